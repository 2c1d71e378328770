#!/bin/bash
# Round-2z profile set, part B (current binary, one MI355X): config 5 shard,
# config-3 phase, gain and tessellated benches with their PMC passes, and the
# per-GPU throughput of the config-4 strong split's shards (--as-shard-of).
set -e
O=${PROF_OUT:-gpurun_out/r2z_prof}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-fits --no-side-legs"
for n in 2 4 8; do
  timeout -k 10 200 python3 -u bench.py --as-shard-of $n $B > $O/shard_of_$n.json 2> $O/shard_of_$n.err
  echo shard $n done
done
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline --no-fits > $O/bench_c5.json 2> $O/bench_c5.err
echo c5 done
tools/pmc_passes.sh $O/c5eval "write fetch" -- python3 bench.py --workload config5 --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c5 "mfma occ valu" -- python3 bench.py --workload config5 --steps 1 --warmup 0 $B
timeout -k 10 200 python3 -u bench.py --workload config3 --steps 10 --no-cpu-baseline --no-fits > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 200 python3 -u bench.py --screen gain --workload config3 --steps 10 --no-cpu-baseline --no-fits > $O/bench_gain_c3.json 2> $O/bench_gain_c3.err
tools/pmc_passes.sh $O/g3eval "write fetch" -- python3 bench.py --screen gain --workload config3 --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/g3 "mfma occ valu" -- python3 bench.py --screen gain --workload config3 --steps 1 --warmup 0 $B
timeout -k 10 200 python3 -u bench.py --screen tess --workload config3 --steps 20 $B > $O/bench_tess_c3.json 2> $O/bench_tess_c3.err
timeout -k 10 200 python3 -u bench.py --screen tess --workload config3 --steps 20 --smooth-pix 0.5 $B > $O/bench_tess_s05_c3.json 2> $O/bench_tess_s05_c3.err
tools/pmc_passes.sh $O/t3eval "write fetch" -- python3 bench.py --screen tess --workload config3 --steps 1 --warmup 0 $B
mkdir -p $O/t3trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/t3trace -o t -- python3 bench.py --screen tess --workload config3 --steps 20 $B > $O/t3trace/bench.json 2> $O/t3trace.err
echo ALL DONE

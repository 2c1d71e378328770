#!/bin/bash
# Round-2g profile set of the current binary (one MI355X): GPU tests, the
# default bench (config 4), its kernel trace, PMC traffic / MFMA / fp64-VALU
# passes of config 4, the config-5 shard and the config-3 gain screens, and
# the config-3 phase bench.
set -e
O=${PROF_OUT:-gpurun_out/r2g_prof}
mkdir -p $O/c4trace
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
echo tests done
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo bench done
B="--no-cpu-baseline --no-fits --no-side-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c4trace -o t -- python3 bench.py $B > $O/c4trace/bench.json 2> $O/c4trace.err
tools/pmc_passes.sh $O/c4eval "write fetch" -- python3 bench.py --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c4 "mfma occ valu" -- python3 bench.py --steps 1 --warmup 0 $B
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline --no-fits > $O/bench_c5.json 2> $O/bench_c5.err
tools/pmc_passes.sh $O/c5eval "write fetch" -- python3 bench.py --workload config5 --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c5 "mfma occ valu" -- python3 bench.py --workload config5 --steps 1 --warmup 0 $B
timeout -k 10 300 python3 -u bench.py --workload config3 --steps 10 --no-cpu-baseline --no-fits > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python3 -u bench.py --screen gain --workload config3 --steps 10 --no-cpu-baseline --no-fits > $O/bench_gain_c3.json 2> $O/bench_gain_c3.err
tools/pmc_passes.sh $O/g3eval "write fetch" -- python3 bench.py --screen gain --workload config3 --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/g3 "mfma occ valu" -- python3 bench.py --screen gain --workload config3 --steps 1 --warmup 0 $B
echo ALL DONE

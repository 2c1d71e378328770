#!/bin/bash
# Round-2d profile set of the current binary (one MI355X): config-4 bench
# kernel trace + stats, PMC traffic / MFMA / occupancy / fp64-VALU passes of
# config 4 and the config-5 shard (fit + eval).
set -e
O=gpurun_out/r2d_prof
mkdir -p $O/c4trace $O/c5trace
export TMPDIR=/tmp
B="--no-cpu-baseline --no-fits --no-side-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c4trace -o t -- python3 bench.py $B > $O/c4trace/bench.json 2> $O/c4trace.err
echo trace4 done
tools/pmc_passes.sh $O/c4eval "write fetch" -- python3 bench.py --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c4 "mfma occ valu" -- python3 bench.py --steps 1 --warmup 0 $B
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c5trace -o t -- python3 bench.py --workload config5 --steps 1 --warmup 1 $B > $O/c5trace/bench.json 2> $O/c5trace.err
echo trace5 done
tools/pmc_passes.sh $O/c5eval "write fetch" -- python3 bench.py --workload config5 --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c5 "mfma occ valu" -- python3 bench.py --workload config5 --steps 1 --warmup 0 $B
echo ALL DONE

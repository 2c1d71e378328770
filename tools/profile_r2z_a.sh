#!/bin/bash
# Round-2z profile set, part A (current binary, one MI355X): GPU tests, the
# default bench (config 4), its kernel trace and the config-4 PMC passes.
# Part B (tools/profile_r2z_b.sh): config 5, config-3 phase and gain.
set -e
O=${PROF_OUT:-gpurun_out/r2z_prof}
mkdir -p $O/c4trace
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo bench done
B="--no-cpu-baseline --no-fits --no-side-legs"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/c4trace -o t -- python3 bench.py $B > $O/c4trace/bench.json 2> $O/c4trace.err
echo trace done
tools/pmc_passes.sh $O/c4eval "write fetch" -- python3 bench.py --eval-only --steps 1 --warmup 0 $B
tools/pmc_passes.sh $O/c4 "mfma occ valu" -- python3 bench.py --steps 1 --warmup 0 $B
echo ALL DONE

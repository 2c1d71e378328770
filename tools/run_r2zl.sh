#!/bin/bash
# Smoothed tessellated fill (sigma 0.5 px, config 1's smoothing) at the
# config-3 shape: bench, kernel trace, PMC write / fetch passes.
set -e
O=gpurun_out/r2zl
mkdir -p $O/trace
export TMPDIR=/tmp
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --smooth-pix 0.5"
timeout -k 10 200 python3 -u bench.py $B --steps 20 > $O/bench.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o t -- python3 bench.py $B --steps 20 > $O/trace/bench.json 2> $O/trace.err
tools/pmc_passes.sh $O/eval "write fetch" -- python3 bench.py $B --steps 1 --warmup 0
echo ALL DONE

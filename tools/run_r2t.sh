#!/bin/bash
# Config-4 step schedule A/B: pipelined (fit of chunk c+1 on reserved CUs
# beside the eval of chunk c) vs serial fit-then-eval on the whole chip.
set -e
O=gpurun_out/r2t
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 10 --warmup 2"
run() { n=$1; shift; timeout -k 10 240 python3 -u bench.py $B "$@" > $O/$n.json 2> $O/$n.err; echo "$n done"; }
run pipe_default
run serial --chunks 1
run pipe_r0 --chunks 2 --reserve-cus 0
run pipe_c4 --chunks 4
run serial_b --chunks 1
run pipe_default_b
echo ALL DONE

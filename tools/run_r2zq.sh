#!/bin/bash
# Four-plane (XX / YY amplitude) smoothed tessellated fill: radii 9-11
# compiled vs the run-time radius kernel (HEAD library), sigma 2.5 (R 10).
set -e
O=gpurun_out/r2zq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --steps 5 --warmup 1 --tess-gain"
for s in 0.5 2.5; do
  SCREENFIT_LIB=$PWD/build_ab/libscreenfit_head.so timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/g_head_s$s.json 2>> $O/err.log
  timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/g_new_s$s.json 2>> $O/err.log
  echo smooth $s
done
echo ALL DONE

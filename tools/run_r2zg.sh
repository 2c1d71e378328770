#!/bin/bash
# Run-time-radius smoothing kernel with 4 taps per loop trip: tessellated
# GPU tests, then smoothed fills at sigma 2.5 / 4 / 6 px (R 10 / 16 / 24),
# the HEAD library (6fa4a8a+, loop not unrolled) beside it.
set -e
O=gpurun_out/r2zo
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --steps 5 --warmup 1"
for s in 2.5 5.0 6.0; do
  SCREENFIT_LIB=$PWD/build_ab/libscreenfit_head.so timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/t3_head_s$s.json 2>> $O/err.log
  timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/t3_new_s$s.json 2>> $O/err.log
  echo smooth $s
done
echo ALL DONE

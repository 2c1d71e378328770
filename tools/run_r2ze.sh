#!/bin/bash
# Wide-tile smoothing kernel: tessellated GPU tests (bitwise vs the round-1
# tile kernel, vs scipy), then smoothed fills at the config-3 shape, new vs
# SF_OPT_TESS_TILE is not reachable from bench -> the HEAD library beside it.
set -e
O=gpurun_out/r2ze
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --steps 10"
for s in 0.5 1.3 4.0; do
  SCREENFIT_LIB=$PWD/build_ab/libscreenfit_head.so timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/t3_head_s$s.json 2>> $O/err.log
  timeout -k 10 200 python -u bench.py $B --smooth-pix $s > $O/t3_new_s$s.json 2>> $O/err.log
  echo smooth $s
done
echo ALL DONE

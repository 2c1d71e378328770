#!/bin/bash
# Tessellated gather with the value-table pre-pass: tests, slots-per-item
# sweep at the config-3 shape (256^2, 102,400 slots), HEAD library beside it.
set -e
O=gpurun_out/r2zc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --steps 20"
BASE=$PWD/build_ab/libscreenfit_head.so
for i in 1 2; do
  SCREENFIT_LIB=$BASE timeout -k 10 120 python -u bench.py $B > $O/t3_head_$i.json 2>> $O/err.log
  timeout -k 10 120 python -u bench.py $B > $O/t3_auto_$i.json 2>> $O/err.log
  for c in 8 16 64; do
    timeout -k 10 120 python -u bench.py $B --tess-slots $c > $O/t3_c${c}_$i.json 2>> $O/err.log
  done
  echo rep $i
done
echo ALL DONE

#!/bin/bash
# Tessellated gather: waves per workgroup x slots per item at the config-3
# shape (256^2, 102,400 slots), after the GPU tess tests.
set -e
O=gpurun_out/r2zd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --screen tess --workload config3 --steps 20"
for i in 1 2; do
  for wk in 4:4 4:8 8:8 8:16 16:16 16:32; do
    w=${wk%:*}; k=${wk#*:}
    timeout -k 10 120 python -u bench.py $B --tess-waves $w --tess-slots $k > $O/t3_w${w}_k${k}_$i.json 2>> $O/err.log
  done
  echo rep $i
done
echo ALL DONE

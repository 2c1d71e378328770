#!/bin/bash
# checksum mode cost at config 5 (register tile, D = 50) and config 4, same box
set -e
O=gpurun_out/r2cs3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2cs3_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs"
for rep in 1; do
for c in on off; do
  timeout -k 10 300 python3 -u bench.py --workload config5 $B --steps 2 --warmup 1 --checksum $c > $O/c5_${c}_$rep.json 2> $O/c5_${c}_$rep.err
  echo "c5 $c $rep done"
done; done
echo ALL DONE

#!/bin/bash
# lean vs general fit pass layout: GPU fit tests, then timing / bit-identity
set -e
O=gpurun_out/r2fa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gain.py tests/test_tec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo tests done
timeout -k 10 200 python3 -u tools/fit_ab.py --workload config4 > $O/ab.txt 2>&1
timeout -k 10 200 python3 -u tools/fit_ab.py --workload config4 --weights random --times 250 >> $O/ab.txt 2>&1
timeout -k 10 300 python3 -u tools/fit_ab.py --workload config5 --reps 3 >> $O/ab.txt 2>&1
echo ALL DONE

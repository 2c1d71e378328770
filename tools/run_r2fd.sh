#!/bin/bash
# fit: slot loads hoisted vs HEAD; fit GPU tests on the new library
set -e
O=gpurun_out/r2fd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gain.py tests/test_tec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo tests done
for v in head new; do
  if [ $v = new ]; then L=ska-sdp-screen-fitting_amd/ska_sdp_screen_fitting_amd/libscreenfit.so; else L=build_ab/$v/libscreenfit.so; fi
  echo "== $v" >> $O/ab.txt
  SCREENFIT_LIB=$L timeout -k 10 200 python3 -u tools/fit_ab.py --workload config4 >> $O/ab.txt 2>&1
  SCREENFIT_LIB=$L timeout -k 10 300 python3 -u tools/fit_ab.py --workload config5 --reps 3 >> $O/ab.txt 2>&1
done
echo ALL DONE

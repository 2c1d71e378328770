#!/bin/bash
# fit kernel register budget A/B: default (1 wave/SIMD budget: 242 VGPRs ->
# 2 waves), min 2 waves/SIMD, min 3 (168 VGPRs, spills); lean layout on/off each
set -e
O=gpurun_out/r2fb
mkdir -p $O
for v in default mw2 mw3; do
  if [ $v = default ]; then L=ska-sdp-screen-fitting_amd/ska_sdp_screen_fitting_amd/libscreenfit.so; else L=build_ab/$v/libscreenfit.so; fi
  echo "== $v" >> $O/ab.txt
  SCREENFIT_LIB=$L timeout -k 10 200 python3 -u tools/fit_ab.py --workload config4 >> $O/ab.txt 2>&1
  SCREENFIT_LIB=$L timeout -k 10 300 python3 -u tools/fit_ab.py --workload config5 --reps 3 >> $O/ab.txt 2>&1
  echo "$v done"
done
echo ALL DONE

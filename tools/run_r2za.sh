#!/bin/bash
# A/B of the pairwise NaN-scrub epilogue (current library) against the HEAD
# library built into build_ab/libscreenfit_base.so, alternating on one box:
# config-3 gain screens, config 4 and config 5 (eval only).
set -e
O=gpurun_out/r2za
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gain.py tests/test_slot_sums.py tests/test_tessellated.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests done
B="--no-cpu-baseline --no-fits --no-side-legs --eval-only"
BASE=$PWD/build_ab/libscreenfit_base.so
for i in 1 2; do
  SCREENFIT_LIB=$BASE timeout -k 10 120 python -u bench.py --screen tess --workload config3 --steps 10 $B > $O/t3_base_$i.json 2>> $O/err.log
  timeout -k 10 120 python -u bench.py --screen tess --workload config3 --steps 10 $B > $O/t3_new_$i.json 2>> $O/err.log
  echo tess $i
done
timeout -k 10 120 python -u bench.py --screen tess --workload config3 --steps 10 --smooth-pix 0.5 $B > $O/t3s_new.json 2>> $O/err.log
for i in 1 2; do
  SCREENFIT_LIB=$BASE timeout -k 10 120 python -u bench.py --screen gain --workload config3 --steps 10 $B > $O/g3_base_$i.json 2>> $O/err.log
  timeout -k 10 120 python -u bench.py --screen gain --workload config3 --steps 10 $B > $O/g3_new_$i.json 2>> $O/err.log
  echo gain $i
done
for i in 1 2; do
  SCREENFIT_LIB=$BASE timeout -k 10 150 python -u bench.py --steps 5 --warmup 1 $B > $O/c4_base_$i.json 2>> $O/err.log
  timeout -k 10 150 python -u bench.py --steps 5 --warmup 1 $B > $O/c4_new_$i.json 2>> $O/err.log
  echo c4 $i
done
for i in 1 2; do
  SCREENFIT_LIB=$BASE timeout -k 10 200 python -u bench.py --workload config5 --steps 1 --warmup 1 $B > $O/c5_base_$i.json 2>> $O/err.log
  timeout -k 10 200 python -u bench.py --workload config5 --steps 1 --warmup 1 $B > $O/c5_new_$i.json 2>> $O/err.log
  echo c5 $i
done
echo ALL DONE

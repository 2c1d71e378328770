set -e
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
V=shb+nt,tile+nt,lds16h+nt,lds8h+nt,lds16+nt
timeout -k 10 200 python3 tools/eval_variants.py --variants $V --reps 5 50:512 20:256 > $O/variants_new.txt 2>&1
SCREENFIT_LIB=$PWD/build_ab/src/ska-sdp-screen-fitting_amd/ska_sdp_screen_fitting_amd/libscreenfit.so timeout -k 10 200 python3 tools/eval_variants.py --variants $V --reps 5 50:512 20:256 > $O/variants_r1.txt 2>&1
timeout -k 10 200 python3 tools/eval_variants.py --variants $V --reps 5 50:512 20:256 > $O/variants_new2.txt 2>&1
tools/pmc_passes.sh $O/d50_shb "occ mfma" -- python3 tools/eval_variants.py --variants shb+nt --reps 2 50:512
tools/pmc_passes.sh $O/d20_lds16 "occ mfma" -- python3 tools/eval_variants.py --variants lds16+nt --reps 2 20:256
echo done

#!/bin/bash
# Energy-attribution builds of libscreenfit.so (kl_eval_impl.h
# SF_EVAL_ENERGY_DIAG): 1 contraction only, 2 epilogue only, 3 stores only,
# 4 empty evaluation launches (the integer prepass alone).  Built on the CPU
# here, shipped to the GPU box in-tree (git-ignored), loaded by bench.py
# through SCREENFIT_LIB; never the product library.
#   tools/energy_variants.sh [DIAG ...]
set -e
cd "$(dirname "$0")/../ska-sdp-screen-fitting_amd/csrc"
mkdir -p variants
for d in ${@:-1 2 3 4}; do
  make -j8 BUILD=build_diag$d EXTRA=-DSF_EVAL_ENERGY_DIAG=$d \
    OUT=variants/libscreenfit_diag$d.so > /dev/null
  echo "built variants/libscreenfit_diag$d.so"
done

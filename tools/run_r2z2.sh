#!/bin/bash
# 256^2 x D = 20 (config 4 shape): every LDS-staged variant x groups, auto map
set -e
O=gpurun_out/r2z2
mkdir -p $O
timeout -k 10 400 python3 -u tools/eval_variants.py --slots 409600 --reps 5 20:256 \
  --variants lds16+nt,lds16h+nt+xi+g2,lds16h+nt+xi+g4,lds8+nt+xi+g2,lds8+nt+xi+g4,lds8h+nt+xi+g2,lds4+nt+xi+g2,lds4+nt+xi+g4,lds4+nt+xi+g1,lds8+nt+xi+g1 > $O/d20xi.txt 2>&1
echo ALL DONE

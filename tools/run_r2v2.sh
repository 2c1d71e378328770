#!/bin/bash
# Pixel bands x XCD map at 512^2, second pass (D = 50 register tile, D = 20 LDS16)
set -e
O=gpurun_out/r2v2
mkdir -p $O
timeout -k 10 300 python3 -u tools/eval_variants.py --slots 409600 --reps 5 50:512 \
  --variants tile+nt,tile+nt+xi+b8,tile+nt+xi+b4,tile+nt+xi+b16,tile+nt+xi+b8+g32,tile+nt+xi+b8+g128,tile+nt+xi+b2,shb+nt+xi+b8 > $O/d50.txt 2>&1
echo d50 done
timeout -k 10 300 python3 -u tools/eval_variants.py --slots 409600 --reps 5 20:512 \
  --variants lds16+nt,lds16+nt+xi,lds16+nt+xi+b2,lds16+nt+xi+b4,lds16+nt+g32,lds16+nt+xi+g32,lds16+nt+xi+b2+g32 > $O/d20.txt 2>&1
echo ALL DONE

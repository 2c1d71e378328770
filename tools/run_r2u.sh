#!/bin/bash
# Pixel-band A/B (SF_OPT_EVAL_BANDS) at 512^2: does keeping each XCD's
# slice of the pixel basis L2-resident lift the 512^2 evaluation?
set -e
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 300 python3 -u tools/eval_variants.py --slots 409600 --reps 5 20:512 20:256 \
  --variants lds16+nt,lds16+nt+b2,lds16+nt+b4,lds16+nt+g2,lds16+nt+g2+b2,lds16+nt+g2+b4,lds16+nt+g4+b4,tile+nt,tile+nt+b4,tile+nt+b8 > $O/d20.txt 2>&1
echo d20 done
timeout -k 10 300 python3 -u tools/eval_variants.py --slots 409600 --reps 5 50:512 \
  --variants tile+nt,tile+nt+b2,tile+nt+b4,tile+nt+b8,tile+nt+b16,tile+nt+g16+b8,tile+nt+xi,tile+nt+xi+b8 > $O/d50.txt 2>&1
echo ALL DONE

set -e
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 300 python3 tools/eval_variants.py --slots 1638400 --reps 3 --variants lds16+nt+g1,lds16+nt+g2,lds16+nt+g4,lds16+nt+g16,lds16h+nt+g1,lds4+nt+g1 20:256 > $O/d20.txt 2>&1
timeout -k 10 300 python3 tools/eval_variants.py --slots 1638400 --reps 3 --variants lds16h+nt+g1,lds16h+nt+g2,lds16h+nt+g16,lds16+nt+g1 7:128 > $O/d7.txt 2>&1
timeout -k 10 300 python3 tools/eval_variants.py --slots 409600 --reps 3 --variants lds4+nt+g1,lds4+nt+g4,lds4+nt+g16,lds16+nt+g1,lds16+nt+g4,tile+nt+g4,tile+nt+g16,tile+nt+g64 36:512 44:512 50:512 > $O/d50.txt 2>&1
echo done

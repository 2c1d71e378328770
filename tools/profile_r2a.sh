#!/bin/bash
# Round-2a profile set (one MI355X): fp64 MFMA probe, PMC passes of the
# evaluation kernels at the config-5 shape (D = 50, 512^2) and config 3/4
# shape (D = 20, 256^2), config-4 kernel trace + traffic passes.
set -e
O=gpurun_out/r2a_prof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_f64_peak > $O/mfma_peak.txt 2>&1
tools/pmc_passes.sh $O/probe "mfma occ" -- ./tools/mfma_f64_peak
for v in shb tile3 lds16h; do
  tools/pmc_passes.sh $O/d50_$v "occ mfma valu lds" -- python3 tools/eval_variants.py --variants $v+nt --reps 2 50:512
done
tools/pmc_passes.sh $O/d20_lds16 "occ mfma valu lds" -- python3 tools/eval_variants.py --variants lds16+nt --reps 2 20:256
# config 4 (bench default): kernel trace of the whole bench, traffic passes
mkdir -p $O/c4trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c4trace -o t -- python3 bench.py --no-cpu-baseline --no-fits --no-side-legs > $O/c4trace/bench.json 2> $O/c4trace.err
tools/pmc_passes.sh $O/c4 "write fetch mfma occ" -- python3 bench.py --eval-only --steps 1 --warmup 0 --no-cpu-baseline --no-fits --no-side-legs
echo ALL DONE

# Bench pipeline variants (fit || eval overlap) on one GPU, one JSON line each.
set -e
mkdir -p gpurun_out/sweep
OUT=gpurun_out/sweep/pipeline.jsonl
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-fits --steps 10 "$@" >> $OUT 2> gpurun_out/sweep/last.err
}
for v in "$@"; do
  run $v
done

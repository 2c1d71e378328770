#!/bin/bash
# The counter tables bench.py reads (profiles/traffic.json, mfma.json,
# fit_flops.json), re-taken on the library in the tree: separate rocprofv3
# PMC passes (tools/pmc_passes.sh) of bench.py runs, one set per workload.
# Run on the GPU box in two halves (each under gpurun's per-call limit):
#   tools/pmc_refresh.sh OUTDIR a     config 4 eval + fit, tessellated fill
#   tools/pmc_refresh.sh OUTDIR b     config 5 eval + fit, gain eval + fit
# then here: tools/pmc_refresh.sh OUTDIR tables   (tools/pmc_traffic.py).
set -e
out=$1
half=$2
B="--no-cpu-baseline --no-fits --no-side-legs --no-child-legs --no-parity"
run() {  # NAME SETS ARGS...
  local name=$1 sets=$2
  shift 2
  tools/pmc_passes.sh "$out/$name" "$sets" -- python3 bench.py $B "$@"
}
case $half in
  a)
    run c4eval "write fetch mfma occ trace" --eval-only --steps 1 --warmup 1
    run c4fit "valu occ trace" --steps 1 --warmup 0
    run t3 "write fetch" --screen tess --workload config3 --eval-only --steps 2 --warmup 1 ;;
  b)
    run c5eval "write fetch mfma occ trace" --workload config5 --eval-only --steps 1 --warmup 0
    run c5fit "valu occ trace" --workload config5 --steps 1 --warmup 0
    run g3eval "write fetch mfma occ trace" --screen gain --workload config3 --eval-only \
      --steps 4 --warmup 1
    run g3fit "valu occ trace" --screen gain --workload config3 --steps 1 --warmup 0 ;;
  tables)
    lab=$(basename "$out")
    # config 4: one 8.192 M-slot call per step (8 one-shot dispatches)
    python3 tools/pmc_traffic.py --traffic-dir "$out/c4eval" --mfma-dir "$out/c4eval" \
      --workload config4 --flags 769 --slots 8192000 --grid 256 --n-dir 20 \
      --eval-kernel "kl_eval_lds_kernel<16 waves>" --label "$lab" \
      --fit-dir "$out/c4fit" --fit-trace-dir "$out/c4fit/trace"
    # config 5: the 16.384 M-slot shard of 64 stations, KL 512^2, D = 50
    python3 tools/pmc_traffic.py --traffic-dir "$out/c5eval" --mfma-dir "$out/c5eval" \
      --workload config5 --flags 769 --slots 16384000 --grid 512 --n-dir 50 \
      --eval-kernel kl_eval_kernel --label "$lab" \
      --fit-dir "$out/c5fit" --fit-trace-dir "$out/c5fit/trace"
    # gain screens on the config-3 shape: three coefficient sets
    python3 tools/pmc_traffic.py --traffic-dir "$out/g3eval" --mfma-dir "$out/g3eval" \
      --workload config3-gain --flags 769 --slots 102400 --grid 256 --n-dir 20 \
      --coef-sets 3 --eval-kernel kl_eval_kernel --label "$lab" \
      --fit-dir "$out/g3fit" --fit-trace-dir "$out/g3fit/trace"
    # tessellated fill (no smoothing) on the config-3 shape
    python3 tools/pmc_traffic.py --traffic-dir "$out/t3" --kernel sf::kl_tess_gather \
      --workload config3-tess --flags 1 --slots 102400 --grid 256 --n-dir 20 \
      --eval-kernel kl_tess_gather_kernel --label "$lab" ;;
  *)
    echo "usage: tools/pmc_refresh.sh OUTDIR a|b|tables" >&2
    exit 2 ;;
esac

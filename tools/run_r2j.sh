set -e
O=gpurun_out/r2j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
B="--no-cpu-baseline --no-fits"
timeout -k 10 300 python -u bench.py $B > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --workload config5 --steps 1 --warmup 1 $B > $O/bench_c5.json 2> $O/bench_c5.err
tools/pmc_passes.sh $O/c5eval "fetch" -- python3 bench.py --workload config5 --eval-only --steps 1 --warmup 0 $B --no-side-legs
tools/pmc_passes.sh $O/c4eval "fetch" -- python3 bench.py --eval-only --steps 1 --warmup 0 $B --no-side-legs
echo done

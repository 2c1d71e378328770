set -e
O=gpurun_out/r2s
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-fits --steps 8 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline --no-fits > $O/bench_c5.json 2> $O/bench_c5.err
echo done

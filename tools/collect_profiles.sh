set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/prof/bench_default.json 2> gpurun_out/prof/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/stats -o s -- python3 bench.py --no-cpu-baseline --no-fits > gpurun_out/prof/bench_stats.json 2> gpurun_out/prof/stats.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/prof/pmcw -o w -- python3 bench.py --eval-only --steps 1 --warmup 0 --no-cpu-baseline --no-fits > gpurun_out/prof/pmcw.json 2> gpurun_out/prof/pmcw.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/prof/pmcf -o f -- python3 bench.py --eval-only --steps 1 --warmup 0 --no-cpu-baseline --no-fits > gpurun_out/prof/pmcf.json 2> gpurun_out/prof/pmcf.err
find gpurun_out/prof -name "*.csv" | sort
tail -c 600 gpurun_out/prof/bench_default.json

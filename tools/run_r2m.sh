set -e
O=gpurun_out/r2m
mkdir -p $O
B="--no-cpu-baseline --no-fits"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 300 python -u bench.py --screen gain --workload config3 --steps 5 $B > $O/gain_c3.json 2> $O/gain_c3.err
timeout -k 10 300 python -u bench.py --screen gain --steps 3 $B > $O/gain_c4.json 2> $O/gain_c4.err
echo done

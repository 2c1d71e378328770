set -e
O=gpurun_out/r2ab
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 5 --warmup 1"
for g in 1 2 4 16; do
timeout -k 10 200 python -u bench.py --workload config2-shape --eval-groups $g $B > $O/c2_g$g.json 2> /dev/null
done
timeout -k 10 200 python -u bench.py $B > $O/c4_default.json 2> /dev/null
timeout -k 10 200 python -u bench.py --workload config3 $B > $O/c3_default.json 2> /dev/null
timeout -k 10 200 python -u bench.py --eval-groups 4 $B > $O/c4_g4.json 2> /dev/null
timeout -k 10 200 python -u bench.py --eval-groups 16 $B > $O/c4_g16.json 2> /dev/null
timeout -k 10 200 python -u bench.py $B > $O/c4_default2.json 2> /dev/null
timeout -k 10 300 python -u bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline --no-fits --no-side-legs > $O/c5_default.json 2> /dev/null
echo done

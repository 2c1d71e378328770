set -e
O=gpurun_out/r2y
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 5 --warmup 1"
for g in 1 2 16 1; do
timeout -k 10 200 python -u bench.py --eval-groups $g $B > $O/c4_g$g.json 2> $O/c4_g$g.err
timeout -k 10 200 python -u bench.py --eval-groups $g --eval-only $B > $O/c4e_g$g.json 2> $O/c4e_g$g.err
done
for g in 1 16; do
timeout -k 10 200 python -u bench.py --workload config2-shape --eval-groups $g $B > $O/c2_g$g.json 2> $O/c2_g$g.err
timeout -k 10 200 python -u bench.py --workload config3 --eval-groups $g $B > $O/c3_g$g.json 2> $O/c3_g$g.err
done
echo done

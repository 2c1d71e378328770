set -e
O=gpurun_out/r2v
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --eval-only --steps 4 --warmup 1"
for g in 1 2 4 8 16; do
timeout -k 10 200 python -u bench.py --eval-groups $g $B > $O/c4_g$g.json 2> $O/c4_g$g.err
done
timeout -k 10 200 python -u bench.py --eval-groups 16 $B > $O/c4_g16b.json 2> $O/c4_g16b.err
timeout -k 10 200 python -u bench.py --eval-groups 1 $B > $O/c4_g1b.json 2> $O/c4_g1b.err
echo done

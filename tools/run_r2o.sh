set -e
O=gpurun_out/r2o
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs"
for g in 16 64 256; do
timeout -k 10 300 python -u bench.py --screen gain --steps 3 --warmup 1 --eval-groups $g $B > $O/gain_c4_g$g.json 2> $O/gain_c4_g$g.err
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --eval-only --eval-groups $g $B > $O/c4_g$g.json 2> $O/c4_g$g.err
timeout -k 10 300 python -u bench.py --workload config5 --steps 1 --warmup 1 --eval-only --eval-groups $g $B > $O/c5_g$g.json 2> $O/c5_g$g.err
done
echo done

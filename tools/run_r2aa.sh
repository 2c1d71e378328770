set -e
O=gpurun_out/r2aa
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 4 --warmup 1 --eval-only"
for x in 0 1; do for g in 1 2 4 8; do
timeout -k 10 200 python -u bench.py --eval-groups $g --eval-xcd-map $x $B > $O/c4_x${x}_g$g.json 2> /dev/null
timeout -k 10 200 python -u bench.py --workload config3 --eval-groups $g --eval-xcd-map $x $B > $O/c3_x${x}_g$g.json 2> /dev/null
done; done
echo done

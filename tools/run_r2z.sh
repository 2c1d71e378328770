set -e
O=gpurun_out/r2z
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 4 --warmup 1 --eval-only"
for g in 1 2 4 8 16; do
timeout -k 10 200 python -u bench.py --eval-groups $g $B > $O/c4_on_g$g.json 2> /dev/null
timeout -k 10 200 python -u bench.py --eval-groups $g --checksum off $B > $O/c4_off_g$g.json 2> /dev/null
timeout -k 10 200 python -u bench.py --eval-groups $g --reserve-cus 0 $B > $O/c4_r0_g$g.json 2> /dev/null
timeout -k 10 200 python -u bench.py --workload config3 --eval-groups $g $B > $O/c3_g$g.json 2> /dev/null
done
echo done

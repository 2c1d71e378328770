set -e
O=gpurun_out/r2n
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs"
for w in config3 config4; do for c in on off; do
timeout -k 10 300 python -u bench.py --screen gain --workload $w --steps 3 --warmup 1 --checksum $c $B > $O/gain_${w}_$c.json 2> $O/gain_${w}_$c.err
done; done
for c in on off; do
timeout -k 10 300 python -u bench.py --workload config5 --steps 1 --warmup 1 --eval-only --checksum $c $B > $O/c5_$c.json 2> $O/c5_$c.err
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --eval-only --checksum $c $B > $O/c4_$c.json 2> $O/c4_$c.err
done
echo done

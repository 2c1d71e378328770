set -e
O=gpurun_out/r2p
mkdir -p $O
B="--no-cpu-baseline --no-fits --no-side-legs --steps 8 --warmup 1"
for rep in 1 2; do for r in 16 24 32 8; do
timeout -k 10 200 python -u bench.py --reserve-cus $r $B > $O/c4_r${r}_$rep.json 2> $O/c4_r${r}_$rep.err
done; done
timeout -k 10 200 python -u bench.py --chunks 4 $B > $O/c4_ch4.json 2> $O/c4_ch4.err
timeout -k 10 200 python -u bench.py --chunks 1 $B > $O/c4_ch1.json 2> $O/c4_ch1.err
echo done

set -e
O=gpurun_out/r2l
mkdir -p $O
B="--no-cpu-baseline --no-fits"
timeout -k 10 300 python -u bench.py --screen gain --workload config3 --steps 5 $B > $O/gain_c3.json 2> $O/gain_c3.err
timeout -k 10 300 python -u bench.py --screen gain --steps 3 $B > $O/gain_c4.json 2> $O/gain_c4.err
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 $B > $O/gloo2_c4.json 2> $O/gloo2_c4.err
echo done

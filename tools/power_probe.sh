#!/bin/bash
# (tools/power_probe.sh OUTDIR BENCH_ARGS...: board power and clocks while a
# bench.py run is in its timed loop; reading only, no settings changed)
# sample the board power / clocks while one eval-only bench runs
out=$1; shift
mkdir -p $out
( timeout -k 10 120 python3 bench.py "$@" > $out/bench.json 2> $out/bench.err ) &
pid=$!
sleep ${PROBE_DELAY:-8}
for i in 1 2 3 4 5 6; do
  timeout 10 rocm-smi --showpower --showclocks --showtemp >> $out/smi.txt 2>&1
  timeout 10 amd-smi metric -p -c 2>/dev/null | head -40 >> $out/amdsmi.txt
  sleep 1
done
wait $pid

#!/bin/bash
# lean fit in the benches + full GPU tests + smoke
set -e
O=gpurun_out/r2fc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
echo tests done
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo smoke done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-fits --steps 10 > $O/c4.json 2> $O/c4.err
echo c4 done
timeout -k 10 400 python3 -u bench.py --workload config5 --no-cpu-baseline --no-fits --steps 2 --warmup 1 > $O/c5.json 2> $O/c5.err
echo ALL DONE

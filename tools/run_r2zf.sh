#!/bin/bash
# Final-binary check: the full GPU suite, smoke(), the default bench.
set -e
O=gpurun_out/r2zp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
echo tests done
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke done
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo ALL DONE

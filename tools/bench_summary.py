#!/usr/bin/env python3
"""One line per bench.py JSON file: value, eval roofline fraction, launch
time, kernel, check.  python tools/bench_summary.py FILE..."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as exc:
        print(f"{path}: {exc}")
        continue
    r = d.get("roofline", {})
    side = d.get("side_legs", {})
    alone = side.get("eval_fp32_sincos", {}).get("frac")
    st = d.get("stages_ms", {})
    print(f"{path.split('/')[-1]:<28} value {d['value'] / 1e6:8.3f} M/s  "
          f"frac {r.get('frac', 0):.4f}  launch {r.get('launch_ms', 0):9.2f} ms  "
          f"alone {alone if alone is None else round(alone, 4)}  "
          f"fit {st.get('fit', 0):7.2f} ms  {r.get('kernel')}  "
          f"check {json.dumps(d.get('check', {}).get('sampled_slots', {}).get('ok'))}")

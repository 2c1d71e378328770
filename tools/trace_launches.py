#!/usr/bin/env python3
"""Average duration of the TIMED evaluation launches of a bench.py run from
its rocprofv3 kernel trace (``--kernel-trace -f csv``): the launches of the
evaluation kernel whose grid is the bench's full grid are taken in start
order, the first ``warmup x chunks`` (warmup steps) are dropped and the next
``steps x chunks`` averaged -- the single-slot launches of the sampled-slot
check and the side legs after the timed region are excluded.

    python tools/trace_launches.py TRACE.csv --warmup 2 --steps 20 --chunks 2
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_csv")
    ap.add_argument("--kernel", default="sf::kl_eval")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--chunks", type=int, default=2)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace_csv)) if a.kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no {a.kernel} launches in {a.trace_csv}")
    gkey = "Grid_Size" if "Grid_Size" in rows[0] else "Grid_Size_X"
    big = max(int(r[gkey]) for r in rows)
    full = sorted((r for r in rows if int(r[gkey]) == big),
                  key=lambda r: int(r["Start_Timestamp"]))
    skip = a.warmup * a.chunks
    timed = full[skip:skip + a.steps * a.chunks]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in timed]
    out = {"kernel": timed[0]["Kernel_Name"].split("(")[0], "grid": big,
           "launches_in_trace": len(rows), "full_grid_launches": len(full),
           "timed_launches": len(dur), "avg_ms": sum(dur) / len(dur),
           "min_ms": min(dur), "max_ms": max(dur)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

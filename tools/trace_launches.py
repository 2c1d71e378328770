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
    ap.add_argument("--gap-us", type=float, default=50.0,
                    help="dispatches closer than this belong to one launch")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace_csv)) if a.kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no {a.kernel} launches in {a.trace_csv}")
    gkey = "Grid_Size" if "Grid_Size" in rows[0] else "Grid_Size_X"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one bench launch = consecutive dispatches of the kernel with no gap
    # (sf_kl_eval splits a call into one-shot launches of <= 2^31 work-items)
    groups = []
    for r in rows:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if groups and t0 - groups[-1]["end"] < a.gap_us * 1000:
            g = groups[-1]
            g["end"] = t1
            g["dispatches"] += 1
            g["work"] += int(r[gkey])
        else:
            groups.append({"start": t0, "end": t1, "dispatches": 1, "work": int(r[gkey])})
    big = max(g["work"] for g in groups)
    full = [g for g in groups if g["work"] >= 0.5 * big]
    skip = a.warmup * a.chunks
    timed = full[skip:skip + a.steps * a.chunks]
    dur = [(g["end"] - g["start"]) * 1e-6 for g in timed]
    out = {"kernel": rows[0]["Kernel_Name"].split("(")[0],
           "dispatches_in_trace": len(rows), "bench_launches": len(full),
           "dispatches_per_launch": timed[0]["dispatches"],
           "timed_launches": len(dur), "avg_ms": sum(dur) / len(dur),
           "min_ms": min(dur), "max_ms": max(dur),
           "note": "a bench launch spans its consecutive dispatches, first "
                   "start to last end"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

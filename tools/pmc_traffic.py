#!/usr/bin/env python3
"""HBM traffic per eval launch from two rocprofv3 PMC passes (separate runs,
per MI355X_MICROARCH.md): WRITE_SIZE and FETCH_SIZE counter CSVs in KB;
FETCH_SIZE is doubled (gfx950 correction in the guide).  Writes
profiles/traffic.json, which bench.py reads when workload / flags / chunks
match its own run.

  python tools/pmc_traffic.py WRITE.csv FETCH.csv --workload config3 \
      --flags 769 --chunks 2 --slots 51200 --grid 256 --n-dir 20 \
      --eval-kernel 'kl_eval_lds_kernel<16 waves>'
"""
import argparse
import csv
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter, kernel="sf::kl_eval"):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"].split("(")[0]
    if not vals:
        raise SystemExit(f"no {kernel} rows with {counter} in {path}")
    return sum(vals) / len(vals), len(vals), name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("write_csv")
    ap.add_argument("fetch_csv")
    ap.add_argument("--workload", default="config3")
    ap.add_argument("--flags", type=int, required=True)
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--slots", type=int, required=True, help="slots per launch")
    ap.add_argument("--grid", type=int, required=True)
    ap.add_argument("--n-dir", type=int, required=True)
    ap.add_argument("--eval-kernel", required=True,
                    help="bench.py's roofline.kernel for the profiled run")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "traffic.json"))
    a = ap.parse_args()
    w_kb, nw, name = per_launch(a.write_csv, "WRITE_SIZE")
    f_kb, nf, _ = per_launch(a.fetch_csv, "FETCH_SIZE")
    wb, fb = w_kb * 1024.0, 2.0 * f_kb * 1024.0
    algo = a.slots * (16 * a.grid * a.grid + 8 * a.n_dir)
    out = {
        "workload": a.workload, "kernel": name, "eval_kernel": a.eval_kernel,
        "flags": a.flags,
        "chunks": a.chunks, "launches_averaged": min(nw, nf),
        "write_bytes": wb, "fetch_bytes_corrected_x2": fb,
        "hbm_bytes_per_launch": wb + fb,
        "algorithmic_bytes_per_launch": algo,
        "ratio_to_algorithmic": (wb + fb) / algo,
        "sources": [os.path.relpath(a.write_csv, REPO), os.path.relpath(a.fetch_csv, REPO)],
        "note": "separate rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE passes of "
                "bench.py --eval-only; KB units; FETCH_SIZE doubled per the "
                "MI355X_MICROARCH.md HBM section",
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

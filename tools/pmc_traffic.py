#!/usr/bin/env python3
"""Per-launch HBM traffic and MFMA / VALU busy of the evaluation kernel from
separate rocprofv3 PMC passes (tools/pmc_passes.sh directories), written as
entries of profiles/traffic.json and profiles/mfma.json (keyed by workload and
bench.py's roofline.kernel), which bench.py reports as roofline.traffic and
mfma.busy_frac_pmc when its run matches.

  python tools/pmc_traffic.py --traffic-dir gpurun_out/X/c4eval \
      --mfma-dir gpurun_out/X/c4 --workload config4 --flags 769 --chunks 2 \
      --slots 4096000 --grid 256 --n-dir 20 \
      --eval-kernel 'kl_eval_lds_kernel<16 waves>'

WRITE_SIZE / FETCH_SIZE are in KB; FETCH_SIZE is doubled (the gfx950
correction of MI355X_MICROARCH.md's HBM section).  Counters are averaged over
the full-grid launches of the evaluation kernel (tools/pmc_summary.py).
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summary(d, kernel, trace=None):
    cmd = [sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), d,
           "--kernel", kernel]
    if trace:
        cmd += ["--trace", trace]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return json.loads(out)


def library_of(d):
    """The library identity pmc_passes.sh recorded beside the passes (in the
    pass directory or its parent); no identity, no table entry."""
    for c in (d, os.path.dirname(os.path.normpath(d))):
        f = os.path.join(c, "library.json")
        if os.path.exists(f):
            return json.load(open(f))
    raise SystemExit(f"no library.json in {d} or its parent: counters without "
                     "the identity of the library they were taken on are not kept")


def upsert(path, entry):
    try:
        tab = json.load(open(path))
    except (OSError, ValueError):
        tab = {}
    if "entries" not in tab:  # the round-1 single-entry file
        tab = {"entries": [tab] if tab else []}
    tab["entries"] = [e for e in tab["entries"]
                      if not (e.get("workload") == entry["workload"]
                              and e.get("eval_kernel") == entry["eval_kernel"])]
    tab["entries"].append(entry)
    json.dump(tab, open(path, "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traffic-dir", help="pmc_passes.sh dir with write/ fetch/")
    ap.add_argument("--mfma-dir", help="pmc_passes.sh dir with mfma/ occ/")
    ap.add_argument("--kernel", default="sf::kl_eval")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--flags", type=int, required=True)
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--slots", type=int, required=True, help="slots per launch")
    ap.add_argument("--grid", type=int, required=True)
    ap.add_argument("--n-dir", type=int, required=True)
    ap.add_argument("--coef-sets", type=int, default=1, help="3 for gain screens")
    ap.add_argument("--eval-kernel", required=True,
                    help="bench.py's roofline.kernel for the profiled run")
    ap.add_argument("--fit-dir", help="pmc_passes.sh dir with valu/ occ/ of a "
                    "fit + eval run: fp64 FLOP/s of the fit kernels")
    ap.add_argument("--label", default="")
    ap.add_argument("--fit-trace-dir", help="a --kernel-trace run of the fit command "
                    "(pmc_passes.sh set trace): the fit kernels' durations")
    a = ap.parse_args()
    algo = a.slots * (16 * a.grid * a.grid + 8 * a.n_dir * a.coef_sets)
    if a.traffic_dir:
        r = summary(a.traffic_dir, a.kernel)
        d = r["derived"]
        wb, fb = d["write_bytes"], d["fetch_bytes_x2"]
        entry = {
            "workload": a.workload, "kernel": r["kernel"], "eval_kernel": a.eval_kernel,
            "library_sha16": library_of(a.traffic_dir)["sha16"],
            "flags": a.flags, "chunks": a.chunks, "launches_averaged": r["dispatches"],
            "write_bytes": wb, "fetch_bytes_corrected_x2": fb,
            "hbm_bytes_per_launch": wb + fb,
            "algorithmic_bytes_per_launch": algo,
            "ratio_to_algorithmic": (wb + fb) / algo,
            "source": os.path.relpath(a.traffic_dir, REPO), "label": a.label,
            "note": "separate rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE passes of "
                    "bench.py --eval-only; FETCH_SIZE doubled (MI355X_MICROARCH.md)",
        }
        upsert(os.path.join(REPO, "profiles", "traffic.json"), entry)
        print(json.dumps(entry, indent=1))
    if a.fit_dir:
        entry = fit_entry(a.fit_dir, a.workload, a.label, a.fit_trace_dir)
        upsert(os.path.join(REPO, "profiles", "fit_flops.json"), entry)
        print(json.dumps(entry, indent=1))
    if a.mfma_dir:
        r = summary(a.mfma_dir, a.kernel)
        d = r["derived"]
        entry = {
            "workload": a.workload, "kernel": r["kernel"], "eval_kernel": a.eval_kernel,
            "library_sha16": library_of(a.mfma_dir)["sha16"],
            "mfma_busy_frac": d.get("mfma_busy_frac"),
            "valu_busy_frac": d.get("valu_busy_frac"),
            "cyc_per_mfma_f64": d.get("cyc_per_mfma_f64"),
            "mfma_f64_tflops_under_pmc": d.get("mfma_f64_tflops"),
            "clock_GHz_under_pmc": d.get("clock_GHz"),
            "launches_averaged": r["dispatches"],
            "source": os.path.relpath(a.mfma_dir, REPO), "label": a.label,
            "note": "rocprofv3 --pmc passes (tools/pmc_passes.sh mfma, occ); "
                    "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE"
                    " / 8 x 256 CUs x 4 SIMDs); valu_busy_frac = 4 x "
                    "SQ_ACTIVE_INST_VALU / same (issue cycles)",
        }
        upsert(os.path.join(REPO, "profiles", "mfma.json"), entry)
        print(json.dumps(entry, indent=1))


def fit_entry(d, workload, label, trace=None):
    """fp64 FLOP/s of the fit kernels (VALU: 64 x (2 FMA + MUL + ADD + TRANS)
    per wave-instruction, SQ_INSTS_VALU_*_F64; no MFMA in the fit): flop
    counts from the PMC passes, durations from the kernel trace of the same
    command when given (``avg_ms``), else the slower durations under
    collection (``avg_ms_under_pmc``)."""
    kernels = {}
    for k in ("kl_fit_pass_kernel", "kl_subset_secular_kernel", "kl_subset_eig_kernel",
              "kl_classify_kernel",
              "kl_assign_kernel", "kl_fit_general_kernel"):
        try:
            r = summary(d, k, trace)
        except subprocess.CalledProcessError:
            continue
        dd = r["derived"]
        kernels[k] = {"kernel": r["kernel"], "dispatches_averaged": r["dispatches"],
                      "avg_ms": r.get("avg_ms_trace"),
                      "avg_ms_under_pmc": r["avg_ms_under_pmc"],
                      "fp64_flop_per_launch": dd.get("valu_fp64_flop"),
                      "fp64_tflops": dd.get("valu_fp64_tflops"),
                      "valu_busy_frac": dd.get("valu_busy_frac")}
    return {"workload": workload, "eval_kernel": "fit", "kernels": kernels,
            "library_sha16": library_of(d)["sha16"],
            "source": os.path.relpath(d, REPO), "label": label,
            "trace": os.path.relpath(trace, REPO) if trace else None,
            "note": "largest-grid launch of each fit kernel in a bench.py "
                    "--steps 1 --warmup 0 run under rocprofv3 --pmc (valu, occ "
                    "passes), durations and rates from a --kernel-trace run of "
                    "the same command; fp64 VALU peak 78.6 TFLOP/s"}


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-call PMC figures of one kernel from the CSVs of tools/pmc_passes.sh:
counters summed over the dispatches of one call and averaged over the calls
(small launches -- cross-checks, single-slot checks -- dropped), plus derived
fractions:

* mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x CUs x 4)
  (GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy cycles sum the SIMDs)
* cyc_per_mfma    = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_VALU_MFMA_F64
* valu_busy_frac  = 4 x SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x CUs x 4)
  (SQ_ACTIVE_INST_* count quad-cycles)
* occupancy       = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / CUs   (waves per CU)
* wait / issue / active shares of SQ_WAVE_CYCLES
* fp64 FLOP       = 64 x (2 FMA + MUL + ADD + TRANS) + 2048 x MFMA_F64 ops

    python tools/pmc_summary.py DIR --kernel kl_eval [--cus 256] [--trace TDIR]

``--trace TDIR``: a --kernel-trace run of the same command (pmc_passes.sh
set ``trace``); ``avg_ms_trace`` is then the kernel's mean duration per call
over the same full-grid dispatches without counter collection (PMC passes
serialise and slow the dispatches), and the derived rates use it.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, kernel):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> v
    meta = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = (path, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[key] = (int(r["Grid_Size"]), r["Kernel_Name"].split("(")[0],
                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         r.get("VGPR_Count"), r.get("LDS_Block_Size"),
                         int(r["Start_Timestamp"]))
    return per, meta


def trace_ms(d, kernel, big):
    """Mean duration (ms) per call of ``kernel``'s dispatches with grid
    ``big`` (the PMC grouping's full grid) in the kernel traces under d."""
    durs = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
        for r in rows:
            g = int(r.get("Grid_Size") or r.get("Grid_Size_X"))
            if g == big:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return (sum(durs) / len(durs), len(durs)) if durs else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="sf::kl_eval",
                    help="substring of the full kernel name (template args included)")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--trace", default=None)
    ap.add_argument("--group", type=int, default=0,
                    help="dispatches per call (default: a call ends at a "
                    "partial-grid dispatch)")
    a = ap.parse_args()
    per, meta = load(a.dir, a.kernel)
    if not per:
        raise SystemExit(f"no {a.kernel} dispatches under {a.dir}")
    big = max(m[0] for m in meta.values())
    # bulk dispatches (cross-check launches of a few slots dropped), grouped
    # into calls: sf_kl_eval splits a call longer than 2^31 work-items into
    # one-shot dispatches, so within each pass file a call is the run of
    # consecutive bulk dispatches ending at a partial-grid one (or --group N
    # dispatches each); counters and durations are summed per call
    groups = []
    for path in sorted({k[0] for k in per}):
        ks = sorted((k for k in per if k[0] == path and meta[k][0] * 64 >= big),
                    key=lambda k: meta[k][5])
        cur = []
        for k in ks:
            cur.append(k)
            if (a.group and len(cur) == a.group) or (not a.group and meta[k][0] < big) \
                    or (not a.group and len({meta[x][0] for x in ks}) == 1):
                groups.append(cur)
                cur = []
        if cur:
            groups.append(cur)
    # average every counter over the calls that collected it
    sums, cnt = defaultdict(float), defaultdict(int)
    for g in groups:
        tot = defaultdict(float)
        for k in g:
            for c, v in per[k].items():
                tot[c] += v
        for c, v in tot.items():
            sums[c] += v
            cnt[c] += 1
    avg = {c: sums[c] / cnt[c] for c in sums}
    dur = sum(meta[k][2] for g in groups for k in g) / len(groups) * 1e-6
    k0 = groups[0][0]
    res = {"kernel": meta[k0][1], "grid": big, "dispatches": len(groups),
           "dispatches_per_call": [len(g) for g in groups],
           "work_items_per_call": sum(meta[k][0] for k in groups[0]),
           "avg_ms_under_pmc": dur, "vgpr": meta[k0][3],
           "lds_bytes": meta[k0][4], "counters": avg}
    # rates over the traced duration when a trace is given (the counters
    # are counts, independent of the slow-down under collection)
    if a.trace:
        tms, tn = trace_ms(a.trace, a.kernel, big)
        calls = max(1, round(sum(len(g) for g in groups) / len(groups)))
        if tms is not None:
            res["avg_ms_trace"] = tms * calls
            res["trace_dispatches"] = tn
            rate_ms = tms * calls
        else:
            res["avg_ms_trace"] = None
            rate_ms = dur
    else:
        rate_ms = dur
    g = avg.get("GRBM_GUI_ACTIVE")
    simd_cyc = g / 8 * a.cus * 4 if g else None
    d = {}
    if g:
        d["clock_GHz"] = g / 8 / (dur * 1e-3) / 1e9
    if simd_cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        d["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cyc
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("SQ_INSTS_VALU_MFMA_F64"):
        d["cyc_per_mfma_f64"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / avg["SQ_INSTS_VALU_MFMA_F64"]
    if simd_cyc and "SQ_ACTIVE_INST_VALU" in avg:
        d["valu_busy_frac"] = 4 * avg["SQ_ACTIVE_INST_VALU"] / simd_cyc
    if "SQ_WAVE_CYCLES" in avg and avg.get("SQ_BUSY_CYCLES"):
        d["waves_per_cu"] = avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"] / a.cus * 8
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
            if c in avg:
                d[c.lower() + "_share"] = avg[c] / avg["SQ_WAVE_CYCLES"]
    f64 = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
           "SQ_INSTS_VALU_TRANS_F64"]
    if all(c in avg for c in f64):
        vflop = 64 * (2 * avg[f64[0]] + avg[f64[1]] + avg[f64[2]] + avg[f64[3]])
        d["valu_fp64_flop"] = vflop
        d["valu_fp64_tflops"] = vflop / (rate_ms * 1e-3) / 1e12
    if "SQ_INSTS_VALU_MFMA_MOPS_F64" in avg:
        # MOPS counts 512-flop units per the rocprof-compute convention
        d["mfma_f64_flop"] = 512 * avg["SQ_INSTS_VALU_MFMA_MOPS_F64"]
        d["mfma_f64_tflops"] = d["mfma_f64_flop"] / (rate_ms * 1e-3) / 1e12
    if "SQ_INSTS_VALU_MFMA_F64" in avg:
        # v_mfma_f64_16x16x4_f64: 16 x 16 x 4 x 2 flop per wave-instruction
        d["mfma_f64_flop_from_insts"] = 2048 * avg["SQ_INSTS_VALU_MFMA_F64"]
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
    if "WRITE_SIZE" in avg:
        d["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in avg:
        d["fetch_bytes_x2"] = 2 * avg["FETCH_SIZE"] * 1024
    res["derived"] = d
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

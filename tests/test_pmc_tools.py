"""The measurement tools that feed the bench line's counter tables
(tools/pmc_summary.py, tools/pmc_traffic.py): durations from a kernel
trace, and no table entry without the identity of the library the
counters were taken on."""

import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _write_counters(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "p_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name",
                                "Counter_Value", "Start_Timestamp", "End_Timestamp",
                                "VGPR_Count", "LDS_Block_Size"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _write_trace(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "t_kernel_trace.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Kernel_Name", "Grid_Size_X", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _fixture(tmp_path):
    """Two calls of a fake fit kernel under PMC (slow: 20 ms each) and the
    same two calls in a trace (12 ms each), plus a small launch to drop."""
    base = dict(Kernel_Name="void sf::kl_fit_pass_kernel<false, 2, true>(int)",
                VGPR_Count="128", LDS_Block_Size="0")
    rows = []
    for i, t0 in enumerate((0, 50_000_000)):
        for c, v in (("SQ_INSTS_VALU_FMA_F64", 1e6), ("SQ_INSTS_VALU_MUL_F64", 0),
                     ("SQ_INSTS_VALU_ADD_F64", 0), ("SQ_INSTS_VALU_TRANS_F64", 0),
                     ("GRBM_GUI_ACTIVE", 8 * 2.0e9 * 0.020)):
            rows.append(dict(base, Dispatch_Id=str(i), Grid_Size="65536", Counter_Name=c,
                             Counter_Value=str(v), Start_Timestamp=str(t0),
                             End_Timestamp=str(t0 + 20_000_000)))
    _write_counters(str(tmp_path / "fit" / "valu"), rows)
    _write_trace(str(tmp_path / "fit" / "trace"), [
        dict(Kernel_Name=base["Kernel_Name"], Grid_Size_X="65536",
             Start_Timestamp=str(t0), End_Timestamp=str(t0 + 12_000_000))
        for t0 in (0, 30_000_000)] + [
        dict(Kernel_Name=base["Kernel_Name"], Grid_Size_X="64",
             Start_Timestamp="90000000", End_Timestamp="90001000")])
    return tmp_path / "fit"


def test_summary_rates_use_the_trace(tmp_path):
    d = _fixture(tmp_path)
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"),
                          str(d), "--kernel", "kl_fit_pass_kernel", "--trace", str(d / "trace")],
                         capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["avg_ms_under_pmc"] == pytest.approx(20.0)
    assert r["avg_ms_trace"] == pytest.approx(12.0)
    # 64 lanes x 2 flop x 1e6 FMA instructions over the traced 12 ms
    assert r["derived"]["valu_fp64_tflops"] == pytest.approx(128e6 / 12e-3 / 1e12)


def test_no_entry_without_library_identity(tmp_path):
    import pmc_traffic
    d = _fixture(tmp_path)
    with pytest.raises(SystemExit):
        pmc_traffic.library_of(str(d / "valu"))
    (d / "library.json").write_text(json.dumps({"sha16": "abcdef0123456789", "bytes": 1}))
    assert pmc_traffic.library_of(str(d / "valu"))["sha16"] == "abcdef0123456789"
    e = pmc_traffic.fit_entry(str(d), "w", "lbl", str(d / "trace"))
    assert e["library_sha16"] == "abcdef0123456789"
    k = e["kernels"]["kl_fit_pass_kernel"]
    assert k["avg_ms"] == pytest.approx(12.0) and k["avg_ms_under_pmc"] == pytest.approx(20.0)

"""bench.py's step schedules on the GPU: the two-coefficient-set schedule
(the fit of step k+1 on a second stream beside the eval of step k) for phase
and gain screens, on the small ``tiny`` workload, checked by the bench's own
sampled-slot comparison against an fp64 restatement and the plane
invariants.  Each run is one child process of bench.py."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", "tiny",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-side-legs",
           "--no-fits", "--no-child-legs", *args]
    if "--cpu-baseline" in args:
        cmd.remove("--cpu-baseline")
        cmd.remove("--no-cpu-baseline")
    if "--parity" in args:
        cmd.remove("--parity")
    else:
        cmd.append("--no-parity")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("screen", ["phase", "gain"])
def test_two_coefficient_sets_schedule(screen):
    extra = ["--screen", "gain"] if screen == "gain" else []
    one = _bench("--coef-sets", "1", *extra)
    two = _bench("--coef-sets", "2", *extra)
    assert one["config"]["schedule"]["coef_sets"] == 1
    assert two["config"]["schedule"]["coef_sets"] == 2
    assert "2 coefficient sets" in two["stages_ms"]["overlap"]
    for line in (one, two):
        s = line["check"]["sampled_slots"]
        assert s["ok"], s
        assert line["value"] > 0
    # the default picks two sets for multi-step gain runs, one for phase
    default = _bench(*extra)
    assert default["config"]["schedule"]["coef_sets"] == (2 if screen == "gain" else 1)


@pytest.mark.gpu
def test_bench_line_carries_parity():
    """The parity object every bench line carries (tools/bench_parity.py):
    the fit of the fixture and of the reference-run synthetic sets, the
    17^2 evaluations and the config-1 / config-2 cubes (made here, the FITS
    legs being off) against the reference's own outputs -- all ok, and the
    process exits 0."""
    line = _bench("--parity")
    par = line["parity"]
    assert par["all_ok"], par
    for k in ("fit_config2", "fit_synth20", "fit_synth50", "eval17", "config1", "config2",
              "fit_amplitude_gain12", "fit_tec14", "gain_cube"):
        assert par[k]["ok"], (k, par[k])
    assert par["fit_synth20"]["orders_equal"] and par["fit_synth50"]["flags_equal"]
    assert par["config1"]["screens_png"]["mismatched_tessellated"] == 0
    assert par["config2"]["cube_from"].startswith("make_aterm_image")
    assert line["library"]["sha16"]


def _assert_contract(line, steps=3, warmup=1):
    """The driver's bench-line contract: the keys, their types and the
    roofline / cpu_baseline objects (BASELINE.json's metric)."""
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert line["metric"] == base["metric"]
    assert line["value"] > 0 and line["unit"] == "screen-slots/s"
    assert line["n_gpus"] == 1 and line["steps"] == steps and line["warmup"] == warmup
    assert line["ms_per_step"] > 0 and line["higher_is_better"] is True
    assert line["scaling"] in ("weak", "strong") and line["vs_baseline"] is None
    assert isinstance(line["dtype"], str) and line["data"] == "synthetic"
    assert isinstance(line["config"]["workload"], str)
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12 and "traffic" in rf
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "screen-slots/s" and cb["cores"] >= 1
    assert cb["kind"] in ("port", "reference") and cb["sample"]


@pytest.mark.gpu
@pytest.mark.parametrize("screen", ["phase", "gain"])
def test_cpu_baseline_leg_checks_the_fit_on_its_sample(screen):
    """The CPU baseline leg's oracle fits (the sample it times) check the
    GPU's fit of the same slots of the benchmarked workload: orders and
    flags equal, coefficients within 1e-8 -- in the line as
    cpu_baseline.oracle_check and parity.fit_oracle_sample; for gain screens
    also the amplitude fit of whole (freq, station, pol) blocks."""
    extra = ["--screen", "gain"] if screen == "gain" else []
    line = _bench("--cpu-baseline", "--cpu-workers", "4", "--no-cpu-reference-path", *extra)
    chk = line["cpu_baseline"]["oracle_check"]
    assert chk["ok"], chk
    assert chk["slots"] >= 16 and chk["orders_differ"] == 0
    assert line["parity"]["fit_oracle_sample"]["ok"]
    assert "_samples" not in line["cpu_baseline"]
    _assert_contract(line)
    if screen == "gain":
        ach = line["cpu_baseline"]["oracle_amp_check"]
        assert ach["ok"] and ach["blocks"] == 4, ach
        assert line["parity"]["fit_oracle_amplitude_blocks"]["ok"]


@pytest.mark.gpu
def test_tess_cpu_baseline_leg_checks_labels_and_fill():
    """--screen tess with its CPU baseline leg: the oracle's label raster
    equals the product's template and the GPU's fill of a non-reference
    slot equals the oracle's gather to 1 ulp -- parity.tess_oracle_sample."""
    line = _bench("--cpu-baseline", "--screen", "tess")
    oc = line["cpu_baseline"]["oracle_check"]
    assert oc["ok"] and oc["labels_differ"] == 0 and oc["max_ulp"] <= 1, oc
    assert line["parity"]["all_ok"] and line["parity"]["tess_oracle_sample"]["ok"]


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["config3", "config5"])
def test_full_size_workload_fit_and_eval_vs_oracle(workload):
    """Configs 3 and 5 at their FULL per-GPU size (config 3: 64 ant x 100 t
    x 16 f x 20 dir, KL 256^2; config 5: the 64-of-512-station shard, 4000 t
    x 64 f x 50 dir = 16.4 M slots, KL 512^2, integer-digit contraction,
    discard + checksum mode), one timed step each as the bench line runs
    them: the GPU fit of the whole workload against the oracle's fits of the
    CPU baseline's sampled slots (orders and flags bit-equal, coefficients
    <= 1e-8), the sampled slots' evaluation against an fp64 restatement of
    kl_screen.py:444-449 and their streamed checksums."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", workload,
           "--steps", "1", "--warmup", "0", "--no-side-legs", "--no-fits",
           "--no-child-legs", "--no-parity", "--cpu-workers", "8", "--cpu-fit-slots", "16",
           "--cpu-eval-slots", "2", "--no-cpu-reference-path"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    S = {"config3": 64 * 100 * 16, "config5": 64 * 4000 * 64}[workload]
    assert line["config"]["slots_per_gpu"] == S
    chk = line["cpu_baseline"]["oracle_check"]
    assert chk["ok"] and chk["orders_differ"] == 0 and chk["slots"] >= 64, chk
    s = line["check"]["sampled_slots"]
    assert s["ok"], s
    if workload == "config5":
        assert s.get("checksums_match") is True
        assert line["dtype"].startswith("i8-digit")

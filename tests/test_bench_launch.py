"""``bench.py --gpus N`` without a launcher starts its own N ranks (CPU).

The driver runs ``python bench.py --gpus N`` at N = 1 and, for the scaling
curve, N = 2 / 4 / 8; torchrun sets WORLD_SIZE for the ranks, a bare command
does not.  bench.py then spawns N child interpreters with the torchrun
environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT),
forwards rank 0's JSON line and fails when any rank fails.  These tests run
the launcher with ``--rehearse-cpu`` (gloo, the shard setup and its
collectives, no kernels) on the tiny workload: the reference's counterpart is
its worker fan-out, stationscreen.py:1056-1077.
"""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*extra, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1")
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *extra],
                          cwd=REPO, env=env, capture_output=True, text=True,
                          timeout=timeout)


def one_line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_ranks(n):
    p = run_bench("--gpus", str(n), "--dist-backend", "gloo", "--workload", "tiny",
                  "--rehearse-cpu")
    assert p.returncode == 0, p.stderr[-2000:]
    line = one_line(p)
    d = line["dist"]
    assert line["n_gpus"] == n and d["world"] == n and d["backend"] == "gloo"
    assert len(d["per_rank"]) == n and len(d["devices"]) == n
    assert [r["rank"] for r in d["per_rank"]] == list(range(n))
    # contiguous antenna shards covering the 80-station array
    spans = [tuple(r["ant"]) for r in d["per_rank"]]
    assert spans[0][0] == 0 and spans[-1][1] == 80
    assert all(spans[k][1] == spans[k + 1][0] for k in range(n - 1))
    # every rank received the same broadcast setup ...
    assert len({r["setup_sha16"] for r in d["per_rank"]}) == 1
    # ... and the same station orders as the unsharded run (max over ranks)
    one = one_line(run_bench("--gpus", "1", "--dist-backend", "gloo", "--workload",
                             "tiny", "--rehearse-cpu"))
    whole = one["dist"]["per_rank"][0]
    assert sum((r["st_order"] for r in d["per_rank"]), []) == whole["st_order"]
    assert d["per_rank"][0]["setup_sha16"] == whole["setup_sha16"]


def test_self_launch_fails_when_a_rank_fails():
    """A rank that exits non-zero (here every rank refuses --rehearse-cpu
    under nccl) makes the launcher exit non-zero with no JSON line."""
    p = run_bench("--gpus", "2", "--dist-backend", "nccl", "--workload", "tiny",
                  "--rehearse-cpu")
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "self-launched job failed" in p.stderr


def test_self_launch_timeout_kills_ranks():
    p = run_bench("--gpus", "2", "--dist-backend", "gloo", "--workload", "tiny",
                  "--rehearse-cpu", "--launch-timeout", "0.05", timeout=60)
    assert p.returncode != 0
    assert "timed out" in p.stderr


def test_world_size_mismatch_still_refused():
    """Under a launcher (WORLD_SIZE set) --gpus must match it."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--rehearse-cpu", "--dist-backend", "gloo"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_force_dist_one_rank_without_launcher():
    """--force-dist at N = 1 with no launcher: a one-rank env:// group, the
    setup collectives run through it (on the GPU box: RCCL)."""
    p = run_bench("--gpus", "1", "--dist-backend", "gloo", "--workload", "tiny",
                  "--rehearse-cpu", "--force-dist")
    assert p.returncode == 0, p.stderr[-2000:]
    # (one process, no launcher to filter its stdout: gloo's own peer
    # message shares it with the JSON line)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])["dist"]
    assert d["backend"] == "gloo" and d["world"] == 1 and len(d["per_rank"]) == 1


def test_power_sampler_reads_hwmon_file(tmp_path):
    """bench.PowerSampler on an hwmon-style file (microwatts): mean board
    power over the sampled window and joules per output byte."""
    import time
    sys.path.insert(0, REPO)
    import bench
    f = tmp_path / "power1_average"
    f.write_text("1250000000\n")                  # 1250 W
    (tmp_path / "freq1_input").write_text("2100000000\n")  # sclk 2.1 GHz
    s = bench.PowerSampler(None, path=str(f))
    with s:
        time.sleep(1.3)
    out = s.summary(out_bytes=6.25e12, seconds=1.0)
    assert out["board_W_mean"] == pytest.approx(1250.0)
    assert out["samples"] >= bench.PowerSampler.MIN_SAMPLES
    assert out["pJ_per_output_byte"] == pytest.approx(200.0)
    assert out["sclk_MHz_mean"] == pytest.approx(2100.0)
    # a run too short for the lagging sensor: no power object
    short = bench.PowerSampler(None, path=str(f))
    with short:
        time.sleep(0.2)
    assert short.summary(1.0, 1.0) is None
    # nothing sampled (never entered): no power object in the line
    assert bench.PowerSampler(None).summary(1.0, 1.0) is None


def test_schedule_is_the_same_at_every_world_size():
    """The driver divides the N = 8 line's rate by the N = 1 line's: both
    must run the same per-GPU schedule (time chunks, coefficient sets, CU
    reservation).  bench.pick_schedule takes no world size; the rehearsal
    line reports what every N would run."""
    lines = {}
    for n in (1, 8):
        p = run_bench("--gpus", str(n), "--dist-backend", "gloo", "--workload", "tiny",
                      "--rehearse-cpu", "--steps", "20")
        assert p.returncode == 0, p.stderr[-2000:]
        lines[n] = one_line(p)
    s1, s8 = lines[1]["config"]["schedule"], lines[8]["config"]["schedule"]
    assert s1 == s8
    assert s1["coef_sets"] == 1 and s1["time_chunks"] == 1
    # the N = 8 line: its parity object holds (every
    # rank's setup = the unsharded run's, station orders concatenate to
    # it, the rank identities pass the nccl one-card check), one per_rank
    # entry per rank, eight distinct device identities
    l8 = lines[8]
    assert l8["parity"]["all_ok"] is True
    assert l8["parity"]["shard_setup"]["ranks"] == 8
    assert l8["parity"]["shard_setup"]["every_rank_equal"]
    assert l8["parity"]["shard_setup"]["station_orders_equal"]
    d = l8["dist"]
    assert [r["rank"] for r in d["per_rank"]] == list(range(8))
    assert len({dv["pci"] for dv in d["devices"]}) == 8 == d["distinct_devices"]
    assert d["nccl_distinct_check"]["ok"] is True
    assert lines[1]["parity"]["all_ok"] is True


def test_child_leg_parity_fails_on_a_broken_leg():
    """a child leg launched with its oracle sample that errored,
    timed out or came back without the sample fails the line's parity
    (bench.child_leg_parity); legs that passed, or did not run, do not."""
    sys.path.insert(0, REPO)
    import bench
    ok = {"max_err": 1e-12, "tol": 1e-8, "ok": True, "slots": 128}
    good = {"config5": {"oracle_requested": True, "oracle_check": dict(ok)},
            "gain_config3": {"oracle_requested": True, "oracle_check": dict(ok),
                             "oracle_amp_check": dict(ok, coef_max_abs_err=1e-13)},
            "tess_config3": {"oracle_requested": True, "oracle_check": dict(ok)}}
    line = {"parity": {"all_ok": True}}
    assert bench.child_leg_parity(good, line) is False
    assert line["parity"]["all_ok"] and len(line["parity"]) == 5
    for broken in ({"error": "exit 134: abort", "oracle_requested": True},
                   {"error": "timed out after 900 s", "oracle_requested": True},
                   {"oracle_requested": True, "value": 1.0}):
        side = dict(good, config5=broken)
        line = {"parity": {"all_ok": True}}
        assert bench.child_leg_parity(side, line) is True
        assert line["parity"]["all_ok"] is False
        assert line["parity"]["fit_oracle_sample_config5"]["ok"] is False
    # a gain leg without its amplitude-block sample
    side = dict(good, gain_config3={"oracle_requested": True, "oracle_check": dict(ok)})
    line = {"parity": {"all_ok": True}}
    assert bench.child_leg_parity(side, line) is True
    # a leg that did not run is not a failure
    line = {"parity": {"all_ok": True}}
    assert bench.child_leg_parity({"config5": good["config5"]}, line) is False


def test_pick_schedule_defaults():
    """Phase screens: one chunk, one coefficient set (at any N); gain: two
    sets over a multi-step run (fit of step k+1 beside the eval of step k)."""
    import argparse
    sys.path.insert(0, REPO)
    import bench
    base = dict(chunks=1, coef_sets=-1, reserve_cus=-1, fit_on_reserved=-1,
                fit_priority=1, steps=20, screen="phase")
    s = bench.pick_schedule(argparse.Namespace(**base), 20, 1000)
    assert (s["time_chunks"], s["coef_sets"], s["pipelined"]) == (1, 1, False)
    g = bench.pick_schedule(argparse.Namespace(**dict(base, screen="gain")), 20, 100)
    assert (g["time_chunks"], g["coef_sets"], g["pipelined"]) == (1, 2, True)
    assert g["reserve_cus"] == 0
    c = bench.pick_schedule(argparse.Namespace(**dict(base, chunks=4)), 20, 100)
    assert (c["time_chunks"], c["reserve_cus"], c["fit_on_reserved"]) == (4, 16, True)


def test_profile_tables_report_only_the_loaded_library(tmp_path, monkeypatch):
    """bench._profile_entry hands out a PMC table entry only when its
    library_sha16 is the library this process loads; an entry taken on
    another build (or with no identity, as before round 5) is withheld and
    named in STALE_COUNTERS."""
    import json as _json
    sys.path.insert(0, REPO)
    import bench
    from ska_sdp_screen_fitting_amd import _lib
    (tmp_path / "profiles").mkdir()
    tab = {"entries": [
        {"workload": "config4", "eval_kernel": "k", "library_sha16": "aaaa", "v": 1},
        {"workload": "config5", "eval_kernel": "k", "library_sha16": "bbbb", "v": 2},
        {"workload": "config3", "eval_kernel": "k", "v": 3}]}
    (tmp_path / "profiles" / "t.json").write_text(_json.dumps(tab))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(_lib, "library_identity", lambda path=None: {"sha16": "aaaa", "bytes": 1})
    bench.STALE_COUNTERS.clear()
    assert bench._profile_entry("t.json", "config4", "k")["v"] == 1
    assert bench._profile_entry("t.json", "config5", "k") is None
    assert bench._profile_entry("t.json", "config3", "k") is None
    assert bench._profile_entry("t.json", "config9", "k") is None
    assert bench.STALE_COUNTERS == {"t.json:config5:k": "bbbb", "t.json:config3:k": None}


def test_committed_tables_carry_library_identity():
    """Every entry the default line and its legs look up (config 4, config 5,
    config-3 gain) carries the identity of the library it was taken on, and
    the fit entries carry trace durations."""
    import json as _json
    for name in ("traffic.json", "mfma.json", "fit_flops.json"):
        tab = _json.load(open(os.path.join(REPO, "profiles", name)))
        keyed = {e["workload"]: e for e in tab["entries"] if e.get("library_sha16")}
        for w in ("config4", "config5", "config3-gain"):
            assert w in keyed, (name, w)
        if name == "fit_flops.json":
            for w in ("config4", "config5", "config3-gain"):
                ks = keyed[w]["kernels"]
                assert ks["kl_fit_pass_kernel"]["avg_ms"] is not None


def test_oracle_sample_check_flags_mismatches():
    """bench._oracle_sample_check (the CPU baseline leg's oracle fits as the
    checker of the GPU's fit of the same slots): equal outputs pass; a
    changed order, a changed flag or a coefficient off by more than the
    tolerance at a well-conditioned slot fail."""
    import numpy as np

    import bench
    from oracle import kl as okl
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions

    T, F, A, D = 6, 1, 3, 8
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D)
    pp = geometry.piercepoints(s.dir_radec)[0]
    basis = okl.Basis(pp)
    coef = np.zeros((T, F, A, D))
    w_out = s.weight.astype(np.float32).copy()
    order_out = np.zeros((T, F, A), np.int32)
    samples = []
    for a in (1, 2):
        ts = np.arange(T)
        res = [okl.fit_slot(s.val[t, 0, a] - s.val[t, 0, 0], s.weight[t, 0, a], 4, 4, basis)
               for t in ts]
        wh = [r[0] for r in res]
        wo = np.array([r[2] for r in res], np.float32)
        od = np.array([r[3] for r in res])
        coef[ts, 0, a] = wh
        w_out[ts, 0, a] = wo
        order_out[ts, 0, a] = od
        samples.append(((ts, 0, a), (wh, wo, od)))
    def gpu(c, w, o):
        return [(c[ts, f, a], w[ts, f, a], o[ts, f, a]) for (ts, f, a), _ in samples]

    ok = bench._oracle_sample_check(samples, gpu(coef, w_out, order_out), pp)
    assert ok["ok"] and ok["slots"] == 2 * T and ok["coef_max_abs_err"] == 0.0
    bad = order_out.copy()
    bad[2, 0, 1] += 1
    assert not bench._oracle_sample_check(samples, gpu(coef, w_out, bad), pp)["ok"]
    badw = w_out.copy()
    badw[3, 0, 2, 0] = 0.0 if badw[3, 0, 2, 0] > 0 else 1.0
    assert not bench._oracle_sample_check(samples, gpu(coef, badw, order_out), pp)["ok"]
    badc = coef.copy()
    badc[1, 0, 2, 3] += 1e-3
    r = bench._oracle_sample_check(samples, gpu(badc, w_out, order_out), pp)
    assert not r["ok"] and r["slots_over_tol"] == 1 and r["over_tol_unexplained"] == 1


def test_baseline_sample_is_the_cpu_baselines_sample():
    """bench.baseline_sample (taken before the parity legs to snapshot the
    GPU's outputs) picks the same slots cpu_baseline fits: deterministic,
    never the reference station, one station and freq per worker."""
    import numpy as np

    import bench
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions

    s = make_solutions(n_ant=5, n_time=9, n_freq=2, n_dir=4)
    setup = {"ref_ant": 1}
    a = bench.baseline_sample(s, setup, 6, slots_fit=4)
    b = bench.baseline_sample(s, setup, 6, slots_fit=4)
    assert len(a) == 6
    for (ts, f, st), (ts2, f2, st2) in zip(a, b):
        assert np.array_equal(ts, ts2) and f == f2 and st == st2
        assert st != 1 and len(set(ts.tolist())) == 4 and f in (0, 1)


def test_oracle_amp_check_flags_mismatches():
    """bench._oracle_amp_check (gain screens: the oracle's amplitude fit of
    whole (freq, station, pol) blocks vs the GPU's): the oracle's own
    outputs pass; a changed order or a coefficient off by 1e-6 fail."""
    import numpy as np

    import bench
    from oracle import kl as okl
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_amplitudes, make_solutions

    T, F, A, D = 8, 2, 4, 6
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D)
    make_amplitudes(s)
    pp = geometry.piercepoints(s.dir_radec)[0]
    basis = okl.Basis(pp)
    order = 3
    blocks = bench.amp_blocks(s, 3)
    gpu = []
    for f, a, p in blocks:
        wh, _, wo, od = okl.process_station_block(
            s.amp_val[:, f, a, :, p].T, s.meta["amp_weight"][:, f, a, :, p].T, order,
            basis, "amplitude", 3, 5.0, True)
        gpu.append((wh.T.copy(), wo.T.copy(), od.astype(np.int32)))
    ok = bench._oracle_amp_check(blocks, gpu, s, pp, order)
    assert ok["ok"] and ok["slots"] == 3 * T, ok
    bad = [(c, w, o.copy()) for c, w, o in gpu]
    bad[1][2][0] += 1
    assert not bench._oracle_amp_check(blocks, bad, s, pp, order)["ok"]
    badc = [(c.copy(), w, o) for c, w, o in gpu]
    badc[2][0][3, 1] += 1e-6
    assert not bench._oracle_amp_check(blocks, badc, s, pp, order)["ok"]


def test_tess_cpu_baseline_checks_labels_and_fill():
    """bench.tess_cpu_baseline (--screen tess): the oracle's label raster
    and gather as the checker of the product's template and of the GPU's
    slot-0 fill -- equal inputs pass, one changed label or a fill off by
    more than 1 ulp fail."""
    import numpy as np
    import torch

    import bench
    from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG, FIELD_RA_DEG,
                                                      FIELD_WIDTH_DEG, make_solutions)
    from ska_sdp_screen_fitting_amd.voronoi_screen import tessellation_template

    cell = 0.2
    s = make_solutions(n_ant=3, n_time=1, n_freq=1, n_dir=6)
    setup = {"ref_phase": torch.from_numpy(np.ascontiguousarray(s.val[:, :, 0, :]))}
    lab, _ = tessellation_template(np.rad2deg(s.dir_radec.astype(np.float64)),
                                   FIELD_RA_DEG, FIELD_DEC_DEG, FIELD_WIDTH_DEG, cell)
    p0 = s.val[0, 0, 1] - s.val[0, 0, 0]  # station 1, referenced to station 0
    slot0 = np.stack([np.cos(p0), np.sin(p0), np.cos(p0), np.sin(p0)]).astype(np.float32)
    slot0 = slot0[:, lab - 1]
    r = bench.tess_cpu_baseline(s, setup, cell, lab, slot0, slot=1)
    assert r["oracle_check"]["ok"], r
    bad = lab.copy()
    bad[3, 4] = bad[3, 4] % 6 + 1
    assert not bench.tess_cpu_baseline(s, setup, cell, bad, slot0, slot=1)["oracle_check"]["ok"]
    off = slot0.copy()
    off[1, 2, 2] = np.nextafter(np.nextafter(off[1, 2, 2], 9.0, dtype=np.float32), 9.0,
                                dtype=np.float32)
    r = bench.tess_cpu_baseline(s, setup, cell, lab, off, slot=1)
    assert r["oracle_check"]["max_ulp"] == 2 and not r["oracle_check"]["ok"]

#!/usr/bin/env python3
"""Benchmark of the KL screen hot path on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic input, on
every GPU: the batched KL fit of all of the rank's slots (``sf_kl_fit``)
followed by the KL pixel evaluation of all of them (``sf_kl_eval``) into an
HBM ring of output cubes.  Default workload = BASELINE.json configs[3], the
config the north_star's targets are quoted on: 256 ant x 1000 time x 32 freq
x 20 dir, KL 256^2 screen, the antenna axis split over the --gpus N ranks
(strong scaling; 8.19 M slots per step in total, discard + checksum mode).
``--workload config3`` is configs[2] per GPU (weak scaling), ``config5``
configs[4]'s per-GPU shard.  Only one-shot setup collectives.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import socket
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))

METRIC = ("screen-slots/sec (ant×time×freq) + FITS-cube wall-clock, "
          "KL 256² screen")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

WORKLOADS = {
    # name: (ant per GPU, times, freqs, dirs, grid side, cellsize)
    "config3": (64, 100, 16, 20, 256, 0.01301),
    "config2-shape": (62, 20, 12, 7, 128, 0.02602),
    "config5-shape": (64, 100, 4, 50, 512, 0.006505),
    # BASELINE.json configs[3]: the whole 256-ant array, sharded over the
    # ranks (strong scaling); D = 20 as config 3
    "config4": (256, 1000, 32, 20, 256, 0.01301),
    # BASELINE.json configs[4] (SKA-Low scale): 64 of its 512 stations per
    # GPU, so --gpus 8 is the whole 512 ant x 4000 t x 64 f x 50 dir array
    "config5": (64, 4000, 64, 50, 512, 0.006505),
    # launcher / collective rehearsals (tests): 80 stations (rank 0 holds
    # the first 10 up to N = 8, as the reference-station choice needs), 32^2
    "tiny": (80, 4, 2, 7, 32, 0.10407),
}
STRONG = {"config4", "tiny"}  # first field = stations of the whole job


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="config4", choices=sorted(WORKLOADS))
    ap.add_argument("--ring-gb", type=float, default=16.0,
                    help="HBM ring for the output cubes (GiB)")
    ap.add_argument("--precise-sincos", action="store_true",
                    help="fp64 sincos epilogue (default: exact fp64 reduction "
                         "of the phase in revolutions + hardware fp32 sincos, "
                         "|err| <= 2.3e-7)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fits", action="store_true",
                    help="skip the FITS-cube wall-clock legs (configs 1-3)")
    ap.add_argument("--no-fits-config3", action="store_true",
                    help="skip only the config-3 (107 GB, KL 256^2) FITS leg")
    ap.add_argument("--cpu-fit-slots", type=int, default=64,
                    help="CPU baseline: fit slots per worker (its oracle fits "
                         "also check the GPU's fit of the same slots)")
    ap.add_argument("--cpu-eval-slots", type=int, default=192,
                    help="CPU baseline: evaluated slots per worker")
    ap.add_argument("--no-cpu-reference-path", action="store_true",
                    help="CPU baseline without the one-core make_aterm_image "
                         "legs of configs 1 / 2")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="CPU baseline pool size; 0 (default): this GPU's "
                         "share of the host (affinity / GPUs per node, capped "
                         "by OMP_NUM_THREADS), see cpu_share()")
    ap.add_argument("--no-side-legs", action="store_true",
                    help="skip the untimed side measurements (fp64-sincos "
                         "eval, fit alone on the whole chip)")
    ap.add_argument("--chunks", type=int, default=1,
                    help="time chunks per step: the fit of chunk c+1 runs on a "
                         "second stream while chunk c is evaluated; 1 "
                         "(default) = fit then eval on the whole chip.  The "
                         "fit is 3 %% (config 4) / 8 %% (config 5) of the eval "
                         "and takes SIMD and CU time from it when overlapped: "
                         "serial config 4 5.92 M slots/s vs 5.81 pipelined "
                         "(profiles/round2t_schedule_ab.txt)")
    ap.add_argument("--coef-sets", type=int, default=-1, choices=(-1, 1, 2),
                    help="coefficient buffers: 2 = the fit of step k+1 writes "
                         "a second set while step k is evaluated (fit || eval "
                         "across steps on two streams, as a caller streaming "
                         "successive solution blocks would run it; the only "
                         "overlap open to gain screens, whose amplitude fit "
                         "sees every time at once); -1 (default): 2 for a "
                         "multi-step gain run (config-3 gain +16 %%), else 1 "
                         "-- at every --gpus N, so the driver's 1 -> 8 curve "
                         "divides like by like (config 4: one or two sets "
                         "measured within 1.9 %%, profiles/round4n_coef_sets_ab.txt)")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="compute units the eval stream leaves to the fit "
                         "stream (pipelined mode); -1 (default): 16 with "
                         "--chunks > 1 and D <= 32 (the fit then runs on "
                         "exactly those), else 0 (with two coefficient sets "
                         "and one chunk, 16 reserved CUs cost gain 40 %%) "
                         "(at D = 50 the eval is compute-bound and the fit "
                         "too heavy for 16 CUs: config 5 +8 %%)")
    ap.add_argument("--fit-on-reserved", type=int, default=-1,
                    help="1: confine the fit stream to the reserved CUs "
                         "(pipelined mode); -1 (default): when D <= 32, where "
                         "the fit of a chunk on the reserved CUs is shorter "
                         "than the evaluation of the previous one")
    ap.add_argument("--fit-priority", type=int, default=1,
                    help="1: fit stream at high priority (pipelined mode)")
    ap.add_argument("--eval-xcd-map", type=int, default=-1,
                    help="SF_OPT_EVAL_XCD_MAP: -1 auto (default), 0 contiguous "
                         "pixel blocks per XCD, 1 interleaved")
    ap.add_argument("--eval-int", type=int, default=-1, choices=(-1, 0),
                    help="SF_OPT_EVAL_INT: -1 the integer-digit contraction where "
                         "it applies (phase screens, D >= 45), 0 fp64 MFMAs")
    ap.add_argument("--eval-groups", type=int, default=0,
                    help="SF_OPT_EVAL_GROUPS: most 16-slot groups per eval work "
                         "item (0 = library default)")
    ap.add_argument("--eval-kernel", type=int, default=0,
                    help="SF_OPT_EVAL_KERNEL: 0 auto (default), else one of "
                         "SF_EVAL_KERNEL_* (A/B runs)")
    ap.add_argument("--eval-bands", type=int, default=0,
                    help="SF_OPT_EVAL_BANDS: pixel bands of an eval launch "
                         "(0 = library default)")
    ap.add_argument("--eval-sleep", type=int, default=0,
                    help="SF_OPT_EVAL_SLEEP: LDS-staged eval waves sleep n x 64 "
                         "cycles before each group's barrier (diagnostic)")
    ap.add_argument("--checksum", default="auto", choices=("auto", "on", "off"),
                    help="per-slot output checksums (sf_kl_eval_sums); auto: on "
                         "for config4 / config5, whose cubes are discarded")
    ap.add_argument("--tess-slots", type=int, default=0,
                    help="SF_OPT_TESS_SLOTS: slots per work item of the "
                         "unsmoothed tessellated fill (0 = library default)")
    ap.add_argument("--tess-waves", type=int, default=0,
                    help="SF_OPT_TESS_WAVES: waves per workgroup of the "
                         "unsmoothed tessellated fill (0 = library default)")
    ap.add_argument("--tess-box", type=int, default=-1, choices=(-1, 0, 1),
                    help="SF_OPT_TESS_BOX: smoothed tessellated fill by interior "
                         "lookups (1), by the wide-tile kernel (0) or auto (-1)")
    ap.add_argument("--tess-gain", action="store_true",
                    help="--screen tess: XX / YY amplitudes too (four "
                         "distinct planes, A cos / A sin)")
    ap.add_argument("--smooth-pix", type=float, default=0.0,
                    help="--screen tess: Gaussian sigma in pixels (<= 6: "
                         "fused in the fill kernel); 0 = make_aterm_image's "
                         "default smooth_deg = 0")
    ap.add_argument("--screen", default="phase", choices=("phase", "gain", "tess"),
                    help="gain: phase + slow XX / YY amplitude screens "
                         "(kl_screen.py:96-125, 319-378): per step the phase "
                         "fit and the two log10-amplitude fits (niter 3, "
                         "block sigma over all times, so one time chunk), "
                         "then the three-contraction gain evaluation; "
                         "tess: the tessellated (Voronoi) fill of every slot "
                         "(voronoi_screen.py:132-216, sf_tess_fill), no fit")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the parity checks against the reference's golden "
                         "outputs (tools/bench_parity.py; on by default, the "
                         "line exits 3 when one fails)")
    ap.add_argument("--eval-only", action="store_true",
                    help="time only sf_kl_eval (profiling)")
    ap.add_argument("--as-shard-of", type=int, default=0,
                    help="strong workloads, one process: run the shard rank 0 "
                         "of an N-way split would run (per-GPU throughput of "
                         "an N-GPU job measured on one GPU; the line's value is "
                         "then the shard's own slots/s, see 'projection')")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse N ranks on a 1-GPU box (setup "
                         "collectives on the CPU, ranks share the device)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group and run the setup "
                         "collectives even at world size 1 (exercises the "
                         "RCCL path on a one-GPU box)")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="launcher / gloo rehearsal without a GPU: every rank "
                         "runs the shard setup and its collectives, no kernels "
                         "(prints a line with value null)")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="--gpus N without a launcher: seconds before the "
                         "self-launched ranks are killed")
    ap.add_argument("--no-child-legs", "--no-config5-leg", action="store_true",
                    dest="no_child_legs",
                    help="skip the child-process legs of the default N = 1 run "
                         "(config 5, gain and tessellated on the config-3 shape)")
    return ap.parse_args()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"bench[{os.environ.get('RANK', '-')}] {time.strftime('%H:%M:%S')} {msg}",
          file=sys.stderr, flush=True)


# --------------------------------------------------------------------------
# Self-launch: ``python bench.py --gpus N`` without torchrun starts N ranks
# itself (one child interpreter per GPU, the torchrun environment), so the
# command form of the N = 1 run works at every N.  The parent never touches
# the GPU; it forwards the ranks' output (rank 0 prints the JSON line) and
# exits non-zero if any rank fails or the job times out.  The reference's
# counterpart is its worker fan-out over processes, stationscreen.py:1056-1077.
# --------------------------------------------------------------------------
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, timeout_s):
    import signal
    import subprocess

    import tempfile

    port = _free_port()
    procs, outs = [], []
    log(f"launching {n} ranks (MASTER 127.0.0.1:{port})")
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", ROLE_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # a rank's stdout goes to a file: libraries print there too (gloo's
        # peer messages), and only rank 0's JSON line may reach our stdout
        outs.append(tempfile.TemporaryFile(mode="w+"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)]
                                      + sys.argv[1:], env=env, stdout=outs[-1]))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def on_signal(signum, _frame):
        stop()
        raise SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, on_signal)
    t_end = time.time() + timeout_s
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with {bad[0][1]}"
            break
        if all(c == 0 for c in codes):
            break
        if time.time() > t_end:
            failed = f"timed out after {timeout_s:.0f} s"
            break
        time.sleep(0.2)
    if failed:
        log(f"self-launched job failed: {failed}; stopping the other ranks")
        stop()
    for r, fh in enumerate(outs):
        fh.seek(0)
        for ln in fh.read().splitlines():
            if r == 0 and not failed and ln.startswith("{"):
                print(ln, flush=True)
            elif ln.strip():
                print(f"[rank {r} stdout] {ln}", file=sys.stderr, flush=True)
        fh.close()
    return 1 if failed else 0


# --------------------------------------------------------------------------
# CPU baseline: the oracle (numpy fp64 restatement of the reference) on a
# bounded slot sample, in a pool of single-threaded workers.
# --------------------------------------------------------------------------
_BLAS_THREADS = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")


def _cpu_worker(job):
    sys.path.insert(0, REPO)
    from oracle import kl as okl  # test infrastructure: baseline leg only

    (phi, w, order, pp, cpix_args, n_eval) = job
    basis = okl.Basis(pp)
    t0 = time.perf_counter()
    coefs, w_outs, orders = [], [], []
    for k in range(phi.shape[0]):
        white, _, w_o, o, _ = okl.fit_slot(phi[k], w[k], order[k], order[k], basis)
        coefs.append(white)
        w_outs.append(w_o)
        orders.append(o)
    t_fit = time.perf_counter() - t0
    x, y = cpix_args
    cpix = okl.cpix_matrix(pp, x, y)
    t0 = time.perf_counter()
    coefs = np.array(coefs)
    for k in range(n_eval):
        ph = okl.eval_phase_screens(coefs[k % len(coefs)][None, :], cpix)
        planes = okl.eval_planes(ph).astype(np.float32)
        del planes
    t_eval = time.perf_counter() - t0
    # the sample's fit outputs go back to the parent as the checker of the
    # GPU's fit of the same slots (_oracle_sample_check)
    return (phi.shape[0], t_fit, n_eval, t_eval,
            (coefs, np.array(w_outs, np.float32), np.array(orders)))


def baseline_sample(sol, setup, n_workers, slots_fit=64):
    """The CPU baseline's fit sample: per worker k, slots_fit random times
    of station k (skipping the reference station) at freq k mod F."""
    T, F, A, _ = sol.val.shape
    ref = setup["ref_ant"]
    rng = np.random.default_rng(1)
    where = []
    for k in range(n_workers):
        a = [a for a in range(A) if a != ref][k % (A - 1)]
        ts = rng.choice(T, size=min(slots_fit, T), replace=False)
        where.append((ts, k % F, a))
    return where


def gpu_sample_outputs(torch, where, coef, w_out, order_out):
    """The GPU fit's outputs at the baseline sample's slots (host copies)."""
    out = []
    for ts, f, a in where:
        ti = torch.as_tensor(ts, device=coef.device)
        out.append((coef[ti, f, a].cpu().numpy(), w_out[ti, f, a].cpu().numpy(),
                    order_out[ti, f, a].cpu().numpy()))
    return out


def amp_blocks(sol, n_blocks=4):
    """Gain screens: the (freq, station, pol) amplitude blocks whose whole
    time series the CPU baseline leg fits with the oracle (the outlier sigma
    couples a block's times, Q6, so a block is the unit)."""
    _, F, A, _ = sol.val.shape
    return [(k % F, (7 * k + 1) % A, k % 2) for k in range(n_blocks)]


def gpu_amp_outputs(blocks, A, stacked, w_out, orders):
    """The GPU amplitude fit's outputs of those blocks (pols stacked along
    the station axis: pol p of station a is column p * A + a)."""
    out = []
    for f, a, p in blocks:
        c = p * A + a
        out.append((stacked[:, f, c].cpu().numpy(), w_out[:, f, c].cpu().numpy(),
                    orders[:, f, c].cpu().numpy()))
    return out


def cpu_baseline(sol, setup, n_workers, rule="", slots_fit=64, slots_eval=192):
    import multiprocessing as mp

    refph = setup["ref_phase"].cpu().numpy()
    jobs = []
    where = baseline_sample(sol, setup, n_workers, slots_fit)
    for ts, f, a in where:
        jobs.append((sol.val[ts, f, a] - refph[ts, f], sol.weight[ts, f, a],
                     [setup["st_order"][a]] * len(ts), setup["piercepoints"],
                     (setup["x"], setup["y"]), slots_eval))
    ctx = mp.get_context("spawn")
    # single-threaded BLAS in every worker: the spawned interpreters read the
    # thread counts from the environment when they import numpy
    saved = {k: os.environ.get(k) for k in _BLAS_THREADS}
    os.environ.update({k: "1" for k in _BLAS_THREADS})
    try:
        t0 = time.perf_counter()
        with ctx.Pool(n_workers) as pool:
            res = pool.map(_cpu_worker, jobs)
        wall = time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    n_fit = sum(r[0] for r in res)
    t_fit = sum(r[1] for r in res)
    n_ev = sum(r[2] for r in res)
    t_ev = sum(r[3] for r in res)
    per_slot = t_fit / n_fit + t_ev / n_ev  # core-seconds per slot (fit + eval)
    P = len(setup["x"]) * len(setup["y"])
    samples = [(wh, r[4]) for wh, r in zip(where, res)]
    # the reference itself, timed during the survey on an 8-vCPU Xeon
    # (SURVEY.md §6): calculate_kl_screen 8.5 us / pixel / slot / core,
    # _fit_screen 68-92 us / slot (unflagged)
    ref_slot_s = 8.5e-6 * P + 80e-6
    return {
        "value": n_workers / per_slot,
        "unit": "screen-slots/s",
        "cores": n_workers,
        "cores_rule": rule,
        "kind": "port",
        "host_cpus": os.cpu_count(),
        "affinity_cpus": _affinity(),
        "sample": (f"oracle (numpy fp64 restatement) on {n_fit} fit slots and "
                   f"{n_ev} {len(setup['x'])}^2 eval slots of the same workload, "
                   f"{n_workers} single-threaded workers, {wall:.1f} s wall; "
                   f"fit {t_fit / n_fit * 1e3:.3f} ms/slot/core, eval "
                   f"{t_ev / n_ev * 1e3:.1f} ms/slot/core"),
        "reference_calibration": {
            "note": ("the reference's own per-slot costs measured in the survey "
                     "(SURVEY.md §6, 8-vCPU Xeon): calculate_kl_screen 8.5 us "
                     "/ pixel / slot / core, _fit_screen ~80 us / slot; its "
                     "Python loop is ~10x slower than this vectorised port"),
            "ref_s_per_slot_core": ref_slot_s,
            "ref_slots_per_s_at_cores": n_workers / ref_slot_s,
        },
        "_samples": samples,
    }


def _oracle_amp_check(blocks, gpu, sol, pp, order):
    """Gain screens: the oracle's amplitude fit (oracle/kl.py
    process_station_block: stationscreen.py:597-782 with the block sigma of
    Q6, niter 3, as KLScreen.fit runs it, kl_screen.py:96-125) of whole
    (freq, station, pol) blocks vs the GPU's stacked-pol fit of the same
    blocks: orders and flags equal, coefficients <= 1e-8 x max(1, |coef|max)."""
    sys.path.insert(0, REPO)
    from oracle import kl as okl  # test infrastructure: the baseline leg's checker

    basis = okl.Basis(pp)
    n = n_ord = n_w = 0
    err_max, scale = 0.0, 1.0
    for g_c, _, _ in gpu:
        scale = max(scale, float(np.nanmax(np.abs(g_c))))
    for (f, a, p), (g_c, g_w, g_o) in zip(blocks, gpu):
        v = sol.amp_val[:, f, a, :, p].T
        w = sol.meta["amp_weight"][:, f, a, :, p].T
        wh, _, wo, od = okl.process_station_block(v, w, order, basis, "amplitude", 3,
                                                  5.0, True)
        n += g_o.shape[0]
        n_ord += int((g_o != od.astype(g_o.dtype)).sum())
        n_w += int((g_w != wo.T).any(axis=-1).sum())
        err_max = max(err_max, float(np.nanmax(np.abs(g_c - wh.T))))
    ok = n_ord == 0 and n_w == 0 and err_max <= 1e-8 * scale
    return {"blocks": len(blocks), "slots": n, "orders_differ": n_ord,
            "weight_rows_differ": n_w, "coef_max_abs_err": err_max,
            "coef_scale": scale, "tol": 1e-8 * scale, "ok": ok,
            "what": "the GPU amplitude fit (stacked pols) vs the oracle's "
                    "process_station_block on whole (freq, station, pol) blocks"}


def _oracle_sample_check(samples, gpu, pp):
    """The CPU baseline's oracle fits (stationscreen.py:597-782 restated,
    oracle/kl.py fit_slot) as the checker of the GPU's fit of the same slots
    of the benchmarked workload (``gpu``: gpu_sample_outputs, taken right
    after the timed steps and side legs, before the parity legs move the
    shared context to other bases): orders and flagged weights bit-equal,
    coefficients <= 1e-8 x max(1, |coef|max) -- the GPU tests' criterion,
    where a slot over it counts as explained only when its order-K normal
    matrix U_k^T W U_k has a singular value <= 1e-3 (the reference's pinv
    cutoff: its own output is chaotic there, tests/test_oracle_golden.py
    ill_conditioned_slots)."""
    sys.path.insert(0, REPO)
    from oracle import kl as okl  # test infrastructure: the baseline leg's checker

    n = n_ord = n_w = 0
    err_max = 0.0
    over = []
    scale = 1.0
    for g_c, _, _ in gpu:
        scale = max(scale, float(np.nanmax(np.abs(g_c))))
    for (_, (wh, wo, od)), (g_c, g_w, g_o) in zip(samples, gpu):
        wh = np.asarray(wh)
        n += len(g_o)
        n_ord += int((g_o != od.astype(g_o.dtype)).sum())
        n_w += int((g_w != wo).sum(axis=-1).astype(bool).sum())
        err = np.abs(g_c - wh).max(axis=-1)
        err_max = max(err_max, float(np.nanmax(err)))
        for k in np.where(~(err <= 1e-8 * scale))[0]:
            over.append((wo[k], int(od[k])))
    basis = okl.Basis(pp)
    unexplained = 0
    for w, o in over:
        unfl = np.where(w > 0)[0]
        _, _, u = okl.calculate_svd(basis.pp[unfl], 100.0, 5.0 / 3.0)
        wd = np.diag(w[unfl].astype(np.float64))
        sv = np.linalg.svd(u[:, :o].T @ (wd @ u)[:, :o], compute_uv=False)
        if o == 0 or sv.min() > 1e-3:
            unexplained += 1
    ok = n_ord == 0 and n_w == 0 and unexplained == 0
    return {"slots": n, "orders_differ": n_ord, "weight_rows_differ": n_w,
            "coef_max_abs_err": err_max, "coef_scale": scale, "tol": 1e-8 * scale,
            "slots_over_tol": len(over), "over_tol_unexplained": unexplained,
            "ok": ok,
            "what": "the GPU fit of the benchmarked workload vs the oracle "
                    "(oracle/kl.py fit_slot, pinned to the reference's outputs) "
                    "on the CPU baseline's sampled slots"}


def tess_cpu_baseline(sol, setup, cell, lab, gpu_slot0, n_slots=64, slot=0):
    """--screen tess, rank 0 at N = 1: the oracle's tessellated path
    (oracle/voronoi.py: label_raster = voronoi_screen.py:218-351 restated
    from the GEOS Polygonizer, gather_planes = voronoi_screen.py:177-214)
    timed on one core for n_slots slots, and as the checker of the product:
    its label raster vs the host template the GPU used, its gather of one
    slot (``slot``: station ``slot`` at time 0, freq 0) vs the GPU's fill of
    it (float32, <= 1 ulp)."""
    sys.path.insert(0, REPO)
    from oracle import voronoi as ov  # test infrastructure: the baseline leg
    from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG, FIELD_RA_DEG,
                                                      FIELD_WIDTH_DEG)

    rd = np.rad2deg(sol.dir_radec.astype(np.float64))
    t0 = time.perf_counter()
    lab_o, _ = ov.label_raster(rd[:, 0], rd[:, 1], FIELD_RA_DEG, FIELD_DEC_DEG,
                               FIELD_WIDTH_DEG, cell)
    t_lab = time.perf_counter() - t0
    A, D = sol.val.shape[2:]
    refph = setup["ref_phase"].cpu().numpy()
    ph = (sol.val[0, 0] - refph[0, 0][None, :])[: max(min(n_slots, A), slot + 1)]
    t0 = time.perf_counter()
    planes = ov.gather_planes(lab_o, ph)
    t_fill = time.perf_counter() - t0
    n = ph.shape[0]
    want = planes[slot]
    ulp = int(np.abs(gpu_slot0.view(np.int32).astype(np.int64)
                     - want.view(np.int32).astype(np.int64)).max())
    labels_differ = int((lab_o != lab).sum())
    ok = labels_differ == 0 and ulp <= 1
    return {
        "value": n / t_fill, "unit": "screen-slots/s", "cores": 1, "kind": "port",
        "sample": (f"oracle gather_planes of {n} slots ({lab.shape[0]}^2, D = {D}) on "
                   f"one core, {t_fill:.2f} s; its label raster {t_lab:.2f} s"),
        "oracle_check": {"labels_differ": labels_differ, "max_ulp": ulp, "slots": 1,
                         "max_err": float(ulp), "tol": 1.0, "ok": ok,
                         "what": "the product's label template vs the oracle's "
                                 "(GEOS-convention rings), and the GPU fill of "
                                 f"slot {slot} (station {slot}, time 0, freq 0) "
                                 "vs the oracle's gather"},
    }


def _affinity():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count()


def _node_gpus():
    """GPUs of the node (not just the ones this process sees): KFD topology
    nodes with a non-zero gfx_target_version; 8 (an MI355X node) when the
    topology is not readable."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for d in os.listdir(root):
            try:
                txt = open(os.path.join(root, d, "properties")).read()
            except OSError:
                continue
            for ln in txt.splitlines():
                k, _, v = ln.partition(" ")
                if k == "gfx_target_version" and v.strip() not in ("", "0"):
                    n += 1
    except OSError:
        pass
    return n or 8


def cpu_share():
    """CPU-baseline pool size: this GPU's share of the host's cores = the
    CPUs this process may run on / the node's GPUs, capped by
    OMP_NUM_THREADS when the job sets it (the GPU box grants 16 host threads
    per GPU that way).  Returns (workers, rule)."""
    aff = _affinity() or 1
    gpus = _node_gpus()
    share = max(1, aff // gpus)
    rule = f"affinity {aff} CPUs / {gpus} GPUs per node = {share}"
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < share:
        share = int(omp)
        rule += f", capped by OMP_NUM_THREADS={omp} (the job's per-GPU CPU grant)"
    return share, rule


def file_write_ceiling(outdir, nbytes, block=1 << 30):
    """The box's file-write rate where the FITS legs write: ``nbytes`` of one
    pre-filled buffer written in ``block`` pieces by plain ``write`` calls
    (what the FITS writer does), then closed; the unlink timed apart."""
    buf = memoryview(np.full(block, 0x3F, np.uint8))
    path = os.path.join(outdir, "write_ceiling.bin")
    t0 = time.perf_counter()
    with open(path, "wb") as fh:
        left = nbytes
        while left > 0:
            fh.write(buf[:min(block, left)])
            left -= block
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    os.remove(path)
    return {"bytes": nbytes, "wall_s": dt, "GB_per_s": nbytes / dt / 1e9,
            "unlink_s": time.perf_counter() - t1,
            "what": "plain write() of one buffer in 1 GiB pieces, same directory"}


def fits_wallclock(config3=True, kept=None):
    """FITS-cube wall-clock of make_aterm_image (the second half of the
    BASELINE.json metric; fit + evaluation + FITS write, host I/O included):

    * config 1 (tessellated 17^2, smooth 0.1 deg) and config 2 (KL 128^2) on
      the reference fixture, best of two runs (the second with the device
      context warm);
    * config 3, the KL 256^2 cube of 64 ant x 100 t x 16 f x 20 dir (107.4 GB,
      synthetic solutions): one run, written as the reference writes a cube
      larger than memory -- one FITS file per time chunk (screen.py:283-317) --
      10 times (10.7 GB) per file, each file deleted when closed (the box has
      less disk than the cube); the unlink time is reported apart, and the
      box's plain file-write rate over one chunk's bytes is measured in the
      same directory right after.

    ``kept``: a dict that receives {config1 / config2: TemporaryDirectory}
    holding the first run's cube, for the parity checks (the caller cleans
    them up)."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import fits_wallclock as fw
    res = {}
    for name in ("config1", "config2"):
        best = None
        for k in range(2):
            if k == 0 and kept is not None:
                kept[name] = tempfile.TemporaryDirectory()
                r = fw.run(name, kept[name].name)
            else:
                with tempfile.TemporaryDirectory() as d:
                    r = fw.run(name, d)
            best = r if best is None or r["wall_s"] < best["wall_s"] else best
        res[name] = {"wall_s": best["wall_s"], "fits_bytes": best["fits_bytes"],
                     "screen_type": best["screen_type"],
                     "grid": 17 if name == "config1" else 128,
                     "slots": best["slots"], "slots_per_s": best["slots_per_s"],
                     "fits_GB_per_s": best["fits_GB_per_s"]}
    if config3:
        with tempfile.TemporaryDirectory() as src:
            h5, slots = fw.synthetic_npz("config3", src)
            with tempfile.TemporaryDirectory() as d:
                r = fw.run("config3", d, h5, slots)
                ceil = file_write_ceiling(d, r["fits_bytes"] // r["files"])
        res["config3"] = {
            "screen_type": "kl", "grid": 256, "slots": slots,
            "wall_s": r["wall_s"], "unlink_s": r["unlink_s"],
            "wall_s_without_unlink": r["wall_s_without_unlink"],
            "fits_bytes": r["fits_bytes"], "files": r["files"],
            "fits_GB_per_s": r["fits_GB_per_s"],
            "fits_GB_per_s_without_unlink": r["fits_GB_per_s_without_unlink"],
            "slots_per_s": slots / r["wall_s"],
            "file_write_ceiling": ceil,
            "frac_of_file_write_ceiling":
                r["fits_GB_per_s_without_unlink"] / ceil["GB_per_s"],
            "what": ("make_aterm_image(screen_type='kl', cellsize_deg=0.01301) "
                     "on synthetic 64 ant x 100 t x 16 f x 20 dir solutions: "
                     "fit + eval + big-endian FITS, 10 time-chunk files of "
                     "10.7 GB, each deleted after close")}
    return res


def cpu_reference_path(cases=("config1", "config2")):
    """BASELINE.json configs[0] / [1] on the CPU, one core (``ncpu=1``): the
    oracle's make_aterm_image path (oracle/pipeline.py: fit, evaluation or
    Voronoi gather + smoothing, FITS write) on the reference fixture, each in
    a child process pinned to one CPU with single-threaded BLAS.  Beside it
    the reference's own timings on the same fixture measured in the survey
    (SURVEY.md §6, 8-vCPU Xeon, ncpu=1)."""
    import subprocess
    import tempfile
    cpu = sorted(os.sched_getaffinity(0))[-1] if hasattr(os, "sched_getaffinity") else 0
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1",
               MKL_NUM_THREADS="1", SF_PIN_CPU=str(cpu))
    # survey: VoronoiScreen.write 1.40 s (17^2, smooth 0.5 px);
    # stationscreen.run 2.80 s + calculate_kl_screen 8.5 us / pixel / slot
    ref_s = {"config1": 1.40, "config2": 2.80 + 8.5e-6 * 128 * 128 * 14880}
    res = {}
    for case in cases:
        with tempfile.TemporaryDirectory() as d:
            p = subprocess.run([sys.executable, "-m", "oracle.pipeline", case, d],
                               cwd=REPO, env=env, capture_output=True, text=True,
                               timeout=300)
        if p.returncode != 0:
            res[case] = {"error": p.stderr[-400:]}
            continue
        r = json.loads(p.stdout.strip().splitlines()[-1])
        r["slots_per_s"] = r["slots"] / r["wall_s"]
        r["cores"] = 1
        r["kind"] = "port"
        r["reference_calibration_s"] = ref_s[case]
        r["reference_calibration_note"] = (
            "survey measurement of the reference itself, ncpu=1 (SURVEY.md §6): "
            + ("VoronoiScreen.write, 17^2, smooth 0.5 px" if case == "config1" else
               "stationscreen.run 2.80 s + calculate_kl_screen at 8.5 us / pixel "
               "/ slot x 128^2 x 14,880 slots (extrapolated from its 17^2 run)"))
        res[case] = r
    return res


def sampled_slots_check(ctx, torch, dev, setup, coef, N, flags, slot_sums,
                        n_evals, fast, cxx=None, cyy=None):
    """Parity of sampled slots of the timed run (not timed): slots 0, S/2 and
    S-1 evaluated alone vs an fp64 torch restatement of kl_screen.py:444-449
    (|d| <= 2e-6 with the fast sincos epilogue, 1e-6 with fp64), and -- in
    checksum mode -- their cube checksums vs the per-slot sums the streamed
    launches accumulated (n_evals identical evaluations of each slot)."""
    D = coef.shape[1]
    P = N * N
    pp = torch.as_tensor(setup["piercepoints"], dtype=torch.float64, device=dev)
    xs = torch.as_tensor(setup["x"], dtype=torch.float64, device=dev)
    ys = torch.as_tensor(setup["y"], dtype=torch.float64, device=dev)
    d2 = ((pp[:, 0][None, None, :] - xs[None, :, None]) ** 2
          + (pp[:, 1][None, None, :] - ys[:, None, None]) ** 2) + pp[:, 2] ** 2
    cpix = (-((d2 / 100.0 ** 2) ** (5.0 / 6.0)) / 2.0).reshape(P, D)
    del d2
    one = torch.empty((1, 4, N, N), dtype=torch.float32, device=dev)
    S = coef.shape[0]
    err, sums_ok, slots = 0.0, True, sorted({0, S // 2, S - 1})
    for k in slots:
        if cxx is None:
            ctx.eval(coef[k:k + 1], 1, one, 1, flags)
        else:
            ctx.eval_gain(coef[k:k + 1], cxx[k:k + 1], cyy[k:k + 1], 1, one, 1, flags)
        torch.cuda.synchronize(dev)
        ph = cpix @ coef[k]
        c, s = torch.cos(ph), torch.sin(ph)
        if cxx is None:
            want = torch.stack([c, s, c, s])
            scale = torch.ones_like(want)
        else:  # kl_screen.py:338-378: 10 ** screen x cos / sin
            ax, ay = 10.0 ** (cpix @ cxx[k]), 10.0 ** (cpix @ cyy[k])
            want = torch.stack([ax * c, ax * s, ay * c, ay * s])
            # gain tolerance relative to max(1, amplitude) (tests/test_gain.py)
            scale = torch.clamp(torch.stack([ax, ax, ay, ay]), min=1.0)
        got = one[0].reshape(4, P).double()
        live = ~torch.isnan(ph)  # NaN pixels are scrubbed to 1 / 0
        if bool(live.any()):
            err = max(err, float(((got - want) / scale)[:, live].abs().max()))
        if slot_sums is not None:
            h = int((one.view(torch.int32).to(torch.int64) & 0xFFFFFFFF).sum())
            sums_ok &= (h * n_evals) % 2 ** 32 == int(slot_sums[k]) % 2 ** 32
    tol = 2e-6 if fast else 1e-6
    res = {"slots": slots, "max_abs_err_vs_fp64": err, "tol": tol,
           "ok": err <= tol}
    if slot_sums is not None:
        res["checksums_match"] = bool(sums_ok)
        res["ok"] = res["ok"] and bool(sums_ok)
    return res


def dist_block(args, world, record):
    """The line's ``dist`` object: backend, world size, every rank's device
    identity (index, PCI address, UUID, host) and its own numbers (slots,
    mean eval-launch time, wall time of the timed steps), gathered from all
    ranks after the timed region."""
    import torch.distributed as dist
    from ska_sdp_screen_fitting_amd.distributed import gather_records
    per_rank = gather_records(record)
    devs = args.idents
    return {"backend": args.dist_backend if dist.is_initialized() else "none",
            "world": world, "devices": devs, "per_rank": per_rank,
            "distinct_devices": len({d.get("uuid") or d.get("pci") for d in devs})}


class PowerSampler:
    """Board power while the timed steps run (read only): the amdgpu hwmon
    power file of this rank's device in sysfs, sampled every 50 ms by a
    thread; when the box exposes none, ``amd-smi metric -p --json`` about
    once a second.  Every KL evaluation runs at the board's power limit
    ("Energy per output byte"), so the line reports the energy
    per output byte beside the rate."""

    MIN_SAMPLES = 20  # ~1 s at the 50 ms sysfs period

    def __init__(self, pci, path=None):
        import glob
        self.path, self.samples, self.source = path, [], path
        self.pci = pci
        self._smi_index = None  # amd-smi's index of this device (fallback)
        dev = f"/sys/bus/pci/devices/{pci}.0" if pci else None
        for name in ("power1_average", "power1_input"):
            if self.path:
                break
            hits = sorted(glob.glob(f"{dev}/hwmon/hwmon*/{name}")) if dev else []
            if hits:
                self.path, self.source = hits[0], hits[0]
        # the shader clock beside it (amdgpu hwmon freq1 = sclk, in Hz)
        fq = os.path.join(os.path.dirname(self.path), "freq1_input") if self.path else None
        self.freq_path = fq if fq and os.path.exists(fq) else None
        self.clocks = []
        if self.path is None and not os.path.exists("/usr/bin/amd-smi") \
                and not os.path.exists("/opt/rocm/bin/amd-smi"):
            self.source = None
        elif self.path is None:
            self.source = "amd-smi metric -p --json"
        self._stop = None
        self._thread = None

    def _read(self):
        if self.path:
            with open(self.path) as fh:
                return int(fh.read().strip()) * 1e-6  # microwatts
        import subprocess
        exe = "/opt/rocm/bin/amd-smi" if os.path.exists("/opt/rocm/bin/amd-smi") else "amd-smi"
        if self._smi_index is None:
            # this rank's card among amd-smi's entries, by PCI address; no
            # match: no reading (never another card's power)
            lst = json.loads(subprocess.run([exe, "list", "--json"], capture_output=True,
                                            text=True, timeout=10).stdout)
            lst = lst if isinstance(lst, list) else [lst]
            want = (self.pci or "").lower()
            # self.pci is domain:bus:device ("0000:05:00"), amd-smi's bdf
            # adds the function ("0000:05:00.0")
            hit = [e.get("gpu") for e in lst
                   if want and str(e.get("bdf", "")).lower().startswith(want + ".")]
            if len(hit) != 1:
                raise LookupError(f"amd-smi: no unique entry for PCI {self.pci}")
            self._smi_index = hit[0]
        out = subprocess.run([exe, "metric", "-p", "--json"], capture_output=True,
                             text=True, timeout=10).stdout
        d = json.loads(out)
        d = d if isinstance(d, list) else [d]
        d = [e for e in d if e.get("gpu") == self._smi_index]
        if len(d) != 1:
            raise LookupError(f"amd-smi metric: no entry for gpu {self._smi_index}")
        d = d[0]
        p = d.get("power", d)
        v = p.get("socket_power", p.get("average_socket_power"))
        v = v.get("value") if isinstance(v, dict) else v
        return float(v)

    def __enter__(self):
        import threading
        if self.source is None:
            return self
        self._stop = threading.Event()

        def run():
            period = 0.05 if self.path else 1.0
            while not self._stop.is_set():
                try:
                    w = self._read()
                    if w > 0:
                        self.samples.append(w)
                    if self.freq_path:
                        with open(self.freq_path) as fh:
                            self.clocks.append(int(fh.read().strip()) * 1e-6)
                except Exception:  # sysfs / amd-smi gone or malformed
                    self.source = None
                    return
                self._stop.wait(period)

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=15)
        return False

    def summary(self, out_bytes, seconds):
        """Mean board power and joules per output byte over the timed steps
        (None when no power source is readable, or when the timed steps
        took under a second: the hwmon reading averages over a window and
        lags a short run, e.g. 0.81 kW for a 0.13 s gain run that draws
        1.37 kW sustained)."""
        if len(self.samples) < self.MIN_SAMPLES or self.source is None:
            return None
        w = float(np.mean(self.samples[1:] if len(self.samples) > 2 else self.samples))
        clk = self.clocks[1:] if len(self.clocks) > 2 else self.clocks
        return {"board_W_mean": w, "samples": len(self.samples),
                "source": self.source,
                "sclk_MHz_mean": float(np.mean(clk)) if clk else None,
                "pJ_per_output_byte": w * seconds / out_bytes * 1e12,
                "what": "mean board power over the timed steps (fit + eval) x their "
                        "wall time / the bytes of output they stored"}


FP64_MFMA_PEAK_TFS = 78.6  # MI355X fp64 matrix peak (AMD spec, dense)
I8_MFMA_PEAK_TOPS = 5000.0  # MI355X int8 matrix peak (dense; 2x bf16)


STALE_COUNTERS = {}  # table -> the stale entry's library, for the line


def _profile_entry(name, workload, kernel):
    """Entry of a profiles/<name>.json table (written by the tools/ that turn
    rocprofv3 PMC passes into per-launch figures) for this workload and
    evaluation kernel, or None -- also None when the entry was taken on
    another build of the library than the one this process loaded (its
    ``library_sha16``, tools/pmc_traffic.py): counters of an older kernel
    are never reported as this one's (the line names the mismatch)."""
    from ska_sdp_screen_fitting_amd._lib import library_identity
    path = os.path.join(REPO, "profiles", name)
    try:
        tab = json.load(open(path))
    except (ValueError, OSError):
        return None
    for e in tab.get("entries", []):
        if e.get("workload") == workload and e.get("eval_kernel") == kernel:
            if e.get("library_sha16") != library_identity()["sha16"]:
                STALE_COUNTERS[f"{name}:{workload}:{kernel}"] = e.get("library_sha16")
                return None
            return e
    return None


def mfma_line(kernel, launch_slots, P, D, launch_s, workload, n_contract=1,
              contraction="f64"):
    """MFMA work of one evaluation launch over the launch time.  fp64
    contraction: executed flops (the k-steps padded to a multiple of 4
    directions) against the fp64 matrix peak; integer-digit contraction
    (kl_eval_int.h): 25 v_mfma_i32_16x16x64_i8 per 16 slots x 16 pixels
    (2 x 16 x 16 x 64 ops each) against the int8 matrix peak.  Both carry the
    algorithmic 2 D flops per pixel per slot; the MFMA-busy fraction from PMC
    counters when profiles/mfma.json holds this workload."""
    ks = (D + 3) // 4
    algo = launch_slots * P * 2.0 * D * n_contract
    if contraction == "i8-digits":
        executed = launch_slots * P * 25 * 2.0 * 64 * n_contract
        res = {"kernel": kernel, "contraction": contraction, "unit": "TOP/s (i8)",
               "peak": I8_MFMA_PEAK_TOPS, "executed": executed / launch_s / 1e12,
               "algorithmic_fp64_equiv_tflops": algo / launch_s / 1e12,
               "ops_per_launch": executed}
        res["frac"] = res["executed"] / I8_MFMA_PEAK_TOPS
    else:
        executed = launch_slots * P * 2.0 * 4 * ks * n_contract
        res = {"kernel": kernel, "contraction": contraction, "unit": "TFLOP/s",
               "peak": FP64_MFMA_PEAK_TFS,
               "executed": executed / launch_s / 1e12,
               "algorithmic": algo / launch_s / 1e12,
               "flops_per_launch": executed}
        res["frac"] = res["executed"] / FP64_MFMA_PEAK_TFS
    e = _profile_entry("mfma.json", workload, kernel)
    if e is not None:
        res["busy_frac_pmc"] = e.get("mfma_busy_frac")
        res["valu_busy_frac_pmc"] = e.get("valu_busy_frac")
    return res


def side_legs(ctx, torch, dev, stream, fit_stream, fit, evaluate, coef, bounds,
              F, A, D, P, out, ring, flags, gain=False, amp=None, fit_ones=None):
    """Untimed side measurements after the timed steps: (1) the evaluation of
    time chunk 0 with the fp64 sincos epilogue (--precise-sincos) beside the
    default fp32 one, (2) the fit of chunk 0 alone on the whole chip, with the
    workload's weights and ("also report an all-ones
    variant") with every weight 1 -- run first, so that the outputs left
    behind are the workload's.  HIP events on the stream each runs on."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS
    t0, t1 = bounds[0]
    n = (t1 - t0) * F * A
    c0 = coef[t0:t1].reshape(-1, D)
    res = {}

    def timed(fn, st, reps=2):
        fn()  # warm (kernel choice, code object)
        ms = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
        return float(np.mean(ms))

    def ev(fl):
        if gain:
            ctx.eval_gain(c0, amp["coef"][0][t0:t1].reshape(-1, D),
                          amp["coef"][1][t0:t1].reshape(-1, D), n, out, ring, fl)
        else:
            ctx.eval(c0, n, out, ring, fl)

    for name, fl in (("eval_fp32_sincos", flags),
                     ("eval_fp64_sincos", flags & ~SF_EVAL_FAST_SINCOS)):
        ctx.set_stream(stream.cuda_stream)
        ms = timed(lambda: ev(fl), stream)
        gbs = n * (16 * P + 8 * D * (3 if gain else 1)) / ms / 1e6
        res[name] = {"kernel": ctx.eval_kernel(fl, gain=gain), "slots": n,
                     "launch_ms": ms, "slots_per_s": n / ms * 1e3,
                     "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}
    if fit_ones is not None:
        ms = timed(lambda: fit_ones(fit_stream), fit_stream)
        res["fit_alone_all_ones_weights"] = {
            "slots": n, "ms": ms, "slots_per_s": n / ms * 1e3,
            "n_masks": ctx.fit_stats().get("n_masks"),
            "what": "the fit of chunk 0 with every weight 1 (no flagged "
                    "directions; the outliers stay in the phases)"}
    ms = timed(lambda: fit(0, fit_stream), fit_stream)
    res["fit_alone_whole_chip"] = {"slots": n, "ms": ms,
                                   "slots_per_s": n / ms * 1e3}
    # the box's store ceiling for context (boxes differ by ~10 %): zero_
    # (hipMemsetAsync) and fill_ of the whole output ring, on the eval stream
    flat = out.view(-1)
    nbytes = flat.numel() * 4
    best = 0.0
    with torch.cuda.stream(stream):
        for fn in (flat.zero_, lambda: flat.fill_(1.0)):
            best = max(best, nbytes / timed(fn, stream) / 1e6)
    res["store_ceiling"] = {"GBs": best, "frac_of_peak": best / HBM_PEAK_GBS,
                            "bytes": nbytes,
                            "what": "max of zero_ (hipMemsetAsync) and fill_ "
                                    "over the output ring"}
    ctx.set_stream(stream.cuda_stream)
    return res


def child_leg(extra, what, timeout_s=420, side=False, oracle=False):
    """One workload of BASELINE.json beside the config-4 line, in a child
    ``bench.py`` (its own device buffers; the parent holds its own and is
    idle meanwhile): its value, eval roofline, checks and wall time; with
    ``side``, also the child's eval alone on the chip (its side leg); with
    ``oracle``, a small CPU baseline of its own (8 workers x 16 fit slots,
    no make_aterm_image legs) whose oracle fits check the child's GPU fit."""
    import subprocess
    base = (["--cpu-workers", "8", "--cpu-fit-slots", "16", "--cpu-eval-slots", "2",
             "--no-cpu-reference-path"] if oracle else ["--no-cpu-baseline"])
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1",
           "--no-fits", "--no-child-legs",
           "--no-parity"] + base + ([] if side else ["--no-side-legs"]) + extra
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True,
                           timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s} s", "args": extra,
                "oracle_requested": oracle}
    wall = time.perf_counter() - t0
    # exit 3: the child's line is printed, its parity (oracle sample) failed
    if p.returncode not in (0, 3) or not p.stdout.strip():
        return {"error": f"exit {p.returncode}: {p.stderr[-600:]}", "args": extra,
                "oracle_requested": oracle}
    r = json.loads(p.stdout.strip().splitlines()[-1])
    rf, chk = r["roofline"], r["check"]
    sm = chk.get("sampled_slots") or {}
    out = {
        "workload": r["config"]["workload"], "args": " ".join(extra),
        "value": r["value"], "unit": r["unit"], "steps": r["steps"],
        "warmup": r["warmup"], "ms_per_step": r["ms_per_step"],
        "dtype": r["dtype"], "stages_ms": r.get("stages_ms"),
        "kernel": rf["kernel"], "launch_ms": rf["launch_ms"],
        "bytes_per_launch": rf["bytes_per_launch"], "achieved_GBs": rf["achieved"],
        "frac": rf["frac"], "traffic": rf["traffic"], "mfma": r.get("mfma"),
        "power": r.get("power"), "check": chk, "child_wall_s": wall, "what": what,
        "oracle_requested": oracle}
    if sm:
        out.update(sampled_slots=sm, checksums_match=sm.get("checksums_match"),
                   max_abs_err_vs_fp64=sm["max_abs_err_vs_fp64"], ok=sm["ok"])
    if oracle and "oracle_check" in (r.get("cpu_baseline") or {}):
        out["oracle_check"] = r["cpu_baseline"]["oracle_check"]
        out["cpu_baseline_sample"] = r["cpu_baseline"].get("sample")
        if "oracle_amp_check" in r["cpu_baseline"]:
            out["oracle_amp_check"] = r["cpu_baseline"]["oracle_amp_check"]
    alone = (r.get("side_legs") or {}).get("eval_fp32_sincos")
    if alone:
        # the same eval with nothing beside it (the step overlaps the fit of
        # the next step with it: DESIGN.md, gain screens)
        out["eval_alone"] = {k: alone[k] for k in ("launch_ms", "achieved_GBs", "frac", "slots")}
    return out


def child_legs():
    """The default line's other BASELINE.json workloads, each observed by
    the same command as the headline:

    * config5: BASELINE.json configs[4] (SKA-Low scale), one timed step
      (after one warmup step) of the shard one of its 8 GPUs runs -- 64 of
      512 stations x 4000 t x 64 f x 50 dir = 16.4 M slots, KL 512^2, fit +
      eval on the integer-digit contraction, discard + checksum mode
      (kl_screen.py:411-449), ~45 GB of device buffers;
    * gain_config3: the gain screens (phase + XX / YY amplitude fits, the
      three-contraction eval with 10 **, kl_screen.py:96-125, 319-378) on
      the config-3 shape, 30 steps, two coefficient sets (the fit of step
      k+1 beside the eval of step k);
    * tess_config3: the tessellated fill (voronoi_screen.py:132-216) on the
      config-3 shape, 10 steps."""
    return {
        "config5": child_leg(
            ["--workload", "config5", "--steps", "1", "--warmup", "1"],
            "one step of config 5's per-GPU shard in a child process "
            "(bench.py --workload config5 --steps 1 --warmup 1), its fit "
            "checked against the oracle on 128 sampled slots", oracle=True),
        "gain_config3": child_leg(
            ["--screen", "gain", "--workload", "config3", "--steps", "30", "--warmup", "2"],
            "gain screens on the config-3 shape in a child process, its phase "
            "fit checked against the oracle on 128 sampled slots and its "
            "amplitude fit on 4 whole (freq, station, pol) blocks", side=True,
            oracle=True),
        "tess_config3": child_leg(
            ["--screen", "tess", "--workload", "config3", "--steps", "10", "--warmup", "2"],
            "tessellated fill on the config-3 shape in a child process, its "
            "label raster and slot-0 fill checked against the oracle", oracle=True),
    }


def child_leg_parity(side, line):
    """Fold the child legs' oracle samples (their CPU baseline legs) into the
    line's parity object; returns True when one failed.  A leg launched with
    its oracle sample that errored, timed out or came back without the sample
    counts as failed (its parity is unproven)."""
    failed = False
    for leg, key, pkey in (("config5", "oracle_check", "fit_oracle_sample_config5"),
                           ("gain_config3", "oracle_check",
                            "fit_oracle_sample_gain_config3"),
                           ("gain_config3", "oracle_amp_check",
                            "fit_oracle_amplitude_blocks_gain_config3"),
                           ("tess_config3", "oracle_check",
                            "tess_oracle_sample_config3")):
        lr = side.get(leg)
        if lr is None:
            continue  # the leg did not run
        c5 = lr.get(key)
        if c5 is None:
            if not lr.get("oracle_requested"):
                continue
            c5 = {"max_err": None, "tol": None, "ok": False, "slots": 0,
                  "error": lr.get("error", f"no {key} in the leg's line")}
        par = line.setdefault("parity", {})
        par[pkey] = {"max_err": c5.get("max_err", c5.get("coef_max_abs_err")),
                     "tol": c5["tol"], "ok": c5["ok"], "slots": c5["slots"]}
        if "error" in c5:
            par[pkey]["error"] = c5["error"]
        if "all_ok" in par:
            par["all_ok"] = par["all_ok"] and c5["ok"]
        failed = failed or not c5["ok"]
    return failed


def setup_digest(setup):
    """sha256 (16 hex digits) of the setup a rank works from: piercepoints,
    grid coordinates, reference-station phases and index."""
    import hashlib
    h = hashlib.sha256()
    for a in (np.asarray(setup["piercepoints"]), np.asarray(setup["x"]),
              np.asarray(setup["y"]), setup["ref_phase"].cpu().numpy()):
        h.update(np.ascontiguousarray(a, np.float64).tobytes())
    h.update(str(setup["ref_ant"]).encode())
    return h.hexdigest()[:16]


def rehearse_cpu(args, dist, world, rank, sol, setup, A, A_total, a0,
                 unsharded_setup=None):
    """--rehearse-cpu: the launcher and the gloo setup collectives without
    a GPU -- every rank builds its shard and runs setup_shard; the line
    reports each rank's shard and a digest of the setup it received (equal
    on every rank).  No kernels run: ``value`` is null.  Its ``parity``
    object: every rank's setup equals the unsharded run's (rebuilt by rank
    0, ``unsharded_setup``), the ranks' station orders concatenate to the
    unsharded run's, and the rank identities pass the nccl one-card check
    (check_distinct_devices, the refusal a real nccl job applies)."""
    t0 = time.perf_counter()
    if dist.is_initialized():
        dist.barrier()
    T, F = sol.val.shape[:2]
    record = {"rank": rank, "ant": [a0, a0 + A], "slots": T * F * A,
              "setup_sha16": setup_digest(setup), "ref_ant": setup["ref_ant"],
              "st_order": setup["st_order"]}
    dist_info = dist_block(args, world, record)
    whole = unsharded_setup() if rank == 0 and unsharded_setup else None
    if dist.is_initialized():
        dist.barrier()
    if rank == 0:
        from ska_sdp_screen_fitting_amd.distributed import check_distinct_devices
        try:
            check_distinct_devices(args.idents, "nccl")
            nccl = {"ok": True}
        except RuntimeError as exc:
            nccl = {"ok": False, "error": str(exc)}
        dist_info["nccl_distinct_check"] = nccl
        parity = {"nccl_distinct_devices": nccl}
        if whole is not None:
            want = setup_digest(whole)
            orders = sum((list(r["st_order"]) for r in dist_info["per_rank"]), [])
            parity["shard_setup"] = {
                "unsharded_setup_sha16": want,
                "every_rank_equal": all(r["setup_sha16"] == want
                                        for r in dist_info["per_rank"]),
                "station_orders_equal": orders == list(whole["st_order"]),
                "ranks": len(dist_info["per_rank"])}
            parity["shard_setup"]["ok"] = (parity["shard_setup"]["every_rank_equal"]
                                           and parity["shard_setup"]["station_orders_equal"])
        parity["all_ok"] = all(v["ok"] for v in parity.values() if isinstance(v, dict))
        line = {"metric": METRIC, "value": None, "unit": "screen-slots/s",
                "n_gpus": world, "steps": 0, "warmup": 0,
                "ms_per_step": None, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic",
                "config": {"workload": f"{args.workload}: {A_total} ant, rehearsal",
                           "parallelism": f"ant-shard x{world}",
                           "schedule": args.schedule},
                "rehearsal": ("cpu: self-launch + gloo setup collectives only, "
                              "no kernels"),
                "setup_s": time.perf_counter() - t0, "dist": dist_info,
                "parity": parity}
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def tess_steps(args, ctx, torch, dev, dist, world, rank, coll_dev, sol, setup,
               A_total, strong):
    """--screen tess: one step = the tessellated fill (gather of the
    referenced per-direction cos / sin by the Voronoi label raster, optional
    fused Gaussian) of every slot of the rank into the HBM ring; the label
    template is built once on the host (voronoi_screen.py:218-351)."""
    from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_NAN_SCRUB, SF_OPT_TESS_BOX,
                                                 SF_OPT_TESS_SLOTS, SF_OPT_TESS_WAVES)
    from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG,
                                                      FIELD_RA_DEG,
                                                      FIELD_WIDTH_DEG)
    from ska_sdp_screen_fitting_amd.voronoi_screen import tessellation_template
    A, T, F, D, N, cell = WORKLOADS[args.workload]
    T, F, A, D = sol.val.shape
    lab, _ = tessellation_template(np.rad2deg(sol.dir_radec.astype(np.float64)),
                                   FIELD_RA_DEG, FIELD_DEC_DEG, FIELD_WIDTH_DEG, cell)
    assert lab.shape == (N, N)
    S, P = T * F * A, N * N
    lab_d = torch.from_numpy(np.ascontiguousarray(lab, np.int32)).to(dev)
    # referenced phases (stationscreen.py:994-997), the fill's input
    ph = (torch.from_numpy(sol.val).to(dev)
          - setup["ref_phase"].to(dev)[:, :, None, :]).reshape(S, D).contiguous()
    ring = int(min(S, max(1, args.ring_gb * 2 ** 30 // (16 * P))))
    out = torch.empty((ring, 4, N, N), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    if args.tess_slots:
        ctx.set_option(SF_OPT_TESS_SLOTS, args.tess_slots)
    if args.tess_waves:
        ctx.set_option(SF_OPT_TESS_WAVES, args.tess_waves)
    ctx.set_option(SF_OPT_TESS_BOX, args.tess_box)
    flags = SF_EVAL_NAN_SCRUB

    amp = {}
    if args.tess_gain:
        # synthetic amplitudes around 1 (log10 sigma 0.1), one set per pol
        g = torch.Generator(device="cpu").manual_seed(7)
        for k in ("amp_xx", "amp_yy"):
            amp[k] = (10.0 ** (0.1 * torch.randn((S, D), generator=g,
                                                 dtype=torch.float64))).to(dev)

    def step():
        ctx.tess_fill(lab_d, N, N, ph, D, S, out, ring_slots=ring,
                      smooth_pix=args.smooth_pix, flags=flags, **amp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = []
    sampler = PowerSampler(args.idents[rank].get("pci"))
    with sampler:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            step()
            e1.record(stream)
            evs.append((e0, e1))
        torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier()
        elapsed = time.perf_counter() - t0
    local_elapsed = elapsed
    power = sampler.summary(float(S) * 16 * P * args.steps, local_elapsed)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if dist.is_initialized():
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    elapsed = tmax.item()
    launch_s = float(np.mean([a.elapsed_time(b) for a, b in evs])) * 1e-3
    dist_info = dist_block(args, world, {
        "rank": rank, "slots": S, "fill_launch_ms": launch_s * 1e3,
        "steps_wall_s": local_elapsed, "device_pci": args.idents[rank]["pci"]})
    # parity spot check of the last ring slots (not timed), without
    # smoothing: cos^2 + sin^2 = 1 (unit amplitudes), or with XX / YY
    # amplitudes the shared angle (Re XX Im YY - Im XX Re YY = 0 relative to
    # |XX| |YY|); and the first slot vs a gather
    chk = out[: min(ring, 16)].double()
    unit_err, check_name = None, "max_abs_cos2_plus_sin2_minus_1"
    if args.smooth_pix == 0 and not args.tess_gain:
        unit_err = float((chk[:, 0] ** 2 + chk[:, 1] ** 2 - 1).abs().max())
    elif args.smooth_pix == 0:
        cross = chk[:, 0] * chk[:, 3] - chk[:, 1] * chk[:, 2]
        mag = (chk[:, 0].hypot(chk[:, 1]) * chk[:, 2].hypot(chk[:, 3])).clamp(min=1e-30)
        unit_err, check_name = float((cross / mag).abs().max()), "max_rel_xx_yy_angle_cross"
    # a slot of a station other than the reference (whose referenced phases
    # are 0: every cell the same value, the labels untested)
    k0 = 1 if setup["ref_ant"] == 0 and A > 1 else 0
    one = torch.empty((1, 4, N, N), dtype=torch.float32, device=dev)
    ctx.tess_fill(lab_d, N, N, ph[k0:k0 + 1], D, 1, one, smooth_pix=0.0, flags=flags)
    p0 = ph[k0].cpu().numpy()
    want = np.stack([np.cos(p0), np.sin(p0), np.cos(p0), np.sin(p0)]).astype(np.float32)
    want = want[:, lab - 1]
    got = one[0].cpu().numpy()
    ulp = int(np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32)).max())
    if rank == 0:
        bytes_launch = S * (16 * P + 8 * D)
        achieved = bytes_launch / launch_s / 1e9
        # the library's choice (tess.hip launch_tess, SF_OPT_TESS_BOX auto)
        R = int(4.0 * args.smooth_pix + 0.5) if args.smooth_pix > 0 else 0
        box = 0 < R <= 24 and (args.tess_box == 1 or (args.tess_box < 0 and
                                                       args.tess_gain and R <= 5))
        kernel = ("kl_tess_gather_kernel" if R == 0 else
                  "kl_tess_box_kernel" if box else "kl_tess_smooth_kernel")
        # PMC traffic (profiles/traffic.json) when measured on this call shape
        traffic = None
        wkey = (args.workload + "-tess" + ("-gain" if args.tess_gain else "")
                + (f"-s{args.smooth_pix:g}" if args.smooth_pix else ""))
        tj = _profile_entry("traffic.json", wkey, kernel)
        if (tj is not None and tj.get("flags") == flags
                and abs(tj.get("algorithmic_bytes_per_launch", 0) - bytes_launch)
                <= 1e-6 * bytes_launch):
            traffic = tj.get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC,
            "value": T * F * (A if args.as_shard_of else A_total) * args.steps / elapsed,
            "unit": "screen-slots/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {
                "workload": (f"{args.workload}-tess: {A_total} ant x {T} time x {F} "
                             f"freq x {D} dir, {A} ant per GPU, tessellated "
                             f"(Voronoi) {N}^2 screen, smooth {args.smooth_pix} px"
                             + (", XX / YY amplitudes" if args.tess_gain else "")),
                "screen": "tess", "slots_per_gpu": S, "grid": N, "n_dir": D,
                "parallelism": f"ant-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel": kernel,
                         "bytes_per_launch": bytes_launch,
                         "launch_ms": launch_s * 1e3},
            "power": power,
            "check": {check_name: unit_err,
                      "slot0_max_ulp_vs_numpy_gather": ulp},
            "dist": dist_info,
        }
        failed = False
        if world == 1 and not args.no_cpu_baseline:
            cb = tess_cpu_baseline(sol, setup, cell, lab, got, slot=k0)
            line["cpu_baseline"] = cb
            oc = cb["oracle_check"]
            line["parity"] = {"tess_oracle_sample": {
                "max_err": oc["max_err"], "tol": oc["tol"], "ok": oc["ok"],
                "slots": oc["slots"], "labels_differ": oc["labels_differ"]},
                "all_ok": oc["ok"]}
            failed = not oc["ok"]
        print(json.dumps(line), flush=True)
        if failed:
            log("PARITY FAILED: the tessellated fill differs from the oracle")
            raise SystemExit(3)
    if dist.is_initialized():
        dist.destroy_process_group()


def pick_schedule(args, D, T):
    """The step's schedule: time chunks, coefficient sets, CU reservation.
    A function of the workload's shape and the command-line options only --
    never of the world size -- so every N of the driver's scaling curve runs
    the same schedule per GPU (the reference's fan-out, stationscreen.py:
    1056-1077, gives each worker the same work; tests/test_bench_launch.py)."""
    gain = args.screen == "gain"
    # the amplitude outlier sigma couples every time of a (freq, station)
    # block (Q6): the gain fit sees all times at once
    n_chunks = 1 if gain else max(1, min(args.chunks, T))
    n_sets = args.coef_sets if args.coef_sets > 0 else (
        2 if gain and args.steps > 1 else 1)
    pipelined = n_chunks > 1 or n_sets > 1
    reserve_cus = args.reserve_cus
    if reserve_cus < 0:
        reserve_cus = 16 if D <= 32 and n_chunks > 1 else 0
    on_reserved = args.fit_on_reserved
    if on_reserved < 0:
        on_reserved = 1 if D <= 32 else 0
    return {"time_chunks": n_chunks, "coef_sets": n_sets, "pipelined": pipelined,
            "reserve_cus": reserve_cus if pipelined else 0,
            "fit_on_reserved": bool(on_reserved and pipelined and reserve_cus > 0),
            "fit_priority": int(args.fit_priority) if pipelined else 0}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the ranks here (the parent never touches the GPU)
        raise SystemExit(launch_ranks(args.gpus, args.launch_timeout))
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse_cpu and args.dist_backend != "gloo":
        raise SystemExit("--rehearse-cpu needs --dist-backend gloo")
    if args.rehearse_cpu:
        gpu, dev = None, torch.device("cpu")
    else:
        n_dev = torch.cuda.device_count()
        # local rank -> visible device; modulo, so a launcher that gives every
        # rank its own one-device HIP_VISIBLE_DEVICES works too (two ranks
        # that resolve to one card are refused below under nccl)
        if n_dev < 1:
            raise SystemExit("bench.py: no GPU visible (torch.cuda.device_count() == 0)")
        gpu = local_rank % n_dev
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    if world > 1 or args.force_dist:
        # --force-dist without a launcher: a one-rank env:// rendezvous
        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"),
                     ("MASTER_ADDR", "127.0.0.1")):
            os.environ.setdefault(k, v)
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    log(f"rank {rank}/{world} backend "
        f"{args.dist_backend if dist.is_initialized() else 'none'} device {dev}")
    # which physical GPU every rank drives, gathered once before any work:
    # under nccl two ranks on one card end the job here
    from ska_sdp_screen_fitting_amd.distributed import (check_distinct_devices,
                                                        device_identity,
                                                        gather_records)
    if args.rehearse_cpu:
        ident = {"index": None, "pci": f"cpu:{socket.gethostname()}:{os.getpid()}",
                 "uuid": "", "name": "cpu (rehearsal)"}
    else:
        ident = device_identity(torch, dev)
    ident = dict(ident, rank=rank, local_rank=local_rank, host=socket.gethostname())
    idents = gather_records(ident)
    try:
        check_distinct_devices(idents, args.dist_backend if world > 1 else "none")
    except RuntimeError as exc:
        raise SystemExit(f"bench.py: {exc}")
    args.idents = idents

    from ska_sdp_screen_fitting_amd import get_context
    from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_FAST_SINCOS,
                                                 SF_EVAL_NAN_SCRUB,
                                                 SF_EVAL_NT_STORES,
                                                 SF_OPT_EVAL_BANDS,
                                                 SF_OPT_EVAL_GROUPS,
                                                 SF_OPT_EVAL_INT,
                                                 SF_OPT_EVAL_KERNEL,
                                                 SF_OPT_EVAL_SLEEP,
                                                 SF_OPT_EVAL_XCD_MAP)
    from ska_sdp_screen_fitting_amd.distributed import setup_shard
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE, library_identity
    from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG,
                                                      FIELD_RA_DEG,
                                                      FIELD_WIDTH_DEG,
                                                      make_amplitudes,
                                                      make_solutions)

    A, T, F, D, N, cell = WORKLOADS[args.workload]
    strong = args.workload in STRONG
    if strong:
        from ska_sdp_screen_fitting_amd.distributed import shard_range
        A_total = A
        if args.as_shard_of and world != 1:
            raise SystemExit("--as-shard-of is a one-process projection")
        a0, a1 = shard_range(A_total, args.as_shard_of or world, rank)
        A = a1 - a0
    else:
        A_total, a0 = A * world, A * rank
    sol = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D,
                         ant_offset=a0, n_ant_total=A_total)
    setup = setup_shard(sol, a0, A_total, FIELD_RA_DEG, FIELD_DEC_DEG,
                        FIELD_WIDTH_DEG, cell,
                        device=coll_dev if dist.is_initialized() else "cpu")
    assert len(setup["x"]) == N
    log(f"shard ready: ant [{a0}, {a0 + A}) of {A_total}, {T * F * A} slots")
    if args.rehearse_cpu:
        args.schedule = pick_schedule(args, D, T)
        # the setup the unsharded (N = 1) run computes, rebuilt by rank 0 on a
        # one-rank group: the rehearsal's parity object compares every
        # rank's received setup with it
        solo = dist.new_group([0]) if dist.is_initialized() else None

        def unsharded_setup():
            whole = make_solutions(n_ant=A_total, n_time=T, n_freq=F, n_dir=D,
                                   ant_offset=0, n_ant_total=A_total)
            return setup_shard(whole, 0, A_total, FIELD_RA_DEG, FIELD_DEC_DEG,
                               FIELD_WIDTH_DEG, cell, group=solo)
        return rehearse_cpu(args, dist, world, rank, sol, setup, A, A_total, a0,
                            unsharded_setup)

    ctx = get_context(gpu)
    if args.screen == "tess":
        return tess_steps(args, ctx, torch, dev, dist, world, rank, coll_dev,
                          sol, setup, A_total, strong)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_basis(setup["piercepoints"], 100, 5.0 / 3.0)
    ctx.set_grid(setup["x"], setup["y"])

    S = T * F * A
    P = N * N
    phase = torch.from_numpy(sol.val).to(dev)
    weight = torch.from_numpy(sol.weight).to(dev)
    refph = setup["ref_phase"].to(dev).contiguous()
    coef = torch.empty_like(phase)
    resid = torch.empty_like(phase)
    w_out = torch.empty_like(weight)
    order_out = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    slot_bytes = 16 * P
    ring = int(min(S, max(1, args.ring_gb * 2 ** 30 // slot_bytes)))
    out = torch.empty((ring, 4, N, N), dtype=torch.float32, device=dev)
    flags = (SF_EVAL_NAN_SCRUB | SF_EVAL_NT_STORES
             | (0 if args.precise_sincos else SF_EVAL_FAST_SINCOS))
    gain = args.screen == "gain"
    amp = None
    if gain:
        # slow XX / YY amplitudes on the phase grid; fitted in log10 space
        # with order min(12, max(3, round(D / 2))), no order scaling, no
        # reference station, 3 iterations (kl_screen.py:96-125)
        make_amplitudes(sol)
        order_amp = min(12, max(3, int(np.round(D / 2))))
        # the two pols stacked along the station axis, one fit call for both
        # (as stationscreen.run does: amplitudes are never referenced and
        # their outlier sigma is per (station, freq) block, so the pols are
        # independent blocks); the evaluation takes each pol's coefficients
        # as its own contiguous [S][D] array (copied per step, 2 x 16 MB)
        v = np.concatenate([sol.amp_val[..., p] for p in range(2)], axis=2)
        w = np.concatenate([sol.meta["amp_weight"][..., p] for p in range(2)], axis=2)
        v = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
        w = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
        amp = {"order": order_amp, "val": v, "w": w, "stacked": torch.empty_like(v),
               "resid": torch.empty_like(v), "w_out": torch.empty_like(w),
               "orders": torch.empty((T, F, 2 * A), dtype=torch.int32, device=dev),
               "coef": [torch.empty((T, F, A, D), dtype=torch.float64, device=dev)
                        for _ in range(2)]}

    # time chunks (the solution layout is time-major, so a chunk is a
    # contiguous slice of every array); phase slots are independent, so the
    # fit of one chunk can run while the previous chunk is evaluated;
    # coefficient sets: step k fits into and evaluates from set k % n_sets
    sched = pick_schedule(args, D, T)
    n_chunks, n_sets = sched["time_chunks"], sched["coef_sets"]
    coef_sets = [coef] + [torch.empty_like(coef) for _ in range(n_sets - 1)]
    # per coefficient set: the stacked fit output and its per-pol copies
    amp_sets = ([(amp["stacked"], amp["coef"])]
                + [(torch.empty_like(amp["stacked"]),
                    [torch.empty_like(x) for x in amp["coef"]])
                   for _ in range(n_sets - 1)]) if gain else None
    pipelined = sched["pipelined"]
    bounds = [(T * c // n_chunks, T * (c + 1) // n_chunks) for c in range(n_chunks)]
    # the eval saturates HBM without every CU: its stream leaves
    # --reserve-cus compute units (spread over the XCDs) to the fit stream, so
    # the fit of the next chunk is not starved by queued eval workgroups
    fit_stream = stream
    masked_handle = fit_handle = None
    if pipelined:
        fit_stream = torch.cuda.Stream(dev, priority=-1 if args.fit_priority else 0)
    # the first fit of a run has the chip to itself (nothing to overlap):
    # it runs on an unrestricted stream even when later fits are confined
    first_fit_stream = fit_stream
    if pipelined:
        reserve_cus = sched["reserve_cus"]
        if reserve_cus > 0:
            n_cu = ctx.device_cus()
            step = max(1, n_cu // reserve_cus)
            # k*step + k%8: one per XCD whether CUs are numbered XCD-major
            # or interleaved across the 8 XCDs
            reserved = [min(n_cu - 1, k * step + k % 8) for k in range(reserve_cus)]
            masked_handle = ctx.stream_create(reserved)
            stream = torch.cuda.ExternalStream(masked_handle, device=dev)
            if sched["fit_on_reserved"]:
                keep = set(reserved)
                fit_handle = ctx.stream_create([c for c in range(n_cu) if c not in keep])
                fit_stream = torch.cuda.ExternalStream(fit_handle, device=dev)

    ctx.set_option(SF_OPT_EVAL_XCD_MAP, args.eval_xcd_map)
    ctx.set_option(SF_OPT_EVAL_GROUPS, args.eval_groups)
    ctx.set_option(SF_OPT_EVAL_INT, args.eval_int)
    ctx.set_option(SF_OPT_EVAL_KERNEL, args.eval_kernel)
    ctx.set_option(SF_OPT_EVAL_BANDS, args.eval_bands)
    ctx.set_option(SF_OPT_EVAL_SLEEP, args.eval_sleep)
    eval_kernel_name = ctx.eval_kernel(flags, gain=gain)
    contraction = ctx.eval_contraction(flags, gain=gain)
    # discard + checksum mode: the cubes go
    # through the HBM ring and every slot's checksum is accumulated
    checksum = args.checksum == "on" or (args.checksum == "auto"
                                         and args.workload in ("config4", "config5"))
    slot_sums = torch.zeros(S, dtype=torch.int32, device=dev) if checksum else None

    def fit(c, fs, b=0, wts=None):
        t0, t1 = bounds[c]
        ctx.set_stream(fs.cuda_stream)
        w_in = weight if wts is None else wts
        ctx.fit(phase[t0:t1], w_in[t0:t1], t1 - t0, F, A, setup["st_order"],
                niter=2, nsigma=5.0, adjust_order=True, ref_ant=setup["ref_ant"],
                coef=coef_sets[b][t0:t1], resid=resid[t0:t1], w_out=w_out[t0:t1],
                order_out=order_out[t0:t1], ant_offset=setup["ant_offset"],
                ref_phase=refph[t0:t1])
        if gain:
            ctx.fit(amp["val"][t0:t1], amp["w"][t0:t1], t1 - t0, F, 2 * A,
                    [amp["order"]] * (2 * A), screen_type=SF_SCREEN_AMPLITUDE,
                    niter=3, nsigma=5.0, adjust_order=True, ref_ant=-1,
                    coef=amp_sets[b][0][t0:t1], resid=amp["resid"][t0:t1],
                    w_out=amp["w_out"][t0:t1], order_out=amp["orders"][t0:t1])

    def stage_amp(c, b=0):
        """Gain: each pol's coefficients of the stacked amplitude fit into its
        own contiguous array, on the eval stream after fit(c) (outside the
        eval kernel's event window)."""
        if not gain:
            return
        t0, t1 = bounds[c]
        stacked, (xx, yy) = amp_sets[b]
        with torch.cuda.stream(stream):
            xx[t0:t1].copy_(stacked[t0:t1, :, :A])
            yy[t0:t1].copy_(stacked[t0:t1, :, A:])

    def evaluate(c, b=0):
        t0, t1 = bounds[c]
        ctx.set_stream(stream.cuda_stream)
        n = (t1 - t0) * F * A
        coef = coef_sets[b]
        cxx = cyy = None
        if gain:
            xx, yy = amp_sets[b][1]
            cxx = xx[t0:t1].reshape(-1, D)
            cyy = yy[t0:t1].reshape(-1, D)
        if checksum:
            ctx.eval_sums(coef[t0:t1].reshape(-1, D), n, out,
                          slot_sums[t0 * F * A:t1 * F * A], ring, coef_xx=cxx,
                          coef_yy=cyy, flags=flags)
        elif gain:
            ctx.eval_gain(coef[t0:t1].reshape(-1, D), cxx, cyy, n, out, ring, flags)
        else:
            ctx.eval(coef[t0:t1].reshape(-1, D), n, out, ring, flags)

    # work items in issue order: every step fits and evaluates all chunks;
    # eval(c) waits for fit(c) (event), fit(c+1) is issued after eval(c) so
    # it overlaps it; fit events bracket the fit stream, eval events the
    # eval stream
    def run_steps(n):
        evs = []
        items = [(k, c) for k in range(n) for c in range(n_chunks)]
        if not items:
            return evs
        fit_done, eval_done = {}, {}

        def issue_fit(i):
            k, c = items[i]
            fs = first_fit_stream if i == 0 else fit_stream
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            lag = n_chunks * n_sets
            if i >= lag:
                # chunk c of this coefficient set is rewritten: wait for the
                # eval that last read it (write-after-read across streams)
                fs.wait_event(eval_done[i - lag])
            if i > 0:
                fs.wait_event(fit_done[i - 1][1])  # fits share the ctx scratch
            e0.record(fs)
            if not args.eval_only:
                fit(c, fs, k % n_sets)
            e1.record(fs)
            fit_done[i] = (e0, e1)

        issue_fit(0)
        for i, (k, c) in enumerate(items):
            stream.wait_event(fit_done[i][1])
            stage_amp(c, k % n_sets)
            e2 = torch.cuda.Event(enable_timing=True)
            e3 = torch.cuda.Event(enable_timing=True)
            e2.record(stream)
            evaluate(c, k % n_sets)
            e3.record(stream)
            eval_done[i] = e3
            if i + 1 < len(items):
                issue_fit(i + 1)
            evs.append((fit_done[i][0], fit_done[i][1], e2, e3))
        return evs

    if args.eval_only:
        for b in range(n_sets):
            for c in range(n_chunks):
                fit(c, first_fit_stream, b)
    log(f"warmup: {args.warmup} steps")
    run_steps(args.warmup)
    torch.cuda.synchronize(dev)

    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    log(f"timed: {args.steps} steps")
    sampler = PowerSampler(args.idents[rank].get("pci"))
    with sampler:
        t0 = time.perf_counter()
        ev = run_steps(args.steps)
        torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier()
        elapsed = time.perf_counter() - t0
    local_elapsed = elapsed
    power = sampler.summary(float(S) * 16 * P * args.steps, local_elapsed)
    ctx.set_stream(stream.cuda_stream)
    fit_stats = ctx.fit_stats() if not args.eval_only else {}
    # per-step stage sums; per-launch eval duration for the roofline
    t_fit = float(np.sum([a.elapsed_time(b) for a, b, _, _ in ev])) * 1e-3 / args.steps
    eval_launch = [c_.elapsed_time(d_) for _, _, c_, d_ in ev]
    t_eval = float(np.sum(eval_launch)) * 1e-3 / args.steps
    t_eval_launch = float(np.mean(eval_launch)) * 1e-3
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if dist.is_initialized():
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    elapsed = tmax.item()

    dist_info = dist_block(args, world, {
        "rank": rank, "slots": S, "eval_launch_ms": t_eval_launch * 1e3,
        "fit_ms_per_step": t_fit * 1e3, "steps_wall_s": local_elapsed,
        "device_pci": args.idents[rank]["pci"]})
    # parity spot check (cheap invariants, not timed): per screen type, the
    # invariant of its planes -- phase screens cos^2 + sin^2 = 1; gain screens
    # Re XX / Im XX and Re YY / Im YY share an angle, so
    # Re XX * Im YY - Im XX * Re YY = 0 relative to |XX| |YY|
    chk = out[: min(ring, 64)].double()
    if gain:
        cross = chk[:, 0] * chk[:, 3] - chk[:, 1] * chk[:, 2]
        mag = (chk[:, 0].hypot(chk[:, 1]) * chk[:, 2].hypot(chk[:, 3])).clamp(min=1e-30)
        check_name = "max_rel_xx_yy_angle_cross"
        unit_err = float((cross / mag).abs().max())
    else:
        check_name = "max_abs_cos2_plus_sin2_minus_1"
        unit_err = float((chk[:, 0] ** 2 + chk[:, 1] ** 2 - 1).abs().max())
    sampled = sampled_slots_check(
        ctx, torch, dev, setup, coef.reshape(-1, D), N, flags, slot_sums,
        args.warmup + args.steps, not args.precise_sincos,
        cxx=amp["coef"][0].reshape(-1, D) if gain else None,
        cyy=amp["coef"][1].reshape(-1, D) if gain else None)

    side = {}
    if not args.no_side_legs and not args.eval_only:
        log("side legs")
        ones = torch.ones_like(weight)
        side = side_legs(ctx, torch, dev, stream, first_fit_stream, fit, evaluate,
                         coef, bounds, F, A, D, P, out, ring, flags, gain, amp,
                         fit_ones=lambda fs: fit(0, fs, 0, ones))
        del ones
    # the CPU baseline's sample of this workload's fit, taken now: the
    # parity and FITS legs below reuse this process's context with other
    # bases and grids
    gpu_sample = gpu_amp = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.eval_only:
        nw_cpu = args.cpu_workers or cpu_share()[0]
        nw_cpu = max(1, nw_cpu)
        for c in range(n_chunks):
            fit(c, stream, 0)
        torch.cuda.synchronize(dev)
        gpu_sample = gpu_sample_outputs(
            torch, baseline_sample(sol, setup, nw_cpu, args.cpu_fit_slots),
            coef_sets[0], w_out, order_out)
        if gain:
            gpu_amp = gpu_amp_outputs(amp_blocks(sol), A, amp_sets[0][0], amp["w_out"],
                                      amp["orders"])
    if (rank == 0 and world == 1 and args.workload == "config4" and not gain
            and not args.no_child_legs and not args.as_shard_of
            and not args.eval_only):
        log("child legs: config 5, gain and tessellated on config 3")
        side.update(child_legs())

    parity_failed = False
    if rank == 0:
        # SURVEY.md §8(d), per step; gain screens read three coefficient sets
        algo_bytes = S * (16 * P + 8 * D * (3 if gain else 1))
        launch_bytes = algo_bytes / n_chunks  # per eval launch (equal chunks)
        achieved = launch_bytes / t_eval_launch / 1e9
        traffic = None
        wkey = args.workload + ("-gain" if gain else "")
        tj = _profile_entry("traffic.json", wkey, eval_kernel_name)
        # the PMC table's figure counts only when it was taken on this very
        # call shape (same flags, chunks and algorithmic bytes per call: a
        # sharded run's calls are smaller than the N = 1 run it was measured on)
        if (tj is not None and tj.get("flags") == flags
                and tj.get("chunks", 1) == n_chunks
                and abs(tj.get("algorithmic_bytes_per_launch", 0) - launch_bytes)
                <= 1e-6 * launch_bytes):
            traffic = tj.get("hbm_bytes_per_launch")
        ceil = side.get("store_ceiling") if side else None
        line = {
            "metric": METRIC,
            "value": T * F * (A if args.as_shard_of else A_total) * args.steps / elapsed,
            "unit": "screen-slots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            # the arithmetic of the contraction: fp64 MFMAs, or (phase, D >=
            # 45) exact int8-digit products of 36- / 44-bit fixed point into
            # int32 modulo 2^32 turns; the fit is fp64 either way
            "dtype": "f64" if contraction == "f64" else "i8-digit fixed point (f64 in)",
            "data": "synthetic",
            "config": {
                "workload": (f"{args.workload}{'-gain' if gain else ''}: {A_total} ant x "
                             f"{T} time x {F} freq x "
                             f"{D} dir, {A} ant per GPU (ant-sharded, "
                             f"{'strong' if strong else 'weak'} scaling), KL {N}^2 "
                             + ("gain screens: phase fit (niter 2) + XX / YY "
                                "log10-amplitude fits (niter 3, order "
                                f"{amp['order']}) + 3-contraction eval with 10**"
                                if gain else
                                "screen, fit (phase, niter 2, adjust_order) + eval")),
                "screen": args.screen,
                "slots_per_gpu": S, "grid": N, "n_dir": D,
                "parallelism": f"ant-shard x{world}",
                "eval_sincos": "fp64" if args.precise_sincos else "fp32-after-fp64-reduction",
                "eval_only": bool(args.eval_only),
                "schedule": sched,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": eval_kernel_name,
                "bytes_per_launch": launch_bytes,
                "launch_ms": t_eval_launch * 1e3,
                "frac_of_box_store_ceiling": achieved / ceil["GBs"] if ceil else None,
            },
            "mfma": mfma_line(eval_kernel_name, S / n_chunks, P, D,
                              t_eval_launch, wkey, 3 if gain else 1, contraction),
            "stages_ms": {"fit": t_fit * 1e3, "eval": t_eval * 1e3,
                          "overlap": ("none" if not pipelined else
                                      "fit(c+1) || eval(c), %d time chunks x %d "
                                      "coefficient sets" % (n_chunks, n_sets))},
            "fit_stats": fit_stats,
            "power": power,
            "check": {check_name: unit_err, "sampled_slots": sampled},
            "dist": dist_info,
        }
        if side:
            line["side_legs"] = side
        if args.as_shard_of:
            # one GPU running the shard of rank 0 of an N-way strong split:
            # nothing in the timed step is shared between ranks, so N such
            # GPUs would process N x this (the driver measures the real curve)
            line["projection"] = {
                "as_shard_of": args.as_shard_of,
                "shard_slots_per_s": line["value"],
                "aggregate_if_n_gpus": line["value"] * args.as_shard_of,
                "note": "one process, rank 0's shard; not an N-GPU measurement"}
        # the fit (slots/s and achieved fp64 FLOP/s): alone
        # on the whole chip (side leg) and per kernel from PMC passes
        fe = _profile_entry("fit_flops.json", wkey, "fit")
        fa = side.get("fit_alone_whole_chip") if side else None
        if fa or fe:
            line["fit"] = {
                "slots_per_s_alone": fa["slots_per_s"] if fa else None,
                "ms_per_step_in_pipeline": t_fit * 1e3,
                "fp64_peak_tflops": FP64_MFMA_PEAK_TFS,
                "kernels_pmc": {k: {"fp64_tflops": v.get("fp64_tflops"),
                                    "avg_ms": v.get("avg_ms"),
                                    "avg_ms_under_pmc": v.get("avg_ms_under_pmc")}
                                for k, v in (fe or {}).get("kernels", {}).items()},
            "kernels_pmc_source": (fe or {}).get("source"),
            }
        kept = {}
        if not args.no_fits and world == 1:
            log("FITS wall-clock legs")
            line["fits_wallclock"] = fits_wallclock(config3=not args.no_fits_config3,
                                                    kept=kept)
        if not args.no_parity:
            # parity of the path against the reference's own outputs (golden
            # files only), on the cubes the FITS legs wrote when they ran
            log("parity checks")
            sys.path.insert(0, os.path.join(REPO, "tools"))
            import bench_parity
            t_par = time.perf_counter()
            line["parity"] = bench_parity.run(
                gpu, flags, {k: v.name for k, v in kept.items()})
            line["parity"]["wall_s"] = time.perf_counter() - t_par
            parity_failed = not line["parity"]["all_ok"]
        for v in kept.values():
            v.cleanup()
        if not args.no_cpu_baseline and world == 1:
            log("CPU baseline")
            nw, rule = cpu_share()
            if args.cpu_workers:
                nw, rule = args.cpu_workers, "--cpu-workers"
            line["cpu_baseline"] = cpu_baseline(sol, setup, max(1, nw), rule,
                                                args.cpu_fit_slots, args.cpu_eval_slots)
            samples = line["cpu_baseline"].pop("_samples")
            if gpu_sample is not None:
                chk = _oracle_sample_check(samples, gpu_sample, setup["piercepoints"])
                line["cpu_baseline"]["oracle_check"] = chk
                line.setdefault("parity", {})["fit_oracle_sample"] = {
                    "max_err": chk["coef_max_abs_err"], "tol": chk["tol"],
                    "ok": chk["ok"], "slots": chk["slots"]}
                if "all_ok" in line["parity"]:
                    line["parity"]["all_ok"] = line["parity"]["all_ok"] and chk["ok"]
                parity_failed = parity_failed or not chk["ok"]
            if gpu_amp is not None:
                ach = _oracle_amp_check(amp_blocks(sol), gpu_amp, sol,
                                        setup["piercepoints"], amp["order"])
                line["cpu_baseline"]["oracle_amp_check"] = ach
                line.setdefault("parity", {})["fit_oracle_amplitude_blocks"] = {
                    "max_err": ach["coef_max_abs_err"], "tol": ach["tol"],
                    "ok": ach["ok"], "slots": ach["slots"]}
                if "all_ok" in line["parity"]:
                    line["parity"]["all_ok"] = line["parity"]["all_ok"] and ach["ok"]
                parity_failed = parity_failed or not ach["ok"]
            # BASELINE.json configs[0] / [1]: the CPU path of make_aterm_image
            # on one core, next to fits_wallclock.config1 / config2
            if not args.no_cpu_reference_path:
                legs = cpu_reference_path()
                fw = line.get("fits_wallclock", {})
                for k, v in legs.items():
                    if k in fw and "wall_s" in v:
                        v["gpu_fits_wall_s"] = fw[k]["wall_s"]
                        v["gpu_speedup"] = v["wall_s"] / fw[k]["wall_s"]
                line["cpu_baseline"]["legs"] = legs
        # the child legs' own oracle samples (their CPU baseline legs)
        if side:
            parity_failed = child_leg_parity(side, line) or parity_failed
        line["library"] = dict(library_identity(), stale_counter_tables=dict(STALE_COUNTERS))
        print(json.dumps(line), flush=True)
    # release the CU-masked stream before the HIP runtime tears down
    torch.cuda.synchronize(dev)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for h in (masked_handle, fit_handle):
        if h is not None:
            ctx.stream_destroy(h)
    if dist.is_initialized():
        # every rank waits for rank 0's line (parity included) before the
        # group goes away
        dist.barrier()
        dist.destroy_process_group()
    if parity_failed:
        log("PARITY FAILED: see the line's 'parity' object")
        raise SystemExit(3)


if __name__ == "__main__":
    main()

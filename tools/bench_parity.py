"""Parity evidence carried by every bench.py line (``parsed.parity``).

Runs outside the timed region, on the product path (the HIP library through
its C ABI and the drop-in ``make_aterm_image``), against the committed
golden data ONLY -- reference outputs generated in the build container by
``tests/golden/make_golden*.py`` and the reference's own rendering
(``tests/golden/screens_png.npz``).  Nothing here imports ``oracle/``; every
expected value is a file the reference produced.

Checks (each reported as ``{max_err, tol, ok, ...}``):

* ``fit_config2`` / ``fit_synth20`` / ``fit_synth50``: the batched KL fit
  (stationscreen.py:433-782: ``_fit_screen``, ``_process_station`` with its
  outlier flags and order adaptation; the round-4 subset Jacobi runs for
  every flagged mask of the synth sets) on the fixture of configs 1-2 and the
  two reference-run synthetic sets: adapted orders and flagged weights
  bit-equal, coefficients and residuals within 1e-8 (x max(1, |coef|max)).
  None of these three sets has an ill-conditioned slot (an atan2 of
  near-zero values where the reference itself is chaotic;
  ``tests/test_bench_parity.py`` pins that the exclusion list is empty).
* ``eval17``: the KL evaluation (kl_screen.py:411-449 + the cos / sin planes
  of :313-380) of the reference-golden coefficients at 17^2 vs the
  reference's own evaluated planes -- D = 7 and 20 on the fp64 MFMA
  contraction, D = 50 on the integer-digit one -- 2e-6 with the fast sincos
  epilogue the bench runs.
* ``config1``: the tessellated FITS cube of make_aterm_image
  (tests/test_fit_screens.py:43-128 with abs(): 1e-4 at the in-image patch
  pixels), its header cards vs the reference's, and plane [t 0, f 3, ant 1,
  Im XX] (and the KL panel beside it, from the reference-golden
  coefficients) vs the colours of the reference's rendered
  resources/screens_.png (scripts/analyze_screens.py:97-223): every one of
  the 2 x 289 pixels must map to the rendered colour.
* ``config2``: the KL 128^2 FITS cube (tests/test_fit_screens.py:131-215
  with abs(): 1e-1 at the patch pixels), the reference's evaluated planes at
  (t 4:6; f, station (3, 7), (9, 44)) within 1e-6, planes 2 / 3 equal to
  0 / 1, and the header cards.
* ``fit_amplitude_gain12`` / ``fit_tec14``: the other soltab types of
  ``stationscreen.run`` against the reference's own fits of them
  (make_golden_gain.py / make_golden_tec.py): the log10-amplitude fit as
  KLScreen.fit calls it (kl_screen.py:96-125: niter 3, the block-coupled
  outlier sigma Q6, both pols) and the tec fit with the reference station and
  with ref_ant = -1 (the precedence quirk Q15); same criteria as the phase fit.
* ``gain_cube``: make_aterm_image on the gain solution set ("gain000" ->
  phase000 + amplitude000: both fits, Screen.interpolate, the three-screen
  evaluation with 10 **, kl_screen.py:319-378) vs the reference's
  make_matrix planes, |d| <= 2e-6 x max(1, |value|).
"""

import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))

FIT_SETS = {"fit_config2": "fixture_kl", "fit_synth20": "synth20",
            "fit_synth50": "synth50"}
FIT_TOL = 1e-8
EVAL_TOL_FAST = 2e-6
PATCH_TOL = {"config1": 1e-4, "config2": 1e-1}
CELL = {"config1": 0.2, "config2": 0.02602}
GRID = {"config1": 17, "config2": 128}
SMOOTH_PIX_CONFIG1 = 0.5  # smooth_deg 0.1 / cellsize 0.2 (screen.py:353-362)


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def _entry(max_err, tol, **kw):
    ok = bool(np.isfinite(max_err) and max_err <= tol)
    for k, v in kw.items():
        if isinstance(v, bool) or k.endswith("_equal"):
            ok = ok and bool(v)
    return dict(max_err=float(max_err), tol=tol, ok=ok, **kw)


def fit_check(ctx, torch, dev, name):
    """GPU fit of a golden set vs the reference's fit of it."""
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    g = golden(name)
    ref = int(g["ref_ant"])
    st = station_orders(g["ant_pos"], ref, int(g["order"]))
    ctx.set_basis(g["piercepoints"])
    T, F, A, D = g["val"].shape
    ph = torch.from_numpy(np.ascontiguousarray(g["val"])).to(dev)
    wt = torch.from_numpy(np.ascontiguousarray(g["weight"])).to(dev)
    coef, resid = torch.empty_like(ph), torch.empty_like(ph)
    w_out = torch.empty_like(wt)
    order = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    ctx.fit(ph, wt, T, F, A, st, niter=2, nsigma=5.0, adjust_order=True,
            ref_ant=ref, coef=coef, resid=resid, w_out=w_out, order_out=order)
    torch.cuda.synchronize(dev)
    coef, resid = coef.cpu().numpy(), resid.cpu().numpy()
    w_out, order = w_out.cpu().numpy(), order.cpu().numpy()
    scale = max(1.0, float(np.abs(g["coef"]).max()))
    cerr = float(np.abs(coef - g["coef"]).max()) / scale
    rerr = float(np.abs(resid - g["resid"]).max())
    return _entry(max(cerr, rerr), FIT_TOL,
                  coef_max_err_scaled=cerr, resid_max_err=rerr,
                  orders_equal=bool(np.array_equal(order, g["orders"])),
                  flags_equal=bool(np.array_equal(w_out.view(np.uint32),
                                                  g["w_out"].view(np.uint32))),
                  slots=int(T * F * A), n_dir=int(D),
                  flagged_entries=int((g["w_out"] == 0).sum()),
                  adapted_orders=int(len(np.unique(g["orders"]))))


def _fit_entry(got, want, tol=FIT_TOL):
    """(coef, resid, w_out, orders) vs the reference's."""
    coef, resid, w_out, orders = got
    wc, wr, ww, wo = want
    scale = max(1.0, float(np.abs(wc).max()))
    cerr = float(np.abs(coef - wc).max()) / scale
    rerr = float(np.abs(resid - wr).max())
    return dict(cerr=cerr, rerr=rerr, orders_equal=bool(np.array_equal(orders, wo)),
                flags_equal=bool(np.array_equal(w_out.view(np.uint32),
                                                np.ascontiguousarray(ww).view(np.uint32))))


def _device_fit(ctx, torch, dev, val, weight, st, **kw):
    T, F, A, D = val.shape
    v = torch.from_numpy(np.ascontiguousarray(val)).to(dev)
    w = torch.from_numpy(np.ascontiguousarray(weight)).to(dev)
    coef, resid = torch.zeros_like(v), torch.zeros_like(v)
    w_out = torch.empty_like(w)
    orders = torch.zeros((T, F, A), dtype=torch.int32, device=dev)
    ctx.fit(v, w, T, F, A, st, coef=coef, resid=resid, w_out=w_out,
            order_out=orders, **kw)
    torch.cuda.synchronize(dev)
    return (coef.cpu().numpy(), resid.cpu().numpy(), w_out.cpu().numpy(),
            orders.cpu().numpy())


def _merge(parts, **kw):
    cerr = max(p["cerr"] for p in parts)
    rerr = max(p["rerr"] for p in parts)
    return _entry(max(cerr, rerr), FIT_TOL, coef_max_err_scaled=cerr, resid_max_err=rerr,
                  orders_equal=all(p["orders_equal"] for p in parts),
                  flags_equal=all(p["flags_equal"] for p in parts), **kw)


def amplitude_check(ctx, torch, dev):
    """The amplitude stationscreen.run of gain12 (both pols, niter 3, no
    reference station, order min(12, max(3, round(D / 2))), kl_screen.py:
    96-125) vs the reference's."""
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE
    g = golden("gain12")
    ctx.set_basis(g["piercepoints"])
    T, F, A, D, P = g["amp_val"].shape
    order = int(g["amp_order"])
    parts = []
    for p in range(P):
        got = _device_fit(ctx, torch, dev, g["amp_val"][..., p], g["amp_weight"][..., p],
                          [order] * A, screen_type=SF_SCREEN_AMPLITUDE, niter=3,
                          nsigma=5.0, adjust_order=True, ref_ant=-1)
        parts.append(_fit_entry(got, (g["amp_coef"][..., p], g["amp_resid"][..., p],
                                      g["amp_w_out"][..., p], g["amp_orders"][..., p])))
    return _merge(parts, slots=int(T * F * A * P), n_dir=int(D),
                  flagged_entries=int((g["amp_w_out"] == 0).sum()))


def tec_check(ctx, torch, dev):
    """The tec stationscreen.run of tec14, with the reference station and
    with ref_ant = -1 (quirk Q15), vs the reference's."""
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_TEC
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    g = golden("tec14")
    ctx.set_basis(g["piercepoints"])
    parts = []
    for case in ("ref", "noref"):
        ref = int(g[f"{case}_ref_ant"])
        st = station_orders(g["ant_pos"], ref, int(g["order"]))
        got = _device_fit(ctx, torch, dev, g["val"], g["weight"], st,
                          screen_type=SF_SCREEN_TEC, niter=int(g["niter"]), nsigma=5.0,
                          adjust_order=True, ref_ant=ref)
        parts.append(_fit_entry(got, tuple(g[f"{case}_{k}"] for k in
                                           ("coef", "resid", "w_out", "orders"))))
    T, F, A, D = g["val"].shape
    return _merge(parts, slots=int(2 * T * F * A), n_dir=int(D), cases=["ref", "noref"])


def gain_cube_check(outdir):
    """make_aterm_image of the gain set (KL, 17^2) vs the reference's
    make_matrix planes at its golden (freq, station) pairs."""
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    g = golden("gain12")
    outroot = os.path.join(outdir, "gain")
    make_aterm_image(os.path.join(GOLDEN, "gain12.npz"), soltabname="gain000",
                     screen_type="kl", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50], skymodel=None,
                     padding_fraction=0, cellsize_deg=0.2, ncpu=0)
    _, cube = sffits.read_cube(outroot + "_0.fits")
    err = 0.0
    for k, (f, a) in enumerate(g["pairs"]):
        ref = g["gain17"][k]
        err = max(err, float((np.abs(cube[:, f, a] - ref) / np.maximum(1.0, np.abs(ref))).max()))
    return _entry(err, EVAL_TOL_FAST, shape_ok=tuple(cube.shape) == (8, 3, 5, 4, 17, 17),
                  pairs=[[int(v) for v in fa] for fa in g["pairs"]])


def eval17_check(ctx, torch, dev, flags):
    """The reference-golden coefficients evaluated at 17^2 vs the
    reference's evaluated cos / sin planes (every golden set)."""
    worst, per = 0.0, {}
    for name in ("fixture_kl", "synth20", "synth50"):
        g = golden(name)
        ctx.set_basis(g["piercepoints"])
        ctx.set_grid(g["x17"], g["y17"])
        err = 0.0
        for k, (f, s) in enumerate(g["pairs17"]):
            c = torch.from_numpy(np.ascontiguousarray(g["coef"][:, f, s, :])).to(dev)
            T = c.shape[0]
            out = torch.empty((T, 4, 17, 17), dtype=torch.float32, device=dev)
            ctx.eval(c, T, out, T, flags)
            torch.cuda.synchronize(dev)
            o = out.cpu().numpy().astype(np.float64)
            err = max(err, float(np.abs(o[:, 0:2] - g["kl17"][k]).max()),
                      float(np.abs(o[:, 2:4] - g["kl17"][k]).max()))
        per[name] = {"max_err": err, "n_dir": int(g["coef"].shape[-1]),
                     "contraction": ctx.eval_contraction(flags),
                     "slots": int(len(g["pairs17"]) * g["coef"].shape[0])}
        worst = max(worst, err)
    return _entry(worst, EVAL_TOL_FAST, sets=per)


def _header_check(hdr, grid):
    want = json.load(open(os.path.join(GOLDEN, "fixture_headers.json")))[str(grid)]
    bad = []
    for k, v in want:
        got = hdr.get(k)
        if isinstance(v, float):
            same = isinstance(got, (int, float)) and abs(got - v) <= 1e-15 * abs(v)
        elif k in ("SIMPLE", "EXTEND"):
            same = got is True
        else:
            same = got == v
        if not same:
            bad.append(k)
    return bad


def _patch_pixels(g, grid, cell):
    from ska_sdp_screen_fitting_amd.geometry import sin_world2pix
    c = grid / 2.0
    px, py = sin_world2pix(g["radec_patch"][:, 0], g["radec_patch"][:, 1],
                           (126.23, 64.5), (c, c), (-cell, cell))
    return px, py


def patch_criterion(cube, g, grid, cell):
    """tests/test_fit_screens.py:103-128 / :190-215 (ref antenna 0), with
    abs(): max |cube[..., p, row, col] - {cos, sin}(phase_corr)| over the
    in-image patch pixels."""
    ph = np.asarray(g["val"])
    corr = ph - ph[:, :, 0:1, :]
    px, py = _patch_pixels(g, grid, cell)
    err, n_in = 0.0, 0
    for i in range(len(px)):
        col, row = int(np.round(px[i])), int(np.round(py[i]))
        if 0 <= row < grid and 0 <= col < grid:
            n_in += 1
            for p, fn in ((0, np.cos), (1, np.sin), (2, np.cos), (3, np.sin)):
                v = np.asarray(cube[:, :, :, p, row, col], np.float64)
                err = max(err, float(np.abs(v - fn(corr[..., i])).max()))
    return err, n_in


def _colours(arr, vmin, vmax, lut):
    """matplotlib Normalize + the 256-entry viridis lookup -> RGB bytes."""
    u = (np.asarray(arr, np.float64) - vmin) / (vmax - vmin)
    return lut[np.clip(np.floor(u * 256.0), 0, 255).astype(int)]


def png_select():
    """The rendered slot (t, f, a, pol) and its phases referenced to the
    fixture's reference station (analyze_screens.get_phase_corrected)."""
    p = golden("screens_png")
    g = golden("fixture_kl")
    t, f, a, pol = (int(v) for v in p["select"])
    ph = g["val"][t, f, a, :] - g["val"][t, f, int(g["ref_ant"]), :]
    return (t, f, a, pol), ph


def png_mismatch(vor, kl, ph):
    """Pixels of the two 17^2 panels whose viridis colour differs from the
    rendered resources/screens_.png; vmin / vmax as get_boundaries
    (scripts/analyze_screens.py:13-66: both panels and values_kl[s])."""
    p = golden("screens_png")
    scalar = np.sin(ph[1])
    vmin = min(kl.min(), vor.min(), scalar)
    vmax = max(kl.max(), vor.max(), scalar)
    bad_vor = int((_colours(vor, vmin, vmax, p["lut"]) != p["vor_rgb"]).any(-1).sum())
    bad_kl = int((_colours(kl, vmin, vmax, p["lut"]) != p["kl_rgb"]).any(-1).sum())
    return bad_vor, bad_kl


def png_check(cube, ctx, torch, dev, flags):
    """Plane [t, f, a, Im XX] of the config-1 cube and the KL panel beside
    it (the reference-golden coefficients evaluated by the HIP kernel at
    17^2) vs the reference's rendered colours (screens_.png)."""
    (t, f, a, pol), ph = png_select()
    g = golden("fixture_kl")
    vor = np.asarray(cube[t, f, a, pol], np.float32)
    ctx.set_basis(g["piercepoints"])
    ctx.set_grid(g["x17"], g["y17"])
    c = torch.from_numpy(np.ascontiguousarray(g["coef"][t, f, a][None])).to(dev)
    out = torch.empty((1, 4, 17, 17), dtype=torch.float32, device=dev)
    ctx.eval(c, 1, out, 1, flags)
    torch.cuda.synchronize(dev)
    kl = out.cpu().numpy()[0, pol]
    bad_vor, bad_kl = png_mismatch(vor, kl, ph)
    return {"select": [t, f, a, pol], "pixels": 2 * vor.size,
            "mismatched_tessellated": bad_vor, "mismatched_kl": bad_kl}


def make_cube(name, outdir):
    """make_aterm_image of config 1 / 2 on the fixture into ``outdir``."""
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    st = "tessellated" if name == "config1" else "kl"
    make_aterm_image(os.path.join(GOLDEN, "fixture_kl.npz"), soltabname="phase000",
                     screen_type=st, outroot=os.path.join(outdir, name),
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50],
                     skymodel=os.path.join(GOLDEN, "skymodel.txt"),
                     padding_fraction=0, cellsize_deg=CELL[name],
                     smooth_deg=0.1 if name == "config1" else 0.0, ncpu=0)


def cube_check(name, outdir, ctx, torch, dev, flags):
    """Checks of the config-1 / config-2 FITS cube make_aterm_image wrote
    into ``outdir`` (``{outdir}/{name}_0.fits``)."""
    from ska_sdp_screen_fitting_amd import fits as sffits
    grid, cell = GRID[name], CELL[name]
    path = os.path.join(outdir, f"{name}_0.fits")
    files = sorted(f for f in os.listdir(outdir) if f.endswith(".fits")
                   and f.startswith(name + "_") and f != f"{name}_template.fits")
    hdr, cube = sffits.read_cube(path, mmap=True)
    g = golden("fixture_kl")
    shape_ok = tuple(cube.shape) == (20, 12, 62, 4, grid, grid)
    bad_hdr = _header_check(hdr, grid)
    perr, n_in = patch_criterion(cube, g, grid, cell)
    res = {"patch_criterion": {"max_err": perr, "tol": PATCH_TOL[name],
                               "in_image_patches": n_in,
                               "ok": bool(perr < PATCH_TOL[name] and n_in >= 5)},
           "header_cards_mismatched": bad_hdr, "files": files, "shape_ok": shape_ok}
    ok = res["patch_criterion"]["ok"] and not bad_hdr and shape_ok and len(files) == 1
    if name == "config1":
        png = png_check(cube, ctx, torch, dev, flags)
        png["ok"] = png["mismatched_tessellated"] == 0 and png["mismatched_kl"] == 0
        res["screens_png"] = png
        ok = ok and png["ok"]
        res.update(max_err=perr, tol=PATCH_TOL[name])
    else:
        t0, t1 = (int(v) for v in g["kl128_t"])
        err, same34 = 0.0, True
        for k, (f, s) in enumerate(g["pairs128"]):
            got = np.asarray(cube[t0:t1, f, s], np.float64)
            err = max(err, float(np.abs(got[:, 0:2] - g["kl128"][k]).max()))
            same34 = same34 and bool(np.array_equal(got[:, 2:4], got[:, 0:2]))
        res["golden_planes"] = {"max_err": err, "tol": 1e-6, "ok": err <= 1e-6,
                                "planes_2_3_equal_0_1": same34,
                                "slices": "t %d:%d, (f, station) %s" % (
                                    t0, t1, [tuple(int(v) for v in fs) for fs in g["pairs128"]])}
        ok = ok and err <= 1e-6 and same34
        res.update(max_err=err, tol=1e-6)
    del cube
    res["ok"] = bool(ok)
    return res


def run(device, flags, cube_dirs=None):
    """All checks on ``device`` with a context of their own (the bench's
    context keeps its basis and grid).  ``cube_dirs``: {config1 / config2:
    directory holding the cube the FITS wall-clock leg wrote}; a cube not
    given is produced here (untimed).  Returns the ``parity`` object."""
    import torch
    from ska_sdp_screen_fitting_amd._lib import Context
    dev = torch.device("cuda", device)
    ctx = Context(device)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    res = {}
    try:
        for key, name in FIT_SETS.items():
            res[key] = fit_check(ctx, torch, dev, name)
        res["eval17"] = eval17_check(ctx, torch, dev, flags)
        res["fit_amplitude_gain12"] = amplitude_check(ctx, torch, dev)
        res["fit_tec14"] = tec_check(ctx, torch, dev)
        with tempfile.TemporaryDirectory() as tmp:
            res["gain_cube"] = gain_cube_check(tmp)
        for name in ("config1", "config2"):
            d = (cube_dirs or {}).get(name)
            if d is not None:
                res[name] = cube_check(name, d, ctx, torch, dev, flags)
                res[name]["cube_from"] = "fits_wallclock leg"
                continue
            with tempfile.TemporaryDirectory() as tmp:
                make_cube(name, tmp)
                res[name] = cube_check(name, tmp, ctx, torch, dev, flags)
                res[name]["cube_from"] = "make_aterm_image run for this check"
    except Exception as exc:  # a crash is a failed check, reported
        res["error"] = f"{type(exc).__name__}: {exc}"
    finally:
        ctx.close()
    res["all_ok"] = "error" not in res and all(
        v.get("ok") for k, v in res.items() if isinstance(v, dict))
    return res

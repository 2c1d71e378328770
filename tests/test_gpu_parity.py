"""HIP path (through the C ABI) vs the reference's golden vectors and the
oracle.  Needs an MI355X: every test is marked ``gpu``.

Tolerances (stated per north_star):
  * fit coefficients / residuals: |d| <= 1e-8 x max(1, |coef|max) (float64
    Jacobi/Cholesky vs LAPACK SVD; rounding-level), orders and flagged
    weights identical;
  * evaluated planes (float32 output of a float64 contraction): |d| <= 1e-6
    vs the reference's float64 cos/sin (fp64 sincos epilogue), 2e-6 with
    SF_EVAL_FAST_SINCOS.
"""

import os
import tempfile

import numpy as np
import pytest

from conftest import FIELD, GOLDEN, load_golden
from oracle import kl as okl

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ctx(dev):
    from ska_sdp_screen_fitting_amd import get_context
    c = get_context(0)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    return c


def gpu_fit(ctx, dev, g, **kw):
    ref = int(g["ref_ant"])
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    st = station_orders(g["ant_pos"], ref, int(g["order"]))
    ctx.set_basis(g["piercepoints"])
    T, F, A, D = g["val"].shape
    ph = torch.from_numpy(np.ascontiguousarray(g["val"])).to(dev)
    wt = torch.from_numpy(np.ascontiguousarray(g["weight"])).to(dev)
    coef = torch.empty_like(ph)
    resid = torch.empty_like(ph)
    w_out = torch.empty_like(wt)
    order = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    ctx.fit(ph, wt, T, F, A, st, ref_ant=ref, coef=coef, resid=resid,
            w_out=w_out, order_out=order, **kw)
    torch.cuda.synchronize()
    return (coef.cpu().numpy(), resid.cpu().numpy(), w_out.cpu().numpy(),
            order.cpu().numpy())


def test_basis_vs_oracle(ctx, golden):
    g = golden
    ctx.set_basis(g["piercepoints"])
    c, pinv, u, eig = ctx.get_basis()
    np.testing.assert_allclose(c, g["C"], rtol=1e-13, atol=0)
    sv = np.linalg.svd(g["C"], compute_uv=False)
    cond = sv.max() / sv[sv > 1e-3].min()
    np.testing.assert_allclose(pinv, g["pinv_c"], rtol=0,
                               atol=1e-13 * cond * np.abs(g["pinv_c"]).max())
    np.testing.assert_allclose(np.abs(eig), sv, rtol=1e-12, atol=1e-12 * sv.max())
    np.testing.assert_allclose(np.abs(u.T @ g["U"]), np.eye(len(sv)), atol=1e-9)


def _ill_conditioned(g):
    from test_oracle_golden import ill_conditioned_slots
    return ill_conditioned_slots(g)


def test_fit_vs_reference_golden(ctx, dev, golden):
    g = golden
    coef, resid, w_out, orders = gpu_fit(ctx, dev, g)
    np.testing.assert_array_equal(orders, g["orders"])
    np.testing.assert_array_equal(w_out, g["w_out"])
    err = np.abs(coef - g["coef"]).max(axis=-1)
    scale = max(1.0, np.abs(g["coef"]).max())
    bad = {tuple(i) for i in np.argwhere(err > 1e-8 * scale)}
    assert bad <= _ill_conditioned(g), sorted(bad)[:10]
    keep = np.ones(err.shape, bool)
    for i in bad:
        keep[i] = False
    print(g["name"], "max coef err", err[keep].max(), "scale", scale)
    rerr = np.abs(resid - g["resid"]).max(axis=-1)
    assert rerr[keep].max() <= 1e-8


@pytest.mark.parametrize("name", ["synth20", "synth50", "synth12tiny"])
def test_fit_fast_equals_general_path(ctx, dev, name):
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_GENERAL
    g = load_golden(name)
    fast = gpu_fit(ctx, dev, g)
    ctx.set_option(SF_OPT_FIT_GENERAL, 1)
    try:
        gen = gpu_fit(ctx, dev, g)
    finally:
        ctx.set_option(SF_OPT_FIT_GENERAL, 0)
    np.testing.assert_array_equal(fast[3], gen[3])
    np.testing.assert_array_equal(fast[2], gen[2])
    bad = _ill_conditioned(g)
    keep = np.ones(fast[0].shape[:3], bool)
    for i in bad:
        keep[i] = False
    np.testing.assert_allclose(fast[0][keep], gen[0][keep], rtol=0, atol=1e-9)


def _wave_count_case(name):
    if name != "config5-density":
        return load_golden(name)
    # config 5's flag density at D = 50: 1 % of (slot, dir) entries zero,
    # 0.5 % outliers (flagged in pass 1) -- hundreds of distinct masks
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=12, n_time=40, n_freq=2, n_dir=50, seed=55,
                       flag_frac=0.01, outlier_frac=0.005)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    return dict(val=s.val, weight=s.weight, ant_pos=s.ant_pos, piercepoints=pp,
                ref_ant=okl.reference_station(s.weight), order=20)


@pytest.mark.parametrize("name", ["synth50", "config5-density", "synth20"])
def test_subset_jacobi_wave_count_is_bit_identical(ctx, dev, name):
    """The subset-basis Jacobi (kl_subset_eig_kernel -> wg_jacobi<NW>,
    stationscreen.py:390-430 / :495-499 per flagged mask) on 1, 2, 3 (the
    default) and 4 waves per mask: the same pool of subset bases, bit for
    bit, and the same orders, flags, coefficients and residuals."""
    from ska_sdp_screen_fitting_amd._lib import (SF_OPT_FIT_EIG_WAVES,
                                                 SF_OPT_FIT_SUBSET_DELETION)
    g = _wave_count_case(name)
    runs = {}
    # the Jacobi solve for every mask (the deletions are the default)
    ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 0)
    try:
        for nw in (3, 1, 2, 4):
            ctx.set_option(SF_OPT_FIT_EIG_WAVES, nw)
            out = gpu_fit(ctx, dev, g)
            runs[nw] = (out, ctx.fit_pool())
    finally:
        ctx.set_option(SF_OPT_FIT_EIG_WAVES, 0)
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 1)
    (ref_out, (ref_masks, ref_pool)) = runs[3]
    assert len(ref_masks) > (100 if name == "config5-density" else 0)
    assert len(np.unique(ref_masks)) == len(ref_masks)
    for nw, (out, (masks, pool)) in runs.items():
        assert np.array_equal(masks, ref_masks), nw
        assert np.array_equal(pool.view(np.uint64), ref_pool.view(np.uint64)), nw
        for a, b in zip(out, ref_out):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), nw


@pytest.mark.parametrize("name", ["synth20", "synth12tiny", "fixture_kl"])
def test_fit_two_slots_per_wave_is_bit_identical(ctx, dev, name):
    """Two slots per wavefront (D <= 32) must not change a single bit: the
    group reductions add in the same order as the 64-lane ones."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_PACK
    g = load_golden(name)
    packed = gpu_fit(ctx, dev, g)
    ctx.set_option(SF_OPT_FIT_PACK, 0)
    try:
        single = gpu_fit(ctx, dev, g)
    finally:
        ctx.set_option(SF_OPT_FIT_PACK, 1)
    for a, b in zip(packed, single):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("name", ["synth20", "synth50", "synth12tiny", "fixture_kl"])
def test_fit_lean_layout_is_bit_identical(ctx, dev, name):
    """The lean pass layout (uniform weights: no per-slot G / subset-basis
    copies in LDS, subset bases read from the pool) must not change a bit;
    sets with unequal weights (synth12tiny) keep the general layout by the
    classify count, so the two runs must agree there too."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_LEAN
    g = load_golden(name)
    lean = gpu_fit(ctx, dev, g)
    ctx.set_option(SF_OPT_FIT_LEAN, 0)
    try:
        general = gpu_fit(ctx, dev, g)
    finally:
        ctx.set_option(SF_OPT_FIT_LEAN, 1)
    for a, b in zip(lean, general):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_fit_vs_oracle_config3_shape(ctx, dev):
    """A larger config-3-shaped synthetic (flags, outliers, adapted orders)."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=8, n_time=24, n_freq=3, n_dir=20, seed=99,
                       flag_frac=0.02, outlier_frac=0.01)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    ref = okl.reference_station(s.weight)
    g = dict(val=s.val, weight=s.weight, ant_pos=s.ant_pos, piercepoints=pp,
             ref_ant=ref, order=19)
    coef, resid, w_out, orders = gpu_fit(ctx, dev, g)
    r = okl.run_phase(s.val, s.weight, s.ant_pos, pp, ref, 19)
    np.testing.assert_array_equal(orders, r["orders"])
    np.testing.assert_array_equal(w_out, r["w_out"])
    np.testing.assert_allclose(coef, r["coef"], rtol=0,
                               atol=1e-8 * max(1.0, np.abs(r["coef"]).max()))
    np.testing.assert_allclose(resid, r["resid"], rtol=0, atol=1e-8)


def test_fit_vs_oracle_max_directions(ctx, dev):
    """D = SF_MAX_DIR (60, the ABI's limit): the largest k-step count, one
    slot per wavefront, subset bases of up to 59 directions; orders and flags
    identical to the oracle, coefficients within 1e-8."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import SF_MAX_DIR
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=4, n_time=6, n_freq=2, n_dir=SF_MAX_DIR, seed=60,
                       flag_frac=0.02, outlier_frac=0.01)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    ref = okl.reference_station(s.weight)
    g = dict(val=s.val, weight=s.weight, ant_pos=s.ant_pos, piercepoints=pp,
             ref_ant=ref, order=20)
    coef, resid, w_out, orders = gpu_fit(ctx, dev, g)
    r = okl.run_phase(s.val, s.weight, s.ant_pos, pp, ref, 20)
    np.testing.assert_array_equal(orders, r["orders"])
    np.testing.assert_array_equal(w_out, r["w_out"])
    np.testing.assert_allclose(coef, r["coef"], rtol=0,
                               atol=1e-8 * max(1.0, np.abs(r["coef"]).max()))
    np.testing.assert_allclose(resid, r["resid"], rtol=0, atol=1e-8)


def test_empty_and_out_of_range_inputs(ctx, dev):
    """S = 0 writes nothing and succeeds (eval, eval_sums, tess_fill);
    D > SF_MAX_DIR is refused with SF_EINVAL before any allocation."""
    from ska_sdp_screen_fitting_amd._lib import SF_MAX_DIR, ScreenFitError
    pp = np.stack([np.linspace(-900, 900, 6), np.linspace(300, -300, 6), np.zeros(6)], 1)
    ctx.set_basis(pp)
    x = np.linspace(-500, 500, 16)
    ctx.set_grid(x, x)
    coef = torch.zeros((1, 6), dtype=torch.float64, device=dev)
    out = torch.full((1, 4, 16, 16), -7.0, dtype=torch.float32, device=dev)
    sums = torch.zeros(1, dtype=torch.int32, device=dev)
    ctx.eval(coef, 0, out, 1)
    ctx.eval_sums(coef, 0, out, sums, 1)
    labels = torch.ones((16, 16), dtype=torch.int32, device=dev)
    ctx.tess_fill(labels, 16, 16, coef, 6, 0, out, 1)
    torch.cuda.synchronize()
    assert bool((out == -7.0).all()) and int(sums[0]) == 0
    big = np.zeros((SF_MAX_DIR + 1, 3))
    big[:, 0] = np.arange(SF_MAX_DIR + 1) * 10.0
    with pytest.raises(ScreenFitError):
        ctx.set_basis(big)
    ctx.set_basis(pp)  # the context stays usable


def test_fit_sharded_equals_unsharded(ctx, dev):
    """ant shards with the reference phases passed in (ref not local)."""
    g = load_golden("synth20")
    coef_all, resid_all, w_all, ord_all = gpu_fit(ctx, dev, g)
    ref = int(g["ref_ant"])
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    st = station_orders(g["ant_pos"], ref, int(g["order"]))
    T, F, A, D = g["val"].shape
    refph = torch.from_numpy(np.ascontiguousarray(g["val"][:, :, ref, :])).to(dev)
    for a0, a1 in ((0, 2), (2, 4), (4, 6)):
        ph = torch.from_numpy(np.ascontiguousarray(g["val"][:, :, a0:a1])).to(dev)
        wt = torch.from_numpy(np.ascontiguousarray(g["weight"][:, :, a0:a1])).to(dev)
        coef = torch.empty_like(ph)
        ctx.fit(ph, wt, T, F, a1 - a0, st[a0:a1], ref_ant=ref, coef=coef,
                ant_offset=a0, ref_phase=refph)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(coef.cpu().numpy(), coef_all[:, :, a0:a1])


def gpu_eval(ctx, dev, pp, x, y, coef_slots, flags=1, ring=None):
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    c = torch.from_numpy(np.ascontiguousarray(coef_slots, np.float64)).to(dev)
    S = c.shape[0]
    R = S if ring is None else ring
    out = torch.full((R, 4, len(y), len(x)), -7.0, dtype=torch.float32, device=dev)
    ctx.eval(c, S, out, R, flags)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("fast", [False, True])
def test_eval_vs_reference_golden(ctx, dev, golden, fast):
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS
    g = golden
    tol = 1e-6
    flags = 1 | (SF_EVAL_FAST_SINCOS if fast else 0)
    for k, (f, s) in enumerate(g["pairs17"]):
        out = gpu_eval(ctx, dev, g["piercepoints"], g["x17"], g["y17"],
                       g["coef"][:, f, s, :], flags)
        ref = g["kl17"][k]  # [t, 2, y, x] float64
        np.testing.assert_allclose(out[:, 0], ref[:, 0], rtol=0, atol=tol)
        np.testing.assert_allclose(out[:, 1], ref[:, 1], rtol=0, atol=tol)
        np.testing.assert_array_equal(out[:, 2], out[:, 0])
        np.testing.assert_array_equal(out[:, 3], out[:, 1])


def test_eval_128_vs_reference_golden(ctx, dev):
    g = load_golden("fixture_kl")
    t0, t1 = g["kl128_t"]
    for k, (f, s) in enumerate(g["pairs128"]):
        out = gpu_eval(ctx, dev, g["piercepoints"], g["x128"], g["y128"],
                       g["coef"][t0:t1, f, s, :])
        np.testing.assert_allclose(out[:, 0:2], g["kl128"][k], rtol=0, atol=1e-6)


@pytest.mark.parametrize("n_dir,grid", [(20, 256), (50, 64), (7, 17), (3, 40),
                                        (60, 48), (2, 16)])
def test_eval_vs_oracle_sizes(ctx, dev, n_dir, grid):
    """Odd grids (scalar stores), every k-step count used by the configs."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=3)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    rng = np.random.default_rng(n_dir)
    coef = rng.normal(0, 0.01, size=(37, n_dir))  # 37: partial slot group
    out = gpu_eval(ctx, dev, pp, x, y, coef)
    cpix = okl.cpix_matrix(pp, x, y)
    want = okl.eval_planes(okl.eval_phase_screens(coef, cpix))
    np.testing.assert_allclose(out.reshape(want.shape), want, rtol=0, atol=1e-6)


@pytest.mark.parametrize("R", [13, 16, 21])
@pytest.mark.parametrize("fast", [False, True])
def test_eval_ring_and_nan_scrub(ctx, dev, R, fast):
    """Ring smaller than the slot count (the per-group ring offset with one
    wrap when R >= 16, the modulo when R < 16), NaN scrub on and off."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS
    g = load_golden("synth20")
    coef = g["coef"].reshape(-1, g["coef"].shape[-1])[:50].copy()
    coef[7, 3] = np.nan
    fl = 1 | (SF_EVAL_FAST_SINCOS if fast else 0)
    out = gpu_eval(ctx, dev, g["piercepoints"], g["x17"], g["y17"], coef, ring=R,
                   flags=fl)
    full = gpu_eval(ctx, dev, g["piercepoints"], g["x17"], g["y17"], coef, flags=fl)
    assert np.all(full[7, 0] == 1.0) and np.all(full[7, 1] == 0.0)
    # every value of a ring entry comes from one of the slots that map to it
    # (which one is unspecified: aliasing slots are stored concurrently, so
    # an entry can interleave them at store granularity)
    for r in range(R):
        cands = np.stack([full[s] for s in range(r, 50, R)])
        assert np.all(np.any(cands == out[r][None], axis=0)), r
    # without the scrub flag NaNs stay NaNs
    raw = gpu_eval(ctx, dev, g["piercepoints"], g["x17"], g["y17"], coef,
                   flags=fl & ~1)
    assert np.all(np.isnan(raw[7]))


def test_make_aterm_image_fixture_kl(tmp_path):
    """End-to-end drop-in on the reference's fixture (tests/test_fit_screens.py
    test_fit_kl_screens, with abs() and exact patch pixels)."""
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.geometry import sin_world2pix
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image

    g = load_golden("fixture_kl")
    outroot = str(tmp_path / "kl")
    make_aterm_image(os.path.join(GOLDEN, "fixture_kl.npz"), soltabname="phase000",
                     screen_type="kl", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50],
                     skymodel=os.path.join(GOLDEN, "skymodel.txt"),
                     solsetname="sol000", padding_fraction=0, cellsize_deg=0.2,
                     smooth_deg=0.1, ncpu=0)
    assert os.path.isfile(outroot + "_0.fits")
    assert os.path.isfile(str(tmp_path / "kl.txt"))
    hdr, cube = sffits.read_cube(outroot + "_0.fits")
    import json
    want_hdr = json.load(open(os.path.join(GOLDEN, "fixture_headers.json")))["17"]
    for k, v in want_hdr:
        if isinstance(v, float):
            assert hdr[k] == pytest.approx(v, rel=1e-15), k
        elif k in ("SIMPLE", "EXTEND"):
            assert hdr[k] is True
        else:
            assert hdr[k] == v, k
    # the reference's own values at the golden slots (fp32 tolerance)
    for k, (f, s) in enumerate(g["pairs17"]):
        np.testing.assert_allclose(cube[:, f, s, 0:2], g["kl17"][k], atol=1e-6)
    # the reference test criterion (threshold 1e-1), two-sided
    ph = np.asarray(g["val"])
    corr = ph - ph[:, :, 0:1, :]
    px, py = sin_world2pix(g["radec_patch"][:, 0], g["radec_patch"][:, 1],
                           (126.23, 64.5), (8.5, 8.5), (-0.2, 0.2))
    n_in = 0
    for i in range(len(px)):
        col, row = int(np.round(px[i])), int(np.round(py[i]))
        if 0 <= row < 17 and 0 <= col < 17:
            n_in += 1
            for p, fn in ((0, np.cos), (1, np.sin), (2, np.cos), (3, np.sin)):
                assert np.all(np.abs(cube[:, :, :, p, row, col] - fn(corr[..., i])) < 1e-1)
    assert n_in >= 5


def test_make_aterm_image_config2_kl128(tmp_path):
    """BASELINE config 2 end to end: make_aterm_image on the fixture, KL,
    cellsize 0.02602 deg (a 128^2 grid, 3.9 GB FITS cube): the reference's
    own evaluated planes at (t 4:6; f, station (3, 7), (9, 44)) within 1e-6,
    the reference's header cards, and its test criterion at the patch pixels
    (tests/test_fit_screens.py:131-215, with abs())."""
    import json
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.geometry import sin_world2pix
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image

    g = load_golden("fixture_kl")
    outroot = str(tmp_path / "kl128")
    make_aterm_image(os.path.join(GOLDEN, "fixture_kl.npz"), soltabname="phase000",
                     screen_type="kl", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50],
                     skymodel=os.path.join(GOLDEN, "skymodel.txt"),
                     solsetname="sol000", padding_fraction=0, cellsize_deg=0.02602,
                     ncpu=0)
    files = open(str(tmp_path / "kl128.txt")).read().split()
    assert files == [outroot + "_0.fits"]
    hdr, cube = sffits.read_cube(outroot + "_0.fits", mmap=True)
    assert cube.shape == (20, 12, 62, 4, 128, 128)
    want_hdr = json.load(open(os.path.join(GOLDEN, "fixture_headers.json")))["128"]
    for k, v in want_hdr:
        if isinstance(v, float):
            assert hdr[k] == pytest.approx(v, rel=1e-15), k
        elif k in ("SIMPLE", "EXTEND"):
            assert hdr[k] is True
        else:
            assert hdr[k] == v, k
    t0, t1 = g["kl128_t"]
    for k, (f, s) in enumerate(g["pairs128"]):
        got = np.asarray(cube[t0:t1, f, s, 0:2], np.float64)
        np.testing.assert_allclose(got, g["kl128"][k], rtol=0, atol=1e-6)
        # planes 2 / 3 repeat 0 / 1 for phase screens
        np.testing.assert_array_equal(np.asarray(cube[t0:t1, f, s, 2:4]),
                                      np.asarray(cube[t0:t1, f, s, 0:2]))
    ph = np.asarray(g["val"])
    corr = ph - ph[:, :, 0:1, :]
    px, py = sin_world2pix(g["radec_patch"][:, 0], g["radec_patch"][:, 1],
                           (126.23, 64.5), (64.0, 64.0), (-0.02602, 0.02602))
    np.testing.assert_allclose(np.stack([px, py]), g["patch_pix128"], atol=1e-9)
    n_in = 0
    for i in range(len(px)):
        col, row = int(np.round(px[i])), int(np.round(py[i]))
        if 0 <= row < 128 and 0 <= col < 128:
            n_in += 1
            for p, fn in ((0, np.cos), (1, np.sin), (2, np.cos), (3, np.sin)):
                err = np.abs(np.asarray(cube[:, :, :, p, row, col]) - fn(corr[..., i]))
                assert np.all(err < 1e-1), (i, p, err.max())
    assert n_in >= 5
    del cube


def test_kl_evaluators_own_their_context(ctx, dev):
    """Two KL evaluators of different bases on same-shaped grids, used
    alternately, and the process-wide context re-based in between (what a
    refit does): each keeps evaluating its own basis."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.kl_screen import KLEvaluator
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    evs, wants = [], []
    rng = np.random.default_rng(11)
    coef = rng.normal(0, 0.01, size=(9, 12))
    for seed in (1, 2):
        s = make_solutions(n_ant=2, n_time=1, n_freq=1, n_dir=12, seed=seed)
        pp, mra, mdec = geometry.piercepoints(s.dir_radec)
        x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                    0.2, mra, mdec)
        evs.append(KLEvaluator(pp, 100.0, 5.0 / 3.0, x, y, 0))
        cpix = okl.cpix_matrix(pp, x, y)
        wants.append(okl.eval_planes(okl.eval_phase_screens(coef, cpix)))
    for rep in range(2):
        for ev, want in zip(evs, wants):
            got = ev.eval_host(coef)
            np.testing.assert_allclose(got.reshape(want.shape), want, rtol=0, atol=2e-6)
        # the fit re-bases the shared context (and clears its grid)
        ctx.set_basis(np.stack([np.linspace(-900, 900, 5), np.zeros(5), np.zeros(5)], 1))


def test_kl_write_smoothing(ctx, dev):
    """KLScreen.write with smooth_pix > 0 (screen.py:353-378): evaluate, then
    the Gaussian, then the NaN scrub -- vs the oracle planes through scipy."""
    from oracle import voronoi as ov
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB
    from ska_sdp_screen_fitting_amd.kl_screen import KLEvaluator
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=1, n_freq=1, n_dir=9, seed=8)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                0.05, mra, mdec)
    ev = KLEvaluator(pp, 100.0, 5.0 / 3.0, x, y, 0)
    rng = np.random.default_rng(3)
    coef = rng.normal(0, 0.01, size=(6, 9))
    coef[2, 4] = np.nan
    c = torch.from_numpy(coef).to(dev)
    out = ev.eval_device(c, flags=SF_EVAL_FAST_SINCOS)
    ev.smooth_device(out, 2.5, SF_EVAL_NAN_SCRUB)
    torch.cuda.synchronize()
    planes = okl.eval_planes(okl.eval_phase_screens(coef, okl.cpix_matrix(pp, x, y)))
    want = ov.smooth(planes.reshape(6, 4, len(y), len(x)).astype(np.float32), 2.5)
    for p in range(4):
        v = want[:, p]
        v[np.isnan(v)] = 0.0 if p % 2 else 1.0
    np.testing.assert_allclose(out.cpu().numpy(), want, rtol=0, atol=2e-6)
    assert np.all(out[2, 0].cpu().numpy() == 1.0)


def test_make_aterm_image_from_h5parm_file(tmp_path):
    """The same drop-in call on a DP3-layout .h5 (built-in HDF5 reader) gives
    the same FITS cube as the .npz input."""
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    cubes = []
    for src, tag in ((os.path.join(GOLDEN, "fixture_kl.npz"), "npz"),
                     (os.path.join(GOLDEN, "h5", "dp3_like.h5"), "h5")):
        outroot = str(tmp_path / tag)
        make_aterm_image(src, soltabname="phase000", screen_type="kl",
                         outroot=outroot,
                         bounds_deg=[124.565, 66.165, 127.895, 62.835],
                         bounds_mid_deg=[126.23, 64.50],
                         skymodel=os.path.join(GOLDEN, "skymodel.txt"),
                         padding_fraction=0, cellsize_deg=0.2, ncpu=0)
        cubes.append(sffits.read_cube(outroot + "_0.fits")[1])
    np.testing.assert_array_equal(cubes[0], cubes[1])


@pytest.mark.parametrize("n_dir,grid", [(20, 256), (7, 128), (24, 60), (50, 64), (3, 40)])
def test_eval_kernels_agree(ctx, dev, n_dir, grid):
    """Every evaluation kernel (register-tile, LDS-staged 1/2/4 KiB runs;
    plain and non-temporal stores; big-endian) writes the same bits, and the
    fp32-sincos result is within 2e-6 of the oracle.  Ragged slot count,
    grids that are not a multiple of the store run, a NaN slot."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import (
        EVAL_KERNEL_NAMES, SF_EVAL_BIG_ENDIAN, SF_EVAL_FAST_SINCOS,
        SF_EVAL_KERNEL_AUTO, SF_EVAL_KERNEL_TILE, SF_EVAL_NT_STORES,
        SF_OPT_EVAL_BANDS, SF_OPT_EVAL_KERNEL, SF_OPT_EVAL_KS_PAD,
        SF_OPT_EVAL_MAX_BLOCKS, SF_OPT_EVAL_XCD_MAP)
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=4)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    rng = np.random.default_rng(n_dir + grid)
    coef = rng.normal(0, 0.01, size=(45, n_dir))
    coef[20:30] *= 300.0  # phases of many turns: the range reduction
    coef[9, n_dir // 2] = np.nan
    coef[31, 0] = np.inf
    base = 1 | SF_EVAL_FAST_SINCOS
    outs = {}
    try:
        for kv in sorted(EVAL_KERNEL_NAMES) + [SF_EVAL_KERNEL_AUTO]:
            ctx.set_option(SF_OPT_EVAL_KERNEL, kv)
            for extra in (0, SF_EVAL_NT_STORES, SF_EVAL_BIG_ENDIAN):
                o = gpu_eval(ctx, dev, pp, x, y, coef, flags=base | extra)
                if extra == SF_EVAL_BIG_ENDIAN:
                    o = o.byteswap()
                outs[(kv, extra)] = o
            # 8 workgroups walking every (pixel block, slot chunk) item: the
            # path large launches take past the 2^32 work-item dispatch limit
            ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 8)
            outs[(kv, "walk")] = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
            ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 0)
            # both workgroup -> pixel-block maps over the XCDs
            for xm in (0, 1):
                ctx.set_option(SF_OPT_EVAL_XCD_MAP, xm)
                outs[(kv, "xcd", xm)] = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
            ctx.set_option(SF_OPT_EVAL_XCD_MAP, -1)
            # band-major work-item order over 2 / 4 pixel bands
            for nb in (2, 4):
                ctx.set_option(SF_OPT_EVAL_BANDS, nb)
                outs[(kv, "bands", nb)] = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
            ctx.set_option(SF_OPT_EVAL_BANDS, 0)
            # zero k-step padding of the contraction
            ctx.set_option(SF_OPT_EVAL_KS_PAD, 2)
            outs[(kv, "pad")] = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
            ctx.set_option(SF_OPT_EVAL_KS_PAD, 0)
            # no NaN scrub: NaN / Inf slots stay NaN in every plane
            o = gpu_eval(ctx, dev, pp, x, y, coef, flags=SF_EVAL_FAST_SINCOS)
            assert np.isnan(o[[9, 31]]).all(), kv
            o[[9, 31]] = 0
            outs[(kv, "noscrub")] = o
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
        ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 0)
        ctx.set_option(SF_OPT_EVAL_XCD_MAP, -1)
        ctx.set_option(SF_OPT_EVAL_KS_PAD, 0)
        ctx.set_option(SF_OPT_EVAL_BANDS, 0)
    ref = outs[(SF_EVAL_KERNEL_TILE, 0)]
    for k, o in outs.items():
        if k[1] == "noscrub":
            o2 = o.copy()
            o2[[9, 31]] = ref[[9, 31]]
            assert np.array_equal(o2.view(np.int32), ref.view(np.int32)), k
        else:
            assert np.array_equal(o.view(np.int32), ref.view(np.int32)), k
    for k in (9, 31):
        assert np.all(ref[k, 0::2] == 1.0) and np.all(ref[k, 1::2] == 0.0)
    cpix = okl.cpix_matrix(pp, x, y)
    good = np.isfinite(coef).all(axis=1)
    want = okl.eval_planes(okl.eval_phase_screens(coef[good], cpix))
    np.testing.assert_allclose(ref[good].reshape(want.shape), want, rtol=0, atol=2e-6)


def test_eval_bands_512(ctx, dev):
    """512^2 x D = 50 (config 5's grid): the auto pixel bands of the register
    tile (8 bands of 128 blocks, interleaved XCD map), explicit 1 / 2 / 16
    bands and both maps, and the auto kernel write the same bits as the
    unbanded contiguous launch; sampled slots match the oracle."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import (
        SF_EVAL_FAST_SINCOS, SF_EVAL_KERNEL_AUTO, SF_EVAL_KERNEL_TILE,
        SF_OPT_EVAL_BANDS, SF_OPT_EVAL_KERNEL, SF_OPT_EVAL_XCD_MAP)
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    n_dir, grid = 50, 512
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=5)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    rng = np.random.default_rng(512)
    coef = rng.normal(0, 0.01, size=(37, n_dir))
    coef[7, 3] = np.nan
    base = 1 | SF_EVAL_FAST_SINCOS
    try:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_TILE)
        ctx.set_option(SF_OPT_EVAL_XCD_MAP, 0)
        ctx.set_option(SF_OPT_EVAL_BANDS, 1)
        ref = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
        for kv, xm, nb in ((SF_EVAL_KERNEL_TILE, -1, 0), (SF_EVAL_KERNEL_TILE, 1, 2),
                           (SF_EVAL_KERNEL_TILE, 0, 16), (SF_EVAL_KERNEL_TILE, 1, 128),
                           (SF_EVAL_KERNEL_AUTO, -1, 0), (SF_EVAL_KERNEL_AUTO, -1, 4)):
            ctx.set_option(SF_OPT_EVAL_KERNEL, kv)
            ctx.set_option(SF_OPT_EVAL_XCD_MAP, xm)
            ctx.set_option(SF_OPT_EVAL_BANDS, nb)
            o = gpu_eval(ctx, dev, pp, x, y, coef, flags=base)
            assert np.array_equal(o.view(np.int32), ref.view(np.int32)), (kv, xm, nb)
            del o
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
        ctx.set_option(SF_OPT_EVAL_XCD_MAP, -1)
        ctx.set_option(SF_OPT_EVAL_BANDS, 0)
    assert np.all(ref[7, 0::2] == 1.0) and np.all(ref[7, 1::2] == 0.0)
    cpix = okl.cpix_matrix(pp, x, y)
    pick = [0, 8, 36]
    want = okl.eval_planes(okl.eval_phase_screens(coef[pick], cpix))
    np.testing.assert_allclose(ref[pick].reshape(want.shape), want, rtol=0, atol=2e-6)


def test_binding_rejects_bad_device_operands(ctx, dev):
    """Wrong dtype / short / strided device buffers raise before any launch."""
    pp = np.stack([np.linspace(-900, 900, 6), np.linspace(300, -300, 6), np.zeros(6)], 1)
    ctx.set_basis(pp)
    x = np.linspace(-500, 500, 16)
    ctx.set_grid(x, x)
    S = 5
    coef = torch.zeros((S, 6), dtype=torch.float64, device=dev)
    out = torch.empty((S, 4, 16, 16), dtype=torch.float32, device=dev)
    with pytest.raises(TypeError):
        ctx.eval(coef.float(), S, out)
    with pytest.raises(ValueError):
        ctx.eval(coef, S, out[: S - 1])
    with pytest.raises(ValueError):
        ctx.eval(coef[:, ::2], S, out)
    ctx.eval(coef, S, out)  # the well-formed call still works
    torch.cuda.synchronize()
    assert torch.all(out[:, 0] == 1.0)


@pytest.mark.parametrize("T", [6, 1000])
def test_fit_vs_oracle_on_bench_workload_sample(ctx, dev, T):
    """The fit exactly as bench.py runs it on config 4 (256 stations, 32
    freqs, D = 20, setup_shard's reference phases and station orders; T
    times) vs the oracle's fit_slot on 6 sampled times of 6 stations x 4
    freqs: orders and flags equal, coefficients within 1e-8 x max(1,
    |coef|max) -- the check the CPU baseline leg makes on its sample."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import WORKLOADS
    from ska_sdp_screen_fitting_amd.distributed import setup_shard
    from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG, FIELD_RA_DEG,
                                                      FIELD_WIDTH_DEG, make_solutions)
    A, _, F, D, N, cell = WORKLOADS["config4"]
    sol = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D, ant_offset=0, n_ant_total=A)
    setup = setup_shard(sol, 0, A, FIELD_RA_DEG, FIELD_DEC_DEG, FIELD_WIDTH_DEG, cell,
                        device="cpu")
    ctx.set_basis(setup["piercepoints"], 100, 5.0 / 3.0)
    phase = torch.from_numpy(sol.val).to(dev)
    weight = torch.from_numpy(sol.weight).to(dev)
    coef = torch.empty_like(phase)
    resid = torch.empty_like(phase)
    w_out = torch.empty_like(weight)
    order_out = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    ctx.fit(phase, weight, T, F, A, setup["st_order"], niter=2, nsigma=5.0,
            adjust_order=True, ref_ant=setup["ref_ant"], coef=coef, resid=resid,
            w_out=w_out, order_out=order_out, ant_offset=setup["ant_offset"],
            ref_phase=setup["ref_phase"].to(dev).contiguous())
    torch.cuda.synchronize()
    g_c, g_w, g_o = coef.cpu().numpy(), w_out.cpu().numpy(), order_out.cpu().numpy()
    ref = setup["ref_ant"]
    phi = sol.val - setup["ref_phase"].numpy()[:, :, None, :]
    basis = okl.Basis(setup["piercepoints"])
    scale = max(1.0, float(np.abs(g_c).max()))
    bad = []
    times = np.random.default_rng(3).choice(T, size=min(6, T), replace=False)
    for a in [x for x in range(A) if x != ref][:6]:
        so = setup["st_order"][a]
        for f in range(4):
            for t in times:
                wh, _, wo, od, nf = okl.fit_slot(phi[t, f, a], sol.weight[t, f, a], so, so,
                                                 basis)
                dc = float(np.abs(g_c[t, f, a] - wh).max())
                if g_o[t, f, a] != int(od) or not np.array_equal(g_w[t, f, a], wo) \
                        or dc > 1e-8 * scale:
                    bad.append((t, f, a, int(so), int(g_o[t, f, a]), int(od),
                                int((g_w[t, f, a] > 0).sum()), int((wo > 0).sum()), nf, dc))
    assert not bad, bad[:12]


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("name", ["synth50", "config5-density", "synth20", "fixture_kl"])
def test_subset_deletion_bases_match_jacobi(ctx, dev, name, mode):
    """SF_OPT_FIT_SUBSET_DELETION: the subset bases by secular-equation
    deletions from the global eigenbasis vs the Jacobi solve of each mask --
    the same masks, eigenvalues to 1e-12 of |lambda|max, each eigenvector
    to the conditioning of its eigenvalue gap (sign free), and the fit's
    orders and flags identical, coefficients within 1e-9 of the golden.
    mode 3: each mask from its nearest ancestor the deletions built; mode 2:
    every mask from the global basis; mode 1 (the default): 3 for a pass
    with many new masks, else 2."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_SUBSET_DELETION
    g = _wave_count_case(name) if name == "config5-density" else load_golden(name)
    ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 0)
    try:
        jac = gpu_fit(ctx, dev, g)
        masks_j, pool_j = ctx.fit_pool()
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, mode)
        dele = gpu_fit(ctx, dev, g)
        masks_d, pool_d = ctx.fit_pool()
    finally:
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 1)
    assert np.array_equal(masks_j, masks_d)
    D = g["val"].shape[-1]
    lmax = 0.0
    worst_l = worst_v = 0.0
    for m, ej, ed in zip(masks_j, pool_j, pool_d):
        n = bin(int(m)).count("1")
        lj, ld_ = ej[D * D:D * D + n], ed[D * D:D * D + n]
        lmax = max(lmax, np.abs(lj).max())
        worst_l = max(worst_l, np.abs(lj - ld_).max())
        Vj = ej[:D * D].reshape(D, D)[:n, :n]
        Vd = ed[:D * D].reshape(D, D)[:n, :n]
        sg = np.sign(np.sum(Vj * Vd, axis=0))
        gap = np.full(n, np.inf)
        srt = np.sort(lj)
        for r in range(n):
            d = np.abs(srt - lj[r])
            d = d[d > 0]
            gap[r] = d.min() if d.size else np.inf
        err = np.abs(Vd * sg - Vj).max(axis=0)
        worst_v = max(worst_v, float(np.max(err * gap / lmax)))
    assert worst_l <= 1e-12 * lmax, (worst_l, lmax)
    assert worst_v <= 1e-12, worst_v
    np.testing.assert_array_equal(dele[3], jac[3])
    np.testing.assert_array_equal(dele[2], jac[2])
    scale = max(1.0, np.abs(jac[0]).max())
    keep = np.ones(jac[0].shape[:3], bool)
    if name != "config5-density":
        for i in _ill_conditioned(g):
            keep[i] = False
    assert np.abs(dele[0] - jac[0])[keep].max() <= 1e-9 * scale


def _deletion_edge_case(name):
    """Flag masks at the deletion kernel's edges: many deletions per mask
    (D = 50, 25 % of the entries zero), the largest D (SF_MAX_DIR = 60),
    a tiny D (masks down to one direction), and directions on a
    square lattice, whose C has six exactly degenerate eigenvalue pairs (the
    close-pole case the kernel hands to the Jacobi)."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    n_dir, flag = {"heavy50": (50, 0.25), "d60": (60, 0.05), "d4": (4, 0.4),
                   "lattice25": (25, 0.05)}[name]
    s = make_solutions(n_ant=8, n_time=30, n_freq=2, n_dir=n_dir, seed=71,
                       flag_frac=flag, outlier_frac=0.005)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    if name == "lattice25":
        g = np.arange(5) - 2.0
        X, Y = np.meshgrid(g, g)
        pp = np.zeros((25, 3))
        pp[:, 0], pp[:, 1] = X.ravel() * 900.0, Y.ravel() * 900.0
    return dict(val=s.val, weight=s.weight, ant_pos=s.ant_pos, piercepoints=pp,
                ref_ant=okl.reference_station(s.weight), order=min(20, n_dir))


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("name", ["heavy50", "d60", "d4", "lattice25"])
def test_subset_deletion_edge_cases(ctx, dev, name, mode):
    """The deletion subset bases vs the Jacobi's at the kernel's edges
    (`_deletion_edge_case`): eigenvalues to 1e-12 of |lambda|max and
    eigenvectors to their gap's conditioning everywhere; orders, flags and
    coefficients as the Jacobi's where no eigenvalue is degenerate; on the
    lattice, the masks whose first deletion meets the degenerate pairs come
    back from the Jacobi fallback bit for bit."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_SUBSET_DELETION
    g = _deletion_edge_case(name)
    ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 0)
    try:
        jac = gpu_fit(ctx, dev, g)
        masks_j, pool_j = ctx.fit_pool()
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, mode)
        dele = gpu_fit(ctx, dev, g)
        masks_d, pool_d = ctx.fit_pool()
    finally:
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 1)
    assert len(masks_j) > (5 if name == "d4" else 20)
    assert np.array_equal(masks_j, masks_d)
    D = g["val"].shape[-1]
    ns = [bin(int(m)).count("1") for m in masks_j]
    if name == "heavy50":
        assert np.mean([D - n for n in ns]) > 8  # many deletions per mask
    if name == "d4":
        assert min(ns) == 1
    lmax = max(np.abs(e[D * D:D * D + n]).max() for e, n in zip(pool_j, ns))
    c = ctx.get_basis()[0]
    worst_l = worst_v = 0.0
    same = 0
    for m, n, ej, ed in zip(masks_j, ns, pool_j, pool_d):
        lj, ld_ = ej[D * D:D * D + n], ed[D * D:D * D + n]
        # both against LAPACK on the principal submatrix of the library's C
        keep = [d for d in range(D) if (int(m) >> d) & 1]
        lref = np.sort(np.linalg.eigvalsh(c[np.ix_(keep, keep)]))
        assert np.abs(np.sort(lj) - lref).max() <= 1e-12 * lmax, ("jacobi", hex(int(m)), lj, lref)
        assert np.abs(np.sort(ld_) - lref).max() <= 1e-12 * lmax, ("deletion", hex(int(m)), ld_, lref)
        same += np.array_equal(ej[:D * D + n].view(np.uint64), ed[:D * D + n].view(np.uint64))
        # columns paired by eigenvalue: two eigenvalues of equal |lambda| and
        # opposite sign (a 2 x 2 subset of a zero-diagonal C: +-b) may come in
        # either order from either solver, as from the reference's SVD
        oj, od = np.argsort(lj, kind="stable"), np.argsort(ld_, kind="stable")
        lj, ld_ = lj[oj], ld_[od]
        worst_l = max(worst_l, np.abs(lj - ld_).max())
        Vj = ej[:D * D].reshape(D, D)[:n, :n][:, oj]
        Vd = ed[:D * D].reshape(D, D)[:n, :n][:, od]
        sg = np.sign(np.sum(Vj * Vd, axis=0))
        gap = np.array([np.min(np.abs(np.delete(lj, r) - lj[r]), initial=np.inf)
                        for r in range(n)])
        gap[~np.isfinite(gap)] = 0.0
        err = np.abs(Vd * sg - Vj).max(axis=0)
        worst_v = max(worst_v, float(np.max(err * gap / lmax)))
    assert worst_l <= 1e-12 * lmax, (worst_l, lmax)
    assert worst_v <= 1e-12, worst_v
    if name == "lattice25":
        assert same > 0  # the fallback ran
        return
    np.testing.assert_array_equal(dele[3], jac[3])
    np.testing.assert_array_equal(dele[2], jac[2])
    # coefficients everywhere: the two-direction masks (d4), whose +-b
    # eigenvalues either solver may order either way, fit on the reference's
    # e_2 column (fit_once), not on the eigenvector order (round 6)
    scale = max(1.0, np.abs(jac[0]).max())
    assert np.abs(dele[0] - jac[0]).max() <= 1e-9 * scale


@pytest.mark.parametrize("name", ["heavy50", "lattice25", "d4", "synth20"])
def test_subset_deletion_modes_bit_identical(ctx, dev, name):
    """The three deletion schedules write the same bits: from
    ancestors (mode 3, one launch per level), from the global basis (mode
    2) and the default (1), over three passes (niter 3, so later passes'
    masks take earlier passes' pool entries as ancestors), also on the
    lattice, where the Jacobi fallback builds some entries: an ancestor is
    taken only if the deletion chain built it, so no mask's bits depend on
    which pass or which other slots produced its parent."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_SUBSET_DELETION
    g = load_golden(name) if name == "synth20" else _deletion_edge_case(name)
    outs = {}
    try:
        for mode in (2, 3, 1):
            ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, mode)
            outs[mode] = gpu_fit(ctx, dev, g, niter=3)
            outs[(mode, "pool")] = ctx.fit_pool()
    finally:
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 1)
    for mode in (3, 1):
        for a, b in zip(outs[mode], outs[2]):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), mode
        ma, pa = outs[(mode, "pool")]
        mb, pb = outs[(2, "pool")]
        assert np.array_equal(ma, mb)
        assert np.array_equal(pa.view(np.uint64), pb.view(np.uint64)), mode


def _golden_soltab(g):
    """A phase soltab + solset of a golden set, as stationscreen.run reads
    them (h5parm.Soltab / Solset)."""
    from ska_sdp_screen_fitting_amd.h5parm import Solset, Soltab
    ss = Solset("sol000", list(g["ant_names"]), g["ant_pos"], list(g["dir_names"]),
                g["dir_radec"])
    st = Soltab("phase000", "phase", ["time", "freq", "ant", "dir"],
                [g["times"], g["freqs"], list(g["ant_names"]), list(g["dir_names"])],
                np.array(g["val"]), np.array(g["weight"]), solset=ss)
    ss.soltabs["phase000"] = st
    return st


def test_threads_fit_on_private_contexts(dev):
    """Two threads run stationscreen.run on different golden sets (synth20,
    synth50: different bases) on one device, interleaved -- each call takes
    a context of its own (_lib.private_context), so neither can re-base the
    other between its set_basis and its fit (the round-5 r5x failure mode of
    one shared context).  Every run matches its reference golden: orders and
    flagged weights bit for bit, coefficients <= 1e-8."""
    import threading
    from ska_sdp_screen_fitting_amd import stationscreen
    from ska_sdp_screen_fitting_amd._lib import get_context
    goldens = {n: load_golden(n) for n in ("synth20", "synth50")}
    # the process-wide context holds a third basis meanwhile
    get_context(0).set_basis(load_golden("fixture_kl")["piercepoints"])
    errors, done = [], {n: 0 for n in goldens}
    start = threading.Barrier(len(goldens))

    def worker(name):
        g = goldens[name]
        try:
            start.wait()
            for it in range(4):
                st = _golden_soltab(g)
                assert stationscreen.run(st, "phase_screen000", order=int(g["order"]),
                                         ref_ant=int(g["ref_ant"])) == 0
                ss = st.get_solset()
                scr = ss.get_soltab("phase_screen000")
                res = ss.get_soltab("phase_screen000resid")
                np.testing.assert_array_equal(res.weight[..., 0], g["orders"])
                np.testing.assert_array_equal(scr.weight, g["w_out"])
                scale = max(1.0, np.abs(g["coef"]).max())
                np.testing.assert_allclose(scr.val, g["coef"], rtol=0, atol=1e-8 * scale)
                done[name] += 1
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((name, repr(e)))

    ths = [threading.Thread(target=worker, args=(n,)) for n in goldens]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errors, errors
    assert all(v == 4 for v in done.values()), done


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("name", ["ties4", "ties6"])
def test_fit_vs_reference_golden_ties(ctx, dev, name, mode):
    """The reference run with many two-direction slots
    (tests/golden/make_golden_ties.py: D = 4 / 6, 40 % flags): its order-1
    fit there keeps LAPACK's first U column e_2 of the tied 2 x 2 subset
    (fit_once, kl_fit_fast.hip), under every subset-basis schedule (the
    Jacobi, deletions from ancestors / the global basis / auto): orders and
    flagged weights bit for bit, coefficients and residuals <= 1e-8 --
    except the slots where the reference's own LAPACK left rounding residue
    in that U (``tie_residue``, recorded by the generator: atan2 of the
    residue)."""
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_SUBSET_DELETION
    g = load_golden(name)
    ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, mode)
    try:
        coef, resid, w_out, orders = gpu_fit(ctx, dev, g)
    finally:
        ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, 1)
    np.testing.assert_array_equal(orders, g["orders"])
    np.testing.assert_array_equal(w_out, g["w_out"])
    keep = ~g["tie_residue"]
    n2 = (g["w_out"] > 0).sum(axis=-1) == 2
    assert (keep & n2).sum() >= 10
    scale = max(1.0, np.abs(g["coef"]).max())
    err = np.abs(coef - g["coef"]).max(axis=-1)
    assert err[keep].max() <= 1e-8 * scale, np.argwhere(err > 1e-8 * scale)[:8]
    assert np.abs(resid - g["resid"]).max(axis=-1)[keep].max() <= 1e-8

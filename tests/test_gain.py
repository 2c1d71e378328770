"""Gain (phase + slow XX/YY amplitude) screens, SURVEY.md §8(f) row 3.

Golden vectors: tests/golden/gain12.npz, made by running the reference itself
(tests/golden/make_golden_gain.py): the amplitude stationscreen.run exactly as
KLScreen.fit calls it (kl_screen.py:96-125), Screen.interpolate
(screen.py:108-154) and KLScreen.make_matrix with amplitudes
(kl_screen.py:319-378).  The tessellated gain planes are checked against the
oracle restatement (the reference's tessellated path needs shapely).

Tolerances: amplitude coefficients |d| <= 1e-8 x max(1, |coef|max) (as the
phase fit); orders and flagged weights identical; interpolation exact (a row
gather); gain planes |d| <= 1e-6 x max(1, amplitude) with fp32 sincos / exp10
(2e-6 fast path).
"""

import os

import numpy as np
import pytest

from conftest import FIELD, GOLDEN, load_golden
from oracle import kl as okl
from oracle import voronoi as ov


@pytest.fixture(scope="module")
def gain():
    return load_golden("gain12")


# ---------------------------------------------------------------- CPU: oracle

def test_oracle_amplitude_fit_vs_reference(gain):
    g = gain
    r = okl.run_amplitude(g["amp_val"], g["amp_weight"], g["piercepoints"],
                          int(g["amp_order"]))
    np.testing.assert_array_equal(r["orders"], g["amp_orders"])
    np.testing.assert_array_equal(r["w_out"], g["amp_w_out"])
    scale = max(1.0, np.abs(g["amp_coef"]).max())
    np.testing.assert_allclose(r["coef"], g["amp_coef"], rtol=0, atol=1e-10 * scale)
    np.testing.assert_allclose(r["resid"], g["amp_resid"], rtol=0, atol=1e-10)
    # the block-coupled sigma flags something beyond the input flags
    assert (g["amp_w_out"] == 0).sum() > (g["amp_weight"] == 0).sum()


def test_oracle_interpolation_vs_reference(gain):
    g = gain
    got = okl.interpolate_nearest(g["amp_coef"], g["amp_times"], g["amp_freqs"],
                                  g["times"], g["freqs"])
    np.testing.assert_array_equal(got, g["amp_interp"])


def test_oracle_gain_planes_vs_reference(gain):
    g = gain
    cpix = okl.cpix_matrix(g["piercepoints"], g["x17"], g["y17"])
    for k, (f, a) in enumerate(g["pairs"]):
        ph = okl.eval_phase_screens(g["coef"][:, f, a, :], cpix)
        ax = 10 ** okl.eval_phase_screens(g["amp_interp"][:, f, a, :, 0], cpix)
        ay = 10 ** okl.eval_phase_screens(g["amp_interp"][:, f, a, :, 1], cpix)
        want = okl.eval_planes(ph, ax, ay).reshape(g["gain17"][k].shape)
        np.testing.assert_allclose(want, g["gain17"][k], rtol=0, atol=1e-12)


# ------------------------------------------------------ CPU: product host code

def test_nearest_index_matches_scipy():
    import scipy.interpolate as si
    from ska_sdp_screen_fitting_amd.screen import nearest_index
    rng = np.random.default_rng(5)
    src = np.sort(rng.random(7)) * 10
    # ties at exact midpoints, points outside both ends, duplicates
    dst = np.concatenate([(src[1:] + src[:-1]) / 2.0, [-3.0, 42.0], src,
                          rng.random(50) * 12 - 1])
    vals = np.arange(7, dtype=np.float64)
    want = si.interp1d(src, vals, kind="nearest", fill_value="extrapolate")(dst)
    np.testing.assert_array_equal(vals[nearest_index(src, dst)], want)


def test_screen_interpolate_vs_reference(gain):
    from ska_sdp_screen_fitting_amd.screen import Screen
    g = gain
    s = Screen("x", None, None, 0.0, 0.0, 1.0, 1.0, amplitude_soltab_name="amp")
    s.vals_ph, s.times_ph, s.freqs_ph = g["coef"], g["times"], g["freqs"]
    s.vals_amp, s.times_amp, s.freqs_amp = g["amp_coef"], g["amp_times"], g["amp_freqs"]
    s.log_amps = True
    s.interpolate()
    np.testing.assert_array_equal(s.vals_amp, g["amp_interp"])
    # tessellated screens interpolate raw amplitudes through log10 space
    s.vals_amp, s.log_amps = 10 ** g["amp_coef"], False
    s.interpolate()
    np.testing.assert_allclose(s.vals_amp, 10 ** g["amp_interp"], rtol=1e-14)
    # a single amplitude time: repeated onto the phase grid
    s.vals_amp = g["amp_coef"][:1, :1]
    s.times_amp = g["amp_times"][:1]
    s.interpolate()
    assert s.vals_amp.shape == g["amp_interp"].shape


# ------------------------------------------------------------------- GPU

def _torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda", 0)


def _ctx(torch, dev):
    from ska_sdp_screen_fitting_amd import get_context
    c = get_context(0)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    return c


@pytest.mark.gpu
def test_amplitude_fit_vs_reference(gain):
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    g = gain
    ctx.set_basis(g["piercepoints"])
    T, F, A, D, P = g["amp_val"].shape
    order = int(g["amp_order"])
    scale = max(1.0, np.abs(g["amp_coef"]).max())
    for p in range(P):
        v = torch.from_numpy(np.ascontiguousarray(g["amp_val"][..., p])).to(dev)
        w = torch.from_numpy(np.ascontiguousarray(g["amp_weight"][..., p])).to(dev)
        coef, resid, w_out = torch.empty_like(v), torch.empty_like(v), torch.empty_like(w)
        orders = torch.empty((T, F, A), dtype=torch.int32, device=dev)
        ctx.fit(v, w, T, F, A, [order] * A, screen_type=SF_SCREEN_AMPLITUDE,
                niter=3, ref_ant=-1, coef=coef, resid=resid, w_out=w_out,
                order_out=orders)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(orders.cpu().numpy(), g["amp_orders"][..., p])
        np.testing.assert_array_equal(w_out.cpu().numpy(), g["amp_w_out"][..., p])
        np.testing.assert_allclose(coef.cpu().numpy(), g["amp_coef"][..., p],
                                   rtol=0, atol=1e-8 * scale)
        np.testing.assert_allclose(resid.cpu().numpy(), g["amp_resid"][..., p],
                                   rtol=0, atol=1e-8)


@pytest.mark.gpu
def test_amplitude_fit_vs_oracle_larger():
    """More stations / times, NaN blocks and all-flagged blocks (skipped)."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE
    from ska_sdp_screen_fitting_amd.synthetic import make_amplitudes, make_solutions
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    s = make_solutions(n_ant=6, n_time=4, n_freq=2, n_dir=20, seed=7)
    make_amplitudes(s, seed=8, flag_frac=0.05, outlier_frac=0.03)
    amp = s.amp_val.copy()
    wt = s.meta["amp_weight"].copy()
    amp[:, 1, 2] = np.nan          # an all-NaN (freq, station) block
    wt[:, 0, 4] = 0.0              # an all-flagged block
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    order = 10
    want = okl.run_amplitude(amp, wt, pp, order)
    ctx.set_basis(pp)
    T, F, A, D, P = amp.shape
    for p in range(P):
        v = torch.from_numpy(np.ascontiguousarray(amp[..., p])).to(dev)
        w = torch.from_numpy(np.ascontiguousarray(wt[..., p])).to(dev)
        coef, resid, w_out = torch.zeros_like(v), torch.zeros_like(v), torch.empty_like(w)
        orders = torch.zeros((T, F, A), dtype=torch.int32, device=dev)
        ctx.fit(v, w, T, F, A, [order] * A, screen_type=SF_SCREEN_AMPLITUDE,
                niter=3, ref_ant=-1, coef=coef, resid=resid, w_out=w_out,
                order_out=orders)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(orders.cpu().numpy(), want["orders"][..., p])
        np.testing.assert_array_equal(w_out.cpu().numpy(), want["w_out"][..., p])
        np.testing.assert_allclose(coef.cpu().numpy(), want["coef"][..., p],
                                   rtol=0, atol=1e-8 * max(1.0, np.abs(want["coef"]).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [False, True])
def test_gain_eval_vs_reference(gain, fast):
    from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_FAST_SINCOS,
                                                 SF_EVAL_NAN_SCRUB)
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    g = gain
    ctx.set_basis(g["piercepoints"])
    ctx.set_grid(g["x17"], g["y17"])
    flags = SF_EVAL_NAN_SCRUB | (SF_EVAL_FAST_SINCOS if fast else 0)
    tol = 2e-6 if fast else 1e-6
    for k, (f, a) in enumerate(g["pairs"]):
        up = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
              (g["coef"][:, f, a, :], g["amp_interp"][:, f, a, :, 0],
               g["amp_interp"][:, f, a, :, 1])]
        S = up[0].shape[0]
        out = torch.full((S, 4, 17, 17), -7.0, dtype=torch.float32, device=dev)
        ctx.eval_gain(up[0], up[1], up[2], S, out, S, flags)
        torch.cuda.synchronize()
        ref = g["gain17"][k]
        amp = np.maximum(1.0, np.abs(ref))
        err = np.abs(out.cpu().numpy() - ref) / amp
        assert err.max() <= tol, err.max()


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [False, True])
def test_gain_eval_finite_groups_and_scrub(gain, fast):
    """Gain planes of 16-slot groups in four regimes against fp64 numpy:
    small amplitudes, |log2 A| up to 100 (finite, large values), a NaN
    amplitude coefficient (its XX planes scrubbed to 1 / 0) and a NaN phase
    coefficient (all four planes scrubbed), in a partial last group; and a
    slot's bits do not depend on the other slots of its group (a NaN slot
    sends the group's phases down the exact reduction, kl_eval_impl.h
    kRevMagic)."""
    from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_FAST_SINCOS,
                                                 SF_EVAL_NAN_SCRUB)
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    g = gain
    pp = g["piercepoints"]
    ctx.set_basis(pp)
    ctx.set_grid(g["x17"], g["y17"])
    cpix = okl.cpix_matrix(pp, g["x17"], g["y17"])
    D = cpix.shape[1]
    cmax = np.abs(cpix).max()
    L = np.log2(10.0)
    rng = np.random.default_rng(11)
    S = 53
    ph = rng.normal(0, 0.01, (S, D))
    amp = [rng.normal(0, 1.0, (S, D)) for _ in range(2)]
    for a in amp:
        # groups 0, 2, 3: sum |coef| log2(10) max|Cpix| = 20 (finite bound)
        a *= 20.0 / (np.abs(a).sum(1, keepdims=True) * L * cmax)
        # group 1: |log2 A| reaches 100 (finite values: A < 2^128), past
        # the bound
        big = a[16:32] * (100.0 / np.abs(a[16:32] @ cpix.T * L).max(1, keepdims=True))
        assert np.any(np.abs(big).sum(1) * L * cmax > 128.0)
        a[16:32] = big
    amp[0][35, 2] = np.nan
    ph[50, 1] = np.nan
    flags = SF_EVAL_NAN_SCRUB | (SF_EVAL_FAST_SINCOS if fast else 0)

    def run(p, ax, ay):
        up = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (p, ax, ay)]
        n = p.shape[0]
        out = torch.full((n, 4, 17, 17), -7.0, dtype=torch.float32, device=dev)
        ctx.eval_gain(up[0], up[1], up[2], n, out, n, flags)
        torch.cuda.synchronize()
        return out.cpu().numpy().reshape(n, 4, -1)

    out = run(ph, amp[0], amp[1])
    phase = ph @ cpix.T
    lx, ly = amp[0] @ cpix.T * L, amp[1] @ cpix.T * L
    with np.errstate(invalid="ignore", over="ignore"):
        want = np.stack([2 ** lx * np.cos(phase), 2 ** lx * np.sin(phase),
                         2 ** ly * np.cos(phase), 2 ** ly * np.sin(phase)], 1)
    want = want.astype(np.float32)
    nan = np.isnan(want)
    want[:, 0::2][nan[:, 0::2]] = 1.0
    want[:, 1::2][nan[:, 1::2]] = 0.0
    assert np.all(out[35, 0] == 1.0) and np.all(out[35, 1] == 0.0)
    assert np.all(out[50] == np.array([1, 0, 1, 0], np.float32)[:, None])
    lmax = np.nan_to_num(np.maximum(np.abs(lx), np.abs(ly)), nan=0.0)[:, None, :]
    tol = (2e-6 if fast else 1e-6) + 1.2e-7 * lmax
    # relative to max(1, A) of the plane's amplitude (A sin is small where
    # sin is: its error is A times that of the fp32 sine)
    with np.errstate(invalid="ignore", over="ignore"):
        ampl = np.stack([2 ** lx, 2 ** lx, 2 ** ly, 2 ** ly], 1)
    ampl = np.maximum(1.0, np.nan_to_num(ampl, nan=1.0))
    err = np.abs(out - want) / ampl
    assert np.all(err <= tol), err.max()
    # slots 0..14 in a group with a NaN slot (checked path) == the same slots
    # in a group of their own, bit for bit
    p2 = np.concatenate([ph[:15], ph[50:51]])
    x2 = np.concatenate([amp[0][:15], amp[0][:1]])
    y2 = np.concatenate([amp[1][:15], amp[1][:1]])
    got = run(p2, x2, y2)
    np.testing.assert_array_equal(got[:15].view(np.uint32), out[:15].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n_dir,grid", [(20, 256), (7, 128), (24, 60), (3, 40),
                                        (44, 32), (50, 64)])
def test_gain_eval_kernels_agree(n_dir, grid):
    """Every gain evaluation kernel -- the register tile and, in a library
    built with -DSF_EVAL_GAIN_LDS=1 (round 6, "Tried" in DESIGN.md), the
    LDS-staged shapes LDS4 / LDS8 / LDS8H / LDS16H (LDS16 mapped to LDS16H;
    the shipped library maps every forced shape to the tile) -- writes the
    same bits as the register tile, with plain, non-temporal
    and big-endian stores, walking workgroups, both XCD maps, short work
    items, and through sf_kl_eval_sums (equal per-slot checksums).  Ragged
    slot count (45: a partial 16-slot group), grids that are not a multiple
    of the LDS store run, NaN / Inf phase and amplitude coefficients (the
    scrubbed products), large amplitudes; D = 50 (past kGainLdsMaxKS) runs
    the register tile under every setting; the tile output is within the
    fast-path tolerance of fp64 numpy."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import (
        EVAL_KERNEL_NAMES, SF_EVAL_BIG_ENDIAN, SF_EVAL_FAST_SINCOS,
        SF_EVAL_KERNEL_AUTO, SF_EVAL_KERNEL_TILE, SF_EVAL_NAN_SCRUB,
        SF_EVAL_NT_STORES, SF_OPT_EVAL_GROUPS, SF_OPT_EVAL_KERNEL,
        SF_OPT_EVAL_MAX_BLOCKS, SF_OPT_EVAL_XCD_MAP)
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=4)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    rng = np.random.default_rng(n_dir * 7 + grid)
    S = 45
    ph = rng.normal(0, 0.01, (S, n_dir))
    ph[20:30] *= 300.0                 # many turns: the exact reduction
    ax = rng.normal(0, 0.002, (S, n_dir))
    ay = rng.normal(0, 0.002, (S, n_dir))
    # large amplitudes: |log2 A| up to 60 (finite in fp32)
    cpix = okl.cpix_matrix(pp, x, y)
    big = ax[33:40] @ cpix.T * np.log2(10.0)
    ax[33:40] *= 60.0 / np.abs(big).max()
    ph[9, n_dir // 2] = np.nan
    ph[31, 0] = np.inf
    ax[12, n_dir - 1] = np.nan         # XX planes scrubbed, YY kept
    ay[41, 0] = np.inf
    up = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (ph, ax, ay)]
    base = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS

    def run(flags, sums=False):
        out = torch.full((S, 4, grid, grid), -7.0, dtype=torch.float32, device=dev)
        if sums:
            cs = torch.zeros(S, dtype=torch.int32, device=dev)
            ctx.eval_sums(up[0], S, out, cs, S, coef_xx=up[1], coef_yy=up[2],
                          flags=flags)
        else:
            ctx.eval_gain(up[0], up[1], up[2], S, out, S, flags)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        if flags & SF_EVAL_BIG_ENDIAN:
            o = o.byteswap()
        return (o, cs.cpu().numpy()) if sums else o

    outs, sums = {}, {}
    try:
        for kv in sorted(EVAL_KERNEL_NAMES) + [SF_EVAL_KERNEL_AUTO]:
            ctx.set_option(SF_OPT_EVAL_KERNEL, kv)
            for extra in (0, SF_EVAL_NT_STORES, SF_EVAL_BIG_ENDIAN):
                outs[(kv, extra)] = run(base | extra)
            outs[(kv, "sums")], sums[kv] = run(base | SF_EVAL_NT_STORES, sums=True)
            ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 8)
            outs[(kv, "walk")] = run(base)
            ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 0)
            for xm in (0, 1):
                ctx.set_option(SF_OPT_EVAL_XCD_MAP, xm)
                outs[(kv, "xcd", xm)] = run(base)
            ctx.set_option(SF_OPT_EVAL_XCD_MAP, -1)
            ctx.set_option(SF_OPT_EVAL_GROUPS, 1)
            outs[(kv, "g1")] = run(base)
            ctx.set_option(SF_OPT_EVAL_GROUPS, 0)
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
        ctx.set_option(SF_OPT_EVAL_MAX_BLOCKS, 0)
        ctx.set_option(SF_OPT_EVAL_XCD_MAP, -1)
        ctx.set_option(SF_OPT_EVAL_GROUPS, 0)
    ref = outs[(SF_EVAL_KERNEL_TILE, 0)]
    for k, o in outs.items():
        assert np.array_equal(o.view(np.int32), ref.view(np.int32)), k
    # the checksum is the sum mod 2^32 of each slot's stored words
    want_sums = ref.reshape(S, -1).view(np.uint32).astype(np.uint64).sum(1) % 2 ** 32
    for kv, cs in sums.items():
        assert np.array_equal(cs.view(np.uint32), want_sums.astype(np.uint32)), kv
    # scrubbed products: NaN phase -> all four planes 1 / 0; NaN log A_XX ->
    # the XX planes
    for k in (9, 31):
        assert np.all(ref[k, 0::2] == 1.0) and np.all(ref[k, 1::2] == 0.0)
    assert np.all(ref[12, 0] == 1.0) and np.all(ref[12, 1] == 0.0)
    good = np.isfinite(ph).all(1) & np.isfinite(ax).all(1) & np.isfinite(ay).all(1)
    L = np.log2(10.0)
    phase = ph[good] @ cpix.T
    lx, ly = ax[good] @ cpix.T * L, ay[good] @ cpix.T * L
    want = np.stack([2 ** lx * np.cos(phase), 2 ** lx * np.sin(phase),
                     2 ** ly * np.cos(phase), 2 ** ly * np.sin(phase)], 1)
    ampl = np.maximum(1.0, np.stack([2 ** lx, 2 ** lx, 2 ** ly, 2 ** ly], 1))
    lmax = np.maximum(np.abs(lx), np.abs(ly))[:, None, :]
    err = np.abs(ref[good].reshape(want.shape) - want) / ampl
    assert np.all(err <= 2e-6 + 1.2e-7 * lmax), err.max()


@pytest.mark.gpu
def test_make_aterm_image_gain_kl(tmp_path, gain):
    """make_aterm_image on a gain solution set (soltab "gain000" -> phase000
    + amplitude000), FITS cube vs the reference's make_matrix output."""
    _torch_dev()
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    g = gain
    outroot = str(tmp_path / "gain")
    make_aterm_image(os.path.join(GOLDEN, "gain12.npz"), soltabname="gain000",
                     screen_type="kl", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50], skymodel=None,
                     padding_fraction=0, cellsize_deg=0.2, ncpu=0)
    _, cube = sffits.read_cube(outroot + "_0.fits")
    assert cube.shape == (8, 3, 5, 4, 17, 17)
    for k, (f, a) in enumerate(g["pairs"]):
        ref = g["gain17"][k]
        err = np.abs(cube[:, f, a] - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 2e-6, (k, err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("smooth", [0.0, 1.3])
def test_tess_gain_vs_oracle(gain, smooth):
    from ska_sdp_screen_fitting_amd.voronoi_screen import tessellation_template
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    g = gain
    radec = np.rad2deg(g["dir_radec"].astype(np.float64))
    lab, _ = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                   FIELD["width"], 0.05)
    ref = int(g["ref_ant"])
    ph = (g["val"] - g["val"][:, :, ref:ref + 1, :]).reshape(-1, 12)
    amp = 10 ** g["amp_interp"].reshape(-1, 12, 2)
    axx, ayy = np.ascontiguousarray(amp[..., 0]), np.ascontiguousarray(amp[..., 1])
    ny, nx = lab.shape
    S = ph.shape[0]
    d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (ph, axx, ayy)]
    lab_d = torch.from_numpy(np.ascontiguousarray(lab, np.int32)).to(dev)
    out = torch.full((S, 4, ny, nx), -5.0, dtype=torch.float32, device=dev)
    ctx.tess_fill(lab_d, nx, ny, d[0], 12, S, out, amp_xx=d[1], amp_yy=d[2],
                  smooth_pix=smooth)
    torch.cuda.synchronize()
    want = ov.gather_planes(lab, ph, axx, ayy)
    if smooth > 0:
        want = ov.smooth(want, smooth)
    np.testing.assert_allclose(out.cpu().numpy(), want, rtol=0,
                               atol=1e-6 * max(1.0, np.abs(want).max()))


@pytest.mark.gpu
def test_stacked_pol_fit_equals_per_pol(gain):
    """stationscreen.run fits the amplitude pols in ONE sf_kl_fit call,
    stacked along the station axis (amplitudes are never referenced and
    their outlier sigma is per (station, freq) block, Q6): bit for bit the
    per-pol fits -- on the reference's gain set and on a larger synthetic
    one with NaN / all-flagged blocks and different flags per pol."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE
    from ska_sdp_screen_fitting_amd.synthetic import make_amplitudes, make_solutions
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    s = make_solutions(n_ant=6, n_time=5, n_freq=3, n_dir=20, seed=17)
    make_amplitudes(s, seed=18, flag_frac=0.05, outlier_frac=0.03)
    amp, wt = s.amp_val.copy(), s.meta["amp_weight"].copy()
    amp[:, 1, 2, :, 0] = np.nan
    wt[:, 0, 4, :, 1] = 0.0
    wt[2, 2, 1, 3, 1] = 0.0  # the pols' flags differ
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    for val, w, pp_, order in ((gain["amp_val"], gain["amp_weight"], gain["piercepoints"],
                                int(gain["amp_order"])), (amp, wt, pp, 10)):
        ctx.set_basis(pp_)
        T, F, A, D, P = val.shape

        def fit(v, ww, n_st):
            v = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
            ww = torch.from_numpy(np.ascontiguousarray(ww)).to(dev)
            out = (torch.zeros_like(v), torch.zeros_like(v), torch.empty_like(ww),
                   torch.zeros((T, F, n_st), dtype=torch.int32, device=dev))
            ctx.fit(v, ww, T, F, n_st, [order] * n_st, screen_type=SF_SCREEN_AMPLITUDE,
                    niter=3, ref_ant=-1, coef=out[0], resid=out[1], w_out=out[2],
                    order_out=out[3])
            torch.cuda.synchronize()
            return [x.cpu().numpy() for x in out]

        stacked = fit(np.concatenate([val[..., p] for p in range(P)], axis=2),
                      np.concatenate([w[..., p] for p in range(P)], axis=2), A * P)
        for p in range(P):
            single = fit(val[..., p], w[..., p], A)
            for a, b in zip(single, stacked):
                assert np.array_equal(a.view(np.uint8),
                                      np.ascontiguousarray(b[:, :, p * A:(p + 1) * A]).view(np.uint8))


def test_oracle_amplitude_ties_vs_reference():
    """tests/golden/ties4amp.npz (make_golden_ties.py amp): the reference's
    amplitude fit as KLScreen.fit calls it at D = 4 with 40 % of the weights
    zero -- 80 (slot, pol) fits with exactly two unflagged directions, whose
    order-1 fit keeps LAPACK's e_2 column of the tied 2 x 2 subset."""
    g = load_golden("ties4amp")
    assert ((g["amp_w_out"] > 0).sum(axis=-2) == 2).sum() >= 40
    r = okl.run_amplitude(g["amp_val"], g["amp_weight"], g["piercepoints"],
                          int(g["amp_order"]))
    np.testing.assert_array_equal(r["orders"], g["amp_orders"])
    np.testing.assert_array_equal(r["w_out"], g["amp_w_out"])
    np.testing.assert_allclose(r["coef"], g["amp_coef"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(r["resid"], g["amp_resid"], rtol=0, atol=1e-10)


@pytest.mark.gpu
def test_amplitude_ties_fit_vs_reference():
    """The GPU amplitude fit (both pols stacked along the station axis in one
    call, as stationscreen.run does) on the two-direction-heavy reference
    run: orders and flags bit-equal, coefficients / residuals <= 1e-8."""
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE
    torch, dev = _torch_dev()
    ctx = _ctx(torch, dev)
    g = load_golden("ties4amp")
    ctx.set_basis(g["piercepoints"])
    T, F, A, D, P = g["amp_val"].shape
    order = int(g["amp_order"])
    v = np.concatenate([g["amp_val"][..., p] for p in range(P)], axis=2)
    w = np.concatenate([g["amp_weight"][..., p] for p in range(P)], axis=2)
    vd = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    wd = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
    coef, resid, w_out = torch.empty_like(vd), torch.empty_like(vd), torch.empty_like(wd)
    orders = torch.empty((T, F, P * A), dtype=torch.int32, device=dev)
    ctx.fit(vd, wd, T, F, P * A, [order] * (P * A), screen_type=SF_SCREEN_AMPLITUDE,
            niter=3, ref_ant=-1, coef=coef, resid=resid, w_out=w_out, order_out=orders)
    torch.cuda.synchronize()
    c, r, wo, o = (x.cpu().numpy() for x in (coef, resid, w_out, orders))
    for p in range(P):
        sl = slice(p * A, (p + 1) * A)
        np.testing.assert_array_equal(o[:, :, sl], g["amp_orders"][..., p])
        np.testing.assert_array_equal(wo[:, :, sl], g["amp_w_out"][..., p])
        np.testing.assert_allclose(c[:, :, sl], g["amp_coef"][..., p], rtol=0, atol=1e-8)
        np.testing.assert_allclose(r[:, :, sl], g["amp_resid"][..., p], rtol=0, atol=1e-8)

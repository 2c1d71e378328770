"""The integer-digit evaluation contraction (kl_eval_int.h, SF_OPT_EVAL_INT).

Phase screens with D >= 45 evaluate Cpix . coef on i8 MFMAs over 6 balanced
base-256 digits of 36- / 44-bit fixed point, exactly modulo 2^32 turns
(kl_screen.py:444-449 contraction, :367-380 epilogue).  Checked here against
the oracle (fp64 numpy restatement of calculate_kl_screen) and against the
fp64 MFMA contraction of the same library (SF_OPT_EVAL_INT = 0):

* finite slots: |d| <= 2e-6 vs the oracle (the fast-epilogue tolerance of
  every evaluation test), <= 3e-7 vs the fp64 contraction (phase error
  < 2^-27 turn plus one fp32 rounding of the reduced phase either way);
* slots the digits cannot carry (NaN / Inf, |coef / 2 pi| beyond ~7.9 turns)
  take the fp64 contraction inside the same launch: bit for bit the fp64
  register tile's output;
* every kernel (register tile, LDS-staged) writes the same bits with it;
* the path really runs: some values differ in the last bits from the fp64
  contraction.
Needs an MI355X: every test is marked ``gpu``.
"""

import numpy as np
import pytest

from conftest import FIELD
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


def grid_for(n_dir, grid, seed):
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=seed)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    return pp, x, y


def run(ctx, dev, coefs, S, grid, int_on, flags, gain=False):
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_EVAL_INT
    ctx.set_option(SF_OPT_EVAL_INT, -1 if int_on else 0)
    try:
        cs = [torch.from_numpy(np.ascontiguousarray(c, np.float64)).to(dev) for c in coefs]
        out = torch.full((S, 4, grid, grid), -7.0, dtype=torch.float32, device=dev)
        if gain:
            ctx.eval_gain(cs[0], cs[1], cs[2], S, out, flags=flags)
        else:
            ctx.eval(cs[0], S, out, flags=flags)
        torch.cuda.synchronize()
        return out.cpu().numpy()
    finally:
        ctx.set_option(SF_OPT_EVAL_INT, -1)


@pytest.mark.parametrize("n_dir,grid", [(50, 64), (45, 128), (60, 96)])
def test_int_phase_vs_fp64_and_oracle(ctx, dev, n_dir, grid):
    from ska_sdp_screen_fitting_amd._lib import (
        EVAL_KERNEL_NAMES, SF_EVAL_FAST_SINCOS, SF_EVAL_KERNEL_AUTO,
        SF_EVAL_KERNEL_SHB, SF_EVAL_KERNEL_TILE, SF_OPT_EVAL_KERNEL)
    pp, x, y = grid_for(n_dir, grid, seed=n_dir)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    rng = np.random.default_rng(grid + n_dir)
    S = 45  # ragged: two whole 16-slot groups and a tail
    coef = rng.normal(0, 0.01, size=(S, n_dir))
    coef[20:30] *= 300.0                 # up to ~1.6 turns per coefficient
    coef[3, 1] = 2 * np.pi * 9.0         # 9 turns: past the digit range
    coef[9, n_dir // 2] = np.nan
    coef[31, 0] = np.inf
    fb = [3, 9, 31]                      # the fp64 rows
    flags = 1 | SF_EVAL_FAST_SINCOS
    # auto: the register tile; SHB holds the pixel digits in LDS (round 4);
    # the LDS-staged kernels take the integer contraction too -- every kernel
    # writes the same bits (below)
    try:
        assert ctx.eval_kernel(flags) == "kl_eval_kernel"
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_SHB)
        assert ctx.eval_kernel(flags) == "kl_eval_kernel<Cpix in LDS>"
        assert ctx.eval_contraction(flags) == "i8-digits"
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
    oi = run(ctx, dev, [coef], S, grid, True, flags)
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_EVAL_WG_WAVES
    try:
        for kv in sorted(EVAL_KERNEL_NAMES):
            ctx.set_option(SF_OPT_EVAL_KERNEL, kv)
            o = run(ctx, dev, [coef], S, grid, True, flags)
            assert np.array_equal(o.view(np.int32), oi.view(np.int32)), kv
        # the register tile with 8-wave (512-pixel) workgroups
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_TILE)
        ctx.set_option(SF_OPT_EVAL_WG_WAVES, 8)
        o = run(ctx, dev, [coef], S, grid, True, flags)
        assert np.array_equal(o.view(np.int32), oi.view(np.int32)), "8 waves"
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
        ctx.set_option(SF_OPT_EVAL_WG_WAVES, 0)
    try:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_TILE)
        of = run(ctx, dev, [coef], S, grid, False, flags)
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
    assert np.array_equal(oi[fb].view(np.int32), of[fb].view(np.int32))
    assert np.all(oi[[9, 31], 0::2] == 1.0) and np.all(oi[[9, 31], 1::2] == 0.0)
    good = [s for s in range(S) if s not in fb]
    np.testing.assert_allclose(oi[good], of[good], rtol=0, atol=3e-7)
    assert not np.array_equal(oi[good].view(np.int32), of[good].view(np.int32))
    cpix = okl.cpix_matrix(pp, x, y)
    ok = np.isfinite(coef).all(axis=1)
    want = okl.eval_planes(okl.eval_phase_screens(coef[ok], cpix))
    np.testing.assert_allclose(oi[ok].reshape(want.shape), want, rtol=0, atol=2e-6)
    # unscrubbed: the NaN / Inf rows stay NaN, the rest is unchanged
    on = run(ctx, dev, [coef], S, grid, True, SF_EVAL_FAST_SINCOS)
    assert np.isnan(on[[9, 31]]).all()
    on[[9, 31]] = oi[[9, 31]]
    assert np.array_equal(on.view(np.int32), oi.view(np.int32))


def test_int_grid_out_of_digit_range_keeps_fp64(ctx, dev):
    """A grid whose |Cpix| exceeds the 36-bit digits (piercepoints ~1e5 TAN
    pixels away: |Cpix| ~ 1e4 > 2^10.9) keeps the fp64 contraction for the
    whole call, and still matches the oracle."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, SF_OPT_EVAL_INT
    rng = np.random.default_rng(3)
    D, grid = 48, 32
    pp = np.stack([rng.uniform(-1e5, 1e5, D), rng.uniform(-1e5, 1e5, D), np.zeros(D)], 1)
    x = np.linspace(-500.0, 500.0, grid)
    ctx.set_basis(pp)
    ctx.set_grid(x, x)
    flags = 1 | SF_EVAL_FAST_SINCOS
    assert ctx.eval_contraction(flags) == "f64"
    coef = rng.normal(0, 1e-4, size=(19, D))
    oi = run(ctx, dev, [coef], 19, grid, True, flags)
    of = run(ctx, dev, [coef], 19, grid, False, flags)
    assert np.array_equal(oi.view(np.int32), of.view(np.int32))
    cpix = okl.cpix_matrix(pp, x, x)
    assert np.abs(cpix).max() > 2 ** 11
    want = okl.eval_planes(okl.eval_phase_screens(coef, cpix))
    np.testing.assert_allclose(oi.reshape(want.shape), want, rtol=0, atol=2e-6)
    # an ordinary grid of the same D does take the integer contraction
    pp2, x2, y2 = grid_for(D, 64, seed=9)
    ctx.set_basis(pp2)
    ctx.set_grid(x2, y2)
    assert ctx.eval_contraction(flags) == "i8-digits"
    ctx.set_option(SF_OPT_EVAL_INT, 0)
    try:
        assert ctx.eval_contraction(flags) == "f64"
    finally:
        ctx.set_option(SF_OPT_EVAL_INT, -1)


def test_int_many_launches_checksums(ctx, dev):
    """A call of more slots than one integer launch holds (1 M slot digit
    buffer): 1.1 M slots into a 32-slot ring in checksum mode; the sums of the
    last slots (second launch) equal those of the same slots evaluated alone,
    and the first slots' likewise."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB
    D, grid = 50, 32
    pp, x, y = grid_for(D, grid, seed=11)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    flags = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS
    assert ctx.eval_contraction(flags) == "i8-digits"
    S = 1_100_000
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    coef = torch.randn((S, D), generator=g, device=dev, dtype=torch.float64) * 0.01
    coef[S - 7, 3] = float("nan")
    ring = 32
    out = torch.empty((ring, 4, grid, grid), dtype=torch.float32, device=dev)
    sums = torch.zeros(S, dtype=torch.int32, device=dev)
    ctx.eval_sums(coef, S, out, sums, ring, flags=flags)
    torch.cuda.synchronize()
    for a, b in ((0, 40), (S - 40, S)):
        part = coef[a:b].contiguous()
        o = torch.empty((b - a, 4, grid, grid), dtype=torch.float32, device=dev)
        s2 = torch.zeros(b - a, dtype=torch.int32, device=dev)
        ctx.eval_sums(part, b - a, o, s2, b - a, flags=flags)
        torch.cuda.synchronize()
        assert torch.equal(s2, sums[a:b]), (a, b)


def test_int_launches_on_two_streams(ctx, dev):
    """Two integer-contraction calls on one context, issued on two streams
    without a host sync between them: the second call's digit prepass
    rewrites the context's slot-digit buffer only after the first call's
    kernel has read it (the kdig_read event), so both results equal the
    same calls run one after the other."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB
    D, grid = 50, 64
    pp, x, y = grid_for(D, grid, seed=13)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    flags = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS
    assert ctx.eval_contraction(flags) == "i8-digits"
    S = 20000
    g = torch.Generator(device=dev)
    g.manual_seed(21)
    ca = torch.randn((S, D), generator=g, device=dev, dtype=torch.float64) * 0.01
    cb = torch.randn((S, D), generator=g, device=dev, dtype=torch.float64) * 0.02
    want = []
    for c in (ca, cb):
        o = torch.empty((S, 4, grid, grid), dtype=torch.float32, device=dev)
        ctx.eval(c, S, o, S, flags)
        torch.cuda.synchronize()
        want.append(o)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = [torch.full((S, 4, grid, grid), -5.0, dtype=torch.float32, device=dev)
            for _ in range(2)]
    torch.cuda.synchronize()
    try:
        for st, c, o in ((s1, ca, outs[0]), (s2, cb, outs[1])):
            ctx.set_stream(st.cuda_stream)
            ctx.eval(c, S, o, S, flags)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for got, w in zip(outs, want):
        assert torch.equal(got.view(torch.int32), w.view(torch.int32))


def test_int_range_check_negative_beta_and_bad_grid(ctx, dev):
    """|Cpix| = (d^2 / r0^2)^(beta / 2) / 2 grows toward the NEAREST grid
    point when beta < 0: a piercepoint 1e-3 from a grid point makes it
    ~5e4 > 2^10.9 at beta = -1, so the call keeps the fp64 contraction (the
    range check takes the nearest point as well as the farthest) and still
    matches the oracle; non-finite grid coordinates are refused."""
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, ScreenFitError
    rng = np.random.default_rng(17)
    D, grid = 48, 32
    x = np.linspace(-500.0, 500.0, grid)
    pp = np.stack([rng.uniform(-400, 400, D), rng.uniform(-400, 400, D), np.zeros(D)], 1)
    pp[7, 0], pp[7, 1] = x[3] + 1e-3, x[5]
    flags = 1 | SF_EVAL_FAST_SINCOS
    ctx.set_basis(pp, 100.0, -1.0)
    ctx.set_grid(x, x)
    try:
        assert ctx.eval_contraction(flags) == "f64"
        coef = rng.normal(0, 1e-7, size=(19, D))
        o = run(ctx, dev, [coef], 19, grid, True, flags)
        cpix = okl.cpix_matrix(pp, x, x, beta=-1.0)
        assert np.abs(cpix).max() > 2 ** 11
        want = okl.eval_planes(okl.eval_phase_screens(coef, cpix))
        np.testing.assert_allclose(o.reshape(want.shape), want, rtol=0, atol=2e-6)
        bad = x.copy()
        bad[4] = np.nan
        with pytest.raises(ScreenFitError):
            ctx.set_grid(bad, x)
    finally:
        ctx.set_basis(pp, 100.0, 5.0 / 3.0)

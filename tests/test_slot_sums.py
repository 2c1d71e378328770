"""Per-slot output checksums (sf_kl_eval_sums): the discard + checksum mode
of the evaluation (whose cubes cannot all
stay resident).  Needs an MI355X: every test is marked ``gpu``.

The checksum of a slot is the sum, mod 2^32, of the 32-bit words of its
[4][ny][nx] cube as stored.  Checked against the same sum taken on the host
from the cube the same launch wrote, for every kernel family, ragged grids,
a ring smaller than the slot count, and the gain (amplitude) path; the cube
bits must equal those of the plain sf_kl_eval / sf_kl_eval_gain launch.
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


def host_sums(cube):
    """[n, 4, ny, nx] float32 -> per-slot sum mod 2^32 of the 32-bit words."""
    w = np.ascontiguousarray(cube).view(np.uint32).reshape(cube.shape[0], -1)
    return (w.astype(np.uint64).sum(axis=1, dtype=np.uint64)
            & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def grid_for(n_dir, grid, seed):
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=2, n_freq=1, n_dir=n_dir, seed=seed)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (grid - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    assert len(x) == grid and len(y) == grid
    return pp, x, y


@pytest.mark.parametrize("n_dir,grid,kernel", [
    (20, 256, "auto"), (20, 256, "tile"), (50, 64, "auto"), (7, 17, "auto"),
    (12, 40, "gain")])
def test_eval_slot_sums(ctx, dev, n_dir, grid, kernel):
    from ska_sdp_screen_fitting_amd._lib import (
        SF_EVAL_FAST_SINCOS, SF_EVAL_KERNEL_AUTO, SF_EVAL_KERNEL_TILE,
        SF_EVAL_NAN_SCRUB, SF_EVAL_NT_STORES, SF_OPT_EVAL_KERNEL)
    pp, x, y = grid_for(n_dir, grid, 5)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    rng = np.random.default_rng(n_dir * grid)
    S = 45  # ragged slot groups
    coef = torch.from_numpy(rng.normal(0, 0.01, size=(S, n_dir))).to(dev)
    coef[11, n_dir // 3] = float("nan")
    gain = kernel == "gain"
    cxx = cyy = None
    if gain:
        cxx = torch.from_numpy(rng.normal(0, 0.05, size=(S, n_dir))).to(dev)
        cyy = torch.from_numpy(rng.normal(0, 0.05, size=(S, n_dir))).to(dev)
    flags = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES
    shape = (S, 4, len(y), len(x))
    try:
        ctx.set_option(SF_OPT_EVAL_KERNEL,
                       SF_EVAL_KERNEL_TILE if kernel == "tile" else SF_EVAL_KERNEL_AUTO)
        out = torch.full(shape, -7.0, dtype=torch.float32, device=dev)
        sums = torch.zeros(S, dtype=torch.int32, device=dev)
        ctx.eval_sums(coef, S, out, sums, S, coef_xx=cxx, coef_yy=cyy, flags=flags)
        # a ring of 7 entries: the sums still cover every slot
        ring = torch.empty((7,) + shape[1:], dtype=torch.float32, device=dev)
        sums7 = torch.zeros(S, dtype=torch.int32, device=dev)
        ctx.eval_sums(coef, S, ring, sums7, 7, coef_xx=cxx, coef_yy=cyy, flags=flags)
        plain = torch.full(shape, -7.0, dtype=torch.float32, device=dev)
        if gain:
            ctx.eval_gain(coef, cxx, cyy, S, plain, S, flags)
        else:
            ctx.eval(coef, S, plain, S, flags)
        torch.cuda.synchronize()
    finally:
        ctx.set_option(SF_OPT_EVAL_KERNEL, SF_EVAL_KERNEL_AUTO)
    o = out.cpu().numpy()
    got = sums.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, host_sums(o))
    np.testing.assert_array_equal(sums7.cpu().numpy().view(np.uint32), got)
    np.testing.assert_array_equal(o.view(np.uint32), plain.cpu().numpy().view(np.uint32))


def test_eval_sums_rejects_bad_operands(ctx, dev):
    pp, x, y = grid_for(6, 16, 2)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    S = 5
    coef = torch.zeros((S, 6), dtype=torch.float64, device=dev)
    out = torch.empty((S, 4, 16, 16), dtype=torch.float32, device=dev)
    with pytest.raises(TypeError):
        ctx.eval_sums(coef, S, out, torch.zeros(S, dtype=torch.int64, device=dev))
    with pytest.raises(ValueError):
        ctx.eval_sums(coef, S, out, torch.zeros(S - 1, dtype=torch.int32, device=dev))


def test_config5_shape_streamed_slots_vs_oracle(ctx, dev):
    """Config-5 pixel grid (D = 50, 512^2) streamed through a 4-entry ring
    with checksums: sampled slots evaluated alone match the streamed
    checksums bit for bit and the oracle within 2e-6 (fp32 sincos)."""
    from ska_sdp_screen_fitting_amd._lib import (
        SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB, SF_EVAL_NT_STORES)
    D, N = 50, 512
    pp, x, y = grid_for(D, N, 9)
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    S = 64
    rng = np.random.default_rng(50)
    coef_np = rng.normal(0, 0.01, size=(S, D))
    coef = torch.from_numpy(coef_np).to(dev)
    flags = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES
    ring = torch.empty((4, 4, N, N), dtype=torch.float32, device=dev)
    sums = torch.zeros(S, dtype=torch.int32, device=dev)
    ctx.eval_sums(coef, S, ring, sums, 4, flags=flags)
    torch.cuda.synchronize()
    got = sums.cpu().numpy().view(np.uint32)
    cpix = okl.cpix_matrix(pp, x, y)
    for k in (0, 29, 63):
        one = torch.empty((1, 4, N, N), dtype=torch.float32, device=dev)
        ctx.eval(coef[k:k + 1], 1, one, 1, flags)
        torch.cuda.synchronize()
        o = one.cpu().numpy()
        assert host_sums(o)[0] == got[k], k
        want = okl.eval_planes(okl.eval_phase_screens(coef_np[k:k + 1], cpix))
        np.testing.assert_allclose(o.reshape(want.shape), want, rtol=0, atol=2e-6)


def test_sharded_gpu_sums_equal_unsharded(ctx, dev):
    """The GPU side of antenna sharding: fit + checksum
    evaluation of each contiguous station shard -- reference phases passed
    in, as distributed.setup_shard hands them to a rank that does not hold
    the reference station -- gives, slot for slot, the same cube checksums
    as the unsharded run on one context."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    A, T, F, D, N = 12, 3, 2, 20, 64
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D, seed=11,
                       flag_frac=0.05, outlier_frac=0.02)
    pp, mra, mdec = geometry.piercepoints(s.dir_radec)
    cell = FIELD["width"] / (N - 0.5)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"],
                                cell, mra, mdec)
    ref = okl.reference_station(s.weight)
    st = station_orders(s.ant_pos, ref, min(20, D - 1))
    ctx.set_basis(pp)
    ctx.set_grid(x, y)
    refph = torch.from_numpy(np.ascontiguousarray(s.val[:, :, ref, :])).to(dev)

    def run(a0, a1, ref_phase):
        ph = torch.from_numpy(np.ascontiguousarray(s.val[:, :, a0:a1])).to(dev)
        wt = torch.from_numpy(np.ascontiguousarray(s.weight[:, :, a0:a1])).to(dev)
        coef = torch.empty_like(ph)
        ctx.fit(ph, wt, T, F, a1 - a0, st[a0:a1], ref_ant=ref, coef=coef,
                ant_offset=a0, ref_phase=ref_phase)
        n = T * F * (a1 - a0)
        out = torch.empty((16, 4, N, N), dtype=torch.float32, device=dev)
        sums = torch.zeros(n, dtype=torch.int32, device=dev)
        ctx.eval_sums(coef.reshape(n, D), n, out, sums, 16, flags=1)
        torch.cuda.synchronize()
        return sums.cpu().numpy().view(np.uint32).reshape(T, F, a1 - a0)

    full = run(0, A, None)
    assert len(np.unique(full)) > T * F * A // 2  # distinct cubes
    for a0, a1 in ((0, 5), (5, 12)):
        np.testing.assert_array_equal(run(a0, a1, refph), full[:, :, a0:a1])

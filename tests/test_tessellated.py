"""Tessellated (Voronoi) path: host template vs the oracle restatement and the
reference's anchors (CPU), fused gather + Gaussian kernel vs the oracle /
scipy.ndimage and the reference test criterion end to end (GPU).

Parity status: the reference's own tessellated path needs shapely, absent
from every interpreter here, so no raster was generated from it; the config-1
raster is pinned at every pixel by the reference's rendering of its own
``tessellated_0.fits`` (tests/test_tess_png_pin.py), and the finer grids by
the reference test's patch-pixel criterion plus the ring convention that
rendering confirms.
"""

import os

import numpy as np
import pytest

from conftest import FIELD, GOLDEN, load_golden
from oracle import voronoi as ov
from ska_sdp_screen_fitting_amd.voronoi_screen import (gaussian_weights,
                                                       read_patch_positions,
                                                       tessellation_template)

SKY = os.path.join(GOLDEN, "skymodel.txt")


def fixture_patches():
    g = load_golden("fixture_kl")
    pos = read_patch_positions(SKY)
    dirs = [str(d) for d in g["dir_names"]]
    return g, np.array([pos[d.strip("[]")] for d in dirs])


def test_patch_positions_vs_astropy():
    g, radec = fixture_patches()
    np.testing.assert_allclose(radec, g["radec_patch"], rtol=0, atol=1e-10)
    pos_o = ov.patch_positions(SKY)
    for k, v in read_patch_positions(SKY).items():
        np.testing.assert_allclose(v, pos_o[k], atol=1e-12)


@pytest.mark.parametrize("cell", [0.2, 0.1, 0.05, 0.02602])
def test_template_matches_oracle(cell):
    """The product's rings (min directed-edge index, clockwise)
    and the oracle's literal GEOS graph walk give the same raster."""
    _, radec = fixture_patches()
    lab, xy = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                    FIELD["width"], cell)
    lab_o, xy_o = ov.label_raster(radec[:, 0], radec[:, 1], FIELD["rad"],
                                  FIELD["dec"], FIELD["width"], cell)
    np.testing.assert_allclose(xy, xy_o, atol=1e-9)
    np.testing.assert_array_equal(lab, lab_o)


def test_template_anchors():
    g, radec = fixture_patches()
    lab, xy = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                    FIELD["width"], 0.2)
    n = lab.shape[0]
    assert n == 17 and lab.min() == 1 and lab.max() == 7
    # patch pixels (via the cube's SIN WCS, golden from astropy) own their label
    px, py = g["patch_pix17"]
    for k in range(len(px)):
        c, r = int(np.round(px[k])), int(np.round(py[k]))
        if 0 <= r < n and 0 <= c < n:
            assert lab[r, c] == k + 1
    # Q10: not the nearest-direction map.  7 of 289 pixels differ with the
    # GEOS ring convention; the survey's probe counted 5 with its own
    # polygonize emulation (rings from Voronoi.regions), whose convention
    # moves (6, 1) and (7, 3) -- two of the pixels that depend on the ring's
    # start vertex / direction (profiles/round3_tess_ring_conventions.txt)
    yy, xx = np.mgrid[0:n, 0:n]
    near = ((xx[..., None] - xy[:, 0]) ** 2 + (yy[..., None] - xy[:, 1]) ** 2).argmin(-1) + 1
    assert np.argwhere(near != lab).tolist() == [[1, 9], [2, 3], [5, 6], [5, 11],
                                                 [6, 1], [6, 10], [7, 3]]


CONFIG_CELLS = [0.2, 0.1, 0.05, 0.02602]


@pytest.mark.parametrize("cell", CONFIG_CELLS)
def test_patch_pixels_own_their_cell(cell):
    """The reference test's anchor (tests/test_make_aterm_images.py: the
    cube at each patch's pixel, via the cube's own SIN WCS, is that patch's
    value) at every cell size the configs use, down to config 2's 128^2."""
    from ska_sdp_screen_fitting_amd import geometry
    g, radec = fixture_patches()
    lab, xy = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                    FIELD["width"], cell)
    n = lab.shape[0]
    assert n == geometry.grid_size(FIELD["width"], cell)
    assert lab.min() == 1 and lab.max() == len(radec)
    px, py = geometry.sin_world2pix(g["radec_patch"][:, 0], g["radec_patch"][:, 1],
                                    (FIELD["rad"], FIELD["dec"]), (n / 2.0, n / 2.0),
                                    (-cell, cell))
    n_in = 0
    for k in range(len(px)):
        c, r = int(np.round(px[k])), int(np.round(py[k]))
        if 0 <= r < n and 0 <= c < n:
            n_in += 1
            assert lab[r, c] == k + 1, (k, r, c, lab[r, c])
    assert n_in >= 5


@pytest.mark.parametrize("cell", CONFIG_CELLS)
def test_no_pixel_claimed_twice(cell):
    """No pixel centre of the fixture's rasters lies on a shared cell edge at
    the configs' cell sizes, so the painting order -- shapely polygonize
    order in the reference, direction order here -- cannot change a label."""
    from ska_sdp_screen_fitting_amd.voronoi_screen import cell_rings, rasterize_cell
    _, radec = fixture_patches()
    rings = cell_rings(radec, FIELD["rad"], FIELD["dec"], FIELD["width"], cell)
    n = tessellation_template(radec, FIELD["rad"], FIELD["dec"], FIELD["width"],
                              cell)[0].shape[0]
    claims = sum(rasterize_cell(r, n).astype(int) for r in rings)
    assert int((claims > 1).sum()) == 0


def test_tie_rule_later_cell_wins():
    """A pixel centre exactly on the edge two cells share is kept by both
    exact border tests (shapely: on the boundary is not disjoint) and takes
    the cell painted last."""
    from ska_sdp_screen_fitting_amd.voronoi_screen import paint_cells, rasterize_cell
    a = [(0.0, 0.0), (5.0, 0.0), (5.0, 9.0), (0.0, 9.0), (0.0, 0.0)]
    b = [(5.0, 0.0), (9.0, 0.0), (9.0, 9.0), (5.0, 9.0), (5.0, 0.0)]
    ma, mb = rasterize_cell(a, 10), rasterize_cell(b, 10)
    assert ma[:, 5].all() and mb[:, 5].all()  # column x = 5: on both edges
    lab = paint_cells([a, b], 10)  # b (label 2) painted last
    assert np.all(lab[:, 5] == 2) and np.all(lab[:, 0] == 1) and np.all(lab[:, 9] == 2)
    lab = paint_cells([b, a], 10)  # a (label 2) painted last
    assert np.all(lab[:, 5] == 2) and np.all(lab[:, 0] == 2) and np.all(lab[:, 9] == 1)


def test_geos_polygonize_restatement():
    """oracle.voronoi.geos_polygonize on two unit squares sharing an edge,
    against the GEOS Polygonizer walked by hand: directed edges in line
    order (de0 a -> b, de1 b -> a); de0 of line 0 runs east with the outer
    face on its right (a counter-clockwise ring: a hole, dropped); de1
    (1,0) -> (0,0) starts square A, clockwise; de2 (1,0) -> (1,1) starts
    square B."""
    from oracle.voronoi import geos_polygonize
    segs = [((0, 0), (1, 0)), ((1, 0), (1, 1)), ((1, 1), (0, 1)), ((0, 1), (0, 0)),
            ((1, 0), (2, 0)), ((2, 0), (2, 1)), ((2, 1), (1, 1))]
    assert geos_polygonize(segs) == [
        [(1.0, 0.0), (0.0, 0.0), (0.0, 1.0), (1.0, 1.0), (1.0, 0.0)],
        [(1.0, 0.0), (1.0, 1.0), (2.0, 1.0), (2.0, 0.0), (1.0, 0.0)]]


@pytest.mark.parametrize("cell", CONFIG_CELLS)
def test_rings_follow_geos_convention(cell):
    """Every cell ring is clockwise and starts at the start vertex of the
    lowest-index directed edge bounding it; cells paint in that order (the
    GEOS Polygonizer convention, voronoi_screen._rings).  The pixels a
    different convention would move are listed per cell size in
    profiles/round3_tess_ring_conventions.txt (tools/tess_ring_conventions.py):
    2 / 289, 1 / 1156, 16 / 4489, 22 / 16384."""
    from oracle.voronoi import geos_polygonize
    from ska_sdp_screen_fitting_amd.voronoi_screen import _rings
    from scipy.spatial import Voronoi
    _, radec = fixture_patches()
    rings, xy, n, order = _rings(radec, FIELD["rad"], FIELD["dec"], FIELD["width"], cell)
    for r in rings:
        area = sum(x0 * y1 - x1 * y0 for (x0, y0), (x1, y1) in zip(r[:-1], r[1:]))
        assert area < 0
    # the oracle's graph walk on the same ridges gives the same rings, in
    # the painting order
    from ska_sdp_screen_fitting_amd import geometry
    k = np.arange(64)
    rad, dec, width = FIELD["rad"], FIELD["dec"], FIELD["width"]
    crval, crpix, cdelt = (rad, dec), (n / 2.0, n / 2.0), (-cell, cell)
    b = (rad + width / 2.0, dec - width / 2.0, rad - width / 2.0, dec + width / 2.0)
    fx0, fy0 = geometry.sin_world2pix(max(b[0], radec[:, 0].max() + 0.1),
                                      min(b[1], radec[:, 1].min() - 0.1), crval, crpix, cdelt)
    fx1, fy1 = geometry.sin_world2pix(min(b[2], radec[:, 0].min() - 0.1),
                                      max(b[3], radec[:, 1].max() + 0.1), crval, crpix, cdelt)
    radius = 2.0 * np.hypot(float(fx1) - float(fx0), float(fy1) - float(fy0))
    outer = xy.mean(axis=0) + radius * np.stack([np.cos(np.pi / 32.0 * k),
                                                 np.sin(np.pi / 32.0 * k)], axis=1)
    vor = Voronoi(np.vstack([xy, outer]))
    walked = geos_polygonize([vor.vertices[r] for r in vor.ridge_vertices if -1 not in r])
    assert walked == [rings[i] for i in order]


@pytest.mark.parametrize("sigma", [0.5, 1.3, 4.2])
def test_gaussian_weights_match_scipy(sigma):
    from scipy.ndimage import _filters
    r, w = gaussian_weights(sigma)
    np.testing.assert_array_equal(w, _filters._gaussian_kernel1d(sigma, 0, r)[::-1])


# ----------------------------------------------------------------- GPU ----
def _tess_gpu(lab, phase, smooth):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ny, nx = lab.shape
    S, D = phase.shape
    lab_d = torch.from_numpy(np.ascontiguousarray(lab, np.int32)).to(dev)
    ph_d = torch.from_numpy(np.ascontiguousarray(phase)).to(dev)
    out = torch.full((S, 4, ny, nx), -5.0, dtype=torch.float32, device=dev)
    ctx.tess_fill(lab_d, nx, ny, ph_d, D, S, out, smooth_pix=smooth)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("cell,smooth", [(0.2, 0.0), (0.2, 0.5), (0.05, 1.3),
                                         (0.02602, 4.0), (0.02602, 10.0),
                                         (0.05, 0.0), (0.02602, 0.0)])
def test_tess_kernel_vs_oracle(cell, smooth):
    """Fused gather + Gaussian (smooth <= 6 px) and, at 10 px (radius 40),
    gather then the separable passes of sf_smooth -- both vs scipy."""
    g, radec = fixture_patches()
    lab, _ = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                   FIELD["width"], cell)
    ref = int(g["ref_ant"])
    ph = (g["val"] - g["val"][:, :, ref:ref + 1, :])[:, 3].reshape(-1, 7)[:150]
    got = _tess_gpu(lab, ph, smooth)
    want = ov.gather_planes(lab, ph)
    if smooth > 0:
        want = ov.smooth(want, smooth)
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-6)
    else:
        # fp64 cos/sin cast once to fp32: at most 1 ulp from numpy's libm
        assert np.max(np.abs(got.view(np.int32) - want.view(np.int32))) <= 1


@pytest.mark.gpu
def test_make_aterm_image_fixture_tessellated(tmp_path):
    """tests/test_fit_screens.py::test_fit_voronoi_screens (abs(), 1e-4)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    g = load_golden("fixture_kl")
    outroot = str(tmp_path / "tessellated")
    make_aterm_image(os.path.join(GOLDEN, "fixture_kl.npz"), soltabname="phase000",
                     screen_type="tessellated", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50], skymodel=SKY,
                     solsetname="sol000", padding_fraction=0, cellsize_deg=0.2,
                     smooth_deg=0.1, ncpu=0)
    for f in ("tessellated_0.fits", "tessellated_template.fits", "tessellated.txt"):
        assert os.path.isfile(str(tmp_path / f)), f
    hdr, cube = sffits.read_cube(outroot + "_0.fits")
    assert cube.shape == (20, 12, 62, 4, 17, 17)
    ph = np.asarray(g["val"])
    corr = ph - ph[:, :, 0:1, :]
    px, py = g["patch_pix17"]
    n_in = 0
    for i in range(len(px)):
        col, row = int(np.round(px[i])), int(np.round(py[i]))
        if 0 <= row < 17 and 0 <= col < 17:
            n_in += 1
            for p, fn in ((0, np.cos), (1, np.sin), (2, np.cos), (3, np.sin)):
                err = np.abs(cube[:, :, :, p, row, col] - fn(corr[..., i]))
                assert np.all(err < 1e-4), (i, p, err.max())
    assert n_in >= 5
    # the whole cube vs the oracle (gather + scipy gaussian, smooth 0.5 px)
    _, radec = fixture_patches()
    lab, _ = tessellation_template(radec, FIELD["rad"], FIELD["dec"],
                                   FIELD["width"], 0.2)
    want = ov.smooth(ov.gather_planes(lab, corr), 0.5)
    np.testing.assert_allclose(cube, want, rtol=0, atol=1e-6)


def _scrub(planes):
    out = planes.copy()
    for p in range(4):
        v = out[..., p, :, :]
        v[np.isnan(v)] = 0.0 if p % 2 else 1.0
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("sigma", [0.7, 10.0, 23.5])
def test_smooth_vs_scipy(sigma):
    """sf_smooth (any radius) vs scipy.ndimage.gaussian_filter per image,
    a non-square grid smaller than the radius, one NaN pixel spreading over
    its neighbourhood, then the scrub (screen.py:353-378 order) and the FITS
    byte swap."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_BIG_ENDIAN, SF_EVAL_NAN_SCRUB
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(int(sigma * 10))
    S, ny, nx = 3, 37, 53
    cube = rng.normal(size=(S, 4, ny, nx)).astype(np.float32)
    cube[1, 2, 5, 7] = np.nan
    want = _scrub(ov.smooth(cube, sigma))
    for flags in (SF_EVAL_NAN_SCRUB, SF_EVAL_NAN_SCRUB | SF_EVAL_BIG_ENDIAN):
        d = torch.from_numpy(cube.copy()).to(dev)
        ctx.smooth(d, nx, ny, 4 * S, sigma, flags)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        if flags & SF_EVAL_BIG_ENDIAN:
            got = got.byteswap()
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-6)
    assert np.isnan(ov.smooth(cube, sigma)[1, 2]).sum() > 1  # it did spread


@pytest.mark.gpu
def test_tess_rejects_bad_labels():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lab = np.ones((8, 8), np.int32)
    lab[3, 3] = 0
    with pytest.raises(ValueError):
        _tess_gpu(lab, np.zeros((2, 3)), 0.0)
    lab[3, 3] = 4
    with pytest.raises(ValueError):
        _tess_gpu(lab, np.zeros((2, 3)), 0.0)


@pytest.mark.gpu
def test_tess_label_check_not_fooled_by_reused_storage():
    """The once-per-template label check is keyed on the tensor object: a
    new, invalid label tensor in the freed block of a validated one (the
    caching allocator hands it straight back, same size, same _version) is
    checked again and refused."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ph = torch.zeros((2, 3), dtype=torch.float64, device=dev)
    out = torch.empty((2, 4, 8, 8), dtype=torch.float32, device=dev)
    good = torch.ones((8, 8), dtype=torch.int32, device=dev)
    ctx.tess_fill(good, 8, 8, ph, 3, 2, out)
    del good
    # (normally the same storage block; refused either way)
    bad = torch.full((8, 8), 9, dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        ctx.tess_fill(bad, 8, 8, ph, 3, 2, out)


@pytest.mark.gpu
@pytest.mark.parametrize("n,S", [(17, 70), (128, 45), (64, 33), (33, 1)])
def test_tess_gather_amplitudes_nan_byteswap(n, S):
    """The unsmoothed table + gather-store kernels (float4 runs when
    n^2 % 4 == 0, scalar tail otherwise; 4 / 8 / 16 waves, slot chunks of
    3 to 64, ragged last chunks): gain tables A cos / A sin,
    NaN phases and amplitudes (scrubbed to 1 / 0, or left NaN), FITS byte
    order -- vs fp64 numpy cast once to fp32 (<= 1 ulp)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_BIG_ENDIAN, SF_EVAL_NAN_SCRUB
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(n * 1000 + S)
    D = 9
    lab = rng.integers(1, D + 1, size=(n, n)).astype(np.int32)
    ph = rng.uniform(-20.0, 20.0, size=(S, D))
    ax = 10.0 ** rng.normal(0.0, 0.3, size=(S, D))
    ay = 10.0 ** rng.normal(0.0, 0.3, size=(S, D))
    ph[S // 2, 3] = np.nan
    ax[S - 1, 5] = np.nan
    tab = np.stack([ax * np.cos(ph), ax * np.sin(ph), ay * np.cos(ph),
                    ay * np.sin(ph)], axis=-1).astype(np.float32)  # [S][D][4]
    want = np.moveaxis(tab[:, lab - 1, :], -1, 1)  # [S][4][n][n]
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in (("lab", lab), ("ph", ph), ("ax", ax), ("ay", ay))}
    from ska_sdp_screen_fitting_amd._lib import SF_OPT_TESS_SLOTS, SF_OPT_TESS_WAVES
    cases = [(fl, 0, 0) for fl in (SF_EVAL_NAN_SCRUB,
                                   SF_EVAL_NAN_SCRUB | SF_EVAL_BIG_ENDIAN, 0)]
    cases += [(SF_EVAL_NAN_SCRUB, w, k) for w, k in ((8, 3), (16, 16), (4, 64))]
    for flags, waves, slots in cases:
        out = torch.full((S, 4, n, n), -5.0, dtype=torch.float32, device=dev)
        ctx.set_option(SF_OPT_TESS_WAVES, waves)
        ctx.set_option(SF_OPT_TESS_SLOTS, slots)
        try:
            ctx.tess_fill(d["lab"], n, n, d["ph"], D, S, out, amp_xx=d["ax"],
                          amp_yy=d["ay"], smooth_pix=0.0, flags=flags)
            torch.cuda.synchronize()
        finally:
            ctx.set_option(SF_OPT_TESS_WAVES, 0)
            ctx.set_option(SF_OPT_TESS_SLOTS, 0)
        got = out.cpu().numpy()
        if flags & SF_EVAL_BIG_ENDIAN:
            got = got.byteswap()
        exp = _scrub(want) if flags & SF_EVAL_NAN_SCRUB else want
        nan = np.isnan(exp)
        assert np.array_equal(np.isnan(got), nan)
        if flags & SF_EVAL_NAN_SCRUB:
            assert not nan.any()
        diff = np.abs(got.view(np.int32).astype(np.int64) - exp.view(np.int32))
        assert diff[~nan].max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("nx,ny,sigma", [(17, 17, 0.5), (53, 37, 1.3), (128, 128, 0.0),
                                         (96, 40, 2.5), (40, 96, 5.0),
                                         (300, 260, 4.0), (64, 64, 6.0), (20, 9, 0.3)])
def test_tess_kernels_agree_with_tile_kernel(nx, ny, sigma):
    """The table + gather (R = 0), interior-lookup smoothing (R <= 24,
    SF_OPT_TESS_BOX = 1) and wide-tile smoothing kernels write the
    same bits as the round-1 fused 16 x 16 tile kernel (SF_OPT_TESS_TILE):
    ragged tiles and slot chunks, NaN phases and amplitudes, labels of every
    cell (noise, so most pixels are cell boundaries) next to a constant
    region (interior pixels), scrub / byte-swap flags."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_BIG_ENDIAN, SF_EVAL_NAN_SCRUB,
                                                 SF_OPT_TESS_BOX, SF_OPT_TESS_TILE)
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(nx * 7 + ny)
    D, S = 11, 21
    lab = rng.integers(1, D + 1, size=(ny, nx)).astype(np.int32)
    lab[: ny // 2, : nx // 2] = 3  # a constant region too
    ph = rng.uniform(-9.0, 9.0, size=(S, D))
    ph[4, 3] = np.nan
    ax = 10.0 ** rng.normal(0.0, 0.3, size=(S, D))
    ax[S - 1, 2] = np.nan
    ay = 10.0 ** rng.normal(0.0, 0.3, size=(S, D))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in (("lab", lab), ("ph", ph), ("ax", ax), ("ay", ay))}
    # without a YY amplitude planes 2 / 3 repeat 0 / 1 (smoothed once)
    for flags, yy in ((SF_EVAL_NAN_SCRUB, None), (SF_EVAL_NAN_SCRUB | SF_EVAL_BIG_ENDIAN, None),
                      (0, None), (SF_EVAL_NAN_SCRUB, t["ay"]), (0, t["ay"])):
        res = []
        for tile, box in ((1, 1), (0, 1), (0, 0)):
            out = torch.full((S, 4, ny, nx), -5.0, dtype=torch.float32, device=dev)
            ctx.set_option(SF_OPT_TESS_TILE, tile)
            ctx.set_option(SF_OPT_TESS_BOX, box)
            try:
                ctx.tess_fill(t["lab"], nx, ny, t["ph"], D, S, out, amp_xx=t["ax"],
                              amp_yy=yy, smooth_pix=sigma, flags=flags)
                torch.cuda.synchronize()
            finally:
                ctx.set_option(SF_OPT_TESS_TILE, 0)
                ctx.set_option(SF_OPT_TESS_BOX, -1)
            res.append(out.cpu().numpy().view(np.uint32))
        for k in (1, 2):
            assert np.array_equal(res[0], res[k]), (k, flags, yy is None,
                                                    int((res[0] != res[k]).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("cell,sigma,gain", [(0.02602, 0.5, False), (0.02602, 0.5, True),
                                             (0.01301, 0.5, True), (0.01301, 2.0, False),
                                             (0.01301, 3.0, True), (0.05, 6.0, False)])
def test_tess_box_kernel_on_voronoi_rasters(cell, sigma, gain):
    """The interior-lookup smoothing kernel on the fixture's own Voronoi
    rasters (large uniform cells: most pixels take the per-cell value)
    writes the same bits as the wide-tile kernel that sums every pixel, and
    matches scipy within 1e-6 (x max(1, A))."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import get_context
    from ska_sdp_screen_fitting_amd._lib import SF_EVAL_NAN_SCRUB, SF_OPT_TESS_BOX
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    g, radec = fixture_patches()
    lab, _ = tessellation_template(radec, FIELD["rad"], FIELD["dec"], FIELD["width"], cell)
    ny, nx = lab.shape
    ref = int(g["ref_ant"])
    ph = (g["val"] - g["val"][:, :, ref:ref + 1, :])[:, 5].reshape(-1, 7)[:40]
    ph[3, 2] = np.nan
    S, D = ph.shape
    rng = np.random.default_rng(3)
    ax = 10.0 ** rng.normal(0.0, 0.1, size=(S, D)) if gain else None
    ay = 10.0 ** rng.normal(0.0, 0.1, size=(S, D)) if gain else None
    dv = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    lab_d = torch.from_numpy(np.ascontiguousarray(lab, np.int32)).to(dev)
    res = []
    for box in (1, 0):
        out = torch.full((S, 4, ny, nx), -5.0, dtype=torch.float32, device=dev)
        ctx.set_option(SF_OPT_TESS_BOX, box)
        try:
            ctx.tess_fill(lab_d, nx, ny, dv(ph), D, S, out, amp_xx=dv(ax), amp_yy=dv(ay),
                          smooth_pix=sigma, flags=SF_EVAL_NAN_SCRUB)
            torch.cuda.synchronize()
        finally:
            ctx.set_option(SF_OPT_TESS_BOX, -1)
        res.append(out.cpu().numpy())
    assert np.array_equal(res[0].view(np.uint32), res[1].view(np.uint32))
    want = _scrub(ov.smooth(ov.gather_planes(lab, ph, ax, ay), sigma))
    scale = np.maximum(1.0, np.abs(want))
    assert np.max(np.abs(res[0] - want) / scale) <= 1e-6


def test_single_direction_template():
    """One direction (make_aterm_images.py:110-112 forces the tessellated
    screen then, Q14): the raster is the rasterized field box
    (voronoi_screen.py:241-259) and the griddata fill around it -- every
    pixel takes label 1; the oracle's restatement agrees."""
    _, radec = fixture_patches()
    one = radec[2:3]
    for cell in (0.2, 0.02602):
        lab, xy = tessellation_template(one, FIELD["rad"], FIELD["dec"], FIELD["width"], cell)
        lab_o, _ = ov.label_raster(one[:, 0], one[:, 1], FIELD["rad"], FIELD["dec"],
                                   FIELD["width"], cell)
        assert lab.min() == 1 and lab.max() == 1
        np.testing.assert_array_equal(lab, lab_o)
        assert xy.shape == (1, 2)


@pytest.mark.gpu
def test_make_aterm_image_one_direction_forces_tessellated(tmp_path):
    """Q14 end to end: a one-direction solution set asked for a KL screen
    is written as a tessellated one (the reference cannot fit a KL screen
    to one direction, make_aterm_images.py:110-112): every pixel of a slot
    is the referenced phase's cos / sin of that direction (the Gaussian of a
    constant image is that constant)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd import fits as sffits
    from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image
    g = load_golden("fixture_kl")
    k = 2
    src = {key: g[key] for key in ("times", "freqs", "ant_names", "ant_pos")}
    src.update(val=g["val"][..., k:k + 1], weight=g["weight"][..., k:k + 1],
               dir_names=g["dir_names"][k:k + 1], dir_radec=g["dir_radec"][k:k + 1])
    path = str(tmp_path / "one.npz")
    np.savez(path, **src)
    outroot = str(tmp_path / "one")
    make_aterm_image(path, soltabname="phase000", screen_type="kl", outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50], skymodel=SKY,
                     padding_fraction=0, cellsize_deg=0.2, smooth_deg=0.1, ncpu=0)
    assert os.path.isfile(outroot + "_template.fits")   # the Voronoi path ran
    _, cube = sffits.read_cube(outroot + "_0.fits")
    assert cube.shape == (20, 12, 62, 4, 17, 17)
    val = np.asarray(g["val"][..., k], np.float64)
    ph = val - val[:, :, 0:1]                            # reference station 0
    for p, fn in ((0, np.cos), (1, np.sin), (2, np.cos), (3, np.sin)):
        want = fn(ph)[..., None, None]
        np.testing.assert_allclose(cube[:, :, :, p], np.broadcast_to(want, cube[:, :, :, p].shape),
                                   rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_tess_fill_threads_on_two_streams():
    """VoronoiScreen.eval_device from two threads, each on its own stream
    (round 6): every call takes a private context, and a context's table /
    smoothing scratch is reused only after its previous fill's event, so
    the interleaved fills equal the same fills run one at a time."""
    import threading
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ska_sdp_screen_fitting_amd.voronoi_screen import VoronoiScreen
    g, radec = fixture_patches()
    lab, _ = tessellation_template(radec, FIELD["rad"], FIELD["dec"], FIELD["width"],
                                   0.05)
    scr = VoronoiScreen.__new__(VoronoiScreen)
    scr.data_rasertize_template = lab
    scr.device = 0
    scr._dev_cache = None
    dev = torch.device("cuda", 0)
    ref = int(g["ref_ant"])
    ph_all = (g["val"] - g["val"][:, :, ref:ref + 1, :]).reshape(-1, 7)
    n, S = 6, 96
    ny, nx = lab.shape
    phs = [torch.from_numpy(np.ascontiguousarray(ph_all[k * S:(k + 1) * S])).to(dev)
           for k in range(2 * n)]
    want = []
    for p in phs:
        o = torch.empty((S, 4, ny, nx), dtype=torch.float32, device=dev)
        scr.eval_device(p, o, smooth_pix=0.5)
        torch.cuda.synchronize()
        want.append(o.cpu().numpy())
    got = [None] * (2 * n)
    errors = []

    def worker(w):
        try:
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                for k in range(w, 2 * n, 2):
                    o = torch.empty((S, 4, ny, nx), dtype=torch.float32, device=dev)
                    scr.eval_device(phs[k], o, smooth_pix=0.5)
                    got[k] = o
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(w,)) for w in (0, 1)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors
    torch.cuda.synchronize()
    for k in range(2 * n):
        np.testing.assert_array_equal(got[k].cpu().numpy(), want[k])

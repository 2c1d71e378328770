"""The oracle (CPU restatement) against golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""

import numpy as np
import pytest

from conftest import FIELD, load_golden
from oracle import geometry as og
from oracle import kl as okl


def test_piercepoints_and_midpoint(golden):
    pp, mra, mdec = og.piercepoints(golden["dir_radec"])
    assert mra == golden["mid_ra"] and mdec == golden["mid_dec"]
    np.testing.assert_allclose(pp, golden["piercepoints"], rtol=0, atol=1e-8)


def test_grid_coords(golden):
    x, y = og.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"], 0.2,
                          float(golden["mid_ra"]), float(golden["mid_dec"]))
    np.testing.assert_allclose(x, golden["x17"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(y, golden["y17"], rtol=0, atol=1e-8)


@pytest.mark.parametrize("n", [17, 128, 256, 512])
def test_grid_coords_sizes(n):
    g = load_golden("fixture_kl")
    cell = {17: 0.2, 128: 0.02602, 256: 0.01301, 512: 0.006505}[n]
    x, y = og.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"], cell,
                          float(g["mid_ra"]), float(g["mid_dec"]))
    assert len(x) == n
    np.testing.assert_allclose(x, g[f"coords{n}_x"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(y, g[f"coords{n}_y"], rtol=0, atol=1e-8)


def test_basis(golden):
    c, pinv, u = okl.calculate_svd(golden["piercepoints"], 100.0, 5.0 / 3.0)
    np.testing.assert_allclose(c, golden["C"], rtol=1e-14, atol=0)
    sv = np.linalg.svd(golden["C"], compute_uv=False)
    cond = sv.max() / sv[sv > 1e-3].min()
    np.testing.assert_allclose(pinv, golden["pinv_c"], rtol=0,
                               atol=1e-14 * cond * np.abs(golden["pinv_c"]).max())
    # U only up to column signs
    np.testing.assert_allclose(np.abs(u.T @ golden["U"]), np.eye(len(c)),
                               atol=1e-9)


def test_reference_station(golden):
    assert okl.reference_station(golden["weight"]) == int(golden["ref_ant"])


def ill_conditioned_slots(g):
    """Slots whose final fit takes atan2 of near-zero values (the reference is
    chaotic there: its own output changes under 1-ulp perturbations)."""
    basis = okl.Basis(g["piercepoints"])
    ref = int(g["ref_ant"])
    val = g["val"] - g["val"][:, :, ref:ref + 1, :]
    bad = set()
    T, F, A, D = val.shape
    for t in range(T):
        for f in range(F):
            for a in range(A):
                o = int(g["orders"][t, f, a])
                w = g["w_out"][t, f, a]
                if o == 0 or a == ref or not np.any(w > 0):
                    continue
                unfl = np.where(w > 0)[0]
                c, pc, u = okl.calculate_svd(basis.pp[unfl], 100.0, 5.0 / 3.0)
                uk = u[:, :o]
                wd = np.diag(w[unfl].astype(np.float64))
                if np.linalg.svd(uk.T @ (wd @ u)[:, :o], compute_uv=False).min() <= 1e-3:
                    bad.add((t, f, a))
    return bad


def test_fit_matches_reference(golden):
    g = golden
    r = okl.run_phase(g["val"], g["weight"], g["ant_pos"], g["piercepoints"],
                      int(g["ref_ant"]), int(g["order"]))
    np.testing.assert_array_equal(r["orders"], g["orders"])
    np.testing.assert_array_equal(r["w_out"], g["w_out"])
    err = np.abs(r["coef"] - g["coef"]).max(axis=-1)
    bad = {tuple(i) for i in np.argwhere(err > 1e-9)}
    assert bad <= ill_conditioned_slots(g), sorted(bad)
    keep = np.ones(err.shape, bool)
    for i in bad:
        keep[i] = False
    scale = max(1.0, np.abs(g["coef"]).max())
    assert np.nanmax(err[keep]) <= 1e-9 * scale
    rerr = np.abs(r["resid"] - g["resid"]).max(axis=-1)
    assert np.nanmax(rerr[keep]) <= 1e-9


def test_eval_matches_reference(golden):
    g = golden
    cpix = okl.cpix_matrix(g["piercepoints"], g["x17"], g["y17"])
    for k, (f, s) in enumerate(g["pairs17"]):
        ph = okl.eval_phase_screens(g["coef"][:, f, s, :], cpix)
        planes = okl.eval_planes(ph)[:, 0:2]
        ref = g["kl17"][k].reshape(planes.shape)
        np.testing.assert_allclose(planes, ref, rtol=0, atol=1e-12)


def test_eval_128_matches_reference():
    g = load_golden("fixture_kl")
    cpix = okl.cpix_matrix(g["piercepoints"], g["x128"], g["y128"])
    t0, t1 = g["kl128_t"]
    for k, (f, s) in enumerate(g["pairs128"]):
        ph = okl.eval_phase_screens(g["coef"][t0:t1, f, s, :], cpix)
        planes = okl.eval_planes(ph)[:, 0:2]
        np.testing.assert_allclose(planes, g["kl128"][k].reshape(planes.shape),
                                   rtol=0, atol=1e-12)


def test_patch_pixels_sin_projection():
    g = load_golden("fixture_kl")
    for n, cell in ((17, 0.2), (128, 0.02602)):
        px, py = og.sin_world2pix(g["radec_patch"][:, 0], g["radec_patch"][:, 1],
                                  (FIELD["rad"], FIELD["dec"]), (n / 2, n / 2),
                                  (-cell, cell))
        np.testing.assert_allclose(px, g[f"patch_pix{n}"][0], atol=1e-8)
        np.testing.assert_allclose(py, g[f"patch_pix{n}"][1], atol=1e-8)


@pytest.mark.parametrize("name", ["ties4", "ties6"])
def test_fit_matches_reference_ties(name):
    """Slots with exactly two unflagged directions (tests/golden/
    make_golden_ties.py, the reference run at D = 4 / 6 with 40 % flags):
    the 2 x 2 subset C = [[0, b], [b, 0]] has |eigenvalues| |b| twice and
    the reference's order-1 fit keeps the first column of LAPACK's U, e_2.
    The oracle (numpy's LAPACK) reproduces the reference's orders, flags and
    coefficients, except at the slots where the reference's LAPACK left
    rounding residue in that U (``tie_residue``: its screen there is atan2
    of the residue)."""
    g = load_golden(name)
    n2 = (g["w_out"] > 0).sum(axis=-1) == 2
    assert n2.sum() >= 10
    r = okl.run_phase(g["val"], g["weight"], g["ant_pos"], g["piercepoints"],
                      int(g["ref_ant"]), int(g["order"]))
    np.testing.assert_array_equal(r["orders"], g["orders"])
    np.testing.assert_array_equal(r["w_out"], g["w_out"])
    keep = ~g["tie_residue"]
    err = np.abs(r["coef"] - g["coef"]).max(axis=-1)
    scale = max(1.0, np.abs(g["coef"]).max())
    assert np.nanmax(err[keep]) <= 1e-9 * scale
    assert np.nanmax(np.abs(r["resid"] - g["resid"]).max(axis=-1)[keep]) <= 1e-9
    assert np.all(err[keep & n2] <= 1e-9 * scale)

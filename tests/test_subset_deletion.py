"""The subset-basis deletion algorithm of kl_subset_secular_kernel
(kl_fit_fast.hip, SF_OPT_FIT_SUBSET_DELETION) restated step for step in
numpy -- secular roots relative to the nearer pole by bracketed Newton,
Loewner-recomputed z, deflation of negligible z, one deletion per flagged
direction in descending order -- against LAPACK's eigendecomposition of the
principal submatrix (stationscreen.py:390-430 computes the subset basis with
an SVD of C[idx][:, idx]).  CPU only: the GPU kernel's own test is
tests/test_gpu_parity.py::test_subset_deletion_bases_match_jacobi."""
import numpy as np
import pytest

from oracle import kl as okl

EPS = np.finfo(np.float64).eps


def _roots(lam, z):
    """Roots of sum z^2 / (lam - mu) between consecutive poles (lam
    ascending): (pole index, tau = root - pole)."""
    n = lam.size
    out = []
    for r in range(n - 1):
        lo, hi = lam[r], lam[r + 1]
        mid = lo + 0.5 * (hi - lo)
        fm = np.sum(z * z / (lam - mid))
        if fm >= 0.0:
            o, a, b = r, 0.0, mid - lo
        else:
            o, a, b = r + 1, mid - hi, 0.0
        zo2 = z[o] * z[o]
        others = np.arange(n) != o
        dl = lam[others] - lam[o]
        zz = z[others] ** 2
        t = 0.5 * (a + b)
        for _ in range(64):
            q = 1.0 / (dl - t)
            rest, drest = np.sum(zz * q), np.sum(zz * q * q)
            f = rest - zo2 / t
            if f == 0.0:
                break
            if f < 0.0:
                a = t
            else:
                b = t
            tn = t - (t * rest - zo2) / (rest + t * drest)
            if abs(tn - t) <= 4 * EPS * abs(t):
                t = tn
                break
            if not (a < tn < b):
                tn = 0.5 * (a + b)
            t = tn
            if not (b - a > 4 * EPS * max(abs(a), abs(b))):
                break
        else:
            raise AssertionError("root did not converge")
        out.append((o, t))
    return out


def delete(lam, U, j):
    """Eigenpairs (lam ascending, U columns) without row / column j."""
    m = lam.size
    z = U[j].copy()
    nd = np.abs(z) > 1e-14 * np.abs(z).max()
    ndi = np.nonzero(nd)[0]
    lz, zn = lam[ndi], z[ndi]
    assert np.all(np.diff(lz) > 1e-12 * np.abs(lam).max())
    roots = _roots(lz, zn)
    nn = ndi.size
    # Loewner
    zh = np.empty(nn)
    for k in range(nn):
        pr = 1.0
        for r, (o, t) in enumerate(roots):
            kp = r if r < k else r + 1
            pr *= ((lz[o] - lz[k]) + t) / (lz[kp] - lz[k])
        zh[k] = np.copysign(np.sqrt(abs(pr)), zn[k])
    W = np.empty((nn, nn - 1))
    for r, (o, t) in enumerate(roots):
        w = zh / ((lz - lz[o]) - t)
        W[:, r] = w / np.sqrt(np.sum(w * w))
    Y = np.concatenate([U[:, ndi] @ W, U[:, ~nd]], axis=1)
    mu = np.concatenate([[lz[o] + t for o, t in roots], lam[~nd]])
    Y = np.delete(Y, j, axis=0)
    o = np.argsort(mu, kind="stable")
    Y = Y[:, o]
    return mu[o], Y / np.sqrt(np.sum(Y * Y, axis=0))


def subset_basis(lam, U, unflagged):
    o = np.argsort(lam, kind="stable")
    lam, U = lam[o], U[:, o]
    for f in range(U.shape[0] - 1, -1, -1):
        if f not in unflagged:
            lam, U = delete(lam, U, f)
    return lam, U


@pytest.mark.parametrize("k", [1, 2, 3, 5])
def test_deletions_match_lapack_on_the_config5_basis(k):
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=1, n_freq=1, n_dir=50)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    c, _, _ = okl.calculate_svd(pp, 100.0, 5.0 / 3.0)
    lam, U = np.linalg.eigh(c)
    rng = np.random.default_rng(k)
    lmax = np.abs(lam).max()
    for _ in range(6):
        flagged = set(rng.choice(50, size=k, replace=False).tolist())
        keep = [d for d in range(50) if d not in flagged]
        mu, Y = subset_basis(lam, U, set(keep))
        l2, V2 = np.linalg.eigh(c[np.ix_(keep, keep)])
        assert np.abs(mu - l2).max() <= 1e-12 * lmax
        assert np.abs(Y.T @ Y - np.eye(len(keep))).max() <= 1e-13
        # eigenvectors to the conditioning of their eigenvalue gaps
        sg = np.sign(np.sum(Y * V2, axis=0))
        gaps = np.array([np.min(np.abs(np.delete(l2, r) - l2[r])) for r in range(len(l2))])
        err = np.abs(Y * sg - V2).max(axis=0)
        assert np.max(err * gaps / lmax) <= 1e-12


def test_ancestor_start_equals_the_chain():
    """SF_OPT_FIT_SUBSET_DELETION = 3 (and 1 on passes with many new masks)
    starts a mask from its nearest chain-built ancestor's pool entry (columns by |mu| descending, re-sorted
    into ascending order by the kernel): an exact permutation of the state
    the chain from the global basis has after the ancestor's deletions, so
    the remaining deletions give the same bits (mode 2 is the chain)."""
    from ska_sdp_screen_fitting_amd import geometry
    from ska_sdp_screen_fitting_amd.synthetic import make_solutions
    s = make_solutions(n_ant=2, n_time=1, n_freq=1, n_dir=20)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    c, _, _ = okl.calculate_svd(pp, 100.0, 5.0 / 3.0)
    lam, U = np.linalg.eigh(c)
    flagged = [17, 9, 4]                   # deleted in this (descending) order
    keep = set(range(20)) - set(flagged)
    mu, Y = subset_basis(lam, U, keep)     # the chain
    # the ancestor: the mask with its lowest flagged direction unflagged
    pa, Ya = subset_basis(lam, U, keep | {4})
    order = np.lexsort((np.arange(pa.size), -np.abs(pa)))  # the pool entry
    ent_l, ent_u = pa[order], Ya[:, order]
    asc = np.lexsort((np.arange(ent_l.size), ent_l))       # back to ascending
    l0, U0 = ent_l[asc], ent_u[:, asc]
    assert np.array_equal(l0, pa) and np.array_equal(U0, Ya)
    mu2, Y2 = delete(l0, U0, 4)            # row 4: every direction below 4 kept
    assert np.array_equal(mu2, mu) and np.array_equal(Y2, Y)

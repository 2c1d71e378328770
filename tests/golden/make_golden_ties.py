#!/opt/conda/bin/python3.9
"""Golden vectors for subset bases with tied |eigenvalues|: run the
reference's own ``stationscreen.run`` (through ``make_golden.run_fit``: the
same interpreter, shims and duck-typed soltab) on small direction counts with
heavy flagging, so that many slots keep exactly two unflagged directions.

Every 2-direction subset of the zero-diagonal C is [[0, b], [b, 0]], whose
singular values are |b| twice: ``scipy.linalg.svd`` (LAPACK gesdd) then
returns U = [[0, 1], [1, 0]] (b < 0) -- unit vectors, not eigenvectors of C --
and the order-1 fit (``_fit_screen``, stationscreen.py:490-534, the order
clipped to n_unflagged - 1 = 1 at :685-686) keeps its first column.  These
sets pin what the reference does there.

Usage:  /opt/conda/bin/python3.9 tests/golden/make_golden_ties.py [amp]
(``amp``: only the amplitude set -- run it under ``timeout``: a slot the
block flags leave with one unflagged direction kills the reference's worker
and the run hangs, see below)
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (shims + reference imports)


def amplitude_case(seed=424):
    """The amplitude fit as KLScreen.fit calls it (kl_screen.py:96-125: order
    min(12, max(3, round(D / 2))) = 3, niter 3, no order scaling, ref_ant -1)
    at D = 4 with 40 % of the weights zero: the block sigma (Q6) and the
    two-direction rule on log10 amplitudes, both pols."""
    from ska_sdp_screen_fitting_amd.synthetic import make_amplitudes
    s = mg.make_solutions(n_ant=6, n_time=6, n_freq=2, n_dir=4, seed=seed)
    make_amplitudes(s, seed=seed + 1, flag_frac=0.4, outlier_frac=0.0)
    w = s.meta["amp_weight"]
    for idx in np.argwhere((w > 0).sum(axis=-2) < 2):   # [t, f, a, pol]
        t, f, a, p = idx
        slot = w[t, f, a, :, p]
        for d in range(slot.size):
            if (slot > 0).sum() >= 2:
                break
            if slot[d] <= 0:
                slot[d] = 1.0
    sol = dict(val=s.val, weight=s.weight, times=s.times, freqs=s.freqs,
               dir_names=s.dir_names, ant_names=s.ant_names,
               dir_radec=s.dir_radec, ant_pos=s.ant_pos)

    class AmpSoltab(mg.DuckSoltab):
        name = "amplitude000"

        def __init__(self, sol, amp, wt):
            super().__init__(sol)
            self.val = np.array(amp, dtype=np.float64)
            self.weight = np.array(wt, dtype=np.float32)
            self.pol = np.array(["XX", "YY"])

        def get_type(self):
            return "amplitude"

        def get_axes_names(self):
            return ["time", "freq", "ant", "dir", "pol"]

    st = AmpSoltab(sol, s.amp_val, w)
    rc = mg.stationscreen.run(st, "amplitude_screen000", order=3, niter=3,
                              ref_ant=-1, scale_order=False, adjust_order=True,
                              ncpu=1)
    assert rc == 0
    ss = st.get_solset()
    scr, res = ss.made["amplitude_screen000"], ss.made["amplitude_screen000resid"]
    w_out = scr.weights.astype(np.float32)
    print("ties4amp slots x pols with 2 unflagged",
          int(((w_out > 0).sum(-2) == 2).sum()))
    np.savez_compressed(
        os.path.join(HERE, "ties4amp.npz"),
        amp_val=s.amp_val, amp_weight=w, dir_radec=s.dir_radec,
        amp_order=3, amp_coef=scr.vals, amp_w_out=w_out, amp_resid=res.vals,
        amp_orders=res.weights[..., 0, :].astype(np.int32),
        piercepoints=ss.obj._v_file.arrays["/sol000/amplitude_screen000/piercepoint"])


def main():
    if sys.argv[1:] == ["amp"]:
        amplitude_case()
        print("done")
        return
    cases = {
        # D = 4 / 6 with 40 % of the (slot, direction) weights zero: masks
        # with exactly two unflagged directions (the 2 x 2 tie), one (K = 0)
        # and none (skipped slots)
        "ties4": dict(n_ant=6, n_time=8, n_freq=2, n_dir=4, seed=404,
                      flag_frac=0.4, outlier_frac=0.02),
        "ties6": dict(n_ant=6, n_time=8, n_freq=2, n_dir=6, seed=606,
                      flag_frac=0.4, outlier_frac=0.02),
    }
    for name, kw in cases.items():
        s = mg.make_solutions(**kw)
        # the reference cannot fit a slot with fewer than two unflagged
        # directions: order min(order, n - 1) = 0 gives pinv of a 0 x 0
        # matrix at stationscreen.py:504 (LAPACK gesdd error, the worker
        # dies); unflag the lowest flagged directions of such slots
        w = s.weight
        for idx in np.argwhere((w > 0).sum(axis=-1) < 2):
            slot = w[tuple(idx)]
            for d in range(slot.size):
                if (slot > 0).sum() >= 2:
                    break
                if slot[d] <= 0:
                    slot[d] = 1.0
        sol = dict(val=s.val, weight=s.weight, times=s.times, freqs=s.freqs,
                   dir_names=s.dir_names, ant_names=s.ant_names,
                   dir_radec=s.dir_radec, ant_pos=s.ant_pos)
        fit = mg.run_fit(sol)
        # slots whose 2-direction subset SVD (the reference's own scipy /
        # LAPACK, stationscreen.py:390-430) is not an exact permutation:
        # there the reference's screen at the first unflagged direction is
        # atan2 of LAPACK rounding residue (its value depends on the LAPACK
        # build), so the tests exclude those slots from value comparisons
        from scipy.linalg import svd
        pp = fit["piercepoints"]
        residue = np.zeros(sol["weight"].shape[:3], bool)
        for wts in (sol["weight"], fit["w_out"]):
            for idx in np.argwhere((wts > 0).sum(axis=-1) == 2):
                unfl = np.where(wts[tuple(idx)] > 0)[0]
                c, _, _ = mg.stationscreen._calculate_svd(pp[unfl], fit["r_0"],
                                                          fit["beta"], 2)
                u = svd(c)[0]
                if not np.all((u == 0.0) | (np.abs(u) == 1.0)):
                    residue[tuple(idx)] = True
        n_unfl = (sol["weight"] > 0).sum(axis=-1)
        print(name, "fit", fit["fit_seconds"], "s ref", fit["ref_ant"],
              "orders", np.unique(fit["orders"], return_counts=True),
              "slots with 2 unflagged", int((n_unfl == 2).sum()),
              "after the fit", int(((fit["w_out"] > 0).sum(-1) == 2).sum()),
              "with SVD residue", int(residue.sum()))
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            val=sol["val"], weight=sol["weight"], times=sol["times"],
            freqs=sol["freqs"], dir_names=np.array(sol["dir_names"]),
            ant_names=np.array(sol["ant_names"]), dir_radec=sol["dir_radec"],
            ant_pos=sol["ant_pos"], ref_ant=fit["ref_ant"],
            order=fit["order"], coef=fit["coef"], w_out=fit["w_out"],
            resid=fit["resid"], orders=fit["orders"],
            piercepoints=fit["piercepoints"], mid_ra=fit["mid_ra"],
            mid_dec=fit["mid_dec"], beta=fit["beta"], r_0=fit["r_0"],
            C=fit["C"], pinv_c=fit["pinv_c"], U=fit["U"], tie_residue=residue)
    # tec screens (stationscreen.py:549-562: no atan2; the screen is C times
    # the fit): the same two-direction rule, niter 3 (the block sigma of Q6)
    s = mg.make_solutions(n_ant=6, n_time=8, n_freq=2, n_dir=4, seed=414,
                          flag_frac=0.4, outlier_frac=0.02)
    w = s.weight
    for idx in np.argwhere((w > 0).sum(axis=-1) < 2):
        slot = w[tuple(idx)]
        for d in range(slot.size):
            if (slot > 0).sum() >= 2:
                break
            if slot[d] <= 0:
                slot[d] = 1.0
    val = s.val * 0.05  # TECU-sized values
    sol = dict(val=val, weight=w, times=s.times, freqs=s.freqs,
               dir_names=s.dir_names, ant_names=s.ant_names,
               dir_radec=s.dir_radec, ant_pos=s.ant_pos)

    class TecSoltab(mg.DuckSoltab):
        name = "tec000"

        def get_type(self):
            return "tec"

    st = TecSoltab(sol)
    ref = mg.reference_station(st.weight, 10)
    rc = mg.stationscreen.run(st, "tec_screen000", order=3, niter=3, ref_ant=ref,
                              scale_order=True, adjust_order=True, ncpu=1)
    assert rc == 0
    ss = st.get_solset()
    scr, res = ss.made["tec_screen000"], ss.made["tec_screen000resid"]
    w_out = scr.weights.astype(np.float32)
    print("ties4tec ref", ref, "slots with 2 unflagged",
          int(((w_out > 0).sum(-1) == 2).sum()))
    np.savez_compressed(
        os.path.join(HERE, "ties4tec.npz"),
        val=val, weight=w, times=s.times, freqs=s.freqs,
        dir_names=np.array(s.dir_names), ant_names=np.array(s.ant_names),
        dir_radec=s.dir_radec, ant_pos=s.ant_pos, ref_ant=ref, order=3, niter=3,
        coef=scr.vals, w_out=w_out, resid=res.vals,
        orders=res.weights[..., 0].astype(np.int32),
        piercepoints=ss.obj._v_file.arrays["/sol000/tec_screen000/piercepoint"])
    print("done")


if __name__ == "__main__":
    main()

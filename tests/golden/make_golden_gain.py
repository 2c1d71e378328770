#!/opt/conda/bin/python3.9
"""Golden vectors for the amplitude / "gain" KL path, produced by running the
reference itself (same interpreter, shims and duck-typed soltabs as
make_golden.py):

* stationscreen.run on an amplitude soltab [time, freq, ant, dir, pol]
  exactly as KLScreen.fit calls it (kl_screen.py:96-125): order
  min(12, max(3, round(D/2))), niter=3, scale_order=False, adjust_order=True,
  ref_ant=-1 -- this exercises the station-block-coupled outlier sigma (Q6);
* Screen.interpolate (screen.py:108-154) of the amplitude screen onto the
  phase time / frequency grid;
* KLScreen.make_matrix with amplitudes (kl_screen.py:319-378).

Usage:  /opt/conda/bin/python3.9 tests/golden/make_golden_gain.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (applies the shims)

import numpy as np  # noqa: E402

from ska_sdp_screen_fitting import stationscreen  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import (make_amplitudes,  # noqa: E402
                                                  make_solutions)


class AmpSoltab(mg.DuckSoltab):
    name = "amplitude000"

    def __init__(self, sol, amp, w, times, freqs):
        super().__init__(sol)
        self.val = np.array(amp, dtype=np.float64)
        self.weight = np.array(w, dtype=np.float32)
        self.time = np.array(times)
        self.freq = np.array(freqs)
        self.pol = np.array(["XX", "YY"])

    def get_type(self):
        return "amplitude"

    def get_axes_names(self):
        return ["time", "freq", "ant", "dir", "pol"]


def main():
    s = make_solutions(n_ant=5, n_time=8, n_freq=3, n_dir=12, seed=33,
                       flag_frac=0.02, outlier_frac=0.01)
    make_amplitudes(s, n_time=4, n_freq=2, seed=34, flag_frac=0.03,
                    outlier_frac=0.02)
    sol = dict(val=s.val, weight=s.weight, times=s.times, freqs=s.freqs,
               dir_names=s.dir_names, ant_names=s.ant_names,
               dir_radec=s.dir_radec, ant_pos=s.ant_pos)
    fit = mg.run_fit(sol)
    D = len(s.dir_names)
    amp_order = min(12, max(3, int(np.round(D / 2))))
    st = AmpSoltab(sol, s.amp_val, s.meta["amp_weight"], s.meta["amp_times"],
                   s.meta["amp_freqs"])
    rc = stationscreen.run(st, "amplitude_screen000", order=amp_order, niter=3,
                           scale_order=False, adjust_order=True, ncpu=1)
    assert rc == 0
    ss = st.get_solset()
    ascr = ss.made["amplitude_screen000"]
    ares = ss.made["amplitude_screen000resid"]
    print("amp fit: orders", np.unique(ares.weights, return_counts=True),
          "flags in", int((s.meta["amp_weight"] == 0).sum()), "out",
          int((ascr.weights == 0).sum()))

    rad, dec, width = 126.23, 64.50, 3.3300000000000054
    scr = mg.make_kl(sol, fit, 0.2, rad, dec, width)
    scr.phase_only = False
    scr.log_amps = True
    scr.vals_amp = ascr.vals
    scr.times_amp = np.array(s.meta["amp_times"])
    scr.freqs_amp = np.array(s.meta["amp_freqs"])
    scr.interpolate()
    pairs = [(0, 1), (2, 3), (1, 0)]
    data = []
    for f, a in pairs:
        data.append(scr.make_matrix(0, 8, f, a, 0.2, None, 1))
    np.savez_compressed(
        os.path.join(HERE, "gain12.npz"),
        val=s.val, weight=s.weight, times=s.times, freqs=s.freqs,
        dir_names=np.array(s.dir_names), ant_names=np.array(s.ant_names),
        dir_radec=s.dir_radec, ant_pos=s.ant_pos,
        ref_ant=fit["ref_ant"], order=fit["order"], coef=fit["coef"],
        piercepoints=fit["piercepoints"], mid_ra=fit["mid_ra"],
        mid_dec=fit["mid_dec"],
        amp_val=s.amp_val, amp_weight=s.meta["amp_weight"],
        amp_times=s.meta["amp_times"], amp_freqs=s.meta["amp_freqs"],
        amp_pol=np.array(["XX", "YY"]), amp_order=amp_order,
        amp_coef=ascr.vals, amp_w_out=ascr.weights.astype(np.float32),
        amp_resid=ares.vals, amp_orders=ares.weights[:, :, :, 0, :].astype(np.int32),
        amp_interp=np.array(scr.vals_amp), pairs=np.array(pairs),
        gain17=np.stack(data), x17=np.array(mg.kl_screen.X_COORD),
        y17=np.array(mg.kl_screen.Y_COORD))
    print("done")


if __name__ == "__main__":
    main()

#!/opt/conda/bin/python3.9
"""Golden vectors for tec screens, produced by running the reference's
stationscreen.run (same interpreter, shims and duck-typed soltabs as
make_golden.py) on a tec soltab:

* case "ref":   ref_ant = 2, scale_order=True  (referenced, ref station skipped)
* case "noref": ref_ant = -1 -- the operator-precedence quirk Q15
  (stationscreen.py:993-996) still references tec to the LAST station;

both with niter=3 so the station-block outlier sigma (quirk Q6) acts twice,
a few tiny (5e-4) weights (the pinv(G) branch), an all-NaN (freq, station)
block and flagged directions.

Usage:  /opt/conda/bin/python3.9 tests/golden/make_golden_tec.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (applies the shims)

import numpy as np  # noqa: E402

from ska_sdp_screen_fitting import stationscreen  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import make_solutions  # noqa: E402


class TecSoltab(mg.DuckSoltab):
    name = "tec000"

    def get_type(self):
        return "tec"


def main():
    s = make_solutions(n_ant=6, n_time=10, n_freq=2, n_dir=14, seed=41,
                       flag_frac=0.03, outlier_frac=0.02,
                       tiny_weight_frac=0.01)
    val = s.val * 0.05          # TECU-sized values
    val[:, 1, 3, :] = np.nan    # an all-NaN block
    sol = dict(val=val, weight=s.weight, times=s.times, freqs=s.freqs,
               dir_names=s.dir_names, ant_names=s.ant_names,
               dir_radec=s.dir_radec, ant_pos=s.ant_pos)
    out = dict(val=val, weight=s.weight, times=s.times, freqs=s.freqs,
               dir_names=np.array(s.dir_names), ant_names=np.array(s.ant_names),
               dir_radec=s.dir_radec, ant_pos=s.ant_pos, order=10, niter=3)
    for case, ref in (("ref", 2), ("noref", -1)):
        st = TecSoltab(sol)
        rc = stationscreen.run(st, "tec_screen000", order=10, niter=3,
                               ref_ant=ref, scale_order=True,
                               adjust_order=True, ncpu=1)
        assert rc == 0
        ss = st.get_solset()
        scr = ss.made["tec_screen000"]
        res = ss.made["tec_screen000resid"]
        out[f"{case}_ref_ant"] = ref
        out[f"{case}_coef"] = scr.vals
        out[f"{case}_w_out"] = scr.weights.astype(np.float32)
        out[f"{case}_resid"] = res.vals
        out[f"{case}_orders"] = res.weights[..., 0].astype(np.int32)
        out["piercepoints"] = ss.obj._v_file.arrays[
            "/sol000/tec_screen000/piercepoint"]
        print(case, "orders", np.unique(out[f"{case}_orders"], return_counts=True),
              "flags in", int((s.weight == 0).sum()), "out",
              int((out[f"{case}_w_out"] == 0).sum()))
    np.savez_compressed(os.path.join(HERE, "tec14.npz"), **out)
    print("done")


if __name__ == "__main__":
    main()

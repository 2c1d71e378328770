#!/opt/conda/bin/python3.9
"""Generate the golden vectors the oracle and the HIP path are pinned to.

Runs the *reference itself* (``/root/reference/src/ska_sdp_screen_fitting``)
under ``/opt/conda/bin/python3.9`` (numpy 1.26.4, scipy 1.7.1, astropy 4.3.1,
h5py 3.3.0) with the import shims recorded in SURVEY.md §8(c):

* numpy aliases removed in numpy >= 1.24 (``np.float`` is used at
  ``utils/processing_utils.py:570``; astropy 4.3.1 needs the others);
* import-only stubs for ``tables`` (PyTables is broken in that env),
  ``lsmtool`` and ``shapely``.  None of them is exercised on the KL path: the
  H5parm is read with h5py into a duck-typed soltab, and the reference's
  ``stationscreen.run`` / ``KLScreen.make_matrix`` / ``make_template_image``
  are then called unchanged.

This script is test infrastructure.  It needs ``/root/reference`` and the
conda interpreter, so it only runs in the build container; its outputs are the
committed ``tests/golden/*.npz`` / ``*.json`` fixtures (data, not source).

Usage:  /opt/conda/bin/python3.9 tests/golden/make_golden.py
"""

import json
import os
import sys
import time
import types
import warnings

warnings.filterwarnings("ignore")

import numpy as np  # noqa: E402

# --- shims (SURVEY.md §8(c) recipe step 1-3) --------------------------------
np.float = float
np.int = int
np.bool = bool
np.object = object
np.str = str
np.asscalar = lambda a: a.item()
np.alen = len

_tables = types.ModuleType("tables")
_tables.__version__ = "3.7.0"


class _Group:  # only referenced by isinstance() in code we do not call
    pass


_tables.Group = _Group
sys.modules["tables"] = _tables
sys.modules["lsmtool"] = types.ModuleType("lsmtool")
for _m in ("shapely", "shapely.geometry", "shapely.ops", "shapely.prepared"):
    sys.modules[_m] = types.ModuleType(_m)
sys.modules["shapely.geometry"].Point = object
sys.modules["shapely.geometry"].Polygon = object
sys.modules["shapely.prepared"].prep = lambda p: p

REF = "/root/reference"
sys.path.insert(0, REF + "/src")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))

import h5py  # noqa: E402
from astropy import wcs as awcs  # noqa: E402
from astropy.coordinates import Angle  # noqa: E402
from astropy.io import fits as pyfits  # noqa: E402

from ska_sdp_screen_fitting import kl_screen, stationscreen  # noqa: E402
from ska_sdp_screen_fitting.utils import processing_utils as misc  # noqa: E402

from ska_sdp_screen_fitting_amd.synthetic import make_solutions  # noqa: E402


# --- duck-typed H5parm soltab / solset (recipe step 4) ----------------------
class _Attrs(dict):
    pass


class _Obj:
    def __init__(self, name):
        self._v_attrs = _Attrs()
        self._v_name = name


class _OutSoltab:
    def __init__(self, soltype, name, axes_names, axes_vals, vals, weights):
        self.soltype = soltype
        self.name = name
        self.axes_names = axes_names
        self.vals = np.array(vals)
        self.weights = np.array(weights)
        self.obj = _Obj(name)

    def add_history(self, _):
        pass


class _File:
    def __init__(self):
        self.arrays = {}

    def create_array(self, where, name, obj=None):
        self.arrays[where + "/" + name] = np.array(obj)


class _SolsetObj:
    def __init__(self):
        self._v_file = _File()


class DuckSolset:
    name = "sol000"

    def __init__(self, sources, ants):
        self._sources = sources
        self._ants = ants
        self.obj = _SolsetObj()
        self.made = {}

    def get_source(self):
        return dict(self._sources)

    def get_ant(self):
        return dict(self._ants)

    def make_soltab(self, soltype, soltab_name=None, axes_names=None,
                    axes_vals=None, vals=None, weights=None, **_):
        st = _OutSoltab(soltype, soltab_name, axes_names, axes_vals, vals,
                        weights)
        self.made[soltab_name] = st
        return st


class DuckSoltab:
    name = "phase000"

    def __init__(self, sol):
        self.val = np.array(sol["val"], dtype=np.float64)
        self.weight = np.array(sol["weight"], dtype=np.float32)
        self.time = np.array(sol["times"], dtype=np.float64)
        self.freq = np.array(sol["freqs"], dtype=np.float64)
        self.dir = np.array(sol["dir_names"]).astype(str)
        self.ant = np.array(sol["ant_names"]).astype(str)
        self._solset = DuckSolset(
            {n: np.array(p, dtype=np.float32)
             for n, p in zip(sol["dir_names"], sol["dir_radec"])},
            {n: np.array(p, dtype=np.float32)
             for n, p in zip(sol["ant_names"], sol["ant_pos"])})

    def get_type(self):
        return "phase"

    def get_axes_names(self):
        return ["time", "freq", "ant", "dir"]

    def get_solset(self):
        return self._solset


def reference_station(weight, max_ind=10):
    """utils/processing_utils.py:538-574 on a [time,freq,ant,dir] weight."""
    w = np.sum(weight, axis=(0, 1, 3), dtype=np.float64)
    max_ind = min(max_ind, w.shape[0])
    return int(np.where(w[:max_ind] == np.max(w[:max_ind]))[0][0])


def run_fit(sol):
    """Call the reference operator exactly as KLScreen.fit does
    (kl_screen.py:95-112)."""
    st = DuckSoltab(sol)
    ref = reference_station(st.weight, 10)
    order = min(20, len(sol["dir_names"]) - 1)
    t0 = time.time()
    rc = stationscreen.run(st, "phase_screen000", order=order, ref_ant=ref,
                           scale_order=True, adjust_order=True, ncpu=1)
    dt = time.time() - t0
    assert rc == 0
    ss = st.get_solset()
    scr = ss.made["phase_screen000"]
    res = ss.made["phase_screen000resid"]
    out = dict(
        ref_ant=ref, order=order, fit_seconds=dt,
        coef=scr.vals, w_out=scr.weights.astype(np.float32),
        resid=res.vals, orders=res.weights[..., 0].astype(np.int32),
        piercepoints=ss.obj._v_file.arrays[
            "/sol000/phase_screen000/piercepoint"],
        mid_ra=float(scr.obj._v_attrs["midra"]),
        mid_dec=float(scr.obj._v_attrs["middec"]),
        beta=float(scr.obj._v_attrs["beta"]),
        r_0=float(scr.obj._v_attrs["r_0"]),
    )
    c, pinv_c, u = stationscreen._calculate_svd(
        out["piercepoints"], out["r_0"], out["beta"], len(sol["dir_names"]))
    out.update(C=c, pinv_c=pinv_c, U=u)
    return out


def make_kl(sol, fit, cellsize, rad, dec, width):
    scr = kl_screen.KLScreen("kl", "unused.h5", "unused.txt", rad, dec,
                             width, width)
    scr.vals_ph = fit["coef"]
    scr.times_ph = np.array(sol["times"])
    scr.freqs_ph = np.array(sol["freqs"])
    scr.source_names = np.array(sol["dir_names"]).astype(str)
    scr.station_names = np.array(sol["ant_names"]).astype(str)
    scr.piercepoints = fit["piercepoints"]
    scr.mid_ra = fit["mid_ra"]
    scr.mid_dec = fit["mid_dec"]
    scr.beta_val = fit["beta"]
    scr.r_0 = fit["r_0"]
    scr.height = 0.0
    scr.ncpu = 1
    return scr


def eval_slots(scr, pairs, t0, t1, cellsize):
    """KLScreen.make_matrix (kl_screen.py:192-380) for (freq, station) pairs.
    Returns planes 0 (cos) and 1 (sin) in float64 plus the X/Y coords."""
    outs = []
    for f, s in pairs:
        data = scr.make_matrix(t0, t1, f, s, cellsize, None, 1)
        outs.append(data[:, 0:2])
        assert np.array_equal(data[:, 0], data[:, 2])
        assert np.array_equal(data[:, 1], data[:, 3])
    return (np.stack(outs), np.array(kl_screen.X_COORD),
            np.array(kl_screen.Y_COORD))


def patch_positions(skymodel):
    """Patch RA/Dec (deg) from the skymodel's patch lines, parsed like
    lsmtool (RA hh:mm:ss, Dec dd.mm.ss)."""
    pos = {}
    for line in open(skymodel):
        parts = [p.strip() for p in line.split(",")]
        if len(parts) == 5 and parts[0] == "" and parts[1] == "":
            ra = Angle(parts[3], unit="hourangle").deg
            d = parts[4].split(".")
            dec = Angle(":".join(d[:3]) + ("." + d[3] if len(d) > 3 else ""),
                        unit="deg").deg
            pos[parts[2]] = (ra, dec)
    return pos


def header_cards(path):
    h = pyfits.getheader(path)
    return [(k, h[k]) for k in h.keys()]


def main():
    rng_pairs = None
    out_dir = HERE
    res_dir = REF + "/resources"
    tmp = "/tmp/sf_golden"
    os.makedirs(tmp, exist_ok=True)

    # ---------------- fixture (configs 1-2) ----------------
    f = h5py.File(res_dir + "/solutions.h5", "r")
    fx = dict(
        val=f["sol000/phase000/val"][:],
        weight=f["sol000/phase000/weight"][:],
        times=f["sol000/phase000/time"][:],
        freqs=f["sol000/phase000/freq"][:],
        dir_names=[x.decode() for x in f["sol000/phase000/dir"][:]],
        ant_names=[x.decode() for x in f["sol000/phase000/ant"][:]],
    )
    src = {r["name"].decode(): r["dir"] for r in f["sol000/source"][:]}
    ants = {r["name"].decode(): r["position"] for r in f["sol000/antenna"][:]}
    fx["dir_radec"] = np.array([src[n] for n in fx["dir_names"]], np.float32)
    fx["ant_pos"] = np.array([ants[n] for n in fx["ant_names"]], np.float32)
    f.close()

    fit = run_fit(fx)
    print("fixture fit", fit["fit_seconds"], "s  ref", fit["ref_ant"],
          "orders", np.unique(fit["orders"], return_counts=True))

    rad, dec = 126.23, 64.50
    bounds = [124.565, 66.165, 127.895, 62.835]
    # padding_fraction=0 arithmetic of make_aterm_images.py:88-97, then the
    # Dec extent (:116-118)
    pad_ra = (bounds[2] - bounds[0]) * (0.0 - 1.0)
    pad_dec = (bounds[3] - bounds[1]) * (0.0 - 1.0)
    bounds = [bounds[0] - pad_ra, bounds[1] - pad_dec, bounds[2] + pad_ra,
              bounds[3] + pad_dec]
    width = bounds[3] - bounds[1]
    print("width", repr(width))
    scr = make_kl(fx, fit, 0.2, rad, dec, width)
    pairs17 = [(0, 0), (0, 1), (5, 30), (11, 61), (7, 13)]
    kl17, x17, y17 = eval_slots(scr, pairs17, 0, 20, 0.2)
    pairs128 = [(3, 7), (9, 44)]
    kl128, x128, y128 = eval_slots(scr, pairs128, 4, 6, 0.02602)
    coords = {}
    for n, cell in ((17, 0.2), (128, 0.02602), (256, 0.01301),
                    (512, 0.006505)):
        scr.make_matrix  # noqa: B018  (coords recomputed below)
        # the coordinate block of make_matrix (kl_screen.py:238-261)
        ximsize = int(np.ceil(scr.width_ra / cell))
        w = awcs.WCS(naxis=2)
        w.wcs.crpix = [ximsize / 2.0, ximsize / 2.0]
        w.wcs.cdelt = np.array([-cell, cell])
        w.wcs.crval = [rad, dec]
        w.wcs.ctype = ["RA---TAN", "DEC--TAN"]
        w.wcs.set_pv([(2, 1, 45.0)])
        ras, decs = [], []
        for i in range(ximsize):
            rd = w.wcs_pix2world(np.array([[i, i]]), 0)[0]
            ras.append(rd[0])
            decs.append(rd[1])
        xy, _, _ = stationscreen._getxy(ras, decs, mid_ra=fit["mid_ra"],
                                        mid_dec=fit["mid_dec"])
        coords[n] = (np.array(ras), np.array(decs), xy[0], xy[1])
        assert ximsize == n, (ximsize, n)
    assert np.array_equal(coords[17][2], x17)
    assert np.array_equal(coords[128][2], x128)

    # FITS template header + patch pixel coordinates via the cube's own WCS
    hdr = {}
    patch_pix = {}
    ppos = patch_positions(res_dir + "/skymodel.txt")
    radec_patch = np.array([ppos[n.strip("[]")] for n in fx["dir_names"]])
    for n, cell in ((17, 0.2), (128, 0.02602)):
        path = f"{tmp}/tmpl_{n}.fits"
        misc.make_template_image(path, rad, dec, ximsize=n, yimsize=n,
                                 cellsize_deg=cell, freqs=fx["freqs"],
                                 times=fx["times"][0:20],
                                 antennas=fx["ant_names"], aterm_type="gain")
        hdr[n] = [(k, v if not isinstance(v, bool) else int(v))
                  for k, v in header_cards(path)]
        wobj = awcs.WCS(pyfits.getheader(path))
        px, py = misc.get_patch_coordinates(radec_patch, wobj)
        patch_pix[n] = np.array([px, py])

    np.savez_compressed(
        os.path.join(out_dir, "fixture_kl.npz"),
        val=fx["val"], weight=fx["weight"], times=fx["times"],
        freqs=fx["freqs"], dir_names=np.array(fx["dir_names"]),
        ant_names=np.array(fx["ant_names"]), dir_radec=fx["dir_radec"],
        ant_pos=fx["ant_pos"],
        ref_ant=fit["ref_ant"], order=fit["order"], coef=fit["coef"],
        w_out=fit["w_out"], resid=fit["resid"], orders=fit["orders"],
        piercepoints=fit["piercepoints"], mid_ra=fit["mid_ra"],
        mid_dec=fit["mid_dec"], beta=fit["beta"], r_0=fit["r_0"],
        C=fit["C"], pinv_c=fit["pinv_c"], U=fit["U"],
        pairs17=np.array(pairs17), kl17=kl17, x17=x17, y17=y17,
        pairs128=np.array(pairs128), kl128_t=np.array([4, 6]), kl128=kl128,
        x128=x128, y128=y128,
        **{f"coords{n}_{k}": v for n, c in coords.items()
           for k, v in zip(("ra", "dec", "x", "y"), c)},
        radec_patch=radec_patch, patch_pix17=patch_pix[17],
        patch_pix128=patch_pix[128],
        fit_seconds=fit["fit_seconds"])
    with open(os.path.join(out_dir, "fixture_headers.json"), "w") as fh:
        json.dump({str(k): v for k, v in hdr.items()}, fh, indent=0)

    # ---------------- synthetic (flags, outliers, tiny weights) -------------
    cases = {
        # D=20: flagged directions, outliers, order adaptation (config-3 shape)
        "synth20": dict(n_ant=6, n_time=6, n_freq=2, n_dir=20, seed=20260,
                        flag_frac=0.03, outlier_frac=0.02),
        # D=12 with weights below the pinv cutoff (stationscreen.py:504)
        "synth12tiny": dict(n_ant=5, n_time=5, n_freq=2, n_dir=12, seed=7,
                            flag_frac=0.05, outlier_frac=0.02,
                            tiny_weight_frac=0.08),
        # D=50 (config-5 direction count), few slots
        "synth50": dict(n_ant=3, n_time=3, n_freq=1, n_dir=50, seed=11,
                        flag_frac=0.01, outlier_frac=0.005),
    }
    for name, kw in cases.items():
        s = make_solutions(**kw)
        sol = dict(val=s.val, weight=s.weight, times=s.times, freqs=s.freqs,
                   dir_names=s.dir_names, ant_names=s.ant_names,
                   dir_radec=s.dir_radec, ant_pos=s.ant_pos)
        if name == "synth20":
            # a fully flagged (station, freq) block and an all-NaN one:
            # both are skipped (stationscreen.py:821-825)
            sol["weight"][:, 1, 3, :] = 0.0
            ref = reference_station(sol["weight"], 10)
            nan_st = [a for a in range(kw["n_ant"]) if a not in (ref, 3)][0]
            sol["val"][:, 0, nan_st, :] = np.nan
        fit = run_fit(sol)
        print(name, "fit", fit["fit_seconds"], "s ref", fit["ref_ant"],
              "orders", np.unique(fit["orders"], return_counts=True))
        scr = make_kl(sol, fit, 0.2, rad, dec, width)
        nf = kw["n_freq"]
        pairs = [(0, 1), (1 % nf, 2), (0, fit["ref_ant"])]
        kl, xs, ys = eval_slots(scr, pairs, 0, kw["n_time"], 0.2)
        np.savez_compressed(
            os.path.join(out_dir, f"{name}.npz"),
            val=sol["val"], weight=sol["weight"], times=sol["times"],
            freqs=sol["freqs"], dir_names=np.array(sol["dir_names"]),
            ant_names=np.array(sol["ant_names"]), dir_radec=sol["dir_radec"],
            ant_pos=sol["ant_pos"], ref_ant=fit["ref_ant"],
            order=fit["order"], coef=fit["coef"], w_out=fit["w_out"],
            resid=fit["resid"], orders=fit["orders"],
            piercepoints=fit["piercepoints"], mid_ra=fit["mid_ra"],
            mid_dec=fit["mid_dec"], beta=fit["beta"], r_0=fit["r_0"],
            C=fit["C"], pinv_c=fit["pinv_c"], U=fit["U"],
            pairs17=np.array(pairs), kl17=kl, x17=xs, y17=ys)
    print("done")


if __name__ == "__main__":
    main()

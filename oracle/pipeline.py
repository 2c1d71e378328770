"""CPU path of ``make_aterm_image`` built from the oracle -- TEST
INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` legs; see oracle/__init__.py).

The reference's own CPU path for BASELINE.json configs 1 and 2, restated
end to end on one core:

* config 1, tessellated (``make_aterm_images.py:120-146`` ->
  ``VoronoiScreen.process`` / ``write``): phases referenced to the reference
  station (voronoi_screen.py:57-102), the label raster
  (voronoi_screen.py:218-351, ``oracle.voronoi.label_raster``), the gather of
  every (time, freq, station) slot (voronoi_screen.py:132-216), the
  per-slot ``gaussian_filter`` (screen.py:353-362) and the FITS cube
  (screen.py:331-382);
* config 2, KL (``KLScreen.fit`` -> ``stationscreen.run`` ->
  ``calculate_kl_screen``): reference station, piercepoints, station orders
  and the fit of every slot (``oracle.kl.run_phase``,
  stationscreen.py:858-1161), the pixel basis (kl_screen.py:411-449), the
  cos / sin planes and the FITS cube.

The FITS file is written in the reference's layout (one primary HDU,
BITPIX -32, big-endian float32, axes [RA, DEC, MATRIX, ANTENNA, FREQ, TIME])
one time row at a time, as ``Screen.write`` streams it.  Only the cards
needed to make the file a valid FITS image are written: the header text is
pinned separately (tests/golden/fixture_headers.json vs the product's
writer); this module exists to time the CPU path, not to check it.

Run as ``python -m oracle.pipeline {config1,config2} OUTDIR`` (bench.py
starts it as a child process pinned to one CPU with single-threaded BLAS)
and it prints one JSON line.
"""

import json
import os
import sys
import time

import numpy as np

from . import geometry as og
from . import kl as okl
from . import voronoi as ov

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(REPO, "tests", "golden", "fixture_kl.npz")
SKYMODEL = os.path.join(REPO, "tests", "golden", "skymodel.txt")
# make_aterm_image(bounds_deg=[124.565, 66.165, 127.895, 62.835],
# bounds_mid_deg=[126.23, 64.50], padding_fraction=0): the reference test's
# field (tests/test_fit_screens.py)
FIELD_RAD, FIELD_DEC = 126.23, 64.50
FIELD_WIDTH = 66.165 - 62.835
BLOCK = 2880


def _card(key, value):
    if isinstance(value, bool):
        v = "T" if value else "F"
    elif isinstance(value, int):
        v = str(value)
    else:
        v = repr(float(value)).upper()
    return f"{key:<8}= {v:>20}".ljust(80).encode("ascii")


class FitsCube:
    """Primary-HDU float32 cube written row by row (big-endian)."""

    def __init__(self, path, shape):
        self.fh = open(path, "wb")
        cards = [_card("SIMPLE", True), _card("BITPIX", -32),
                 _card("NAXIS", len(shape))]
        cards += [_card(f"NAXIS{k + 1}", int(n)) for k, n in enumerate(shape[::-1])]
        cards.append(b"END".ljust(80))
        hdr = b"".join(cards)
        self.fh.write(hdr + b" " * ((-len(hdr)) % BLOCK))
        self.nbytes = 0

    def write(self, block):
        b = np.ascontiguousarray(block, dtype=">f4").tobytes()
        self.fh.write(b)
        self.nbytes += len(b)

    def close(self):
        self.fh.write(b"\0" * ((-self.nbytes) % BLOCK))
        self.fh.close()


def _scrub(planes):
    """NaN -> 1 (real) / 0 (imaginary) planes (screen.py:364-378)."""
    for p in range(4):
        v = planes[..., p, :, :]
        v[np.isnan(v)] = 0.0 if p % 2 else 1.0
    return planes


def _fixture():
    return np.load(FIXTURE)


def tessellated_path(outdir, cellsize_deg=0.2, smooth_deg=0.1, keep=False):
    """Config 1: make_aterm_image(screen_type="tessellated") on the fixture."""
    t0 = time.perf_counter()
    g = _fixture()
    val = np.asarray(g["val"], np.float64)
    ref = okl.reference_station(g["weight"])
    ph = val - val[:, :, ref:ref + 1, :]                      # :57-102
    pos = ov.patch_positions(SKYMODEL)
    radec = np.array([pos[str(d).strip("[]")] for d in g["dir_names"]])
    lab, _ = ov.label_raster(radec[:, 0], radec[:, 1], FIELD_RAD, FIELD_DEC,
                             FIELD_WIDTH, cellsize_deg)
    n = lab.shape[0]
    smooth_pix = smooth_deg / cellsize_deg
    T, F, A, _ = ph.shape
    path = os.path.join(outdir, "cpu_tessellated_0.fits")
    cube = FitsCube(path, (T, F, A, 4, n, n))
    for t in range(T):
        planes = ov.gather_planes(lab, ph[t])                 # [F, A, 4, n, n]
        if smooth_pix > 0:
            planes = ov.smooth(planes, smooth_pix)
        cube.write(_scrub(planes))
    cube.close()
    wall = time.perf_counter() - t0
    size = os.path.getsize(path)
    if not keep:
        os.remove(path)
    return {"case": "config1", "screen_type": "tessellated", "grid": n,
            "smooth_pix": smooth_pix, "slots": T * F * A, "wall_s": wall,
            "fits_bytes": size}


def kl_path(outdir, cellsize_deg=0.02602, order=None):
    """Config 2: make_aterm_image(screen_type="kl") on the fixture."""
    t0 = time.perf_counter()
    g = _fixture()
    val = np.asarray(g["val"], np.float64)
    weight = np.asarray(g["weight"], np.float32)
    T, F, A, D = val.shape
    if order is None:
        order = min(20, D - 1)                               # kl_screen.py:81
    ref = okl.reference_station(weight)
    pp, mid_ra, mid_dec = og.piercepoints(g["dir_radec"])
    fit = okl.run_phase(val, weight, g["ant_pos"], pp, ref, order)
    t_fit = time.perf_counter() - t0
    x, y = og.grid_coords(FIELD_RAD, FIELD_DEC, FIELD_WIDTH, cellsize_deg,
                          mid_ra, mid_dec)
    cpix = okl.cpix_matrix(pp, x, y)
    ny, nx = len(y), len(x)
    path = os.path.join(outdir, "cpu_kl_0.fits")
    cube = FitsCube(path, (T, F, A, 4, ny, nx))
    for t in range(T):
        coef = fit["coef"][t].reshape(F * A, D)
        planes = okl.eval_planes(okl.eval_phase_screens(coef, cpix))
        cube.write(_scrub(planes.reshape(F, A, 4, ny, nx)))
    cube.close()
    wall = time.perf_counter() - t0
    size = os.path.getsize(path)
    os.remove(path)
    return {"case": "config2", "screen_type": "kl", "grid": nx, "slots": T * F * A,
            "wall_s": wall, "fit_s": t_fit, "fits_bytes": size}


def main():
    case, outdir = sys.argv[1], sys.argv[2]
    pin = os.environ.get("SF_PIN_CPU")
    if pin is not None and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {int(pin)})
    fn = {"config1": tessellated_path, "config2": kl_path}[case]
    r = fn(outdir)
    r["threads"] = {k: os.environ.get(k) for k in
                    ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    try:
        r["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        r["affinity_cpus"] = None
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""FITS-cube wall-clock of make_aterm_image (the second half of the
BASELINE.json metric) on the reference fixture:

  config 1: tessellated, 0.2 deg cells (17^2), smooth 0.1 deg
  config 2: KL, 128^2 grid (cellsize 0.02602)
  (optional) KL 256^2 on the fixture

Prints one JSON line per case: wall-clock of make_aterm_image (fit + eval +
FITS write, host I/O included) and the cube size.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))

from ska_sdp_screen_fitting_amd.make_aterm_images import make_aterm_image  # noqa: E402

FIX = os.path.join(REPO, "tests", "golden", "fixture_kl.npz")
SKY = os.path.join(REPO, "tests", "golden", "skymodel.txt")
CASES = {
    "config1": ("tessellated", 0.2, 0.1),
    "config2": ("kl", 0.02602, 0.0),
    "kl256": ("kl", 0.01301, 0.0),
}


def run(name, outdir):
    st, cell, smooth = CASES[name]
    outroot = os.path.join(outdir, name)
    t0 = time.perf_counter()
    make_aterm_image(FIX, soltabname="phase000", screen_type=st, outroot=outroot,
                     bounds_deg=[124.565, 66.165, 127.895, 62.835],
                     bounds_mid_deg=[126.23, 64.50], skymodel=SKY,
                     padding_fraction=0, cellsize_deg=cell, smooth_deg=smooth,
                     ncpu=0)
    dt = time.perf_counter() - t0
    size = sum(os.path.getsize(os.path.join(outdir, f)) for f in os.listdir(outdir)
               if f.startswith(name) and f.endswith(".fits"))
    return {"case": name, "screen_type": st, "cellsize_deg": cell,
            "wall_s": dt, "fits_bytes": size, "slots": 14880,
            "slots_per_s": 14880 / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["config1", "config2"])
    ap.add_argument("--outdir", default=None)
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    for name in a.cases:
        for k in range(a.repeat):
            with tempfile.TemporaryDirectory(dir=a.outdir) as d:
                r = run(name, d)
            r["repeat"] = k
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

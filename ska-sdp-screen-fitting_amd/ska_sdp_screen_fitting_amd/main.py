"""Command-line entry point, mirroring ``ska-sdp-screen-fitting`` (main.py:13-78)."""

import argparse

from .make_aterm_images import make_aterm_image


def start(argv=None):
    p = argparse.ArgumentParser(description="Make a-term images from solutions")
    p.add_argument("h5parmfile", help="Filename of input H5parm (or converted .npz)")
    p.add_argument("--soltabname", default="phase000")
    p.add_argument("--screen_type", default="tessellated")
    p.add_argument("--outroot", default="")
    p.add_argument("--bounds_deg", default=None)
    p.add_argument("--bounds_mid_deg", default=None)
    p.add_argument("--skymodel", default=None)
    p.add_argument("--solsetname", default="sol000")
    p.add_argument("--padding_fraction", default=1.4, type=float)
    p.add_argument("--cellsize_deg", default=0.2, type=float)
    p.add_argument("--smooth_deg", default=0, type=float)
    p.add_argument("--ncpu", default=0, type=int)
    a = p.parse_args(argv)
    make_aterm_image(a.h5parmfile, soltabname=a.soltabname,
                     screen_type=a.screen_type, outroot=a.outroot,
                     bounds_deg=a.bounds_deg, bounds_mid_deg=a.bounds_mid_deg,
                     skymodel=a.skymodel, solsetname=a.solsetname,
                     padding_fraction=a.padding_fraction,
                     cellsize_deg=a.cellsize_deg, smooth_deg=a.smooth_deg,
                     ncpu=a.ncpu)


if __name__ == "__main__":
    start()

"""``make_aterm_image`` -- the drop-in entry point (make_aterm_images.py:15-153
of the reference), same signature and side effects, GPU-backed KL and
tessellated paths."""

import os

from .h5parm import H5parm
from .kl_screen import KLScreen
from .voronoi_screen import VoronoiScreen


def make_aterm_image(h5parmfile, soltabname="phase000", screen_type="tessellated",
                     outroot="", bounds_deg=None, bounds_mid_deg=None,
                     skymodel=None, solsetname="sol000", padding_fraction=1.4,
                     cellsize_deg=0.2, smooth_deg=0, ncpu=0):
    """Make a-term FITS images.  Returns None (as the reference does)."""
    if "gain" in soltabname:
        soltab_amp = soltabname.replace("gain", "amplitude")
        soltab_ph = soltabname.replace("gain", "phase")
    else:
        soltab_amp = None
        soltab_ph = soltabname

    if isinstance(bounds_deg, str):
        bounds_deg = [float(f.strip()) for f in bounds_deg.strip("[]").split(";")]
    if isinstance(bounds_mid_deg, str):
        bounds_mid_deg = [float(f.strip()) for f in bounds_mid_deg.strip("[]").split(";")]
    bounds_deg = list(bounds_deg)  # the reference pads the caller's list in place
    if padding_fraction is not None:
        padding_fraction = float(padding_fraction)
        padding_ra = (bounds_deg[2] - bounds_deg[0]) * (padding_fraction - 1.0)
        padding_dec = (bounds_deg[3] - bounds_deg[1]) * (padding_fraction - 1.0)
        bounds_deg[0] -= padding_ra
        bounds_deg[1] -= padding_dec
        bounds_deg[2] += padding_ra
        bounds_deg[3] += padding_dec
    cellsize_deg = float(cellsize_deg)
    smooth_deg = float(smooth_deg)
    smooth_pix = smooth_deg / cellsize_deg
    if screen_type == "kl":
        smooth_pix = 0.0

    # one direction forces the tessellated screen (Q14)
    h5 = H5parm(h5parmfile)
    soltab = h5.get_solset(solsetname).get_soltab(soltab_ph)
    if len(soltab.dir) == 1:
        screen_type = "tessellated"
    h5.close()

    width_deg = bounds_deg[3] - bounds_deg[1]
    rootname = os.path.basename(outroot)
    if screen_type == "kl":
        screen = KLScreen(rootname, h5parmfile, skymodel, bounds_mid_deg[0],
                          bounds_mid_deg[1], width_deg, width_deg,
                          solset_name=solsetname, phase_soltab_name=soltab_ph,
                          amplitude_soltab_name=soltab_amp)
    elif screen_type == "tessellated":
        screen = VoronoiScreen(rootname, h5parmfile, skymodel, bounds_mid_deg[0],
                               bounds_mid_deg[1], width_deg, width_deg,
                               solset_name=solsetname, phase_soltab_name=soltab_ph,
                               amplitude_soltab_name=soltab_amp)
    else:
        raise ValueError(f"unknown screen_type {screen_type!r}")
    screen.process(ncpu=ncpu)
    outdir = os.path.dirname(outroot)
    screen.write(outdir, cellsize_deg, smooth_pix=smooth_pix, ncpu=ncpu)

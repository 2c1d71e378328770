"""Oracle restatement of the tessellated (Voronoi) screen -- TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows voronoi_screen.py:57-351 and utils/processing_utils.py:295-334 of the
reference:

* ``patch_positions``  <- lsmtool ``getPatchPositions`` on the patch lines of
  the sky model (RA "hh:mm:ss", Dec "dd.mm.ss");
* ``label_raster``     <- ``make_rasertize_template`` (:218-351): SIN pixel
  coordinates of the patches, field box, 64-point outer ring, scipy Voronoi,
  one polygon per direction, ``rasterize`` (Pillow polygon fill+outline, then
  the exact border test of the outline pixels), ``griddata(nearest)`` for
  uncovered pixels;
* ``gather_planes``    <- ``make_matrix`` (:132-216);
* ``smooth``           <- the per-(time, freq, station) ``gaussian_filter``
  of ``Screen.write`` (screen.py:353-362), through scipy.ndimage itself.

Third-party pieces: Pillow is the reference's own dependency (pinned 9.0.1;
Pillow 8.4.0 and 12.2.0 gave identical masks on the fixture, SURVEY §8(a)
a14).  shapely (pinned 1.8.0) is absent from every interpreter here, so its
two uses are restated: ``polygonize`` of the finite Voronoi ridges == the
bounded Voronoi regions of the direction points (the outer ring bounds them),
and ``disjoint(point)`` == "strictly outside the closed convex cell" (exact
orientation tests on float coordinates).  PARITY STATUS: the reference's
tessellated path cannot run in this image (needs shapely), so label rasters
are pinned only by the reference test criterion (patch pixels,
tests/test_fit_screens.py:43-128) and the survey's probe counts; interior
labels are otherwise unpinned.
"""

import numpy as np
import scipy.interpolate as si
from PIL import Image, ImageDraw
from scipy import ndimage
from scipy.spatial import Voronoi

from .geometry import sin_world2pix


def _sexagesimal(s, hours):
    s = s.strip()
    neg = s.startswith("-")
    parts = s.lstrip("+-").replace(":", ".").split(".")
    d, m = float(parts[0]), float(parts[1])
    sec = float(parts[2] + ("." + parts[3] if len(parts) > 3 else ""))
    v = d + m / 60.0 + sec / 3600.0
    v = -v if neg else v
    return v * 15.0 if hours else v


def patch_positions(skymodel):
    pos = {}
    for line in open(skymodel, encoding="utf8"):
        parts = [p.strip() for p in line.split(",")]
        if len(parts) == 5 and parts[0] == "" and parts[1] == "" and parts[2]:
            pos[parts[2]] = (_sexagesimal(parts[3], True),
                             _sexagesimal(parts[4], False))
    return pos


def _strictly_outside(poly, x, y):
    """shapely prepared.disjoint(Point) for a convex polygon ring."""
    n = len(poly)
    # orientation of the ring
    area = 0.0
    for k in range(n):
        x0, y0 = poly[k]
        x1, y1 = poly[(k + 1) % n]
        area += x0 * y1 - x1 * y0
    sgn = 1.0 if area > 0 else -1.0
    for k in range(n):
        x0, y0 = poly[k]
        x1, y1 = poly[(k + 1) % n]
        cr = (x1 - x0) * (y - y0) - (y1 - y0) * (x - x0)
        if cr * sgn < 0:
            return True
    return False


def rasterize(verts, shape):
    """utils/processing_utils.py:295-334 on an array of ones."""
    data = np.ones(shape)
    mask = Image.new("L", (shape[0], shape[1]), 0)
    ImageDraw.Draw(mask).polygon(verts, outline=1, fill=1)
    data *= np.array(mask)
    mask = Image.new("L", (shape[0], shape[1]), 0)
    ImageDraw.Draw(mask).polygon(verts, outline=1, fill=0)
    xs, ys = np.where(np.array(mask).transpose())
    ring = verts[:-1] if verts[0] == verts[-1] else verts
    for xm, ym in zip(xs, ys):
        if _strictly_outside(ring, float(xm), float(ym)):
            data[int(ym), int(xm)] = 0
    return data


def _cell(vor, k):
    reg = vor.regions[vor.point_region[k]]
    assert -1 not in reg and len(reg) >= 3
    v = vor.vertices[reg]
    c = v.mean(axis=0)
    order = np.argsort(np.arctan2(v[:, 1] - c[1], v[:, 0] - c[0]))
    ring = [tuple(map(float, p)) for p in v[order]]
    return ring + [ring[0]]


def label_raster(ra_deg, dec_deg, rad, dec, width, cellsize):
    """Label template (values 1..D), shape (ny, nx)."""
    n = int(np.ceil(width / cellsize))
    crval, crpix, cdelt = (rad, dec), (n / 2.0, n / 2.0), (-cellsize, cellsize)
    ra_deg = np.asarray(ra_deg, np.float64)
    dec_deg = np.asarray(dec_deg, np.float64)
    px, py = sin_world2pix(ra_deg, dec_deg, crval, crpix, cdelt)
    xy = np.stack([px, py], axis=1)
    b = [rad + width / 2.0, dec - width / 2.0, rad - width / 2.0, dec + width / 2.0]
    fmin = sin_world2pix(max(b[0], ra_deg.max() + 0.1), min(b[1], dec_deg.min() - 0.1),
                         crval, crpix, cdelt)
    fmax = sin_world2pix(min(b[2], ra_deg.min() - 0.1), max(b[3], dec_deg.max() + 0.1),
                         crval, crpix, cdelt)
    fmin = (float(fmin[0]), float(fmin[1]))
    fmax = (float(fmax[0]), float(fmax[1]))
    if len(xy) == 1:
        polys = [[fmin, (fmin[0], fmax[1]), fmax, (fmax[0], fmin[1]), fmin]]
    else:
        nouter = 64
        ang = np.array([np.pi / (nouter / 2.0) * i for i in range(nouter)])
        radius = 2.0 * np.sqrt((fmax[0] - fmin[0]) ** 2 + (fmax[1] - fmin[1]) ** 2)
        outer = xy.mean(axis=0) + radius * np.stack([np.cos(ang), np.sin(ang)], 1)
        vor = Voronoi(np.vstack([xy, outer]))
        polys = [_cell(vor, k) for k in range(len(xy))]
    tmpl = np.zeros((n, n))
    for k, verts in enumerate(polys):
        r = rasterize(verts, (n, n)) * (k + 1)
        filled = r > 0
        tmpl[filled] = r[filled]
    zero = np.where(tmpl == 0)
    if len(zero[0]) > 0:
        nz = np.where(tmpl != 0)
        tmpl[zero] = si.griddata((nz[0], nz[1]), tmpl[nz], (zero[0], zero[1]),
                                 method="nearest")
    return tmpl.astype(np.int32), xy


def gather_planes(label, phase, amp_xx=None, amp_yy=None):
    """voronoi_screen.py:177-214 for [..., D] values -> [..., 4, ny, nx]
    float32 (the cast the FITS store applies, screen.py:343)."""
    phase = np.asarray(phase, np.float64)
    if amp_xx is None:
        amp_xx = np.ones_like(phase)
    if amp_yy is None:
        amp_yy = amp_xx
    idx = label - 1
    c, s = np.cos(phase), np.sin(phase)
    planes = [amp_xx * c, amp_xx * s, amp_yy * c, amp_yy * s]
    return np.stack([p[..., idx] for p in planes], axis=-3).astype(np.float32)


def smooth(planes, smooth_pix):
    """screen.py:353-362: gaussian_filter(sigma=(0, s, s)) of each slot's
    float32 [4, ny, nx] block."""
    out = np.empty_like(planes)
    flat = planes.reshape(-1, *planes.shape[-3:])
    o = out.reshape(flat.shape)
    for k in range(flat.shape[0]):
        o[k] = ndimage.gaussian_filter(flat[k], sigma=(0, smooth_pix, smooth_pix),
                                       order=0)
    return out

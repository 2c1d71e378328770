"""Host-side geometry of the KL path (closed-form gnomonic / orthographic).

The reference obtains these from astropy.wcs (not available on the GPU box);
they are O(D + N) host computations that set up the device work:

* ``piercepoints``  <- stationscreen._calculate_piercepoints + _getxy +
  _radec2xy + _make_wcs (stationscreen.py:70-110, 138-231, 275-300): TAN
  projection with CRPIX 1000, CDELT -/+0.0005 deg about a data-chosen
  midpoint; float32 source directions converted to degrees in float32 (Q11);
* ``grid_coords``   <- the coordinate block of KLScreen.make_matrix
  (kl_screen.py:238-261): image TAN WCS (CRPIX N/2, CDELT -/+cell), pixel ->
  world for the diagonal pixels (i, i) only (Q8), then the piercepoint TAN;
* ``sin_world2pix`` <- the RA---SIN / DEC--SIN axes of the FITS cube
  (processing_utils.py:232-246), used to locate patch pixels.

Formulas are the standard closed forms (Calabretta & Greisen 2002) with the
native longitude of the celestial pole at 180 deg; PV2_1 has no effect on TAN.
"""

import numpy as np

_R2D = 180.0 / np.pi
_D2R = np.pi / 180.0


def tan_world2pix(ra, dec, crval, crpix, cdelt):
    """Gnomonic world -> pixel, 0-based pixel origin."""
    a = (np.asarray(ra, np.float64) - crval[0]) * _D2R
    d = np.asarray(dec, np.float64) * _D2R
    d0 = crval[1] * _D2R
    cosc = np.sin(d0) * np.sin(d) + np.cos(d0) * np.cos(d) * np.cos(a)
    x = np.cos(d) * np.sin(a) / cosc * _R2D
    y = (np.cos(d0) * np.sin(d) - np.sin(d0) * np.cos(d) * np.cos(a)) / cosc * _R2D
    return crpix[0] - 1.0 + x / cdelt[0], crpix[1] - 1.0 + y / cdelt[1]


def tan_pix2world(px, py, crval, crpix, cdelt):
    """Gnomonic pixel -> world, 0-based pixel origin; RA in [0, 360)."""
    x = (np.asarray(px, np.float64) + 1.0 - crpix[0]) * cdelt[0] * _D2R
    y = (np.asarray(py, np.float64) + 1.0 - crpix[1]) * cdelt[1] * _D2R
    d0 = crval[1] * _D2R
    den = np.cos(d0) - y * np.sin(d0)
    ra = crval[0] + np.arctan2(x, den) * _R2D
    dec = np.arctan2(np.sin(d0) + y * np.cos(d0), np.hypot(x, den)) * _R2D
    return np.mod(ra, 360.0), dec


def sin_world2pix(ra, dec, crval, crpix, cdelt):
    """Orthographic (SIN) world -> pixel, 0-based pixel origin."""
    a = (np.asarray(ra, np.float64) - crval[0]) * _D2R
    d = np.asarray(dec, np.float64) * _D2R
    d0 = crval[1] * _D2R
    x = np.cos(d) * np.sin(a) * _R2D
    y = (np.cos(d0) * np.sin(d) - np.sin(d0) * np.cos(d) * np.cos(a)) * _R2D
    return crpix[0] - 1.0 + x / cdelt[0], crpix[1] - 1.0 + y / cdelt[1]


_PP_CRPIX = (1000.0, 1000.0)
_PP_CDELT = (-0.0005, 0.0005)


def _pp_xy(ra_deg, dec_deg, ref_ra, ref_dec):
    return tan_world2pix(ra_deg, dec_deg, (float(ref_ra), float(ref_dec)),
                         _PP_CRPIX, _PP_CDELT)


def midpoint(ra_deg, dec_deg):
    """Data-chosen projection centre (stationscreen.py:158-180): the RA / Dec
    of the first source, in x- / y-sorted order, whose x / y exceeds the
    middle of the range."""
    if len(ra_deg) < 2:
        return ra_deg[0], dec_deg[0]
    x, y = _pp_xy(ra_deg, dec_deg, ra_deg[0], dec_deg[0])
    xmid = x.min() + (x.max() - x.min()) / 2.0
    ymid = y.min() + (y.max() - y.min()) / 2.0
    xs = np.argsort(x)
    ys = np.argsort(y)
    ix = np.nonzero(x[xs] > xmid)[0]
    iy = np.nonzero(y[ys] > ymid)[0]
    if ix.size == 0 or iy.size == 0:
        return ra_deg[0], dec_deg[0]
    return ra_deg[xs[ix[0]]], dec_deg[ys[iy[0]]]


def piercepoints(dir_radec):
    """[D, 3] piercepoints (x, y, 0) in 0.0005-deg TAN pixels plus the
    midpoint (mid_ra, mid_dec) in degrees."""
    src = np.asarray(dir_radec, dtype=np.float32)
    ra_deg = np.rad2deg(src[:, 0])   # float32 on purpose (Q11)
    dec_deg = np.rad2deg(src[:, 1])
    mid_ra, mid_dec = midpoint(ra_deg, dec_deg)
    x, y = _pp_xy(ra_deg, dec_deg, mid_ra, mid_dec)
    pp = np.zeros((src.shape[0], 3))
    pp[:, 0] = x
    pp[:, 1] = y
    return pp, float(mid_ra), float(mid_dec)


def grid_size(width_deg, cellsize_deg):
    """int(ceil(width / cell)) (kl_screen.py:238-239, screen.py:180-181)."""
    return int(np.ceil(width_deg / cellsize_deg))


def grid_coords(rad, dec, width_deg, cellsize_deg, mid_ra, mid_dec):
    """X_COORD, Y_COORD of kl_screen.py:238-259."""
    n = grid_size(width_deg, cellsize_deg)
    i = np.arange(n, dtype=np.float64)
    ra, de = tan_pix2world(i, i, (rad, dec), (n / 2.0, n / 2.0),
                           (-cellsize_deg, cellsize_deg))
    x, y = _pp_xy(ra, de, mid_ra, mid_dec)
    return np.asarray(x), np.asarray(y)

"""Oracle restatement of the host geometry on the KL path (test infrastructure).

Restates, in the wcslib formulation (celestial -> native spherical rotation,
then the zenithal projection), what the reference gets from astropy.wcs:

* ``_make_wcs``/``_radec2xy``/``_getxy``  (stationscreen.py:138-231, 275-300):
  TAN, CRPIX 1000, CDELT -/+0.0005 deg, origin-0 world->pixel;
* the image TAN WCS of ``KLScreen.make_matrix`` (kl_screen.py:238-259):
  CRPIX N/2, CDELT -/+cell, origin-0 pixel->world on the DIAGONAL pixels only
  (quirk Q8: pixel (i, j) is evaluated at (X[i], Y[j]));
* ``_calculate_piercepoints`` (stationscreen.py:70-110): float32 source
  directions, degrees computed in float32 (quirk Q11);
* the SIN WCS of the output FITS cube (processing_utils.py:232-246), used by
  the reference test to find the patch pixels (tests/test_fit_screens.py:75-81).

``PV2_1 = 45`` set by ``set_pv`` has no effect on TAN (TAN takes no
parameters); LONPOLE defaults to 180 deg for a zenithal projection whose
reference point is not the pole.
"""

import numpy as np

R2D = 180.0 / np.pi
D2R = np.pi / 180.0


def _cel2native(ra, dec, ra0, dec0, lonpole=180.0):
    """(ra, dec) -> native (phi, theta), degrees; wcslib sphs2x for a
    zenithal projection with the native pole at (ra0, dec0)."""
    da = (np.asarray(ra, np.float64) - ra0) * D2R
    d = np.asarray(dec, np.float64) * D2R
    d0 = dec0 * D2R
    x = np.sin(d) * np.cos(d0) - np.cos(d) * np.sin(d0) * np.cos(da)
    y = -np.cos(d) * np.sin(da)
    phi = lonpole + np.arctan2(y, x) * R2D
    theta = np.arcsin(np.clip(np.sin(d) * np.sin(d0)
                              + np.cos(d) * np.cos(d0) * np.cos(da), -1, 1))
    return phi, theta * R2D


def _native2cel(phi, theta, ra0, dec0, lonpole=180.0):
    """Inverse of _cel2native (wcslib sphx2s)."""
    dp = (np.asarray(phi, np.float64) - lonpole) * D2R
    t = np.asarray(theta, np.float64) * D2R
    d0 = dec0 * D2R
    x = np.sin(t) * np.cos(d0) - np.cos(t) * np.sin(d0) * np.cos(dp)
    y = -np.cos(t) * np.sin(dp)
    ra = ra0 + np.arctan2(y, x) * R2D
    dec = np.arcsin(np.clip(np.sin(t) * np.sin(d0)
                            + np.cos(t) * np.cos(d0) * np.cos(dp), -1, 1))
    return np.mod(ra, 360.0), dec * R2D


def tan_world2pix(ra, dec, crval, crpix, cdelt):
    """TAN world->pixel, origin 0 (astropy ``wcs_world2pix(.., 0)``)."""
    phi, theta = _cel2native(ra, dec, crval[0], crval[1])
    r = R2D / np.tan(theta * D2R)
    x = r * np.sin(phi * D2R)
    y = -r * np.cos(phi * D2R)
    return crpix[0] - 1.0 + x / cdelt[0], crpix[1] - 1.0 + y / cdelt[1]


def tan_pix2world(px, py, crval, crpix, cdelt):
    """TAN pixel->world, origin 0 (astropy ``wcs_pix2world(.., 0)``)."""
    x = (np.asarray(px, np.float64) + 1.0 - crpix[0]) * cdelt[0]
    y = (np.asarray(py, np.float64) + 1.0 - crpix[1]) * cdelt[1]
    r = np.hypot(x, y)
    phi = np.arctan2(x, -y) * R2D
    theta = np.arctan2(R2D, r) * R2D
    return _native2cel(phi, theta, crval[0], crval[1])


def sin_world2pix(ra, dec, crval, crpix, cdelt):
    """SIN (orthographic) world->pixel, origin 0: the FITS cube's RA---SIN /
    DEC--SIN axes (processing_utils.py:232-246)."""
    phi, theta = _cel2native(ra, dec, crval[0], crval[1])
    r = R2D * np.cos(theta * D2R)
    x = r * np.sin(phi * D2R)
    y = -r * np.cos(phi * D2R)
    return crpix[0] - 1.0 + x / cdelt[0], crpix[1] - 1.0 + y / cdelt[1]


_PP_CRPIX = (1000.0, 1000.0)
_PP_CDELT = (-0.0005, 0.0005)


def radec2xy(ra_list, dec_list, ref_ra=None, ref_dec=None):
    """stationscreen.py:189-231."""
    if ref_ra is None:
        ref_ra = ra_list[0]
    if ref_dec is None:
        ref_dec = dec_list[0]
    x, y = tan_world2pix(np.asarray(ra_list, np.float64),
                         np.asarray(dec_list, np.float64),
                         (float(ref_ra), float(ref_dec)), _PP_CRPIX, _PP_CDELT)
    return list(x), list(y)


def getxy(ra_list, dec_list, mid_ra=None, mid_dec=None):
    """stationscreen.py:138-186 (data-chosen midpoint when mid is None)."""
    if mid_ra is None or mid_dec is None:
        x, y = radec2xy(ra_list, dec_list)
        if len(x) > 1:
            xmid = min(x) + (max(x) - min(x)) / 2.0
            ymid = min(y) + (max(y) - min(y)) / 2.0
            xind = np.argsort(x)
            yind = np.argsort(y)
            try:
                midxind = np.where(np.array(x)[xind] > xmid)[0][0]
                midyind = np.where(np.array(y)[yind] > ymid)[0][0]
                mid_ra = ra_list[xind[midxind]]
                mid_dec = dec_list[yind[midyind]]
            except IndexError:
                mid_ra, mid_dec = ra_list[0], dec_list[0]
        else:
            mid_ra, mid_dec = ra_list[0], dec_list[0]
    x, y = radec2xy(ra_list, dec_list, mid_ra, mid_dec)
    return np.array([x, y]), mid_ra, mid_dec


def piercepoints(dir_radec):
    """stationscreen.py:70-110 + run :1050-1052: one (x, y, 0) row per
    direction (first station only), degrees computed in float32 (Q11)."""
    src = np.asarray(dir_radec, dtype=np.float32)
    ra_deg = np.rad2deg(src.T[0])
    dec_deg = np.rad2deg(src.T[1])
    xy, mid_ra, mid_dec = getxy(ra_deg, dec_deg)
    pp = np.zeros((src.shape[0], 3))
    pp[:, 0] = xy[0]
    pp[:, 1] = xy[1]
    return pp, float(mid_ra), float(mid_dec)


def grid_coords(rad, dec, width_deg, cellsize_deg, mid_ra, mid_dec):
    """kl_screen.py:238-261: X_COORD / Y_COORD from the diagonal pixels."""
    n = int(np.ceil(width_deg / cellsize_deg))
    idx = np.arange(n, dtype=np.float64)
    ra, de = tan_pix2world(idx, idx, (rad, dec), (n / 2.0, n / 2.0),
                           (-cellsize_deg, cellsize_deg))
    xy, _, _ = getxy(list(ra), list(de), mid_ra=mid_ra, mid_dec=mid_dec)
    return xy[0], xy[1]

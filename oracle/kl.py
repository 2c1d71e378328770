"""Oracle restatement of the KL fit and KL evaluation (test infrastructure).

Follows, function by function, the reference at ``/root/reference``
(src/ska_sdp_screen_fitting/...):

* ``calculate_svd``      <- stationscreen.py:390-430
* ``fit_screen``         <- stationscreen.py:433-594 (phase and tec)
* ``flag_outliers_slot`` <- stationscreen.py:303-350 restricted to one slot
* ``circ_chi2``          <- stationscreen.py:353-387
* ``fit_slot``           <- stationscreen.py:597-782 restricted to one slot
* ``run_phase``          <- stationscreen.py:858-1161 (+ 785-855)
* ``cpix_matrix`` / ``eval_phase_screens`` / ``eval_planes``
                         <- kl_screen.py:411-449 and :367-380

Why a per-slot restatement of ``_process_station`` is exact for phase/tec:
``_flag_outliers`` takes the circular std per time across directions
(``axis=0`` of a [dir, time] block), the order floor ``station_order`` is
``screen_order[0]`` and every time starts with the same order
(stationscreen.py:1040-1045), ``sign``/``hit_*`` reset per time, and
``prev_redchi2`` is only read at ``oindx > 0`` after being written at
``oindx - 1`` of the same time.  The weight aliasing quirk (Q2:
``_flag_outliers`` mutates and returns ``init_station_weights``, so the
"weights unchanged" test at :695-698 is always true) is reproduced
explicitly.  The only cross-time coupling left is the block-level skip of
fully flagged / all-NaN (station, freq) blocks (:817-825), handled in
``run_phase``.

``pinv(.., rcond=1e-3)`` has scipy >= 1.7 semantics: absolute cutoff
``s > 1e-3`` with ``rtol = 0`` (scipy/linalg/basic.py:1326-1328 in scipy 1.7.1).
"""

import numpy as np

PINV_ATOL = 1e-3


def pinv_abs(a, atol=PINV_ATOL):
    """scipy.linalg.pinv(a, rcond=atol) under scipy 1.7: keep s > atol."""
    a = np.asarray(a, dtype=np.float64)
    if a.size == 0:
        return a.T.copy()
    u, s, vh = np.linalg.svd(a, full_matrices=False)
    rank = int(np.sum(s > atol))
    u = u[:, :rank] / s[:rank]
    return (u @ vh[:rank]).T


def calculate_svd(pp, r_0, beta):
    """stationscreen.py:390-430 -> (C, pinv(C), U)."""
    pp = np.asarray(pp, dtype=np.float64)
    diff = pp[:, None, :] - pp[None, :, :]
    d2 = np.sum(diff ** 2, axis=2)
    c = -((d2 / r_0 ** 2) ** (beta / 2.0)) / 2.0
    pinv_c = pinv_abs(c)
    u, _, _ = np.linalg.svd(c)
    return c, pinv_c, u


def normalize_phase(phase):
    """utils/processing_utils.py:73-98."""
    out = np.fmod(phase, 2.0 * np.pi)
    nans = np.isnan(out)
    np.putmask(out, nans, 0)
    out[out < -np.pi] += 2.0 * np.pi
    out[out > np.pi] -= 2.0 * np.pi
    np.putmask(out, nans, np.nan)
    return out


def nancircstd(samples, axis=None):
    """utils/processing_utils.py:101-132 (is_phase=True)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        x1 = np.sin(samples)
        x2 = np.cos(samples)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            r = np.hypot(np.nanmean(x1, axis=axis), np.nanmean(x2, axis=axis))
        return np.sqrt(-2 * np.log(r))


def flag_outliers_slot(w, resid, nsigma):
    """stationscreen.py:303-350, phase type, one time slot (the std is per
    time across directions, :337).  Returns a new weight vector."""
    w = w.copy()
    if not np.any(w > 0.0):
        return w
    res = normalize_phase(resid.copy())
    res_nan = res.copy()
    res_nan[w == 0.0] = np.nan
    std = nancircstd(res_nan)
    with np.errstate(invalid="ignore"):
        w[np.abs(res) > nsigma * std] = 0.0
    return w


def circ_chi2(samples, weights):
    """stationscreen.py:353-387 (squares of sin/cos, quirk Q7)."""
    unfl = weights > 0.0
    if not np.any(unfl):
        return 0.0
    x1 = np.sin(samples[unfl])
    x2 = np.cos(samples[unfl])
    m1, sw = np.average(x1 ** 2, weights=weights[unfl], returned=True)
    m2, sw = np.average(x2 ** 2, weights=weights[unfl], returned=True)
    return (1.0 - np.hypot(m1, m2)) * sw


class Basis:
    """The shared KL basis (FULL_MATRICES + piercepoints)."""

    def __init__(self, pp, r_0=100.0, beta=5.0 / 3.0):
        self.pp = np.asarray(pp, dtype=np.float64)
        self.r_0 = float(r_0)
        self.beta = float(beta)
        self.c, self.pinv_c, self.u = calculate_svd(self.pp, self.r_0, self.beta)


def fit_screen(phi, w, order, basis, screen_type="phase"):
    """stationscreen.py:433-594 for one slot: returns (white[D], resid[D])."""
    d_all = phi.shape[0]
    unfl = np.where(w > 0.0)[0]
    n = unfl.size
    pp_unfl = basis.pp[unfl]
    wd = np.diag(np.asarray(w, np.float64)[unfl])
    if n == d_all:
        c, pinv_c, u = basis.c, basis.pinv_c, basis.u  # Q1: global matrices
    else:
        c, pinv_c, u = calculate_svd(pp_unfl, basis.r_0, basis.beta)
    uk = u[:, :order]
    arg1 = uk.T @ (wd @ u)[:, :order]
    inv_u = pinv_abs(arg1)

    def project(rhs):
        rr1 = uk.T @ (wd @ rhs)
        return pinv_c @ (uk @ (inv_u @ rr1))

    if screen_type == "phase":
        re = project(np.cos(phi[unfl]))
        im = project(np.sin(phi[unfl]))
        screen = np.arctan2(c @ im, c @ re)
    elif screen_type == "tec":
        screen = c @ project(phi[unfl])
    elif screen_type == "amplitude":
        screen = c @ project(np.log10(phi[unfl]))
    else:
        raise ValueError(screen_type)
    white = pinv_c @ screen

    if n != d_all:
        screen_all = np.zeros(d_all)
        screen_all[unfl] = screen
        for f in np.where(w <= 0.0)[0]:
            d2 = np.sum(np.square(pp_unfl - basis.pp[f]), axis=1)
            cval = -((d2 / basis.r_0 ** 2) ** (basis.beta / 2.0)) / 2.0
            screen_all[f] = cval @ white
        white_all = basis.pinv_c @ screen_all
        if screen_type == "amplitude":
            resid_all = phi - 10 ** screen_all
        else:
            resid_all = phi - screen_all
    else:
        white_all = white
        if screen_type == "amplitude":
            resid_all = phi - 10 ** (c @ white)
        else:
            resid_all = phi - c @ white
    return white_all, resid_all


def fit_slot(phi, w, order, station_order, basis, niter=2, nsigma=5.0,
             adjust_order=True, screen_type="phase"):
    """stationscreen.py:597-782 for one (station, freq, pol, time) slot.

    Returns (white[D], resid[D], w_out[D] float32, order_out, n_fits)."""
    d = phi.shape[0]
    w = np.asarray(w, np.float32).copy()
    screen = np.zeros(d)
    resid = np.zeros(d)
    order = float(order)
    station_order = float(station_order)
    nfits = 0
    for it in range(niter):
        if it > 0 and screen_type == "phase":
            w = flag_outliers_slot(w, resid.copy(), nsigma)
        elif it > 0:
            raise NotImplementedError("oracle: phase only beyond iteration 0")
        norderiter = 4 if (adjust_order and it > 0) else 1
        n_unfl = int(np.sum(w > 0.0))
        if n_unfl == 0:
            continue
        if order > n_unfl - 1:
            order = float(n_unfl - 1)
        hit_upper = hit_lower = hit_upper2 = hit_lower2 = False
        sign = 1.0
        prev_redchi2 = 0.0
        for oindx in range(norderiter):
            skip_fit = False
            if it > 0:
                # Q2: station_weights is prev_station_weights -> always equal
                if not adjust_order:
                    break
                if oindx == 0:
                    skip_fit = True
            if not np.all(w == 0.0) and not skip_fit:
                screen, resid = fit_screen(phi, w, int(order), basis,
                                           screen_type)
                nfits += 1
            if hit_lower2 or hit_upper2:
                break
            if adjust_order and it > 0:
                redchi2 = circ_chi2(resid, w) / (n_unfl - order)
                if oindx > 0:
                    if redchi2 > 1.0 and prev_redchi2 < redchi2:
                        sign *= -1
                    if redchi2 < 1.0 and prev_redchi2 > redchi2:
                        sign *= -1
                prev_redchi2 = redchi2
                order_factor = (n_unfl - order) ** 0.2
                target = float(order) - sign * order_factor * (1.0 - redchi2)
                target = max(station_order, target)
                target = min(int(round(target)), n_unfl - 1)
                if target <= 0:
                    target = min(station_order, n_unfl - 1)
                if target == order:
                    break
                if target == n_unfl - 1:
                    if hit_upper:
                        hit_upper2 = True
                    hit_upper = True
                if target == station_order:
                    if hit_lower:
                        hit_lower2 = True
                    hit_lower = True
                order = float(target)
    return screen, resid, w, order, nfits


def reference_station(weight, max_ind=10):
    """utils/processing_utils.py:538-574 on a [time, freq, ant, dir] weight."""
    w = np.sum(weight, axis=(0, 1, 3), dtype=np.float64)
    max_ind = min(max_ind, w.shape[0])
    return int(np.where(w[:max_ind] == np.max(w[:max_ind]))[0][0])


def station_orders(ant_pos, ref_ant, order, min_order=5, scale_order=True,
                   scale_dist=None):
    """stationscreen.py:999-1034 (float32 distances, Q11)."""
    n = len(ant_pos)
    if not scale_order or ref_ant == -1:
        return [order] * n
    pos = [np.asarray(p, dtype=np.float32) for p in ant_pos]
    ref = pos[ref_ant]
    dist = [np.sqrt((ref[0] - p[0]) ** 2 + (ref[1] - p[1]) ** 2
                    + (ref[2] - p[2]) ** 2) for p in pos]
    if scale_dist is None:
        scale_dist = max(dist)
    out = []
    for k in range(n):
        # float32 sqrt; python int * float32 scalar -> float64 under numpy<2
        v = float(order) * float(np.sqrt(np.float32(dist[k] / scale_dist)))
        out.append(max(min_order, min(order, int(v))))
    return out


def run_phase(val, weight, ant_pos, pp, ref_ant, order, r_0=100.0,
              beta=5.0 / 3.0, niter=2, nsigma=5.0, min_order=5,
              scale_order=True, adjust_order=True, slot_filter=None):
    """stationscreen.run for a scalar-phase soltab ([time, freq, ant, dir]).

    Returns dict(coef, resid, w_out, orders) in the soltab layout.
    ``slot_filter(t, f, a) -> bool`` restricts the work to a slot sample (the
    unselected slots are left at zero) for the bounded CPU baseline.
    """
    val = np.array(val, dtype=np.float64)
    weight = np.asarray(weight, dtype=np.float32)
    nt, nf, na, nd = val.shape
    if ref_ant != -1:
        val = val - val[:, :, ref_ant:ref_ant + 1, :]  # :994-997
    st_order = station_orders(ant_pos, ref_ant, order, min_order, scale_order)
    basis = Basis(pp, r_0, beta)
    coef = np.zeros_like(val)
    resid = np.zeros_like(val)
    w_out = weight.copy()
    orders = np.zeros((nt, nf, na), dtype=np.int32)
    for f in range(nf):
        for a in range(na):
            if a == ref_ant:
                continue
            if np.all(np.isnan(val[:, f, a, :])) or np.all(weight[:, f, a, :] == 0):
                continue
            for t in range(nt):
                if slot_filter is not None and not slot_filter(t, f, a):
                    continue
                white, res, w, o, _ = fit_slot(
                    val[t, f, a], weight[t, f, a], st_order[a], st_order[a],
                    basis, niter, nsigma, adjust_order)
                coef[t, f, a] = white
                resid[t, f, a] = res
                w_out[t, f, a] = w
                orders[t, f, a] = int(o)
    return dict(coef=coef, resid=resid, w_out=w_out, orders=orders,
                st_order=st_order, basis=basis)


def cpix_matrix(pp, x_coord, y_coord, r_0=100.0, beta=5.0 / 3.0):
    """kl_screen.py:444-448: C_pix[(j, i), d] for pixel (y=j, x=i) at
    (X[i], Y[j], 0) -- one row per output pixel in FITS order (y-major)."""
    pp = np.asarray(pp, dtype=np.float64)
    xx = np.asarray(x_coord, np.float64)[None, :, None]
    yy = np.asarray(y_coord, np.float64)[:, None, None]
    d2 = (pp[None, None, :, 0] - xx) ** 2 + (pp[None, None, :, 1] - yy) ** 2
    d2 = d2 + pp[None, None, :, 2] ** 2
    c = -((d2 / (r_0 ** 2)) ** (beta / 2.0)) / 2.0
    return c.reshape(len(y_coord) * len(x_coord), pp.shape[0])


def eval_phase_screens(coef_slots, cpix):
    """kl_screen.py:411-449 for a batch: phase[s, pixel] = C_pix @ coef[s]."""
    return np.asarray(coef_slots, np.float64) @ cpix.T


def eval_planes(phase, amp_xx=None, amp_yy=None):
    """kl_screen.py:367-380: the 4 Jones planes (Re XX, Im XX, Re YY, Im YY),
    float64, [..., 4, pixel]."""
    c, s = np.cos(phase), np.sin(phase)
    if amp_xx is None:
        return np.stack([c, s, c, s], axis=-2)
    return np.stack([amp_xx * c, amp_xx * s, amp_yy * c, amp_yy * s], axis=-2)


def process_station_block(vals, wts, order0, basis, screen_type, niter=2,
                          nsigma=5.0, adjust_order=True):
    """stationscreen.py:597-782 for a whole [D, T] station block (any screen
    type; amplitude / tec flag with ONE sigma over the block, quirk Q6).
    Returns (white [D, T], resid [D, T], w [D, T], orders [T])."""
    d, t_n = vals.shape
    screen = np.zeros((d, t_n))
    resid = np.zeros((d, t_n))
    order = np.full(t_n, float(order0))
    station_order = float(order0)
    w = np.asarray(wts, np.float32).copy()
    for it in range(niter):
        if it > 0:
            if screen_type in ("phase", "tec"):
                diff = resid.copy()
            else:
                diff = np.log10(vals) - np.log10(np.abs(vals - resid))
            nonfl = np.where(w > 0.0)
            if nonfl[0].size > 0:
                if screen_type == "phase":
                    r = normalize_phase(diff)
                    rn = r.copy()
                    rn[np.where(w == 0.0)] = np.nan
                    std = nancircstd(rn, axis=0)
                else:
                    r = diff
                    std = np.sqrt(np.average(r[nonfl] ** 2, weights=w[nonfl], axis=0))
                with np.errstate(invalid="ignore"):
                    w[np.where(np.abs(r) > nsigma * std)] = 0.0
        norderiter = 4 if (adjust_order and it > 0) else 1
        for t in range(t_n):
            n_unfl = int(np.sum(w[:, t] > 0.0))
            if n_unfl == 0:
                continue
            if order[t] > n_unfl - 1:
                order[t] = n_unfl - 1
            hit_upper = hit_lower = hit_upper2 = hit_lower2 = False
            sign = 1.0
            prev = 0.0
            for oi in range(norderiter):
                skip = False
                if it > 0:
                    if not adjust_order:
                        break
                    if oi == 0:
                        skip = True
                if not np.all(w[:, t] == 0.0) and not skip:
                    wh, rs = fit_screen(vals[:, t], w[:, t], int(order[t]), basis,
                                        screen_type)
                    screen[:, t] = wh
                    resid[:, t] = rs
                if hit_lower2 or hit_upper2:
                    break
                if adjust_order and it > 0:
                    if screen_type == "phase":
                        redchi2 = circ_chi2(resid[:, t], w[:, t]) / (n_unfl - order[t])
                    elif screen_type == "amplitude":
                        sd = np.log10(vals[:, t]) - np.log10(np.abs(vals[:, t] - resid[:, t]))
                        redchi2 = np.sum(np.square(sd) * w[:, t]) / (n_unfl - order[t])
                    else:
                        redchi2 = np.sum(np.square(resid[:, t]) * w[:, t]) / (n_unfl - order[t])
                    if oi > 0:
                        if redchi2 > 1.0 and prev < redchi2:
                            sign *= -1
                        if redchi2 < 1.0 and prev > redchi2:
                            sign *= -1
                    prev = redchi2
                    factor = (n_unfl - order[t]) ** 0.2
                    target = float(order[t]) - sign * factor * (1.0 - redchi2)
                    target = max(station_order, target)
                    target = min(int(round(target)), n_unfl - 1)
                    if target <= 0:
                        target = min(station_order, n_unfl - 1)
                    if target == order[t]:
                        break
                    if target == n_unfl - 1:
                        if hit_upper:
                            hit_upper2 = True
                        hit_upper = True
                    if target == station_order:
                        if hit_lower:
                            hit_lower2 = True
                        hit_lower = True
                    order[t] = target
    return screen, resid, w, order


def run_amplitude(val, weight, pp, order, r_0=100.0, beta=5.0 / 3.0, niter=3,
                  nsigma=5.0, adjust_order=True):
    """stationscreen.run on an amplitude soltab [time, freq, ant, dir, pol] as
    KLScreen.fit calls it (kl_screen.py:117-125: ref_ant=-1,
    scale_order=False)."""
    val = np.asarray(val, np.float64)
    weight = np.asarray(weight, np.float32)
    nt, nf, na, nd, npol = val.shape
    basis = Basis(pp, r_0, beta)
    coef = np.zeros_like(val)
    resid = np.zeros_like(val)
    w_out = weight.copy()
    orders = np.zeros((nt, nf, na, npol), np.int32)
    for p in range(npol):
        for f in range(nf):
            for a in range(na):
                v = val[:, f, a, :, p].T
                w = weight[:, f, a, :, p].T
                if np.all(np.isnan(v)) or np.all(w == 0):
                    continue
                sc, rs, ww, oo = process_station_block(v, w, order, basis,
                                                       "amplitude", niter,
                                                       nsigma, adjust_order)
                coef[:, f, a, :, p] = sc.T
                resid[:, f, a, :, p] = rs.T
                w_out[:, f, a, :, p] = ww.T
                orders[:, f, a, p] = oo.astype(np.int32)
    return dict(coef=coef, resid=resid, w_out=w_out, orders=orders)


def run_soltab(val, weight, ant_pos, pp, ref_ant, order, screen_type,
               r_0=100.0, beta=5.0 / 3.0, niter=2, nsigma=5.0, min_order=5,
               scale_order=True, adjust_order=True):
    """stationscreen.run (:858-1161) for one polarization [time, freq, ant,
    dir] of any screen type, block by block through process_station_block:
    referencing with the Q15 precedence (:993-996; tec with ref_ant == -1
    subtracts the LAST station), the reference-station skip for phase / tec
    (:818-820) and the all-NaN / all-flagged skip (:822-827)."""
    val = np.array(val, dtype=np.float64)
    weight = np.asarray(weight, dtype=np.float32)
    nt, nf, na, nd = val.shape
    if ref_ant != -1 and screen_type == "phase" or screen_type == "tec":
        val = val - val[:, :, ref_ant:ref_ant + 1 if ref_ant != -1 else None, :]
    st_order = station_orders(ant_pos, ref_ant, order, min_order, scale_order)
    basis = Basis(pp, r_0, beta)
    coef = np.zeros_like(val)
    resid = np.zeros_like(val)
    w_out = weight.copy()
    orders = np.zeros((nt, nf, na), dtype=np.int32)
    for f in range(nf):
        for a in range(na):
            if a == ref_ant and screen_type in ("phase", "tec"):
                continue
            v = val[:, f, a, :].T
            w = weight[:, f, a, :].T
            if np.all(np.isnan(v)) or np.all(w == 0):
                continue
            sc, rs, ww, oo = process_station_block(v, w, st_order[a], basis,
                                                   screen_type, niter, nsigma,
                                                   adjust_order)
            coef[:, f, a] = sc.T
            resid[:, f, a] = rs.T
            w_out[:, f, a] = ww.T
            orders[:, f, a] = oo.astype(np.int32)
    return dict(coef=coef, resid=resid, w_out=w_out, orders=orders)


def interpolate_nearest(vals, src_times, src_freqs, dst_times, dst_freqs):
    """screen.py:108-154 on log-amplitude coefficients: scipy interp1d
    (kind="nearest", fill_value="extrapolate") along time then frequency."""
    import scipy.interpolate as si
    out = np.asarray(vals)
    if len(src_times) == 1:
        shape = list(out.shape)
        shape[0] = len(dst_times)
        shape[1] = len(dst_freqs)
        return np.resize(out, shape)
    if out.shape[0] != len(dst_times):
        out = si.interp1d(src_times, out, axis=0, kind="nearest",
                          fill_value="extrapolate")(dst_times)
    if out.shape[1] != len(dst_freqs):
        out = si.interp1d(src_freqs, out, axis=1, kind="nearest",
                          fill_value="extrapolate")(dst_freqs)
    return out

"""``stationscreen.run`` on the MI355X: the batched KL screen fit.

Same signature, argument meaning, return codes and soltab side effects as the
reference operator (stationscreen.py:858-1161), but every (station, time,
freq) slot is fitted on the GPU through the C ABI ``sf_kl_fit``: the
classify / mask-assign / subset-eigenbasis kernels and ``kl_fit_pass_kernel``
of csrc/kl_fit_fast.hip (one slot per wavefront, two per wavefront in 32-lane
groups for D <= 32; eigenbasis solve), with ``kl_fit_general_kernel``
(csrc/kl_fit.hip) for slots whose weights sit at the pinv cutoff.  The host does
only the O(A + D) setup: piercepoints and midpoint, per-station orders, the
shared basis upload, and the soltab bookkeeping.
"""

import logging

import numpy as np

from . import geometry
from ._lib import SF_SCREEN_AMPLITUDE, SF_SCREEN_PHASE, SF_SCREEN_TEC, private_context

log = logging.getLogger("ska_sdp_screen_fitting_amd.stationscreen")


def station_orders(station_positions, ref_ant, order, min_order=5,
                   scale_order=True, scale_dist=None):
    """Initial per-station order (stationscreen.py:999-1034), with the
    float32 distance arithmetic of the H5parm antenna table (Q11)."""
    n = len(station_positions)
    if not scale_order or ref_ant == -1:
        return [int(order)] * n
    pos = np.asarray(station_positions, dtype=np.float32)
    d = pos - pos[ref_ant]
    dist = np.sqrt(d[:, 0] ** 2 + d[:, 1] ** 2 + d[:, 2] ** 2)  # float32
    if scale_dist is None:
        scale_dist = dist.max()
    # sqrt in float32, then the product with the Python int in float64 (the
    # reference's numpy<2 scalar promotion)
    root = np.sqrt((dist / np.float32(scale_dist)).astype(np.float32))
    return [max(min_order, min(int(order), int(float(order) * float(v))))
            for v in root]


def _device_fit(phase, weight, pp, st_order, screen_type, niter, nsigma,
                adjust_order, ref_ant, beta, r_0, device=0):
    """Run sf_kl_fit on host arrays [T, F, A, D]; returns host arrays."""
    import torch

    T, F, A, D = phase.shape
    dev = torch.device("cuda", device)
    # a context of its own for the basis + fit sequence: another thread's
    # fit or screen cannot re-base it between the two
    with private_context(device) as ctx, torch.cuda.device(dev):
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        ctx.set_basis(pp, r_0, beta)
        ph = torch.from_numpy(np.ascontiguousarray(phase, np.float64)).to(dev)
        wt = torch.from_numpy(np.ascontiguousarray(weight, np.float32)).to(dev)
        coef = torch.empty_like(ph)
        resid = torch.empty_like(ph)
        w_out = torch.empty_like(wt)
        order_out = torch.empty((T, F, A), dtype=torch.int32, device=dev)
        ctx.fit(ph, wt, T, F, A, st_order, screen_type=screen_type,
                niter=niter, nsigma=nsigma, adjust_order=adjust_order,
                ref_ant=ref_ant, coef=coef, resid=resid, w_out=w_out,
                order_out=order_out)
        torch.cuda.current_stream(dev).synchronize()
        return (coef.cpu().numpy(), resid.cpu().numpy(), w_out.cpu().numpy(),
                order_out.cpu().numpy())


def run(soltab, outsoltab, order=12, beta=5.0 / 3.0, niter=2, nsigma=5.0,
        ref_ant=-1, scale_order=True, scale_dist=None, min_order=5,
        adjust_order=True, ncpu=0, device=0):
    """Fit station screens to a phase, tec or amplitude soltab
    (stationscreen.py:858).  Amplitude screens are fitted to log10 of the
    amplitudes, per polarization, with one outlier sigma per (station, freq)
    block (stationscreen.py:535-548, 669-700).

    Writes ``outsoltab`` (white KL coefficients, weights after flagging) and
    ``outsoltab + "resid"`` (residuals, orders as weights) into the soltab's
    solset, with attributes beta, r_0, height, midra, middec and the
    ``piercepoint`` array.  Returns 0, or 1 for an unsupported soltab type.
    ``ncpu`` is accepted for signature compatibility (the fit runs on the
    GPU).
    """
    del ncpu
    screen_type = soltab.get_type()
    if screen_type not in ("phase", "tec", "amplitude"):
        log.error('Screens can only be fit to soltabs of type "phase", '
                  '"tec", or "amplitude".')
        return 1

    axis_names = soltab.get_axes_names()
    val = np.asarray(soltab.val, dtype=np.float64)
    weight = np.asarray(soltab.weight, dtype=np.float32)
    order_axes = [axis_names.index(a) for a in ("time", "freq", "ant", "dir")]
    has_pol = "pol" in axis_names
    if has_pol:
        order_axes.append(axis_names.index("pol"))
    val = np.transpose(val, order_axes)
    weight = np.transpose(weight, order_axes)
    if not has_pol:
        val = val[..., np.newaxis]
        weight = weight[..., np.newaxis]
    n_times, n_freqs, n_stations, n_sources, n_pols = val.shape

    solset = soltab.get_solset()
    source_names = list(soltab.dir[:])
    source_dict = solset.get_source()
    source_positions = np.array([source_dict[s] for s in source_names], dtype=np.float32)
    station_names = list(soltab.ant[:])
    station_dict = solset.get_ant()
    station_positions = np.array([station_dict[s] for s in station_names], dtype=np.float32)

    if isinstance(ref_ant, str):
        if n_stations == 1 or ref_ant not in station_names:
            ref_ant = -1
        else:
            ref_ant = station_names.index(ref_ant)
    st_order = station_orders(station_positions, ref_ant, order, min_order,
                              scale_order, scale_dist)
    r_0 = 100
    pp, mid_ra, mid_dec = geometry.piercepoints(source_positions)

    stype = {"phase": SF_SCREEN_PHASE, "tec": SF_SCREEN_TEC,
             "amplitude": SF_SCREEN_AMPLITUDE}[screen_type]
    coef = np.zeros(val.shape)
    resid = np.zeros(val.shape)
    w_out = np.zeros(weight.shape, dtype=np.float32)
    orders = np.zeros((n_times, n_freqs, n_stations, n_pols))
    if stype == SF_SCREEN_AMPLITUDE and n_pols > 1:
        # amplitude screens are never referenced (stationscreen.py:994 applies
        # to phase / tec) and their outlier sigma is per (station, freq) block
        # (Q6): the pols are independent station blocks, so ONE fit of the
        # pols stacked along the station axis gives every pol's result bit
        # for bit, with the fixed per-call costs (host syncs, mask table,
        # latency-bound subset bases -- shared when the pols' flags agree)
        # paid once (tests/test_gain.py::test_stacked_pol_fit_equals_per_pol)
        c, r, w, o = _device_fit(
            np.concatenate([val[..., p] for p in range(n_pols)], axis=2),
            np.concatenate([weight[..., p] for p in range(n_pols)], axis=2),
            pp, np.tile(st_order, n_pols), stype, niter, nsigma, adjust_order,
            -1, beta, r_0, device)
        for pol in range(n_pols):
            sl = slice(pol * n_stations, (pol + 1) * n_stations)
            coef[..., pol], resid[..., pol], w_out[..., pol] = c[:, :, sl], r[:, :, sl], w[:, :, sl]
            orders[..., pol] = o[:, :, sl]
    else:
        for pol in range(n_pols):
            c, r, w, o = _device_fit(val[..., pol], weight[..., pol], pp, st_order,
                                     stype, niter, nsigma, adjust_order, ref_ant,
                                     beta, r_0, device)
            coef[..., pol], resid[..., pol], w_out[..., pol] = c, r, w
            orders[..., pol] = o

    times, freqs = np.asarray(soltab.time), np.asarray(soltab.freq)
    axes = ["time", "freq", "ant", "dir"]
    axes_vals = [times, freqs, station_names, source_names]
    res_w = np.repeat(orders[:, :, :, np.newaxis, :], n_sources, axis=3)
    if has_pol:
        axes = axes + ["pol"]
        axes_vals = axes_vals + [soltab.pol[:]]
    else:
        coef, resid, w_out, res_w = (x[..., 0] for x in (coef, resid, w_out, res_w))
    screen_st = solset.make_soltab(f"{screen_type}screen", outsoltab,
                                   axes_names=axes, axes_vals=axes_vals,
                                   vals=coef, weights=w_out)
    solset.make_soltab(f"{screen_type}screenresid", outsoltab + "resid",
                       axes_names=axes, axes_vals=axes_vals, vals=resid,
                       weights=res_w)
    screen_st.attrs.update(beta=beta, r_0=r_0, height=0.0, midra=mid_ra,
                           middec=mid_dec)
    screen_st.piercepoint = pp
    return 0

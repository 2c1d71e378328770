"""KL (Karhunen-Loeve) screens on the MI355X (kl_screen.py:22-449 of the
reference).

``KLScreen`` keeps the reference's constructor and methods.  ``fit`` runs the
batched GPU fit (``stationscreen.run`` -> ``sf_kl_fit``: the fit-pass,
subset-eigenbasis and classify kernels of csrc/kl_fit_fast.hip);
``make_matrix`` and ``write`` evaluate the screens with ``sf_kl_eval`` (the
LDS-staged ``kl_eval_lds_kernel`` or the register-tile ``kl_eval_kernel`` of
csrc/kl_eval.hip, chosen per D: an MFMA float64 contraction + sincos
epilogue) instead of a per-pixel Python loop in a process pool.
"""

import multiprocessing

import numpy as np

from . import geometry
from . import stationscreen
from ._lib import (SF_EVAL_BIG_ENDIAN, SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB,
                   SF_EVAL_NT_STORES, Context)
from .h5parm import H5parm, get_reference_station
from .screen import Screen

# NaN scrub (screen.py:368-378) + exact fp64 reduction of the phase in
# revolutions / hardware fp32 sincos + streaming stores
DEFAULT_FLAGS = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES


def read_patch_names(skymodel_filename):
    """Patch names of a makesourcedb sky model (the patch lines ``, , name,
    ra, dec``), i.e. the keys of lsmtool ``getPatchPositions()``."""
    names = []
    with open(skymodel_filename, encoding="utf8") as fh:
        for line in fh:
            parts = [p.strip() for p in line.split(",")]
            if len(parts) >= 5 and parts[0] == "" and parts[1] == "" and parts[2]:
                names.append(parts[2])
    return names


class KLEvaluator:
    """Device state for evaluating KL screens on one grid.  Owns its sf_ctx:
    the basis and pixel grid it sets stay put whatever other screens or the
    fit (which takes a ``private_context`` per call) set meanwhile."""

    def __init__(self, piercepoints, r_0, beta, x_coord, y_coord, device=0):
        import torch

        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.ctx = Context(device)
        self.pp = np.asarray(piercepoints, np.float64)
        self.D = self.pp.shape[0]
        self.nx, self.ny = len(x_coord), len(y_coord)
        with torch.cuda.device(self.dev):
            self.ctx.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
            self.ctx.set_basis(self.pp, r_0, beta)
            self.ctx.set_grid(x_coord, y_coord)

    def eval_device(self, coef_dev, out_dev=None, flags=DEFAULT_FLAGS):
        """coef_dev: device [S, D] float64 -> device [S, 4, ny, nx] float32."""
        torch = self.torch
        S = coef_dev.shape[0]
        if out_dev is None:
            out_dev = torch.empty((S, 4, self.ny, self.nx), dtype=torch.float32,
                                  device=self.dev)
        with torch.cuda.device(self.dev):
            self.ctx.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
            self.ctx.eval(coef_dev, S, out_dev, S, flags)
        return out_dev

    def eval_gain_device(self, coef_dev, xx_dev, yy_dev, out_dev=None,
                         flags=DEFAULT_FLAGS):
        """Phase + XX / YY log10-amplitude coefficients (device [S, D] each)
        -> device [S, 4, ny, nx] gain planes."""
        torch = self.torch
        S = coef_dev.shape[0]
        if out_dev is None:
            out_dev = torch.empty((S, 4, self.ny, self.nx), dtype=torch.float32,
                                  device=self.dev)
        with torch.cuda.device(self.dev):
            self.ctx.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
            self.ctx.eval_gain(coef_dev, xx_dev, yy_dev, S, out_dev, S, flags)
        return out_dev

    def smooth_device(self, out_dev, smooth_pix, flags):
        """Screen.write's Gaussian (screen.py:353-362) in place on a device
        cube [S, 4, ny, nx]; scrub / byte swap in ``flags`` after it."""
        torch = self.torch
        with torch.cuda.device(self.dev):
            self.ctx.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
            self.ctx.smooth(out_dev, self.nx, self.ny, 4 * out_dev.shape[0],
                            smooth_pix, flags)
        return out_dev

    def _upload(self, a):
        a = np.ascontiguousarray(a, np.float64)
        return self.torch.from_numpy(a.reshape(-1, self.D)).to(self.dev)

    def eval_host(self, coef, amp_xx=None, amp_yy=None, flags=DEFAULT_FLAGS):
        """coef (and optional log10-amplitude coefs): host [..., D] -> host
        float32 [..., 4, ny, nx]."""
        coef = np.asarray(coef)
        lead = coef.shape[:-1]
        c = self._upload(coef)
        if amp_xx is None:
            out = self.eval_device(c, flags=flags)
        else:
            out = self.eval_gain_device(c, self._upload(amp_xx),
                                        self._upload(amp_yy), flags=flags)
        return out.cpu().numpy().reshape(lead + (4, self.ny, self.nx))


class KLScreen(Screen):
    """Class for KL (Karhunen-Lo`eve) screens (kl_screen.py:22)."""

    def __init__(self, name, h5parm_filename, skymodel_filename, rad, dec,
                 width_ra, width_dec, solset_name="sol000",
                 phase_soltab_name="phase000", amplitude_soltab_name=None):
        super().__init__(name, h5parm_filename, skymodel_filename, rad, dec,
                         width_ra, width_dec, solset_name=solset_name,
                         phase_soltab_name=phase_soltab_name,
                         amplitude_soltab_name=amplitude_soltab_name)
        self.height = None
        self.beta_val = None
        self.r_0 = None
        self.piercepoints = None
        self.mid_ra = None
        self.mid_dec = None
        self._evaluators = {}

    def fit(self):
        """Fit screens to the input solutions (kl_screen.py:61-155): phases
        with per-station orders referenced to a central station; for gain
        solutions also the XX / YY log10 amplitudes (order
        min(12, max(3, round(D / 2))), 3 iterations, no order scaling)."""
        self._evaluators = {}  # a refit invalidates the evaluated basis
        h5 = H5parm(self.input_h5parm_filename)
        solset = h5.get_solset(self.input_solset_name)
        soltab_ph = solset.get_soltab(self.input_phase_soltab_name)
        dirs = [str(d) for d in soltab_ph.dir]
        if self.input_skymodel_filename is not None:
            patches = set(read_patch_names(self.input_skymodel_filename))
            missing = [d for d in dirs if d.strip("[]") not in patches]
            if missing:  # the reference raises KeyError here (kl_screen.py:79)
                raise KeyError(f"directions not in the sky model: {missing}")
        ref_ind = get_reference_station(soltab_ph, 10)
        screen_order = min(20, len(dirs) - 1)
        stationscreen.run(soltab_ph, "phase_screen000", order=screen_order,
                          ref_ant=ref_ind, scale_order=True, adjust_order=True,
                          ncpu=self.ncpu or 0, device=self.device)
        if not self.phase_only:
            soltab_amp = solset.get_soltab(self.input_amplitude_soltab_name)
            order_amp = min(12, max(3, int(np.round(len(dirs) / 2))))
            stationscreen.run(soltab_amp, "amplitude_screen000", order=order_amp,
                              niter=3, scale_order=False, adjust_order=True,
                              ncpu=self.ncpu or 0, device=self.device)
            sta = solset.get_soltab("amplitude_screen000")
            self.log_amps = True
            self.vals_amp = sta.val
            self.times_amp = np.asarray(sta.time)
            self.freqs_amp = np.asarray(sta.freq)
        st = solset.get_soltab("phase_screen000")
        self.vals_ph = st.val
        self.times_ph = np.asarray(st.time)
        self.freqs_ph = np.asarray(st.freq)
        self.source_names = st.dir
        self.source_dict = solset.get_source()
        self.source_positions = [self.source_dict[s] for s in self.source_names]
        self.station_names = st.ant
        self.station_dict = solset.get_ant()
        self.station_positions = [self.station_dict[s] for s in self.station_names]
        self.height = st.attrs["height"]
        self.beta_val = st.attrs["beta"]
        self.r_0 = st.attrs["r_0"]
        self.piercepoints = np.array(st.piercepoint)
        self.mid_ra = st.attrs["midra"]
        self.mid_dec = st.attrs["middec"]
        h5.close()

    def get_memory_usage(self, cellsize_deg):
        """GB per time slot, the reference's estimate (kl_screen.py:157-190:
        int() sizes, /10 overhead, x ncpu) so that time chunking matches."""
        ncpu = self.ncpu or multiprocessing.cpu_count()
        ximsize = int(self.width_ra / cellsize_deg)
        yimsize = int(self.width_dec / cellsize_deg)
        nbytes = 8 * len(self.freqs_ph) * len(self.station_names) * 4 * yimsize * ximsize
        return nbytes / 1024 ** 3 / 10 * ncpu

    def evaluator(self, cellsize_deg):
        key = float(cellsize_deg)
        ev = self._evaluators.get(key)
        if ev is None:
            x, y = geometry.grid_coords(self.rad, self.dec, self.width_ra,
                                        cellsize_deg, self.mid_ra, self.mid_dec)
            ev = KLEvaluator(self.piercepoints, self.r_0, self.beta_val, x, y,
                             self.device)
            self._evaluators = {key: ev}
        return ev

    def make_matrix(self, t_start_index, t_stop_index, freq_ind, stat_ind,
                    cellsize_deg, out_dir, ncpu):
        """(t_stop - t_start, 4, ny, nx) float64 (kl_screen.py:192-380): the
        raw cos / sin (x 10 ** amplitude) planes, NaN where a coefficient is
        NaN -- the reference scrubs NaNs only in ``Screen.write``, after the
        optional smoothing (screen.py:353-378), and so does ``write_chunk``.
        The values carry the float32 rounding of the FITS cube (Q12)."""
        del out_dir, ncpu
        sl = np.s_[t_start_index:t_stop_index, freq_ind, stat_ind, :]
        coef = np.asarray(self.vals_ph)[sl]
        ev = self.evaluator(cellsize_deg)
        flags = DEFAULT_FLAGS & ~SF_EVAL_NAN_SCRUB
        if self.phase_only:
            return ev.eval_host(coef, flags=flags).astype(np.float64)
        amp = np.asarray(self.vals_amp)[sl]
        return ev.eval_host(coef, amp[..., 0], amp[..., 1],
                            flags=flags).astype(np.float64)

    def write_chunk(self, writer, g_start, g_stop, cellsize_deg, smooth_pix,
                    max_batch_bytes=1 << 30):
        """All (freq, station) screens of times [g_start, g_stop): device
        batches of whole time rows in FITS byte order, streamed through
        pinned buffers to the file while the next batch is evaluated."""
        from .streaming import PinnedPipeline
        torch = __import__("torch")
        ev = self.evaluator(cellsize_deg)
        vals = np.asarray(self.vals_ph)
        n_f, n_a, D = vals.shape[1], vals.shape[2], vals.shape[3]
        per_slot = 16 * ev.nx * ev.ny
        row_bytes = n_f * n_a * per_slot
        rows = max(1, int(max_batch_bytes // row_bytes))
        rows = min(rows, g_stop - g_start)
        coef = ev._upload(vals[g_start:g_stop])
        if not self.phase_only:
            amp = np.asarray(self.vals_amp)[g_start:g_stop]
            c_xx, c_yy = ev._upload(amp[..., 0]), ev._upload(amp[..., 1])
        pipe = PinnedPipeline(torch, ev.dev, rows * row_bytes)
        try:
            for t0 in range(g_start, g_stop, rows):
                t1 = min(g_stop, t0 + rows)
                s0, s1 = (t0 - g_start) * n_f * n_a, (t1 - g_start) * n_f * n_a
                slot, buf = pipe.device_buffer((s1 - s0) * per_slot)
                out = buf.view(torch.float32).view(s1 - s0, 4, ev.ny, ev.nx)
                fin = SF_EVAL_NAN_SCRUB | SF_EVAL_BIG_ENDIAN
                # with smoothing, scrub and byte swap come after the Gaussian
                # (screen.py:353-378 smooths, then replaces NaNs)
                flags = DEFAULT_FLAGS | fin if smooth_pix <= 0 else \
                    DEFAULT_FLAGS & ~SF_EVAL_NAN_SCRUB
                if self.phase_only:
                    ev.eval_device(coef[s0:s1], out, flags)
                else:
                    ev.eval_gain_device(coef[s0:s1], c_xx[s0:s1], c_yy[s0:s1],
                                        out, flags)
                if smooth_pix > 0:
                    ev.smooth_device(out, smooth_pix, fin)
                pipe.submit(slot, (s1 - s0) * per_slot, writer)
        finally:
            pipe.close()

"""Screen base class: the a-term FITS writer around the device kernels.

Mirrors ``Screen`` of the reference (screen.py:19-411): same constructor,
``process``/``write``/``interpolate``/``make_matrix``/``get_memory_usage``
methods and the same FITS products (``{name}_{g}.fits`` per time chunk and
``{name}.txt`` listing them).  ``write`` evaluates a whole time chunk at once
on the GPU (all frequencies and stations in one kernel launch per device
batch) instead of looping ``make_matrix`` over (freq, station).
"""

import logging
import os

import numpy as np

from . import fits


def _angle_deg(v):
    """astropy ``Angle(str).to('deg')`` for the sexagesimal forms rapthor
    passes ("12h34m56s", "12:34:56", "+65d13m47s", or plain degrees)."""
    if not isinstance(v, str):
        return v
    s = v.strip().lower()
    hours = "h" in s
    for ch in "hdms:":
        s = s.replace(ch, " ")
    parts = s.split()
    sign = -1.0 if parts[0].startswith("-") else 1.0
    vals = [abs(float(p)) for p in parts]
    while len(vals) < 3:
        vals.append(0.0)
    deg = sign * (vals[0] + vals[1] / 60.0 + vals[2] / 3600.0)
    return deg * 15.0 if hours else deg


def available_memory_gb():
    """utils/processing_utils.py:599-614 (floored GB)."""
    try:
        import psutil
        return int(np.floor(psutil.virtual_memory().available / 1024 ** 3))
    except ImportError:  # pragma: no cover
        pages = os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
        return int(np.floor(pages / 1024 ** 3))


def time_chunks(times, mem_per_slot_gb, available_gb=None):
    """Gap + memory splitting of the time axis (screen.py:283-317, Q9).
    Returns the chunk end indices."""
    times = np.asarray(times)
    if len(times) > 2:
        delta = times[1:] - times[:-1]
        width = np.min(delta)
        gaps_ind = np.nonzero(delta > width * 1.2)[0] + 1
        gaps_ind = np.append(gaps_ind, np.array([len(times)]))
    else:
        gaps_ind = np.array([len(times)])
    if len(times) > 2:
        if available_gb is None:
            available_gb = available_memory_gb()
        max_ntimes = max(1, int(available_gb / mem_per_slot_gb))
        check = True
        while check:
            check = False
            g_start = 0
            for gnum, g_stop in enumerate(gaps_ind.copy()):
                if g_stop - g_start > max_ntimes:
                    gaps_ind = np.insert(gaps_ind, gnum,
                                         np.array([g_start + int((g_stop - g_start) / 2)]))
                    check = True
                    break
                g_start = g_stop
    return [int(g) for g in gaps_ind]


def nearest_index(src, dst):
    """Index of the nearest ``src`` sample for every ``dst`` point, ties to
    the lower sample, clamped at the ends (scipy interp1d kind="nearest"
    with fill_value="extrapolate")."""
    src = np.asarray(src, np.float64)
    order = np.argsort(src, kind="mergesort")
    xs = src[order]
    bounds = (xs[1:] + xs[:-1]) / 2.0
    idx = np.searchsorted(bounds, np.asarray(dst, np.float64), side="left")
    return order[np.clip(idx, 0, len(xs) - 1)]


def resample_axis(src, vals, dst, axis, kind="nearest"):
    """One axis of Screen.interpolate; "nearest" is an exact row gather."""
    if kind == "nearest":
        return np.take(vals, nearest_index(src, dst), axis=axis)
    import scipy.interpolate as si
    return si.interp1d(src, vals, axis=axis, kind=kind,
                       fill_value="extrapolate")(dst)


class Screen:
    """Master class for a-term screens (screen.py:19)."""

    def __init__(self, name, h5parm_filename, skymodel_filename, rad, dec,
                 width_ra, width_dec, solset_name="sol000",
                 phase_soltab_name="phase000", amplitude_soltab_name=None):
        self.name = name
        self.log = logging.getLogger(f"rapthor:{self.name}")
        self.input_h5parm_filename = h5parm_filename
        self.input_skymodel_filename = skymodel_filename
        self.input_solset_name = solset_name
        self.input_phase_soltab_name = phase_soltab_name
        self.input_amplitude_soltab_name = amplitude_soltab_name
        self.phase_only = amplitude_soltab_name is None
        self.rad = _angle_deg(rad)
        self.dec = _angle_deg(dec)
        width = max(width_ra, width_dec)  # square images (screen.py:77-81)
        self.width_ra = width
        self.width_dec = width
        self.log_amps = False
        self.times_amp = None
        self.times_ph = []
        self.vals_amp = None
        self.vals_ph = None
        self.freqs_amp = None
        self.freqs_ph = None
        self.station_names = None
        self.source_names = None
        self.source_dict = None
        self.source_positions = None
        self.station_dict = None
        self.station_positions = None
        self.ncpu = None
        self.device = 0

    def fit(self):
        """Implemented by the subclasses."""

    def interpolate(self, interp_kind="nearest"):
        """Put the slow amplitudes on the fast-phase time / frequency grid
        (screen.py:108-154): interpolation in log10 space along time, then
        frequency, extrapolating at the ends; KL screens already hold log10
        values (``log_amps``), tessellated ones hold amplitudes."""
        if self.phase_only:
            return
        vals = np.asarray(self.vals_amp)
        n_t, n_f = np.shape(self.vals_ph)[:2]
        if len(self.times_amp) == 1:
            shape = list(vals.shape)
            shape[0], shape[1] = n_t, n_f
            self.vals_amp = np.resize(vals, shape)
            return
        logvals = vals if self.log_amps else np.log10(vals)
        if vals.shape[0] != n_t:
            logvals = resample_axis(self.times_amp, logvals, self.times_ph, 0,
                                    interp_kind)
        if vals.shape[1] != n_f:
            logvals = resample_axis(self.freqs_amp, logvals, self.freqs_ph, 1,
                                    interp_kind)
        self.vals_amp = logvals if self.log_amps else 10 ** logvals

    def grid_size(self, cellsize_deg):
        return (int(np.ceil(self.width_ra / cellsize_deg)),
                int(np.ceil(self.width_dec / cellsize_deg)))

    def make_matrix(self, t_start_index, t_stop_index, freq_ind, stat_ind,
                    cellsize_deg, out_dir, ncpu):
        """(t_stop - t_start, 4, ny, nx) values; defined by the subclasses."""
        raise NotImplementedError

    def get_memory_usage(self, cellsize_deg):
        """GB per time slot; defined by the subclasses."""
        raise NotImplementedError

    def write_chunk(self, writer, g_start, g_stop, cellsize_deg, smooth_pix):
        """Evaluate times [g_start, g_stop) and stream them to ``writer``;
        defined by the subclasses."""
        raise NotImplementedError

    def write(self, out_dir, cellsize_deg, smooth_pix=0, ncpu=0):
        """Write the a-term screens to FITS cubes (screen.py:260-394)."""
        self.ncpu = ncpu
        gaps_ind = time_chunks(self.times_ph, self.get_memory_usage(cellsize_deg))
        nx, ny = self.grid_size(cellsize_deg)
        outfiles = []
        g_start = 0
        for gnum, g_stop in enumerate(gaps_ind):
            outfile = os.path.join(out_dir, f"{self.name}_{gnum}.fits")
            cards = fits.aterm_header(self.rad, self.dec, nx, ny, cellsize_deg,
                                      self.freqs_ph, self.times_ph[g_start:g_stop],
                                      len(self.station_names))
            shape = (g_stop - g_start, len(self.freqs_ph), len(self.station_names),
                     4, ny, nx)
            writer = fits.CubeWriter(outfile, cards, shape)
            try:
                self.write_chunk(writer, g_start, g_stop, cellsize_deg, smooth_pix)
            finally:
                writer.close()
            outfiles.append(outfile)
            g_start = g_stop
        with open(os.path.join(out_dir, f"{self.name}.txt"), "w",
                  encoding="utf8") as fh:
            fh.writelines([o + "\n" for o in outfiles])
        return outfiles

    def process(self, ncpu=0):
        """Fit, then interpolate (screen.py:396-411)."""
        self.ncpu = ncpu
        self.fit()
        self.interpolate()

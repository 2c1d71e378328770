"""Synthetic solution cubes of the shapes named in BASELINE.json.

The reference ships one small fixture (resources/solutions.h5: 20 t x 12 f x
62 ant x 7 dir).  Configs 3-5 are synthetic; this module makes them with the
recipe of SURVEY.md §8(d), seed 20260:

* field: rad=126.23, dec=64.50, width 3.33 deg (square, ceil(width/cell) pixels);
* directions: D sources uniform in a disc of radius 1.5 deg about the field
  centre, stored as float32 radians exactly like the H5parm ``source`` table
  (``utils/h5parm.py:750-767``);
* stations: LOFAR CS001HBA0 ITRF position plus uniform +-20 km offsets (float32,
  like the H5parm ``antenna`` table);
* times: 8.0111 s spacing, no gaps; freqs: 122.2 MHz + 4.05 MHz k;
* phases: smooth linear+quadratic gradient across the directions per
  (ant, time, freq) with 0.3 rad rms, plus N(0, 0.05) noise; a fraction of the
  entries get a +2 rad outlier (drives ``_flag_outliers``,
  ``stationscreen.py:303-350``);
* weights: 1.0 with a fraction of (slot, dir) set to 0 (drives the flagged
  branch of ``_fit_screen``, ``stationscreen.py:495-499, 565-582``).

Layouts follow the H5parm scalarphase soltab: ``val[time, freq, ant, dir]``
float64 and ``weight[time, freq, ant, dir]`` float32.  Only numpy is used, so
the same generator runs under the reference's interpreter (golden vectors) and
on the GPU box (benchmark inputs).
"""

from dataclasses import dataclass, field

import numpy as np

FIELD_RA_DEG = 126.23
FIELD_DEC_DEG = 64.50
FIELD_WIDTH_DEG = 3.3300000000000054  # make_aterm_images.py:116-118 arithmetic
CS001 = (3826896.2, 460979.47, 5064658.0)

# cellsizes that give the named grid sides under ceil(width / cell)
# (3.33/N has a 5e-15 excess and gives N+1)
CELLSIZE_FOR_GRID = {17: 0.2, 128: 0.02602, 256: 0.01301, 512: 0.006505}


@dataclass
class SolutionSet:
    """In-memory equivalent of one H5parm scalarphase soltab + its solset.

    Mirrors the pieces of ``Soltab``/``Solset`` the KL path reads
    (``stationscreen.py:936-979``, ``kl_screen.py:66-155``).
    """

    val: np.ndarray            # [time, freq, ant, dir] float64 (radians)
    weight: np.ndarray         # [time, freq, ant, dir] float32
    times: np.ndarray          # [time] float64 (s)
    freqs: np.ndarray          # [freq] float64 (Hz)
    ant_names: list            # [ant] str
    ant_pos: np.ndarray        # [ant, 3] float32 ITRF (m)
    dir_names: list            # [dir] str, H5parm style "[Patch_k]"
    dir_radec: np.ndarray      # [dir, 2] float32 radians
    soltype: str = "phase"
    amp_val: np.ndarray = None  # optional amplitude soltab [time, freq, ant, dir, pol]
    meta: dict = field(default_factory=dict)

    @property
    def shape(self):
        return self.val.shape


def make_solutions(n_ant, n_time, n_freq, n_dir, seed=20260, flag_frac=0.01,
                   outlier_frac=0.005, ant_offset=0, n_ant_total=None,
                   tiny_weight_frac=0.0, field_ra=FIELD_RA_DEG,
                   field_dec=FIELD_DEC_DEG, disc_deg=1.5):
    """Make a synthetic scalarphase solution set.

    ``ant_offset`` / ``n_ant_total`` produce one ant-shard of a larger array
    (every shard sees the same directions, times and freqs; stations and
    phases are drawn per station from a per-station stream so the shard is
    identical to the matching slice of the full set).
    """
    if n_ant_total is None:
        n_ant_total = ant_offset + n_ant
    rng = np.random.default_rng(seed)

    # directions: uniform in a disc (same for every shard)
    r = disc_deg * np.sqrt(rng.random(n_dir))
    th = 2.0 * np.pi * rng.random(n_dir)
    dec = field_dec + r * np.sin(th)
    ra = field_ra + r * np.cos(th) / np.cos(np.deg2rad(dec))
    dir_radec = np.deg2rad(np.stack([ra, dec], axis=1)).astype(np.float32)
    dir_names = [f"[Patch_{k}]" for k in range(n_dir)]

    times = 4987958432.341753 + 8.0111 * np.arange(n_time)
    freqs = 122.2e6 + 4.05e6 * np.arange(n_freq)

    # direction-space basis for the smooth gradient (unit-rms per term)
    x = (ra - field_ra) * np.cos(np.deg2rad(field_dec))
    y = dec - field_dec
    basis = np.stack([x, y, x * x, x * y, y * y], axis=0)
    basis -= basis.mean(axis=1, keepdims=True)
    basis /= np.sqrt((basis ** 2).mean(axis=1, keepdims=True)) + 1e-30

    ant_pos = np.empty((n_ant, 3), dtype=np.float32)
    val = np.empty((n_time, n_freq, n_ant, n_dir), dtype=np.float64)
    weight = np.ones((n_time, n_freq, n_ant, n_dir), dtype=np.float32)
    for a in range(n_ant):
        ga = ant_offset + a
        srng = np.random.default_rng([seed, ga])
        off = srng.uniform(-20e3, 20e3, size=3) if ga > 0 else np.zeros(3)
        ant_pos[a] = (np.array(CS001) + off).astype(np.float32)
        coeff = srng.normal(0.0, 0.3 / np.sqrt(5.0), size=(n_time, n_freq, 5))
        ph = coeff @ basis
        ph += srng.normal(0.0, 0.05, size=ph.shape)
        out = srng.random(ph.shape) < outlier_frac
        ph[out] += 2.0
        val[:, :, a, :] = ph
        fl = srng.random(ph.shape) < flag_frac
        w = np.ones(ph.shape, dtype=np.float32)
        w[fl] = 0.0
        if tiny_weight_frac > 0:
            tiny = (srng.random(ph.shape) < tiny_weight_frac) & ~fl
            w[tiny] = np.float32(5e-4)
        weight[:, :, a, :] = w
    ant_names = [f"ST{ant_offset + a:04d}" for a in range(n_ant)]
    return SolutionSet(val=val, weight=weight, times=times, freqs=freqs,
                       ant_names=ant_names, ant_pos=ant_pos, dir_names=dir_names,
                       dir_radec=dir_radec,
                       meta=dict(seed=seed, n_ant_total=n_ant_total,
                                 ant_offset=ant_offset))


def make_amplitudes(sol, n_time=None, n_freq=None, seed=20261, flag_frac=0.01,
                    outlier_frac=0.005, rms_log=0.05):
    """Synthetic XX/YY amplitude soltab ([time, freq, ant, dir, pol]) on a
    (possibly coarser) time / frequency grid spanning the phase grid: a smooth
    log10-amplitude gradient across directions plus noise; outliers get x3.
    Stored in ``sol.amp_*`` (the slow-amplitude half of a "gain" solution)."""
    T, F, A, D = sol.val.shape
    n_time = n_time or T
    n_freq = n_freq or F
    rng = np.random.default_rng(seed)
    t = np.linspace(sol.times[0], sol.times[-1], n_time)
    f = np.linspace(sol.freqs[0], sol.freqs[-1], n_freq)
    ra = sol.dir_radec[:, 0].astype(np.float64)
    de = sol.dir_radec[:, 1].astype(np.float64)
    basis = np.stack([ra - ra.mean(), de - de.mean()], axis=0)
    basis /= np.sqrt((basis ** 2).mean(axis=1, keepdims=True)) + 1e-30
    coeff = rng.normal(0.0, rms_log, size=(n_time, n_freq, A, 2, 2))
    logamp = np.einsum("tfapk,kd->tfadp", coeff, basis)
    logamp += rng.normal(0.0, rms_log / 5, size=logamp.shape)
    amp = 10.0 ** logamp
    out = rng.random(amp.shape) < outlier_frac
    amp[out] *= 3.0
    w = np.ones(amp.shape, np.float32)
    w[rng.random(amp.shape) < flag_frac] = 0.0
    sol.amp_val = amp
    sol.meta["amp_weight"] = w
    sol.meta["amp_times"] = t
    sol.meta["amp_freqs"] = f
    return sol

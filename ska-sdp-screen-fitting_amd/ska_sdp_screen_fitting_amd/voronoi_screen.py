"""Tessellated (Voronoi) screens (voronoi_screen.py:24-351 of the reference).

The label raster ("template") is host setup, computed once per run: patch
positions from the sky model, SIN pixel coordinates, a Voronoi tessellation
closed by a 64-point outer ring, one polygon per direction rasterized with
Pillow exactly as ``utils/processing_utils.rasterize`` does (fill + outline
with rounded vertices, then an exact border test of the outline pixels,
quirk Q10) and a nearest-label fallback for uncovered pixels.  The per-slot
work -- gather of each direction's (amplitude x) cos / sin into its cells and
the optional Gaussian smoothing of ``Screen.write`` (screen.py:353-362) --
runs on the GPU through ``sf_tess_fill``: a per-slot value-table kernel, then
the gather-store kernel (no smoothing) or the wide-tile smoothing kernel
(csrc/tess.hip).
"""

import os

import numpy as np
import scipy.interpolate as si
from PIL import Image, ImageDraw
from scipy.spatial import Voronoi

from . import fits, geometry
from ._lib import SF_EVAL_BIG_ENDIAN, SF_EVAL_NAN_SCRUB, private_context
from .h5parm import H5parm, get_reference_station
from .screen import Screen


def parse_angle(text, hours):
    """lsmtool patch-position strings: RA "hh:mm:ss.s", Dec "dd.mm.ss.s"."""
    t = text.strip()
    sign = -1.0 if t.startswith("-") else 1.0
    t = t.lstrip("+-")
    f = t.split(":") if ":" in t else t.split(".", 2)
    val = float(f[0]) + float(f[1]) / 60.0 + float(f[2]) / 3600.0
    return sign * val * (15.0 if hours else 1.0)


def read_patch_positions(skymodel_filename):
    """{patch name: (ra_deg, dec_deg)} from the patch lines of a sky model."""
    out = {}
    with open(skymodel_filename, encoding="utf8") as fh:
        for line in fh:
            p = [x.strip() for x in line.split(",")]
            if len(p) == 5 and p[0] == "" and p[1] == "" and p[2]:
                out[p[2]] = (parse_angle(p[3], True), parse_angle(p[4], False))
    return out


def _on_or_inside(ring, x, y):
    """Not shapely-disjoint: winding number != 0 or on an edge."""
    wn = 0
    for (x0, y0), (x1, y1) in zip(ring[:-1], ring[1:]):
        cr = (x1 - x0) * (y - y0) - (x - x0) * (y1 - y0)
        if cr == 0.0 and min(x0, x1) <= x <= max(x0, x1) and \
                min(y0, y1) <= y <= max(y0, y1):
            return True
        if y0 <= y < y1 and cr > 0:
            wn += 1
        elif y1 <= y < y0 and cr < 0:
            wn -= 1
    return wn != 0


def rasterize_cell(ring, n):
    """utils/processing_utils.py:295-334 for one closed ring, n x n image:
    returns a boolean mask [y, x]."""
    img = Image.new("L", (n, n), 0)
    ImageDraw.Draw(img).polygon(ring, outline=1, fill=1)
    mask = np.array(img) > 0
    edge = Image.new("L", (n, n), 0)
    ImageDraw.Draw(edge).polygon(ring, outline=1, fill=0)
    ey, ex = np.nonzero(np.array(edge))
    for x, y in zip(ex, ey):
        if not _on_or_inside(ring, float(x), float(y)):
            mask[y, x] = False
    return mask


def tessellation_template(patch_radec, rad, dec, width_deg, cellsize_deg):
    """voronoi_screen.py:218-351 -> (labels [ny, nx] int32 in 1..D, patch xy).
    Cells are painted in shapely.ops.polygonize order (later cells win a
    shared pixel)."""
    rings, xy, n, order = _rings(patch_radec, rad, dec, width_deg, cellsize_deg)
    return paint_cells(rings, n, order), xy


def _rings(patch_radec, rad, dec, width_deg, cellsize_deg):
    """Voronoi cell rings in pixel coordinates (voronoi_screen.py:230-309):
    SIN pixel positions of the patches, the field box, a 64-point outer ring
    closing the tessellation; each direction's bounded region as
    ``shapely.ops.polygonize`` of the bounded ridges returns it (:311-317).

    The ring convention follows the GEOS Polygonizer algorithm (restated
    literally, as a graph walk, in oracle/voronoi.py::geos_polygonize): every
    ridge j = (a, b) of ``ridge_vertices`` adds directed edges 2j (a -> b)
    and 2j + 1 (b -> a); a ring keeps its face on the right, so a cell's
    exterior is clockwise; it starts at the start vertex of the lowest-index
    directed edge that bounds the cell, and the polygons come out in the
    order of those indices.  Pillow's outline (and so the outline pixels
    the exact test sees) depends on the ring's start and direction, and the
    painting order on the polygon order.  Returns (rings in direction order,
    xy, n, painting order of the directions)."""
    n = geometry.grid_size(width_deg, cellsize_deg)
    crval, crpix, cdelt = (rad, dec), (n / 2.0, n / 2.0), (-cellsize_deg, cellsize_deg)
    ra = np.asarray(patch_radec, np.float64)[:, 0]
    de = np.asarray(patch_radec, np.float64)[:, 1]
    xy = np.stack(geometry.sin_world2pix(ra, de, crval, crpix, cdelt), axis=1)
    bnd = (rad + width_deg / 2.0, dec - width_deg / 2.0,
           rad - width_deg / 2.0, dec + width_deg / 2.0)
    x0, y0 = geometry.sin_world2pix(max(bnd[0], ra.max() + 0.1),
                                    min(bnd[1], de.min() - 0.1), crval, crpix, cdelt)
    x1, y1 = geometry.sin_world2pix(min(bnd[2], ra.min() - 0.1),
                                    max(bnd[3], de.max() + 0.1), crval, crpix, cdelt)
    x0, y0, x1, y1 = float(x0), float(y0), float(x1), float(y1)
    if len(xy) == 1:
        rings = [[(x0, y0), (x0, y1), (x1, y1), (x1, y0), (x0, y0)]]
    else:
        k = np.arange(64)
        radius = 2.0 * np.hypot(x1 - x0, y1 - y0)
        ring_pts = xy.mean(axis=0) + radius * np.stack(
            [np.cos(np.pi / 32.0 * k), np.sin(np.pi / 32.0 * k)], axis=1)
        vor = Voronoi(np.vstack([xy, ring_pts]))
        # lowest directed-edge index (and its start vertex) bounding each cell
        first = {}
        j = 0
        for (va, vb), (p, q) in zip(vor.ridge_vertices, vor.ridge_points):
            if va == -1 or vb == -1:
                continue
            a, b = vor.vertices[va], vor.vertices[vb]
            for c in (p, q):
                if c < len(xy):
                    # cell c on the right of a -> b: the forward edge 2j
                    right = ((b[0] - a[0]) * (xy[c, 1] - a[1])
                             - (b[1] - a[1]) * (xy[c, 0] - a[0])) < 0
                    de, start = (2 * j, va) if right else (2 * j + 1, vb)
                    if c not in first or de < first[c][0]:
                        first[c] = (de, start)
            j += 1
        rings = []
        for i in range(len(xy)):
            reg = vor.regions[vor.point_region[i]]
            if -1 in reg or i not in first:
                raise ValueError("unbounded Voronoi cell for a direction")
            v = vor.vertices[reg]
            ctr = v.mean(axis=0)
            cw = np.argsort(-np.arctan2(v[:, 1] - ctr[1], v[:, 0] - ctr[0]))
            idx = [reg[k] for k in cw]
            k0 = idx.index(first[i][1])
            idx = idx[k0:] + idx[:k0]
            pts = [(float(vor.vertices[k][0]), float(vor.vertices[k][1])) for k in idx]
            rings.append(pts + [pts[0]])
        order = sorted(range(len(xy)), key=lambda c: first[c][0])
        return rings, xy, n, order
    return rings, xy, n, [0]


def paint_cells(rings, n, order=None):
    """voronoi_screen.py:319-349: rasterize every cell ring (label = index +
    1) in ``order`` (default: list order; the reference paints in polygonize
    order) -- a pixel claimed by two cells (its centre exactly on their
    shared edge: the exact border test keeps it in both) takes the later one
    -- then give uncovered pixels the nearest painted label (griddata
    'nearest' in index space).  On the fixture no pixel is claimed twice at
    0.2, 0.1, 0.05 or 0.02602 deg (tests/test_tessellated.py)."""
    labels = np.zeros((n, n), np.int32)
    for i in (range(len(rings)) if order is None else order):
        labels[rasterize_cell(rings[i], n)] = i + 1
    empty = labels == 0
    if empty.any():
        iy, ix = np.nonzero(~empty)
        zy, zx = np.nonzero(empty)
        labels[empty] = si.griddata((iy, ix), labels[~empty], (zy, zx),
                                    method="nearest")
    return labels


def cell_rings(patch_radec, rad, dec, width_deg, cellsize_deg):
    """The closed pixel-space rings of tessellation_template (for tests)."""
    return _rings(patch_radec, rad, dec, width_deg, cellsize_deg)[0]


def gaussian_weights(smooth_pix, truncate=4.0):
    """scipy.ndimage._gaussian_kernel1d (order 0): radius and weights."""
    sigma = float(smooth_pix)
    radius = int(truncate * sigma + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    return radius, phi / phi.sum()


class VoronoiScreen(Screen):
    """Class for Voronoi screens (voronoi_screen.py:24)."""

    def __init__(self, name, h5parm_filename, skymodel_filename, rad, dec,
                 width_ra, width_dec, solset_name="sol000",
                 phase_soltab_name="phase000", amplitude_soltab_name=None):
        super().__init__(name, h5parm_filename, skymodel_filename, rad, dec,
                         width_ra, width_dec, solset_name=solset_name,
                         phase_soltab_name=phase_soltab_name,
                         amplitude_soltab_name=amplitude_soltab_name)
        self.data_rasertize_template = None
        self.polygons = None
        self._dev_cache = None

    def fit(self):
        """Reference the phases to one station (voronoi_screen.py:57-102);
        gain solutions also keep the raw XX / YY amplitudes
        [time, freq, ant, dir, pol] for interpolation."""
        h5 = H5parm(self.input_h5parm_filename)
        solset = h5.get_solset(self.input_solset_name)
        st = solset.get_soltab(self.input_phase_soltab_name)
        ref = get_reference_station(st, 10)
        vals = np.array(st.val, dtype=np.float64)
        vals = vals - vals[:, :, ref:ref + 1, :]
        self.vals_ph = vals
        self.times_ph = np.asarray(st.time)
        self.freqs_ph = np.asarray(st.freq)
        if self.phase_only:
            self.vals_amp = None  # ones (phase only)
            self.times_amp, self.freqs_amp = self.times_ph, self.freqs_ph
        else:
            sta = solset.get_soltab(self.input_amplitude_soltab_name)
            names = sta.get_axes_names()
            order = [names.index(a) for a in ("time", "freq", "ant", "dir", "pol")]
            self.log_amps = False
            self.vals_amp = np.transpose(np.asarray(sta.val, np.float64), order)
            self.times_amp = np.asarray(sta.time)
            self.freqs_amp = np.asarray(sta.freq)
        self.source_names = st.dir
        self.source_dict = solset.get_source()
        self.source_positions = [self.source_dict[s] for s in self.source_names]
        self.station_names = st.ant
        self.station_dict = solset.get_ant()
        self.station_positions = [self.station_dict[s] for s in self.station_names]
        h5.close()

    def get_memory_usage(self, cellsize_deg):
        """voronoi_screen.py:104-130 (x10 overhead, no ncpu factor)."""
        ximsize = int(self.width_ra / cellsize_deg)
        yimsize = int(self.width_dec / cellsize_deg)
        nbytes = 8 * len(self.freqs_ph) * len(self.station_names) * 4 * yimsize * ximsize
        return nbytes / 1024 ** 3 * 10

    def make_rasertize_template(self, cellsize_deg, out_dir):
        """voronoi_screen.py:218-351; also writes {name}_template.fits."""
        n = geometry.grid_size(self.width_ra, cellsize_deg)
        path = os.path.join(out_dir, f"{self.name}_template.fits")
        cards = fits.aterm_header(self.rad, self.dec, n, n, cellsize_deg,
                                  self.freqs_ph, self.times_ph[0:1],
                                  len(self.station_names))
        w = fits.CubeWriter(path, cards, (1, len(self.freqs_ph),
                                          len(self.station_names), 4, n, n))
        w.write(np.zeros((1, len(self.freqs_ph), len(self.station_names), 4, n, n),
                         np.float32))
        w.close()
        pos = read_patch_positions(self.input_skymodel_filename)
        radec = np.array([pos[str(s).strip("[]")] for s in self.source_names])
        self.data_rasertize_template, self.polygons = tessellation_template(
            radec, self.rad, self.dec, self.width_ra, cellsize_deg)
        self._dev_cache = None

    def _device(self):
        import torch
        if self._dev_cache is None:
            dev = torch.device("cuda", self.device)
            lab = torch.from_numpy(self.data_rasertize_template.astype(np.int32)).to(dev)
            self._dev_cache = (dev, lab)
        return self._dev_cache

    def eval_device(self, ph_dev, out_dev, smooth_pix=0.0,
                    flags=SF_EVAL_NAN_SCRUB, amp_xx=None, amp_yy=None):
        """device [S, D] referenced phases (and optional XX / YY amplitudes,
        device [S, D]) -> device [S, 4, ny, nx]."""
        import torch
        dev, lab = self._device()
        ny, nx = self.data_rasertize_template.shape
        S, D = ph_dev.shape
        # the fill's scratch (table, smoothing buffers) is the context's: a
        # context of its own per call.  The call returns with its kernels
        # queued, so the context carries an event of its last fill: the next
        # holder's stream waits for it before reusing the scratch (another
        # thread's stream is not ordered after this one)
        with private_context(self.device) as ctx, torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            busy = getattr(ctx, "tess_busy", None)
            if busy is not None:
                stream.wait_event(busy)
            ctx.set_stream(stream.cuda_stream)
            ctx.tess_fill(lab, nx, ny, ph_dev, D, S, out_dev, amp_xx=amp_xx,
                          amp_yy=amp_yy, smooth_pix=smooth_pix, flags=flags)
            ctx.tess_busy = torch.cuda.Event()
            ctx.tess_busy.record(stream)
        return out_dev

    def _upload(self, a):
        import torch
        dev, _ = self._device()
        a = np.ascontiguousarray(a, np.float64)
        return torch.from_numpy(a.reshape(-1, a.shape[-1])).to(dev)

    def eval_host(self, phase, smooth_pix=0.0, amp_xx=None, amp_yy=None,
                  flags=SF_EVAL_NAN_SCRUB):
        """[..., D] referenced phases (optional amplitudes) -> float32
        [..., 4, ny, nx] (gather + optional Gaussian smoothing) on the GPU."""
        import torch
        dev, _ = self._device()
        lead = np.shape(phase)[:-1]
        ny, nx = self.data_rasertize_template.shape
        ph = self._upload(phase)
        axx = None if amp_xx is None else self._upload(amp_xx)
        ayy = None if amp_yy is None else self._upload(amp_yy)
        out = torch.empty((ph.shape[0], 4, ny, nx), dtype=torch.float32, device=dev)
        self.eval_device(ph, out, smooth_pix, flags, amp_xx=axx, amp_yy=ayy)
        return out.cpu().numpy().reshape(lead + (4, ny, nx))

    def make_matrix(self, t_start_index, t_stop_index, freq_ind, stat_ind,
                    cellsize_deg, out_dir, ncpu):
        """(t_stop - t_start, 4, ny, nx) float64 (voronoi_screen.py:132-216):
        the gathered (amplitude x) cos / sin, NaN where a phase is NaN; the
        NaN scrub belongs to ``Screen.write`` (screen.py:364-378)."""
        del ncpu
        if self.data_rasertize_template is None:
            self.make_rasertize_template(cellsize_deg, out_dir)
        sl = np.s_[t_start_index:t_stop_index, freq_ind, stat_ind, :]
        ph = self.vals_ph[sl]
        if self.phase_only:
            return self.eval_host(ph, flags=0).astype(np.float64)
        amp = np.asarray(self.vals_amp)[sl]
        return self.eval_host(ph, amp_xx=amp[..., 0], amp_yy=amp[..., 1],
                              flags=0).astype(np.float64)

    def write(self, out_dir, cellsize_deg, smooth_pix=0, ncpu=0):
        if self.data_rasertize_template is None:
            self.make_rasertize_template(cellsize_deg, out_dir)
        return super().write(out_dir, cellsize_deg, smooth_pix=smooth_pix, ncpu=ncpu)

    def write_chunk(self, writer, g_start, g_stop, cellsize_deg, smooth_pix,
                    max_batch_bytes=1 << 30):
        """Gather + smoothing of times [g_start, g_stop) in FITS byte order,
        streamed through pinned buffers (see streaming.py)."""
        import torch
        from .streaming import PinnedPipeline
        dev, _ = self._device()
        ny, nx = self.data_rasertize_template.shape
        n_f, n_a, D = self.vals_ph.shape[1:]
        per_slot = 16 * nx * ny
        row_bytes = n_f * n_a * per_slot
        rows = min(max(1, int(max_batch_bytes // row_bytes)), g_stop - g_start)
        ph = self._upload(self.vals_ph[g_start:g_stop])
        axx = ayy = None
        if not self.phase_only:
            amp = np.asarray(self.vals_amp)[g_start:g_stop]
            axx, ayy = self._upload(amp[..., 0]), self._upload(amp[..., 1])
        pipe = PinnedPipeline(torch, dev, rows * row_bytes)
        try:
            for t0 in range(g_start, g_stop, rows):
                t1 = min(g_stop, t0 + rows)
                s0, s1 = (t0 - g_start) * n_f * n_a, (t1 - g_start) * n_f * n_a
                slot, buf = pipe.device_buffer((s1 - s0) * per_slot)
                out = buf.view(torch.float32).view(s1 - s0, 4, ny, nx)
                self.eval_device(ph[s0:s1], out, smooth_pix,
                                 SF_EVAL_NAN_SCRUB | SF_EVAL_BIG_ENDIAN,
                                 amp_xx=None if axx is None else axx[s0:s1],
                                 amp_yy=None if ayy is None else ayy[s0:s1])
                pipe.submit(slot, (s1 - s0) * per_slot, writer)
        finally:
            pipe.close()

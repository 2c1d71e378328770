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
a14).  shapely (pinned 1.8.0, GEOS) is absent from every interpreter here, so
its two uses are restated from their published algorithms:
``geos_polygonize`` walks the GEOS Polygonizer's planar graph (directed-edge
insertion order, counter-clockwise edge stars, clockwise shells; the ring
start vertex and direction, which Pillow's outline depends on, and the
polygon order come from it), and ``disjoint(point)`` == "strictly outside
the closed convex cell" (exact orientation tests on float coordinates).
scipy 1.7.1 (the reference's era) and 1.15.3 give bit-identical Voronoi
vertices and ridge order on the fixture at every config cell size.  PARITY
STATUS: the reference's tessellated path cannot run in this image (needs
shapely).  The config-1 raster (0.2 deg, 17^2) is pinned by the reference's
own rendering of its ``tessellated_0.fits`` (resources/screens_.png, decoded
by tests/golden/decode_screens_png.py; tests/test_tess_png_pin.py): all 289
pixels, including the 2 whose label depends on the ring convention, and
every other ring start / direction that moves a pixel is contradicted by it.
At the finer cell sizes (1 / 1156 at 0.1 deg ... 22 / 16384 at 0.02602 deg,
profiles/round3_tess_ring_conventions.txt) the same convention decides a few
pixels that no reference output shows: those follow the convention pinned
at 0.2 deg, not an observed GEOS raster.
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


def _quadrant(dx, dy):
    """geos::geom::Quadrant::quadrant: NE 0, NW 1, SW 2, SE 3."""
    if dx >= 0:
        return 0 if dy >= 0 else 3
    return 1 if dy >= 0 else 2


def _orientation(p1, p2, q):
    """geos::algorithm::Orientation::index: +1 q left of p1->p2 (CCW), -1
    right, 0 collinear (exact: Fraction arithmetic on the float inputs)."""
    from fractions import Fraction as Fr
    det = ((Fr(p2[0]) - Fr(p1[0])) * (Fr(q[1]) - Fr(p1[1]))
           - (Fr(p2[1]) - Fr(p1[1])) * (Fr(q[0]) - Fr(p1[0])))
    return (det > 0) - (det < 0)


def geos_polygonize(segments):
    """shapely.ops.polygonize of two-point LineStrings, restated from the
    GEOS Polygonizer algorithm (operation/polygonize: PolygonizeGraph,
    EdgeRing; the JTS design it ports):

    * every line adds its directed edges in input order: de0 start -> end,
      then de1 end -> start (PlanarGraph::add); nodes are keyed by exact
      coordinates;
    * around each node the outgoing edges are sorted counter-clockwise by
      quadrant, then orientation (DirectedEdge::compareDirection), and the
      edge arriving along outgoing edge e_k continues on e_(k+1)
      (computeNextCWEdges): every ring keeps its face on the right;
    * rings are collected by walking the directed edges in insertion order,
      starting a ring at each edge not yet in one (getEdgeRings), its
      coordinates from that edge's start node on (EdgeRing::getCoordinates);
    * rings that are not counter-clockwise are shells (EdgeRing::isHole):
      the polygons, in that order, exteriors exactly as walked.

    No dangles or cut edges arise from the bounded ridges of a Voronoi
    diagram closed by an outer ring of points (every ridge separates two
    cells, or a cell and the outer face); they are asserted absent.
    Returns a list of closed rings [(x, y), ..., first]."""
    nodes = {}
    des = []  # (from node key, to node key, line index)
    for j, (a, b) in enumerate(segments):
        a, b = (float(a[0]), float(a[1])), (float(b[0]), float(b[1]))
        if a == b:
            continue
        for u, v in ((a, b), (b, a)):
            nodes.setdefault(u, []).append(len(des))
            des.append((u, v, j))
    sym = [i ^ 1 for i in range(len(des))]
    nxt = [None] * len(des)
    import functools

    def cmp(i, k):
        (p0, p1, _), (q0, q1, _) = des[i], des[k]
        qa = _quadrant(p1[0] - p0[0], p1[1] - p0[1])
        qb = _quadrant(q1[0] - q0[0], q1[1] - q0[1])
        if qa != qb:
            return 1 if qa > qb else -1
        return _orientation(q0, q1, p1)  # > 0: des[i] is CCW of des[k]

    for key, out in nodes.items():
        assert len(out) >= 2, "dangle"
        out = sorted(out, key=functools.cmp_to_key(cmp))
        for k in range(len(out)):
            nxt[sym[out[k]]] = out[(k + 1) % len(out)]
    ring_of = [-1] * len(des)
    rings = []
    for start in range(len(des)):
        if ring_of[start] >= 0:
            continue
        ring, de = [], start
        while True:
            ring_of[de] = len(rings)
            ring.append(des[de][0])
            de = nxt[de]
            if de == start:
                break
        rings.append(ring + [ring[0]])
    for i in range(len(des)):
        assert ring_of[i] != ring_of[sym[i]], "cut edge"
    shells = []
    for r in rings:
        area = sum(x0 * y1 - x1 * y0 for (x0, y0), (x1, y1) in zip(r[:-1], r[1:]))
        if area < 0:  # not CCW
            shells.append(r)
    return shells


def _contains(ring, x, y):
    """Point strictly inside a convex closed ring (either orientation)."""
    s = [(bx - ax) * (y - ay) - (by - ay) * (x - ax)
         for (ax, ay), (bx, by) in zip(ring[:-1], ring[1:])]
    return all(v > 0 for v in s) or all(v < 0 for v in s)


def label_raster(ra_deg, dec_deg, rad, dec, width, cellsize):
    """Label template (values 1..D), shape (ny, nx), with the cells as the
    reference gets them from
    shapely.ops.polygonize of the bounded Voronoi ridges
    (voronoi_screen.py:311-349): ``geos_polygonize`` rings (orientation,
    start vertex) rasterized in polygonize order, each labelled with the
    direction it contains."""
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
    tmpl = np.zeros((n, n))
    if len(xy) == 1:
        # one direction: the field box as the single polygon (:283-293); the
        # nearest-label fill below then covers the rest of the image
        x0, y0 = float(fmin[0]), float(fmin[1])
        x1, y1 = float(fmax[0]), float(fmax[1])
        tmpl = rasterize([(x0, y0), (x0, y1), (x1, y1), (x1, y0), (x0, y0)], (n, n))
    else:
        nouter = 64
        ang = np.array([np.pi / (nouter / 2.0) * i for i in range(nouter)])
        radius = 2.0 * np.sqrt((float(fmax[0]) - float(fmin[0])) ** 2
                               + (float(fmax[1]) - float(fmin[1])) ** 2)
        outer = xy.mean(axis=0) + radius * np.stack([np.cos(ang), np.sin(ang)], 1)
        vor = Voronoi(np.vstack([xy, outer]))
        segs = [vor.vertices[r] for r in vor.ridge_vertices if -1 not in r]
        for ring in geos_polygonize(segs):
            idx = [k for k in range(len(xy)) if _contains(ring, xy[k, 0], xy[k, 1])]
            assert len(idx) == 1
            r = rasterize(ring, (n, n)) * (idx[0] + 1)
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

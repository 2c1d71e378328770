"""Minimal streaming FITS writer for a-term cubes (no astropy on the GPU box).

Produces the primary-HDU file that the reference builds with
``make_template_image`` (processing_utils.py:144-292) and fills in
``Screen.write`` (screen.py:331-382): BITPIX -32, axes
[RA, DEC, MATRIX, ANTENNA, FREQ, TIME] (numpy order [time, freq, ant, 4, y, x]),
big-endian float32, header cards in the reference's order.  Data are written
in time-major chunks so a cube never has to exist whole in host memory.
"""

import numpy as np

BLOCK = 2880


def _fmt_value(v):
    if isinstance(v, bool):
        return f"{'T' if v else 'F':>20}"
    if isinstance(v, (int, np.integer)):
        return f"{int(v):>20d}"
    if isinstance(v, (float, np.floating)):
        # 16 significant digits, like the astropy writer the reference uses
        s = f"{float(v):.16G}"
        if "E" in s:
            mant, exp = s.split("E")
            if "." not in mant:
                mant += ".0"
            s = f"{mant}E{int(exp):+03d}"
        elif "." not in s and "INF" not in s and "NAN" not in s:
            s += ".0"
        return f"{s:>20}"
    sval = str(v).replace("'", "''")
    return f"'{sval:<8}'".ljust(20)


def card(key, value):
    c = f"{key:<8}= {_fmt_value(value)}"
    if len(c) > 80:
        raise ValueError(f"FITS card too long: {c}")
    return c.ljust(80)


def aterm_header(rad, dec, nx, ny, cellsize_deg, freqs, times, n_ant):
    """Header cards of make_template_image(..., aterm_type='gain')."""
    freqs = np.asarray(freqs, np.float64)
    times = np.asarray(times, np.float64)
    nt, nf = len(times), len(freqs)
    cards = [("SIMPLE", True), ("BITPIX", -32), ("NAXIS", 6),
             ("NAXIS1", nx), ("NAXIS2", ny), ("NAXIS3", 4), ("NAXIS4", n_ant),
             ("NAXIS5", nf), ("NAXIS6", nt), ("EXTEND", True),
             ("CRVAL1", float(rad)), ("CDELT1", -float(cellsize_deg)),
             ("CRPIX1", nx / 2.0), ("CUNIT1", "deg"), ("CTYPE1", "RA---SIN"),
             ("CRVAL2", float(dec)), ("CDELT2", float(cellsize_deg)),
             ("CRPIX2", ny / 2.0), ("CUNIT2", "deg"), ("CTYPE2", "DEC--SIN"),
             ("CRVAL3", 0.0), ("CDELT3", 1.0), ("CRPIX3", 1.0), ("CUNIT3", ""),
             ("CTYPE3", "MATRIX"),
             ("CRVAL4", 0.0), ("CDELT4", 1.0), ("CRPIX4", 1.0), ("CUNIT4", ""),
             ("CTYPE4", "ANTENNA")]
    ref_freq = float(freqs[0])
    del_freq = float(np.min(freqs[1:] - freqs[:-1])) if nf > 1 else 1e8
    cards += [("RESTFRQ", ref_freq), ("CRVAL5", ref_freq), ("CDELT5", del_freq),
              ("CRPIX5", 1.0), ("CUNIT5", "Hz"), ("CTYPE5", "FREQ")]
    if nt > 1:
        deltas = times[1:] - times[:-1]
        del_time = float(np.min(deltas[:-1])) if nt > 2 else float(deltas[0])
    else:
        del_time = 1.0
    cards += [("CRVAL6", float(times[0])), ("CDELT6", del_time), ("CRPIX6", 1.0),
              ("CUNIT6", "s"), ("CTYPE6", "TIME"), ("EQUINOX", 2000.0),
              ("TELESCOP", "LOFAR")]
    return cards


def header_bytes(cards):
    text = "".join(card(k, v) for k, v in cards) + "END".ljust(80)
    pad = (-len(text)) % BLOCK
    return (text + " " * pad).encode("ascii")


class CubeWriter:
    """Stream a float32 cube into a FITS primary HDU, time-major."""

    def __init__(self, path, cards, shape):
        self.path = path
        self.shape = tuple(shape)
        self.expected = int(np.prod(self.shape)) * 4
        self.written = 0
        self.fh = open(path, "wb")
        self.fh.write(header_bytes(cards))

    def write(self, block):
        """Append the next time rows (any float32 array in C order)."""
        a = np.ascontiguousarray(block, dtype=">f4")
        self.fh.write(a.tobytes())
        self.written += a.nbytes

    def write_raw(self, buf):
        """Append bytes that are already big-endian float32 (device stores
        with SF_EVAL_BIG_ENDIAN)."""
        self.fh.write(buf)
        self.written += len(buf)

    def close(self):
        if self.fh is None:
            return
        if self.written != self.expected:
            self.fh.close()
            self.fh = None
            raise ValueError(f"{self.path}: wrote {self.written} of {self.expected} bytes")
        self.fh.write(b"\0" * ((-self.written) % BLOCK))
        self.fh.close()
        self.fh = None


def read_cube(path, mmap=False):
    """Read back (header dict, data) of a file written by CubeWriter (tests);
    ``mmap``: the data as a read-only big-endian memory map instead of a copy
    (cubes of several GB)."""
    hdr = {}
    off = 0
    with open(path, "rb") as fh:
        while True:
            c = fh.read(80).decode("ascii")
            off += 80
            if not c or c.startswith("END"):
                break
            if c[8:10] == "= ":
                k, v = c[:8].strip(), c[10:].strip()
                if v.startswith("'"):
                    v = v[1:v.rindex("'")].rstrip()
                elif v in ("T", "F"):
                    v = v == "T"
                else:
                    try:
                        v = int(v)
                    except ValueError:
                        v = float(v)
                hdr[k] = v
        off += (-off) % BLOCK
        n = hdr["NAXIS"]
        shape = tuple(hdr[f"NAXIS{n - i}"] for i in range(n))
        if mmap:
            return hdr, np.memmap(path, dtype=">f4", mode="r", offset=off, shape=shape)
        fh.seek(off)
        count = int(np.prod(shape))
        data = np.frombuffer(fh.read(4 * count), dtype=">f4", count=count)
    return hdr, data.reshape(shape)

"""Read-only HDF5 subset for H5parm solution files.

The reference reads H5parms through PyTables (utils/h5parm.py:1-1400); the
GPU box has neither PyTables nor h5py, so this module parses the file format
directly (numpy views over an ``mmap``) for the structures DP3, PyTables and
h5py write into solution files:

* superblock versions 0-3; object headers v1 and v2 ("OHDR"/"OCHK"), with
  continuation blocks;
* old-style groups (symbol table: v1 B-tree of "SNOD" nodes + local heap)
  and compact new-style groups (link messages);
* dataspaces (scalar / simple), datatypes: fixed-point, IEEE float (f2/f4/f8,
  either byte order), fixed strings, compound, array, variable-length
  strings (global heap "GCOL");
* data layouts: compact, contiguous, chunked with a v1 B-tree index
  (layout message v3), with the deflate, shuffle and fletcher32 filters;
* attributes (message versions 1-3).

Anything else (dense link / attribute storage in fractal heaps, v4 chunk
indexes, szip / blosc filters, external storage) raises ``NotImplementedError``
naming the structure, rather than returning wrong data.
"""

import mmap
import zlib

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5FormatError(ValueError):
    """The file is not HDF5 or is damaged."""


def _unsupported(what):
    raise NotImplementedError(f"HDF5 feature not supported by this reader: {what}")


class _Cursor:
    """Little-endian reader over the file buffer with the file's offset /
    length sizes."""

    def __init__(self, f, pos):
        self.f = f
        self.buf = f.buf
        self.pos = pos

    def u(self, n):
        v = int.from_bytes(self.buf[self.pos:self.pos + n], "little")
        self.pos += n
        return v

    def u8(self):
        return self.u(1)

    def u16(self):
        return self.u(2)

    def u32(self):
        return self.u(4)

    def off(self):
        v = self.u(self.f.so)
        return UNDEF if v == (1 << (8 * self.f.so)) - 1 else v + self.f.base

    def length(self):
        return self.u(self.f.sl)

    def raw(self, n):
        b = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return b

    def skip(self, n):
        self.pos += n

    def align(self, k, origin=0):
        self.pos += (-(self.pos - origin)) % k


# ----------------------------------------------------------------- datatypes

class _VlenString:
    """Marker for variable-length strings (read through the global heap)."""

    def __init__(self, size):
        self.itemsize = size


def _parse_datatype(c):
    cv = c.u8()
    cls, ver = cv & 0x0F, cv >> 4
    b0, b1, b2 = c.u8(), c.u8(), c.u8()
    bits = b0 | (b1 << 8) | (b2 << 16)
    size = c.u32()
    if cls == 0:  # fixed point
        c.skip(4)
        order = ">" if b0 & 1 else "<"
        kind = "i" if b0 & 0x08 else "u"
        return np.dtype(f"{order}{kind}{size}")
    if cls == 1:  # floating point
        c.skip(12)
        if b0 & 0x40:
            _unsupported("VAX float byte order")
        order = ">" if b0 & 1 else "<"
        if size not in (2, 4, 8):
            _unsupported(f"{size}-byte float")
        return np.dtype(f"{order}f{size}")
    if cls == 3:  # fixed string
        return np.dtype(f"S{size}")
    if cls == 4:  # bitfield
        c.skip(4)
        return np.dtype(f"V{size}")
    if cls == 5:  # opaque
        tag = c.raw(bits & 0xFF)
        del tag
        return np.dtype(f"V{size}")
    if cls == 6:  # compound
        n = bits & 0xFFFF
        names, formats, offsets = [], [], []
        for _ in range(n):
            s = c.pos
            end = c.buf.find(b"\x00", s)
            name = bytes(c.buf[s:end]).decode("ascii", "replace")
            c.pos = end + 1
            if ver < 3:
                c.align(8, s)
            if ver == 1:
                moff = c.u32()
                ndim = c.u8()
                c.skip(3 + 4 + 4)
                dims = [c.u32() for _ in range(4)][:ndim]
                mt = _parse_datatype(c)
                if ndim:
                    mt = np.dtype((mt, tuple(dims)))
            else:
                if ver == 2:
                    moff = c.u32()
                else:
                    nb = max(1, (size.bit_length() + 7) // 8)
                    moff = c.u(nb)
                mt = _parse_datatype(c)
            if isinstance(mt, _VlenString):
                _unsupported("variable-length string inside a compound")
            names.append(name)
            formats.append(mt)
            offsets.append(moff)
        return np.dtype({"names": names, "formats": formats, "offsets": offsets,
                         "itemsize": size})
    if cls == 9:  # variable length
        vtype = bits & 0x0F
        base = _parse_datatype(c)
        if vtype == 1:
            return _VlenString(size)
        del base
        _unsupported("variable-length sequence")
    if cls == 10:  # array
        ndim = c.u8()
        if ver < 3:
            c.skip(3)
        dims = [c.u32() for _ in range(ndim)]
        if ver < 3:
            c.skip(4 * ndim)
        base = _parse_datatype(c)
        return np.dtype((base, tuple(dims)))
    if cls == 8:  # enumeration: read as the base integer type
        n = bits & 0xFFFF
        base = _parse_datatype(c)
        for _ in range(n):
            s = c.pos
            end = c.buf.find(b"\x00", s)
            c.pos = end + 1
            if ver < 3:
                c.align(8, s)
        c.skip(n * base.itemsize)
        return base
    _unsupported(f"datatype class {cls}")


def _parse_dataspace(c):
    ver = c.u8()
    ndim = c.u8()
    flags = c.u8()
    if ver == 1:
        c.skip(5)
        stype = 1 if ndim > 0 else 0
    else:
        stype = c.u8()
    dims = tuple(c.length() for _ in range(ndim))
    if flags & 1:
        for _ in range(ndim):
            c.length()
    if ver == 1 and flags & 2:
        c.skip(4 * ndim)
    if stype == 2:
        return None  # null dataspace
    return dims


# ---------------------------------------------------------------- file / objects

class _Message:
    __slots__ = ("mtype", "pos", "size")

    def __init__(self, mtype, pos, size):
        self.mtype, self.pos, self.size = mtype, pos, size


class File:
    """``File(path)``: root ``Group`` of an HDF5 file, read-only."""

    def __init__(self, path):
        self.path = path
        self._fh = open(path, "rb")
        try:
            self.buf = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        except ValueError as exc:  # empty file
            self._fh.close()
            raise H5FormatError(f"{path}: empty file") from exc
        self.base = 0
        sb = None
        for cand in (0, 512, 1024, 2048, 4096, 8192, 16384):
            if self.buf[cand:cand + 8] == SIGNATURE:
                sb = cand
                break
        if sb is None:
            self.close()
            raise H5FormatError(f"{path}: no HDF5 signature")
        c = _Cursor(self, sb + 8)
        self.version = c.u8()
        if self.version in (0, 1):
            c.skip(4)  # free-space, root symtab, reserved, shared msg versions
            self.so, self.sl = c.u8(), c.u8()
            c.skip(1)
            c.skip(4 + 4)  # group K values, consistency flags
            if self.version == 1:
                c.skip(4)
            self.base = c.u(self.so)
            c.skip(3 * self.so)  # free space, EOF, driver info
            c.skip(self.so)  # root link name offset
            root = c.u(self.so) + self.base
        elif self.version in (2, 3):
            self.so, self.sl = c.u8(), c.u8()
            c.skip(1)
            self.base = c.u(self.so)
            c.skip(2 * self.so)  # superblock extension, EOF
            root = c.u(self.so) + self.base
        else:
            self.close()
            raise H5FormatError(f"{path}: superblock version {self.version}")
        self.root = Group(self, root, "/")

    def close(self):
        if getattr(self, "buf", None) is not None:
            self.buf.close()
            self.buf = None
        if self._fh:
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __getitem__(self, path):
        return self.root[path]

    def keys(self):
        return self.root.keys()

    @property
    def attrs(self):
        return self.root.attrs

    # -- object headers -----------------------------------------------------

    def messages(self, addr):
        """All messages of the object header at ``addr`` (continuations
        followed)."""
        out = []
        if self.buf[addr:addr + 4] == b"OHDR":
            c = _Cursor(self, addr + 4)
            ver = c.u8()
            if ver != 2:
                raise H5FormatError(f"OHDR version {ver}")
            flags = c.u8()
            if flags & 0x20:
                c.skip(16)
            if flags & 0x10:
                c.skip(4)
            size0 = c.u(1 << (flags & 3))
            self._v2_block(c.pos, c.pos + size0, flags, out)
        else:
            c = _Cursor(self, addr)
            ver = c.u8()
            if ver != 1:
                raise H5FormatError(f"object header version {ver} at {addr}")
            c.skip(1)
            nmsg = c.u16()
            c.skip(4)
            hsize = c.u32()
            c.skip(4)  # v1 header is padded to 16 bytes
            blocks = [(c.pos, hsize)]
            while blocks and len(out) < nmsg + 64:
                start, size = blocks.pop(0)
                p = start
                while p + 8 <= start + size:
                    mc = _Cursor(self, p)
                    mtype, msize = mc.u16(), mc.u16()
                    mc.skip(4)
                    if mtype == 0x10:
                        cc = _Cursor(self, mc.pos)
                        blocks.append((cc.off(), cc.length()))
                    else:
                        out.append(_Message(mtype, mc.pos, msize))
                    p = mc.pos + msize
        return out

    def _v2_block(self, start, end, flags, out):
        p = start
        hdr = 6 if flags & 0x04 else 4
        while end - p >= hdr:
            c = _Cursor(self, p)
            mtype = c.u8()
            msize = c.u16()
            mflags = c.u8()
            if flags & 0x04:
                c.skip(2)
            if mtype == 0x10:
                cc = _Cursor(self, c.pos)
                caddr, clen = cc.off(), cc.length()
                if self.buf[caddr:caddr + 4] != b"OCHK":
                    raise H5FormatError("bad OCHK")
                self._v2_block(caddr + 4, caddr + clen - 4, flags, out)
            elif mtype != 0:
                out.append(_Message(mtype, c.pos, msize))
            del mflags
            p = c.pos + msize

    def attributes(self, msgs):
        attrs = {}
        for m in msgs:
            if m.mtype == 0x0C:
                name, val = self._attribute(m.pos)
                attrs[name] = val
            elif m.mtype == 0x15:
                c = _Cursor(self, m.pos)
                c.skip(1)
                fl = c.u8()
                if fl & 1:
                    c.skip(2)
                heap = c.off()
                if heap != UNDEF:
                    _unsupported("dense attribute storage (fractal heap)")
        return attrs

    def _attribute(self, pos):
        c = _Cursor(self, pos)
        ver = c.u8()
        flags = c.u8()
        nlen, tlen, slen = c.u16(), c.u16(), c.u16()
        if ver >= 3:
            c.skip(1)  # name character set
        if flags & 3:
            _unsupported("shared datatype / dataspace in an attribute")
        name = bytes(self.buf[c.pos:c.pos + nlen]).split(b"\x00")[0].decode("utf8")
        c.pos += nlen if ver > 1 else nlen + (-nlen % 8)
        tpos = c.pos
        dt = _parse_datatype(_Cursor(self, tpos))
        c.pos = tpos + (tlen if ver > 1 else tlen + (-tlen % 8))
        spos = c.pos
        dims = _parse_dataspace(_Cursor(self, spos))
        c.pos = spos + (slen if ver > 1 else slen + (-slen % 8))
        if dims is None:
            return name, None
        n = int(np.prod(dims)) if dims else 1
        if isinstance(dt, _VlenString):
            vals = [self._vlen_string(c.pos + k * (4 + self.so + 4)) for k in range(n)]
            arr = np.array(vals, dtype=object).reshape(dims) if dims else vals[0]
            return name, arr
        raw = self.buf[c.pos:c.pos + n * dt.itemsize]
        arr = np.frombuffer(raw, dtype=dt, count=n).copy()
        if not dims:
            return name, arr[0]
        return name, arr.reshape(dims)

    def _vlen_string(self, pos):
        c = _Cursor(self, pos)
        length = c.u32()
        heap = c.off()
        index = c.u32()
        if length == 0 or heap == UNDEF:
            return ""
        return self._global_heap_object(heap, index)[:length].decode("utf8", "replace")

    def _global_heap_object(self, addr, index):
        if self.buf[addr:addr + 4] != b"GCOL":
            raise H5FormatError("bad global heap collection")
        c = _Cursor(self, addr + 8)
        size = c.length()
        end = addr + size
        while c.pos + 8 + self.sl <= end:
            idx = c.u16()
            c.skip(6)
            osize = c.length()
            if idx == 0:
                break
            if idx == index:
                return bytes(self.buf[c.pos:c.pos + osize])
            c.pos += osize + (-osize % 8)
        raise H5FormatError(f"global heap object {index} not found")

    # -- groups -----------------------------------------------------------

    def links(self, msgs):
        """name -> object header address for a group's header messages."""
        links = {}
        for m in msgs:
            if m.mtype == 0x11:  # symbol table
                c = _Cursor(self, m.pos)
                btree, heap = c.off(), c.off()
                self._symtab_links(btree, self._local_heap(heap), links)
            elif m.mtype == 0x06:  # link
                c = _Cursor(self, m.pos)
                c.skip(1)
                fl = c.u8()
                ltype = c.u8() if fl & 0x08 else 0
                if fl & 0x04:
                    c.skip(8)
                if fl & 0x10:
                    c.skip(1)
                nlen = c.u(1 << (fl & 3))
                name = c.raw(nlen).decode("utf8")
                if ltype == 0:
                    links[name] = c.off()
            elif m.mtype == 0x02:  # link info
                c = _Cursor(self, m.pos)
                c.skip(1)
                fl = c.u8()
                if fl & 1:
                    c.skip(8)
                heap = c.off()
                if heap != UNDEF:
                    _unsupported("dense link storage (fractal heap)")
        return links

    def _local_heap(self, addr):
        if self.buf[addr:addr + 4] != b"HEAP":
            raise H5FormatError("bad local heap")
        c = _Cursor(self, addr + 8)
        c.length()
        c.length()
        return c.off()

    def _heap_name(self, data, off):
        s = data + off
        return bytes(self.buf[s:self.buf.find(b"\x00", s)]).decode("utf8")

    def _symtab_links(self, node, heap, links):
        if self.buf[node:node + 4] == b"SNOD":
            c = _Cursor(self, node + 6)
            n = c.u16()
            for _ in range(n):
                name_off = c.u(self.so)
                addr = c.off()
                c.skip(8 + 16)
                links[self._heap_name(heap, name_off)] = addr
            return
        if self.buf[node:node + 4] != b"TREE":
            raise H5FormatError("bad group B-tree node")
        c = _Cursor(self, node + 4)
        ntype, _level, used = c.u8(), c.u8(), c.u16()
        if ntype != 0:
            raise H5FormatError("group B-tree of wrong type")
        c.skip(2 * self.so)
        for _ in range(used):
            c.length()  # key
            self._symtab_links(c.off(), heap, links)

    # -- chunked data ---------------------------------------------------------

    def chunks(self, node, ndim):
        """[(offsets, filter_mask, size, address)] of a v1 chunk B-tree."""
        out = []
        stack = [node]
        while stack:
            a = stack.pop()
            if self.buf[a:a + 4] != b"TREE":
                raise H5FormatError("bad chunk B-tree node")
            c = _Cursor(self, a + 4)
            ntype, level, used = c.u8(), c.u8(), c.u16()
            if ntype != 1:
                raise H5FormatError("chunk B-tree of wrong type")
            c.skip(2 * self.so)
            for _ in range(used):
                size = c.u32()
                mask = c.u32()
                offs = tuple(c.u(8) for _ in range(ndim + 1))[:ndim]
                child = c.off()
                if level == 0:
                    out.append((offs, mask, size, child))
                else:
                    stack.append(child)
        return out


def _unfilter(data, filters, mask, itemsize):
    for k in range(len(filters) - 1, -1, -1):
        if mask & (1 << k):
            continue
        fid, cd = filters[k]
        if fid == 1:
            data = zlib.decompress(data)
        elif fid == 2:
            n = len(data) // itemsize
            data = np.frombuffer(data, np.uint8, n * itemsize).reshape(
                itemsize, n).T.tobytes() + data[n * itemsize:]
        elif fid == 3:
            data = data[:-4]
        else:
            _unsupported(f"filter id {fid}")
        del cd
    return data


class _Node:
    def __init__(self, f, addr, name):
        self.file = f
        self.addr = addr
        self.name = name
        self._msgs = f.messages(addr)
        self._attrs = None

    @property
    def attrs(self):
        if self._attrs is None:
            self._attrs = self.file.attributes(self._msgs)
        return self._attrs


class Group(_Node):
    """An HDF5 group: ``keys()``, ``[name]`` (also "a/b/c" paths),
    ``attrs``."""

    def __init__(self, f, addr, name):
        super().__init__(f, addr, name)
        self._links = f.links(self._msgs)

    def keys(self):
        return list(self._links)

    def __contains__(self, name):
        try:
            self[name]
        except KeyError:
            return False
        return True

    def __iter__(self):
        return iter(self._links)

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, Group) or part not in node._links:
                raise KeyError(f"{path!r} not in {self.file.path}:{self.name}")
            addr = node._links[part]
            child = node.name.rstrip("/") + "/" + part
            msgs = self.file.messages(addr)
            is_ds = any(m.mtype == 0x08 for m in msgs)
            node = Dataset(self.file, addr, child) if is_ds else Group(self.file, addr, child)
        return node


class Dataset(_Node):
    """An HDF5 dataset: ``shape``, ``dtype``, ``attrs``, ``[()]`` /
    ``read()`` -> numpy array (native byte order)."""

    def __init__(self, f, addr, name):
        super().__init__(f, addr, name)
        self.shape = ()
        self.dtype = None
        self._layout = None
        self._filters = []
        for m in self._msgs:
            c = _Cursor(f, m.pos)
            if m.mtype == 0x01:
                self.shape = _parse_dataspace(c) or ()
            elif m.mtype == 0x03:
                self.dtype = _parse_datatype(c)
            elif m.mtype == 0x08:
                self._layout = m
            elif m.mtype == 0x0B:
                self._filters = self._parse_filters(c)
            elif m.mtype == 0x17:
                _unsupported("external data storage")

    @staticmethod
    def _parse_filters(c):
        ver = c.u8()
        n = c.u8()
        if ver == 1:
            c.skip(6)
        out = []
        for _ in range(n):
            fid = c.u16()
            nlen = c.u16() if (ver == 1 or fid >= 256) else 0
            c.u16()  # flags
            ncv = c.u16()
            if nlen:
                c.skip(nlen + ((-nlen % 8) if ver == 1 else 0))
            cd = [c.u32() for _ in range(ncv)]
            if ver == 1 and ncv % 2:
                c.skip(4)
            out.append((fid, cd))
        return out

    def __len__(self):
        return self.shape[0]

    @property
    def size(self):
        return int(np.prod(self.shape)) if self.shape else 1

    def __getitem__(self, key):
        return self.read()[key]

    def read(self):
        f = self.file
        dt = self.dtype
        if isinstance(dt, _VlenString):
            return self._read_vlen()
        n = self.size
        c = _Cursor(f, self._layout.pos)
        ver = c.u8()
        if ver not in (3, 4):
            _unsupported(f"data layout message version {ver}")
        cls = c.u8()
        if cls == 0:  # compact
            size = c.u16()
            raw = bytes(f.buf[c.pos:c.pos + size])
            arr = np.frombuffer(raw, dt, n)
        elif cls == 1:  # contiguous
            addr, size = c.off(), c.length()
            if addr == UNDEF:
                arr = np.zeros(n, dt)
            else:
                arr = np.frombuffer(f.buf, dt, n, addr)
        elif cls == 2:
            if ver != 3:
                _unsupported("layout v4 chunk indexes")
            ndim = c.u8()
            btree = c.off()
            cdims = [c.u32() for _ in range(ndim)][:-1]
            arr = self._read_chunked(btree, cdims)
        else:
            _unsupported(f"layout class {cls}")
        arr = np.array(arr).reshape(self.shape)
        return arr.astype(arr.dtype.newbyteorder("=")) if arr.dtype.byteorder == ">" else arr

    def _read_chunked(self, btree, cdims):
        f = self.file
        dt = self.dtype
        out = np.zeros(self.shape, dt)
        if btree == UNDEF:
            return out
        nd = len(self.shape)
        for offs, mask, size, addr in f.chunks(btree, nd):
            raw = bytes(f.buf[addr:addr + size])
            if self._filters:
                raw = _unfilter(raw, self._filters, mask, dt.itemsize)
            chunk = np.frombuffer(raw, dt, int(np.prod(cdims))).reshape(cdims)
            sl_out = tuple(slice(o, min(o + cd, s)) for o, cd, s in zip(offs, cdims, self.shape))
            sl_in = tuple(slice(0, s.stop - s.start) for s in sl_out)
            out[sl_out] = chunk[sl_in]
        return out

    def _read_vlen(self):
        f = self.file
        c = _Cursor(f, self._layout.pos)
        c.skip(1)
        if c.u8() != 1:
            _unsupported("non-contiguous variable-length dataset")
        addr = c.off()
        step = 4 + f.so + 4
        vals = [f._vlen_string(addr + k * step) for k in range(self.size)]
        return np.array(vals, dtype=object).reshape(self.shape)


# ===================================================================== writer

_K_LEAF, _K_NODE = 4, 16  # symbol-table node K values written in the superblock


def _pad8(b):
    return b + b"\x00" * (-len(b) % 8)


def _u(v, n):
    return int(v).to_bytes(n, "little")


def _enc_datatype(dt):
    """HDF5 datatype message body (version 1 encodings) for a numpy dtype."""
    dt = np.dtype(dt)
    if dt.subdtype is not None:
        _unsupported("top-level array datatype (use a compound member)")
    if dt.names:
        members = b""
        for name in dt.names:
            fdt, off = dt.fields[name][:2]
            base, shape = (fdt.subdtype if fdt.subdtype else (fdt, ()))
            if len(shape) > 4:
                _unsupported("compound member with more than 4 dims")
            dims = list(shape) + [0] * (4 - len(shape))
            members += _pad8(name.encode() + b"\x00")
            members += _u(off, 4) + _u(len(shape), 1) + b"\x00" * 3
            members += b"\x00" * 8 + b"".join(_u(d, 4) for d in dims)
            members += _enc_datatype(base)
        return bytes([0x16]) + _u(len(dt.names), 3) + _u(dt.itemsize, 4) + members
    order = 1 if dt.byteorder == ">" else 0
    if dt.kind == "f":
        spec = {2: (15, 10, 5, 10, 15), 4: (31, 23, 8, 23, 127),
                8: (63, 52, 11, 52, 1023)}[dt.itemsize]
        sign, eloc, esize, msize, bias = spec
        return (bytes([0x11, 0x20 | order, sign, 0]) + _u(dt.itemsize, 4)
                + _u(0, 2) + _u(8 * dt.itemsize, 2) + bytes([eloc, esize, 0, msize])
                + _u(bias, 4))
    if dt.kind in "iu":
        b0 = order | (0x08 if dt.kind == "i" else 0)
        return (bytes([0x10, b0, 0, 0]) + _u(dt.itemsize, 4) + _u(0, 2)
                + _u(8 * dt.itemsize, 2))
    if dt.kind == "S":
        return bytes([0x13, 0x01, 0, 0]) + _u(dt.itemsize, 4)  # null-padded ASCII
    _unsupported(f"writing dtype {dt}")


def _enc_dataspace(shape):
    if not shape:  # version 2 carries an explicit scalar type
        return bytes([2, 0, 0, 0])
    return (bytes([1, len(shape), 0, 0]) + b"\x00" * 4
            + b"".join(_u(d, 8) for d in shape))


def _as_array(value):
    a = np.asarray(value)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf8")
    if a.dtype.kind == "S" and a.dtype.itemsize == 0:
        a = a.astype("S1")
    if a.dtype.kind == "b":
        a = a.astype(np.uint8)
    if a.dtype.byteorder == ">" and a.dtype.kind in "fiu":
        a = a.astype(a.dtype.newbyteorder("<"))
    return a


class Writer:
    """Build a new HDF5 file (superblock v0, v1 object headers, symbol-table
    groups, contiguous datasets) -- the layout DP3 and PyTables files use, so
    PyTables, h5py and this module's reader all open it.

    ``w = Writer(); w.dataset("/sol000/phase000/val", arr, attrs={...});
    w.group_attrs("/sol000", {...}); w.save(path)``.
    """

    def __init__(self):
        self.tree = {"attrs": {}, "children": {}}

    def _node(self, path, create_group=True):
        node = self.tree
        for part in [p for p in path.split("/") if p]:
            ch = node["children"]
            if part not in ch:
                if not create_group:
                    raise KeyError(path)
                ch[part] = {"attrs": {}, "children": {}}
            node = ch[part]
        return node

    def group_attrs(self, path, attrs):
        self._node(path)["attrs"].update(attrs)

    def dataset(self, path, data, attrs=None):
        parent, _, name = path.rstrip("/").rpartition("/")
        node = self._node(parent)
        node["children"][name] = {"data": _as_array(data), "attrs": dict(attrs or {})}

    # -- serialisation ----------------------------------------------------

    def save(self, path):
        buf = bytearray(b"\x00" * 96)  # superblock, patched at the end

        def alloc(nbytes):
            buf.extend(b"\x00" * (-len(buf) % 8))
            addr = len(buf)
            buf.extend(b"\x00" * nbytes)
            return addr

        def put(addr, b):
            buf[addr:addr + len(b)] = b

        def header(messages):
            body = b""
            for mtype, data in messages:
                data = _pad8(data)
                body += _u(mtype, 2) + _u(len(data), 2) + b"\x00" * 4 + data
            hdr = (bytes([1, 0]) + _u(len(messages), 2) + _u(1, 4)
                   + _u(len(body), 4) + b"\x00" * 4)
            addr = alloc(len(hdr) + len(body))
            put(addr, hdr + body)
            return addr

        def attr_messages(attrs):
            out = []
            for name, value in attrs.items():
                a = _as_array(value)
                nm = name.encode() + b"\x00"
                dt = _enc_datatype(a.dtype)
                ds = _enc_dataspace(a.shape)
                msg = (bytes([1, 0]) + _u(len(nm), 2) + _u(len(dt), 2) + _u(len(ds), 2)
                       + _pad8(nm) + _pad8(dt) + _pad8(ds)
                       + np.asarray(a, order="C").tobytes())
                out.append((0x0C, msg))
            return out

        def write_dataset(node):
            a = np.asarray(node["data"], order="C")
            raw = a.tobytes()
            daddr = alloc(len(raw)) if raw else UNDEF
            if raw:
                put(daddr, raw)
            msgs = [(0x01, _enc_dataspace(a.shape)),
                    (0x03, _enc_datatype(a.dtype)),
                    (0x05, bytes([2, 1, 2, 0])),  # fill value: early alloc, never write
                    (0x08, bytes([3, 1]) + _u(daddr, 8) + _u(len(raw), 8))]
            return header(msgs + attr_messages(node["attrs"]))

        def write_group(node):
            names = sorted(node["children"])
            if len(names) > 2 * _K_LEAF * 2 * _K_NODE:
                _unsupported("group with more than 256 members")
            kids = {}
            for n in names:
                ch = node["children"][n]
                kids[n] = write_dataset(ch) if "data" in ch else write_group(ch)[0]
            # local heap: "" at offset 0, then the names (8-byte padded)
            heap_data = bytearray(b"\x00" * 8)
            offs = {}
            for n in names:
                offs[n] = len(heap_data)
                heap_data += _pad8(n.encode() + b"\x00")
            heap_data += b"\x00" * max(0, 16 - len(heap_data))  # non-trivial segment
            seg = alloc(len(heap_data))
            put(seg, bytes(heap_data))
            heap = alloc(32)
            # free-list head 1 = "no free block" (the library's H5HL_FREE_NULL)
            put(heap, b"HEAP" + bytes([0, 0, 0, 0]) + _u(len(heap_data), 8)
                + _u(1, 8) + _u(seg, 8))
            # symbol-table leaves of at most 2K entries, one level-0 B-tree node
            leaves = [names[i:i + 2 * _K_LEAF] for i in range(0, len(names), 2 * _K_LEAF)] or [[]]
            snods = []
            for leaf in leaves:
                ent = b""
                for n in leaf:
                    ent += _u(offs[n], 8) + _u(kids[n], 8) + b"\x00" * 24
                a = alloc(8 + 2 * _K_LEAF * 40)
                put(a, b"SNOD" + bytes([1, 0]) + _u(len(leaf), 2) + ent)
                snods.append((a, leaf))
            tree = alloc(24 + (2 * _K_NODE + 1) * 8 + 2 * _K_NODE * 8)
            body = b"TREE" + bytes([0, 0]) + _u(len(snods) if names else 0, 2)
            body += _u(UNDEF, 8) + _u(UNDEF, 8) + _u(0, 8)
            if names:
                for a, leaf in snods:
                    body += _u(a, 8) + _u(offs[leaf[-1]], 8)
            put(tree, body)
            msgs = [(0x11, _u(tree, 8) + _u(heap, 8))]
            return header(msgs + attr_messages(node["attrs"])), tree, heap

        root, rtree, rheap = write_group(self.tree)
        sb = (SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + _u(_K_LEAF, 2)
              + _u(_K_NODE, 2) + _u(0, 4) + _u(0, 8) + _u(UNDEF, 8)
              + _u(len(buf), 8) + _u(UNDEF, 8)
              + _u(0, 8) + _u(root, 8) + _u(1, 4) + _u(0, 4) + _u(rtree, 8) + _u(rheap, 8))
        put(0, sb)
        with open(path, "wb") as fh:
            fh.write(bytes(buf))

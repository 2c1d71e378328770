"""ctypes binding of libscreenfit.so (the C ABI declared in include/screenfit.h).

There is no fallback: if the library is missing or no gfx950 device is
usable, every compute entry point raises :class:`ScreenFitError`.
"""

import contextlib
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCREENFIT_LIB", os.path.join(_HERE, "libscreenfit.so"))

SF_SCREEN_PHASE = 0
SF_SCREEN_TEC = 1
SF_SCREEN_AMPLITUDE = 2
SF_EVAL_NAN_SCRUB = 1
SF_EVAL_FAST_SINCOS = 1 << 8
SF_EVAL_NT_STORES = 1 << 9
SF_EVAL_BIG_ENDIAN = 1 << 10
SF_MAX_DIR = 60
SF_OPT_FIT_GENERAL = 1
SF_OPT_EVAL_KERNEL = 2
SF_OPT_EVAL_MAX_BLOCKS = 3
SF_OPT_FIT_PACK = 4
SF_OPT_EVAL_KS_PAD = 5
SF_OPT_EVAL_SLEEP = 6
SF_OPT_EVAL_XCD_MAP = 7
SF_OPT_EVAL_GROUPS = 8
SF_OPT_EVAL_BANDS = 9
SF_OPT_FIT_LEAN = 10
SF_OPT_TESS_SLOTS = 11
SF_OPT_TESS_WAVES = 12
SF_OPT_TESS_TILE = 13
SF_OPT_TESS_BOX = 14
SF_OPT_EVAL_INT = 15
SF_OPT_EVAL_WG_WAVES = 16
SF_OPT_FIT_EIG_WAVES = 17
SF_OPT_FIT_SUBSET_DELETION = 18
SF_EVAL_KERNEL_AUTO = 0
SF_EVAL_KERNEL_TILE = 1
SF_EVAL_KERNEL_LDS4 = 2
SF_EVAL_KERNEL_LDS8 = 3
SF_EVAL_KERNEL_LDS16 = 4
SF_EVAL_KERNEL_LDS8H = 5
SF_EVAL_KERNEL_LDS16H = 6
SF_EVAL_KERNEL_TILE3 = 7
SF_EVAL_KERNEL_SHB = 8
EVAL_KERNEL_NAMES = {SF_EVAL_KERNEL_TILE: "kl_eval_kernel",
                     SF_EVAL_KERNEL_LDS4: "kl_eval_lds_kernel<4 waves>",
                     SF_EVAL_KERNEL_LDS8: "kl_eval_lds_kernel<8 waves>",
                     SF_EVAL_KERNEL_LDS16: "kl_eval_lds_kernel<16 waves>",
                     SF_EVAL_KERNEL_LDS8H: "kl_eval_lds_kernel<8 waves, 2 tiles>",
                     SF_EVAL_KERNEL_LDS16H: "kl_eval_lds_kernel<16 waves, 2 tiles>",
                     SF_EVAL_KERNEL_TILE3: "kl_eval_kernel<3 waves/SIMD>",
                     SF_EVAL_KERNEL_SHB: "kl_eval_kernel<Cpix in LDS>"}

# every symbol include/screenfit.h declares (checked by tests/test_capi.py)
EXPORTED = (
    "sf_version", "sf_last_error", "sf_create", "sf_destroy", "sf_set_stream",
    "sf_synchronize", "sf_set_option", "sf_get_eval_kernel", "sf_get_eval_contraction", "sf_alloc", "sf_free", "sf_copy_h2d", "sf_copy_d2h",
    "sf_set_basis", "sf_get_basis", "sf_kl_fit", "sf_get_fit_stats", "sf_get_fit_pool",
    "sf_stream_create", "sf_stream_destroy", "sf_device_cus",
    "sf_set_grid", "sf_kl_eval", "sf_kl_eval_gain", "sf_kl_eval_sums",
    "sf_tess_fill", "sf_smooth",
)


_identity = {}


def library_identity(path=None):
    """sha256 (first 16 hex digits) and size of the library file this
    process loads: the key the measurement tables under profiles/ carry, so
    counters taken on another build are not reported as this one's."""
    import hashlib
    p = os.path.realpath(path or LIB_PATH)
    if p not in _identity:
        h = hashlib.sha256()
        with open(p, "rb") as fh:
            for blk in iter(lambda: fh.read(1 << 20), b""):
                h.update(blk)
        _identity[p] = {"sha16": h.hexdigest()[:16], "bytes": os.path.getsize(p)}
    return dict(_identity[p])


class ScreenFitError(RuntimeError):
    """Raised for any failure of the HIP library (including its absence)."""


class FitParams(ctypes.Structure):
    _fields_ = [("screen_type", ctypes.c_int), ("niter", ctypes.c_int),
                ("nsigma", ctypes.c_double), ("adjust_order", ctypes.c_int),
                ("ref_ant", ctypes.c_int), ("ant_offset", ctypes.c_int),
                ("ref_phase", ctypes.c_void_p)]


_lib = None
_lib_lock = threading.Lock()


def load_library(path=None):
    """Load (once) and return the ctypes handle of libscreenfit.so."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ScreenFitError(
                f"libscreenfit.so not found at {p}: build it with "
                "`make -C ska-sdp-screen-fitting_amd/csrc` (or "
                "__graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(p)
        vp, ip, c_int, c_dbl = (ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                ctypes.c_int, ctypes.c_double)
        i64 = ctypes.c_int64
        sig = {
            "sf_version": ([], ctypes.c_char_p),
            "sf_last_error": ([], ctypes.c_char_p),
            "sf_create": ([c_int, ctypes.POINTER(vp)], c_int),
            "sf_destroy": ([vp], c_int),
            "sf_set_stream": ([vp, vp], c_int),
            "sf_synchronize": ([vp], c_int),
            "sf_set_option": ([vp, c_int, c_int], c_int),
            "sf_get_eval_kernel": ([vp, c_int, ctypes.c_uint, ip], c_int),
            "sf_get_eval_contraction": ([vp, c_int, ctypes.c_uint, ip], c_int),
            "sf_alloc": ([vp, ctypes.c_size_t, ctypes.POINTER(vp)], c_int),
            "sf_free": ([vp, vp], c_int),
            "sf_copy_h2d": ([vp, vp, vp, ctypes.c_size_t], c_int),
            "sf_copy_d2h": ([vp, vp, vp, ctypes.c_size_t], c_int),
            "sf_set_basis": ([vp, vp, c_int, c_dbl, c_dbl], c_int),
            "sf_get_basis": ([vp, vp, vp, vp, vp], c_int),
            "sf_kl_fit": ([vp, vp, vp, c_int, c_int, c_int, ip,
                           ctypes.POINTER(FitParams), vp, vp, vp, vp], c_int),
            "sf_get_fit_stats": ([vp, ip, ip], c_int),
            "sf_get_fit_pool": ([vp, vp, vp, c_int, ip], c_int),
            "sf_set_grid": ([vp, vp, c_int, vp, c_int], c_int),
            "sf_kl_eval": ([vp, vp, i64, vp, i64, ctypes.c_uint], c_int),
            "sf_stream_create": ([vp, ctypes.POINTER(c_int), c_int,
                                  ctypes.POINTER(vp)], c_int),
            "sf_stream_destroy": ([vp, vp], c_int),
            "sf_device_cus": ([vp, ctypes.POINTER(c_int)], c_int),
            "sf_kl_eval_gain": ([vp, vp, vp, vp, i64, vp, i64, ctypes.c_uint],
                                c_int),
            "sf_kl_eval_sums": ([vp, vp, vp, vp, i64, vp, i64, ctypes.c_uint, vp],
                                c_int),
            "sf_tess_fill": ([vp, vp, c_int, c_int, vp, vp, vp, c_int, i64, vp,
                              i64, c_dbl, ctypes.c_uint], c_int),
            "sf_smooth": ([vp, vp, c_int, c_int, i64, c_dbl, ctypes.c_uint], c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if path is None:
            _lib = lib
        return lib


def _check(rc, what):
    if rc != 0:
        msg = load_library().sf_last_error().decode(errors="replace")
        raise ScreenFitError(f"{what} failed ({rc}): {msg}")


_TORCH_DTYPES = {np.float64: "torch.float64", np.float32: "torch.float32",
                 np.int32: "torch.int32", np.int64: "torch.int64"}


def _dev(x, dtype, numel, name, device=None):
    """Pointer of a device operand after checking what the kernels assume:
    a contiguous CUDA tensor of ``dtype`` with at least ``numel`` elements on
    the context's ``device`` (a short, mistyped or foreign-device buffer would
    be overrun or dereferenced by the wrong GPU).  Raw integer pointers are
    the caller's responsibility."""
    if x is None or isinstance(x, int):
        return x
    if not hasattr(x, "data_ptr"):
        raise TypeError(f"{name}: expected a device tensor, got {type(x).__name__}")
    if not x.is_cuda:
        raise ValueError(f"{name}: must be a device (cuda) tensor")
    if device is not None and x.device.index != device:
        raise ValueError(f"{name}: on cuda:{x.device.index}, the context is on "
                         f"cuda:{device}")
    if str(x.dtype) != _TORCH_DTYPES[dtype]:
        raise TypeError(f"{name}: dtype {x.dtype}, expected {_TORCH_DTYPES[dtype]}")
    if not x.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if x.numel() < numel:
        raise ValueError(f"{name}: {x.numel()} elements, the call needs {numel}")
    return x.data_ptr()


class Context:
    """One sf_ctx bound to one device.  Methods mirror the C ABI."""

    def __init__(self, device=0):
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        _check(self.lib.sf_create(device, ctypes.byref(h)), "sf_create")
        self.h = h
        self.D = 0
        self.grid = None
        self.options = {}  # sf_set_option values set through this object

    def close(self):
        if self.h:
            self.lib.sf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, x, dtype, numel, name):
        return _dev(x, dtype, numel, name, self.device)

    def set_stream(self, stream_handle):
        _check(self.lib.sf_set_stream(self.h, stream_handle), "sf_set_stream")

    def set_option(self, option, value):
        _check(self.lib.sf_set_option(self.h, int(option), int(value)),
               "sf_set_option")
        self.options[int(option)] = int(value)

    def eval_kernel(self, flags, gain=False):
        """Name of the evaluation kernel sf_kl_eval runs for these flags
        (with the workgroup width when SF_OPT_EVAL_WG_WAVES = 8 takes effect:
        the integer-digit contraction on the register tile only)."""
        k = ctypes.c_int()
        _check(self.lib.sf_get_eval_kernel(self.h, int(bool(gain)), int(flags),
                                           ctypes.byref(k)), "sf_get_eval_kernel")
        name = EVAL_KERNEL_NAMES[k.value]
        if (self.options.get(SF_OPT_EVAL_WG_WAVES, 0) == 8
                and k.value in (SF_EVAL_KERNEL_TILE, SF_EVAL_KERNEL_TILE3)
                and self.eval_contraction(flags, gain) == "i8-digits"):
            name += " (8-wave workgroups)"
        return name

    def eval_contraction(self, flags, gain=False):
        """'f64' (fp64 MFMAs) or 'i8-digits' (the integer-digit contraction)
        for the evaluation sf_kl_eval runs with these flags."""
        k = ctypes.c_int()
        _check(self.lib.sf_get_eval_contraction(self.h, int(bool(gain)), int(flags),
                                                ctypes.byref(k)), "sf_get_eval_contraction")
        return "i8-digits" if k.value == 1 else "f64"

    def synchronize(self):
        _check(self.lib.sf_synchronize(self.h), "sf_synchronize")

    def set_basis(self, pp, r0=100.0, beta=5.0 / 3.0):
        pp = np.ascontiguousarray(pp, dtype=np.float64)
        assert pp.ndim == 2 and pp.shape[1] == 3
        _check(self.lib.sf_set_basis(self.h, pp.ctypes.data, pp.shape[0],
                                     float(r0), float(beta)), "sf_set_basis")
        self.D = pp.shape[0]
        self.grid = None

    def get_basis(self):
        D = self.D
        c, pinv, u = (np.empty((D, D)) for _ in range(3))
        eig = np.empty(D)
        _check(self.lib.sf_get_basis(self.h, c.ctypes.data, pinv.ctypes.data,
                                     u.ctypes.data, eig.ctypes.data),
               "sf_get_basis")
        return c, pinv, u, eig

    def fit(self, phase, weight, T, F, A, station_order, screen_type=0,
            niter=2, nsigma=5.0, adjust_order=True, ref_ant=-1, coef=None,
            resid=None, w_out=None, order_out=None, ant_offset=0,
            ref_phase=None):
        """sf_kl_fit on device buffers (torch tensors or raw pointers)."""
        so = np.ascontiguousarray(station_order, dtype=np.int32)
        if so.shape != (A,):
            raise ValueError(f"station_order: shape {so.shape}, expected ({A},)")
        n = int(T) * int(F) * int(A) * self.D
        prm = FitParams(int(screen_type), int(niter), float(nsigma),
                        int(bool(adjust_order)), int(ref_ant), int(ant_offset),
                        self._dev(ref_phase, np.float64, int(T) * int(F) * self.D,
                             "ref_phase"))
        _check(self.lib.sf_kl_fit(
            self.h, self._dev(phase, np.float64, n, "phase"),
            self._dev(weight, np.float32, n, "weight"), int(T), int(F), int(A),
            so.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
            ctypes.byref(prm), self._dev(coef, np.float64, n, "coef"),
            self._dev(resid, np.float64, n, "resid"),
            self._dev(w_out, np.float32, n, "w_out"),
            self._dev(order_out, np.int32, n // max(self.D, 1), "order_out")),
            "sf_kl_fit")

    def fit_stats(self):
        nm, ng = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.sf_get_fit_stats(self.h, ctypes.byref(nm), ctypes.byref(ng)),
               "sf_get_fit_stats")
        return {"n_masks": nm.value, "n_general": ng.value}

    def fit_pool(self):
        """The subset bases decomposed so far (sf_get_fit_pool), sorted by
        mask: (masks uint64 [n], entries float64 [n][D*D + D])."""
        n = ctypes.c_int(0)
        _check(self.lib.sf_get_fit_pool(self.h, None, None, 0, ctypes.byref(n)),
               "sf_get_fit_pool")
        D = self.D
        masks = np.zeros(n.value, np.uint64)
        ent = np.zeros((n.value, D * D + D))
        if n.value:
            _check(self.lib.sf_get_fit_pool(self.h, masks.ctypes.data, ent.ctypes.data,
                                            n.value, ctypes.byref(n)), "sf_get_fit_pool")
        order = np.argsort(masks, kind="stable")
        masks, ent = masks[order], ent[order]
        # only the leading n x n block and n eigenvalues of an n-direction
        # mask are written; the rest of the entry is stale scratch
        for k, m in enumerate(masks):
            n = bin(int(m)).count("1")
            u = ent[k, :D * D].reshape(D, D)
            u[n:, :] = 0.0
            u[:, n:] = 0.0
            ent[k, D * D + n:] = 0.0
        return masks, ent

    def set_grid(self, x, y):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        _check(self.lib.sf_set_grid(self.h, x.ctypes.data, x.size,
                                    y.ctypes.data, y.size), "sf_set_grid")
        self.grid = (x.size, y.size)

    def _out_numel(self, S, ring):
        nx, ny = self.grid if self.grid else (0, 0)
        return min(int(S), ring) * 4 * nx * ny

    def eval(self, coef, S, out, ring_slots=None,
             flags=SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES):
        ring = max(int(S if ring_slots is None else ring_slots), 1)
        _check(self.lib.sf_kl_eval(
            self.h, self._dev(coef, np.float64, int(S) * self.D, "coef"), int(S),
            self._dev(out, np.float32, self._out_numel(S, ring), "out"), ring,
            int(flags)), "sf_kl_eval")


    def device_cus(self):
        n = ctypes.c_int(0)
        _check(self.lib.sf_device_cus(self.h, ctypes.byref(n)), "sf_device_cus")
        return n.value

    def stream_create(self, reserve_cus=()):
        """Raw HIP stream (int handle) whose kernels avoid ``reserve_cus``;
        wrap with ``torch.cuda.ExternalStream``."""
        arr = (ctypes.c_int * max(1, len(reserve_cus)))(*reserve_cus)
        out = ctypes.c_void_p()
        _check(self.lib.sf_stream_create(self.h, arr, len(reserve_cus),
                                         ctypes.byref(out)), "sf_stream_create")
        return out.value

    def stream_destroy(self, stream):
        _check(self.lib.sf_stream_destroy(self.h, ctypes.c_void_p(stream)),
               "sf_stream_destroy")

    def eval_gain(self, coef_ph, coef_xx, coef_yy, S, out, ring_slots=None,
                  flags=SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES):
        ring = max(int(S if ring_slots is None else ring_slots), 1)
        n = int(S) * self.D
        _check(self.lib.sf_kl_eval_gain(
            self.h, self._dev(coef_ph, np.float64, n, "coef_ph"),
            self._dev(coef_xx, np.float64, n, "coef_xx"),
            self._dev(coef_yy, np.float64, n, "coef_yy"), int(S),
            self._dev(out, np.float32, self._out_numel(S, ring), "out"), ring,
            int(flags)), "sf_kl_eval_gain")

    def eval_sums(self, coef, S, out, sums, ring_slots=None, coef_xx=None,
                  coef_yy=None,
                  flags=SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES):
        """sf_kl_eval_sums: evaluate (phase, or gain with coef_xx / coef_yy)
        and add (mod 2^32) each slot's output checksum -- the sum mod 2^32 of
        its stored 32-bit words -- to ``sums`` (int32 device tensor of >= S
        elements, zeroed by the caller; int32 holds the uint32 bits)."""
        ring = max(int(S if ring_slots is None else ring_slots), 1)
        n = int(S) * self.D
        _check(self.lib.sf_kl_eval_sums(
            self.h, self._dev(coef, np.float64, n, "coef"),
            self._dev(coef_xx, np.float64, n, "coef_xx"),
            self._dev(coef_yy, np.float64, n, "coef_yy"), int(S),
            self._dev(out, np.float32, self._out_numel(S, ring), "out"), ring,
            int(flags), self._dev(sums, np.int32, int(S), "sums")), "sf_kl_eval_sums")

    def tess_fill(self, labels, nx, ny, phase, D, S, out, ring_slots=None,
                  amp_xx=None, amp_yy=None, smooth_pix=0.0,
                  flags=SF_EVAL_NAN_SCRUB):
        ring = max(int(S if ring_slots is None else ring_slots), 1)
        n = int(S) * int(D)
        if hasattr(labels, "min") and labels.numel():
            # validated once per label tensor OBJECT (held by a weak
            # reference, so a new tensor in the freed storage of the old one
            # is validated again), its in-place version and D: every chunk of
            # a Screen.write passes the same template, and min / max are two
            # reductions + two host syncs
            import weakref
            prev = getattr(self, "_labels_ok", None)
            key = (labels._version, int(D))
            if prev is None or prev[0]() is not labels or prev[1] != key:
                lo, hi = int(labels.min()), int(labels.max())
                if lo < 1 or hi > int(D):
                    raise ValueError(f"labels: values {lo}..{hi} outside 1..{D}")
                self._labels_ok = (weakref.ref(labels), key)
        _check(self.lib.sf_tess_fill(
            self.h, self._dev(labels, np.int32, int(nx) * int(ny), "labels"),
            int(nx), int(ny), self._dev(phase, np.float64, n, "phase"),
            self._dev(amp_xx, np.float64, n, "amp_xx"),
            self._dev(amp_yy, np.float64, n, "amp_yy"), int(D), int(S),
            self._dev(out, np.float32, min(int(S), ring) * 4 * int(nx) * int(ny), "out"),
            ring, float(smooth_pix), int(flags)), "sf_tess_fill")


    def smooth(self, cube, nx, ny, n_img, smooth_pix, flags=0):
        """sf_smooth: Screen.write's Gaussian in place on n_img float32
        images [n_img][ny][nx] (n_img = 4 x slots), scrub / byte swap in
        ``flags`` applied after smoothing."""
        _check(self.lib.sf_smooth(
            self.h, self._dev(cube, np.float32, int(n_img) * int(nx) * int(ny), "cube"),
            int(nx), int(ny), int(n_img), float(smooth_pix), int(flags)), "sf_smooth")


_contexts = {}
_ctx_lock = threading.Lock()


def get_context(device=0):
    """Process-wide context per device (bound to torch's current stream by
    the callers that use torch).  Its basis, grid, options and scratch are
    shared by every holder: for a single-threaded caller (the bench, the
    tests) -- the product paths take a ``private_context`` instead."""
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
    return ctx


_idle = {}
# idle contexts kept per device (more are closed: a context keeps the device
# scratch of the largest call it ran)
_IDLE_MAX = 4


@contextlib.contextmanager
def private_context(device=0):
    """A context this block holds alone: taken from the device's idle list
    (or created) and returned to it on exit, so a caller's set_basis / fit /
    tess_fill sequence never sees a basis, grid or scratch buffer another
    thread set meanwhile.  The reference's counterpart is its module-global
    state per worker process (stationscreen.py:918-919, kl_screen.py:223-226);
    there one screen at a time per process, here any number of threads, one
    context each while they run (at most as many contexts as ever ran
    concurrently)."""
    with _ctx_lock:
        idle = _idle.setdefault(device, [])
        ctx = idle.pop() if idle else None
    if ctx is None:
        ctx = Context(device)
    try:
        yield ctx
    finally:
        with _ctx_lock:
            keep = len(_idle[device]) < _IDLE_MAX
            if keep:
                _idle[device].append(ctx)
        if not keep:
            ctx.close()  # sf_destroy: hipFree waits for the device

/*
 * screenfit.h -- C ABI of the MI355X-native KL a-term screen library
 * (libscreenfit.so, hand-written HIP for gfx950).
 *
 * Drop-in boundary for the hot path of ska-sdp-screen-fitting v0.1.0
 * (reference at /root/reference, paths below relative to
 * src/ska_sdp_screen_fitting/).  The reference is pure Python with no FFI;
 * each entry point names the Python interface it replaces:
 *
 *   sf_set_basis  <- stationscreen._calculate_piercepoints / _calculate_svd
 *                    (stationscreen.py:70-110, 390-430; run :1046-1053)
 *   sf_kl_fit     <- stationscreen.run -> _process_single_freq ->
 *                    _process_station -> _fit_screen
 *                    (stationscreen.py:858-1161, 785-855, 597-782, 433-594)
 *   sf_set_grid   <- KLScreen.make_matrix coordinate block
 *                    (kl_screen.py:228-261)
 *   sf_kl_eval    <- KLScreen.make_matrix + calculate_kl_screen + the NaN
 *                    scrub of Screen.write (kl_screen.py:192-449,
 *                    screen.py:343-378)
 *
 * Conventions
 *  - Plain C types only.  Return 0 on success, a negative errno-style code
 *    on failure (SF_EINVAL bad shape/argument, SF_ENOMEM, SF_EIO HIP
 *    failure, SF_ENODEV no usable gfx950 device); sf_last_error() gives a
 *    thread-local message.
 *  - Array arguments of sf_kl_fit / sf_kl_eval are DEVICE pointers (HBM,
 *    e.g. from sf_alloc or any HIP allocator); small geometry arrays
 *    (piercepoints, grid coordinates, per-station orders) are HOST pointers.
 *    The caller owns every buffer it passes; the library never frees caller
 *    memory.  Device scratch (basis, pixel matrix) is owned by the context.
 *  - Work is enqueued on the context's stream (sf_set_stream); calls return
 *    once enqueued except sf_set_basis/sf_get_basis/sf_copy_* which
 *    synchronise.  Calls on one context must be serialised by the caller;
 *    contexts on different devices may be driven from different threads.
 *  - Slot layout is the H5parm scalarphase layout [time][freq][ant][dir]
 *    (stationscreen.py:936-963, kl_screen.py:269-272): slot index
 *    s = (t * F + f) * A + a.  The evaluated cube is the FITS a-term cube
 *    layout [time][freq][ant][4][y][x] (screen.py:319-351), native-endian
 *    float32, planes (Re XX, Im XX, Re YY, Im YY).
 */
#ifndef SCREENFIT_H
#define SCREENFIT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SF_OK 0
#define SF_EINVAL (-22)
#define SF_ENOMEM (-12)
#define SF_EIO (-5)
#define SF_ENODEV (-19)

#define SF_MAX_DIR 60 /* directions per slot (one wavefront lane each; LDS-bound) */

/* screen types of stationscreen.run (stationscreen.py:922-928) */
#define SF_SCREEN_PHASE 0
#define SF_SCREEN_TEC 1
#define SF_SCREEN_AMPLITUDE 2 /* log10 fit; sigma per station block (Q6) */

/* sf_kl_eval flags */
#define SF_EVAL_NAN_SCRUB 1u /* NaN -> 1 (real planes), 0 (imag) (screen.py:368-378) */
#define SF_EVAL_FAST_SINCOS (1u << 8) /* exact fp64 reduction of the phase in
                                         revolutions + hardware fp32 sincos
                                         (|err| <= 2.3e-7) instead of fp64
                                         sincos */
#define SF_EVAL_NT_STORES (1u << 9) /* non-temporal (streaming) cube stores */
#define SF_EVAL_BIG_ENDIAN (1u << 10) /* store big-endian float32 (the FITS
                                         byte order), for direct file writes */

typedef struct sf_ctx sf_ctx;

/* Operator parameters of stationscreen.run (stationscreen.py:858-871). */
typedef struct sf_fit_params {
  int screen_type;  /* SF_SCREEN_PHASE, _TEC or _AMPLITUDE */
  int niter;        /* outlier-flagging iterations (phase: 2) */
  double nsigma;    /* outlier threshold in circular sigmas (5.0) */
  int adjust_order; /* adapt the order toward reduced chi^2 ~ 1 (1) */
  int ref_ant;      /* GLOBAL reference station index, -1 = none */
  int ant_offset;   /* global index of this call's station 0 (ant shards) */
  const double* ref_phase; /* device [T][F][D] phases of the reference
                              station when it is not in this shard; NULL =
                              read them from station ref_ant - ant_offset */
} sf_fit_params;

/* Library / device management */
const char* sf_version(void);
const char* sf_last_error(void);
int sf_create(int device, sf_ctx** out);
int sf_destroy(sf_ctx* ctx);
int sf_set_stream(sf_ctx* ctx, void* hip_stream); /* NULL = default stream */
int sf_synchronize(sf_ctx* ctx);
/* A HIP stream whose kernels may only use the compute units NOT listed in
 * reserve_cus (CU indices 0..n_cu-1; the reserved units stay free for work
 * on other streams, e.g. the fit of the next time chunk while the current
 * chunk is evaluated).  n_reserve = 0 gives an ordinary stream. */
int sf_stream_create(sf_ctx* ctx, const int* reserve_cus, int n_reserve,
                     void** hip_stream);
int sf_stream_destroy(sf_ctx* ctx, void* hip_stream);
int sf_device_cus(sf_ctx* ctx, int* n_cu);
/* Options: SF_OPT_FIT_GENERAL = 1 routes every slot through the general
 * (per-slot Jacobi) fit kernel instead of the mask-cached eigenbasis
 * pipeline; both give the reference's results (used to cross-check). */
#define SF_OPT_FIT_GENERAL 1
/* SF_OPT_EVAL_KERNEL selects the evaluation kernel of sf_kl_eval (all give
 * the same values): AUTO (default), TILE = register-tile stores (4 slots x
 * 256 B per store instruction; always used for fp64 sincos and gain
 * screens), LDS4 / LDS8 / LDS16 = LDS-staged stores with 1 / 2 / 4 KiB
 * contiguous runs per (slot, plane). */
#define SF_OPT_EVAL_KERNEL 2
/* SF_OPT_EVAL_MAX_BLOCKS caps the workgroups of an evaluation launch (0 =
 * the dispatch limit); each workgroup then walks several (pixel block, slot
 * chunk) items.  For tests of that walk. */
#define SF_OPT_EVAL_MAX_BLOCKS 3
/* SF_OPT_FIT_PACK = 0 runs one slot per wavefront in the fit also for
 * D <= 32 (default 1: two slots per wavefront; same results bit for bit). */
#define SF_OPT_FIT_PACK 4
/* SF_OPT_EVAL_KS_PAD = n (0..3) runs the evaluation contraction with n extra
 * all-zero k-steps of 4 directions (same values; tuning / diagnostics). */
#define SF_OPT_EVAL_KS_PAD 5
/* SF_OPT_EVAL_SLEEP = n: LDS-staged evaluation waves sleep n x 64 cycles
 * after each 16-slot contraction (store-throttling experiments; default 0). */
#define SF_OPT_EVAL_SLEEP 6
/* SF_OPT_EVAL_XCD_MAP: workgroup -> pixel-block map of the evaluation
 * kernels.  0: XCD x (workgroups are dealt round-robin over the 8 XCDs)
 * takes a contiguous eighth of the pixel blocks; 1: XCD x takes the pixel
 * blocks pb = x (mod 8); -1 (default): 1 when an XCD's eighth is at most 8
 * pixel blocks (256^2 with 4 KiB runs: +2-3 % measured), else 0. */
#define SF_OPT_EVAL_XCD_MAP 7
/* SF_OPT_EVAL_GROUPS = g (1..256, power of two; 0 = auto: 64 for the
 * register-tile kernels, 16 for the LDS-staged ones): most 16-slot groups per
 * evaluation work item (each item loads its pixel block's basis once, so
 * longer items re-read less of it). */
#define SF_OPT_EVAL_GROUPS 8
/* SF_OPT_EVAL_BANDS = b (1..128, power of two; 0 = auto): the evaluation
 * runs its work items band-major over b pixel bands (every slot chunk of the
 * first 1/b of the pixel blocks, then the next ...), so each XCD's live slice
 * of the pixel basis is 1/b of its share.  Auto: bands of 128 pixel blocks
 * (with the interleaved XCD map) for the register-tile kernels on grids of
 * >= 1024 blocks (512^2 and up), else 1.  Ignored where the pixel blocks of a
 * band would not divide by 8.  Outputs are identical for every b. */
#define SF_OPT_EVAL_BANDS 9
/* SF_OPT_FIT_LEAN = 0 / 1 (default 1): when every slot's unflagged weights
 * are equal (counted by the classify kernel), the fit passes run a variant
 * with no per-slot normal-matrix / subset-basis copies in LDS (flagged slots
 * read their subset basis from the pool), for 2.7-4x the resident waves.
 * Same results bit for bit; 0 forces the general layout. */
#define SF_OPT_FIT_LEAN 10
/* SF_OPT_TESS_SLOTS = n (0 = auto 16, else 1..256): slots per work item of
 * the unsmoothed tessellated fill (the item's value-table slice sits in
 * LDS); SF_OPT_TESS_WAVES = 4, 8 or 16 (0 = auto 16): its waves per
 * workgroup, each writing whole 4 KiB runs of its own slots.  Outputs are
 * identical for every setting. */
#define SF_OPT_TESS_SLOTS 11
#define SF_OPT_TESS_WAVES 12
/* SF_OPT_TESS_TILE = 1 runs sf_tess_fill (radius <= 24) on the round-1 fused
 * 16 x 16 tile kernel instead of the table + gather / wide-tile smoothing
 * kernels (same bits; for cross-checks). */
#define SF_OPT_TESS_TILE 13
/* SF_OPT_TESS_BOX = 1: sf_tess_fill with smoothing (radius <= 24) stores
 * the pixels whose whole (2R + 1)^2 neighbourhood is one cell from a
 * per-(slot, cell) value and sums only the others (kl_tess_box_kernel); 0:
 * the wide-tile kernel that sums every pixel; -1 (default): the first for
 * four planes (XX / YY amplitudes) at radius <= 5, else the second.  Same
 * bits. */
#define SF_OPT_TESS_BOX 14
/* SF_OPT_EVAL_INT = 0 evaluates with the fp64 MFMA contraction everywhere;
 * -1 (default): the integer-digit contraction -- Cpix and the coefficients
 * as 6 balanced base-256 digits of 36- / 44-bit fixed point, contracted
 * exactly on i8 MFMAs (64x the fp64 MFMA rate per product) modulo 2^32
 * turns -- for phase screens with D >= 45, on the fast (hardware sincos)
 * epilogue with float4-aligned output (gain screens keep fp64); slots whose
 * coefficients are not finite or out of the digit range take the fp64
 * contraction.  |error| < 2^-27 turn of phase over the allowed ranges
 * (7.06e-9 turn at D = 60, |coef / 2 pi| = 8.03 turns, |Cpix| = 1905 with
 * every rounding aligned; ~2^-32 at the BASELINE configs), below the fp32
 * rounding of the reduced phase (up to 2^-26 turn); it runs in the register
 * tile, the SHB tile (pixel digits shared in LDS by 4 waves) and the
 * LDS-staged kernels alike (same bits; sf_get_eval_kernel /
 * sf_get_eval_contraction say which). */
#define SF_OPT_EVAL_INT 15
/* SF_OPT_EVAL_WG_WAVES: waves per workgroup of the integer-digit register
 * tile -- 4 (0 = default: 256 pixels, 1 KiB store runs per (slot, plane)) or
 * 8 (512 pixels, 2 KiB runs).  Same bits.  It acts ONLY on the register tile
 * (SF_EVAL_KERNEL_TILE / TILE3) running the integer-digit contraction
 * (sf_get_eval_contraction == 1); the fp64 contraction, the LDS-staged
 * kernels and SF_EVAL_KERNEL_SHB always run 4-wave workgroups and ignore it
 * (the Python binding's eval_kernel() names the 8-wave variant when it runs). */
#define SF_OPT_EVAL_WG_WAVES 16
/* SF_OPT_FIT_EIG_WAVES: waves per flagged-direction mask of the subset-basis
 * Jacobi in sf_kl_fit -- 1..4 (0 = default: 3).  Every count writes the same
 * bits (the rotations and their per-element arithmetic do not depend on how
 * a round's column pairs are split over the waves). */
#define SF_OPT_FIT_EIG_WAVES 17
/* SF_OPT_FIT_SUBSET_DELETION: the flagged-direction subset bases by
 * secular-equation deletions (Loewner-corrected vectors), one per flagged
 * direction, the Jacobi solve only for the masks the deletions cannot
 * separate.  3 = each mask starts from its nearest ancestor in the mask
 * table that the deletions built (the mask with its lowest flagged
 * directions unflagged; the global basis when none is), one launch per
 * number of flagged directions; 2 = every mask from the global basis, one
 * launch; 1 (default) = 3 for a fit pass with many new masks, else 2;
 * 0 = the Jacobi solve for every mask.  1, 2 and 3 write the same bits. */
#define SF_OPT_FIT_SUBSET_DELETION 18
#define SF_EVAL_KERNEL_AUTO 0
#define SF_EVAL_KERNEL_TILE 1
#define SF_EVAL_KERNEL_LDS4 2
#define SF_EVAL_KERNEL_LDS8 3
#define SF_EVAL_KERNEL_LDS16 4
#define SF_EVAL_KERNEL_LDS8H 5 /* LDS-staged, 2 MFMA tiles per wave (large D) */
#define SF_EVAL_KERNEL_LDS16H 6
#define SF_EVAL_KERNEL_TILE3 7 /* register tile at 3 waves per SIMD */
#define SF_EVAL_KERNEL_SHB 8 /* register tile, Cpix (or its digits) shared in LDS by 4 waves */
/* The evaluation kernel sf_kl_eval (gain = 0) or sf_kl_eval_gain (gain = 1)
 * runs for the current grid and these flags on a 16-byte aligned output
 * (one of SF_EVAL_KERNEL_TILE / _LDS4 / _LDS8 / _LDS16). */
int sf_get_eval_kernel(sf_ctx* ctx, int gain, unsigned flags, int* kernel);
/* The contraction of that evaluation: SF_EVAL_CONTRACTION_F64 (fp64 MFMAs) or
 * SF_EVAL_CONTRACTION_I8_DIGITS (the integer-digit contraction,
 * SF_OPT_EVAL_INT). */
#define SF_EVAL_CONTRACTION_F64 0
#define SF_EVAL_CONTRACTION_I8_DIGITS 1
int sf_get_eval_contraction(sf_ctx* ctx, int gain, unsigned flags, int* contraction);
int sf_set_option(sf_ctx* ctx, int option, int value);
int sf_alloc(sf_ctx* ctx, size_t bytes, void** dev_ptr);
int sf_free(sf_ctx* ctx, void* dev_ptr);
int sf_copy_h2d(sf_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
int sf_copy_d2h(sf_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);

/*
 * Shared KL basis from the D piercepoints (host, [D][3] float64, the
 * "piercepoint" array of the screen soltab): C[i][j] =
 * -(|pp_i - pp_j|^2 / r0^2)^(beta/2) / 2, its pseudo-inverse with absolute
 * cutoff 1e-3 (scipy>=1.7 pinv(rcond=1e-3) semantics) and U = the left
 * singular vectors of C ordered by descending singular value.  Computed on
 * the device (wavefront Jacobi eigen-solver).  1 <= D <= SF_MAX_DIR.
 */
int sf_set_basis(sf_ctx* ctx, const double* pp_host, int D, double r0,
                 double beta);
/* Copy the device basis back (host [D][D] each; any pointer may be NULL). */
int sf_get_basis(sf_ctx* ctx, double* c_host, double* pinv_c_host,
                 double* u_host, double* eig_host);

/*
 * Batched KL least-squares fit of all T*F*A slots (one scalar-phase or tec
 * soltab, one pol).  Device inputs: phase [T][F][A][D] float64 (radians,
 * NOT yet referenced -- the reference-station subtraction of
 * stationscreen.py:994-997 is done here), weight [T][F][A][D] float32.
 * Host input: station_order [A] (the initial per-station order,
 * stationscreen.py:999-1034).  Device outputs (any may be NULL except
 * coef): coef [T][F][A][D] float64 (the "phase_screen000" values),
 * resid [T][F][A][D] float64, w_out [T][F][A][D] float32 (weights after
 * outlier flagging), order_out [T][F][A] int32 (orders, the weights of the
 * "...resid" soltab).  Requires sf_set_basis with the same D.
 */
int sf_kl_fit(sf_ctx* ctx, const double* phase, const float* weight, int T,
              int F, int A, const int* station_order_host,
              const sf_fit_params* params, double* coef, double* resid,
              float* w_out, int32_t* order_out);

/* Statistics of the last sf_kl_fit (synchronises): number of distinct
 * flagged-direction masks whose subset basis was decomposed, and number of
 * slots that took the general (tiny-weight) path. */
int sf_get_fit_stats(sf_ctx* ctx, int* n_masks, int* n_general);

/* The subset bases the last sf_kl_fit decomposed (a test / inspection
 * hook; every call renumbers and rebuilds its pool): up to max_masks
 * entries, each its direction mask (masks_host[i], bit d = direction d
 * unflagged, n bits set) and a [D][D] block whose leading n x n part holds
 * the subset's eigenvectors (row = unflagged direction in index order,
 * columns sorted by |lambda| descending) followed by D slots whose first n
 * hold its eigenvalues (entries_host[i * (D*D + D)]); the rest of an entry
 * is unspecified.  Entries are in the order the
 * masks were numbered, which is not deterministic; *n_masks = how many
 * exist.  Synchronises. */
int sf_get_fit_pool(sf_ctx* ctx, uint64_t* masks_host, double* entries_host,
                    int max_masks, int* n_masks);

/*
 * Pixel grid of the a-term image: X[nx], Y[ny] screen coordinates of the
 * diagonal pixels (kl_screen.py:247-259, quirk Q8: pixel (y=j, x=i) is
 * evaluated at (X[i], Y[j])).  Builds the [nx*ny][D] pixel basis on the
 * device in MFMA fragment order.  Requires sf_set_basis first.
 */
int sf_set_grid(sf_ctx* ctx, const double* x_host, int nx,
                const double* y_host, int ny);

/*
 * KL pixel evaluation of S slots: phase[s][p] = sum_d Cpix[p][d]*coef[s][d]
 * (float64, MFMA), written as the 4 Jones planes (cos, sin, cos, sin) in
 * float32 to out[(s % ring_slots)][4][ny][nx] (device).  ring_slots >= S
 * writes every slot to its own place; smaller rings let a benchmark stream
 * an output volume larger than HBM.  coef: device [S][D] float64.
 */
int sf_kl_eval(sf_ctx* ctx, const double* coef, int64_t S, float* out,
               int64_t ring_slots, unsigned flags);

/*
 * Gain screens (kl_screen.py:319-378): three KL screens on the same pixel
 * basis -- phase and the XX / YY log10-amplitude screens -- written as
 * (10^xx cos, 10^xx sin, 10^yy cos, 10^yy sin).  Device coef arrays [S][D].
 */
int sf_kl_eval_gain(sf_ctx* ctx, const double* coef_phase,
                    const double* coef_xx, const double* coef_yy, int64_t S,
                    float* out, int64_t ring_slots, unsigned flags);
/* sf_kl_eval / sf_kl_eval_gain (coef_xx = coef_yy = NULL: phase screens)
 * that also ADD, mod 2^32, to slot_sums[s] (device, uint32, zeroed by the
 * caller) the checksum of slot s's output: the sum mod 2^32 of the 4 N^2
 * 32-bit words written for it (as stored, after the NaN scrub / byte swap;
 * SURVEY.md §8(d) "per-slot sum of fp32 words").  Order-free
 * integer sums, so a slot streamed through a ring in a large run and the same
 * slot evaluated alone give the same value: the discard + checksum mode of
 * volumes that do not fit HBM. */
int sf_kl_eval_sums(sf_ctx* ctx, const double* coef_phase,
                    const double* coef_xx, const double* coef_yy, int64_t S,
                    float* out, int64_t ring, unsigned flags,
                    uint32_t* slot_sums);

/*
 * Tessellated (Voronoi) screens: fill every pixel with the values of the
 * direction whose cell contains it, then (smooth_pix > 0) apply the Gaussian
 * of Screen.write.  Replaces VoronoiScreen.make_matrix + the smoothing loop
 * (voronoi_screen.py:132-216, screen.py:353-362).  Device inputs: labels
 * [ny][nx] int32 in 1..D (the template of make_rasertize_template), phase
 * [S][D] float64 (already referenced), amp_xx / amp_yy [S][D] float64 or NULL
 * (phase-only: amplitude 1).  Output as sf_kl_eval.  smooth_pix <= 6 runs
 * fused in one LDS-tiled kernel; larger values (any sigma, as scipy) gather
 * first and then run the passes of sf_smooth, which needs ring_slots >= S.
 * A label outside 1..D (the template never makes one) gives NaN pixels (1 / 0
 * under SF_EVAL_NAN_SCRUB); no table entry is read for it.
 */
int sf_tess_fill(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                 const double* phase, const double* amp_xx,
                 const double* amp_yy, int D, int64_t S, float* out,
                 int64_t ring_slots, double smooth_pix, unsigned flags);

/*
 * The Gaussian smoothing of Screen.write (screen.py:353-362:
 * scipy.ndimage.gaussian_filter(., sigma=(0, smooth_pix, smooth_pix)) per
 * image, float32 between the y and x passes, 'reflect' borders, truncate
 * 4 sigma) in place on n_img images [n_img][ny][nx] float32 on the device --
 * the cube [S][4][ny][nx] is n_img = 4 S images (n_img must be a multiple of
 * 4).  SF_EVAL_NAN_SCRUB / SF_EVAL_BIG_ENDIAN in flags apply after smoothing,
 * as the reference scrubs after smoothing: evaluate without them, then
 * smooth with them.  Any smooth_pix (device pass buffer <= 256 MiB).
 */
int sf_smooth(sf_ctx* ctx, float* cube, int nx, int ny, int64_t n_img,
              double smooth_pix, unsigned flags);

#ifdef __cplusplus
}
#endif
#endif /* SCREENFIT_H */

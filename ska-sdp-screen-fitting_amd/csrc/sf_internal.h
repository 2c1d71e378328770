// sf_internal.h -- shared definitions of libscreenfit (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "screenfit.h"

namespace sf {

// error plumbing -------------------------------------------------------------
void set_error(const std::string& msg);

#define SF_HIP(call)                                                        \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) {                                                 \
      ::sf::set_error(std::string(#call) + ": " + hipGetErrorString(e_));   \
      return SF_EIO;                                                        \
    }                                                                       \
  } while (0)

#define SF_REQUIRE(cond, code, msg) \
  do {                              \
    if (!(cond)) {                  \
      ::sf::set_error(msg);         \
      return (code);                \
    }                               \
  } while (0)

// pixel tiling of the evaluation kernel (kl_eval.hip) -------------------------
constexpr int kTiles = 4;                       // 16x16 MFMA tiles per wave, interleaved
constexpr int kWavePix = 16 * kTiles;           // 64 consecutive pixels per wave
constexpr int kEvalWaves = 4;                   // waves per workgroup
constexpr int kBlockPix = kWavePix * kEvalWaves; // 256 pixels per workgroup

// integer-digit contraction (kl_eval_int.h): balanced base-256 digits per
// operand
constexpr int kDigits = 6;

}  // namespace sf

struct sf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // shared KL basis (sf_set_basis)
  int D = 0;
  double r0 = 100.0;
  double beta = 5.0 / 3.0;
  double* d_pp = nullptr;      // [D][3]
  double* d_c = nullptr;       // [D][D]
  double* d_pinv = nullptr;    // [D][D]
  double* d_u = nullptr;       // [D][D] (columns sorted by |lambda| desc)
  double* d_eig = nullptr;     // [D]    (signed eigenvalues, sorted)
  // pixel grid (sf_set_grid)
  int nx = 0, ny = 0;
  int64_t n_pix = 0;
  int64_t n_pix_blocks = 0;    // workgroup pixel blocks (kBlockPix)
  int ksteps = 0;              // ceil(D / 4)
  double* d_cfrag = nullptr;   // [wave pixel blocks][ksteps][kTiles][64]
  // fixed-point phase epilogue: a lane's |coef| sum (turns) below rev_thr
  // bounds its phases below 2^17 turns (kl_eval_impl.h group_rev_safe)
  double rev_thr = 0.0;
  // integer-digit contraction (kl_eval_int.h): Cpix as 6 balanced base-256
  // digits of rint(Cpix * 2^36) in i8 MFMA B-fragment order (phase screens,
  // D >= 45), and whether the grid fits the digits
  int8_t* d_cdig = nullptr;    // [wave pixel blocks][6][kTiles][64][16 B]
  int dig_ok = 0;              // 1: max |Cpix| * 2^36 fits 6 digits
  int eval_int = -1;           // SF_OPT_EVAL_INT (-1 auto, 0 off)
  int eval_wg_waves = 0;       // SF_OPT_EVAL_WG_WAVES (0 = 4, or 8)
  // per-call slot digits of the integer contraction (kl_kdig_kernel)
  int8_t* d_kdig = nullptr;    // [slot][6][64]
  uint8_t* d_kflag = nullptr;  // [slot]: 1 = integer path
  int64_t kdig_slots = 0;      // slots the buffers hold
  // recorded after every launch that reads d_kdig / d_kflag: the next
  // prepass (on whatever stream) waits for it before rewriting them
  hipEvent_t kdig_read = nullptr;
  double h_pp[3 * SF_MAX_DIR] = {};  // host copy of the piercepoints
  // fit scratch
  uint8_t* d_skip = nullptr;   // [F][A] block skip flags
  size_t skip_cap = 0;
  int* d_st_order = nullptr;   // [A]
  size_t st_order_cap = 0;
  // mask-keyed cache of flagged-subset bases (kl_fit_fast.hip)
  unsigned long long* d_keys = nullptr;  // hash table keys (0 = empty)
  int* d_ids = nullptr;                  // hash table values (-1 = unassigned)
  size_t table_cap = 0;                  // power of two
  unsigned long long* d_pool_mask = nullptr;  // [pool_cap] mask of pool entry
  double* d_pool = nullptr;              // [pool_cap][D*D + D] (U_sub, lam)
  int fit_eig_waves = 0;                 // SF_OPT_FIT_EIG_WAVES (0 = 3)
  int fit_subset_deletion = 1;           // SF_OPT_FIT_SUBSET_DELETION: 1 from ancestors (default), 2 from the global basis, 0 Jacobi
  size_t pool_cap = 0;
  uint8_t* d_pool_status = nullptr;      // [>= pool entries] deletion kernel: 0 done, 1 Jacobi
  size_t pool_status_cap = 0;
  int pool_D = 0;
  int* d_pos = nullptr;                  // [S] table slot of the current mask
  uint8_t* d_class = nullptr;            // [S] 0 fast, 1 skipped, 2 slow
  double* d_sigma = nullptr;             // [F][A] tec/amplitude block sigma
  size_t sigma_cap = 0;
  size_t slot_cap = 0;
  int* d_counters = nullptr;  // [0] ids, [1] range start, [2] slow, [3] error,
                              // [4] non-uniform-weight slots
  double* d_scratch = nullptr;           // resid / state when caller passes NULL
  size_t scratch_cap = 0;
  float* d_wscratch = nullptr;
  int32_t* d_oscratch = nullptr;
  // Gaussian weights of sf_tess_fill / sf_smooth, pass buffer of sf_smooth
  double* d_gw = nullptr;
  size_t gw_cap = 0;                     // doubles
  double gw_sigma = -1.0;                // sigma whose weights d_gw holds
  float* d_trash = nullptr;  // 1 KiB sink of the eval's out-of-range stores
  float* d_smooth = nullptr;
  size_t smooth_cap = 0;                 // bytes
  float* d_tess_tab = nullptr;           // tessellated value table [S][D+1][4]
  size_t tess_tab_cap = 0;               // bytes
  // fast-path switch (SCREENFIT_FIT=general forces the general kernel)
  int force_general = 0;
  // evaluation kernel (SF_OPT_EVAL_KERNEL)
  int eval_kernel = SF_EVAL_KERNEL_AUTO;
  int64_t eval_max_blocks = 0;  // SF_OPT_EVAL_MAX_BLOCKS (0 = dispatch limit)
  int eval_ks_pad = 0;          // SF_OPT_EVAL_KS_PAD: extra zero k-steps
  int eval_sleep = 0;           // SF_OPT_EVAL_SLEEP: x 64 cycles per group
  int eval_xcd_map = -1;        // SF_OPT_EVAL_XCD_MAP (-1 = auto)
  int eval_groups = 0;          // SF_OPT_EVAL_GROUPS (0 = auto = 256)
  int eval_bands = 0;           // SF_OPT_EVAL_BANDS (0 = auto = 1)
  int tess_slots = 0;           // SF_OPT_TESS_SLOTS (0 = auto = 16)
  int tess_waves = 0;           // SF_OPT_TESS_WAVES (0 = auto = 16)
  int tess_tile = 0;            // SF_OPT_TESS_TILE (1: round-1 fused tile kernel)
  int tess_box = -1;            // SF_OPT_TESS_BOX (-1 auto, 0 wide-tile, 1 interior lookups)
  int fit_pack = 1;             // SF_OPT_FIT_PACK: 2 slots per wave for D <= 32
  int fit_lean = 1;             // SF_OPT_FIT_LEAN: lean pass when weights are uniform
};

namespace sf {
// Does the integer-digit contraction (kl_eval_int.h) serve this call?  Phase
// screens from D = 45 (below, the fp64 MFMA share of the SIMD is small and
// the LDS-staged kernels are store-bound already) on the fast epilogue with
// float4-aligned output; SF_OPT_EVAL_INT = 0 and grids whose |Cpix| does not
// fit the digits keep the fp64 contraction.
inline bool eval_int_applies(const sf_ctx* ctx, bool gain, unsigned flags,
                             bool out_aligned16) {
  return !gain && ctx->dig_ok && ctx->d_cdig && ctx->eval_int != 0 &&
         (flags & SF_EVAL_FAST_SINCOS) && ctx->n_pix % 4 == 0 && out_aligned16 &&
         ctx->ksteps >= 12;
}

struct RefSpec {
  int sub = -1;                 // local station whose phases are subtracted
  const double* refph = nullptr;  // or: external reference phases [T][F][D]
  int skip = -1;                // local station skipped as the reference
};
RefSpec ref_spec(const sf_fit_params* p, int A);
int launch_skip(sf_ctx* ctx, const double* phase, const float* weight, int T,
                int F, int A, const RefSpec& r);
int launch_fit_general(sf_ctx* ctx, const int* slot_list, const int* n_list,
                       int64_t max_slots, const double* phase,
                       const float* weight, int T, int F, int A,
                       const sf_fit_params* p, const RefSpec& r, double* coef,
                       double* resid, float* w_out, int32_t* order_out);
int launch_basis(sf_ctx* ctx);
int launch_cpix(sf_ctx* ctx, const double* d_x, const double* d_y);
int launch_cdig(sf_ctx* ctx, const double* d_x, const double* d_y, int* d_bad);
int launch_fit(sf_ctx* ctx, const double* phase, const float* weight, int T,
               int F, int A, const sf_fit_params* p, double* coef,
               double* resid, float* w_out, int32_t* order_out);
int pick_eval_kernel(const sf_ctx* ctx, bool gain, unsigned flags,
                     bool out_aligned16);
int launch_eval(sf_ctx* ctx, const double* coef, const double* cxx,
                const double* cyy, int64_t S, float* out, int64_t ring,
                unsigned flags, unsigned* sums);
int launch_tess(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                const double* phase, const double* amp_xx,
                const double* amp_yy, int D, int64_t S, float* out,
                int64_t ring, const double* d_w, int R, unsigned flags);
int launch_tess_tile(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                const double* phase, const double* amp_xx,
                const double* amp_yy, int D, int64_t S, float* out,
                int64_t ring, const double* d_w, int R, unsigned flags);
int launch_smooth(sf_ctx* ctx, float* cube, int nx, int ny, int64_t n_img,
                  const double* d_w, int R, unsigned flags);
constexpr int kTessMaxR = 24;  // Gaussian radius of the fused tess kernel
}  // namespace sf

// kl_eval.hip -- KL screen -> pixel-grid evaluation on gfx950.
//
// Replaces KLScreen.make_matrix + calculate_kl_screen (kl_screen.py:192-449):
// for every slot s and pixel p
//     phase[s][p] = sum_d Cpix[p][d] * coef[s][d]          (float64)
//     out[s][0|2][p] = cos(phase), out[s][1|3][p] = sin(phase)  (float32)
// Cpix is the same for every slot (kl_screen.py:446-448 depends only on the
// piercepoints, r0, beta and the pixel coordinates), so the evaluation is one
// dense (S x D) x (D x P) contraction followed by an elementwise epilogue --
// HBM-write-bound (16 B written per pixel per slot).
//
// Mapping (one 64-lane wave):
//   * v_mfma_f64_16x16x4_f64 with A = coef (16 slots x 4 dirs) and B = Cpix^T
//     (4 dirs x 16 pixels); kTiles = 4 B tiles whose columns interleave so
//     that lane l owns the 4 CONSECUTIVE pixels 4*(l&15) + t of a 64-pixel
//     run -> every store is a 16-B float4, 16 lanes cover 256 contiguous B.
//   * the wave keeps its Cpix fragments (ksteps x 4 doubles) in registers for
//     its whole lifetime and streams slot groups of 16 through the MFMA.
//   * an fp64 MFMA holds its SIMD's VALU for its whole 64 cycles (measured:
//     tools/coexec_probe.hip), so contraction and epilogue ADD on a SIMD:
//     the epilogue is cut to ~7 VALU issues per value (kl_eval_impl.h).
//   * block index -> (pixel block, slot chunk) is XCD-aware: the 8 XCDs each
//     own 1/8 of the pixel blocks, so their Cpix slices stay in their L2.
// Two store mappings share this contraction (same bits out):
//   * kl_eval_kernel (register tile): each lane stores its own MFMA outputs,
//     so one store instruction covers 4 slots x 256 B;
//   * kl_eval_lds_kernel: the reduced phases go through LDS and each wave
//     writes 1-4 KiB contiguous runs per (slot, plane) -- the choice up to
//     D = 44; the register tile takes larger D, fp64 sincos and gain screens
//     (profiles/round2c_eval_sweep.txt).
// This unit holds the pixel basis, the kernel choice and the dispatch on the
// k-step count; the kernels and their launch templates are in
// kl_eval_impl.h, instantiated per KS in kl_eval_ks1..5.hip.

#include "kl_eval_impl.h"

namespace sf {

// launch_eval_pick<KS> is instantiated in kl_eval_ks*.hip
SF_EVAL_KS_LIST(SF_EVAL_EXTERN)

__device__ inline double pix_cov(double ppx, double ppy, double ppz, double x,
                                 double y, double r0sq, double half_beta) {
#pragma clang fp contract(off)
  // numpy: sum(square(PIERCEPOINTS - (x, y, 0)), axis=1) -> ((.)+(.))+(.)
  const double dx = ppx - x;
  const double dy = ppy - y;
  const double dz = ppz - 0.0;
  const double d2 = (dx * dx + dy * dy) + dz * dz;
  return -pow(d2 / r0sq, half_beta) / 2.0;
}

// Cpix in MFMA B-fragment order: [wave pixel block][kstep][tile][lane].
__global__ __launch_bounds__(256) void kl_cpix_kernel(
    const double* __restrict__ pp, int D, double r0, double beta,
    const double* __restrict__ xs, int nx, const double* __restrict__ ys,
    int ny, int ksteps, int64_t n_elems, double* __restrict__ cfrag) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_elems) return;
  const int l = (int)(e & 63);
  const int t = (int)((e >> 6) % kTiles);
  const int64_t rest = (e >> 6) / kTiles;
  const int kk = (int)(rest % ksteps);
  const int64_t wpb = rest / ksteps;
  const int64_t p = wpb * kWavePix + (int64_t)(l & 15) * kTiles + t;
  const int d = 4 * kk + (l >> 4);
  double v = 0.0;
  if (p < (int64_t)nx * ny && d < D) {
    const int i = (int)(p % nx), j = (int)(p / nx);
    v = pix_cov(pp[3 * d], pp[3 * d + 1], pp[3 * d + 2], xs[i], ys[j],
                r0 * r0, beta / 2.0);
  }
  cfrag[e] = v;
}

int launch_cpix(sf_ctx* ctx, const double* d_x, const double* d_y) {
  const int64_t n_wpb = ctx->n_pix_blocks * kEvalWaves;
  const int64_t n = n_wpb * ctx->ksteps * kTiles * 64;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(kl_cpix_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     ctx->stream, ctx->d_pp, ctx->D, ctx->r0, ctx->beta, d_x,
                     ctx->nx, d_y, ctx->ny, ctx->ksteps, n, ctx->d_cfrag);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

// Pixel digits of the integer contraction (kl_eval_int.h): digit i of a
// wave pixel block in v_mfma_i32_16x16x64_i8 B order -- lane l, byte jb holds
// direction d = 16 (l >> 4) + jb of pixel column l & 15 of tile t, i.e. digit
// i of rint(Cpix[p][d] * 2^36) (0 past D or the grid).  Cpix is
// kl_cpix_kernel's value bit for bit (pix_cov).
// A value that is not finite or does not fit the 6 digits (the host's range
// check is a bound, not a proof) sets *bad, and sf_set_grid keeps the fp64
// contraction for the grid.
__global__ __launch_bounds__(256) void kl_cdig_kernel(
    const double* __restrict__ pp, int D, double r0, double beta,
    const double* __restrict__ xs, int nx, const double* __restrict__ ys,
    int ny, int64_t n_frag, v4i* __restrict__ cdig, int* __restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_frag) return;
  const int l = (int)(e & 63);
  const int t = (int)((e >> 6) % kTiles);
  const int64_t rest = (e >> 6) / kTiles;
  const int i = (int)(rest % kDigits);
  const int64_t wpb = rest / kDigits;
  const int64_t p = wpb * kWavePix + (int64_t)(l & 15) * kTiles + t;
  union {
    v4i v;
    int8_t b[16];
  } u;
#pragma unroll 1
  for (int jb = 0; jb < 16; ++jb) {
    const int d = 16 * (l >> 4) + jb;
    int8_t val = 0;
    if (d < D && p < (int64_t)nx * ny) {
      const int ix = (int)(p % nx), iy = (int)(p / nx);
      const double c = pix_cov(pp[3 * d], pp[3 * d + 1], pp[3 * d + 2], xs[ix], ys[iy],
                               r0 * r0, beta / 2.0);
      const double y = ldexp(c, kSigma);
      const bool fin = __builtin_isfinite(y) && fabs(y) < 4.6e18;  // llrint range
      int8_t dg[kDigits];
      const long long rem = dig_split(fin ? (long long)rint(y) : 0ll, dg);
      if (!fin || rem != 0) atomicOr(bad, 1);
      val = dg[i];
    }
    u.b[jb] = val;
  }
  cdig[e] = u.v;
}

int launch_cdig(sf_ctx* ctx, const double* d_x, const double* d_y, int* d_bad) {
  const int64_t n_wpb = ctx->n_pix_blocks * kEvalWaves;
  const int64_t n = n_wpb * kDigits * kTiles * 64;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(kl_cdig_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     ctx->stream, ctx->d_pp, ctx->D, ctx->r0, ctx->beta, d_x,
                     ctx->nx, d_y, ctx->ny, n, reinterpret_cast<v4i*>(ctx->d_cdig),
                     d_bad);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

// Kernel sf_kl_eval runs for this context, output alignment and flags.
int pick_eval_kernel(const sf_ctx* ctx, bool gain, unsigned flags,
                     bool out_aligned16) {
  // the LDS-staged kernel covers phase screens with the fast (hardware) sincos
  // epilogue and float4-aligned output; everything else (fp64 sincos, gain
  // screens, odd grids) takes the register-tile kernel
  const bool lds_ok = !gain && (flags & SF_EVAL_FAST_SINCOS) &&
                      (ctx->n_pix % 4 == 0) && out_aligned16;
  const int opt = ctx->eval_kernel;
  if (gain) {
    // round 6: gain screens on the LDS-staged kernels whose three-plane tile
    // fits LDS (LDS16's 1024-pixel run does not: LDS16H instead), fast
    // epilogue, float4-aligned output, up to kGainLdsMaxKS k-steps including
    // any zero padding
    const bool glds = (flags & SF_EVAL_FAST_SINCOS) && ctx->n_pix % 4 == 0 &&
                      out_aligned16 && ctx->ksteps + ctx->eval_ks_pad <= kGainLdsMaxKS;
    switch (opt) {
      case SF_EVAL_KERNEL_LDS4:
      case SF_EVAL_KERNEL_LDS8:
      case SF_EVAL_KERNEL_LDS8H:
      case SF_EVAL_KERNEL_LDS16H:
        return glds ? opt : SF_EVAL_KERNEL_TILE;
      case SF_EVAL_KERNEL_LDS16:
        return glds ? SF_EVAL_KERNEL_LDS16H : SF_EVAL_KERNEL_TILE;
      case SF_EVAL_KERNEL_TILE3:
        return opt;
      case SF_EVAL_KERNEL_AUTO:
        return glds ? kGainLdsAuto : SF_EVAL_KERNEL_TILE;
      default:
        return SF_EVAL_KERNEL_TILE;
    }
  }
  // the integer-digit contraction (phase D >= 45) runs on the register tile,
  // the SHB tile (pixel digits in LDS) and the LDS-staged kernels (same bits)
  const bool ic = eval_int_applies(ctx, gain, flags, out_aligned16);
  // (auto: the register tile -- 512^2 x D = 50 0.744 with 4-group items;
  // the LDS-staged shapes 0.66-0.70, profiles/round3y_eval_items_512.txt)
  if (ic && opt == SF_EVAL_KERNEL_AUTO) return SF_EVAL_KERNEL_TILE;
  if (opt == SF_EVAL_KERNEL_SHB)
    return (!gain && ctx->n_pix % 4 == 0 && out_aligned16) ? opt : SF_EVAL_KERNEL_TILE;
  if (opt == SF_EVAL_KERNEL_TILE || opt == SF_EVAL_KERNEL_TILE3) return opt;
  if (!lds_ok) return SF_EVAL_KERNEL_TILE;
  if (opt != SF_EVAL_KERNEL_AUTO) return opt;
  // measured on MI355X with the v_sin / v_cos epilogue (tools/eval_variants.py,
  // profiles/round2c_eval_sweep.txt): the LDS-staged kernels' long store runs
  // win up to D = 44 (16 waves up to D = 32, 4 waves / 1 KiB runs beyond,
  // where the 16-wave barrier starts to serialise MFMA and stores; 16 waves
  // with half tiles for D <= 12); from D = 45 the register tile (2 waves /
  // SIMD, Cpix fragments in registers) is 4-10 % ahead of every LDS shape
  if (ctx->ksteps <= 3) return SF_EVAL_KERNEL_LDS16H;
  if (ctx->ksteps <= 8) return SF_EVAL_KERNEL_LDS16;
  if (ctx->ksteps <= 11) return SF_EVAL_KERNEL_LDS4;
  return SF_EVAL_KERNEL_TILE;
}

int launch_eval(sf_ctx* ctx, const double* coef, const double* cxx,
                const double* cyy, int64_t S, float* out, int64_t ring,
                unsigned flags, unsigned* sums) {
  // the kernels keep slot and ring indices in 32 bits; a ring longer than
  // the launch changes nothing (slot s -> ring entry s % ring = s)
  if (S > INT32_MAX) {
    set_error("sf_kl_eval: more than 2^31 - 1 slots in one call");
    return SF_EINVAL;
  }
  if (ring > S) ring = S > 0 ? S : 1;
  // zero k-step padding (SF_OPT_EVAL_KS_PAD) only for the LDS-staged
  // kernels, which take the real k-step count for their Cpix indexing
  const int v = pick_eval_kernel(ctx, cxx != nullptr, flags,
                                 (reinterpret_cast<uintptr_t>(out) & 15) == 0);
  const bool lds = v != SF_EVAL_KERNEL_TILE && v != SF_EVAL_KERNEL_TILE3 &&
                   v != SF_EVAL_KERNEL_SHB;
  int ks = ctx->ksteps + (lds ? ctx->eval_ks_pad : 0);
  flags &= ~(kEvalXcdInterleave | kEvalBandMask);
  if (ctx->eval_xcd_map > 0) flags |= kEvalXcdInterleave;
  if (ks > 15) ks = ctx->ksteps;
  switch (ks) {
#define SF_KS(k) \
  case k:        \
    return launch_eval_pick<k>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
    SF_KS(1) SF_KS(2) SF_KS(3) SF_KS(4) SF_KS(5) SF_KS(6) SF_KS(7) SF_KS(8)
    SF_KS(9) SF_KS(10) SF_KS(11) SF_KS(12) SF_KS(13) SF_KS(14) SF_KS(15)
#undef SF_KS
    default:
      set_error("sf_kl_eval: unsupported number of directions");
      return SF_EINVAL;
  }
}

}  // namespace sf

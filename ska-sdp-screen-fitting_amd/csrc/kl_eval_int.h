// kl_eval_int.h -- the integer-digit contraction of the evaluation (round 3).
//
// The evaluation contraction rev[s][p] = sum_d Cpix[p][d] * coef[s][d] / 2 pi
// (kl_screen.py:444-449) runs on v_mfma_f64_16x16x4_f64, which on gfx950 is
// 64 cycles for 1024 products and holds the SIMD's VALU meanwhile: at D = 50
// (config 5) the fp64 MFMA alone is ~0.5 of the SIMD time and the chip clocks
// down under it (1.71 GHz under PMC).  v_mfma_i32_16x16x64_i8 does 16384
// exact int8 products into int32 in 16 cycles (tools/i8_mfma_probe.hip: 64x
// the fp64 rate per product; the int32 sums wrap modulo 2^32).  The phase is
// only needed modulo one turn, to about 2^-26 turn (the fp32 rounding of the
// reduced phase), so:
//
//   * Cq = rint(Cpix * 2^36) and cq = rint(coef / 2 pi * 2^44) are split into
//     6 balanced base-256 digits each (Cq = sum_i a_i 256^i, a_i in
//     [-128, 127]); the grid must have |Cpix| < 2^10.9 (sf_set_grid checks),
//     a slot -8.031 <= coef / 2 pi <= 7.969 turns (the digit range: the
//     prepass checks, per slot);
//   * sum_d Cq cq 2^-80 turn = sum_{i,j} P_ij 2^(8 (i + j) - 80) with
//     P_ij = sum_d a_i[d] b_j[d] over the D <= 64 directions of one MFMA's
//     K, exact in int32 (|P| < 2^23);
//   * in units of 2^-32 turn a diagonal k = i + j weighs 2^(8 k - 48): the
//     diagonals k >= 10 are whole turns and vanish modulo 2^32, k <= 3 add
//     less than 1/4 unit together -- 25 digit pairs (k = 4..9) of one i8
//     MFMA each give the phase as a 32-bit fixed-point turn, wrapped: the
//     quantity the fixed-point fp64 epilogue reads off its accumulator
//     (kl_eval_impl.h kRevMagic), at half the MFMA cycles of the 13 fp64
//     k-steps of D = 50;
//   * error (turns): Cq rounding sum |coef / 2 pi| 2^-37 (<= 3.51e-9 at
//     D = 60 x 8.031 turns), cq rounding sum |Cpix| 2^-45 (<= 3.25e-9 at
//     60 x 1904.6), the dropped diagonals and the shifts of the combine
//     <= 1.3 units (3.0e-10): < 7.06e-9 < 2^-27 turn over the allowed
//     ranges (an adversarial case with every rounding aligned reaches
//     6.2e-9, tests/test_int_digits.py), ~2^-32 at the BASELINE configs;
//     the fp32 rounding of the reduced phase is up to 2^-26.
//
// Used for phase screens from D = 45 (the register tile's range), fast
// epilogue: below, the LDS-staged fp64 kernels are store-bound already.  Gain
// screens keep the fp64 MFMAs: their three contractions need all three slot
// row sets (and 3 x 7 combine ops per value) live at once, which spilled 47
// VGPRs in the register tile (0.48 vs 0.62 of 8 TB/s, DESIGN.md "Tried").
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sf_internal.h"

namespace sf {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kSigma = 36;       // Cq = rint(Cpix * 2^36)
constexpr int kTauPhase = 44;    // cq = rint(coef / 2 pi * 2^44)
#ifndef SF_DIG_ORDER
#define SF_DIG_ORDER 0
#endif
#ifndef SF_DIAG_LO
#define SF_DIAG_LO 4
#endif
constexpr int kDiagLo = SF_DIAG_LO;  // lowest diagonal kept (4 or 5)
static_assert(kDiagLo == 4 || kDiagLo == 5, "kept diagonals: 4..9 or 5..9");
constexpr int kDiagHi = 9;       // highest diagonal below a whole turn
constexpr int kNDiag = kDiagHi - kDiagLo + 1;

// the integer contraction's operands of one evaluation launch
struct DigArgs {
  const v4i* cdig = nullptr;       // pixel digit fragments (sf_ctx::d_cdig)
  const int8_t* kdig = nullptr;    // slot digit rows [slot][6][64]
  const uint8_t* kflag = nullptr;  // [slot]: 1 = integer path
};

// balanced base-256 digits of v (v = sum_i b_i 256^i, b_i in [-128, 127]);
// returns what is left above the kDigits digits (0 iff v fits)
__device__ __forceinline__ long long dig_split(long long v, int8_t (&b)[kDigits]) {
#pragma unroll
  for (int i = 0; i < kDigits; ++i) {
    const int lo = (int)(v & 0xff);
    const int bi = lo >= 128 ? lo - 256 : lo;
    b[i] = (int8_t)bi;
    v = (v - bi) >> 8;
  }
  return v;
}

// the 6 diagonal sums -> the phase in units of 2^-32 turn, wrapped: diagonal
// k weighs 2^(8 (k - 6)); the two lowest are folded in with arithmetic
// shifts (< 1.004 units of truncation), the rest wrap modulo 2^32
__device__ __forceinline__ int dig_combine(int p4, int p5, int p6, int p7, int p8, int p9) {
  int t = p5 + (p4 >> 8);
  t = p6 + (t >> 8);
  return (int)((unsigned)t + ((unsigned)p7 << 8) + ((unsigned)p8 << 16) +
               ((unsigned)p9 << 24));
}

// Slot digits (prepass of every integer evaluation launch): one wave per
// slot, lane d = direction (K position).  Row j of a slot holds digit j of
// its fixed-point coefficients (0 past D); kflag[s] = 1 when every
// coefficient is finite and fits, else the slot takes the fp64 contraction.
// (A template only so that every unit including this header may hold it.)
template <int kUnused = 0>
__global__ __launch_bounds__(256) void kl_kdig_kernel(
    const double* __restrict__ coef, int D, int64_t S, double prescale,
    int8_t* __restrict__ kdig, uint8_t* __restrict__ kflag) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;  // whole waves
  const int d = threadIdx.x & 63;
  const double x = d < D ? coef[s * D + d] * prescale : 0.0;
  const double y = ldexp(x, kTauPhase);
  bool ok = __builtin_isfinite(x) && fabs(y) < 4.6e18;  // llrint range
  int8_t dg[kDigits];
  const long long rem = dig_split(ok ? (long long)rint(y) : 0ll, dg);
  ok = __builtin_amdgcn_ballot_w64(!(ok && rem == 0)) == 0;
#pragma unroll
  for (int j = 0; j < kDigits; ++j) kdig[(s * kDigits + j) * 64 + d] = ok ? dg[j] : (int8_t)0;
  if (d == 0) kflag[s] = ok ? 1 : 0;
}

// slot of the group row an A-lane feeds: the i32 MFMA puts A row m in
// accumulator (lane 16 (m >> 2) + col, register m & 3), the fp64 one (whose
// store mapping the epilogue follows) row (l >> 4) + 4 r in (lane l,
// register r); feeding row m with slot (m >> 2) + 4 (m & 3) lands every slot
// where the fp64 contraction puts it
__device__ __forceinline__ int dig_row_slot(int l) {
  const int m = l & 15;
  return (m >> 2) + 4 * (m & 3);
}

// the lane's 16 bytes (directions 16 (l >> 4) ..) of each digit row of its
// slot (slots past S read slot S - 1: their output rows are never stored)
struct DigRows {
  v4i w[kDigits];
};

__device__ __forceinline__ void dig_load(DigRows& r, const int8_t* __restrict__ kdig,
                                         int64_t s, int64_t S, int l) {
  const int8_t* row = kdig + (s < S ? s : S - 1) * (kDigits * 64) + 16 * (l >> 4);
#pragma unroll
  for (int n = 0; n < kDigits; ++n) r.w[n] = *reinterpret_cast<const v4i*>(row + n * 64);
}

// one 16-slot group against one 16-pixel tile (pixel digit fragments
// bd[i] = digit i): the six diagonal sums of the 25 pairs, combined
__device__ __forceinline__ v4i dig_contract(const DigRows& r, const v4i (&bd)[kDigits]) {
  v4i acc[kNDiag];
#pragma unroll
  for (int k = 0; k < kNDiag; ++k) acc[k] = v4i{0, 0, 0, 0};
#if SF_DIG_ORDER == 0
  // pixel digit outer: consecutive MFMAs feed different accumulators
#pragma unroll
  for (int i = 0; i < kDigits; ++i)
#pragma unroll
    for (int k = kDiagLo; k <= kDiagHi; ++k)
      if (k - i >= 0 && k - i < kDigits)
        acc[k - kDiagLo] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            r.w[k - i], bd[i], acc[k - kDiagLo], 0, 0, 0);
#else
  // round robin over the diagonals: the m-th pair of every diagonal, then
  // the (m+1)-th -- an accumulator is fed again only after the others
#pragma unroll
  for (int m = 0; m < kDigits; ++m)
#pragma unroll
    for (int k = kDiagLo; k <= kDiagHi; ++k) {
      const int i = (k - kDigits + 1 > 0 ? k - kDigits + 1 : 0) + m;
      if (i <= k && i < kDigits)
        acc[k - kDiagLo] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            r.w[k - i], bd[i], acc[k - kDiagLo], 0, 0, 0);
    }
#endif
  v4i R;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    R[e] = kDiagLo == 4
               ? dig_combine(acc[0][e], acc[1][e], acc[2][e], acc[3][e], acc[4][e], acc[5][e])
               : dig_combine(0, acc[0][e], acc[1][e], acc[2][e], acc[3][e], acc[kNDiag - 1][e]);
  return R;
}

}  // namespace sf

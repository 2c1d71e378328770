// kl_eval_impl.h -- the evaluation kernels and their launch templates,
// shared by kl_eval.hip (pixel basis, kernel choice, dispatch on the k-step
// count) and the kl_eval_ks*.hip units that instantiate launch_eval_pick<KS>
// for a few KS each, so the five units compile in parallel.  See kl_eval.hip
// for the design notes.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "kl_eval_int.h"
#include "sf_internal.h"

namespace sf {

typedef double v4d __attribute__((ext_vector_type(4)));

// Energy attribution builds (tools/energy_variants.sh; never the shipped
// library): the register tile with one component removed, so the board
// power of each variant splits a kernel's joules per output byte into its
// parts -- 1: contraction only (no sincos / amplitude: the reduced phase and
// the raw log-amplitudes are stored), 2: epilogue only (no MFMA: the
// accumulators take a loaded coefficient / digit row), 3: stores only
// (neither: lane-dependent constants), 4: no evaluation kernel work at all
// (the launch returns at once; the integer path's slot-digit prepass still
// runs).  The same stores in the same pattern in every variant.
#ifndef SF_EVAL_ENERGY_DIAG
#define SF_EVAL_ENERGY_DIAG 0
#endif
constexpr int kEnergyDiag = SF_EVAL_ENERGY_DIAG;



// f64 16x16x4 accumulator layout on gfx950: lane l, register r holds
// D[row = (l >> 4) + 4 r][col = l & 15] (cdna_hip_programming.md §3).
__device__ __forceinline__ int acc_row(int l, int r) { return (l >> 4) + 4 * r; }

// Fast epilogue (SF_EVAL_FAST_SINCOS): the contraction runs on coefficients
// pre-scaled by 1 / 2 pi, so it yields the phase in REVOLUTIONS; the fp64
// reduction rev - rint(rev) to [-1/2, 1/2] is exact, the result is rounded to
// float (<= 1.5e-8 rev = 9.4e-8 rad) and fed to the hardware v_sin_f32 /
// v_cos_f32, whose argument is in revolutions (max |err| 1.25e-7 over
// [-1/2, 1/2] measured on MI355X, profiles/round2a_coexec_probe.txt): ~7 VALU
// issues per value instead of the ~25 of a polynomial sincos.  On gfx950 the
// fp64 MFMA holds the SIMD's VALU for its whole 64 cycles (same probe: MFMA
// and VALU waves on one SIMD take the SUM of their times), so every VALU
// cycle of the epilogue adds to the contraction's.
constexpr double kInv2Pi = 0.15915494309189535;

// fp32 revolutions in [-1/2, 1/2] of a phase given in revolutions; NaN / Inf
// -> 0 when scrubbing, i.e. cos 1 and sin 0 (screen.py:368-378 NaN scrub)
__device__ __forceinline__ float rev_reduce(double rev, bool scrub) {
  const float f = (float)(rev - rint(rev));
  return (scrub && __builtin_isnan(f)) ? 0.0f : f;
}

// rev_reduce of N (2 or 4) phases at once: v_cmp_u of a PAIR flags either
// being NaN, so N / 2 compares collect a lane flag and the N selects run only
// when some lane of the wave has a NaN (a wave-uniform branch; same bits as N
// rev_reduce calls)
template <int N>
__device__ __forceinline__ void rev_reduce_n(float (&f)[N], const double (&rev)[N],
                                             bool scrub) {
  static_assert(N % 2 == 0, "pairs");
  bool bad = false;
#pragma unroll
  for (int t = 0; t < N; ++t) f[t] = (float)(rev[t] - rint(rev[t]));
#pragma unroll
  for (int t = 0; t < N; t += 2) bad |= __builtin_isunordered(f[t], f[t + 1]);
  if (scrub && __builtin_amdgcn_ballot_w64(bad) != 0) {
#pragma unroll
    for (int t = 0; t < N; ++t) f[t] = __builtin_isnan(f[t]) ? 0.0f : f[t];
  }
}

// Fixed-point phase reduction (fast epilogue, round 3).  The phase
// contraction starts its accumulators at kRevMagic = 1.5 * 2^20 instead of 0,
// so the fp64 MFMA result is y = M + rev with ulp 2^-32 wherever |rev| <
// 2^19: the low dword of y is frac(rev) * 2^32 as a two's-complement int,
// i.e. the phase reduced to [-1/2, 1/2) turn in 32-bit fixed point, already
// rounded by the accumulation (<= KS * 2^-32 turn).  One v_cvt_f32_i32 and
// one v_mul_f32 then give the float argument of v_sin / v_cos, where the
// exact reduction rev - rint(rev) took v_rndne_f64 + v_add_f64 +
// v_cvt_f32_f64 (4.4 issue cycles each, profiles/round3b_valu_cost.txt):
// float(lo) * 2^-32 == float(rev' - rint(rev')) for rev' = y - M exactly.
// A 16-slot group takes this path only when every lane's coefficient sum
// bounds its phases below 2^17 turns (group_rev_safe: a lane holds a quarter
// of a slot's directions, so sum |coef| / 2 pi < rev_thr = 2^15 / max |Cpix|
// per lane) -- which also proves them finite, so no NaN scrub is needed
// there; any other group (NaN / Inf coefficients, huge phases) takes the
// exact path on rev' = y - M, NaN / Inf propagating.  The check costs KS
// fp64 adds per lane and group, about what the fixed point saves per value
// at D = 50 -- where the fixed point also measured 3-4 % slower in the
// config-5 bench (profiles/round3m_eval_fixed_point_ab.txt) -- so it is
// used up to kMagicMaxKS k-steps (D <= 44, the LDS-staged kernels' range),
// the exact reduction above; every kernel variant of a given D takes the
// same path and writes the same bits.
constexpr double kRevMagic = 1572864.0;          // 1.5 * 2^20
constexpr float kTwoM32 = 2.3283064365386963e-10f;  // 2^-32
constexpr int kMagicMaxKS = 11;
// gain screens on the LDS-staged kernels (round 6, "Tried" in DESIGN.md):
// bit-equal to the register tile but slower (0.48-0.56 vs 0.66 of 8 TB/s),
// so the shipped library compiles none (1.9 MB of code objects); a variant
// build with -DSF_EVAL_GAIN_LDS=1 has them for kGainLdsMaxKS k-steps, where
// SF_OPT_EVAL_KERNEL forces them (the auto choice stays on the tile)
#ifndef SF_EVAL_GAIN_LDS
#define SF_EVAL_GAIN_LDS 0
#endif
constexpr int kGainLdsMaxKS = SF_EVAL_GAIN_LDS ? 11 : 0;
constexpr int kGainLdsAuto = SF_EVAL_KERNEL_TILE;

template <int KS>
__device__ __forceinline__ bool group_rev_safe(const double (&af)[KS], double thr) {
  double sum = 0.0;
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) sum += fabs(af[kk]);
  return __builtin_amdgcn_ballot_w64(!(sum < thr)) == 0;  // NaN: not safe
}

__device__ __forceinline__ float rev_fixed(double y) {
  const int lo = (int)(unsigned)__double_as_longlong(y);
  return (float)lo * kTwoM32;
}

// rev_reduce_n of magic-started accumulators: fixed point when the group is
// safe, else the exact reduction of y - M (scrub as rev_reduce_n)
template <int N>
__device__ __forceinline__ void rev_reduce_magic(float (&f)[N], const double (&y)[N],
                                                 bool safe, double a0, bool scrub) {
  if (safe) {
#pragma unroll
    for (int t = 0; t < N; ++t) f[t] = rev_fixed(y[t]);
  } else {
    double rv[N];
#pragma unroll
    for (int t = 0; t < N; ++t) rv[t] = y[t] - a0;
    rev_reduce_n<N>(f, rv, scrub);
  }
}

// v_sin_f32 / v_cos_f32 return NaN for a NaN argument (checked by the
// unscrubbed cases of tests/test_gpu_parity.py::test_eval_kernels_agree)
__device__ __forceinline__ void sincos_rev(float f, float& s, float& c) {
  s = __builtin_amdgcn_sinf(f);
  c = __builtin_amdgcn_cosf(f);
}

// The two halves of load_coef, for software pipelining: load_coef_raw
// issues the KS loads of a group's fragments (clamped addresses, no use of
// the data), coef_finish applies the scale and zeroes the lanes past S or D
// once they have landed.  The register tile issues group g + 1's loads before
// group g's MFMAs, so their L2 round trip hides behind a whole group of MFMA
// and epilogue work instead of stalling the wave at the top of every group
// (vmcnt counts loads and stores in issue order: waiting for loads issued
// before group g's stores does not wait for the stores).
template <int KS>
__device__ __forceinline__ void load_coef_raw(double (&v)[KS],
                                              const double* __restrict__ coef,
                                              int64_t s0, int64_t S, int D, int l) {
  const int64_t s = s0 + (l & 15);
  const double* row = coef + (s < S ? s : S - 1) * D;
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int d = 4 * kk + (l >> 4);
    v[kk] = row[d < D ? d : D - 1];
  }
}

// select without a branch: an all-ones / all-zeros mask on the bits (the
// compiler turns a plain `ok ? x : 0.0` over a whole fragment into an
// exec-masked region with its own load waits)
__device__ __forceinline__ double keep_if(bool ok, double x) {
  const unsigned long long m = ok ? ~0ull : 0ull;
  return __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, x) & m);
}

template <int KS>
__device__ __forceinline__ void coef_finish(double (&af)[KS], const double (&v)[KS],
                                            int64_t s0, int64_t S, int D, int l,
                                            double scale) {
  const bool srow = s0 + (l & 15) < S;
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    af[kk] = keep_if(srow && 4 * kk + (l >> 4) < D, v[kk] * scale);
}

// MFMA A fragments of a 16-slot group: lane l holds coef[s0 + (l & 15)]
// [4 kk + (l >> 4)] for every k-step (0 past S or D), times `scale`.  The
// loads are unconditional (clamped addresses, then a select), so all KS of
// them are in flight together: a guarded load compiles to a branch around
// it and a wait after it, i.e. KS serial round trips to L2 per group.
template <int KS>
__device__ __forceinline__ void load_coef(double (&af)[KS],
                                          const double* __restrict__ coef,
                                          int64_t s0, int64_t S, int D, int l,
                                          double scale) {
  const int64_t s = s0 + (l & 15);
  const bool srow = s < S;
  const double* row = coef + (srow ? s : S - 1) * D;
  double v[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int d = 4 * kk + (l >> 4);
    v[kk] = row[d < D ? d : D - 1];
  }
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int d = 4 * kk + (l >> 4);
    af[kk] = (srow && d < D) ? v[kk] * scale : 0.0;
  }
}

// Workgroup index -> (pixel block, slot chunk).  XCD-aware when the pixel
// blocks divide by 8: consecutive workgroups go to the 8 XCDs round-robin,
// so XCD x owns pixel blocks [x*per, (x+1)*per) -- or, with the interleaved
// map (SF_OPT_EVAL_XCD_MAP), pb = x (mod 8) -- and their Cpix slices stay
// in its L2.  The eval kernels walk bb = blockIdx.x, += gridDim.x (a
// multiple of 8, so a workgroup stays on its XCD's pixel blocks): one HSA
// dispatch counts at most 2^32 work-items, which config 5 (16 M slots per
// GPU at 512^2) would exceed with one workgroup per (pixel block, chunk).
// Internal flag bit (never set by callers: sf_kl_eval masks it): XCD x takes
// the pixel blocks pb = x (mod 8) instead of a contiguous eighth.
constexpr unsigned kEvalXcdInterleave = 1u << 30;
// Internal flag bits 27-29: log2 of the pixel bands (SF_OPT_EVAL_BANDS).  With
// B bands the work items run band-major -- every slot chunk of band 0's pixel
// blocks, then band 1's, ... -- and the XCD map applies within a band, so an
// XCD's live Cpix slice is 1/B of its share: at 512^2 it outgrows the 4 MiB L2
// (D = 20: 5.2 MB, D = 50: 13.6 MB per XCD) unless banded.
constexpr int kEvalBandShift = 27;
constexpr unsigned kEvalBandMask = 7u << kEvalBandShift;

__device__ __forceinline__ void eval_block(int64_t bb, int64_t n_pb, int64_t n_sc,
                                           int64_t& pb, int64_t& sc,
                                           unsigned flags) {
  const int lb = (flags & kEvalBandMask) >> kEvalBandShift;
  int64_t band = 0;
  if (lb) {
    // the launcher sets bands only when n_pb / B divides by 8
    n_pb >>= lb;
    const int64_t per_band = n_pb * n_sc;
    band = bb / per_band;
    bb -= band * per_band;
  }
  if ((n_pb & 7) == 0) {
    const int64_t per = n_pb >> 3;
    const int64_t x = bb & 7, i = bb >> 3;
    pb = (flags & kEvalXcdInterleave) ? (i % per) * 8 + x : x * per + (i % per);
    sc = i / per;
  } else {
    pb = bb % n_pb;
    sc = bb / n_pb;
  }
  pb += band * n_pb;
}

// log2 of the pixel bands of a launch over n_pb blocks: SF_OPT_EVAL_BANDS,
// else auto_bands, while each band's blocks still divide by 8
inline unsigned eval_band_flags(const sf_ctx* ctx, int64_t n_pb, int auto_bands = 1) {
  int b = ctx->eval_bands ? ctx->eval_bands : auto_bands, lb = 0;
  while (b > 1 && ((n_pb % ((int64_t)8 * b)) != 0)) b >>= 1;
  while ((1 << lb) < b) ++lb;
  return (unsigned)lb << kEvalBandShift;
}

// Precise epilogue (no SF_EVAL_FAST_SINCOS): sin / cos(2 pi rev) in fp64 to
// ~1e-16, then one cast to float (the reference's fp64 cos / sin cast at the
// FITS store, Q12).  rev - rint(rev) and the quarter-turn split are exact;
// the remaining |t| <= 1/8 turn is scaled by 2 pi (relative error 1e-16) and
// fed to Taylor polynomials to x^15 / x^16 on |x| <= pi/4 (truncation
// <= 1e-15): ~20 fp64 VALU issues per value instead of ocml's sincos with its
// large-argument reduction.  NaN / Inf in, NaN out.
__device__ __forceinline__ void sincos_rev_f64(double rev, float& s, float& c) {
  const double fr = rev - rint(rev);            // [-1/2, 1/2] turn, exact
  const double q = rint(fr * 4.0);              // quarter turns, -2..2
  const double x = fma(-q, 0.25, fr) * 6.283185307179586;  // |x| <= pi/4
  const double x2 = x * x;
  double ps = fma(x2, 7.647163731819816e-13, -1.6059043836821613e-10);
  ps = fma(x2, ps, 2.505210838544172e-08);
  ps = fma(x2, ps, -2.7557319223985893e-06);
  ps = fma(x2, ps, 1.984126984126984e-04);
  ps = fma(x2, ps, -8.333333333333333e-03);
  ps = fma(x2, ps, 1.6666666666666666e-01);
  const double sx = fma(-x * x2, ps, x);        // x - x^3 / 6 + ...
  double pc = fma(x2, -1.1470745597729725e-11, 2.08767569878681e-09);
  pc = fma(x2, pc, -2.755731922398589e-07);
  pc = fma(x2, pc, 2.48015873015873e-05);
  pc = fma(x2, pc, -1.3888888888888889e-03);
  pc = fma(x2, pc, 4.1666666666666664e-02);
  pc = fma(x2, pc, -0.5);
  const double cx = fma(x2, pc, 1.0);           // 1 - x^2 / 2 + ...
  const int iq = (int)q & 3;
  const double a = (iq & 1) ? cx : sx;
  const double b = (iq & 1) ? sx : cx;
  s = (float)((iq & 2) ? -a : a);
  c = (float)(((iq + 1) & 2) ? -b : b);
}

// ph in revolutions (the coefficients are scaled by 1 / 2 pi as loaded):
// FAST = hardware fp32 sincos (rev_reduce), else sincos_rev_f64
template <bool FAST>
__device__ __forceinline__ void jones_sincos(double ph, float& s, float& c,
                                             bool scrub) {
  if (FAST) {
    sincos_rev(rev_reduce(ph, scrub), s, c);
  } else {
    sincos_rev_f64(ph, s, c);
  }
}

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bswapf(float x) {
  return __uint_as_float(__builtin_bswap32(__float_as_uint(x)));
}

// Per-slot output checksum (sf_kl_eval_sums): the sum, mod 2^32, of the
// 32-bit words the slot's cube holds (as stored: after the NaN scrub and any
// byte swap).  Integer adds commute, so the value does not depend on which
// lanes / waves / workgroups contribute in which order.  32-bit wrap-around
// adds (v_add3_u32 chains) keep the epilogue cost at ~0.5 VALU op per word.
__device__ __forceinline__ unsigned fbits(float x) { return __float_as_uint(x); }

// Sum over the 16 lanes of each DPP row (every lane of the row receives it):
// VALU-only butterflies, no LDS round trips.
__device__ __forceinline__ unsigned row_sum16(unsigned v) {
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// Transposed sum of four per-lane partials p[r] (r = 0..3) over the 16 lanes
// of each DPP row: lane i of the row returns the row total of p[i >> 2]
// (every lane of quad i >> 2 gets it).  Halving the values at each of the
// first two steps (exchange with lane i ^ 8, then with lane i ^ 7, keeping
// the r the lane's bits 3, 2 name) costs 11 VALU ops instead of the 16 of
// four row_sum16.
__device__ __forceinline__ unsigned row_sum16_x4(const unsigned (&p)[4], int i) {
  const bool b3 = i & 8, b2 = i & 4;
  // step 1, partner i ^ 8 (row_ror:8): keep r in {2 b3, 2 b3 + 1}
  const unsigned x0 = b3 ? p[0] : p[2], x1 = b3 ? p[1] : p[3];
  const unsigned q0 = (b3 ? p[2] : p[0]) +
                      (unsigned)__builtin_amdgcn_update_dpp(0, (int)x0, 0x128, 0xF, 0xF, false);
  const unsigned q1 = (b3 ? p[3] : p[1]) +
                      (unsigned)__builtin_amdgcn_update_dpp(0, (int)x1, 0x128, 0xF, 0xF, false);
  // step 2, partner i ^ 7 (row_half_mirror: same bit 3, other bit 2): keep
  // r = 2 b3 + b2; lane i now covers lanes {i, i^8, i^7, i^15}, and the four
  // lanes of a quad cover the row
  const unsigned w = b2 ? q0 : q1;
  unsigned v = (b2 ? q1 : q0) +
               (unsigned)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad [1,0,3,2]
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad [2,3,0,1]
  return v;
}

template <bool NT>
__device__ __forceinline__ void store4(float* p, v4f v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
  else *reinterpret_cast<v4f*>(p) = v;
}

// amplitude screens are log10 values: 10 ** screen (kl_screen.py:338-365);
// fast path: the XX / YY coefficients are pre-scaled by log2(10), so the
// contraction gives log2 A, rounded to float for v_exp_f32 (1 ulp)
constexpr double kLog2of10 = 3.321928094887362;
__device__ __forceinline__ float amp2f(double log2a) {
  return __builtin_amdgcn_exp2f((float)log2a);
}

// SHB ("shared B"): the 4 waves of a workgroup share ONE 64-pixel block,
// whose Cpix fragments sit in LDS (KS x 2 KiB) instead of 8*KS registers per
// wave, and take its 16-slot groups round-robin -- the register tile at
// ~half the VGPRs, so large D (config 5: D = 50) runs 4 waves per SIMD
// without spilling; same MFMA operands in the same order, same bits.
// BEM: byte order of the stores -- 0 little-endian, 1 big-endian (FITS),
// 2 chosen per launch from SF_EVAL_BIG_ENDIAN (a branch around two copies of
// the epilogue; the hot float4 / fast-sincos variants are compiled per byte
// order instead: with the branch the compiler's wait for the next group's
// coefficient loads also waits for most of this group's stores)
// DIRECT: every group of the launch is 16 live slots that do not wrap round
// the ring, in 64-pixel blocks inside the grid (launch_eval_ks sends a ragged
// tail to the general kernel): lane row (l >> 4) + 4 r of a group stores to
// lane_base + 16 r P -- one base per group instead of, per row, a ring index,
// a 64-bit product and the trash select (a run-time choice between the two
// would again be a branch round the stores, see BEM)
// NWV: waves per workgroup (the workgroup's pixel block is NWV x 64 pixels;
// the integer tile can run 8, SF_OPT_EVAL_WG_WAVES)
template <int KS, int MINW, bool VEC4, bool FAST, bool NT, bool GAIN,
          bool SHB = false, int BEM = 2, bool DIRECT = false, bool IC = false,
          int NWV = kEvalWaves>
__global__ __launch_bounds__(64 * NWV, MINW) void kl_eval_kernel(
    const double* __restrict__ cfrag, const double* __restrict__ coef,
    const double* __restrict__ coef_xx, const double* __restrict__ coef_yy,
    int D, int64_t S, int64_t P, int64_t n_pb, int64_t n_sc, int chunk_groups,
    float* __restrict__ out, int64_t ring, int64_t ring_base, unsigned flags,
    unsigned* __restrict__ sums, float* __restrict__ trash, double rev_thr,
    DigArgs dg) {
  constexpr int kFrag = KS * kTiles * 64;  // Cpix doubles of a wave pixel block
  if constexpr (kEnergyDiag == 4) return;
  constexpr bool kNoContract = kEnergyDiag == 2 || kEnergyDiag == 3;
  // IC: the integer-digit contraction (kl_eval_int.h) instead of the fp64
  // MFMAs; slots it cannot carry take the fp64 contraction with the Cpix
  // fragments read from memory.  IC + SHB: the pixel digit fragments of the
  // workgroup's 64-pixel block sit in LDS (24 KiB) instead of 96 VGPRs per
  // wave, read one tile at a time (round 4: 3 waves / SIMD instead of 2)
  static_assert(!IC || (FAST && !GAIN), "integer contraction: fast phase screens");
  static_assert(NWV == kEvalWaves || (IC && !SHB), "8-wave workgroups: integer register tile");
  // fixed-point phase reduction (kRevMagic) for D <= 44
  constexpr bool kMagic = FAST && KS <= kMagicMaxKS && !IC;
  // SHB: the fp64 Cpix fragments, or (IC) the pixel digit fragments
  // [digit][tile][lane] of the wave block (kDigits x kTiles x 64 x 16 B)
  constexpr int kShDoubles = SHB ? (IC ? kDigits * kTiles * 64 * 2 : kFrag) : 1;
  __shared__ double bsh[kShDoubles];
  const int l = threadIdx.x & 63;
  // wave index, wave-uniform: keeps slot / ring arithmetic on the SALU
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware block -> (pixel block, slot chunk); SHB: n_pb counts 64-pixel
  // wave blocks, else 256-pixel workgroup blocks
  const int64_t n_blocks = n_pb * n_sc;
  for (int64_t bb = blockIdx.x; bb < n_blocks; bb += gridDim.x) {
    int64_t pb, sc;
    eval_block(bb, n_pb, n_sc, pb, sc, flags);
    if (sc >= n_sc) continue;  // uniform per workgroup
    const int64_t wpb = SHB ? pb : pb * NWV + w;
    const int64_t p0 = wpb * kWavePix + (int64_t)(l & 15) * kTiles;
    if constexpr (SHB) {
      __syncthreads();  // the previous item's reads of bsh are done
      if (wpb * kWavePix < P) {
        if constexpr (IC) {
          constexpr int kN = kDigits * kTiles * 64;
          v4i* dst = reinterpret_cast<v4i*>(bsh);
          const v4i* src = dg.cdig + wpb * kN;
          for (int i = threadIdx.x; i < kN; i += 256) dst[i] = src[i];
        } else {
          for (int i = threadIdx.x; i < kFrag; i += 256) bsh[i] = cfrag[wpb * kFrag + i];
        }
      }
      __syncthreads();
    }
    if (wpb * kWavePix >= P) continue;

    double bf[SHB || IC ? 1 : KS][kTiles];
    if constexpr (!SHB && !IC) {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int t = 0; t < kTiles; ++t)
          bf[kk][t] = cfrag[((wpb * KS + kk) * kTiles + t) * 64 + l];
    }
    // IC: the pixel digit fragments [tile][digit] (IC + SHB: read per tile
    // from LDS in the group loop instead)
    v4i bd[kTiles][IC && !SHB ? kDigits : 1];
    if constexpr (IC && !SHB) {
#pragma unroll
      for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int i = 0; i < kDigits; ++i)
          bd[t][i] = dg.cdig[((wpb * kDigits + i) * kTiles + t) * 64 + l];
    }
    auto bval = [&](int kk, int t) -> double {
      if constexpr (SHB) return bsh[(kk * kTiles + t) * 64 + l];
      else return bf[kk][t];
    };

    const bool scrub = flags & SF_EVAL_NAN_SCRUB;
    const bool be = flags & SF_EVAL_BIG_ENDIAN;
    const int64_t slot_base = sc * (int64_t)chunk_groups * 16;
    // checksums: the slot sums of 4 groups of this wave are parked one per
    // lane (lane 16 k + 4 r + gq <- slot row 4 r + k of the gq-th group, the
    // layout row_sum16_x4 leaves) and leave as ONE 64-lane atomic instead of
    // 16 (atomics run at the memory side, one wave-instruction per ~50 ns per
    // CU); slots past S are never added
    unsigned pend = 0u;
    uint32_t pslot = ~0u;
    int gq = 0;
    auto flush_sums = [&]() {
      // phase screens on the float4 path sum planes 0 / 1 only (2 / 3 repeat
      // them): doubled here, once per flush instead of once per row
      if (pslot < (uint32_t)S) atomicAdd(sums + pslot, (VEC4 && !GAIN) ? 2u * pend : pend);
      pend = 0u;
      pslot = ~0u;
      gq = 0;
    };
    // coefficient fragments, loaded one group ahead: the raw loads of group
    // g + 1 go out before group g's MFMAs and stores (load_coef_raw) and are
    // finished (scaled, masked) at the end of group g; gain: the XX / YY
    // loads go out with the phase ones
    constexpr int kGStep = SHB ? kEvalWaves : 1;
    const double sx = FAST ? kLog2of10 : 1.0;
    double rf[KS], rx[GAIN ? KS : 1], ry[GAIN ? KS : 1];
    double af[KS], ax[GAIN ? KS : 1], ay[GAIN ? KS : 1];
    bool safe = false;
    // IC: the digit rows and the slot flags, one group ahead (the A-lane
    // feeding group row m holds slot dig_row_slot); unconditional loads of a
    // clamped slot (a load behind a branch is a serial round trip), slots
    // past S count as carried
    const int rs = dig_row_slot(l);
    DigRows wp;
    bool okp = true;
    auto load_flag = [&](int64_t s) {
      const uint8_t f = dg.kflag[s < S ? s : S - 1];
      okp = s >= S || f != 0;
    };
    if constexpr (IC) {
      const int64_t sw = slot_base + (SHB ? w : 0) * 16;
      dig_load(wp, dg.kdig, sw + rs, S, l);
      load_flag(sw + rs);
      // everything loaded so far must have landed before the group loop (as
      // the Cpix fragments below): else the compiler, merging this path with
      // the loop's back edge, waits at the loop top with a count that covers
      // the previous group's stores as well
      if constexpr (!SHB) {
#pragma unroll
        for (int t = 0; t < kTiles; ++t)
#pragma unroll
          for (int i = 0; i < kDigits; ++i) asm volatile("" ::"v"(bd[t][i]));
      }
#pragma unroll
      for (int n = 0; n < kDigits; ++n) asm volatile("" ::"v"(wp.w[n]));
      asm volatile("" ::"s"(__builtin_amdgcn_ballot_w64(okp)));
    } else {
      const int64_t s0 = slot_base + (SHB ? w : 0) * 16;
      load_coef_raw<KS>(rf, coef, s0, S, D, l);
      coef_finish<KS>(af, rf, s0, S, D, l, kInv2Pi);  // phase in turns
      if constexpr (kMagic) safe = group_rev_safe<KS>(af, rev_thr);
      if constexpr (GAIN) {
        load_coef_raw<KS>(rx, coef_xx, s0, S, D, l);
        load_coef_raw<KS>(ry, coef_yy, s0, S, D, l);
        coef_finish<KS>(ax, rx, s0, S, D, l, sx);
        coef_finish<KS>(ay, ry, s0, S, D, l, sx);
      }
      // the Cpix fragments too must have landed before the group loop: else
      // the compiler, merging this path with the loop's back edge, waits for
      // them inside the loop with a count that covers the previous group's
      // stores as well
      if constexpr (!SHB) {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int t = 0; t < kTiles; ++t) asm volatile("" ::"v"(bf[kk][t]));
      }
    }
    for (int g = SHB ? w : 0; g < chunk_groups; g += kGStep) {
      const int64_t s0 = slot_base + (int64_t)g * 16;
      if (s0 >= S) break;
      // SHB: keep the Cpix reads inside the loop (in LDS, not hoisted into
      // registers, which is the point)
      if constexpr (SHB) asm volatile("" ::: "memory");
      // the next group's loads (a clamped dummy past the chunk or S)
      const int64_t s1 = s0 + 16 * kGStep;
      if constexpr (!IC) {
        load_coef_raw<KS>(rf, coef, s1, S, D, l);
        if constexpr (GAIN) {
          load_coef_raw<KS>(rx, coef_xx, s1, S, D, l);
          load_coef_raw<KS>(ry, coef_yy, s1, S, D, l);
        }
      }
      // ring slot of the group's first slot (S, ring < 2^31: launch_eval);
      // the 16 rows follow it with at most one wrap when the ring is >= 16
      // slots -- scalar, no per-lane 64-bit modulo
      const uint32_t ring0 = (uint32_t)(s0 + ring_base) % (uint32_t)ring;
      // fast epilogue: fixed-point phase accumulators (kRevMagic)
      const double a0 = kMagic ? kRevMagic : 0.0;
      v4d acc[kTiles];
      // gain: the XX / YY log-amplitude screens share the pixel basis
      v4d accx[GAIN ? kTiles : 1], accy[GAIN ? kTiles : 1];
      // fast epilogue: the reduced phases of the group's 4 x 4 values
      float frg[4][kTiles];
      if constexpr (!IC) {
#pragma unroll
        for (int t = 0; t < kTiles; ++t) acc[t] = v4d{a0, a0, a0, a0};
        if constexpr (kNoContract) {
          // energy diagnostic: a loaded coefficient instead of the products
#pragma unroll
          for (int t = 0; t < kTiles; ++t) acc[t] += af[t % KS];
          if constexpr (GAIN) {
#pragma unroll
            for (int t = 0; t < kTiles; ++t) {
              accx[t] = v4d{ax[t % KS], ax[t % KS], ax[t % KS], ax[t % KS]};
              accy[t] = v4d{ay[t % KS], ay[t % KS], ay[t % KS], ay[t % KS]};
            }
          }
        } else {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int t = 0; t < kTiles; ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[kk], bval(kk, t),
                                                          acc[t], 0, 0, 0);
        if constexpr (GAIN) {
#pragma unroll
          for (int t = 0; t < kTiles; ++t) {
            accx[t] = v4d{0.0, 0.0, 0.0, 0.0};
            accy[t] = v4d{0.0, 0.0, 0.0, 0.0};
          }
#pragma unroll
          for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int t = 0; t < kTiles; ++t) {
              accx[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ax[kk], bval(kk, t), accx[t], 0, 0, 0);
              accy[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ay[kk], bval(kk, t), accy[t], 0, 0, 0);
            }
        }
        }
        // fixed point or exact by ONE wave-uniform branch per group (per-row
        // branches measured 4 % slower at D = 50); gain screens scrub the
        // products, phase screens the reduced argument (cos 1, sin 0)
        if constexpr (FAST) {
          if (safe) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int t = 0; t < kTiles; ++t) frg[r][t] = rev_fixed(acc[t][r]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              double rv[kTiles];
#pragma unroll
              for (int t = 0; t < kTiles; ++t) rv[t] = acc[t][r] - a0;
              rev_reduce_n<kTiles>(frg[r], rv, !GAIN && scrub);
            }
          }
        }
      } else {
        // ---- integer-digit contraction (kl_eval_int.h)
        // rows the digits cannot carry (bit 4 (l >> 4) + r <-> lane l's
        // register r): this group's flags, loaded one group ahead
        const unsigned long long badp = __builtin_amdgcn_ballot_w64(!okp) & 0xffffull;
        const int rowbit = 4 * (l >> 4);
#pragma unroll
        for (int t = 0; t < kTiles; ++t) {
          v4i R;
          if constexpr (kNoContract) {
            R = wp.w[t % kDigits];  // energy diagnostic: no MFMA
            if constexpr (!SHB) R ^= bd[t][0];
          } else if constexpr (SHB) {
            const v4i* bs = reinterpret_cast<const v4i*>(bsh);
            v4i bt[kDigits];
#pragma unroll
            for (int i = 0; i < kDigits; ++i) bt[i] = bs[(i * kTiles + t) * 64 + l];
            R = dig_contract(wp, bt);
          } else {
            R = dig_contract(wp, bd[t]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) frg[r][t] = (float)R[r] * kTwoM32;
        }
        // the next group's rows and flags (wp is free now)
        dig_load(wp, dg.kdig, s1 + rs, S, l);
        load_flag(s1 + rs);
        // fp64 contraction of the rows the digits cannot carry (non-finite
        // or out-of-range coefficients; rare), one k-step at a time (few
        // registers beside the digit fragments), Cpix fragments from memory:
        // the same products in the same order as the fp64 register tile, the
        // exact reduction
        if (badp != 0ull) {
          const int64_t sa = s0 + (l & 15);
          const double* row = coef + (sa < S ? sa : S - 1) * D;
          v4d ac[kTiles];
#pragma unroll
          for (int t = 0; t < kTiles; ++t) ac[t] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
          for (int kk = 0; kk < KS; ++kk) {
            const int d = 4 * kk + (l >> 4);
            const double a = keep_if(sa < S && d < D, row[d < D ? d : D - 1] * kInv2Pi);
#pragma unroll
            for (int t = 0; t < kTiles; ++t)
              ac[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                  a, cfrag[((wpb * KS + kk) * kTiles + t) * 64 + l], ac[t], 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double rv[kTiles];
            float f[kTiles];
#pragma unroll
            for (int t = 0; t < kTiles; ++t) rv[t] = ac[t][r];
            rev_reduce_n<kTiles>(f, rv, scrub);
            const bool b = (badp >> (rowbit + r)) & 1ull;
#pragma unroll
            for (int t = 0; t < kTiles; ++t) frg[r][t] = b ? f[t] : frg[r][t];
          }
        }
      }
      // this lane's checksum partial of each of its 4 slot rows
      unsigned part[4] = {0u, 0u, 0u, 0u};
      // one MFMA accumulator row: 4 slot rows x this lane's 4 pixels; BE
      // (FITS byte order) as a compile-time branch of the whole row
      // DIRECT: the lane's row base of this group (see the template notes)
      float* const lane_base = out + ((int64_t)(ring0 + (uint32_t)(l >> 4)) * 4) * P + p0;
      auto row_out = [&](int r, auto be_tag) {
        constexpr bool kBE = decltype(be_tag)::value;
        constexpr bool kDirect = VEC4 && DIRECT;
        const int row = acc_row(l, r);
        const int64_t s = s0 + row;
        // float4 path: rows past S and the float4s past P store into the
        // context's trash block instead of branching round the stores, so
        // every path through the epilogue issues the same 16 stores and the
        // compiler can wait for the next group's coefficient loads with
        // vmcnt(16) instead of vmcnt(0) (i.e. for this group's stores too)
        const bool live = s < S && (!VEC4 || p0 < P);
        if (!VEC4 && s >= S) return;  // uniform over the 16 lanes of a slot row
        uint32_t so = ring0 + (uint32_t)row;
        if (ring >= 16) {
          if (so >= (uint32_t)ring) so -= (uint32_t)ring;
        } else {
          so %= (uint32_t)ring;
        }
        // planes 0..3 = Re XX, Im XX, Re YY, Im YY
        float pv[4][kTiles];
        // per-value NaN scrub (gain, fp64 sincos): v_cmp_u of a PAIR of
        // values flags either being NaN, so 2 compares per pixel collect a
        // lane flag, and the 8 selects per pixel run only when some lane of
        // the wave has a NaN (a wave-uniform branch; same bits either way)
        constexpr bool kScrubValues = GAIN || !FAST;
        bool bad = false;
        // fast epilogue: this row's reduced arguments (frg, above)
        const float(&fr)[kTiles] = frg[r];
#pragma unroll
        for (int t = 0; t < kTiles; ++t) {
          float sf, cf;
          if constexpr (kEnergyDiag == 3) {
            // energy diagnostic: stores only
            pv[0][t] = pv[2][t] = (float)(l + t);
            pv[1][t] = pv[3][t] = (float)(r - t);
            continue;
          } else if constexpr (kEnergyDiag == 1) {
            // energy diagnostic: the contraction's values, no sincos / exp2
            pv[0][t] = pv[2][t] = fr[t];
            pv[1][t] = pv[3][t] = fr[t];
            if constexpr (GAIN) {
              pv[2][t] = (float)accx[t][r];
              pv[3][t] = (float)accy[t][r];
            }
            continue;
          }
          if (GAIN) {
            // a NaN phase stays NaN through A * cos and is scrubbed below,
            // as the reference scrubs the product (screen.py:368-378)
            if (FAST)
              sincos_rev(fr[t], sf, cf);
            else
              jones_sincos<false>(acc[t][r], sf, cf, false);
            if (FAST) {
              // fp32 amplitude x fp32 cos / sin: within 2e-6 x max(1, A)
              const float ax = amp2f(accx[t][r]);
              const float ay = amp2f(accy[t][r]);
              pv[0][t] = ax * cf;
              pv[1][t] = ax * sf;
              pv[2][t] = ay * cf;
              pv[3][t] = ay * sf;
            } else {
              // reference: A (fp64) * cos (fp64), one cast at the FITS store
              const double ax = exp10(accx[t][r]);
              const double ay = exp10(accy[t][r]);
              pv[0][t] = (float)(ax * (double)cf);
              pv[1][t] = (float)(ax * (double)sf);
              pv[2][t] = (float)(ay * (double)cf);
              pv[3][t] = (float)(ay * (double)sf);
            }
          } else {
            // FAST: NaN scrubbed on the reduced argument (cos 1, sin 0)
            if constexpr (FAST && !GAIN) sincos_rev(fr[t], sf, cf);
            else jones_sincos<FAST>(acc[t][r], sf, cf, scrub);
            pv[0][t] = pv[2][t] = cf;
            pv[1][t] = pv[3][t] = sf;
          }
          if (kScrubValues)
            bad |= __builtin_isunordered(pv[0][t], pv[1][t]) |
                   __builtin_isunordered(pv[2][t], pv[3][t]);
        }
        if (kScrubValues && scrub && __builtin_amdgcn_ballot_w64(bad) != 0) {
#pragma unroll
          for (int t = 0; t < kTiles; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (isnan(pv[q][t])) pv[q][t] = (q & 1) ? 0.0f : 1.0f;
        }
        if (kBE) {
#pragma unroll
          for (int t = 0; t < kTiles; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) pv[q][t] = bswapf(pv[q][t]);
        }
        unsigned cs = 0u;
        if (VEC4) {
          // P % 4 == 0: a lane's 4 pixels are all inside the grid or all out
          // (the last wave block of a grid that is not a multiple of 64)
          float* o;
          int64_t qstride = P;
          if constexpr (kDirect) {
            o = lane_base + (int64_t)(16 * r) * P;
          } else {
            o = live ? out + ((int64_t)so * 4) * P + p0 : trash + 4 * l;
            qstride = live ? P : 0;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const v4f v = {pv[q][0], pv[q][1], pv[q][2], pv[q][3]};
            store4<NT>(o + q * qstride, v);
          }
          if (sums) {
            // phase screens store (cos, sin) twice: sum the planes once
            // (the flush doubles the total)
#pragma unroll
            for (int q = 0; q < (GAIN ? 4 : 2); ++q)
#pragma unroll
              for (int t = 0; t < kTiles; ++t) cs += fbits(pv[q][t]);
            if constexpr (!kDirect) cs = live ? cs : 0u;
          }
        } else {
          float* o = out + ((int64_t)so * 4) * P + p0;
#pragma unroll
          for (int t = 0; t < kTiles; ++t) {
            if (p0 + t < P) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                o[q * P + t] = pv[q][t];
                if (sums) cs += fbits(pv[q][t]);
              }
            }
          }
        }
        if (sums) part[r] = cs;  // the 16 lanes of the row sum it below
      };
      auto rows_out = [&](auto be_tag) {
#pragma unroll
        for (int r = 0; r < 4; ++r) row_out(r, be_tag);
      };
      if constexpr (BEM == 1) {
        rows_out(std::true_type{});
      } else if constexpr (BEM == 0) {
        rows_out(std::false_type{});
      } else if (be) {
        rows_out(std::true_type{});
      } else {
        rows_out(std::false_type{});
      }
      if (sums) {
        const unsigned tot = row_sum16_x4(part, l & 15);
        if ((l & 3) == gq) {
          pend = tot;
          pslot = (uint32_t)(s0 + 4 * ((l >> 2) & 3) + (l >> 4));
        }
        if (++gq == 4) flush_sums();
      }
      if constexpr (!IC) {
        coef_finish<KS>(af, rf, s1, S, D, l, kInv2Pi);
        if constexpr (kMagic) safe = group_rev_safe<KS>(af, rev_thr);
        if constexpr (GAIN) {
          coef_finish<KS>(ax, rx, s1, S, D, l, sx);
          coef_finish<KS>(ay, ry, s1, S, D, l, sx);
        }
      }
    }
    if (sums) flush_sums();
  }  // workgroup walk
}

// LDS-staged variant (phase screens, fast sincos epilogue): the same MFMA
// contraction, but the stores are re-mapped so that one wave writes long
// contiguous runs.  A workgroup of NW waves covers RUN = 64*NW consecutive
// pixels; per 16-slot group every wave drops its 16 x 64 reduced phases
// (rev_reduce: fp32 revolutions, exactly the value the register-tile
// kernel feeds to v_sin / v_cos) into LDS, and after one
// barrier wave w takes slots w*16/NW.. and, per slot, sweeps the RUN pixels
// plane by plane: RUN*4 contiguous bytes per (slot, plane) instead of 256 B.
// The LDS tile is double-buffered, so one barrier per group suffices (a
// wave reaches the barrier of group g only after reading group g-1).
// TPW = MFMA tiles per wave: 4 (the wave owns a whole 64-pixel block, as in
// the register-tile kernel) or 2 (two waves share a block, each holding half
// of its Cpix fragments -- half the registers, for large D).
// GAIN (round 6): the tile holds three fp32 planes per value -- the reduced
// phase, log2 A_XX and log2 A_YY, exactly the values the register tile feeds
// to v_sin / v_cos and v_exp_f32 -- and the store waves run the whole gain
// epilogue.  Two buffers (one barrier per group) while they fit the 160 KiB
// of LDS, else one buffer and a second barrier once every wave has read it.
template <int NW, int TPW, bool GAIN = false>
struct EvalLds {
  static constexpr int kWavesPerBlock = kTiles / TPW;
  static constexpr int kRun = kWavePix * NW / kWavesPerBlock;  // pixels per workgroup
  static constexpr int kStride = kRun + 4;      // padded LDS row (floats)
  static constexpr int kSlotsPerWave = 16 / NW;
  static constexpr int kChunks = kRun / 256;    // 1-KiB store runs per plane
  static constexpr int kPlanes = GAIN ? 3 : 1;  // fp32 values per (slot, pixel)
  static constexpr int kBufBytes = kPlanes * 16 * kStride * 4;
  static constexpr int kCsumBytes = 2 * 16 * 16 * 4;
  // gain: one buffer always (the 1-KiB-run shapes then fit 2-3 workgroups
  // per CU instead of 1: double-buffered, every SIMD of the CU ran its
  // contraction and its stores in lockstep, 0.40-0.54 of 8 TB/s)
  static constexpr int kBufs = !GAIN && 2 * kBufBytes + kCsumBytes <= 163840 ? 2 : 1;
  static constexpr bool kFits = kBufs * kBufBytes + kCsumBytes <= 163840;
  static_assert(kRun % 256 == 0 && 16 % NW == 0, "bad LDS eval shape");
};

template <int KS, int NW, int TPW, bool NT, bool IC = false, bool GAIN = false>
__global__ __launch_bounds__(64 * NW) void kl_eval_lds_kernel(
    const double* __restrict__ cfrag, const double* __restrict__ coef,
    const double* __restrict__ coef_xx, const double* __restrict__ coef_yy, int D,
    int ks_real, int64_t S, int64_t P, int64_t n_pb, int64_t n_sc,
    int chunk_groups, float* __restrict__ out, int64_t ring, int64_t ring_base,
    unsigned flags,
    int sleep, unsigned* __restrict__ sums, double rev_thr, DigArgs dg) {
  using L = EvalLds<NW, TPW, GAIN>;
  static_assert(L::kFits, "LDS eval shape exceeds 160 KiB");
  static_assert(!(IC && GAIN), "integer contraction: phase screens");
  // IC: the integer-digit contraction (kl_eval_int.h) feeds the same LDS
  // tile with the same reduced phases as the register tile's IC variant;
  // GAIN: planes [1] / [2] hold log2 A_XX / A_YY
  __shared__ float tile[L::kBufs][L::kPlanes][16][L::kStride];
  // checksums: slot sums of up to 16 groups per half ([half][group % 16]
  // [row]); wave 0 adds a half's 256 consecutive slots with 4 64-lane
  // atomics once the next half has begun, instead of one atomic per (wave,
  // slot) -- atomics run at the memory side, one wave-instruction per ~50 ns
  // per CU
  __shared__ unsigned csum[2][16][16];
  const int l = threadIdx.x & 63;
  // wave index, wave-uniform: keeps slot / ring arithmetic on the SALU
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_blocks = n_pb * n_sc;
  for (int64_t bb = blockIdx.x; bb < n_blocks; bb += gridDim.x) {
    int64_t pb, sc;
    eval_block(bb, n_pb, n_sc, pb, sc, flags);
    if (sc >= n_sc) continue;  // uniform per workgroup
    const int wblk = w / L::kWavesPerBlock;         // 64-pixel block in the run
    const int t0 = (w % L::kWavesPerBlock) * TPW;   // first tile of this wave
    const int64_t wpb = pb * (NW / L::kWavesPerBlock) + wblk;
    const bool live = wpb * kWavePix < P;  // waves past the grid still sync

    double bf[IC ? 1 : KS][TPW];
    if constexpr (!IC) {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
          bf[kk][t] = (live && kk < ks_real)
                          ? cfrag[((wpb * ks_real + kk) * kTiles + t0 + t) * 64 + l]
                          : 0.0;
    }
    v4i bd[TPW][IC ? kDigits : 1];
    if constexpr (IC) {
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int i = 0; i < kDigits; ++i)
          bd[t][i] = live ? dg.cdig[((wpb * kDigits + i) * kTiles + t0 + t) * 64 + l]
                          : v4i{0, 0, 0, 0};
    }

    const bool scrub = flags & SF_EVAL_NAN_SCRUB;
    const bool be = flags & SF_EVAL_BIG_ENDIAN;
    const int64_t pix0 = pb * L::kRun;
    const int64_t slot_base = sc * (int64_t)chunk_groups * 16;
    // wave 0: add the csum entries of groups [g0, g0 + ng) (one half)
    auto flush_sums = [&](int g0, int ng) {
      const unsigned(*cs)[16] = csum[(g0 >> 4) & 1];
      for (int i = l; i < ng * 16; i += 64) {
        const int64_t s = slot_base + (int64_t)g0 * 16 + i;
        if (s < S) atomicAdd(sums + s, cs[i >> 4][i & 15]);
      }
    };
    int ng_done = 0;
    for (int g = 0; g < chunk_groups; ++g) {
      const int64_t s0 = slot_base + (int64_t)g * 16;
      if (s0 >= S) break;  // uniform per workgroup
      ng_done = g + 1;
      const int bi = L::kBufs == 2 ? (g & 1) : 0;
      float(*buf)[L::kStride] = tile[bi][0];
      // ---- contraction: 16 slots x this wave's 64 pixels
      if constexpr (IC) {
        // integer digits; rows the digits cannot carry (bit 4 (l >> 4) + r)
        // take the fp64 contraction, Cpix fragments from memory
        const int rs = dig_row_slot(l);
        DigRows wr;
        dig_load(wr, dg.kdig, s0 + rs, S, l);
        const int64_t sfl = s0 + rs;
        const uint8_t fv = dg.kflag[sfl < S ? sfl : S - 1];
        const unsigned long long bad =
            __builtin_amdgcn_ballot_w64(!(sfl >= S || fv != 0)) & 0xffffull;
        float red[4][TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          const v4i R = dig_contract(wr, bd[t]);
#pragma unroll
          for (int r = 0; r < 4; ++r) red[r][t] = (float)R[r] * kTwoM32;
        }
        if (bad != 0ull && live) {
          const int64_t sa = s0 + (l & 15);
          const double* row = coef + (sa < S ? sa : S - 1) * D;
          v4d ac[TPW];
#pragma unroll
          for (int t = 0; t < TPW; ++t) ac[t] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
          for (int kk = 0; kk < ks_real; ++kk) {
            const int d = 4 * kk + (l >> 4);
            const double a = keep_if(sa < S && d < D, row[d < D ? d : D - 1] * kInv2Pi);
#pragma unroll
            for (int t = 0; t < TPW; ++t)
              ac[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                  a, cfrag[((wpb * ks_real + kk) * kTiles + t0 + t) * 64 + l], ac[t], 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double rv[TPW];
            float f[TPW];
#pragma unroll
            for (int t = 0; t < TPW; ++t) rv[t] = ac[t][r];
            rev_reduce_n<TPW>(f, rv, scrub);
            const bool b = (bad >> (4 * (l >> 4) + r)) & 1ull;
#pragma unroll
            for (int t = 0; t < TPW; ++t) red[r][t] = b ? f[t] : red[r][t];
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* dst = &buf[acc_row(l, r)][wblk * kWavePix + (l & 15) * kTiles + t0];
          if (TPW == 4)
            *reinterpret_cast<v4f*>(dst) =
                v4f{red[r][0], red[r][1 % TPW], red[r][2 % TPW], red[r][3 % TPW]};
          else
            *reinterpret_cast<v2f*>(dst) = v2f{red[r][0], red[r][1 % TPW]};
        }
      } else {
      double af[KS];
      load_coef<KS>(af, coef, s0, S, D, l, kInv2Pi);
      // fixed-point phase accumulators (kRevMagic) while the REAL k-step
      // count (ks_real: KS may be zero-padded) is in the fixed-point range,
      // as the register tile of the same D
      const bool magic = ks_real <= kMagicMaxKS;
      const double a0 = magic ? kRevMagic : 0.0;
      const bool safe = magic && group_rev_safe<KS>(af, rev_thr);
      // gain: the XX / YY log-amplitude coefficients scaled by log2(10), as
      // the register tile's fast path (kLog2of10)
      double ax[GAIN ? KS : 1], ay[GAIN ? KS : 1];
      if constexpr (GAIN) {
        load_coef<KS>(ax, coef_xx, s0, S, D, l, kLog2of10);
        load_coef<KS>(ay, coef_yy, s0, S, D, l, kLog2of10);
      }
      v4d acc[TPW];
      v4d accx[GAIN ? TPW : 1], accy[GAIN ? TPW : 1];
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] = v4d{a0, a0, a0, a0};
      if constexpr (kEnergyDiag == 3) {
        // energy diagnostic: no contraction (the LDS tile, barrier and
        // stores stay)
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = v4d{af[0], af[0], bf[0][t], bf[0][t]};
        if constexpr (GAIN) {
#pragma unroll
          for (int t = 0; t < TPW; ++t) accx[t] = accy[t] = acc[t];
        }
      } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[kk], bf[kk][t],
                                                        acc[t], 0, 0, 0);
      }
      const int col = wblk * kWavePix + (l & 15) * kTiles + t0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float red[TPW];
        double rv[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) rv[t] = acc[t][r];
        // gain screens scrub the products (the store side), not the phase
        rev_reduce_magic<TPW>(red, rv, safe, a0, !GAIN && scrub);
        float* dst = &buf[acc_row(l, r)][col];
        if (TPW == 4)
          *reinterpret_cast<v4f*>(dst) = v4f{red[0], red[1], red[2 % TPW], red[3 % TPW]};
        else
          *reinterpret_cast<v2f*>(dst) = v2f{red[0], red[1 % TPW]};
      }
      if constexpr (GAIN && kEnergyDiag != 3) {
        // the log-amplitude contractions after the phase one is in LDS (its
        // accumulators free again): the same products in the same order per
        // accumulator as the register tile (kl_eval_kernel GAIN), the same bits
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          accx[t] = v4d{0.0, 0.0, 0.0, 0.0};
          accy[t] = v4d{0.0, 0.0, 0.0, 0.0};
        }
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            accx[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ax[kk], bf[kk][t], accx[t], 0, 0, 0);
            accy[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ay[kk], bf[kk][t], accy[t], 0, 0, 0);
          }
      }
      if constexpr (GAIN) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // log2 A rounded to float: amp2f's argument
          float lx[TPW], ly[TPW];
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            lx[t] = (float)accx[t][r];
            ly[t] = (float)accy[t][r];
          }
          float* dx = &tile[bi][GAIN ? 1 : 0][acc_row(l, r)][col];
          float* dy = &tile[bi][GAIN ? 2 : 0][acc_row(l, r)][col];
          if (TPW == 4) {
            *reinterpret_cast<v4f*>(dx) = v4f{lx[0], lx[1 % TPW], lx[2 % TPW], lx[3 % TPW]};
            *reinterpret_cast<v4f*>(dy) = v4f{ly[0], ly[1 % TPW], ly[2 % TPW], ly[3 % TPW]};
          } else {
            *reinterpret_cast<v2f*>(dx) = v2f{lx[0], lx[1 % TPW]};
            *reinterpret_cast<v2f*>(dy) = v2f{ly[0], ly[1 % TPW]};
          }
        }
      }
      }  // fp64 contraction
      for (int z = 0; z < sleep; ++z) __builtin_amdgcn_s_sleep(1);
      __syncthreads();
      // every wave wrote its sums of groups < g before this barrier
      if (sums && w == 0 && g >= 16 && (g & 15) == 0) flush_sums(g - 16, 16);
      // ---- stores: wave w owns kSlotsPerWave slots of the group
      // BE (FITS byte order) as a compile-time branch of a whole slot
      auto slot_out = [&](int j, auto be_tag) {
        constexpr bool kBE = decltype(be_tag)::value;
        const int row = w * L::kSlotsPerWave + j;
        const int64_t s = s0 + row;
        if (s >= S) return;  // uniform per wave
        float cv[L::kChunks][4], sv[L::kChunks][4];
#pragma unroll
        for (int c = 0; c < L::kChunks; ++c) {
          const v4f rv = *reinterpret_cast<const v4f*>(&buf[row][c * 256 + 4 * l]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float sn, cs;
            if constexpr (kEnergyDiag == 3) {
              sn = rv[e];  // energy diagnostic: no sincos
              cs = -rv[e];
            } else {
              sincos_rev(rv[e], sn, cs);
            }
            if (kBE) {
              cs = bswapf(cs);
              sn = bswapf(sn);
            }
            cv[c][e] = cs;
            sv[c][e] = sn;
          }
        }
        // S, ring < 2^31 (launch_eval): 32-bit scalar modulo
        const int64_t so = (uint32_t)(s + ring_base) % (uint32_t)ring;
        float* o = out + (so * 4) * P + pix0 + 4 * l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int c = 0; c < L::kChunks; ++c) {
            if (pix0 + c * 256 + 4 * l < P) {
              const v4f v = (q & 1) ? v4f{sv[c][0], sv[c][1], sv[c][2], sv[c][3]}
                                    : v4f{cv[c][0], cv[c][1], cv[c][2], cv[c][3]};
              store4<NT>(o + q * P + c * 256, v);
            }
          }
        }
        if (sums) {
          // planes 0 / 2 hold cos, 1 / 3 sin: every value is stored twice
          unsigned cs = 0u;
#pragma unroll
          for (int c = 0; c < L::kChunks; ++c)
            if (pix0 + c * 256 + 4 * l < P)
#pragma unroll
              for (int e = 0; e < 4; ++e) cs += fbits(cv[c][e]) + fbits(sv[c][e]);
          cs = row_sum16(2u * cs);
          // the 4 row totals, uniform (scalar) values
          const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)cs, 0) +
                               (unsigned)__builtin_amdgcn_readlane((int)cs, 16) +
                               (unsigned)__builtin_amdgcn_readlane((int)cs, 32) +
                               (unsigned)__builtin_amdgcn_readlane((int)cs, 48);
          if (l == 0) csum[(g >> 4) & 1][g & 15][row] = tot;
        }
      };
      if constexpr (GAIN) {
        // this wave's values of the group, read before any is used: with one
        // buffer the next group's writes wait at a second barrier for every
        // wave's reads, not for its stores
        v4f rph[L::kSlotsPerWave][L::kChunks], rlx[L::kSlotsPerWave][L::kChunks],
            rly[L::kSlotsPerWave][L::kChunks];
#pragma unroll
        for (int j = 0; j < L::kSlotsPerWave; ++j) {
          const int row = w * L::kSlotsPerWave + j;
#pragma unroll
          for (int c = 0; c < L::kChunks; ++c) {
            rph[j][c] = *reinterpret_cast<const v4f*>(&tile[bi][0][row][c * 256 + 4 * l]);
            rlx[j][c] = *reinterpret_cast<const v4f*>(&tile[bi][GAIN ? 1 : 0][row][c * 256 + 4 * l]);
            rly[j][c] = *reinterpret_cast<const v4f*>(&tile[bi][GAIN ? 2 : 0][row][c * 256 + 4 * l]);
          }
        }
        if constexpr (L::kBufs == 1) __syncthreads();
        // the register tile's gain epilogue (fast path) value for value:
        // A = v_exp_f32 of log2 A, fp32 A x cos / sin, per-value NaN scrub
        // of the products (screen.py:368-378), byte swap, 4 distinct planes
        auto gain_out = [&](int j, auto be_tag) {
          constexpr bool kBE = decltype(be_tag)::value;
          const int row = w * L::kSlotsPerWave + j;
          const int64_t s = s0 + row;
          if (s >= S) return;  // uniform per wave
          const int64_t so = (uint32_t)(s + ring_base) % (uint32_t)ring;
          float* o = out + (so * 4) * P + pix0 + 4 * l;
          unsigned cs = 0u;
          // one 1-KiB chunk per plane at a time (fewer live registers)
#pragma unroll
          for (int c = 0; c < L::kChunks; ++c) {
            float pv[4][4];
            bool bad = false;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float sn, cn, xa, ya;
              if constexpr (kEnergyDiag == 3) {
                // energy diagnostic: stores only (no sincos / exp2)
                sn = rph[j][c][e];
                cn = -sn;
                xa = rlx[j][c][e];
                ya = rly[j][c][e];
              } else {
                sincos_rev(rph[j][c][e], sn, cn);
                xa = __builtin_amdgcn_exp2f(rlx[j][c][e]);
                ya = __builtin_amdgcn_exp2f(rly[j][c][e]);
              }
              pv[0][e] = xa * cn;
              pv[1][e] = xa * sn;
              pv[2][e] = ya * cn;
              pv[3][e] = ya * sn;
              bad |= __builtin_isunordered(pv[0][e], pv[1][e]) |
                     __builtin_isunordered(pv[2][e], pv[3][e]);
            }
            if (scrub && __builtin_amdgcn_ballot_w64(bad) != 0) {
#pragma unroll
              for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  if (isnan(pv[q][e])) pv[q][e] = (q & 1) ? 0.0f : 1.0f;
            }
            if (kBE) {
#pragma unroll
              for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) pv[q][e] = bswapf(pv[q][e]);
            }
            if (pix0 + c * 256 + 4 * l < P) {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                store4<NT>(o + q * P + c * 256, v4f{pv[q][0], pv[q][1], pv[q][2], pv[q][3]});
              // checksum of the stored words (all four planes differ)
              if (sums) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                  for (int e = 0; e < 4; ++e) cs += fbits(pv[q][e]);
              }
            }
          }
          if (sums) {
            cs = row_sum16(cs);
            const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)cs, 0) +
                                 (unsigned)__builtin_amdgcn_readlane((int)cs, 16) +
                                 (unsigned)__builtin_amdgcn_readlane((int)cs, 32) +
                                 (unsigned)__builtin_amdgcn_readlane((int)cs, 48);
            if (l == 0) csum[(g >> 4) & 1][g & 15][row] = tot;
          }
        };
        if (be) {
#pragma unroll
          for (int j = 0; j < L::kSlotsPerWave; ++j) gain_out(j, std::true_type{});
        } else {
#pragma unroll
          for (int j = 0; j < L::kSlotsPerWave; ++j) gain_out(j, std::false_type{});
        }
      } else if (be) {
#pragma unroll
        for (int j = 0; j < L::kSlotsPerWave; ++j) slot_out(j, std::true_type{});
      } else {
#pragma unroll
        for (int j = 0; j < L::kSlotsPerWave; ++j) slot_out(j, std::false_type{});
      }
    }
    // the next workgroup item reuses the LDS tiles from buffer 0
    __syncthreads();
    if (sums) {
      // the last (partial) half: every wave's sums are in after the barrier
      if (w == 0 && ng_done > 0) {
        const int g0 = ((ng_done - 1) >> 4) << 4;
        flush_sums(g0, ng_done - g0);
      }
      __syncthreads();  // before a next item's waves write csum again
    }
  }  // workgroup walk
}

// Grid of an eval launch: one workgroup per (pixel block, slot chunk) up to
// the dispatch limit of 2^32 work-items (kept at 2^31), a multiple of 8 so
// the XCD mapping of eval_block holds for every item a workgroup walks.
inline int64_t eval_grid(const sf_ctx* ctx, int64_t n_pb, int64_t n_sc,
                         int threads) {
  int64_t n = n_pb * n_sc;
  if ((n_pb & 7) == 0) n = ((n + 7) / 8) * 8;
  int64_t cap = ((int64_t)1 << 31) / threads;
  if (ctx->eval_max_blocks > 0 && ctx->eval_max_blocks < cap)
    cap = ctx->eval_max_blocks;
  cap = cap < 8 ? 8 : cap & ~(int64_t)7;
  return n < cap ? n : cap;
}

// 16-slot groups per (pixel block, slot chunk) work item: as many as keep
// >= min_items items (the grid fills the chip), at most max_groups
// (SF_OPT_EVAL_GROUPS, else 64 for the register tile, 16 for the LDS-staged
// kernels).  Every item loads its pixel block's Cpix fragments once, so long
// chunks keep that reload small against the item's output: at 512^2 x D = 50
// the Cpix of one XCD's pixel blocks (13.6 MB) outgrows its 4 MiB L2, and 16
// groups per item re-read 3.6 TB of it per 8.2 M-slot launch (FETCH_SIZE,
// 10 % of the writes; 64 groups: 0.9 TB, +2 %); at 256^2 x D = 20 the slices
// stay in L2 and 16 groups keep each XCD's coefficient rows there too
// (profiles/round2e_eval_groups_ab.txt, round2f_eval_groups_bench.txt).
inline int eval_chunk_groups(int64_t n_pb, int64_t S, int max_groups,
                             int64_t min_items) {
  int groups = max_groups;
  while (groups > 1 && n_pb * ((S + 16 * groups - 1) / (16 * groups)) < min_items)
    groups >>= 1;
  return groups;
}


// Slots per launch that keep one workgroup per work item: the dispatch caps
// a grid at 2^31 work-items (eval_grid); past that the workgroups would walk
// several items each, which measured 3-8 % slower than one-shot workgroups
// dispatched in slot order (profiles/round2k_eval_split.txt), so a call
// longer than that is split into consecutive launches.
inline int64_t eval_launch_slots(const sf_ctx* ctx, int64_t n_pb, int groups,
                                 int threads) {
  int64_t cap = ((int64_t)1 << 31) / threads;
  if (ctx->eval_max_blocks > 0) return INT64_MAX;  // the walk test keeps one launch
  const int64_t chunks = cap / n_pb;
  return (chunks < 1 ? 1 : chunks) * 16 * groups;
}

template <int KS, int MINW>
int launch_eval_ks(sf_ctx* ctx, const double* coef,
                          const double* cxx, const double* cyy, int64_t S_all,
                          float* out, int64_t ring, unsigned flags,
                          unsigned* sums) {
  const int64_t P = ctx->n_pix;
  const int64_t n_pb = ctx->n_pix_blocks;
  // (64 groups also at 512^2: 8 measured 0.725 vs 0.691 of 8 TB/s in
  // tools/eval_variants.py but 0.703 vs 0.714 in the config-5 bench step,
  // profiles/round3y_eval_items_512.txt, round3ad_c5_fp64_g8.json)
  const int groups = eval_chunk_groups(n_pb, S_all, ctx->eval_groups ? ctx->eval_groups : 64, 2048);
  const int64_t per = eval_launch_slots(ctx, n_pb, groups, 256);
  // large grids (>= 1024 blocks of 256 px: 512^2 and up): auto bands of 128
  // blocks with the XCD-interleaved map -- 512^2 x D = 50 0.706 -> 0.732 of
  // 8 TB/s; 2, 4 or 16 bands and the contiguous map measured no better
  // (profiles/round2u_eval_bands.txt)
  const int auto_bands = n_pb >= 1024 ? (int)(n_pb / 128 < 128 ? n_pb / 128 : 128) : 1;
  unsigned fl = flags | eval_band_flags(ctx, n_pb, auto_bands);
  if (ctx->eval_xcd_map < 0 && ctx->eval_bands == 0 && auto_bands > 1)
    fl |= kEvalXcdInterleave;
  for (int64_t b = 0; b < S_all; b += per) {
  const int64_t S = S_all - b < per ? S_all - b : per;
  const int64_t n_sc = (S + 16 * groups - 1) / (16 * groups);
  const int64_t nblk = eval_grid(ctx, n_pb, n_sc, 256);
  const double* cb = coef + b * ctx->D;
  const double* cxb = cxx ? cxx + b * ctx->D : nullptr;
  const double* cyb = cyy ? cyy + b * ctx->D : nullptr;
  unsigned* sb = sums ? sums + b : nullptr;
  const bool vec4 = (P % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  const bool fast = flags & SF_EVAL_FAST_SINCOS;
  const bool nt = flags & SF_EVAL_NT_STORES;
  const bool gain = cxx != nullptr;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  // float4 + fast sincos, 64-pixel blocks inside the grid and a ring of
  // whole 16-slot groups: the direct-addressing kernel over the whole groups
  // of the launch, the general one over a ragged tail (< 16 slots)
  // (up to D = 44: at D = 50 it measured 2 % slower, like the fixed-point
  // reduction -- profiles/round3o_eval_direct_ab.txt)
  const bool direct = KS <= kMagicMaxKS && vec4 && fast && P % kWavePix == 0 &&
                      ring % 16 == 0 && (b % ring) % 16 == 0;
  const int64_t S_dir = direct ? (S & ~(int64_t)15) : 0;
#define SF_LAUNCH_BD(V, F, N, G, B, DIR, SL, NSC, NBLK, OFF)                   \
  hipLaunchKernelGGL((kl_eval_kernel<KS, MINW, V, F, N, G, false, B, DIR>),     \
                     dim3((unsigned)(NBLK)), dim3(256), 0, ctx->stream,         \
                     ctx->d_cfrag, cb + (OFF) * ctx->D,                        \
                     cxb ? cxb + (OFF) * ctx->D : nullptr,                     \
                     cyb ? cyb + (OFF) * ctx->D : nullptr, ctx->D, SL, P, n_pb, \
                     NSC, groups, out, ring, (b + (OFF)) % ring, fl,           \
                     sb ? sb + (OFF) : nullptr, ctx->d_trash, ctx->rev_thr, DigArgs{})
#define SF_LAUNCH_B(V, F, N, G, B)                                              \
  do {                                                                          \
    if constexpr (KS <= kMagicMaxKS) {                                          \
      if (S_dir > 0) {                                                          \
        const int64_t nsc_d = (S_dir + 16 * groups - 1) / (16 * groups);        \
        SF_LAUNCH_BD(V, F, N, G, B, true, S_dir, nsc_d,                        \
                     eval_grid(ctx, n_pb, nsc_d, 256), (int64_t)0);            \
      }                                                                         \
    }                                                                           \
    if (S > S_dir) {                                                            \
      const int64_t nsc_t = (S - S_dir + 16 * groups - 1) / (16 * groups);      \
      SF_LAUNCH_BD(V, F, N, G, B, false, S - S_dir, nsc_t,                     \
                   eval_grid(ctx, n_pb, nsc_t, 256), S_dir);                   \
    }                                                                           \
  } while (0)
#define SF_LAUNCH(V, F, N, G) \
  SF_LAUNCH_BD(V, F, N, G, 2, false, S, n_sc, nblk, (int64_t)0)
#define SF_LAUNCH_G(V, F, N) \
  do {                       \
    if (gain)                \
      SF_LAUNCH(V, F, N, true); \
    else                     \
      SF_LAUNCH(V, F, N, false); \
  } while (0)
  // float4 + fast sincos (every hot call): the byte order compiled in
#define SF_LAUNCH_GB(N)                                  \
  do {                                                   \
    if (gain) {                                          \
      if (be) SF_LAUNCH_B(true, true, N, true, 1);       \
      else SF_LAUNCH_B(true, true, N, true, 0);          \
    } else {                                             \
      if (be) SF_LAUNCH_B(true, true, N, false, 1);      \
      else SF_LAUNCH_B(true, true, N, false, 0);         \
    }                                                    \
  } while (0)
  if (vec4) {
    if (fast) {
      if (nt) SF_LAUNCH_GB(true); else SF_LAUNCH_GB(false);
    } else {
      if (nt) SF_LAUNCH_G(true, false, true); else SF_LAUNCH_G(true, false, false);
    }
  } else {
    if (fast) SF_LAUNCH_G(false, true, false); else SF_LAUNCH_G(false, false, false);
  }
#undef SF_LAUNCH_GB
#undef SF_LAUNCH_G
#undef SF_LAUNCH
#undef SF_LAUNCH_B
#undef SF_LAUNCH_BD
  SF_HIP(hipGetLastError());
  }
  return SF_OK;
}

// SHB register tile (phase screens, float4-aligned output): one workgroup
// per (64-pixel wave block, chunk of 4 x 16 groups of 16 slots)
template <int KS>
int launch_eval_shb(sf_ctx* ctx, const double* coef, int64_t S_all,
                           float* out, int64_t ring, unsigned flags,
                           unsigned* sums) {
  const int64_t P = ctx->n_pix;
  const int64_t n_wpb = ctx->n_pix_blocks * kEvalWaves;
  const int groups = eval_chunk_groups(n_wpb, S_all, ctx->eval_groups ? ctx->eval_groups : 64, 4096);
  const int64_t per = eval_launch_slots(ctx, n_wpb, groups, 256);
  for (int64_t b = 0; b < S_all; b += per) {
  const int64_t S = S_all - b < per ? S_all - b : per;
  const int64_t n_sc = (S + 16 * groups - 1) / (16 * groups);
  const int64_t nblk = eval_grid(ctx, n_wpb, n_sc, 256);
  const double* cb = coef + b * ctx->D;
  unsigned* sb = sums ? sums + b : nullptr;
  const bool fast = flags & SF_EVAL_FAST_SINCOS;
  const bool nt = flags & SF_EVAL_NT_STORES;
#define SF_LAUNCH_SHB(F, N)                                                     \
  hipLaunchKernelGGL((kl_eval_kernel<KS, 4, true, F, N, false, true>),          \
                     dim3((unsigned)nblk), dim3(256), 0, ctx->stream,           \
                     ctx->d_cfrag, cb, nullptr, nullptr, ctx->D, S, P, n_wpb, \
                     n_sc, groups, out, ring, b % ring,                         \
                     flags | eval_band_flags(ctx, n_wpb), sb, ctx->d_trash,     \
                     ctx->rev_thr, DigArgs{})
  if (fast) {
    if (nt) SF_LAUNCH_SHB(true, true); else SF_LAUNCH_SHB(true, false);
  } else {
    if (nt) SF_LAUNCH_SHB(false, true); else SF_LAUNCH_SHB(false, false);
  }
#undef SF_LAUNCH_SHB
  SF_HIP(hipGetLastError());
  }
  return SF_OK;
}

// Slots per launch of the integer contraction: its per-slot digit rows
// (384 B) live in a context buffer of at most this many slots; launches of
// 1 M slots are ~0.7 s at 512^2 x D = 50, so the cut costs no measurable tail
constexpr int64_t kDigChunk = (int64_t)1 << 20;

inline int ensure_kdig(sf_ctx* ctx, int64_t slots) {
  if (ctx->kdig_slots >= slots) return SF_OK;
  // (hipFree waits for the device, so no reader of the old buffers remains)
  (void)hipFree(ctx->d_kdig);
  (void)hipFree(ctx->d_kflag);
  ctx->d_kdig = nullptr;
  ctx->d_kflag = nullptr;
  ctx->kdig_slots = 0;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->d_kdig), (size_t)slots * kDigits * 64) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&ctx->d_kflag), (size_t)slots) != hipSuccess) {
    set_error("sf_kl_eval: hipMalloc of the integer-contraction digits failed");
    return SF_ENOMEM;
  }
  ctx->kdig_slots = slots;
  return SF_OK;
}

// Prepass of one integer-contraction launch: the digit rows and flags of S
// slots.  The buffers are the context's, so a launch on another stream may
// still be reading them: the prepass waits for the last reader first
// (kdig_read, recorded by kdig_done after every integer launch; on the same
// stream the wait is already satisfied by stream order).
inline int run_kdig(sf_ctx* ctx, const double* cb, int64_t S) {
  if (!ctx->kdig_read)
    SF_HIP(hipEventCreateWithFlags(&ctx->kdig_read, hipEventDisableTiming));
  else
    SF_HIP(hipStreamWaitEvent(ctx->stream, ctx->kdig_read, 0));
  hipLaunchKernelGGL(kl_kdig_kernel<0>, dim3((unsigned)((S + 3) / 4)), dim3(256), 0,
                     ctx->stream, cb, ctx->D, S, kInv2Pi, ctx->d_kdig, ctx->d_kflag);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

// after the launch that read the digits run_kdig wrote
inline int kdig_done(sf_ctx* ctx) {
  SF_HIP(hipEventRecord(ctx->kdig_read, ctx->stream));
  return SF_OK;
}

inline DigArgs dig_args(const sf_ctx* ctx, int64_t off) {
  DigArgs dg;
  dg.cdig = reinterpret_cast<const v4i*>(ctx->d_cdig);
  dg.kdig = ctx->d_kdig + off * kDigits * 64;
  dg.kflag = ctx->d_kflag + off;
  return dg;
}

template <int KS, int NW, int TPW, bool GAIN = false>
int launch_eval_lds(sf_ctx* ctx, const double* coef, const double* cxx,
                    const double* cyy, int64_t S_all, float* out, int64_t ring,
                    unsigned flags, unsigned* sums) {
  const int64_t P = ctx->n_pix;
  const int64_t run = EvalLds<NW, TPW, GAIN>::kRun;
  const int64_t n_pb = (P + run - 1) / run;
  // Small grids (n_pb <= 64: 256^2 and below, pixel blocks dealt to the XCDs
  // interleaved): the shortest items whose Cpix reload (8 x 4 KS bytes per
  // pixel) stays <= ~1/3 of their output (16 x 16 g bytes per pixel):
  // KS <= 2 -> 1 group, 3-5 -> 2, 6-11 -> 4, else 8.  Measured in the bench
  // setting (profiles/round2l_eval_chunks.txt): 256^2 x D = 20 0.72 (16
  // groups) -> 0.79 (2 groups) of 8 TB/s, 1 group 0.67; 128^2 x D = 7 0.61
  // -> 0.75 (1 group).  Larger grids keep 16 (their Cpix outgrows L2 and the
  // long items won at 512^2, round2k_eval_split.txt).
  const int def_groups = n_pb > 64 ? 16 : KS <= 2 ? 1 : KS <= 5 ? 2 : KS <= 11 ? 4 : 8;
  const int groups = eval_chunk_groups(n_pb, S_all,
                                       ctx->eval_groups ? ctx->eval_groups : def_groups, 1024);
  int64_t per = eval_launch_slots(ctx, n_pb, groups, 64 * NW);
  // the integer-digit contraction: per-launch slot digits (run_kdig), at
  // most kDigChunk slots per launch
  const bool ic = !GAIN && eval_int_applies(ctx, false, flags,
                                            (reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (ic) {
    const int64_t gs = 16 * (int64_t)groups;
    const int64_t cap = kDigChunk < gs ? gs : (kDigChunk / gs) * gs;
    if (per > cap) per = cap;
    const int rc = ensure_kdig(ctx, S_all < per ? S_all : per);
    if (rc != SF_OK) return rc;
  }
  for (int64_t b = 0; b < S_all; b += per) {
  const int64_t S = S_all - b < per ? S_all - b : per;
  const int64_t n_sc = (S + 16 * groups - 1) / (16 * groups);
  const int64_t nblk = eval_grid(ctx, n_pb, n_sc, 64 * NW);
  const double* cb = coef + b * ctx->D;
  const double* cxb = GAIN ? cxx + b * ctx->D : nullptr;
  const double* cyb = GAIN ? cyy + b * ctx->D : nullptr;
  unsigned* sb = sums ? sums + b : nullptr;
  if (ic) {
    const int rc = run_kdig(ctx, cb, S);
    if (rc != SF_OK) return rc;
  }
  // auto XCD map: interleave the pixel blocks over the XCDs when each XCD's
  // contiguous eighth would be <= 8 blocks (measured: 256^2 at 4 KiB runs
  // +2-3 %, 512^2 -3 %; profiles/round1e_eval_xcd_map.txt)
  unsigned fl = flags;
  if (ctx->eval_xcd_map < 0 && (n_pb & 7) == 0 && n_pb / 8 <= 8)
    fl |= kEvalXcdInterleave;
  fl |= eval_band_flags(ctx, n_pb);
#define SF_LAUNCH_LDS(N, I)                                                             \
  hipLaunchKernelGGL((kl_eval_lds_kernel<KS, NW, TPW, N, I, GAIN>), dim3((unsigned)nblk), \
                     dim3(64 * NW), 0, ctx->stream, ctx->d_cfrag, cb, cxb, cyb, ctx->D,   \
                     ctx->ksteps, S, P, n_pb, n_sc, groups, out, ring, b % ring, fl,      \
                     ctx->eval_sleep, sb, ctx->rev_thr, I ? dig_args(ctx, 0) : DigArgs{})
  // (the integer variant only where it can apply: D >= 45)
  if (ic) {
    if constexpr (KS >= 12 && !GAIN) {
      if (flags & SF_EVAL_NT_STORES) SF_LAUNCH_LDS(true, true);
      else SF_LAUNCH_LDS(false, true);
    }
  } else {
    if (flags & SF_EVAL_NT_STORES) SF_LAUNCH_LDS(true, false);
    else SF_LAUNCH_LDS(false, false);
  }
#undef SF_LAUNCH_LDS
  SF_HIP(hipGetLastError());
  if (ic) {
    const int rc = kdig_done(ctx);
    if (rc != SF_OK) return rc;
  }
  }
  return SF_OK;
}

// The register tile on the integer-digit contraction (phase, D >= 45);
// NWV = 4 (256-pixel workgroup blocks) or 8 (512, SF_OPT_EVAL_WG_WAVES)
template <int KS, int NWV>
int launch_eval_int_nw(sf_ctx* ctx, const double* coef, int64_t S_all, float* out,
                       int64_t ring, unsigned flags, unsigned* sums) {
  const int64_t P = ctx->n_pix;
  constexpr int kThreads = 64 * NWV;
  // workgroup pixel blocks of NWV x 64 pixels (the wave blocks of the Cpix /
  // digit fragments are 64 pixels either way)
  const int64_t n_pb = (ctx->n_pix_blocks * kEvalWaves + NWV - 1) / NWV;
  const int64_t n_pb256 = ctx->n_pix_blocks;
  // large grids (>= 1024 blocks of 256 px: 512^2 and up): items of 4 groups
  // (the digit fragments are 6 KB per wave block, a quarter of the fp64 ones,
  // so short items cost little reload): 512^2 x D = 50 0.691 (64 groups) ->
  // 0.744 of 8 TB/s, 2 / 8 groups 0.723 / 0.731
  // (profiles/round3y_eval_items_512.txt)
  const int def_groups = n_pb256 >= 1024 ? 4 : 64;
  const int groups = eval_chunk_groups(n_pb, S_all, ctx->eval_groups ? ctx->eval_groups : def_groups,
                                       2048 * kEvalWaves / NWV);
  const int64_t gs = 16 * (int64_t)groups;
  int64_t per = eval_launch_slots(ctx, n_pb, groups, kThreads);
  const int64_t cap = kDigChunk < gs ? gs : (kDigChunk / gs) * gs;
  if (per > cap) per = cap;
  {
    const int rc = ensure_kdig(ctx, S_all < per ? S_all : per);
    if (rc != SF_OK) return rc;
  }
  // bands / XCD map as the fp64 register tile (launch_eval_ks): bands of
  // 128 x 256 pixels
  const int auto_bands = n_pb256 >= 1024 ? (int)(n_pb256 / 128 < 128 ? n_pb256 / 128 : 128) : 1;
  unsigned fl = flags | eval_band_flags(ctx, n_pb, auto_bands);
  if (ctx->eval_xcd_map < 0 && ctx->eval_bands == 0 && auto_bands > 1)
    fl |= kEvalXcdInterleave;
  const bool nt = flags & SF_EVAL_NT_STORES;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  for (int64_t b = 0; b < S_all; b += per) {
    const int64_t S = S_all - b < per ? S_all - b : per;
    const double* cb = coef + b * ctx->D;
    unsigned* sb = sums ? sums + b : nullptr;
    {
      const int rc = run_kdig(ctx, cb, S);
      if (rc != SF_OK) return rc;
    }
    // (direct addressing: measured 2 % slower at D = 50 with fp64, not used)
    const int64_t nsc = (S + gs - 1) / gs;
    const unsigned nblk = (unsigned)eval_grid(ctx, n_pb, nsc, kThreads);
#define SF_LAUNCH_IC(N, B)                                                                 \
  hipLaunchKernelGGL((kl_eval_kernel<KS, 2, true, true, N, false, false, B, false, true, NWV>), \
                     dim3(nblk), dim3(kThreads), 0, ctx->stream, ctx->d_cfrag, cb, nullptr,     \
                     nullptr, ctx->D, S, P, n_pb, nsc, groups, out, ring, b % ring, fl,         \
                     sb, ctx->d_trash, ctx->rev_thr, dig_args(ctx, 0))
    if constexpr (KS >= 12) {
      if (nt) {
        if (be) SF_LAUNCH_IC(true, 1); else SF_LAUNCH_IC(true, 0);
      } else {
        if (be) SF_LAUNCH_IC(false, 1); else SF_LAUNCH_IC(false, 0);
      }
    }
#undef SF_LAUNCH_IC
    SF_HIP(hipGetLastError());
    {
      const int rc = kdig_done(ctx);
      if (rc != SF_OK) return rc;
    }
  }
  return SF_OK;
}

template <int KS>
int launch_eval_int(sf_ctx* ctx, const double* coef, int64_t S_all, float* out,
                    int64_t ring, unsigned flags, unsigned* sums) {
  if (ctx->eval_wg_waves == 8)
    return launch_eval_int_nw<KS, 8>(ctx, coef, S_all, out, ring, flags, sums);
  return launch_eval_int_nw<KS, kEvalWaves>(ctx, coef, S_all, out, ring, flags, sums);
}

// The integer-digit contraction on the SHB tile (SF_EVAL_KERNEL_SHB with the
// integer contraction): the 4 waves of a workgroup share one 64-pixel block,
// its pixel digits in LDS, and take its 16-slot groups round-robin
template <int KS>
int launch_eval_int_shb(sf_ctx* ctx, const double* coef, int64_t S_all, float* out,
                        int64_t ring, unsigned flags, unsigned* sums) {
  const int64_t P = ctx->n_pix;
  const int64_t n_wpb = ctx->n_pix_blocks * kEvalWaves;
  // groups per item: 4 per wave (the register tile's 4-group items)
  const int groups = eval_chunk_groups(n_wpb, S_all, ctx->eval_groups ? ctx->eval_groups : 16, 4096);
  const int64_t gs = 16 * (int64_t)groups;
  int64_t per = eval_launch_slots(ctx, n_wpb, groups, 256);
  const int64_t cap = kDigChunk < gs ? gs : (kDigChunk / gs) * gs;
  if (per > cap) per = cap;
  {
    const int rc = ensure_kdig(ctx, S_all < per ? S_all : per);
    if (rc != SF_OK) return rc;
  }
  // pixel bands as the register tile's (bands of 128 x 256 pixels)
  const int64_t n_pb = ctx->n_pix_blocks;
  const int auto_bands = n_pb >= 1024 ? (int)(n_pb / 128 < 128 ? n_pb / 128 : 128) : 1;
  unsigned fl = flags | eval_band_flags(ctx, n_wpb, auto_bands);
  if (ctx->eval_xcd_map < 0 && ctx->eval_bands == 0 && auto_bands > 1)
    fl |= kEvalXcdInterleave;
  const bool nt = flags & SF_EVAL_NT_STORES;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  for (int64_t b = 0; b < S_all; b += per) {
    const int64_t S = S_all - b < per ? S_all - b : per;
    const double* cb = coef + b * ctx->D;
    unsigned* sb = sums ? sums + b : nullptr;
    {
      const int rc = run_kdig(ctx, cb, S);
      if (rc != SF_OK) return rc;
    }
    const int64_t nsc = (S + gs - 1) / gs;
    const unsigned nblk = (unsigned)eval_grid(ctx, n_wpb, nsc, 256);
#define SF_LAUNCH_ICS(N, B)                                                              \
  hipLaunchKernelGGL((kl_eval_kernel<KS, 3, true, true, N, false, true, B, false, true>), \
                     dim3(nblk), dim3(256), 0, ctx->stream, ctx->d_cfrag, cb, nullptr,   \
                     nullptr, ctx->D, S, P, n_wpb, nsc, groups, out, ring, b % ring, fl, \
                     sb, ctx->d_trash, ctx->rev_thr, dig_args(ctx, 0))
    if constexpr (KS >= 12) {
      if (nt) {
        if (be) SF_LAUNCH_ICS(true, 1); else SF_LAUNCH_ICS(true, 0);
      } else {
        if (be) SF_LAUNCH_ICS(false, 1); else SF_LAUNCH_ICS(false, 0);
      }
    }
#undef SF_LAUNCH_ICS
    SF_HIP(hipGetLastError());
    {
      const int rc = kdig_done(ctx);
      if (rc != SF_OK) return rc;
    }
  }
  return SF_OK;
}

template <int KS>
int launch_eval_pick(sf_ctx* ctx, const double* coef, const double* cxx,
                            const double* cyy, int64_t S, float* out,
                            int64_t ring, unsigned flags,
                            unsigned* sums) {
  const bool aligned = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const int v = pick_eval_kernel(ctx, cxx != nullptr, flags, aligned);
  // the integer-digit contraction: the LDS-staged kernels take it themselves,
  // the register tile through launch_eval_int
  if (eval_int_applies(ctx, cxx != nullptr, flags, aligned)) {
    if (v == SF_EVAL_KERNEL_TILE || v == SF_EVAL_KERNEL_TILE3)
      return launch_eval_int<KS>(ctx, coef, S, out, ring, flags, sums);
    if (v == SF_EVAL_KERNEL_SHB)
      return launch_eval_int_shb<KS>(ctx, coef, S, out, ring, flags, sums);
  }
  // gain screens (round 6): the LDS-staged shapes whose three-plane tile
  // fits LDS (pick_eval_kernel maps LDS16 to LDS16H), up to kGainLdsMaxKS
  if (cxx != nullptr) {
    if constexpr (KS <= kGainLdsMaxKS) {
      switch (v) {
        case SF_EVAL_KERNEL_LDS4:
          return launch_eval_lds<KS, 4, 4, true>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
        case SF_EVAL_KERNEL_LDS8:
          return launch_eval_lds<KS, 8, 4, true>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
        case SF_EVAL_KERNEL_LDS8H:
          return launch_eval_lds<KS, 8, 2, true>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
        case SF_EVAL_KERNEL_LDS16H:
          return launch_eval_lds<KS, 16, 2, true>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
        default:
          break;
      }
    }
    // (pick_eval_kernel gives gain screens no other LDS-staged shape)
    if (v != SF_EVAL_KERNEL_TILE && v != SF_EVAL_KERNEL_TILE3) {
      set_error("sf_kl_eval_gain: no LDS-staged gain kernel for this shape");
      return SF_EINVAL;
    }
  }
  switch (v) {
    case SF_EVAL_KERNEL_LDS4:
      return launch_eval_lds<KS, 4, 4>(ctx, coef, nullptr, nullptr, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_LDS8:
      return launch_eval_lds<KS, 8, 4>(ctx, coef, nullptr, nullptr, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_LDS16:
      return launch_eval_lds<KS, 16, 4>(ctx, coef, nullptr, nullptr, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_LDS8H:
      return launch_eval_lds<KS, 8, 2>(ctx, coef, nullptr, nullptr, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_LDS16H:
      return launch_eval_lds<KS, 16, 2>(ctx, coef, nullptr, nullptr, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_SHB:
      return launch_eval_shb<KS>(ctx, coef, S, out, ring, flags, sums);
    case SF_EVAL_KERNEL_TILE3:
      // below 8 k-steps the register tile fits 4 waves/SIMD anyway
      return launch_eval_ks<KS, (KS >= 8 ? 3 : 2)>(ctx, coef, cxx, cyy, S, out,
                                                   ring, flags, sums);
    default:
      return launch_eval_ks<KS, 2>(ctx, coef, cxx, cyy, S, out, ring, flags, sums);
  }
}

#define SF_EVAL_PICK_ARGS                                                    \
  sf_ctx* ctx, const double* coef, const double* cxx, const double* cyy,   \
      int64_t S, float* out, int64_t ring, unsigned flags, unsigned* sums
#define SF_EVAL_KS_LIST(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define SF_EVAL_EXTERN(k) extern template int launch_eval_pick<k>(SF_EVAL_PICK_ARGS);
#define SF_EVAL_INSTANTIATE(k) template int launch_eval_pick<k>(SF_EVAL_PICK_ARGS);

}  // namespace sf

// kl_fit.hip -- shared KL basis and the batched per-slot KL least-squares fit
// (gfx950, float64).
//
// Restates on the GPU (not a translation -- one wavefront per slot, one lane
// per direction, LDS-resident basis) the reference operator
// stationscreen.run (stationscreen.py:858-1161):
//   * kl_basis_kernel   <- _calculate_svd (stationscreen.py:390-430)
//   * kl_skip_kernel    <- the (station, freq) block skip of
//                          _process_single_freq (stationscreen.py:817-825)
//   * kl_fit_kernel     <- _process_station (stationscreen.py:597-782) with
//                          _fit_screen (:433-594), _flag_outliers (:303-350),
//                          _circ_chi2 (:353-387) for one slot per wavefront.
// Every phase slot is independent (see oracle/kl.py for the argument), so a
// slot is the unit of parallelism.
#include <hip/hip_runtime.h>

#include <cmath>

#include "sf_internal.h"
#include "sf_wave.h"

namespace sf {

constexpr double kPinvAtol = 1e-3;  // pinv(rcond=1e-3), scipy>=1.7 semantics
constexpr int kMaxSweeps = 40;

__host__ __device__ inline int odd_ld(int n) { return n | 1; }

// C[i][j] = -(|pp_i - pp_j|^2 / r0^2)^(beta/2) / 2 with numpy's evaluation
// order ((dx^2 + dy^2) + dz^2), no contraction.
__device__ inline double kl_cov(const double* pi, const double* pj,
                                double r0sq, double half_beta) {
#pragma clang fp contract(off)
  const double dx = pi[0] - pj[0];
  const double dy = pi[1] - pj[1];
  const double dz = pi[2] - pj[2];
  const double d2 = (dx * dx + dy * dy) + dz * dz;
  return -pow(d2 / r0sq, half_beta) / 2.0;
}

// ---------------------------------------------------------------------------
// basis: one wavefront. C, eigen-decomposition by Jacobi, U sorted by
// descending |lambda| (= svd(C)[0] up to column signs), pinv with absolute
// cutoff.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void kl_basis_kernel(
    const double* __restrict__ pp, int D, double r0, double beta,
    double* __restrict__ c_out, double* __restrict__ pinv_out,
    double* __restrict__ u_out, double* __restrict__ eig_out) {
  extern __shared__ double smem[];
  const int ld = odd_ld(D);
  double* a = smem;
  double* v = a + D * ld;
  double2* cs = reinterpret_cast<double2*>(v + D * ld);
  int2* pr = reinterpret_cast<int2*>(cs + 64);      // 64 int2 + 64 int
  int* perm = reinterpret_cast<int*>(pr + 96);
  const int i = lane();
  const double r0sq = r0 * r0, hb = beta / 2.0;
  if (i < D) {
    for (int j = 0; j < D; ++j) {
      const double c = kl_cov(pp + 3 * i, pp + 3 * j, r0sq, hb);
      a[i * ld + j] = c;
      c_out[i * D + j] = c;
    }
  }
  lds_sync();
  wave_jacobi(a, v, cs, pr, D, ld, kMaxSweeps);
  wave_eig_order(a, D, ld, perm);
  if (i < D) {
    for (int r = 0; r < D; ++r) u_out[i * D + r] = v[i * ld + perm[r]];
    const int pr = perm[i];
    eig_out[i] = a[pr * ld + pr];
    for (int j = 0; j < D; ++j) {
      double s = 0.0;
      for (int r = 0; r < D; ++r) {
        const int m = perm[r];
        const double lam = a[m * ld + m];
        if (fabs(lam) > kPinvAtol) s += v[i * ld + m] * (v[j * ld + m] / lam);
      }
      pinv_out[i * D + j] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// (station, freq) block skip: all phases NaN after referencing, or all
// weights zero (stationscreen.py:821-825).  One wavefront per block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void kl_skip_kernel(
    const double* __restrict__ phase, const float* __restrict__ weight, int T,
    int F, int A, int D, int ref, const double* __restrict__ refph,
    uint8_t* __restrict__ skip) {
  const int blk = blockIdx.x;  // f * A + a
  const int f = blk / A, a = blk % A;
  const int d = lane();
  bool any_val = false, any_w = false;
  for (int t = 0; t < T; ++t) {
    if (d < D) {
      const int64_t base = ((int64_t)(t * F + f) * A) * D;
      double ph = phase[base + (int64_t)a * D + d];
      if (refph) ph -= refph[(int64_t)(t * F + f) * D + d];
      else if (ref >= 0) ph -= phase[base + (int64_t)ref * D + d];
      any_val |= !isnan(ph);
      any_w |= weight[base + (int64_t)a * D + d] != 0.0f;
    }
    // a block is kept as soon as it has one finite phase and one non-zero
    // weight: stop there (every 8 times, a wave-uniform test)
    if ((t & 7) == 7 && __any(any_val) && __any(any_w)) break;
  }
  const bool av = __any(any_val), aw = __any(any_w);
  if (d == 0) skip[blk] = (!av || !aw) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// per-slot fit
// ---------------------------------------------------------------------------
struct FitLds {
  // shared by the workgroup
  double* C;     // [D][ld]
  double* U;     // [D][ld], columns sorted
  double* eig;   // [64]
  // per wave
  double* V;     // [D][ld] eigenvectors of C_sub (unsorted columns)
  double* M1;    // [D][ld] scratch
  double* M2;    // [D][ld] normal matrix / scratch
  double* lam;   // [64] eigenvalues of C_sub by rank
  double* vec;   // [6][64] broadcast vectors
  int* idx;      // [64] subset -> direction
  int* perm;     // [64] rank -> column of V
  double2* cs;   // [64] Jacobi rotations
  int2* pr;      // [64] + 64 int: Jacobi round pairs / partners
};

__host__ __device__ inline size_t fit_shared_bytes(int D) {
  return (size_t)(2 * D * odd_ld(D) + 64) * sizeof(double);
}
__host__ __device__ inline size_t fit_wave_bytes(int D) {
  return (size_t)(3 * D * odd_ld(D) + 64 + 6 * 64) * sizeof(double) +
         (size_t)(64 + 64) * sizeof(int) + 64 * sizeof(double2) +
         96 * sizeof(int2);
}

struct SubsetState {
  int n;        // number of unflagged directions
  bool full;    // n == D: use the shared basis (quirk Q1)
  double wmin;  // smallest unflagged weight
};

// Cache the basis of the unflagged subset (stationscreen.py:493-499).
__device__ void setup_subset(const FitLds& L, int D, int ld, double w_d,
                             SubsetState& st) {
  const int d = lane();
  const bool unfl = (d < D) && (w_d > 0.0);
  const uint64_t mask = __ballot(unfl);
  const int n = __popcll(mask);
  st.n = n;
  st.full = (n == D);
  double wm = unfl ? w_d : INFINITY;
  wm = -wave_max(-wm);
  st.wmin = wm;
  if (unfl) {
    const int p = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    L.idx[p] = d;
  }
  lds_sync();
  if (st.full) return;  // shared U / eig (already sorted)
  if (n == 0) return;
  // C_sub = C[idx][:, idx], eigen-decomposed in M1 / V
  if (d < n) {
    const int r = L.idx[d];
    for (int q = 0; q < n; ++q) L.M1[d * ld + q] = L.C[r * ld + L.idx[q]];
  }
  lds_sync();
  wave_jacobi(L.M1, L.V, L.cs, L.pr, n, ld, kMaxSweeps);
  wave_eig_order(L.M1, n, ld, L.perm);
  if (d < n) {
    const int m = L.perm[d];
    L.lam[d] = L.M1[m * ld + m];
  }
  lds_sync();
}

// column `rank` of the (sorted) U of the current subset, row p
__device__ __forceinline__ double ucol(const FitLds& L, const SubsetState& st,
                                       int ld, int p, int rank) {
  return st.full ? L.U[p * ld + rank] : L.V[p * ld + L.perm[rank]];
}

// y = pinv(C_sub) x for x held one element per lane (lanes < n), through
// the eigen-decomposition: y = sum_{|lam|>atol} u_r (u_r^T x) / lam_r.
__device__ double apply_pinv(const FitLds& L, const SubsetState& st, int ld,
                             double x, double* vtmp) {
  const int p = lane();
  const int n = st.n;
  if (p < n) vtmp[p] = x;
  lds_sync();
  double t = 0.0;
  if (p < n) {
    for (int q = 0; q < n; ++q) t += ucol(L, st, ld, q, p) * vtmp[q];
    const double lam = st.full ? L.eig[p] : L.lam[p];
    t = (fabs(lam) > kPinvAtol) ? t / lam : 0.0;
  }
  lds_sync();
  if (p < n) vtmp[p] = t;
  lds_sync();
  double y = 0.0;
  if (p < n)
    for (int r = 0; r < n; ++r) y += ucol(L, st, ld, p, r) * vtmp[r];
  lds_sync();
  return y;
}

// full-basis pinv (shared U / eig), x on lanes < D
__device__ double apply_pinv_full(const FitLds& L, int D, int ld, double x,
                                  double* vtmp) {
  SubsetState full{D, true, 0.0};
  return apply_pinv(L, full, ld, x, vtmp);
}

// y_p = sum_q C[idx p][idx q] x_q  (lanes < n)
__device__ double apply_csub(const FitLds& L, int n, int ld, double x,
                             double* vtmp) {
  const int p = lane();
  if (p < n) vtmp[p] = x;
  lds_sync();
  double y = 0.0;
  if (p < n) {
    const int r = L.idx[p];
    for (int q = 0; q < n; ++q) y += L.C[r * ld + L.idx[q]] * vtmp[q];
  }
  lds_sync();
  return y;
}

// One _fit_screen call (stationscreen.py:433-594) at order K.  Inputs per
// direction lane d: phi_d, w_d.  Outputs per direction lane: white_d,
// resid_d.
__device__ void fit_screen(const FitLds& L, const SubsetState& st, int D,
                           int ld, int K, int screen_type, double phi_d,
                           double w_d, double& white_d, double& resid_d) {
#pragma clang fp contract(off)
  const int lp = lane();
  const int n = st.n;
  double* v0 = L.vec;
  double* v1 = L.vec + 64;
  double* v2 = L.vec + 128;
  double* v3 = L.vec + 192;
  // gather the unflagged directions onto lanes p < n
  if (lp < D) {
    v0[lp] = phi_d;
    v1[lp] = w_d;
  }
  lds_sync();
  double phi_p = 0.0, w_p = 0.0;
  if (lp < n) {
    phi_p = v0[L.idx[lp]];
    w_p = v1[L.idx[lp]];
  }
  lds_sync();
  double rc, rs;
  if (screen_type == SF_SCREEN_PHASE) {
    double sn, cn;
    sincos(phi_p, &sn, &cn);
    rc = w_p * cn;   // W cos(phi)
    rs = w_p * sn;   // W sin(phi)
  } else {
    rc = w_p * phi_p;
    rs = 0.0;
  }
  if (lp < n) {
    v0[lp] = rc;
    v1[lp] = rs;
    v2[lp] = w_p;
  }
  lds_sync();
  // rr1 = U_k^T W r  (lane k < K);  G = U_k^T W U_k (row k)
  double g1 = 0.0, g2 = 0.0;
  if (lp < K) {
    for (int p = 0; p < n; ++p) {
      const double u = ucol(L, st, ld, p, lp);
      g1 += u * v0[p];
      g2 += u * v1[p];
    }
    for (int j = 0; j < K; ++j) {
      double s = 0.0;
      for (int p = 0; p < n; ++p)
        s += ucol(L, st, ld, p, lp) * (v2[p] * ucol(L, st, ld, p, j));
      L.M2[lp * ld + j] = s;
    }
  }
  lds_sync();
  // inv_u = pinv(G, atol=1e-3) applied to rr1.  lambda_min(G) >= min w over
  // the unflagged rows (U_k has orthonormal columns over exactly those rows),
  // so for wmin above the cutoff pinv == inverse: Cholesky.  Otherwise the
  // eigen path reproduces the truncation.
  double a1 = g1, a2 = g2;
  if (K > 0) {
    if (st.wmin > kPinvAtol * (1.0 + 1e-9)) {
      wave_cholesky_solve2(L.M2, K, ld, a1, a2);
    } else {
      wave_jacobi(L.M2, L.M1, L.cs, L.pr, K, ld, kMaxSweeps);
      if (lp < K) {
        v0[lp] = g1;
        v1[lp] = g2;
      }
      lds_sync();
      double t1 = 0.0, t2 = 0.0;
      if (lp < K) {
        for (int q = 0; q < K; ++q) {
          t1 += L.M1[q * ld + lp] * v0[q];
          t2 += L.M1[q * ld + lp] * v1[q];
        }
        const double mu = L.M2[lp * ld + lp];
        if (fabs(mu) > kPinvAtol) {
          t1 /= mu;
          t2 /= mu;
        } else {
          t1 = t2 = 0.0;
        }
      }
      lds_sync();
      if (lp < K) {
        v2[lp] = t1;
        v3[lp] = t2;
      }
      lds_sync();
      a1 = a2 = 0.0;
      if (lp < K)
        for (int m = 0; m < K; ++m) {
          a1 += L.M1[lp * ld + m] * v2[m];
          a2 += L.M1[lp * ld + m] * v3[m];
        }
      lds_sync();
    }
  }
  // h = U_k a  (lane p < n)
  if (lp < K) {
    v0[lp] = a1;
    v1[lp] = a2;
  }
  lds_sync();
  double h1 = 0.0, h2 = 0.0;
  if (lp < n)
    for (int k = 0; k < K; ++k) {
      const double u = ucol(L, st, ld, lp, k);
      h1 += u * v0[k];
      h2 += u * v1[k];
    }
  lds_sync();
  double screen;
  if (n == 2 && K == 1) {
    // two unflagged directions: the reference's U_k = e_2 (see fit_once in
    // kl_fit_fast.hip); v0..v2 were overwritten above, so the second
    // direction's terms are gathered again
    if (lp < D) {
      v0[lp] = phi_d;
      v1[lp] = w_d;
    }
    lds_sync();
    const double w2 = v1[L.idx[1]];
    const double ph2 = v0[L.idx[1]];
    lds_sync();
    const double iw = w2 > kPinvAtol ? 1.0 / w2 : 0.0;
    double t_re, t_im = 0.0;
    if (screen_type == SF_SCREEN_PHASE) {
      double sn, cn;
      sincos(ph2, &sn, &cn);
      t_re = iw * (w2 * cn);
      t_im = iw * (w2 * sn);
    } else {
      t_re = iw * (w2 * ph2);
    }
    screen = lp != 1 ? 0.0 : screen_type == SF_SCREEN_PHASE ? atan2(t_im, t_re) : t_re;
  } else if (screen_type == SF_SCREEN_PHASE) {
    const double re = apply_pinv(L, st, ld, h1, v3);
    const double im = apply_pinv(L, st, ld, h2, v3);
    const double cre = apply_csub(L, n, ld, re, v3);
    const double cim = apply_csub(L, n, ld, im, v3);
    screen = atan2(cim, cre);
  } else {
    const double tf = apply_pinv(L, st, ld, h1, v3);
    screen = apply_csub(L, n, ld, tf, v3);
  }
  const double white = apply_pinv(L, st, ld, screen, v3);
  if (st.full) {
    white_d = white;
    const double cw = apply_csub(L, n, ld, white, v3);  // idx = identity
    resid_d = phi_d - cw;
    return;
  }
  // flagged directions: screen from the unflagged white coefficients, then
  // re-whitened with the full pinv (stationscreen.py:565-582)
  if (lp < n) {
    v0[lp] = screen;
    v1[lp] = white;
  }
  lds_sync();
  const bool unfl = (lp < D) && (w_d > 0.0);
  const uint64_t mask = __ballot(unfl);
  double screen_all = 0.0;
  if (lp < D) {
    if (unfl) {
      const int p = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      screen_all = v0[p];
    } else {
      for (int p = 0; p < n; ++p) screen_all += L.C[lp * ld + L.idx[p]] * v1[p];
    }
  }
  lds_sync();
  white_d = apply_pinv_full(L, D, ld, screen_all, v3);
  resid_d = phi_d - screen_all;
}

__global__ __launch_bounds__(256) void kl_fit_general_kernel(
    const int* __restrict__ slot_list, const int* __restrict__ n_list,
    const double* __restrict__ phase, const float* __restrict__ weight,
    int T, int F, int A, int D, const int* __restrict__ st_order,
    const uint8_t* __restrict__ skip, const double* __restrict__ refph,
    const double* __restrict__ g_c,
    const double* __restrict__ g_u, const double* __restrict__ g_eig,
    int screen_type, int niter, double nsigma, int adjust_order, int ref,
    int ref_skip, double* __restrict__ coef, double* __restrict__ resid_out,
    float* __restrict__ w_out, int32_t* __restrict__ order_out) {
#pragma clang fp contract(off)
  extern __shared__ double smem[];
  const int ld = odd_ld(D);
  const int nwaves = blockDim.x / 64;
  const int wv = threadIdx.x / 64;
  const int d = lane();
  FitLds L;
  L.C = smem;
  L.U = L.C + D * ld;
  L.eig = L.U + D * ld;
  char* wbase = reinterpret_cast<char*>(L.eig + 64) + (size_t)wv * fit_wave_bytes(D);
  L.V = reinterpret_cast<double*>(wbase);
  L.M1 = L.V + D * ld;
  L.M2 = L.M1 + D * ld;
  L.lam = L.M2 + D * ld;
  L.vec = L.lam + 64;
  L.idx = reinterpret_cast<int*>(L.vec + 6 * 64);
  L.perm = L.idx + 64;
  L.cs = reinterpret_cast<double2*>(L.perm + 64);
  L.pr = reinterpret_cast<int2*>(L.cs + 64);
  // shared basis -> LDS
  for (int e = threadIdx.x; e < D * D; e += blockDim.x) {
    const int r = e / D, c = e % D;
    L.C[r * ld + c] = g_c[e];
    L.U[r * ld + c] = g_u[e];
  }
  for (int e = threadIdx.x; e < D; e += blockDim.x) L.eig[e] = g_eig[e];
  __syncthreads();

  // either all slots or the slots of a device-side list (the slow path of
  // kl_fit_fast.hip: tiny weights, mask-pool overflow)
  const int64_t S = slot_list ? (int64_t)n_list[0] : (int64_t)T * F * A;
  for (int64_t j = (int64_t)blockIdx.x * nwaves + wv; j < S;
       j += (int64_t)gridDim.x * nwaves) {
    const int64_t s = slot_list ? (int64_t)slot_list[j] : j;
    const int a = (int)(s % A);
    const int f = (int)((s / A) % F);
    const int64_t base = s * D;
    double phi_d = 0.0;
    float w_f = 0.0f;
    if (d < D) {
      phi_d = phase[base + d];
      if (refph) phi_d -= refph[(s / A) * D + d];
      else if (ref >= 0) phi_d -= phase[base + (int64_t)(ref - a) * D + d];
      w_f = weight[base + d];
    }
    const bool skipped = (ref_skip >= 0 && a == ref_skip) || skip[f * A + a];
    if (skipped) {
      if (d < D) {
        coef[base + d] = 0.0;
        if (resid_out) resid_out[base + d] = 0.0;
        if (w_out) w_out[base + d] = w_f;
      }
      if (d == 0 && order_out) order_out[s] = 0;
      continue;
    }
    double w_d = (double)w_f;
    double order = (double)st_order[a];
    const double station_order = order;
    double white_d = 0.0, resid_d = 0.0;
    SubsetState st{-1, false, 0.0};
    bool mask_valid = false;
    for (int it = 0; it < niter; ++it) {
      if (it > 0 && screen_type == SF_SCREEN_PHASE) {
        // _flag_outliers on this slot (stationscreen.py:303-350): circular
        // std across directions of the wrapped residual, flagged -> NaN
        const bool live = d < D;
        const bool any_unfl = __any(live && w_d > 0.0);
        if (any_unfl) {
          double r = fmod(resid_d, 2.0 * M_PI);
          if (r < -M_PI) r += 2.0 * M_PI;
          if (r > M_PI) r -= 2.0 * M_PI;
          const bool inc = live && (w_d != 0.0) && !isnan(r);
          double sn = 0.0, cn = 0.0;
          if (inc) sincos(r, &sn, &cn);
          const double cnt = wave_sum(inc ? 1.0 : 0.0);
          const double ms = wave_sum(sn) / cnt;
          const double mc = wave_sum(cn) / cnt;
          const double stdv = sqrt(-2.0 * log(hypot(ms, mc)));
          const bool outl = live && (fabs(r) > nsigma * stdv);
          if (outl) w_d = 0.0;
          if (__any(outl)) mask_valid = false;
        }
      }
      const int norderiter = (adjust_order && it > 0) ? 4 : 1;
      const uint64_t um = __ballot(d < D && w_d > 0.0);
      const int n_unfl = __popcll(um);
      if (n_unfl == 0) continue;
      if (order > n_unfl - 1) order = n_unfl - 1;
      bool hit_upper = false, hit_lower = false, hit_upper2 = false,
           hit_lower2 = false;
      double sign = 1.0, prev_redchi2 = 0.0;
      for (int oi = 0; oi < norderiter; ++oi) {
        bool skip_fit = false;
        if (it > 0) {
          // quirk Q2: the weights always compare equal to "previous"
          if (!adjust_order) break;
          if (oi == 0) skip_fit = true;
        }
        if (!skip_fit) {
          if (!mask_valid) {
            setup_subset(L, D, ld, w_d, st);
            mask_valid = true;
          }
          fit_screen(L, st, D, ld, (int)order, screen_type, phi_d, w_d,
                     white_d, resid_d);
        }
        if (hit_lower2 || hit_upper2) break;
        if (adjust_order && it > 0) {
          double redchi2;
          const bool unfl = d < D && w_d > 0.0;
          if (screen_type == SF_SCREEN_PHASE) {
            // _circ_chi2: squares of sin / cos (quirk Q7)
            double sn = 0.0, cn = 0.0;
            if (unfl) sincos(resid_d, &sn, &cn);
            const double ww = unfl ? w_d : 0.0;
            const double sw = wave_sum(ww);
            const double m1 = wave_sum(sn * sn * ww) / sw;
            const double m2 = wave_sum(cn * cn * ww) / sw;
            redchi2 = (1.0 - hypot(m1, m2)) * sw / (n_unfl - order);
          } else {
            const double ww = unfl ? w_d : 0.0;
            redchi2 = wave_sum(resid_d * resid_d * ww) / (n_unfl - order);
          }
          if (oi > 0) {
            if (redchi2 > 1.0 && prev_redchi2 < redchi2) sign = -sign;
            if (redchi2 < 1.0 && prev_redchi2 > redchi2) sign = -sign;
          }
          prev_redchi2 = redchi2;
          const double order_factor = pow((double)n_unfl - order, 0.2);
          double target = order - sign * order_factor * (1.0 - redchi2);
          target = fmax(station_order, target);
          target = fmin(rint(target), (double)(n_unfl - 1));
          if (target <= 0.0) target = fmin(station_order, (double)(n_unfl - 1));
          if (target == order) break;
          if (target == n_unfl - 1) {
            if (hit_upper) hit_upper2 = true;
            hit_upper = true;
          }
          if (target == station_order) {
            if (hit_lower) hit_lower2 = true;
            hit_lower = true;
          }
          order = target;
        }
      }
    }
    if (d < D) {
      coef[base + d] = white_d;
      if (resid_out) resid_out[base + d] = resid_d;
      if (w_out) w_out[base + d] = (float)w_d;
    }
    if (d == 0 && order_out) order_out[s] = (int32_t)order;
  }
}

int launch_basis(sf_ctx* ctx) {
  const int D = ctx->D;
  const int ld = odd_ld(D);
  const size_t shm = (size_t)2 * D * ld * sizeof(double) + 64 * sizeof(double2) +
                     96 * sizeof(int2) + 64 * sizeof(int);
  hipLaunchKernelGGL(kl_basis_kernel, dim3(1), dim3(64), shm, ctx->stream,
                     ctx->d_pp, D, ctx->r0, ctx->beta, ctx->d_c, ctx->d_pinv,
                     ctx->d_u, ctx->d_eig);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

// Referencing / ref-station skip parameters of one sf_kl_fit call
// (stationscreen.py:994-997, :818), including the operator-precedence quirk
// Q15 (tec is always referenced, to the last (local) station when
// ref_ant == -1).
RefSpec ref_spec(const sf_fit_params* p, int A) {
  RefSpec r;
  const int ref = (p->ref_ant == -1) ? -1 : p->ref_ant - p->ant_offset;
  if (p->screen_type == SF_SCREEN_AMPLITUDE) return r;  // never referenced
  if (p->screen_type == SF_SCREEN_PHASE) {
    if (p->ref_ant != -1) {
      if (p->ref_phase) r.refph = p->ref_phase; else r.sub = ref;
    }
  } else {
    if (p->ref_ant == -1) r.sub = A - 1;
    else if (p->ref_phase) r.refph = p->ref_phase;
    else r.sub = ref;
  }
  if (ref >= 0 && ref < A) r.skip = ref;
  return r;
}

int launch_skip(sf_ctx* ctx, const double* phase, const float* weight, int T,
                int F, int A, const RefSpec& r) {
  hipLaunchKernelGGL(kl_skip_kernel, dim3(F * A), dim3(64), 0, ctx->stream,
                     phase, weight, T, F, A, ctx->D, r.sub, r.refph, ctx->d_skip);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

int launch_fit_general(sf_ctx* ctx, const int* slot_list, const int* n_list,
                       int64_t max_slots, const double* phase,
                       const float* weight, int T, int F, int A,
                       const sf_fit_params* p, const RefSpec& r, double* coef,
                       double* resid, float* w_out, int32_t* order_out) {
  const int D = ctx->D;
  const size_t shared = fit_shared_bytes(D);
  const size_t wave = fit_wave_bytes(D);
  int nw = 4;
  while (nw > 1 && shared + nw * wave > 80 * 1024) --nw;
  const size_t shm = shared + nw * wave;
  int64_t blocks = (max_slots + nw - 1) / nw;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (shm > 64 * 1024)
    SF_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&kl_fit_general_kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipLaunchKernelGGL(kl_fit_general_kernel, dim3((unsigned)blocks),
                     dim3(64 * nw), shm, ctx->stream, slot_list, n_list, phase,
                     weight, T, F, A, D, ctx->d_st_order, ctx->d_skip, r.refph,
                     ctx->d_c, ctx->d_u, ctx->d_eig, p->screen_type, p->niter,
                     p->nsigma, p->adjust_order, r.sub, r.skip, coef, resid,
                     w_out, order_out);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

}  // namespace sf

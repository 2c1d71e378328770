// kl_fit_fast.hip -- the production KL fit pipeline (gfx950, float64).
//
// Same result as kl_fit_general_kernel (and the reference operator
// stationscreen.run, stationscreen.py:597-782 / 433-594), restructured for
// throughput:
//
//  1. flagged-direction subsets are decomposed ONCE PER UNIQUE FLAG MASK
//     (the reference recomputes _calculate_svd for every slot with a flagged
//     direction, stationscreen.py:495-499): a device hash table maps each
//     64-bit unflagged-mask to an entry of a pool of subset bases (U_sub
//     sorted by |lambda|, lambda), filled by a wavefront Jacobi kernel;
//  2. the least-squares solve runs in the eigenbasis of C.  With
//     C = U Lambda U^T, pinv(C) U_k = U_k Lambda_k^+ and C pinv(C) U_k =
//     U_k (Lambda_k Lambda_k^+), so
//        C re = U_k m(a_c),  a_c = (U_k^T W U_k)^+ U_k^T W cos(phi)
//        white = U Lambda^+ U^T screen,  C white = U (Lambda Lambda^+) U^T screen
//     (m = mask of |lambda| > 1e-3).  No C / pinv(C) mat-vecs remain, and for
//     uniform unflagged weights (the common 0/1 case) U_k^T W U_k = w I;
//  3. slots with a weight in (0, 1.001e-3] -- where the 1e-3 pinv cutoff on
//     U_k^T W U_k can truncate -- are routed to kl_fit_general_kernel, which
//     keeps the reference's exact pinv semantics through a Jacobi solve.
//
// The outlier-flagging iterations become passes over all slots; between
// passes the new masks are inserted, numbered and decomposed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "sf_internal.h"
#include "sf_wave.h"

namespace sf {

constexpr double kAtol = 1e-3;             // pinv(rcond=1e-3)
constexpr size_t kLdsBytes = 160 * 1024;   // LDS of one gfx950 CU
constexpr double kTinyW = 1e-3 * 1.001;    // slow-path threshold on weights
constexpr unsigned long long kEmptyKey = 0ull;

__host__ __device__ inline int ldo(int n) { return n | 1; }

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Insert `key` (non-zero) into the open-addressing table; returns its slot
// or -3 when the table is full.  Only ever inserts, never waits on other
// threads (ids are assigned by a later kernel).
__device__ int table_insert(unsigned long long* keys, int cap,
                            unsigned long long key) {
  int h = (int)(mix64(key) & (unsigned long long)(cap - 1));
  for (int probe = 0; probe < cap; ++probe) {
    // a plain load first: most slots share a few masks, whose entries are
    // taken long before most inserts arrive -- no atomic on those
    unsigned long long prev = keys[h];
    if (prev == kEmptyKey) prev = atomicCAS(keys + h, kEmptyKey, key);
    if (prev == kEmptyKey || prev == key) return h;
    h = (h + 1) & (cap - 1);
  }
  return -3;
}

// The slot of `key` in the table, or -1 (read-only: the table does not
// change while the subset bases are decomposed).
__device__ int table_find(const unsigned long long* keys, int cap,
                          unsigned long long key) {
  int h = (int)(mix64(key) & (unsigned long long)(cap - 1));
  for (int probe = 0; probe < cap; ++probe) {
    const unsigned long long k = keys[h];
    if (k == key) return h;
    if (k == kEmptyKey) return -1;
    h = (h + 1) & (cap - 1);
  }
  return -1;
}

__device__ __forceinline__ double phase_ref(const double* phase,
                                            const double* refph, int sub,
                                            int64_t s, int a, int A, int D,
                                            int d) {
  double v = phase[s * D + d];
  if (refph) v -= refph[(s / A) * D + d];
  else if (sub >= 0) v -= phase[(s + (sub - a)) * D + d];
  return v;
}

// ---------------------------------------------------------------------------
// 1. classify slots, initialise the per-slot state, insert initial masks.
//    A slot is a group of GW = pow2 >= D lanes (64 / GW slots per wavefront),
//    lane d of the group handles direction d, so every load and store of the
//    [S][D] arrays is contiguous across the wave.
// ---------------------------------------------------------------------------
template <int GW>
__global__ __launch_bounds__(256) void kl_classify_kernel(
    const float* __restrict__ weight, int64_t S, int F, int A, int D,
    const int* __restrict__ st_order, const uint8_t* __restrict__ skip,
    int ref_skip, unsigned long long* __restrict__ keys, int cap,
    int* __restrict__ pos, uint8_t* __restrict__ cls,
    int* __restrict__ counters,
    double* __restrict__ coef, double* __restrict__ resid,
    float* __restrict__ w_out, int32_t* __restrict__ order_out) {
  constexpr int kPerWave = 64 / GW;
  const int l = lane();
  const int g = l / GW;   // slot group within the wave
  const int d = l % GW;   // direction
  const int64_t s = ((int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) *
                        kPerWave + g;
  const bool live = s < S && d < D;
  float x = 0.0f;
  if (live) {
    x = weight[s * D + d];
    w_out[s * D + d] = x;
  }
  // the group's unflagged-direction bits and tiny-weight vote
  const unsigned long long bm = __ballot(live && x > 0.0f);
  const unsigned long long bt = __ballot(live && x > 0.0f && (double)x <= kTinyW);
  const unsigned long long gmask = (GW == 64) ? ~0ull : ((1ull << GW) - 1ull);
  const unsigned long long mask = (bm >> (g * GW)) & gmask;
  const bool tiny = ((bt >> (g * GW)) & gmask) != 0ull;
  // unequal positive weights in the slot (U_k^T W U_k != w I): compared with
  // the group's first unflagged weight; zeroing weights (outlier flags) keeps
  // a uniform slot uniform, so one count per fit decides the pass kernel
  const float w_first = __shfl(x, g * GW + (mask ? __builtin_ctzll(mask) : 0));
  const unsigned long long bn = __ballot(live && x > 0.0f && x != w_first);
  const bool nonuniform = ((bn >> (g * GW)) & gmask) != 0ull;
  if (s >= S) return;
  const int a = (int)(s % A);
  const int f = (int)((s / A) % F);
  // zero outputs only where no pass writes them: skipped blocks (class 1);
  // the passes write every other slot (pass 0 starts from zero coefficients
  // and residuals without reading them)
  if (live && (a == ref_skip || skip[f * A + a])) {
    coef[s * D + d] = 0.0;
    resid[s * D + d] = 0.0;
  }
  if (d != 0) return;
  if (a == ref_skip || skip[f * A + a]) {  // stationscreen.py:818-825
    cls[s] = 1;
    order_out[s] = 0;
    pos[s] = -2;
    return;
  }
  order_out[s] = st_order[a];
  if (tiny) atomicAdd(counters + 2, 1);
  else if (nonuniform) atomicAdd(counters + 4, 1);
  cls[s] = tiny ? 2 : 0;
  const unsigned long long full = (D == 64) ? ~0ull : ((1ull << D) - 1ull);
  if (mask == full) pos[s] = -1;
  else if (mask == 0ull) pos[s] = -2;
  else pos[s] = table_insert(keys, cap, mask);
}

// 2. number the newly inserted masks (one thread per table entry)
__global__ __launch_bounds__(256) void kl_assign_kernel(
    const unsigned long long* __restrict__ keys, int cap, int* __restrict__ ids,
    unsigned long long* __restrict__ pool_mask, int pool_cap,
    int* __restrict__ counters, int D) {
  // grid-stride over the table (a power of two >= 64: every wave's lanes
  // take the same trips)
  int lvl = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i - lane() < cap;
       i += gridDim.x * blockDim.x) {
    const unsigned long long k = i < cap ? keys[i] : kEmptyKey;
    const bool fresh = k != kEmptyKey && ids[i] < 0;
    // ids: one atomic per wavefront (the pool's order is immaterial: every
    // entry is decomposed on its own, sf_get_fit_pool callers sort by mask)
    const unsigned long long nb = __ballot(fresh);
    if (nb == 0ull) continue;  // wave-uniform: most of the table is empty
    int base = 0;
    if (lane() == 0) base = atomicAdd(counters, __popcll(nb));
    base = __shfl(base, 0);
    if (fresh) {
      const int id = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(nb >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)nb, 0));
      ids[i] = id;
      if (id < pool_cap) pool_mask[id] = k;
      lvl = max(lvl, D - __popcll(k));
    }
  }
  // the most flagged directions among the new masks (the deletion levels):
  // one atomic per wavefront
  for (int o = 32; o > 0; o >>= 1) lvl = max(lvl, __shfl_xor(lvl, o));
  if (lane() == 0 && lvl > 0) atomicMax(counters + 5, lvl);
}

// 3. subset bases of the masks numbered [counters[1], counters[0]):
//    C_sub = C[idx][:, idx] -> Jacobi -> U_sub sorted by |lambda| desc.
//    A pool mask leaves at least one direction out (the full mask is the
//    global basis, kl_classify_kernel), so the LDS matrices are sized for
//    D - 1 rows: at D = 50 a wave's 40,720 bytes let 4 waves share a CU's
//    160 KiB (43,104 bytes, sized for D, let 3).
__host__ __device__ inline int subset_ld(int D) { return ldo(D > 1 ? D - 1 : 1); }
__host__ __device__ inline int subset_rows(int D) { return D > 1 ? D - 1 : 1; }
// NW: waves per mask of the subset Jacobi (wg_jacobi); the library runs 3
// (kEigWavesDefault), SF_OPT_FIT_EIG_WAVES picks 1..4 -- the same bits at
// every count (tests/test_gpu_parity.py::test_subset_jacobi_wave_count_*)
constexpr int kEigWavesDefault = 3;
template <int NW>
__global__ __launch_bounds__(64 * NW) void kl_subset_eig_kernel(
    const double* __restrict__ g_c, int D,
    const unsigned long long* __restrict__ pool_mask, int pool_cap,
    int* __restrict__ counters, double* __restrict__ pool,
    const uint8_t* __restrict__ done) {
  extern __shared__ double smem[];
  const int ld = subset_ld(D);
  double* a = smem;
  double* v = a + subset_rows(D) * ld;
  double2* cs = reinterpret_cast<double2*>(v + subset_rows(D) * ld);
  int2* pr = reinterpret_cast<int2*>(cs + 64);  // 64 int2 + 64 int
  int* perm = reinterpret_cast<int*>(pr + 96);
  int* idx = perm + 64;
  const int first = counters[1];
  const int last = min(counters[0], pool_cap);
  const int l = lane();
  const bool w0 = threadIdx.x < 64;  // NW waves per mask
  for (int id = first + blockIdx.x; id < last; id += gridDim.x) {
    // masks the deletion kernel already decomposed (status 0)
    if (done && done[id] == 0) continue;
    const unsigned long long m = pool_mask[id];
    const bool in = (l < D) && ((m >> l) & 1ull);
    const int n = __popcll(m);
    if (n >= D) {  // cannot happen (full masks never enter the pool): flag it
      if (threadIdx.x == 0) atomicOr(counters + 3, 8);
      continue;
    }
    if (w0 && in) {
      const int p = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      idx[p] = l;
    }
    __syncthreads();
    if (w0 && l < n) {
      const int r = idx[l];
      for (int q = 0; q < n; ++q) a[l * ld + q] = g_c[r * D + idx[q]];
    }
    __syncthreads();
    wg_jacobi<NW>(a, v, cs, pr, n, ld, 40);
    __syncthreads();
    if (w0) wave_eig_order(a, n, ld, perm);
    double* e = pool + (size_t)id * (D * D + D);
    if (w0 && l < n) {
      for (int r = 0; r < n; ++r) e[l * D + r] = v[l * ld + perm[r]];
      const int pr = perm[l];
      e[D * D + l] = a[pr * ld + pr];
    }
    __syncthreads();
  }
}

// 3b. subset bases by deletions (round 5): the eigenpairs of the principal
//     submatrix C_sub = C[idx][:, idx] follow from those of C = U diag(lam)
//     U^T one deleted direction j at a time.  With z = row j of U, the
//     eigenvalues mu of the matrix without row / column j are the roots of
//         f(mu) = sum_i z_i^2 / (lam_i - mu) = 0
//     (det(C_j - mu) / det(C - mu) = [(C - mu)^-1]_jj), one between each
//     pair of consecutive poles, and its eigenvectors are U w with w_i ~
//     z_i / (lam_i - mu) (row j of U w is f(mu) = 0).  Each root is found
//     relative to its nearer pole (tau = mu - pole, Newton on tau rest(tau) -
//     z_pole^2 inside a bisection bracket), and the z_i are recomputed from
//     the roots by Loewner's formula before the vectors are formed
//     (Gu & Eisenstat: the vectors then come out orthogonal to rounding).
//     A direction whose z_i is negligible keeps its eigenpair (deflation).
//     One wavefront per mask, k deletions for k flagged directions (in
//     descending direction order, so the row of direction f is f), lane =
//     root / row; O(k n^2) per lane against the Jacobi's ~8 sweeps of n - 1
//     rounds.  Cases it does not take -- two poles closer than 1e-12 of the
//     spectrum, a root that does not converge -- are left to the Jacobi
//     kernel (status 1).  Eigenvalues to ~1e-15 of |lam|max and
//     eigenvectors to the conditioning LAPACK's have (~1e-11 for
//     close pairs), tests/test_gpu_parity.py::test_subset_secular_*.
//
//     Ancestors (level > 0): the launch takes the masks with `level` flagged
//     directions, launches run level 1, 2, ... in order, and a mask starts
//     from its nearest decomposed ancestor -- the mask with its lowest
//     flagged directions unflagged, whose deletions are the first ones of
//     its own (found in the mask table; decomposed by an earlier pass, or by
//     this call's lower levels without falling back) -- so a mask whose
//     parent is in the pool costs one deletion instead of one per flagged
//     direction.  level 0: every new mask from the global basis.  Either
//     way a mask's basis is bit for bit the chain's from the global basis:
//     an ancestor is taken only if the chain built it (status 0; status is
//     kept for every pool entry of the call, the host sets 1 before a pass's
//     launches, so an entry the Jacobi built is never a start).
__global__ __launch_bounds__(64) void kl_subset_secular_kernel(
    const double* __restrict__ g_u, const double* __restrict__ g_eig, int D,
    const unsigned long long* __restrict__ pool_mask, int pool_cap,
    int* __restrict__ counters, double* __restrict__ pool,
    uint8_t* __restrict__ status, const unsigned long long* __restrict__ keys,
    const int* __restrict__ ids, int table_cap, int level) {
#pragma clang fp contract(off)
  extern __shared__ double smem[];
  const int ld = D | 1;
  double* U = smem;            // [D][ld] current eigenvectors (row = direction)
  double* W = U + D * ld;      // [D][ld] w (row = non-deflated pole, col = root), then U w
  double* lam = W + D * ld;    // [64] current eigenvalues, ascending
  double* lz = lam + 64;       // [64] the non-deflated ones
  double* zh = lz + 64;        // [64] their z (then Loewner's)
  double* tau = zh + 64;       // [64] root - its pole
  double* nlam = tau + 64;     // [64] next eigenvalues (unsorted)
  int* ndi = reinterpret_cast<int*>(nlam + 64);  // [64] non-deflated pole -> column
  int* orig = ndi + 64;        // [64] root -> its pole (index into lz)
  int* src = orig + 64;        // [64] next slot -> root r, or -1 - deflated column
  int* perm = src + 64;        // [64] an order
  const int l = lane();
  const int first = counters[1];
  const int last = min(counters[0], pool_cap);
  constexpr double kEps = 2.220446049250313e-16;
  for (int id = first + blockIdx.x; id < last; id += gridDim.x) {
    const unsigned long long msk = pool_mask[id];
    const int n = __popcll(msk);
    if (level > 0 && D - n != level) continue;  // another launch's
    if (n >= D) {
      if (l == 0) status[id] = 1;
      continue;
    }
    // ---- the nearest decomposed ancestor (wave-uniform search)
    const unsigned long long full = D == 64 ? ~0ull : (1ull << D) - 1ull;
    unsigned long long anc = full;
    int aid = -1;
    if (level > 0) {
      unsigned long long a = msk;
      for (;;) {
        const unsigned long long fl = full & ~a;
        a |= fl & (~fl + 1ull);  // unflag the lowest flagged direction
        if (a == full) break;
        const int h = table_find(keys, table_cap, a);
        const int pid = h >= 0 ? ids[h] : -1;
        // chain-built ancestors only (status 0, kept across the passes of
        // the call): an entry the Jacobi decomposed is not the chain's bits
        if (pid >= 0 && pid < pool_cap && status[pid] == 0) {
          anc = a;
          aid = pid;
          break;
        }
      }
    }
    int m;
    if (aid < 0) {
      // ---- the global basis in ascending eigenvalue order
      const double li = l < D ? g_eig[l] : 0.0;
      int rk = 0;
      if (l < D)
        for (int k = 0; k < D; ++k) {
          const double lk = g_eig[k];
          rk += (lk < li) || (lk == li && k < l);
        }
      if (l < D) perm[rk] = l;
      lds_sync();
      if (l < D) lam[l] = g_eig[perm[l]];
      for (int e = l; e < D * D; e += 64) {
        const int p = e / D, c = e % D;
        U[p * ld + c] = g_u[p * D + perm[c]];
      }
      m = D;
    } else {
      // ---- the ancestor's pool entry (rows = its directions ascending,
      //      columns by |mu| descending) in ascending eigenvalue order
      m = __popcll(anc);
      const double* ea = pool + (size_t)aid * (D * D + D);
      const double li = l < m ? ea[D * D + l] : 0.0;
      int rk = 0;
      if (l < m)
        for (int k = 0; k < m; ++k) {
          const double lk = ea[D * D + k];
          rk += (lk < li) || (lk == li && k < l);
        }
      if (l < m) perm[rk] = l;
      lds_sync();
      if (l < m) lam[l] = ea[D * D + perm[l]];
      for (int e = l; e < m * m; e += 64) {
        const int p = e / m, c = e % m;
        U[p * ld + c] = ea[p * D + perm[c]];
      }
    }
    lds_sync();
    bool ok = true;
    for (int f = D - 1; f >= 0 && ok; --f) {
      if ((msk >> f) & 1ull) continue;  // unflagged: stays
      if (!((anc >> f) & 1ull)) continue;  // deleted in the ancestor
      const int j = f;                  // its row (every deleted row so far is > f)
      // ---- z, deflation of negligible components
      const double z = l < m ? U[j * ld + l] : 0.0;
      const double zmax = wave_max(fabs(z));
      const double lmax = wave_max(l < m ? fabs(lam[l]) : 0.0);
      const bool nd = l < m && fabs(z) > 1e-14 * zmax;
      const unsigned long long ndm = __ballot(nd);
      const int nn = __popcll(ndm);
      const int kk = __builtin_amdgcn_mbcnt_hi((uint32_t)(ndm >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)ndm, 0));
      if (nd) {
        ndi[kk] = l;
        lz[kk] = lam[l];
        zh[kk] = z;
      }
      lds_sync();
      // two non-deflated poles too close to separate a root between them
      const bool close = l + 1 < nn && lz[l + 1] - lz[l] <= 1e-12 * lmax;
      if (__ballot(close) != 0ull) {
        ok = false;
        break;
      }
      // ---- roots: lane r < nn - 1 between poles r and r + 1, as
      //      tau = mu - (nearer pole); Newton on tau rest(tau) - z_pole^2
      //      (the nearer pole's term divided out) inside a bisection bracket
      double t = 0.0;
      int o = 0;
      bool conv = true;
      if (l + 1 < nn) {
        const double lo = lz[l], hi = lz[l + 1];
        const double mid = lo + 0.5 * (hi - lo);
        double fm = 0.0;  // only its sign is used
#pragma unroll 4
        for (int k = 0; k < nn; ++k) {
          const double zk = zh[k];
          const double x = lz[k] - mid;
          double q = __builtin_amdgcn_rcp(x);
          q = q * (2.0 - x * q);
          fm += zk * zk * q;
        }
        double a, b;
        if (fm >= 0.0) {
          o = l;
          a = 0.0;
          b = mid - lo;
        } else {
          o = l + 1;
          a = mid - hi;
          b = 0.0;
        }
        const double lo_ = lz[o];
        const double zo = zh[o];
        const double zo2 = zo * zo;
        t = 0.5 * (a + b);
        conv = false;
        for (int it = 0; it < 64; ++it) {
          double rest = 0.0, drest = 0.0;
#pragma unroll 4
          for (int k = 0; k < nn; ++k) {
            const double zk = zh[k];
            const double x = (lz[k] - lo_) - t;
            // 1 / x: the hardware reciprocal and one Newton step (to ~1 ulp)
            double q = __builtin_amdgcn_rcp(x);
            q = q * (2.0 - x * q);
            q = k == o ? 0.0 : q;
            const double zq = zk * zk * q;
            rest += zq;
            drest += zq * q;
          }
          const double fv = rest - zo2 / t;  // increasing in t
          if (fv == 0.0) {
            conv = true;
            break;
          }
          if (fv < 0.0) a = t; else b = t;
          double tn = t - (t * rest - zo2) / (rest + t * drest);
          if (fabs(tn - t) <= 4.0 * kEps * fabs(t)) {
            t = tn;
            conv = true;
            break;
          }
          if (!(tn > a && tn < b)) tn = 0.5 * (a + b);
          t = tn;
          if (!(b - a > 4.0 * kEps * fmax(fabs(a), fabs(b)))) {
            conv = true;
            break;
          }
        }
        tau[l] = t;
        orig[l] = o;
      }
      if (__ballot(!conv) != 0ull) {
        ok = false;
        break;
      }
      lds_sync();
      // ---- Loewner: z_k^2 = prod_r (mu_r - lam_k) / prod_{k' != k} (lam_k' - lam_k),
      //      root r paired with pole r (r < k) or r + 1 (r >= k)
      double zn = 0.0;
      if (l < nn) {
        const double lk = lz[l];
        double pr = 1.0;
#pragma unroll 4
        for (int r = 0; r + 1 < nn; ++r) {
          const int kp = r < l ? r : r + 1;
          pr *= ((lz[orig[r]] - lk) + tau[r]) / (lz[kp] - lk);
        }
        zn = sqrt(fabs(pr));
        if (zh[l] < 0.0) zn = -zn;
      }
      lds_sync();
      if (l < nn) zh[l] = zn;
      lds_sync();
      // ---- w columns (lane r = root), normalised
      if (l + 1 < nn) {
        const double ol = lz[o];
        double nrm = 0.0;
#pragma unroll 4
        for (int k = 0; k < nn; ++k) {
          const double w = zh[k] / ((lz[k] - ol) - t);
          W[k * ld + l] = w;
          nrm += w * w;
        }
        const double inv = 1.0 / sqrt(nrm);
        for (int k = 0; k < nn; ++k) W[k * ld + l] *= inv;
      }
      // next eigenvalues: the roots (slots 0 .. nn - 2), then the deflated
      // poles (slots nn - 1 ..)
      const int dk = l - kk;  // deflated lanes below this one
      if (l + 1 < nn) {
        nlam[l] = lz[o] + t;
        src[l] = l;
      }
      if (l < m && !nd) {
        nlam[nn - 1 + dk] = lam[l];
        src[nn - 1 + dk] = -1 - l;
      }
      lds_sync();
      // ---- U w into W's root columns (column r is read whole by every
      //      lane before any lane writes it), deflated columns copied
      if (l < m) {
        // four root columns at a time: each U element read once per four
        // products; no deflation (the common case) reads U's columns directly
        const bool dense = nn == m;
        int r = 0;
        for (; r + 4 < nn; r += 4) {
          double y0 = 0.0, y1 = 0.0, y2 = 0.0, y3 = 0.0;
#pragma unroll 2
          for (int k = 0; k < nn; ++k) {
            const double u = U[l * ld + (dense ? k : ndi[k])];
            const double* wk = W + k * ld + r;
            y0 += u * wk[0];
            y1 += u * wk[1];
            y2 += u * wk[2];
            y3 += u * wk[3];
          }
          lds_sync();
          W[l * ld + r] = y0;
          W[l * ld + r + 1] = y1;
          W[l * ld + r + 2] = y2;
          W[l * ld + r + 3] = y3;
        }
        for (; r + 1 < nn; ++r) {
          double y = 0.0;
          for (int k = 0; k < nn; ++k) y += U[l * ld + (dense ? k : ndi[k])] * W[k * ld + r];
          lds_sync();
          W[l * ld + r] = y;
        }
        for (int c = 0; c < m - nn; ++c) {
          const int sc = src[nn - 1 + c];
          W[l * ld + nn - 1 + c] = U[l * ld + (-1 - sc)];
        }
      }
      // ascending order of the m - 1 next eigenvalues
      const int m1 = m - 1;
      if (l < m1) {
        const double v = nlam[l];
        int r2 = 0;
#pragma unroll 4
        for (int k = 0; k < m1; ++k) {
          const double w = nlam[k];
          r2 += (w < v) || (w == v && k < l);
        }
        perm[r2] = l;
      }
      lds_sync();
      // ---- next U: rows without j, columns ascending
      if (l < m && l != j) {
        const int pn = l < j ? l : l - 1;
        for (int c = 0; c < m1; ++c) U[pn * ld + c] = W[l * ld + perm[c]];
      }
      lds_sync();
      if (l < m1) lam[l] = nlam[perm[l]];
      // column norms without row j (lane = column, rows summed in order;
      // ~1 to rounding: row j of U w is f(mu) = 0), then each row rescaled
      if (l < m1) {
        double nr = 0.0;
#pragma unroll 4
        for (int r = 0; r < m1; ++r) {
          const double y = U[r * ld + l];
          nr += y * y;
        }
        tau[l] = sqrt(nr);
      }
      lds_sync();
      if (l < m1)
        for (int c = 0; c < m1; ++c) U[l * ld + c] = U[l * ld + c] / tau[c];
      lds_sync();
      m = m1;
    }
    if (!ok) {
      if (l == 0) status[id] = 1;
      continue;
    }
    // ---- pool entry: columns by |mu| descending (wave_eig_order's rule)
    if (l < m) {
      const double v = fabs(lam[l]);
      int r2 = 0;
      for (int k = 0; k < m; ++k) {
        const double w = fabs(lam[k]);
        r2 += (w > v) || (w == v && k < l);
      }
      perm[r2] = l;
    }
    lds_sync();
    double* e = pool + (size_t)id * (D * D + D);
    if (l < m) {
      for (int r = 0; r < m; ++r) e[l * D + r] = U[l * ld + perm[r]];
      e[D * D + l] = lam[perm[l]];
    }
    if (l == 0) status[id] = 0;
    lds_sync();
  }
}

// ---------------------------------------------------------------------------
// 4. one fit pass (iteration `it` of _process_station) over the slots of one
//    class; one wavefront per slot.  SLOW (class 2: a weight in (0, 1.001e-3])
//    solves U_k^T W U_k by a Jacobi eigen-decomposition with the 1e-3 pinv
//    cutoff; the fast class uses w I (uniform weights) or Cholesky.
// ---------------------------------------------------------------------------
struct FastLds {
  const double* U;    // [D][ld] full basis, columns sorted
  const double* C;    // [D][cld]: LDS, or global for the one-slot pass
  int cld;            // row stride of C
  const double* lam;  // [64]
  double* Vs;         // per wave: subset basis [D][ld]
  double* lams;       // per wave [64]
  double* G;          // per wave [D][ld]
  double* M;          // per wave [D][ld] (SLOW: eigenvectors of G)
  double* vec;        // per wave [6][64]
  double2* cs;        // per wave [64]   (SLOW: Jacobi scratch)
  int2* pr;           // per wave [96]   (SLOW: Jacobi scratch)
};

// U (and C, except in the one-slot pass, which reads C from L2: at D = 50
// that halves the workgroup's shared LDS so 4 waves per SIMD fit) + lambda
__host__ __device__ inline size_t fast_shared_bytes(int D, bool c_global) {
  return (size_t)((c_global ? 1 : 2) * D * ldo(D) + 64) * sizeof(double);
}
__host__ __device__ inline size_t fast_wave_bytes(int D, bool slow, bool lean = false) {
  if (lean) return (size_t)6 * 64 * sizeof(double);  // the vectors only
  return (size_t)((slow ? 3 : 2) * D * ldo(D) + 64 + 6 * 64) * sizeof(double) +
         (slow ? 64 * sizeof(double2) + 96 * sizeof(int2) : 0);
}

struct Basis {
  int n;
  bool full;
  int ld;             // row stride of U
  const double* U;    // LDS (full basis, or a copied subset) or the global pool
  const double* lam;
};

// The fp64 transcendentals of the fit pass, inlined or called (NI).  Inlined
// into the two-slots-per-wave pass, their polynomial constants were hoisted
// out of the slot loop into ~100 VGPRs (235-256 VGPRs: 2 waves per SIMD for
// a latency-bound kernel); called, that pass fits 128 VGPRs at 4 waves per
// SIMD (config-4 fit 34 -> 28 ms, gain fits faster still).  The one-slot
// pass (D > 32) calls them too, with C read from L2 so that its LDS admits
// the same 4 waves per SIMD (calls alone, LDS-capped at 3, were slower).
// The SLOW class keeps them inlined.  Same functions either way, same bits.
__device__ __noinline__ void nl_sincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __noinline__ double nl_atan2(double y, double x) { return atan2(y, x); }
__device__ __noinline__ double nl_log10(double x) { return log10(x); }
__device__ __noinline__ double nl_pow(double x, double y) { return pow(x, y); }
__device__ __noinline__ double nl_log(double x) { return log(x); }
__device__ __noinline__ double nl_fmod(double x, double y) { return fmod(x, y); }

template <bool NI>
struct FitMath {
  static __device__ __forceinline__ void sin_cos(double x, double* s, double* c) {
    if constexpr (NI) nl_sincos(x, s, c); else sincos(x, s, c);
  }
  static __device__ __forceinline__ double arctan2(double y, double x) {
    if constexpr (NI) return nl_atan2(y, x); else return atan2(y, x);
  }
  static __device__ __forceinline__ double lg10(double x) {
    if constexpr (NI) return nl_log10(x); else return log10(x);
  }
  static __device__ __forceinline__ double power(double x, double y) {
    if constexpr (NI) return nl_pow(x, y); else return pow(x, y);
  }
  static __device__ __forceinline__ double ln(double x) {
    if constexpr (NI) return nl_log(x); else return log(x);
  }
  static __device__ __forceinline__ double mod(double x, double y) {
    if constexpr (NI) return nl_fmod(x, y); else return fmod(x, y);
  }
};

template <bool NI = false>
__device__ __forceinline__ double model_value(int screen_type, double x) {
  // amplitude screens are log10 values (stationscreen.py:535-548, 576-588)
  return screen_type == SF_SCREEN_AMPLITUDE ? FitMath<NI>::power(10.0, x) : x;
}

// One _fit_screen (stationscreen.py:433-594) in the eigenbasis.  Lanes p < n
// carry the unflagged directions (phi_p, w_p); returns, per DIRECTION lane d,
// white_d and resid_d.
template <bool SLOW, int SPW, bool LEAN>
__device__ void fit_once(const FastLds& L, const Basis& B, int D, int ld,
                         int K, int screen_type, bool uniform, double wu,
                         double phi_p, double w_p, double phi_d, double w_d,
                         double& white_d, double& resid_d) {
#pragma clang fp contract(off)
  using G = Group<SPW>;
  using M = FitMath<!SLOW>;
  constexpr bool NI = !SLOW;
  // mat-vec loops: four terms' loads in flight, the sums still in order (the
  // same bits); the lean layout only (the general one would spill)
  constexpr int kMatVecUnroll = LEAN ? 4 : 1;
  const int l = G::lane();
  const int n = B.n;
  double* v0 = L.vec;
  double* v1 = L.vec + 64;
  double* v2 = L.vec + 128;
  double* v3 = L.vec + 192;
  double rc = 0.0, rs = 0.0;
  if (l < n) {
    if (screen_type == SF_SCREEN_PHASE) {
      double sn, cn;
      M::sin_cos(phi_p, &sn, &cn);
      rc = w_p * cn;
      rs = w_p * sn;
    } else if (screen_type == SF_SCREEN_AMPLITUDE) {
      rc = w_p * M::lg10(phi_p);
    } else {
      rc = w_p * phi_p;
    }
    v0[l] = rc;
    v1[l] = rs;
    v2[l] = w_p;
  }
  lds_sync();
  // Two unflagged directions (order clipped to n - 1 = 1): their C is
  // [[0, b], [b, 0]], singular values |b| twice, and the reference's
  // svd(C)[0] (LAPACK gesdd, stationscreen.py:427) is [[0, 1], [1, 0]] --
  // unit vectors, not eigenvectors -- whose first column e_2 it keeps
  // (:490-534): inv_u = pinv([w_2]) (0 below the 1e-3 cutoff), the fit
  // C pinv(C) e_2 inv_u w_2 x_2 = (0, t), and the screen (0, atan2(t_im,
  // t_re)) -- 0 = atan2(+0, +0) where the BLAS products leave +0
  // (tests/golden/make_golden_ties.py pins it; LAPACK builds whose SVD
  // leaves rounding residue there give atan2 of that residue instead)
  const bool tie2 = n == 2 && K == 1;
  double t_re = 0.0, t_im = 0.0;
  if (tie2) {
    const double w2 = v2[1];
    const double iw = w2 > kAtol ? 1.0 / w2 : 0.0;
    t_re = iw * v0[1];
    t_im = iw * v1[1];
  }
  double a1 = 0.0, a2 = 0.0;
  if (l < K) {
#pragma unroll kMatVecUnroll
    for (int p = 0; p < n; ++p) {
      const double u = B.U[p * B.ld + l];
      a1 += u * v0[p];
      a2 += u * v1[p];
    }
  }
  if (K > 0) {
    if (!SLOW && (LEAN || uniform)) {
      // U_k^T (w I) U_k = w I  (U_k orthonormal over the unflagged rows)
      a1 /= wu;
      a2 /= wu;
    } else {
      if (l < K) {
        for (int j = 0; j < K; ++j) {
          double s = 0.0;
          for (int p = 0; p < n; ++p)
            s += B.U[p * B.ld + l] * (v2[p] * B.U[p * B.ld + j]);
          L.G[l * ld + j] = s;
        }
      }
      lds_sync();
      if (!SLOW) {
        wave_cholesky_solve2<SPW>(L.G, K, ld, a1, a2);
      } else {
        // pinv(G, atol=1e-3) = sum_{|mu| > 1e-3} z z^T / mu (scipy >= 1.7)
        wave_jacobi(L.G, L.M, L.cs, L.pr, K, ld, 40);
        if (l < K) {
          v0[l] = a1;
          v1[l] = a2;
        }
        lds_sync();
        double t1 = 0.0, t2 = 0.0;
        if (l < K) {
          for (int q = 0; q < K; ++q) {
            t1 += L.M[q * ld + l] * v0[q];
            t2 += L.M[q * ld + l] * v1[q];
          }
          const double mu = L.G[l * ld + l];
          if (fabs(mu) > kAtol) {
            t1 /= mu;
            t2 /= mu;
          } else {
            t1 = t2 = 0.0;
          }
        }
        lds_sync();
        if (l < K) {
          v2[l] = t1;
          v3[l] = t2;
        }
        lds_sync();
        a1 = a2 = 0.0;
        if (l < K)
          for (int m = 0; m < K; ++m) {
            a1 += L.M[l * ld + m] * v2[m];
            a2 += L.M[l * ld + m] * v3[m];
          }
      }
    }
  }
  lds_sync();
  // C re = U_k m(a): keep the components whose eigenvalue survives the cutoff
  if (l < K) {
    const bool keep = fabs(B.lam[l]) > kAtol;
    v0[l] = keep ? a1 : 0.0;
    v1[l] = keep ? a2 : 0.0;
  }
  lds_sync();
  double screen = 0.0;
  if (l < n) {
    double cre = 0.0, cim = 0.0;
#pragma unroll kMatVecUnroll
    for (int k = 0; k < K; ++k) {
      const double u = B.U[l * B.ld + k];
      cre += u * v0[k];
      cim += u * v1[k];
    }
    screen = (screen_type == SF_SCREEN_PHASE) ? M::arctan2(cim, cre) : cre;
    if (tie2)
      screen = l != 1 ? 0.0 : (screen_type == SF_SCREEN_PHASE) ? M::arctan2(t_im, t_re) : t_re;
  }
  lds_sync();
  if (l < n) v2[l] = screen;
  lds_sync();
  // s_hat = U^T screen; white = U Lambda^+ s_hat; C white = U (Lambda Lambda^+) s_hat
  if (l < n) {
    double sh = 0.0;
#pragma unroll kMatVecUnroll
    for (int p = 0; p < n; ++p) sh += B.U[p * B.ld + l] * v2[p];
    const double lm = B.lam[l];
    const bool keep = fabs(lm) > kAtol;
    v0[l] = keep ? sh / lm : 0.0;
    v1[l] = keep ? sh : 0.0;
  }
  lds_sync();
  double white = 0.0, cw = 0.0;
  if (l < n) {
#pragma unroll kMatVecUnroll
    for (int r = 0; r < n; ++r) {
      const double u = B.U[l * B.ld + r];
      white += u * v0[r];
      cw += u * v1[r];
    }
  }
  lds_sync();
  if (B.full) {
    white_d = white;
    resid_d = phi_d - model_value<NI>(screen_type, cw);
    return;
  }
  // flagged directions (stationscreen.py:565-582): screen from the subset's
  // white coefficients, then re-whitened with the full pinv(C)
  if (l < n) {
    v0[l] = screen;
    v1[l] = white;
  }
  lds_sync();
  const bool unfl = (l < D) && (w_d > 0.0);
  const unsigned long long m = G::ballot(unfl);
  double sall = 0.0;
  if (l < D) {
    if (unfl) {
      const int p = G::rank(m);
      sall = v0[p];
    } else {
      // C[l][idx p]: idx p = p-th set bit of m
      unsigned long long mm = m;
      int p = 0;
      while (mm) {
        const int q = __builtin_ctzll(mm);
        sall += L.C[l * L.cld + q] * v1[p];
        mm &= mm - 1;
        ++p;
      }
    }
  }
  lds_sync();
  if (l < D) v2[l] = sall;
  lds_sync();
  if (l < D) {
    double sh = 0.0;
#pragma unroll kMatVecUnroll
    for (int p = 0; p < D; ++p) sh += L.U[p * ld + l] * v2[p];
    const double lm = L.lam[l];
    v0[l] = fabs(lm) > kAtol ? sh / lm : 0.0;
  }
  lds_sync();
  double wa = 0.0;
  if (l < D)
#pragma unroll kMatVecUnroll
    for (int r = 0; r < D; ++r) wa += L.U[l * ld + r] * v0[r];
  lds_sync();
  white_d = wa;
  resid_d = phi_d - model_value<NI>(screen_type, sall);
}

// residual as the outlier test / chi^2 see it (stationscreen.py:660-668,
// 733-746): phase & tec use the residual, amplitude the log10 ratio
template <bool NI = false>
__device__ __forceinline__ double screen_diff(int screen_type, double val,
                                              double resid) {
  if (screen_type == SF_SCREEN_AMPLITUDE)
    return FitMath<NI>::lg10(val) - FitMath<NI>::lg10(fabs(val - resid));
  return resid;
}

// LEAN (fast class, every slot's unflagged weights equal -- the 0/1 weights
// of the benchmarks): no per-slot G / subset-basis copies in LDS -- a flagged
// slot reads its subset basis straight from the pool (L1/L2) -- so the
// per-slot LDS is the 3 KiB of vectors and 2.7x (D = 20) to 4x (D = 50) more
// waves fit on a CU; the kernel is latency-bound, so occupancy is its speed.
#ifndef SF_FIT_MINW
#define SF_FIT_MINW 4  // waves per SIMD of the two-slot fast pass (128 VGPRs)
#endif
template <bool SLOW, int SPW, bool LEAN>
__global__ __launch_bounds__(256, SLOW ? 1 : SF_FIT_MINW) void kl_fit_pass_kernel(
    int it, int niter, int64_t S, int F, int A, int D,
    const double* __restrict__ phase, const double* __restrict__ refph,
    int ref_sub, const double* __restrict__ g_u, const double* __restrict__ g_c,
    const double* __restrict__ g_eig, const int* __restrict__ st_order,
    const uint8_t* __restrict__ cls, int* __restrict__ pos,
    const int* __restrict__ ids, unsigned long long* __restrict__ keys, int cap,
    const double* __restrict__ pool, int pool_cap, int* __restrict__ counters,
    int screen_type, double nsigma, int adjust_order, double* __restrict__ coef,
    double* __restrict__ resid, float* __restrict__ w_out,
    int32_t* __restrict__ order_out) {
#pragma clang fp contract(off)
  extern __shared__ double smem[];
  const int ld = ldo(D);
  using G = Group<SPW>;
  using M = FitMath<!SLOW>;
  constexpr bool NI = !SLOW;
  constexpr bool CG = SPW == 1;  // C read from global (L2), not LDS
  const int nwaves = blockDim.x / 64;
  const int nslots = nwaves * SPW;                  // slots in flight per WG
  const int wv = (threadIdx.x / 64) * SPW + G::index();  // slot of the WG
  const int d = G::lane();
  double* sU = smem;
  double* sC = CG ? nullptr : sU + D * ld;
  double* sl = sU + (CG ? 1 : 2) * D * ld;
  for (int e = threadIdx.x; e < D * D; e += blockDim.x) {
    const int r = e / D, c = e % D;
    sU[r * ld + c] = g_u[e];
    if (!CG) sC[r * ld + c] = g_c[e];
  }
  for (int e = threadIdx.x; e < 64; e += blockDim.x) sl[e] = e < D ? g_eig[e] : 0.0;
  __syncthreads();
  FastLds L;
  L.U = sU;
  L.C = CG ? g_c : sC;
  L.cld = CG ? D : ld;
  L.lam = sl;
  double* wb = sl + 64 + (size_t)wv * (fast_wave_bytes(D, SLOW, LEAN) / sizeof(double));
  if (LEAN) {
    L.Vs = L.G = L.M = L.lams = nullptr;
    L.vec = wb;
    L.cs = nullptr;
    L.pr = nullptr;
  } else {
    L.Vs = wb;
    L.G = wb + D * ld;
    L.M = L.G + D * ld;
    L.lams = (SLOW ? L.M + D * ld : L.G + D * ld);
    L.vec = L.lams + 64;
    L.cs = reinterpret_cast<double2*>(L.vec + 6 * 64);
    L.pr = reinterpret_cast<int2*>(L.cs + 64);
  }
  const uint8_t want = SLOW ? 2 : 0;

  for (int64_t s = (int64_t)blockIdx.x * nslots + wv; s < S;
       s += (int64_t)gridDim.x * nslots) {
    // the slot's independent loads go out together (class, mask position,
    // phases, weights, state): checked one after another they were 4-5
    // serial global round trips per slot, the pass's main cost.  The rare
    // SLOW class tests its class first (it skips almost every slot).
    if (SLOW && cls[s] != want) continue;
    const uint8_t cl = SLOW ? want : cls[s];
    const int a = (int)(s % A);
    const int p0 = pos[s];
    const int64_t base = s * D;
    double phi_d = 0.0, w_d = 0.0, white_d = 0.0, resid_d = 0.0;
    if (d < D) {
      phi_d = phase_ref(phase, refph, ref_sub, s, a, A, D, d);
      w_d = (double)w_out[base + d];
      // pass 0 starts from zero (kl_classify_kernel leaves them unwritten)
      white_d = it == 0 ? 0.0 : coef[base + d];
      resid_d = it == 0 ? 0.0 : resid[base + d];
    }
    double order = (double)order_out[s];
    const double station_order = (double)st_order[a];
    if (cl != want) continue;
    int id = -1;
    if (p0 >= 0) {
      id = ids[p0];
      if (id < 0 || id >= pool_cap) {  // cannot happen: flag it loudly
        if (d == 0) atomicOr(counters + 3, 1);
        continue;
      }
    } else if (p0 == -3) {
      if (d == 0) atomicOr(counters + 3, 2);
      continue;
    }
    const bool unfl = (d < D) && (w_d > 0.0);
    const unsigned long long um = G::ballot(unfl);
    const int n_unfl = __popcll(um);

    Basis B;
    B.n = n_unfl;
    B.full = (n_unfl == D);
    B.ld = ld;
    if (B.full) {
      B.U = L.U;
      B.lam = L.lam;
    } else if (n_unfl > 0) {
      const double* e = pool + (size_t)id * (D * D + D);
      if (LEAN) {
        B.U = e;
        B.ld = D;
        B.lam = e + D * D;
      } else {
        for (int r = 0; r < n_unfl; ++r)
          if (d < n_unfl) L.Vs[r * ld + d] = e[r * D + d];
        if (d < n_unfl) L.lams[d] = e[D * D + d];
        lds_sync();
        B.U = L.Vs;
        B.lam = L.lams;
      }
    }
    // unflagged directions onto lanes p < n
    double phi_p = 0.0, w_p = 0.0;
    {
      double* v4 = L.vec + 256;
      double* v5 = L.vec + 320;
      if (unfl) {
        const int p = G::rank(um);
        v4[p] = phi_d;
        v5[p] = w_d;
      }
      lds_sync();
      if (d < n_unfl) {
        phi_p = v4[d];
        w_p = v5[d];
      }
      lds_sync();
    }
    const double wmax = G::max(unfl ? w_d : -INFINITY);
    const double wmin = -G::max(unfl ? -w_d : -INFINITY);
    const bool uniform = (wmax == wmin);
    if (LEAN && n_unfl > 0 && !uniform) {  // classify counted none: flag it loudly
      if (d == 0) atomicOr(counters + 3, 4);
      continue;
    }

    if (n_unfl > 0) {
      if (order > n_unfl - 1) order = n_unfl - 1;
      if (it == 0) {
        fit_once<SLOW, SPW, LEAN>(L, B, D, ld, (int)order, screen_type, uniform, wmin,
                       phi_p, w_p, phi_d, w_d, white_d, resid_d);
      } else if (adjust_order) {
        bool hit_upper = false, hit_lower = false, hit_upper2 = false,
             hit_lower2 = false;
        double sign = 1.0, prev_redchi2 = 0.0;
        for (int oi = 0; oi < 4; ++oi) {
          // oi == 0: the weights always compare equal (quirk Q2) -> no fit
          if (oi > 0)
            fit_once<SLOW, SPW, LEAN>(L, B, D, ld, (int)order, screen_type, uniform, wmin,
                           phi_p, w_p, phi_d, w_d, white_d, resid_d);
          if (hit_lower2 || hit_upper2) break;
          double redchi2;
          if (screen_type == SF_SCREEN_PHASE) {
            double sn = 0.0, cn = 0.0;
            if (unfl) M::sin_cos(resid_d, &sn, &cn);
            const double ww = unfl ? w_d : 0.0;
            const double sw = G::sum(ww);
            const double m1 = G::sum(sn * sn * ww) / sw;
            const double m2 = G::sum(cn * cn * ww) / sw;
            redchi2 = (1.0 - hypot(m1, m2)) * sw / (n_unfl - order);
          } else {
            // np.sum(square(diff) * w) over all directions
            double t = 0.0;
            if (d < D) {
              const double sd = screen_diff<NI>(screen_type, phi_d, resid_d);
              t = (sd * sd) * w_d;
            }
            redchi2 = G::sum(t) / (n_unfl - order);
          }
          if (oi > 0) {
            if (redchi2 > 1.0 && prev_redchi2 < redchi2) sign = -sign;
            if (redchi2 < 1.0 && prev_redchi2 > redchi2) sign = -sign;
          }
          prev_redchi2 = redchi2;
          const double order_factor = M::power((double)n_unfl - order, 0.2);
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
    // phase: outlier flagging for the next pass, per slot (the circular
    // sigma is per time across directions, stationscreen.py:303-350);
    // tec / amplitude: one sigma per station block -> kl_block_sigma/flag
    if (it + 1 < niter && screen_type == SF_SCREEN_PHASE) {
      const bool live = d < D;
      if (G::any(live && w_d > 0.0)) {
        double r = M::mod(resid_d, 2.0 * M_PI);
        if (r < -M_PI) r += 2.0 * M_PI;
        if (r > M_PI) r -= 2.0 * M_PI;
        const bool inc = live && (w_d != 0.0) && !isnan(r);
        double sn = 0.0, cn = 0.0;
        if (inc) M::sin_cos(r, &sn, &cn);
        const double cnt = G::sum(inc ? 1.0 : 0.0);
        const double ms = G::sum(sn) / cnt;
        const double mc = G::sum(cn) / cnt;
        const double stdv = sqrt(-2.0 * M::ln(hypot(ms, mc)));
        const bool outl = live && (fabs(r) > nsigma * stdv);
        if (outl) w_d = 0.0;
        if (G::any(outl)) {
          const unsigned long long nm = G::ballot(live && w_d > 0.0);
          if (d == 0) pos[s] = (nm == 0ull) ? -2 : table_insert(keys, cap, nm);
        }
      }
    }
    if (d < D) {
      coef[base + d] = white_d;
      resid[base + d] = resid_d;
      w_out[base + d] = (float)w_d;
    }
    if (d == 0) order_out[s] = (int32_t)order;
  }
}

// 5. tec / amplitude outlier sigma per (station, freq) block
//    (stationscreen.py:338-344: fancy indexing flattens the block, so ONE
//    weighted rms over all its times and directions, quirk Q6)
__global__ __launch_bounds__(256) void kl_block_sigma_kernel(
    int T, int F, int A, int D, const double* __restrict__ phase,
    const double* __restrict__ refph, int ref_sub,
    const uint8_t* __restrict__ skip, int ref_skip, int screen_type,
    const double* __restrict__ resid, const float* __restrict__ w_out,
    double* __restrict__ sigma) {
  __shared__ double red[2][256];
  const int blk = blockIdx.x;  // f * A + a
  const int f = blk / A, a = blk % A;
  double sw = 0.0, swr = 0.0;
  if (!(skip[blk] || a == ref_skip)) {
    for (int e = threadIdx.x; e < T * D; e += blockDim.x) {
      const int t = e / D, d = e % D;
      const int64_t s = ((int64_t)t * F + f) * A + a;
      const double w = (double)w_out[s * D + d];
      if (w > 0.0) {
        const double v = phase_ref(phase, refph, ref_sub, s, a, A, D, d);
        const double sd = screen_diff(screen_type, v, resid[s * D + d]);
        swr += w * (sd * sd);
        sw += w;
      }
    }
  }
  red[0][threadIdx.x] = sw;
  red[1][threadIdx.x] = swr;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) sigma[blk] = sqrt(red[1][0] / red[0][0]);
}

// 6. apply the block sigma: |diff| > nsigma sigma -> weight 0, new mask
__global__ __launch_bounds__(256) void kl_block_flag_kernel(
    int64_t S, int F, int A, int D, const double* __restrict__ phase,
    const double* __restrict__ refph, int ref_sub,
    const uint8_t* __restrict__ cls, int screen_type, double nsigma,
    const double* __restrict__ sigma, const double* __restrict__ resid,
    float* __restrict__ w_out, unsigned long long* __restrict__ keys, int cap,
    int* __restrict__ pos) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S || (cls[s] != 0 && cls[s] != 2)) return;
  const int a = (int)(s % A);
  const int f = (int)((s / A) % F);
  const double sig = sigma[f * A + a];
  unsigned long long m = 0ull;
  bool changed = false;
  for (int d = 0; d < D; ++d) {
    float w = w_out[s * D + d];
    const double v = phase_ref(phase, refph, ref_sub, s, a, A, D, d);
    const double sd = screen_diff(screen_type, v, resid[s * D + d]);
    if (fabs(sd) > nsigma * sig && w != 0.0f) {
      w = 0.0f;
      w_out[s * D + d] = w;
      changed = true;
    }
    if (w > 0.0f) m |= 1ull << d;
  }
  if (changed) {
    const unsigned long long full = (D == 64) ? ~0ull : ((1ull << D) - 1ull);
    pos[s] = (m == 0ull) ? -2 : (m == full ? -1 : table_insert(keys, cap, m));
  }
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------
namespace {

template <typename T>
int grow(T** p, size_t& cap, size_t need, bool keep = false) {
  if (*p && cap >= need) return SF_OK;
  T* q = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&q), need * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc failed (fit scratch)");
    return SF_ENOMEM;
  }
  // callers synchronise the context stream before growing, so the old
  // buffer is no longer written by queued kernels
  if (keep && *p && cap > 0 &&
      hipMemcpy(q, *p, cap * sizeof(T), hipMemcpyDeviceToDevice) != hipSuccess) {
    (void)hipFree(q);
    set_error("hipMemcpy failed (fit scratch grow)");
    return SF_EIO;
  }
  if (*p) (void)hipFree(*p);
  *p = q;
  cap = need;
  return SF_OK;
}

size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

#define SF_TRYF(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != SF_OK) return rc_;  \
  } while (0)

static int ensure_pool(sf_ctx* ctx, size_t need) {
  const size_t entry = (size_t)ctx->D * ctx->D + ctx->D;
  if (ctx->pool_D != ctx->D) {
    if (ctx->d_pool) (void)hipFree(ctx->d_pool);
    if (ctx->d_pool_mask) (void)hipFree(ctx->d_pool_mask);
    ctx->d_pool = nullptr;
    ctx->d_pool_mask = nullptr;
    ctx->pool_cap = 0;
    ctx->pool_D = ctx->D;
  }
  if (ctx->pool_cap >= need) return SF_OK;
  size_t cap = ctx->pool_cap ? ctx->pool_cap : 1024;
  while (cap < need) cap *= 2;
  size_t pc = ctx->pool_cap * entry, mc = ctx->pool_cap;
  SF_TRYF(grow(&ctx->d_pool, pc, cap * entry, true));
  SF_TRYF(grow(&ctx->d_pool_mask, mc, cap, true));
  ctx->pool_cap = cap;
  return SF_OK;
}

// pool_mask[id] for ids assigned beyond a previous pool capacity
__global__ __launch_bounds__(256) void kl_fill_mask_kernel(
    const unsigned long long* __restrict__ keys, const int* __restrict__ ids,
    int cap, unsigned long long* __restrict__ pool_mask, int lo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  if (keys[i] != kEmptyKey && ids[i] >= lo) pool_mask[ids[i]] = keys[i];
}

// new masks of a pass from which SF_OPT_FIT_SUBSET_DELETION = 1 starts
// deletions from ancestors (below it: one launch from the global basis)
constexpr int kAncestorMinMasks = 8192;

// number new masks, make sure the pool holds them, decompose them
static int number_and_decompose(sf_ctx* ctx, int* n_slow, int* n_nonuniform) {
  SF_HIP(hipMemcpyAsync(ctx->d_counters + 1, ctx->d_counters, sizeof(int),
                        hipMemcpyDeviceToDevice, ctx->stream));
  SF_HIP(hipMemsetAsync(ctx->d_counters + 5, 0, sizeof(int), ctx->stream));
  const int cap = (int)ctx->table_cap;
  const int old_cap = (int)ctx->pool_cap;
  hipLaunchKernelGGL(kl_assign_kernel, dim3(std::min((cap + 255) / 256, 8192)), dim3(256), 0,
                     ctx->stream, ctx->d_keys, cap, ctx->d_ids,
                     ctx->d_pool_mask, old_cap, ctx->d_counters, ctx->D);
  SF_HIP(hipGetLastError());
  int cnt[6];
  SF_HIP(hipMemcpyAsync(cnt, ctx->d_counters, 6 * sizeof(int),
                        hipMemcpyDeviceToHost, ctx->stream));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  *n_slow = cnt[2];
  *n_nonuniform = cnt[4];
  if (cnt[0] > old_cap) {
    SF_TRYF(ensure_pool(ctx, (size_t)cnt[0]));
    hipLaunchKernelGGL(kl_fill_mask_kernel, dim3((cap + 255) / 256), dim3(256),
                       0, ctx->stream, ctx->d_keys, ctx->d_ids, cap,
                       ctx->d_pool_mask, old_cap);
    SF_HIP(hipGetLastError());
  }
  const int n_new = cnt[0] - cnt[1];
  const uint8_t* done = nullptr;
  if (n_new > 0 && ctx->fit_subset_deletion && ctx->D <= 64) {
    // subset bases by deletions first (kl_subset_secular_kernel); the
    // Jacobi below takes the masks it left (status 1)
    // (the status of every pool entry of the call is kept: a later pass's
    // masks take an earlier pass's entries as ancestors only if the chain
    // built them; the stream was synchronised above, so the copy is safe)
    SF_TRYF(grow(&ctx->d_pool_status, ctx->pool_status_cap, ctx->pool_cap, true));
    SF_HIP(hipMemsetAsync(ctx->d_pool_status + cnt[1], 1, (size_t)n_new, ctx->stream));
    const int D = ctx->D;
    const int ldd = D | 1;
    const size_t shm = (size_t)2 * D * ldd * sizeof(double) + 6 * 64 * sizeof(double) +
                       4 * 64 * sizeof(int);
    if (shm > 64 * 1024)
      SF_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&kl_subset_secular_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    const int blocks = n_new < 16384 ? n_new : 16384;
    // levels 1 .. (most flagged directions), each mask from its nearest
    // decomposed ancestor (option 3, and option 1 -- the default -- when the
    // pass has kAncestorMinMasks new masks or more), or one launch, every
    // mask from the global basis (option 2, and option 1 below that count):
    // the same bits either way.  The level launches are serial, one per
    // level; they pay off where the deletions they save are many (config 5:
    // ~113 k masks, 229 -> 192 ms per fit) and cost where the masks are few
    // and deep (the gain step's amplitude fit: block flags, up to D - 1
    // flagged directions per mask, ~31 level launches per step: 10.4 ->
    // 18.7 ms per step)
    const bool anc = ctx->fit_subset_deletion == 3 ||
                     (ctx->fit_subset_deletion == 1 && n_new >= kAncestorMinMasks);
    const int levels = anc ? cnt[5] : 0;
    for (int lv = levels > 0 ? 1 : 0; lv <= levels; ++lv) {
      hipLaunchKernelGGL(kl_subset_secular_kernel, dim3(blocks), dim3(64), shm, ctx->stream,
                         ctx->d_u, ctx->d_eig, D, ctx->d_pool_mask, (int)ctx->pool_cap,
                         ctx->d_counters, ctx->d_pool, ctx->d_pool_status, ctx->d_keys,
                         ctx->d_ids, cap, lv);
      SF_HIP(hipGetLastError());
    }
    done = ctx->d_pool_status;
  }
  if (n_new > 0) {
    const int D = ctx->D;
    const size_t shm = (size_t)2 * subset_rows(D) * subset_ld(D) * sizeof(double) +
                       64 * sizeof(double2) + 96 * sizeof(int2) +
                       128 * sizeof(int);
    const int blocks = n_new < 8192 ? n_new : 8192;
    const int nw = ctx->fit_eig_waves > 0 ? ctx->fit_eig_waves : kEigWavesDefault;
#define SF_LAUNCH_EIG(NW)                                                              \
  do {                                                                                 \
    if (shm > 64 * 1024)                                                               \
      SF_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&kl_subset_eig_kernel<NW>), \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm)); \
    hipLaunchKernelGGL(kl_subset_eig_kernel<NW>, dim3(blocks), dim3(64 * NW), shm,     \
                       ctx->stream, ctx->d_c, D, ctx->d_pool_mask, (int)ctx->pool_cap, \
                       ctx->d_counters, ctx->d_pool, done);                            \
  } while (0)
    switch (nw) {
      case 1: SF_LAUNCH_EIG(1); break;
      case 2: SF_LAUNCH_EIG(2); break;
      case 4: SF_LAUNCH_EIG(4); break;
      default: SF_LAUNCH_EIG(3); break;
    }
#undef SF_LAUNCH_EIG
    SF_HIP(hipGetLastError());
  }
  return SF_OK;
}

template <bool SLOW, int SPW, bool LEAN>
static int launch_pass_spw(sf_ctx* ctx, int it, const sf_fit_params* p,
                           const RefSpec& r, int64_t S, int F, int A,
                           const double* phase, double* coef, double* resid,
                           float* w_out, int32_t* order_out) {
  const int D = ctx->D;
  const size_t shared = fast_shared_bytes(D, SPW == 1);
  const size_t slot = fast_wave_bytes(D, SLOW, LEAN);  // per-slot LDS scratch
  // waves per workgroup (<= 4): the most resident waves per CU under the
  // 160 KiB LDS of a gfx950 CU (the per-slot subset basis is D^2 doubles,
  // so at D = 50 only 2 waves fit; the smaller workgroup wins ties)
  int nw = 1, best = 0;
  for (int k = 1; k <= 4; ++k) {
    const size_t per_wg = shared + (size_t)k * SPW * slot;
    if (per_wg > kLdsBytes) break;
    const int waves = k * (int)(kLdsBytes / per_wg);
    if (waves > best) {
      best = waves;
      nw = k;
    }
  }
  const size_t shm = shared + (size_t)nw * SPW * slot;
  if (shm > 64 * 1024)
    SF_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&kl_fit_pass_kernel<SLOW, SPW, LEAN>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  int64_t blocks = (S + nw * SPW - 1) / (nw * SPW);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL((kl_fit_pass_kernel<SLOW, SPW, LEAN>), dim3((unsigned)blocks),
                     dim3(64 * nw), shm, ctx->stream, it, p->niter, S, F, A, D,
                     phase, r.refph, r.sub, ctx->d_u, ctx->d_c, ctx->d_eig,
                     ctx->d_st_order, ctx->d_class, ctx->d_pos, ctx->d_ids,
                     ctx->d_keys, (int)ctx->table_cap, ctx->d_pool,
                     (int)ctx->pool_cap, ctx->d_counters, p->screen_type,
                     p->nsigma, p->adjust_order, coef, resid, w_out, order_out);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

// The fast class packs two slots into one wavefront (two 32-lane groups)
// while the directions fit in half a wave: D <= 20 leaves 44 of 64 lanes
// idle otherwise, and the per-slot instruction stream is the fit's cost.
template <bool SLOW>
static int launch_pass(sf_ctx* ctx, int it, const sf_fit_params* p,
                       const RefSpec& r, int64_t S, int F, int A,
                       const double* phase, double* coef, double* resid,
                       float* w_out, int32_t* order_out, bool lean) {
  const bool pack = !SLOW && ctx->D <= 32 && ctx->fit_pack;
  if (!SLOW && lean && ctx->fit_lean) {
    if (pack)
      return launch_pass_spw<false, 2, true>(ctx, it, p, r, S, F, A, phase, coef,
                                             resid, w_out, order_out);
    return launch_pass_spw<false, 1, true>(ctx, it, p, r, S, F, A, phase, coef,
                                           resid, w_out, order_out);
  }
  if (pack)
    return launch_pass_spw<SLOW, 2, false>(ctx, it, p, r, S, F, A, phase, coef,
                                           resid, w_out, order_out);
  return launch_pass_spw<SLOW, 1, false>(ctx, it, p, r, S, F, A, phase, coef, resid,
                                         w_out, order_out);
}

int launch_fit(sf_ctx* ctx, const double* phase, const float* weight, int T,
               int F, int A, const sf_fit_params* p, double* coef,
               double* resid, float* w_out, int32_t* order_out) {
  const int D = ctx->D;
  const int64_t S = (int64_t)T * F * A;
  const RefSpec r = ref_spec(p, A);
  SF_TRYF(launch_skip(ctx, phase, weight, T, F, A, r));

  static const char* env = std::getenv("SCREENFIT_FIT");
  if (ctx->force_general || (env && env[0] == 'g')) {
    if (p->screen_type == SF_SCREEN_AMPLITUDE ||
        (p->niter > 1 && p->screen_type != SF_SCREEN_PHASE)) {
      set_error("the general fit kernel handles phase (any niter) and tec (niter 1) only");
      return SF_EINVAL;
    }
    return launch_fit_general(ctx, nullptr, nullptr, S, phase, weight, T, F, A,
                              p, r, coef, resid, w_out, order_out);
  }
  // scratch for outputs the caller does not want (they carry pass state)
  if (!resid) {
    SF_TRYF(grow(&ctx->d_scratch, ctx->scratch_cap, (size_t)S * D));
    resid = ctx->d_scratch;
  }
  if (!w_out || !order_out) {
    size_t wc = 0, oc = 0;
    if (ctx->d_wscratch) (void)hipFree(ctx->d_wscratch);
    if (ctx->d_oscratch) (void)hipFree(ctx->d_oscratch);
    ctx->d_wscratch = nullptr;
    ctx->d_oscratch = nullptr;
    SF_TRYF(grow(&ctx->d_wscratch, wc, (size_t)S * D));
    SF_TRYF(grow(&ctx->d_oscratch, oc, (size_t)S));
    if (!w_out) w_out = ctx->d_wscratch;
    if (!order_out) order_out = ctx->d_oscratch;
  }
  if (ctx->slot_cap < (size_t)S) {
    size_t c1 = 0, c3 = 0;
    if (ctx->d_pos) (void)hipFree(ctx->d_pos);
    if (ctx->d_class) (void)hipFree(ctx->d_class);
    ctx->d_pos = nullptr;
    ctx->d_class = nullptr;
    SF_TRYF(grow(&ctx->d_pos, c1, (size_t)S));
    SF_TRYF(grow(&ctx->d_class, c3, (size_t)S));
    ctx->slot_cap = (size_t)S;
  }
  if (ctx->sigma_cap < (size_t)F * A) {
    size_t c = 0;
    if (ctx->d_sigma) (void)hipFree(ctx->d_sigma);
    ctx->d_sigma = nullptr;
    SF_TRYF(grow(&ctx->d_sigma, c, (size_t)F * A));
    ctx->sigma_cap = (size_t)F * A;
  }
  // every pass inserts at most one mask per slot
  const size_t tcap = next_pow2((size_t)(2 * p->niter + 2) * (size_t)S + 64);
  if (ctx->table_cap < tcap) {
    size_t c1 = 0, c2 = 0;
    if (ctx->d_keys) (void)hipFree(ctx->d_keys);
    if (ctx->d_ids) (void)hipFree(ctx->d_ids);
    ctx->d_keys = nullptr;
    ctx->d_ids = nullptr;
    SF_TRYF(grow(&ctx->d_keys, c1, tcap));
    SF_TRYF(grow(&ctx->d_ids, c2, tcap));
    ctx->table_cap = tcap;
  }
  if (!ctx->d_counters) {
    size_t c = 0;
    SF_TRYF(grow(&ctx->d_counters, c, 8));
  }
  SF_TRYF(ensure_pool(ctx, 1024));
  const int cap = (int)ctx->table_cap;
  SF_HIP(hipMemsetAsync(ctx->d_keys, 0, ctx->table_cap * sizeof(unsigned long long),
                        ctx->stream));
  SF_HIP(hipMemsetAsync(ctx->d_ids, 0xff, ctx->table_cap * sizeof(int), ctx->stream));
  SF_HIP(hipMemsetAsync(ctx->d_counters, 0, 8 * sizeof(int), ctx->stream));

  {
    // lane groups of GW >= D lanes per slot, 4 waves per workgroup
    const int gw = D <= 8 ? 8 : D <= 16 ? 16 : D <= 32 ? 32 : 64;
    const int64_t per_block = 4 * (64 / gw);
    const dim3 grid((unsigned)((S + per_block - 1) / per_block));
#define SF_CLASSIFY(W)                                                          \
  hipLaunchKernelGGL(kl_classify_kernel<W>, grid, dim3(256), 0, ctx->stream,    \
                     weight, S, F, A, D, ctx->d_st_order, ctx->d_skip, r.skip,  \
                     ctx->d_keys, cap, ctx->d_pos, ctx->d_class,               \
                     ctx->d_counters, coef, resid, w_out, order_out)
    switch (gw) {
      case 8: SF_CLASSIFY(8); break;
      case 16: SF_CLASSIFY(16); break;
      case 32: SF_CLASSIFY(32); break;
      default: SF_CLASSIFY(64); break;
    }
#undef SF_CLASSIFY
    SF_HIP(hipGetLastError());
  }

  const bool block_flags = p->screen_type != SF_SCREEN_PHASE;
  for (int it = 0; it < p->niter; ++it) {
    int n_slow = 0, n_nonuniform = 0;
    SF_TRYF(number_and_decompose(ctx, &n_slow, &n_nonuniform));
    SF_TRYF(launch_pass<false>(ctx, it, p, r, S, F, A, phase, coef, resid,
                               w_out, order_out, n_nonuniform == 0));
    if (n_slow > 0)
      SF_TRYF(launch_pass<true>(ctx, it, p, r, S, F, A, phase, coef, resid,
                                w_out, order_out, false));
    if (block_flags && it + 1 < p->niter) {
      hipLaunchKernelGGL(kl_block_sigma_kernel, dim3(F * A), dim3(256), 0,
                         ctx->stream, T, F, A, D, phase, r.refph, r.sub,
                         ctx->d_skip, r.skip, p->screen_type, resid, w_out,
                         ctx->d_sigma);
      SF_HIP(hipGetLastError());
      hipLaunchKernelGGL(kl_block_flag_kernel, dim3((unsigned)((S + 255) / 256)),
                         dim3(256), 0, ctx->stream, S, F, A, D, phase, r.refph,
                         r.sub, ctx->d_class, p->screen_type, p->nsigma,
                         ctx->d_sigma, resid, w_out, ctx->d_keys, cap,
                         ctx->d_pos);
      SF_HIP(hipGetLastError());
    }
  }
  int err = 0;
  SF_HIP(hipMemcpyAsync(&err, ctx->d_counters + 3, sizeof(int),
                        hipMemcpyDeviceToHost, ctx->stream));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  // error bits of the fit pass: 1 / 2 the mask table (lookup miss / subset
  // basis missing), 8 a full mask in the subset pool, 4 the lean layout met a slot whose unflagged weights are
  // not uniform (kl_classify_kernel counted it uniform: an internal
  // inconsistency, the slot was left unwritten)
  SF_REQUIRE((err & 3) == 0, SF_EIO, "sf_kl_fit: internal mask table overflow");
  SF_REQUIRE((err & 4) == 0, SF_EIO,
             "sf_kl_fit: lean fit pass saw non-uniform weights in a slot "
             "classified uniform (slot left unwritten)");
  SF_REQUIRE((err & 8) == 0, SF_EIO,
             "sf_kl_fit: a mask with every direction unflagged entered the "
             "subset-basis pool (its basis is the global one; left unbuilt)");
  return SF_OK;
}

}  // namespace sf

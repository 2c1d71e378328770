// sf_wave.h -- wavefront-level (64-lane) float64 building blocks for the KL
// fit: reductions, a symmetric Jacobi eigen-solver and a Cholesky solver.
//
// Layout convention: an n x n matrix (n <= 64) lives in LDS with row stride
// `ld` (odd, so that lane i reading row i with ds_read_b64 hits 32 distinct
// bank pairs); lane i owns row i.  All control flow in here is wave-uniform.
#pragma once

#include <hip/hip_runtime.h>

namespace sf {

__device__ __forceinline__ int lane() { return __lane_id(); }

// Order this wave's LDS traffic: every LDS op issued so far has completed
// before anything after it (LDS ops of one wave are otherwise only ordered
// per address by the hardware; the memory clobber stops compiler motion).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ double wave_sum(double v) {
  // xor butterfly: every lane ends with the same bits (a+b == b+a)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double bcast(double v, int src) {
  return __shfl(v, src, 64);
}

// Lane group of one slot when a wavefront carries SPW independent slots
// (SPW = 1: the whole wave; SPW = 2: two 32-lane halves, for D <= 32).
// Every reduction / vote / broadcast stays inside the group, and with
// SPW = 1 each is the exact 64-lane operation above (same order of adds),
// so packing slots changes no result bit.
template <int SPW>
struct Group {
  static constexpr int kWidth = 64 / SPW;
  __device__ static int lane() { return __lane_id() & (kWidth - 1); }
  __device__ static int first() { return __lane_id() & ~(kWidth - 1); }
  __device__ static int index() { return __lane_id() / kWidth; }
  __device__ static double sum(double v) {
#pragma unroll
    for (int o = kWidth / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
  __device__ static double max(double v) {
#pragma unroll
    for (int o = kWidth / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
  }
  __device__ static double bcast(double v, int src) {
    return __shfl(v, first() + src, 64);
  }
  // the group's vote bits, bit i = group lane i
  __device__ static unsigned long long ballot(bool x) {
    const unsigned long long m = __ballot(x);
    if (SPW == 1) return m;
    return (m >> first()) & ((1ull << kWidth) - 1);
  }
  __device__ static bool any(bool x) { return ballot(x) != 0ull; }
  // number of set bits of the group mask m below this lane
  __device__ static int rank(unsigned long long m) {
    if (SPW == 1)
      return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    return __popcll(m & ((1ull << lane()) - 1));
  }
};

// Round-robin (chess tournament) pairing of m = n + (n & 1) players over
// m - 1 rounds; player m - 1 is fixed.  Returns the partner of i in round r
// (a partner >= n means "sits out this round").
__device__ __forceinline__ int rr_partner(int i, int r, int m) {
  const int mm = m - 1;
  if (i == mm) return r;
  if (i == r) return mm;
  // 2r - i lies in (-mm, 2mm): one conditional add / subtract, no modulo
  int p = 2 * r - i;
  if (p < 0) p += mm;
  if (p >= mm) p -= mm;
  return p;
}

// Cyclic Jacobi eigen-decomposition of the symmetric n x n matrix `a`
// (in place; on exit diag(a) = eigenvalues) accumulating the eigenvectors in
// the columns of `v`.  `cs` is LDS scratch of 64 double2 (the rotation of
// each row/column this round), `pr` LDS scratch of 64 int2 (the round's
// column pairs) and 64 ints (each row's partner).
// Each round applies the n/2 disjoint rotations of a round-robin pairing at
// once, A <- J^T A J, V <- V J: lane i owns row i; the element (i, j) update
// reads A_ij, A_i,pj, A_pi,j, A_pi,pj, so a chunk of column pairs is read by
// the whole wave before any of it is written (lds_sync between).  The loop
// over column pairs is branch-free (an unpaired column is paired with
// itself under the identity rotation), so the reads of a chunk issue
// back-to-back.
__device__ inline int wave_jacobi(double* a, double* v, double2* cs, int2* pr,
                                  int n, int ld, int max_sweeps) {
#pragma clang fp contract(off)
  const int i = lane();
  const bool own = i < n;
  const int m = n + (n & 1);
  const int npairs = m / 2;
  int* part = reinterpret_cast<int*>(pr + 64);
  for (int j = 0; j < n; ++j)
    if (own) v[i * ld + j] = (i == j) ? 1.0 : 0.0;
  lds_sync();
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    double off = 0.0, dia = 0.0;
    if (own) {
      for (int j = 0; j < n; ++j) {
        const double x = a[i * ld + j];
        if (j == i) dia += x * x; else off += x * x;
      }
    }
    off = wave_sum(off);
    dia = wave_sum(dia);
    // converged once the off-diagonal mass is at the rounding floor:
    // ||offdiag||_F <= 1e-13 ||A||_F (quadratic convergence gets there one
    // sweep after ~1e-7; a stricter test never triggers for n >= 10)
    if (!(off > 1e-26 * (off + dia))) break;
    for (int r = 0; r < m - 1; ++r) {
      // pair k of round r: (m-1, r) for k = 0, else (r+k, r-k) mod (m-1);
      // a pair with the dummy player n (n odd) becomes (j, j)
      if (i < npairs) {
        int p, q;
        if (i == 0) {
          p = r;
          q = m - 1;
        } else {
          p = r + i;
          if (p >= m - 1) p -= m - 1;
          q = r - i;
          if (q < 0) q += m - 1;
        }
        if (q >= n) q = p;
        if (p >= n) p = q;
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        const double apq = a[p * ld + q];
        if (p != q && apq != 0.0) {
          const double app = a[p * ld + p];
          const double aqq = a[q * ld + q];
          const double tau = (aqq - app) / (2.0 * apq);
          double t;
          if (fabs(tau) > 1e150) {
            t = 0.5 / tau;
          } else {
            t = 1.0 / (fabs(tau) + sqrt(1.0 + tau * tau));
            if (tau < 0.0) t = -t;
          }
          c = 1.0 / sqrt(1.0 + t * t);
          s = t * c;
        }
        pr[i] = make_int2(p, q);
        cs[p] = make_double2(c, -s);  // row/col p: x_p' = c x_p - s x_q
        part[p] = q;
        if (q != p) {
          cs[q] = make_double2(c, s);  // row/col q: x_q' = c x_q + s x_p
          part[q] = p;
        }
      }
      lds_sync();
      const double2 ri = own ? cs[i] : make_double2(1.0, 0.0);
      const int pir = own ? part[i] : 0;
      // lanes that own no row read (and discard) row 0: every LDS address
      // stays inside the n x ld matrices the caller sized
      const int row = own ? i : 0;
      constexpr int CH = 4;  // column pairs per chunk
      for (int k0 = 0; k0 < npairs; k0 += CH) {
        double na[CH], nb[CH], nv[CH], nw[CH];
        int jj[CH], qq[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = min(k0 + u, npairs - 1);
          const int2 jq = pr[k];
          const int j = jq.x, pj = jq.y;
          jj[u] = j;
          qq[u] = pj;
          const double2 rj = cs[j];
          const double2 rq = cs[pj];
          const double aij = a[row * ld + j];
          const double aiq = a[row * ld + pj];
          const double apj = a[pir * ld + j];
          const double apq = a[pir * ld + pj];
          const double vij = v[row * ld + j];
          const double viq = v[row * ld + pj];
          // row rotation then column rotation, summed symmetrically
          const double r_j = ri.x * aij + ri.y * apj;   // R_ij
          const double r_q = ri.x * aiq + ri.y * apq;   // R_i,pj
          na[u] = rj.x * r_j + rj.y * r_q;              // A''_ij
          nb[u] = rq.x * r_q + rq.y * r_j;              // A''_i,pj
          nv[u] = rj.x * vij + rj.y * viq;
          nw[u] = rq.x * viq + rq.y * vij;
        }
        lds_sync();
        if (own) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            a[i * ld + jj[u]] = na[u];
            v[i * ld + jj[u]] = nv[u];
            if (qq[u] != jj[u]) {
              a[i * ld + qq[u]] = nb[u];
              v[i * ld + qq[u]] = nw[u];
            }
          }
        }
        lds_sync();
      }
    }
  }
  return sweep;
}

// wave_jacobi on a workgroup of NW waves (64 NW threads): the same rounds,
// rotations and per-element arithmetic -- so the same bits -- with each
// round's column pairs split between the waves (consecutive shares; lane i
// of every wave owns row i) and a workgroup barrier where the
// one-wave version relies on wave order: after wave 0 computes the round's
// rotations, and at the end of every round.  The waves write disjoint
// columns within a round, and every read of a round precedes its barrier.
// With one wave per SIMD the one-wave solve sat exposed to every LDS and
// fp64 latency; more waves split each round's update work and overlap
// (config 5: 2 waves 405 -> 334 ms of fit, 3 waves 309 ms, 4 waves slower).
template <int NW = 2>
__device__ inline int wg_jacobi(double* a, double* v, double2* cs, int2* pr,
                                int n, int ld, int max_sweeps) {
#pragma clang fp contract(off)
  const int i = lane();
  const int w = threadIdx.x >> 6;
  const bool own = i < n;
  const int m = n + (n & 1);
  const int npairs = m / 2;
  const int share = (npairs + NW - 1) / NW;  // column pairs per wave
  const int kb = min(w * share, npairs);
  const int ke = min(kb + share, npairs);
  int* part = reinterpret_cast<int*>(pr + 64);
  for (int j = w; j < n; j += NW)
    if (own) v[i * ld + j] = (i == j) ? 1.0 : 0.0;
  __syncthreads();
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    // both waves reduce the same rows in the same order: the same decision
    double off = 0.0, dia = 0.0;
    if (own) {
      for (int j = 0; j < n; ++j) {
        const double x = a[i * ld + j];
        if (j == i) dia += x * x; else off += x * x;
      }
    }
    off = wave_sum(off);
    dia = wave_sum(dia);
    if (!(off > 1e-26 * (off + dia))) break;
    for (int r = 0; r < m - 1; ++r) {
      if (w == 0 && i < npairs) {
        int p, q;
        if (i == 0) {
          p = r;
          q = m - 1;
        } else {
          p = r + i;
          if (p >= m - 1) p -= m - 1;
          q = r - i;
          if (q < 0) q += m - 1;
        }
        if (q >= n) q = p;
        if (p >= n) p = q;
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        const double apq = a[p * ld + q];
        if (p != q && apq != 0.0) {
          const double app = a[p * ld + p];
          const double aqq = a[q * ld + q];
          const double tau = (aqq - app) / (2.0 * apq);
          double t;
          if (fabs(tau) > 1e150) {
            t = 0.5 / tau;
          } else {
            t = 1.0 / (fabs(tau) + sqrt(1.0 + tau * tau));
            if (tau < 0.0) t = -t;
          }
          c = 1.0 / sqrt(1.0 + t * t);
          s = t * c;
        }
        pr[i] = make_int2(p, q);
        cs[p] = make_double2(c, -s);
        part[p] = q;
        if (q != p) {
          cs[q] = make_double2(c, s);
          part[q] = p;
        }
      }
      __syncthreads();
      const double2 ri = own ? cs[i] : make_double2(1.0, 0.0);
      const int pir = own ? part[i] : 0;
      // lanes that own no row read (and discard) row 0: every LDS address
      // stays inside the n x ld matrices the caller sized
      const int row = own ? i : 0;
      constexpr int CH = 4;  // column pairs per chunk
      for (int k0 = kb; k0 < ke; k0 += CH) {
        double na[CH], nb[CH], nv[CH], nw[CH];
        int jj[CH], qq[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = min(k0 + u, ke - 1);
          const int2 jq = pr[k];
          const int j = jq.x, pj = jq.y;
          jj[u] = j;
          qq[u] = pj;
          const double2 rj = cs[j];
          const double2 rq = cs[pj];
          const double aij = a[row * ld + j];
          const double aiq = a[row * ld + pj];
          const double apj = a[pir * ld + j];
          const double apq = a[pir * ld + pj];
          const double vij = v[row * ld + j];
          const double viq = v[row * ld + pj];
          const double r_j = ri.x * aij + ri.y * apj;
          const double r_q = ri.x * aiq + ri.y * apq;
          na[u] = rj.x * r_j + rj.y * r_q;
          nb[u] = rq.x * r_q + rq.y * r_j;
          nv[u] = rj.x * vij + rj.y * viq;
          nw[u] = rq.x * viq + rq.y * vij;
        }
        lds_sync();
        if (own) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            a[i * ld + jj[u]] = na[u];
            v[i * ld + jj[u]] = nv[u];
            if (qq[u] != jj[u]) {
              a[i * ld + qq[u]] = nb[u];
              v[i * ld + qq[u]] = nw[u];
            }
          }
        }
        lds_sync();
      }
      __syncthreads();
    }
  }
  return sweep;
}

// Rank of lane i's eigenvalue by descending |lambda| (ties by index), i.e.
// the column order of U from svd() of a symmetric matrix.  Writes
// perm[rank] = i for i < n.
__device__ inline void wave_eig_order(const double* a, int n, int ld,
                                      int* perm) {
  const int i = lane();
  if (i < n) {
    const double li = fabs(a[i * ld + i]);
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const double lj = fabs(a[j * ld + j]);
      rank += (lj > li) || (lj == li && j < i);
    }
    perm[rank] = i;
  }
  lds_sync();
}

// In-place Cholesky G = L L^T of the SPD k x k matrix g (lower triangle
// used), then solves G x = b for two right-hand sides held one element per
// lane (b1, b2 on lanes < k).  Returns the solutions in the same layout.
template <int SPW = 1>
__device__ inline void wave_cholesky_solve2(double* g, int k, int ld,
                                            double& b1, double& b2) {
  using G = Group<SPW>;
  const int i = G::lane();
  for (int c = 0; c < k; ++c) {
    const double piv = sqrt(g[c * ld + c]);
    lds_sync();
    double lic = 0.0;
    if (i > c && i < k) {
      lic = g[i * ld + c] / piv;
      g[i * ld + c] = lic;
    }
    if (i == c) g[c * ld + c] = piv;
    lds_sync();
    if (i > c && i < k) {
      for (int j = c + 1; j <= i; ++j) g[i * ld + j] -= lic * g[j * ld + c];
    }
    lds_sync();
  }
  // forward: L y = b
  for (int c = 0; c < k; ++c) {
    const double lcc = g[c * ld + c];
    const double y1 = G::bcast(b1, c) / lcc;
    const double y2 = G::bcast(b2, c) / lcc;
    if (i == c) { b1 = y1; b2 = y2; }
    if (i > c && i < k) {
      const double lic = g[i * ld + c];
      b1 -= lic * y1;
      b2 -= lic * y2;
    }
  }
  // backward: L^T x = y
  for (int c = k - 1; c >= 0; --c) {
    const double lcc = g[c * ld + c];
    const double x1 = G::bcast(b1, c) / lcc;
    const double x2 = G::bcast(b2, c) / lcc;
    if (i == c) { b1 = x1; b2 = x2; }
    if (i < c) {
      const double lci = g[c * ld + i];
      b1 -= lci * x1;
      b2 -= lci * x2;
    }
  }
}

}  // namespace sf

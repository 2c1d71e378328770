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
// the columns of `v`.  `cs` is LDS scratch of 64 double2 for the rotations of
// one round.  Each round applies n/2 disjoint rotations A <- J^T A J at once;
// the update of element (i, j) reads A_ij, A_{pi,j}, A_{i,pj}, A_{pi,pj}
// (pi, pj = round partners), so every read of a column pair happens before
// any write to it (lds_sync between the two phases).
__device__ inline int wave_jacobi(double* a, double* v, double2* cs, int n,
                                  int ld, int max_sweeps) {
#pragma clang fp contract(off)
  const int i = lane();
  const bool own = i < n;
  const int m = n + (n & 1);
  // V = I
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
      // rotation of the pair containing lane i, computed by its smaller member
      const int pi = (i < m) ? rr_partner(i, r, m) : i;
      if (own && pi < n && i < pi) {
        const double app = a[i * ld + i];
        const double aqq = a[pi * ld + pi];
        const double apq = a[i * ld + pi];
        double c = 1.0, s = 0.0;
        if (apq != 0.0) {
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
        cs[i] = make_double2(c, -s);  // row/col of p: x_p' = c x_p - s x_q
        cs[pi] = make_double2(c, s);  // row/col of q: x_q' = c x_q + s x_p
      } else if (own && pi >= n) {
        cs[i] = make_double2(1.0, 0.0);
      }
      lds_sync();
      const double2 ri = own ? cs[i] : make_double2(1.0, 0.0);
      const int pir = (own && pi < n) ? pi : i;
      // A'' = J^T A J, processed in column pairs (j, pj), chunked so that the
      // reads of a chunk precede its writes for the whole wave.
      constexpr int CH = 8;
      for (int j0 = 0; j0 < n; j0 += CH) {
        double na[CH], nb[CH], nv[CH], nw[CH];
        int jj[CH], pjj[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int j = j0 + u;
          int pj = (j < n) ? rr_partner(j, r, m) : n;
          jj[u] = j;
          pjj[u] = pj;
          na[u] = nb[u] = nv[u] = nw[u] = 0.0;
          if (own && j < n && (pj >= n || j < pj)) {
            const double2 rj = cs[j];
            if (pj >= n) {
              // column j unpaired this round
              const double aij = a[i * ld + j];
              const double apj = a[pir * ld + j];
              na[u] = ri.x * aij + ri.y * apj;
              nv[u] = v[i * ld + j];
            } else {
              const double2 rq = cs[pj];
              const double aij = a[i * ld + j];
              const double aiq = a[i * ld + pj];
              const double apj = a[pir * ld + j];
              const double apq = a[pir * ld + pj];
              // row rotation then column rotation, summed symmetrically
              const double r_j = ri.x * aij + ri.y * apj;   // R_ij
              const double r_q = ri.x * aiq + ri.y * apq;   // R_i,pj
              na[u] = rj.x * r_j + rj.y * r_q;              // A''_ij
              nb[u] = rq.x * r_q + rq.y * r_j;              // A''_i,pj
              const double vij = v[i * ld + j];
              const double viq = v[i * ld + pj];
              nv[u] = rj.x * vij + rj.y * viq;
              nw[u] = rq.x * viq + rq.y * vij;
            }
          }
        }
        lds_sync();
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int j = jj[u], pj = pjj[u];
          if (own && j < n && (pj >= n || j < pj)) {
            a[i * ld + j] = na[u];
            v[i * ld + j] = nv[u];
            if (pj < n) {
              a[i * ld + pj] = nb[u];
              v[i * ld + pj] = nw[u];
            }
          }
        }
      }
      lds_sync();
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
__device__ inline void wave_cholesky_solve2(double* g, int k, int ld,
                                            double& b1, double& b2) {
  const int i = lane();
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
    const double y1 = bcast(b1, c) / lcc;
    const double y2 = bcast(b2, c) / lcc;
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
    const double x1 = bcast(b1, c) / lcc;
    const double x2 = bcast(b2, c) / lcc;
    if (i == c) { b1 = x1; b2 = x2; }
    if (i < c) {
      const double lci = g[c * ld + i];
      b1 -= lci * x1;
      b2 -= lci * x2;
    }
  }
}

}  // namespace sf

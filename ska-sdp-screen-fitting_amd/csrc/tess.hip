// tess.hip -- tessellated (Voronoi) screen fill + Gaussian smoothing, fused.
//
// Replaces VoronoiScreen.make_matrix (voronoi_screen.py:132-216) and the
// per-(time, freq, station) scipy.ndimage.gaussian_filter of Screen.write
// (screen.py:353-362):
//   out[s][p][y][x] = g(value_p[s][label[y][x] - 1]),  value_p in
//     {A_xx cos(phi), A_xx sin(phi), A_yy cos(phi), A_yy sin(phi)}
// with g = identity or the separable Gaussian (axis y then axis x, float32
// between the passes, 'reflect' borders, scipy's symmetric-kernel summation
// order in float64).  sf_tess_fill runs a per-slot value-table pass and then
// kl_tess_gather_kernel (no smoothing) or kl_tess_smooth_kernel (radius <=
// kMaxR), both below; kl_tess_kernel, the round-1 fused kernel (one
// workgroup = a 16 x 16 output tile and a chunk of slots, label tile + halo
// in LDS), stays for cross-checks (SF_OPT_TESS_TILE).  In every variant the
// only large HBM traffic is the 16 B / pixel / slot output write.
#include <hip/hip_runtime.h>

#include <cmath>

#include "sf_internal.h"

namespace sf {

constexpr int kTT = 16;       // output tile side
constexpr int kMaxR = kTessMaxR;  // fused-tile Gaussian radius (sigma <= 6 px)
constexpr int kTessSlots = 64;  // slots per workgroup

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // scipy.ndimage mode 'reflect' (d c b a | a b c d | d c b a) in closed
  // form: period 2n, the second half mirrored -- O(1) for any offset
  if (i >= 0 && i < n) return i;
  int m = i % (2 * n);
  if (m < 0) m += 2 * n;
  return m < n ? m : 2 * n - 1 - m;
}

__global__ __launch_bounds__(256) void kl_tess_kernel(
    const int32_t* __restrict__ labels, int nx, int ny,
    const double* __restrict__ phase, const double* __restrict__ amp_xx,
    const double* __restrict__ amp_yy, int D, int64_t S,
    float* __restrict__ out, int64_t ring, const double* __restrict__ gw,
    int R, unsigned flags) {
#pragma clang fp contract(off)
  __shared__ int lab[(kTT + 2 * kMaxR) * (kTT + 2 * kMaxR)];
  __shared__ float table[65 * 4];  // + one NaN row for invalid labels
  __shared__ float ybuf[4 * kTT * (kTT + 2 * kMaxR)];
  __shared__ double w[2 * kMaxR + 1];
  const int tiles_x = (nx + kTT - 1) / kTT;
  const int tile = blockIdx.x;
  const int tx0 = (tile % tiles_x) * kTT;
  const int ty0 = (tile / tiles_x) * kTT;
  const int64_t s0 = (int64_t)blockIdx.y * kTessSlots;
  const int H = kTT + 2 * R;  // halo tile side
  for (int e = threadIdx.x; e < H * H; e += blockDim.x) {
    const int hy = e / H, hx = e % H;
    const int gy = reflect_idx(ty0 + hy - R, ny);
    const int gx = reflect_idx(tx0 + hx - R, nx);
    const int lb = labels[(int64_t)gy * nx + gx] - 1;
    lab[e] = (lb >= 0 && lb < D) ? lb : D;  // entry D: the NaN row
  }
  for (int e = threadIdx.x; e < 2 * R + 1; e += blockDim.x) w[e] = gw[e];
  if (threadIdx.x < 4) table[D * 4 + threadIdx.x] = __builtin_nanf("");
  const int oy = threadIdx.x / kTT, ox = threadIdx.x % kTT;
  const int gy = ty0 + oy, gx = tx0 + ox;
  const bool live = gy < ny && gx < nx;
  const int64_t P = (int64_t)nx * ny;
  const bool scrub = flags & SF_EVAL_NAN_SCRUB;
  for (int64_t k = 0; k < kTessSlots; ++k) {
    const int64_t s = s0 + k;
    if (s >= S) break;
    __syncthreads();
    if (threadIdx.x < D) {
      const int d = threadIdx.x;
      double sn, cn;
      sincos(phase[s * D + d], &sn, &cn);
      const double ax = amp_xx ? amp_xx[s * D + d] : 1.0;
      const double ay = amp_yy ? amp_yy[s * D + d] : ax;
      table[d * 4 + 0] = (float)(ax * cn);
      table[d * 4 + 1] = (float)(ax * sn);
      table[d * 4 + 2] = (float)(ay * cn);
      table[d * 4 + 3] = (float)(ay * sn);
    }
    __syncthreads();
    float v[4];
    if (R == 0) {
      const int l = lab[oy * H + ox];
#pragma unroll
      for (int p = 0; p < 4; ++p) v[p] = table[l * 4 + p];
    } else {
      // pass 1 (axis y) over the tile rows and all halo columns
      for (int e = threadIdx.x; e < kTT * H; e += blockDim.x) {
        const int r = e / H, c = e % H;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          double acc = (double)table[lab[(r + R) * H + c] * 4 + p] * w[R];
          for (int j = R; j >= 1; --j) {
            const double a = table[lab[(r + R - j) * H + c] * 4 + p];
            const double b = table[lab[(r + R + j) * H + c] * 4 + p];
            acc += (a + b) * w[R - j];
          }
          ybuf[(p * kTT + r) * H + c] = (float)acc;
        }
      }
      __syncthreads();
      // pass 2 (axis x)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float* row = ybuf + (p * kTT + oy) * H + R + ox;
        double acc = (double)row[0] * w[R];
        for (int j = R; j >= 1; --j) acc += ((double)row[-j] + (double)row[j]) * w[R - j];
        v[p] = (float)acc;
      }
    }
    if (live) {
      float* o = out + ((s % ring) * 4) * P + (int64_t)gy * nx + gx;
      // a label outside 1..D (never made by the template) reads no table
      // entry: its pixels are NaN (1 / 0 under the scrub), see sf_tess_fill
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float x = v[p];
        if (scrub && isnan(x)) x = (p & 1) ? 0.0f : 1.0f;
        if (flags & SF_EVAL_BIG_ENDIAN)
          x = __uint_as_float(__builtin_bswap32(__float_as_uint(x)));
        o[p * P] = x;
      }
    }
  }
}

// Unsmoothed fill (R = 0, the make_aterm_image default smooth_deg = 0): a
// pure gather-store, laid out for HBM writes, in two kernels.
//  * kl_tess_table_kernel: per (slot, direction) the float4 {A_xx cos, A_xx
//    sin, A_yy cos, A_yy sin} (fp64 sincos and products, one cast -- the
//    bits of kl_tess_kernel) with the NaN scrub and the byte swap already
//    applied (the output IS the table entry when nothing is smoothed, so
//    scrubbing the entry equals scrubbing the pixel), plus entry D for
//    labels outside 1..D: once per slot instead of once per (slot, pixel
//    block).  [S][D + 1] float4 in a context scratch buffer.
//  * kl_tess_gather_kernel: a workgroup owns a run of kGatherRun consecutive
//    pixels and a chunk of slots; it copies the chunk's table slice to LDS,
//    and each wave takes every NW-th slot of the chunk over the
//    whole run (16 labels per lane in registers): per slot 16 entry reads
//    (ds_read_b128) and 16 float4 stores, i.e. one wave writes a 4 KiB
//    contiguous run per (slot, plane) -- the LDS-staged eval's store shape.
constexpr int kGatherRun = 1024;       // pixels per workgroup (4 KiB per plane)
// one slot per wave per work item, 16 waves: 0.816 of 8 TB/s at 256^2 x
// 102,400 slots vs 0.73-0.77 for 4 / 8 waves or 2+ slots per wave
// (profiles/round2zd_tess_gather_sweep.txt)
constexpr int kGatherWavesAuto = 16;   // waves per workgroup (SF_OPT_TESS_WAVES)
constexpr int kGatherSlotsAuto = 16;   // slots per work item (SF_OPT_TESS_SLOTS)

typedef float tess_v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void kl_tess_table_kernel(
    const double* __restrict__ phase, const double* __restrict__ amp_xx,
    const double* __restrict__ amp_yy, int D, int64_t S,
    tess_v4f* __restrict__ tab, unsigned flags) {
  const int DT = D + 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S * DT) return;
  const int64_t s = e / DT;
  const int d = (int)(e - s * DT);
  float v[4];
  if (d < D) {
    const int64_t i = s * D + d;
    double sn, cn;
    sincos(phase[i], &sn, &cn);
    const double ax = amp_xx ? amp_xx[i] : 1.0;
    const double ay = amp_yy ? amp_yy[i] : ax;
    v[0] = (float)(ax * cn);
    v[1] = (float)(ax * sn);
    v[2] = (float)(ay * cn);
    v[3] = (float)(ay * sn);
  } else {
    v[0] = v[1] = v[2] = v[3] = __builtin_nanf("");
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if ((flags & SF_EVAL_NAN_SCRUB) && isnan(v[p])) v[p] = (p & 1) ? 0.0f : 1.0f;
    if (flags & SF_EVAL_BIG_ENDIAN)
      v[p] = __uint_as_float(__builtin_bswap32(__float_as_uint(v[p])));
  }
  tab[e] = tess_v4f{v[0], v[1], v[2], v[3]};
}

template <int NW, bool VEC4>
__global__ __launch_bounds__(64 * NW) void kl_tess_gather_kernel(
    const int32_t* __restrict__ labels, int64_t P,
    const tess_v4f* __restrict__ tab, int D, int64_t S,
    float* __restrict__ out, int64_t ring, int64_t ring_base, int64_t n_pb,
    int64_t n_sc, int chunk) {
  extern __shared__ tess_v4f gtab[];  // [chunk][D + 1]
  constexpr int kC = kGatherRun / 256;  // 1 KiB pieces of a wave's run
  const int DT = D + 1;
  const int l = threadIdx.x & 63;
  // wave index, wave-uniform: slot and ring arithmetic stay on the SALU
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t bb = blockIdx.x; bb < n_pb * n_sc; bb += gridDim.x) {
    const int64_t pb = bb % n_pb, sc = bb / n_pb;
    const int64_t s0 = sc * chunk;
    const int ns = (int)((S - s0) < chunk ? (S - s0) : chunk);
    __syncthreads();  // the previous item's table reads are done
    for (int e = threadIdx.x; e < ns * DT; e += blockDim.x) gtab[e] = tab[s0 * DT + e];
    __syncthreads();
    // every wave covers the whole run (pixels 256 c + 4 l + j) for its own
    // slots k = w, w + NW, ...: per (slot, plane) one wave writes
    // kGatherRun * 4 contiguous bytes
    const int64_t p0 = pb * kGatherRun + 4 * l;
    int lab[kC][4];
#pragma unroll
    for (int c = 0; c < kC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t p = p0 + 256 * c + j;
        const int lb = p < P ? labels[p] - 1 : 0;
        lab[c][j] = (lb >= 0 && lb < D) ? lb : D;
      }
    for (int k = w; k < ns; k += NW) {
      const tess_v4f* t = gtab + k * DT;
      tess_v4f v[kC][4];
#pragma unroll
      for (int c = 0; c < kC; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[c][j] = t[lab[c][j]];
      // ring slot (ring < 2^31: sf_tess_fill)
      const int64_t so = (s0 + k + ring_base) % ring;
      float* o = out + so * 4 * P + p0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < kC; ++c) {
          if (VEC4) {
            if (p0 + 256 * c < P)
              __builtin_nontemporal_store(
                  tess_v4f{v[c][0][q], v[c][1][q], v[c][2][q], v[c][3][q]},
                  reinterpret_cast<tess_v4f*>(o + q * P + 256 * c));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (p0 + 256 * c + j < P) o[q * P + 256 * c + j] = v[c][j][q];
          }
        }
    }
  }
}

// Smoothed fill (0 < R <= kMaxR): wide tiles for long store runs.  A
// workgroup (4 waves) owns a tile of kSmTH rows x kSmTW pixels (wave w:
// rows w, w + 4, 4 pixels per lane, 1 KiB contiguous per (slot, plane)) and a
// chunk of slots.  The tile's labels + halo sit in LDS as bytes (D <= 64,
// entry D = NaN for labels outside 1..D); per slot the raw value table
// (kl_tess_table_kernel without scrub / swap, widened to double) goes to
// LDS, the y pass writes the halo columns of the tile rows (fp64 sums in
// scipy's order -- centre, then the pairs from the outermost in -- rounded
// to float like scipy's float32 intermediate), the x pass
// each wave's row, then the NaN scrub and byte swap (the reference scrubs
// after smoothing).  The same arithmetic in the same order as
// kl_tess_kernel: the same bits.
constexpr int kSmTW = 256;
// tile rows by radius: 4 for R <= 2 (0.5 px: 18.1 vs 20.1 ms with 8), 8 above
// (more rows per y-pass window: 1.3 / 2 px 26.4 / 38.4 -> 25.1 / 36.2 ms;
// profiles/round2zi_tess_smooth_rows.txt)
__host__ __device__ constexpr int smooth_rows(int R) { return (R >= 1 && R <= 2) ? 4 : 8; }
constexpr int kSmSlots = 8;

// RT > 0: the radius at compile time (taps unrolled, so the label and table
// reads of a tap window go out together; LDS sized for RT: more resident
// workgroups); RT = 0: any R <= kMaxR at run time.
template <int RT, int NP>
__global__ __launch_bounds__(256) void kl_tess_smooth_kernel(
    const int32_t* __restrict__ labels, int nx, int ny,
    const tess_v4f* __restrict__ tab, int D, int64_t S,
    float* __restrict__ out, int64_t ring, int64_t ring_base,
    const double* __restrict__ gw, int R_arg, int64_t n_tiles, int64_t n_sc,
    unsigned flags) {
#pragma clang fp contract(off)
  // NP = 2: planes 2 / 3 repeat planes 0 / 1 (no YY amplitude: A_yy = A_xx),
  // so only two planes are smoothed and each is stored twice
  typedef double vacc_t __attribute__((ext_vector_type(NP)));
  typedef float vyf_t __attribute__((ext_vector_type(NP)));
  auto widen = [](const auto& v) {
    vacc_t r;
#pragma unroll
    for (int p = 0; p < NP; ++p) r[p] = (double)v[p];
    return r;
  };
  constexpr int kR = RT > 0 ? RT : kMaxR;  // LDS sizing
  constexpr int kSmTH = smooth_rows(RT);
  const int R = RT > 0 ? RT : R_arg;
  // RT > 0: every tap unrolled; a run-time R: 4 taps per trip, so the label
  // and table reads of 4 taps go out together
  constexpr int kTapUnroll = RT > 0 ? RT : 4;
  __shared__ unsigned char lab[(kSmTH + 2 * kR) * (kSmTW + 2 * kR)];
  // y-pass results: float, as scipy's float32 intermediate image
  __shared__ vyf_t ybuf[kSmTH * (kSmTW + 2 * kR)];
  __shared__ vacc_t tbl[2][65];
  __shared__ double w[2 * kR + 1];
  const int DT = D + 1;
  const int W2 = kSmTW + 2 * R;  // halo tile width
  const int H2 = kSmTH + 2 * R;
  const int tiles_x = (nx + kSmTW - 1) / kSmTW;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool scrub = flags & SF_EVAL_NAN_SCRUB;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  const int64_t P = (int64_t)nx * ny;
  for (int e = threadIdx.x; e < 2 * R + 1; e += blockDim.x) w[e] = gw[e];
  for (int64_t bb = blockIdx.x; bb < n_tiles * n_sc; bb += gridDim.x) {
    const int64_t tile = bb % n_tiles, sc = bb / n_tiles;
    const int tx0 = (int)(tile % tiles_x) * kSmTW;
    const int ty0 = (int)(tile / tiles_x) * kSmTH;
    const int64_t s0 = sc * kSmSlots;
    const int ns = (int)((S - s0) < kSmSlots ? (S - s0) : kSmSlots);
    __syncthreads();  // the previous item is done with lab / tbl / ybuf
    for (int e = threadIdx.x; e < H2 * W2; e += blockDim.x) {
      const int hy = e / W2, hx = e - hy * W2;
      const int gy = reflect_idx(ty0 + hy - R, ny);
      const int gx = reflect_idx(tx0 + hx - R, nx);
      const int lb = labels[(int64_t)gy * nx + gx] - 1;
      lab[e] = (unsigned char)((lb >= 0 && lb < D) ? lb : D);
    }
    for (int e = threadIdx.x; e < DT; e += blockDim.x) {
      tbl[0][e] = widen(tab[s0 * DT + e]);
    }
    for (int k = 0; k < ns; ++k) {
      __syncthreads();  // tbl[k & 1] (and, at k = 0, lab) complete; ybuf free
      const vacc_t* t = tbl[k & 1];
      // y pass over the tile rows and every halo column; compile-time R: an
      // item = (column, half of the tile rows): it slides one kYR + 2R
      // window of table values (read once) down its kYR rows; half-height
      // items split the W2 > 256 columns' tail trip in two
      if constexpr (RT > 0) {
        constexpr int kYR = kSmTH / 2;
        constexpr int HW = kYR + 2 * RT;
        for (int e = threadIdx.x; e < 2 * W2; e += blockDim.x) {
          const int g = e >= W2;
          const int c = e - g * W2;
          const int r0 = g * kYR;
          vacc_t win[HW];
#pragma unroll
          for (int h = 0; h < HW; ++h) win[h] = t[lab[(r0 + h) * W2 + c]];
#pragma unroll
          for (int r = 0; r < kYR; ++r) {
            vacc_t acc = win[r + RT] * w[RT];
#pragma unroll
            for (int j = RT; j >= 1; --j)
              acc += (win[r + RT - j] + win[r + RT + j]) * w[RT - j];
            vyf_t y;
#pragma unroll
            for (int p = 0; p < NP; ++p) y[p] = (float)acc[p];
            ybuf[(r0 + r) * W2 + c] = y;
          }
        }
      } else
      for (int e = threadIdx.x; e < kSmTH * W2; e += blockDim.x) {
        const int r = e / W2, c = e - r * W2;
        const unsigned char* col = lab + (r + R) * W2 + c;
        vacc_t acc = t[col[0]] * w[R];
#pragma unroll kTapUnroll
        for (int j = R; j >= 1; --j) {
          const vacc_t a = t[col[-j * W2]], b = t[col[j * W2]];
          acc += (a + b) * w[R - j];
        }
        vyf_t y;
#pragma unroll
        for (int p = 0; p < NP; ++p) y[p] = (float)acc[p];
        ybuf[e] = y;
      }
      // the next slot's table, into the other buffer (its last readers
      // finished the y pass of slot k - 1 before the barrier above)
      if (k + 1 < ns)
        for (int e = threadIdx.x; e < DT; e += blockDim.x) {
          tbl[(k + 1) & 1][e] = widen(tab[(s0 + k + 1) * DT + e]);
        }
      __syncthreads();
      // x pass: wave w takes rows w, w + 4, ...; 4 pixels per lane
      const int gx0 = tx0 + 4 * l;
      for (int rr = wv; rr < kSmTH; rr += 4) {
      const int gy = ty0 + rr;
      if (gy >= ny || gx0 >= nx) continue;
      float v[4][4];  // [pixel][plane]
      // compile-time R: the lane's 4 pixels share one 4 + 2R window
      constexpr int XW = RT > 0 ? 4 + 2 * RT : 1;
      vacc_t xwin[XW];
      if constexpr (RT > 0) {
        const vyf_t* base = ybuf + rr * W2 + 4 * l;
#pragma unroll
        for (int h = 0; h < XW; ++h) xwin[h] = widen(base[h]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vacc_t acc;
        if constexpr (RT > 0) {
          acc = xwin[RT + i] * w[RT];
#pragma unroll
          for (int j = RT; j >= 1; --j)
            acc += (xwin[RT + i - j] + xwin[RT + i + j]) * w[RT - j];
        } else {
          const vyf_t* row = ybuf + rr * W2 + R + 4 * l + i;
          acc = widen(row[0]) * w[R];
#pragma unroll kTapUnroll
          for (int j = R; j >= 1; --j) {
            acc += (widen(row[-j]) + widen(row[j])) * w[R - j];
          }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float x = (float)acc[p % NP];
          if (scrub && isnan(x)) x = (p & 1) ? 0.0f : 1.0f;
          if (be) x = __uint_as_float(__builtin_bswap32(__float_as_uint(x)));
          v[i][p] = x;
        }
      }
      const int64_t so = (s0 + k + ring_base) % ring;
      float* o = out + so * 4 * P + (int64_t)gy * nx + gx0;
      const bool vec = (nx % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (vec) {
          __builtin_nontemporal_store(tess_v4f{v[0][p], v[1][p], v[2][p], v[3][p]},
                                      reinterpret_cast<tess_v4f*>(o + p * P));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (gx0 + i < nx) o[p * P + i] = v[i][p];
        }
      }
      }  // rows of this wave
    }
  }
}

// Smoothed fill with interior lookups (round 3; kl_tess_box_kernel).  The
// unsmoothed image of a slot is piecewise constant: every pixel holds one of
// the D + 1 table values, chosen by the label raster, which is the same for
// every slot.  Where the whole (2R + 1)^2 box around a pixel carries one
// label L, both passes of the Gaussian see 2R + 1 equal inputs, so the
// pixel's smoothed value is a function of the table entry alone: computed
// once per (slot, entry) with scipy's arithmetic in scipy's order (y sum of
// equal doubles -> float -> x sum of equal doubles -> float -> scrub -> swap)
// it is bit for bit what the full two-pass sum gives there.  Per tile the
// kernel finds (once, for all the item's slots) the vertically uniform
// y-pass windows (vlab) and the box-uniform pixels (plab), and lists the
// others; per slot it then runs the y pass only over the listed windows, the
// x pass only over the listed (boundary) pixels -- reading a uniform
// window's y value from the per-entry table -- and stores every pixel from
// either the per-entry final value or the boundary result.  At sigma 0.5 px
// (R = 2) about a fifth of a 256^2 Voronoi raster of 20 cells is boundary,
// so the fp64 VALU work of the passes (3 ops per tap per plane, scipy's
// order: the reason kl_tess_smooth_kernel is VALU-bound) shrinks ~5x and the
// fill approaches the gather kernel's store rate.  Same bits as
// kl_tess_smooth_kernel and kl_tess_kernel.
constexpr int kBoxTH = 4;       // tile rows (one per wave)
constexpr int kBoxSlots = 32;   // slots per work item (the tile setup amortises over them)
constexpr int kBoxMaxR = 24;

template <int RT, int NP>
__global__ __launch_bounds__(256) void kl_tess_box_kernel(
    const int32_t* __restrict__ labels, int nx, int ny,
    const tess_v4f* __restrict__ tab, int D, int64_t S,
    float* __restrict__ out, int64_t ring, int64_t ring_base,
    const double* __restrict__ gw, int R_arg, int64_t n_tiles, int64_t n_sc,
    unsigned flags) {
#pragma clang fp contract(off)
  typedef double vacc_t __attribute__((ext_vector_type(NP)));
  typedef float vyf_t __attribute__((ext_vector_type(NP)));
  auto widen = [](const auto& v) {
    vacc_t r;
#pragma unroll
    for (int p = 0; p < NP; ++p) r[p] = (double)v[p];
    return r;
  };
  constexpr int kR = RT > 0 ? RT : kBoxMaxR;  // LDS sizing
  constexpr int kW2 = kSmTW + 2 * kR;
  constexpr unsigned char kMixed = 0xFF;       // D <= 64 < 0xFF
  constexpr int kTapUnroll = RT > 0 ? RT : 4;
  const int R = RT > 0 ? RT : R_arg;
  const int W2 = kSmTW + 2 * R;
  const int H2 = kBoxTH + 2 * R;
  __shared__ unsigned char lab[(kBoxTH + 2 * kR) * kW2];  // halo labels
  __shared__ unsigned char vlab[kBoxTH * kW2];   // uniform y window: its label
  __shared__ __attribute__((aligned(16))) unsigned char plab[kBoxTH * kSmTW];  // uniform box: its label
  __shared__ unsigned short ylist[kBoxTH * kW2];  // mixed y windows
  __shared__ unsigned short xlist[kBoxTH * kSmTW];  // mixed (boundary) pixels
  __shared__ int n_list[2];
  __shared__ vacc_t tbl[2][65];     // raw table entries, widened
  __shared__ vyf_t yu[2][65];       // y pass of a uniform window, per entry
  __shared__ tess_v4f xu[2][65];    // final value of a uniform box, per entry
  __shared__ vyf_t ybuf[kBoxTH * kW2];    // y pass of the mixed windows
  __shared__ tess_v4f xout[kBoxTH * kSmTW];  // final value of the mixed pixels
  __shared__ double w[2 * kR + 1];
  const int DT = D + 1;
  const int tiles_x = (nx + kSmTW - 1) / kSmTW;
  const int tid = threadIdx.x, l = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool scrub = flags & SF_EVAL_NAN_SCRUB;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  const int64_t P = (int64_t)nx * ny;
  const bool vec = (nx % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  for (int e = tid; e < 2 * R + 1; e += blockDim.x) w[e] = gw[e];
  // per-entry tables of slot s into buffer b: the raw entry, its uniform y
  // value and its uniform-box final value (scipy's order on equal inputs)
  auto entry_tables = [&](int64_t s, int b) {
    for (int e = tid; e < DT; e += blockDim.x) {
      const vacc_t t = widen(tab[s * DT + e]);
      tbl[b][e] = t;
      vacc_t acc = t * w[R];
      for (int j = R; j >= 1; --j) acc += (t + t) * w[R - j];
      vyf_t y;
#pragma unroll
      for (int p = 0; p < NP; ++p) y[p] = (float)acc[p];
      yu[b][e] = y;
      const vacc_t yd = widen(y);
      acc = yd * w[R];
      for (int j = R; j >= 1; --j) acc += (yd + yd) * w[R - j];
      tess_v4f v;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float x = (float)acc[p % NP];
        if (scrub && isnan(x)) x = (p & 1) ? 0.0f : 1.0f;
        if (be) x = __uint_as_float(__builtin_bswap32(__float_as_uint(x)));
        v[p] = x;
      }
      xu[b][e] = v;
    }
  };
  for (int64_t bb = blockIdx.x; bb < n_tiles * n_sc; bb += gridDim.x) {
    const int64_t tile = bb % n_tiles, sc = bb / n_tiles;
    const int tx0 = (int)(tile % tiles_x) * kSmTW;
    const int ty0 = (int)(tile / tiles_x) * kBoxTH;
    const int64_t s0 = sc * kBoxSlots;
    const int ns = (int)((S - s0) < kBoxSlots ? (S - s0) : kBoxSlots);
    __syncthreads();  // the previous item is done with every LDS array
    // ---- tile setup, once for the item's slots
    for (int e = tid; e < H2 * W2; e += blockDim.x) {
      const int hy = e / W2, hx = e - hy * W2;
      const int gy = reflect_idx(ty0 + hy - R, ny);
      const int gx = reflect_idx(tx0 + hx - R, nx);
      const int lb = labels[(int64_t)gy * nx + gx] - 1;
      lab[e] = (unsigned char)((lb >= 0 && lb < D) ? lb : D);
    }
    if (tid < 2) n_list[tid] = 0;
    entry_tables(s0, 0);
    __syncthreads();
    for (int e = tid; e < kBoxTH * W2; e += blockDim.x) {
      const int r = e / W2, c = e - r * W2;
      const unsigned char L = lab[r * W2 + c];
      bool uni = true;
      for (int h = 1; h <= 2 * R; ++h) uni &= lab[(r + h) * W2 + c] == L;
      vlab[e] = uni ? L : kMixed;
      if (!uni) ylist[atomicAdd(&n_list[0], 1)] = (unsigned short)e;
    }
    __syncthreads();
    for (int e = tid; e < kBoxTH * kSmTW; e += blockDim.x) {
      const int r = e / kSmTW, x = e - r * kSmTW;
      const unsigned char* v = vlab + r * W2 + x;
      const unsigned char L = v[0];
      bool uni = L != kMixed;
      for (int j = 1; j <= 2 * R; ++j) uni &= v[j] == L;
      plab[e] = uni ? L : kMixed;
      if (!uni && ty0 + r < ny && tx0 + x < nx)
        xlist[atomicAdd(&n_list[1], 1)] = (unsigned short)e;
    }
    __syncthreads();
    const int ny_list = n_list[0], nx_list = n_list[1];
    for (int k = 0; k < ns; ++k) {
      const int b = k & 1;
      const vacc_t* t = tbl[b];
      // y pass of the mixed windows (fp64 in scipy's order, float result)
      for (int i = tid; i < ny_list; i += blockDim.x) {
        const int e = ylist[i];
        const int r = e / W2, c = e - r * W2;
        const unsigned char* col = lab + (r + R) * W2 + c;
        vacc_t acc = t[col[0]] * w[R];
#pragma unroll kTapUnroll
        for (int j = R; j >= 1; --j) acc += (t[col[-j * W2]] + t[col[j * W2]]) * w[R - j];
        vyf_t y;
#pragma unroll
        for (int p = 0; p < NP; ++p) y[p] = (float)acc[p];
        ybuf[e] = y;
      }
      __syncthreads();
      // x pass of the mixed pixels: a window's y value from ybuf (mixed) or
      // from the per-entry table (uniform)
      for (int i = tid; i < nx_list; i += blockDim.x) {
        const int e = xlist[i];
        const int r = e / kSmTW, x = e - r * kSmTW;
        const int c0 = r * W2 + x + R;
        auto ycol = [&](int c) -> vacc_t {
          const unsigned char L = vlab[c];
          return widen(L != kMixed ? yu[b][L] : ybuf[c]);
        };
        vacc_t acc = ycol(c0) * w[R];
#pragma unroll kTapUnroll
        for (int j = R; j >= 1; --j) acc += (ycol(c0 - j) + ycol(c0 + j)) * w[R - j];
        tess_v4f v;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float xv = (float)acc[p % NP];
          if (scrub && isnan(xv)) xv = (p & 1) ? 0.0f : 1.0f;
          if (be) xv = __uint_as_float(__builtin_bswap32(__float_as_uint(xv)));
          v[p] = xv;
        }
        xout[e] = v;
      }
      __syncthreads();
      // stores: wave w writes tile row w, 4 pixels per lane (1 KiB runs per
      // plane); then the next slot's per-entry tables into the other buffer
      {
        const int gy = ty0 + wv, gx0 = tx0 + 4 * l;
        if (gy < ny && gx0 < nx) {
          const int e0 = wv * kSmTW + 4 * l;
          const unsigned pl = *reinterpret_cast<const unsigned*>(plab + e0);
          tess_v4f v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const unsigned L = (pl >> (8 * i)) & 0xFF;
            v[i] = L != kMixed ? xu[b][L] : xout[e0 + i];
          }
          const int64_t so = (s0 + k + ring_base) % ring;
          float* o = out + so * 4 * P + (int64_t)gy * nx + gx0;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            if (vec) {
              __builtin_nontemporal_store(tess_v4f{v[0][p], v[1][p], v[2][p], v[3][p]},
                                          reinterpret_cast<tess_v4f*>(o + p * P));
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (gx0 + i < nx) o[p * P + i] = v[i][p];
            }
          }
        }
      }
      if (k + 1 < ns) entry_tables(s0 + k + 1, b ^ 1);
      __syncthreads();
    }
  }
}

// Separable Gaussian of Screen.write for any radius (screen.py:353-362:
// scipy.ndimage.gaussian_filter(img, sigma=(0, s, s)) per (time, freq,
// station), i.e. per image of the [.][4][ny][nx] cube): one 1-D pass per
// launch, axis y then axis x, float64 sums in scipy's order (centre first,
// then the symmetric pairs from the outermost in), float32 between the
// passes, 'reflect' borders.  The LDS tiles of kl_tess_smooth_kernel cover
// R <= kMaxR; this pair of kernels (one thread per output pixel, neighbours
// from L1 / L2) covers every R, with the NaN scrub and byte swap of the cube
// after the second pass (the reference scrubs after smoothing).
__global__ __launch_bounds__(256) void smooth_pass_kernel(
    const float* __restrict__ in, float* __restrict__ out, int nx, int ny,
    int64_t n, const double* __restrict__ gw, int R, int axis,
    unsigned flags) {
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t P = (int64_t)nx * ny;
  const int64_t img = e / P;
  const int rem = (int)(e - img * P);
  const int y = rem / nx, x = rem % nx;
  const float* base = in + img * P;
  auto at = [&](int o) -> double {
    return axis == 0 ? (double)base[(int64_t)reflect_idx(y + o, ny) * nx + x]
                     : (double)base[(int64_t)y * nx + reflect_idx(x + o, nx)];
  };
  double acc = at(0) * gw[R];
  for (int j = R; j >= 1; --j) acc += (at(-j) + at(j)) * gw[R - j];
  float v = (float)acc;
  if (flags & SF_EVAL_NAN_SCRUB) {
    // plane = image index mod 4 (cube [.][4][ny][nx]): 1.0 real, 0.0 imag
    if (isnan(v)) v = (img & 1) ? 0.0f : 1.0f;
  }
  if (flags & SF_EVAL_BIG_ENDIAN)
    v = __uint_as_float(__builtin_bswap32(__float_as_uint(v)));
  out[e] = v;
}

int launch_smooth(sf_ctx* ctx, float* cube, int nx, int ny, int64_t n_img,
                  const double* d_w, int R, unsigned flags) {
  const int64_t P = (int64_t)nx * ny;
  // the y pass goes to scratch, the x pass back into the cube, in chunks
  // of images that keep the scratch at <= 256 MiB
  int64_t chunk = ((int64_t)256 << 20) / (P * (int64_t)sizeof(float));
  if (chunk < 4) chunk = 4;
  chunk &= ~(int64_t)3;  // whole [4][ny][nx] slot cubes (plane = img % 4)
  if (chunk > n_img) chunk = n_img;
  const size_t need = (size_t)(chunk * P) * sizeof(float);
  if (ctx->smooth_cap < need) {
    if (ctx->d_smooth) (void)hipFree(ctx->d_smooth);
    ctx->d_smooth = nullptr;
    ctx->smooth_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->d_smooth), need) != hipSuccess) {
      set_error("sf_smooth: hipMalloc of the pass buffer failed");
      return SF_ENOMEM;
    }
    ctx->smooth_cap = need;
  }
  for (int64_t i0 = 0; i0 < n_img; i0 += chunk) {
    const int64_t ni = (n_img - i0 < chunk) ? n_img - i0 : chunk;
    const int64_t n = ni * P;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    float* c = cube + i0 * P;
    hipLaunchKernelGGL(smooth_pass_kernel, dim3(blocks), dim3(256), 0,
                       ctx->stream, c, ctx->d_smooth, nx, ny, n, d_w, R, 0, 0u);
    SF_HIP(hipGetLastError());
    hipLaunchKernelGGL(smooth_pass_kernel, dim3(blocks), dim3(256), 0,
                       ctx->stream, ctx->d_smooth, c, nx, ny, n, d_w, R, 1,
                       flags);
    SF_HIP(hipGetLastError());
  }
  return SF_OK;
}

// The value table of at most `per` slots (<= 256 MiB of scratch, a multiple
// of `chunk`) in the context's scratch buffer.
static int tess_table_alloc(sf_ctx* ctx, int64_t S, int64_t DT, int chunk,
                            int64_t* per_out) {
  int64_t per = (((int64_t)256 << 20) / (DT * 16)) / chunk * chunk;
  if (per < chunk) per = chunk;
  if (per > S) per = S;
  const size_t need = (size_t)(per * DT) * 16;
  if (ctx->tess_tab_cap < need) {
    if (ctx->d_tess_tab) (void)hipFree(ctx->d_tess_tab);
    ctx->d_tess_tab = nullptr;
    ctx->tess_tab_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->d_tess_tab), need) != hipSuccess) {
      set_error("sf_tess_fill: hipMalloc of the value table failed");
      return SF_ENOMEM;
    }
    ctx->tess_tab_cap = need;
  }
  *per_out = per;
  return SF_OK;
}

int launch_tess(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                const double* phase, const double* amp_xx,
                const double* amp_yy, int D, int64_t S, float* out,
                int64_t ring, const double* d_w, int R, unsigned flags) {
  const int64_t P = (int64_t)nx * ny;
  const int64_t DT = D + 1;
  // smoothing: the interior-lookup kernel or the wide-tile kernel
  // (SF_OPT_TESS_BOX; auto: interior lookups for four planes at R <= 5, where
  // the wide-tile kernel is fp64-VALU-bound -- sigma 0.25 / 0.5 / 0.75 / 1 /
  // 1.25 px: 0.66 / 0.51 / 0.42 / 0.35 / 0.31 -> 0.73 / 0.73 / 0.59 / 0.44 /
  // 0.37 of 8 TB/s; with two planes, or at R = 8, the wide-tile kernel's
  // sliding windows win: profiles/round3p_tess_box_sweep.txt)
  const bool box = R > 0 && R <= kBoxMaxR &&
                   (ctx->tess_box == 1 || (ctx->tess_box < 0 && amp_yy && R <= 5));
  int chunk = box ? kBoxSlots : kSmSlots;
  if (R == 0) {
    // the item's table slice in LDS: at most 64 KiB (63 slots at D = 64)
    chunk = ctx->tess_slots > 0 ? ctx->tess_slots : kGatherSlotsAuto;
    if (chunk * DT * 16 > 65536) chunk = (int)(65536 / (DT * 16));
  }
  int64_t per = 0;
  const int rc = tess_table_alloc(ctx, S, DT, chunk, &per);
  if (rc != SF_OK) return rc;
  tess_v4f* tab = reinterpret_cast<tess_v4f*>(ctx->d_tess_tab);
  // unsmoothed, the table entries are the pixels: scrub / swap them there
  const unsigned tab_flags = R == 0 ? flags : 0u;
  for (int64_t b = 0; b < S; b += per) {
    const int64_t Sb = S - b < per ? S - b : per;
    const int64_t n_tab = Sb * DT;
    hipLaunchKernelGGL(kl_tess_table_kernel, dim3((unsigned)((n_tab + 255) / 256)),
                       dim3(256), 0, ctx->stream, phase + b * D,
                       amp_xx ? amp_xx + b * D : nullptr,
                       amp_yy ? amp_yy + b * D : nullptr, D, Sb, tab, tab_flags);
    SF_HIP(hipGetLastError());
    const int64_t n_sc = (Sb + chunk - 1) / chunk;
    if (box) {
      const int64_t n_tiles = (int64_t)((nx + kSmTW - 1) / kSmTW) * ((ny + kBoxTH - 1) / kBoxTH);
      int64_t grid = n_tiles * n_sc;
      const int64_t cap = ((int64_t)1 << 31) / 256;
      if (grid > cap) grid = cap;  // workgroups walk the remaining items
#define SF_BOX(RT)                                                                  \
  do {                                                                              \
    if (amp_yy)                                                                     \
      hipLaunchKernelGGL((kl_tess_box_kernel<RT, 4>), dim3((unsigned)grid),         \
                         dim3(256), 0, ctx->stream, labels, nx, ny, tab, D, Sb, out, \
                         ring, b % ring, d_w, R, n_tiles, n_sc, flags);             \
    else                                                                            \
      hipLaunchKernelGGL((kl_tess_box_kernel<RT, 2>), dim3((unsigned)grid),         \
                         dim3(256), 0, ctx->stream, labels, nx, ny, tab, D, Sb, out, \
                         ring, b % ring, d_w, R, n_tiles, n_sc, flags);             \
  } while (0)
      // compiled radii: sigma up to 2 px (R <= 8); wider ones run the
      // run-time radius variant
      switch (R) {
        case 1: SF_BOX(1); break;
        case 2: SF_BOX(2); break;
        case 3: SF_BOX(3); break;
        case 4: SF_BOX(4); break;
        case 5: SF_BOX(5); break;
        case 6: SF_BOX(6); break;
        case 7: SF_BOX(7); break;
        case 8: SF_BOX(8); break;
        default: SF_BOX(0);
      }
#undef SF_BOX
      SF_HIP(hipGetLastError());
      continue;
    }
    if (R > 0) {
      const int rows = smooth_rows(R);  // the kernel's kSmTH (8 for every R > 2)
      const int64_t n_tiles = (int64_t)((nx + kSmTW - 1) / kSmTW) * ((ny + rows - 1) / rows);
      int64_t grid = n_tiles * n_sc;
      const int64_t cap = ((int64_t)1 << 31) / 256;
      if (grid > cap) grid = cap;  // workgroups walk the remaining items
#define SF_SMOOTH(RT)                                                               \
  do {                                                                              \
    if (amp_yy)                                                                     \
      hipLaunchKernelGGL((kl_tess_smooth_kernel<RT, 4>), dim3((unsigned)grid),      \
                         dim3(256), 0, ctx->stream, labels, nx, ny, tab, D, Sb, out, \
                         ring, b % ring, d_w, R, n_tiles, n_sc, flags);             \
    else                                                                            \
      hipLaunchKernelGGL((kl_tess_smooth_kernel<RT, 2>), dim3((unsigned)grid),      \
                         dim3(256), 0, ctx->stream, labels, nx, ny, tab, D, Sb, out, \
                         ring, b % ring, d_w, R, n_tiles, n_sc, flags);             \
  } while (0)
#define SF_SMOOTH2(RT)                                                              \
  hipLaunchKernelGGL((kl_tess_smooth_kernel<RT, 2>), dim3((unsigned)grid), dim3(256), \
                     0, ctx->stream, labels, nx, ny, tab, D, Sb, out, ring, b % ring,  \
                     d_w, R, n_tiles, n_sc, flags)
      switch (R) {
        case 1: SF_SMOOTH(1); break;
        case 2: SF_SMOOTH(2); break;
        case 3: SF_SMOOTH(3); break;
        case 4: SF_SMOOTH(4); break;
        case 5: SF_SMOOTH(5); break;
        case 6: SF_SMOOTH(6); break;
        case 7: SF_SMOOTH(7); break;
        case 8: SF_SMOOTH(8); break;
        // R = 9..11 compiled for both plane counts, 12..24 for two planes
        // only (four would spill); four-plane calls there take the run-time
        // radius kernel
        case 9: SF_SMOOTH(9); break;
        case 10: SF_SMOOTH(10); break;
        case 11: SF_SMOOTH(11); break;
        case 12: if (!amp_yy) { SF_SMOOTH2(12); break; } SF_SMOOTH(0); break;
        case 13: if (!amp_yy) { SF_SMOOTH2(13); break; } SF_SMOOTH(0); break;
        case 14: if (!amp_yy) { SF_SMOOTH2(14); break; } SF_SMOOTH(0); break;
        case 15: if (!amp_yy) { SF_SMOOTH2(15); break; } SF_SMOOTH(0); break;
        case 16: if (!amp_yy) { SF_SMOOTH2(16); break; } SF_SMOOTH(0); break;
        case 17: if (!amp_yy) { SF_SMOOTH2(17); break; } SF_SMOOTH(0); break;
        case 18: if (!amp_yy) { SF_SMOOTH2(18); break; } SF_SMOOTH(0); break;
        case 19: if (!amp_yy) { SF_SMOOTH2(19); break; } SF_SMOOTH(0); break;
        case 20: if (!amp_yy) { SF_SMOOTH2(20); break; } SF_SMOOTH(0); break;
        case 21: if (!amp_yy) { SF_SMOOTH2(21); break; } SF_SMOOTH(0); break;
        case 22: if (!amp_yy) { SF_SMOOTH2(22); break; } SF_SMOOTH(0); break;
        case 23: if (!amp_yy) { SF_SMOOTH2(23); break; } SF_SMOOTH(0); break;
        case 24: if (!amp_yy) { SF_SMOOTH2(24); break; } SF_SMOOTH(0); break;
        default: SF_SMOOTH(0);
      }
#undef SF_SMOOTH
#undef SF_SMOOTH2
      SF_HIP(hipGetLastError());
      continue;
    }
    const int64_t n_pb = (P + kGatherRun - 1) / kGatherRun;
    const size_t lds = (size_t)chunk * DT * 16;
    const bool vec4 = (P % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    int64_t grid = n_pb * n_sc;
    const int nw = ctx->tess_waves > 0 ? ctx->tess_waves : kGatherWavesAuto;
    const int64_t cap = ((int64_t)1 << 31) / (64 * nw);
    if (grid > cap) grid = cap;  // workgroups walk the remaining items
#define SF_GATHER(NW, V)                                                          \
  hipLaunchKernelGGL((kl_tess_gather_kernel<NW, V>), dim3((unsigned)grid),       \
                     dim3(64 * NW), lds, ctx->stream, labels, P, tab, D, Sb, out, \
                     ring, b % ring, n_pb, n_sc, chunk)
    if (vec4) {
      if (nw == 4) SF_GATHER(4, true);
      else if (nw == 8) SF_GATHER(8, true);
      else SF_GATHER(16, true);
    } else {
      SF_GATHER(4, false);
    }
#undef SF_GATHER
    SF_HIP(hipGetLastError());
  }
  return SF_OK;
}

// The round-1 fused tile kernel (16 x 16 tiles, table built per tile), kept
// for cross-checks (SF_OPT_TESS_TILE): same bits as launch_tess.
int launch_tess_tile(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                     const double* phase, const double* amp_xx,
                     const double* amp_yy, int D, int64_t S, float* out,
                     int64_t ring, const double* d_w, int R, unsigned flags) {
  const int tiles = ((nx + kTT - 1) / kTT) * ((ny + kTT - 1) / kTT);
  const int64_t chunks = (S + kTessSlots - 1) / kTessSlots;
  hipLaunchKernelGGL(kl_tess_kernel, dim3(tiles, (unsigned)chunks), dim3(256),
                     0, ctx->stream, labels, nx, ny, phase, amp_xx, amp_yy, D,
                     S, out, ring, d_w, R, flags);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

}  // namespace sf

// tess.hip -- tessellated (Voronoi) screen fill + Gaussian smoothing, fused.
//
// Replaces VoronoiScreen.make_matrix (voronoi_screen.py:132-216) and the
// per-(time, freq, station) scipy.ndimage.gaussian_filter of Screen.write
// (screen.py:353-362):
//   out[s][p][y][x] = g(value_p[s][label[y][x] - 1]),  value_p in
//     {A_xx cos(phi), A_xx sin(phi), A_yy cos(phi), A_yy sin(phi)}
// with g = identity or the separable Gaussian (axis y then axis x, float32
// between the passes, 'reflect' borders, scipy's symmetric-kernel summation
// order in float64).  One workgroup = a 16 x 16 output tile and a chunk of
// slots; the label tile (+halo) stays in LDS for the whole chunk, so the only
// HBM traffic is the 16 B / pixel / slot output write.
#include <hip/hip_runtime.h>

#include <cmath>

#include "sf_internal.h"

namespace sf {

constexpr int kTT = 16;       // output tile side
constexpr int kMaxR = kTessMaxR;  // fused-tile Gaussian radius (sigma <= 6 px)
constexpr int kTessSlots = 64;  // slots per workgroup

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // scipy.ndimage mode 'reflect': d c b a | a b c d | d c b a
  while (i < 0 || i >= n) {
    if (i < 0) i = -i - 1;
    if (i >= n) i = 2 * n - i - 1;
  }
  return i;
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
// pure gather-store, laid out for HBM writes.  A workgroup owns a run of
// kGatherRun consecutive pixels (4 per lane, 1 KiB per wave and plane) and a
// chunk of kGatherSlots slots: it first builds the chunk's value table in LDS
// -- per (slot, direction) the float4 {A_xx cos, A_xx sin, A_yy cos, A_yy
// sin} with the NaN scrub and the byte swap already applied (the output IS
// the table entry when nothing is smoothed, so scrubbing the entry equals
// scrubbing the pixel) -- keeps its 4 labels in registers, and then per slot
// reads 4 table entries (ds_read_b128) and writes 4 float4 stores, one per
// plane: 4 KiB contiguous runs per (slot, plane) per workgroup.  Same fp64
// sincos and casts as kl_tess_kernel, so the same bits.
constexpr int kGatherWaves = 4;
constexpr int kGatherRun = 64 * 4 * kGatherWaves;  // pixels per workgroup
constexpr int kGatherSlots = 32;                   // slots per work item

template <bool VEC4>
__global__ __launch_bounds__(64 * kGatherWaves) void kl_tess_gather_kernel(
    const int32_t* __restrict__ labels, int64_t P,
    const double* __restrict__ phase, const double* __restrict__ amp_xx,
    const double* __restrict__ amp_yy, int D, int64_t S,
    float* __restrict__ out, int64_t ring, int64_t n_pb, int64_t n_sc,
    unsigned flags) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  extern __shared__ v4f gtab[];  // [kGatherSlots][D + 1]
  const int DT = D + 1;          // entry D: invalid labels (NaN / scrubbed)
  const bool scrub = flags & SF_EVAL_NAN_SCRUB;
  const bool be = flags & SF_EVAL_BIG_ENDIAN;
  auto fin = [&](float x, int p) {
    if (scrub && isnan(x)) x = (p & 1) ? 0.0f : 1.0f;
    if (be) x = __uint_as_float(__builtin_bswap32(__float_as_uint(x)));
    return x;
  };
  for (int64_t bb = blockIdx.x; bb < n_pb * n_sc; bb += gridDim.x) {
    const int64_t pb = bb % n_pb, sc = bb / n_pb;
    const int64_t s0 = sc * kGatherSlots;
    const int ns = (int)((S - s0) < kGatherSlots ? (S - s0) : kGatherSlots);
    __syncthreads();  // the previous item's table reads are done
    for (int e = threadIdx.x; e < ns * DT; e += blockDim.x) {
      const int k = e / DT, d = e - k * DT;
      v4f v;
      if (d < D) {
        const int64_t i = (s0 + k) * D + d;
        double sn, cn;
        sincos(phase[i], &sn, &cn);
        const double ax = amp_xx ? amp_xx[i] : 1.0;
        const double ay = amp_yy ? amp_yy[i] : ax;
        v = v4f{(float)(ax * cn), (float)(ax * sn), (float)(ay * cn), (float)(ay * sn)};
      } else {
        const float q = __builtin_nanf("");
        v = v4f{q, q, q, q};
      }
      gtab[e] = v4f{fin(v[0], 0), fin(v[1], 1), fin(v[2], 2), fin(v[3], 3)};
    }
    __syncthreads();
    const int64_t p0 = pb * kGatherRun + 4 * (int64_t)threadIdx.x;
    if (p0 >= P) continue;  // after the barrier: nothing below syncs
    int lab[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int lb = (p0 + j < P) ? labels[p0 + j] - 1 : 0;
      lab[j] = (lb >= 0 && lb < D) ? lb : D;
    }
    for (int k = 0; k < ns; ++k) {
      const v4f* t = gtab + k * DT;
      const v4f a = t[lab[0]], b = t[lab[1]], c = t[lab[2]], d = t[lab[3]];
      float* o = out + ((s0 + k) % ring) * 4 * P + p0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (VEC4) {
          __builtin_nontemporal_store(v4f{a[q], b[q], c[q], d[q]},
                                      reinterpret_cast<v4f*>(o + q * P));
        } else {
          const float v[4] = {a[q], b[q], c[q], d[q]};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (p0 + j < P) o[q * P + j] = v[j];
        }
      }
    }
  }
}

// Separable Gaussian of Screen.write for any radius (screen.py:353-362:
// scipy.ndimage.gaussian_filter(img, sigma=(0, s, s)) per (time, freq,
// station), i.e. per image of the [.][4][ny][nx] cube): one 1-D pass per
// launch, axis y then axis x, float64 sums in scipy's order (centre first,
// then the symmetric pairs from the outermost in), float32 between the
// passes, 'reflect' borders.  The fused LDS tile of kl_tess_kernel covers
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

int launch_tess(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                const double* phase, const double* amp_xx,
                const double* amp_yy, int D, int64_t S, float* out,
                int64_t ring, const double* d_w, int R, unsigned flags) {
  if (R == 0) {
    const int64_t P = (int64_t)nx * ny;
    const int64_t n_pb = (P + kGatherRun - 1) / kGatherRun;
    const int64_t n_sc = (S + kGatherSlots - 1) / kGatherSlots;
    int64_t grid = n_pb * n_sc;
    const int64_t cap = ((int64_t)1 << 31) / (64 * kGatherWaves);
    if (grid > cap) grid = cap;  // workgroups walk the remaining items
    const size_t lds = (size_t)kGatherSlots * (D + 1) * 4 * sizeof(float);
    const bool vec4 = (P % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    if (vec4)
      hipLaunchKernelGGL(kl_tess_gather_kernel<true>, dim3((unsigned)grid),
                         dim3(64 * kGatherWaves), lds, ctx->stream, labels, P,
                         phase, amp_xx, amp_yy, D, S, out, ring, n_pb, n_sc, flags);
    else
      hipLaunchKernelGGL(kl_tess_gather_kernel<false>, dim3((unsigned)grid),
                         dim3(64 * kGatherWaves), lds, ctx->stream, labels, P,
                         phase, amp_xx, amp_yy, D, S, out, ring, n_pb, n_sc, flags);
    SF_HIP(hipGetLastError());
    return SF_OK;
  }
  const int tiles = ((nx + kTT - 1) / kTT) * ((ny + kTT - 1) / kTT);
  const int64_t chunks = (S + kTessSlots - 1) / kTessSlots;
  hipLaunchKernelGGL(kl_tess_kernel, dim3(tiles, (unsigned)chunks), dim3(256),
                     0, ctx->stream, labels, nx, ny, phase, amp_xx, amp_yy, D,
                     S, out, ring, d_w, R, flags);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

}  // namespace sf

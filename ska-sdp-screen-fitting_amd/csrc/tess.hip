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
  const int tiles = ((nx + kTT - 1) / kTT) * ((ny + kTT - 1) / kTT);
  const int64_t chunks = (S + kTessSlots - 1) / kTessSlots;
  hipLaunchKernelGGL(kl_tess_kernel, dim3(tiles, (unsigned)chunks), dim3(256),
                     0, ctx->stream, labels, nx, ny, phase, amp_xx, amp_yy, D,
                     S, out, ring, d_w, R, flags);
  SF_HIP(hipGetLastError());
  return SF_OK;
}

}  // namespace sf

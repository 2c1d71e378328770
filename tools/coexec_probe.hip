// Two probes for the evaluation epilogue design on gfx950:
//  (1) co-execution: waves 0-3 of a 512-thread workgroup (one per SIMD) run
//      v_mfma_f64_16x16x4_f64 chains, waves 4-7 (the same SIMDs) run VALU
//      chains (fp32 FMA, fp64 FMA or v_sin_f32); time of each alone and of
//      both together -- sum => the pipes serialise, max => they overlap;
//  (2) accuracy of the hardware v_sin_f32 / v_cos_f32 (argument in
//      revolutions) over [-0.5, 0.5] against fp64 sin / cos(2 pi x).
//   hipcc --offload-arch=gfx950 -O3 tools/coexec_probe.hip -o tools/coexec_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

// mode bit 0: MFMA waves work, bit 1: VALU waves work; vk = VALU kind
__global__ __launch_bounds__(512) void coexec(double* out, int iters, int mode, int vk) {
  const int w = threadIdx.x >> 6;
  double acc_s = 0;
  if (w < 4) {
    if (mode & 1) {
      v4d acc[4];
      for (int i = 0; i < 4; ++i) acc[i] = v4d{0, 0, 0, 0};
      double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
      for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 4; ++i) acc_s += acc[i][0] + acc[i][3];
    }
  } else if (mode & 2) {
    // 16 VALU instructions per MFMA of the partner wave (iters x 4 MFMA)
    if (vk == 0) {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
      for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16 * 8; ++u)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = fmaf(x[i], 0.999f, 0.5f);
      }
      for (int i = 0; i < 8; ++i) acc_s += x[i];
    } else if (vk == 1) {
      double x[8];
      for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
      for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16 * 8; ++u)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = fma(x[i], 0.999, 0.5);
      }
      for (int i = 0; i < 8; ++i) acc_s += x[i];
    } else {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-5f + i * 0.01f;
      for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16 * 8; ++u)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_sinf(x[i]);
      }
      for (int i = 0; i < 8; ++i) acc_s += x[i];
    }
  }
  if (acc_s == 1234.5678) out[threadIdx.x] = acc_s;
}

// per-block max |error| of v_sin_f32 / v_cos_f32 vs fp64 sin / cos(2 pi x)
__global__ __launch_bounds__(256) void sin_acc(long n, double* err) {
  __shared__ double es[256], ec[256];
  double ms = 0, mc = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float x = -0.5f + (float)((double)i / n);
    const float s = __builtin_amdgcn_sinf(x), c = __builtin_amdgcn_cosf(x);
    const double xs = 6.283185307179586 * (double)x;
    ms = fmax(ms, fabs((double)s - sin(xs)));
    mc = fmax(mc, fabs((double)c - cos(xs)));
  }
  es[threadIdx.x] = ms;
  ec[threadIdx.x] = mc;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 256; ++i) {
      ms = fmax(ms, es[i]);
      mc = fmax(mc, ec[i]);
    }
    err[2 * blockIdx.x] = ms;
    err[2 * blockIdx.x + 1] = mc;
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  double* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  const char* vk_name[3] = {"fp32 fma", "fp64 fma", "v_sin_f32"};
  for (int vk = 0; vk < 3; ++vk) {
    for (int mode = 1; mode <= 3; ++mode) {
      hipLaunchKernelGGL(coexec, dim3(cus), dim3(512), 0, 0, d, 64, mode, vk);
      hipEventRecord(e0);
      hipLaunchKernelGGL(coexec, dim3(cus), dim3(512), 0, 0, d, iters, mode, vk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("coexec %-9s %s: %.3f ms\n", vk_name[vk],
             mode == 1 ? "MFMA only" : mode == 2 ? "VALU only" : "MFMA+VALU", ms);
    }
  }
  const long n = 1L << 28;
  const int nb = 1024;
  hipLaunchKernelGGL(sin_acc, dim3(nb), dim3(256), 0, 0, n, d);
  static double h[2 * 1024];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double ms = 0, mc = 0;
  for (int i = 0; i < nb; ++i) {
    ms = fmax(ms, h[2 * i]);
    mc = fmax(mc, h[2 * i + 1]);
  }
  printf("v_sin_f32 max abs err %.3g, v_cos_f32 max abs err %.3g over %ld points in [-0.5, 0.5] rev\n",
         ms, mc, n);
  hipFree(d);
  return 0;
}

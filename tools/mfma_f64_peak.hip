// fp64 MFMA throughput probe (v_mfma_f64_16x16x4_f64) on gfx950: every wave
// issues ITERS x NACC MFMAs on NACC independent accumulators; the chip rate
// in TFLOP/s and the cycles per MFMA per SIMD at the measured clock follow.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_peak.hip -o tools/mfma_f64_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0) {
  v4d acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = v4d{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  // unrolled by 32 so the accumulators stay in place (a rolled loop makes
  // the compiler copy them through VGPRs every iteration)
  for (int it = 0; it < iters; it += 32) {
#pragma unroll
    for (int u = 0; u < 32; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i)
        acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;  // keep the loop alive
}

template <int NACC>
static void run(int blocks_per_cu, int waves_per_block, double* d) {
  int dev = 0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  const int iters = 4096;
  dim3 grid(cus * blocks_per_cu), block(64 * waves_per_block);
  hipLaunchKernelGGL(mfma_loop<NACC>, grid, block, 0, 0, d, 32, 1.0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<NACC>, grid, block, 0, 0, d, iters, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = (double)grid.x * waves_per_block;
  const double n_mfma = waves * iters * NACC;
  const double tf = n_mfma * 2048.0 / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD at 2.4 GHz if every SIMD were busy
  const double per_simd = n_mfma / (cus * 4.0);
  printf("NACC=%d waves/CU=%d: %.3f ms, %.1f TFLOP/s, %.1f cyc/MFMA/SIMD @2.4GHz\n",
         NACC, blocks_per_cu * waves_per_block, ms, tf, ms * 1e-3 * 2.4e9 / per_simd);
}

int main() {
  double* d;
  hipMalloc(&d, 4096 * sizeof(double));
  run<1>(1, 4, d);
  run<4>(1, 4, d);
  run<4>(2, 4, d);
  run<8>(2, 4, d);
  run<4>(4, 4, d);
  hipFree(d);
  return 0;
}

// v_mfma_i32_16x16x64_i8 probe on gfx950, before the integer-digit evaluation
// contraction relies on it:
//  1. operand / result lane maps with exact random int8 data: lane l holds
//     A[row l & 15][k = 16 (l >> 4) + j] and B[k = 16 (l >> 4) + j][col l & 15]
//     in byte j of its 16-byte fragment (the contraction only needs A and B to
//     share the k map), D[row 4 (l >> 4) + r][col l & 15] in register r;
//  2. int32 accumulation wraps modulo 2^32 (C near INT32_MAX);
//  3. issue rate: cycles per MFMA per SIMD with 4 independent accumulators,
//     beside the fp64 16x16x4 loop, and the shader clock each loop ran at
//     (s_memtime ticks / event time).
//   hipcc --offload-arch=gfx950 -O3 tools/i8_mfma_probe.hip -o tools/i8_mfma_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const int8_t* A, const int8_t* B, const int* C, int* D) {
  const int l = threadIdx.x;
  union { v4i v; int8_t b[16]; } a, b;
  for (int j = 0; j < 16; ++j) {
    const int k = 16 * (l >> 4) + j;
    a.b[j] = A[(l & 15) * 64 + k];
    b.b[j] = B[k * 16 + (l & 15)];
  }
  v4i c;
  for (int r = 0; r < 4; ++r) c[r] = C[(4 * (l >> 4) + r) * 16 + (l & 15)];
  const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, b.v, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = d[r];
}

template <bool I8>
__global__ __launch_bounds__(256) void rate_kernel(int* out, unsigned long long* ticks,
                                                   int iters) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  v4i ai[4];
  v4d ad[4];
  for (int i = 0; i < 4; ++i) {
    ai[i] = v4i{0, 0, 0, 0};
    ad[i] = v4d{0, 0, 0, 0};
  }
  const v4i a = v4i{(int)threadIdx.x, 3, -5, 7};
  const v4i b = v4i{11, (int)threadIdx.x * 3, 1, -2};
  const double x = 1.0 + threadIdx.x * 1e-9, y = 1.0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; it += 16) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (I8)
          ai[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, ai[i], 0, 0, 0);
        else
          ad[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, ad[i], 0, 0, 0);
      }
  }
  long long s = 0;
  for (int i = 0; i < 4; ++i)
    s += ai[i][0] + ai[i][1] + ai[i][2] + ai[i][3] +
         (long long)(ad[i][0] + ad[i][1] + ad[i][2] + ad[i][3]);
  if (s == 123456789) out[threadIdx.x] = (int)s;  // keep the loop
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

static int check_layout() {
  std::vector<int8_t> A(16 * 64), B(64 * 16);
  std::vector<int> C(256), D(256), want(256);
  srand(7);
  for (auto& v : A) v = (int8_t)(rand() & 255);
  for (auto& v : B) v = (int8_t)(rand() & 255);
  for (int i = 0; i < 256; ++i) C[i] = (i % 3 == 0) ? 2147483000 : (rand() % 2001) - 1000;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      long long s = C[i * 16 + j];
      for (int k = 0; k < 64; ++k) s += (long long)A[i * 64 + k] * B[k * 16 + j];
      want[i * 16 + j] = (int)(uint32_t)(uint64_t)s;  // modulo 2^32
    }
  int8_t *dA, *dB;
  int *dC, *dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dC, 1024);
  hipMalloc(&dD, 1024);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
  hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
  int bad = 0, wrapped = 0;
  for (int i = 0; i < 256; ++i) {
    bad += D[i] != want[i];
    wrapped += (C[i] == 2147483000) && (want[i] < 0);
  }
  printf("layout: %d / 256 mismatches (%d results wrapped past INT32_MAX)\n", bad, wrapped);
  hipFree(dA);
  hipFree(dB);
  hipFree(dC);
  hipFree(dD);
  return bad;
}

template <bool I8>
static void rate(int* d, unsigned long long* ticks, int cus) {
  const int iters = 8192, blocks = cus * 2;  // 2 x 4 waves per CU: 2 per SIMD
  hipLaunchKernelGGL(rate_kernel<I8>, dim3(blocks), dim3(256), 0, 0, d, ticks, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(rate_kernel<I8>, dim3(blocks), dim3(256), 0, 0, d, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> t(blocks);
  hipMemcpy(t.data(), ticks, blocks * 8, hipMemcpyDeviceToHost);
  double tick_avg = 0;
  for (auto v : t) tick_avg += (double)v / blocks;
  const double per_simd = (double)blocks * 4 * iters * 4 / (cus * 4.0);  // MFMAs per SIMD
  const double clk = tick_avg / (ms * 1e-3);
  printf("%s: %.3f ms, %.1f cycles per MFMA per SIMD at the measured %.2f GHz "
         "(s_memtime ticks %.3g per wave)\n",
         I8 ? "v_mfma_i32_16x16x64_i8 " : "v_mfma_f64_16x16x4_f64",
         ms, ms * 1e-3 * clk / per_simd, clk * 1e-9, tick_avg);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("%s, %d CUs\n", p.gcnArchName, p.multiProcessorCount);
  const int bad = check_layout();
  int* d;
  unsigned long long* ticks;
  hipMalloc(&d, 4096);
  hipMalloc(&ticks, 8 * p.multiProcessorCount * 2);
  rate<true>(d, ticks, p.multiProcessorCount);
  rate<false>(d, ticks, p.multiProcessorCount);
  rate<true>(d, ticks, p.multiProcessorCount);
  return bad ? 1 : 0;
}

// Pure-store HBM bandwidth probe (float4 stores, plain vs non-temporal), to
// calibrate what a write-bound kernel can reach on this MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void fill(float4* __restrict__ p4, size_t n, float v) {
  v4f* p = reinterpret_cast<v4f*>(p4);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    v4f x = {v, v + 1, v + 2, v + 3};
    if (NT) __builtin_nontemporal_store(x, p + i);
    else p[i] = x;
  }
}

__global__ __launch_bounds__(256) void copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)16 << 30;
  const size_t n = bytes / 16;
  float4* p;
  float4* q;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&q, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {1024, 4096, 16384, 65536}) {
    for (int nt = 0; nt < 2; ++nt) {
      float best = 1e9;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        if (nt) hipLaunchKernelGGL(fill<true>, dim3(grid), dim3(256), 0, 0, p, n, 1.0f);
        else hipLaunchKernelGGL(fill<false>, dim3(grid), dim3(256), 0, 0, p, n, 1.0f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      printf("store grid=%6d nt=%d: %.1f GB/s\n", grid, nt, bytes / (best * 1e-3) / 1e9);
    }
  }
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(copy, dim3(16384), dim3(256), 0, 0, p, q, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  printf("copy (read+write): %.1f GB/s\n", 2 * bytes / (best * 1e-3) / 1e9);
  float ms;
  hipEventRecord(e0);
  hipMemsetAsync(p, 0, bytes);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("hipMemset: %.1f GB/s\n", bytes / (ms * 1e-3) / 1e9);
  return 0;
}

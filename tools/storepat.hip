// Store-pattern probe: the eval kernel's exact output address pattern with no
// compute, versus longer contiguous runs, to see what the pattern alone can
// reach.  out[S][4][P] float32, P = 256^2, 16 GiB.
//   A: eval mapping -- wave = 64 px x 16 slots; one float4 store instruction
//      covers 4 slots x 256 B (per plane)
//   B: wave = 256 px x 4 slots; one instruction covers 1 slot x 1 KiB
//   C: grid-stride fill (upper bound)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st(float* p, v4f v) {
  __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
}

constexpr long P = 65536;

__global__ __launch_bounds__(256) void patA(float* out, long S, long n_pb) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long b = blockIdx.x;
  const long per = n_pb >> 3, x = b & 7, i = b >> 3;
  const long pb = x * per + (i % per), sc = i / per;
  const long p0 = (pb * 4 + w) * 64 + (l & 15) * 4;
  for (int g = 0; g < 16; ++g) {
    const long s0 = sc * 256 + g * 16;
    if (s0 >= S) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + (l >> 4) + 4 * r;
      float* o = out + s * 4 * P + p0;
      v4f v = {1.f, 2.f, 3.f, (float)r};
#pragma unroll
      for (int q = 0; q < 4; ++q) st(o + q * P, v);
    }
  }
}

__global__ __launch_bounds__(256) void patB(float* out, long S, long n_pb) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long b = blockIdx.x;
  const long per = n_pb >> 3, x = b & 7, i = b >> 3;
  const long pb = x * per + (i % per), sc = i / per;
  const long p0 = pb * 256 + l * 4;
  for (int g = 0; g < 16; ++g) {
    const long s0 = sc * 256 + g * 16;
    if (s0 >= S) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + w * 4 + r;
      float* o = out + s * 4 * P + p0;
      v4f v = {1.f, 2.f, 3.f, (float)r};
#pragma unroll
      for (int q = 0; q < 4; ++q) st(o + q * P, v);
    }
  }
}

// D: wave = 1024 px x 1 slot per group row: 4 consecutive 1 KiB stores per
// (slot, plane) -> 4 KiB contiguous per wave
__global__ __launch_bounds__(256) void patD(float* out, long S, long n_pb4) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long b = blockIdx.x;
  const long per = n_pb4 >> 3, x = b & 7, i = b >> 3;
  const long pb = x * per + (i % per), sc = i / per;
  const long p0 = pb * 1024 + l * 4;
  for (int g = 0; g < 16; ++g) {
    const long s0 = sc * 256 + g * 16;
    if (s0 >= S) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + w * 4 + r;
      float* o = out + s * 4 * P + p0;
      v4f v = {1.f, 2.f, 3.f, (float)r};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int h = 0; h < 4; ++h) st(o + q * P + h * 256, v);
    }
  }
}

// E: each wave owns a contiguous chunk and streams through it
__global__ __launch_bounds__(256) void patE(float* out, long n4, long per_wave) {
  const int l = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long base = wave * per_wave;
  for (long i = 0; i < per_wave; i += 64) {
    const long k = base + i + l;
    if (k < n4) {
      v4f v = {1.f, 2.f, 3.f, 4.f};
      st(out + 4 * k, v);
    }
  }
}

__global__ __launch_bounds__(256) void patC(float* out, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    v4f v = {1.f, 2.f, 3.f, 4.f};
    st(out + 4 * i, v);
  }
}

int main() {
  const long S = 16384;
  const size_t bytes = (size_t)S * 4 * P * 4;
  float* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  const long n_pb = P / 256, n_sc = S / 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int k = 0; k < 5; ++k) {
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(patA, dim3(n_pb * n_sc), dim3(256), 0, 0, out, S, n_pb);
      if (k == 1) hipLaunchKernelGGL(patB, dim3(n_pb * n_sc), dim3(256), 0, 0, out, S, n_pb);
      if (k == 2) hipLaunchKernelGGL(patC, dim3(16384), dim3(256), 0, 0, out, (long)(bytes / 16));
      if (k == 3) hipLaunchKernelGGL(patD, dim3(n_pb / 4 * n_sc), dim3(256), 0, 0, out, S, n_pb / 4);
      if (k == 4) {
        const long n4 = (long)(bytes / 16), waves = 16384L * 4;
        hipLaunchKernelGGL(patE, dim3(16384), dim3(256), 0, 0, out, n4, (n4 + waves - 1) / waves);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    printf("pattern %c: %.1f GB/s (%.3f ms)\n", "ABCDE"[k], bytes / (best * 1e-3) / 1e9, best);
  }
  return 0;
}

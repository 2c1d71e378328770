// Issue cost on gfx950 of the VALU instructions the evaluation epilogues
// use, one wave per SIMD (256-thread workgroups, one per CU) and four waves
// per SIMD: 8 independent register streams per lane, each instruction
// written as inline asm so the count is exact.  Prints cycles per wave
// instruction per SIMD (clock from the device's reported clock rate, so
// compare the rows with each other, not with the guide's constants).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_cost_probe.hip -o tools/valu_cost_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ __launch_bounds__(1024) void probe(float* out, int iters) {
  float f[8];
  double d[8];
  int i32[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    f[k] = 0.01f * (threadIdx.x + k);
    d[k] = 1.37 * (threadIdx.x + k) + 0.25;
    i32[k] = threadIdx.x * 977 + k;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#define OP(k)                                                                        \
  if constexpr (K == 0) asm volatile("v_mul_f32 %0, %0, %0" : "+v"(f[k]));          \
  if constexpr (K == 1) asm volatile("v_add_f64 %0, %0, %0" : "+v"(d[k]));          \
  if constexpr (K == 2) asm volatile("v_rndne_f64 %0, %0" : "+v"(d[k]));            \
  if constexpr (K == 3) asm volatile("v_fract_f64 %0, %0" : "+v"(d[k]));            \
  if constexpr (K == 4) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[k]) : "v"(d[k])); \
  if constexpr (K == 5) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(i32[k]));        \
  if constexpr (K == 6) asm volatile("v_exp_f32 %0, %0" : "+v"(f[k]));              \
  if constexpr (K == 7) asm volatile("v_sin_f32 %0, %0" : "+v"(f[k]));              \
  if constexpr (K == 8) asm volatile("v_cmp_u_f32 vcc, %0, %0" : : "v"(f[k]) : "vcc"); \
  if constexpr (K == 9) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[k]));      \
  if constexpr (K == 10) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[k]));         \
  if constexpr (K == 11) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[k]) : "v"(f[k])); \
  if constexpr (K == 12) asm volatile("v_cndmask_b32 %0, %0, %0, vcc" : "+v"(i32[k]) : : "vcc"); \
  if constexpr (K == 13) asm volatile("v_add_u32 %0, %0, %0" : "+v"(i32[k]));
      R8(OP)
#undef OP
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += f[k] + (float)d[k] + (float)i32[k];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

static const char* kName[] = {"v_mul_f32", "v_add_f64", "v_rndne_f64", "v_fract_f64",
                              "v_cvt_f32_f64", "v_cvt_f32_i32", "v_exp_f32",
                              "v_sin_f32", "v_cmp_u_f32", "v_fma_f64", "v_mul_f64",
                              "v_cvt_f64_f32", "v_cndmask_b32", "v_add_u32"};

template <int K>
static void run(int cus, double ghz, float* d, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 2048;
  for (int wps : {1, 4}) {
    const int threads = 256 * wps;
    hipLaunchKernelGGL(probe<K>, dim3(cus), dim3(threads), 0, 0, d, 16);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<K>, dim3(cus), dim3(threads), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double inst = (double)iters * 16 * 8 * wps;  // per SIMD
    printf("%-14s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (%.3f ms)\n",
           kName[K], wps, ms * 1e-3 * ghz * 1e9 / inst, ms);
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate * 1e-6;
  printf("%d CUs, reported clock %.3f GHz\n", cus, ghz);
  float* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  run<0>(cus, ghz, d, e0, e1);
  run<1>(cus, ghz, d, e0, e1);
  run<2>(cus, ghz, d, e0, e1);
  run<3>(cus, ghz, d, e0, e1);
  run<4>(cus, ghz, d, e0, e1);
  run<5>(cus, ghz, d, e0, e1);
  run<6>(cus, ghz, d, e0, e1);
  run<7>(cus, ghz, d, e0, e1);
  run<8>(cus, ghz, d, e0, e1);
  run<9>(cus, ghz, d, e0, e1);
  run<10>(cus, ghz, d, e0, e1);
  run<11>(cus, ghz, d, e0, e1);
  run<12>(cus, ghz, d, e0, e1);
  run<13>(cus, ghz, d, e0, e1);
  hipFree(d);
  return 0;
}

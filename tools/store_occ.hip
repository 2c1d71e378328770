// Store-ceiling probe for the evaluation's output stream: what sets the
// chip's store rate -- resident waves per CU, work-item shape, or address
// order?  out = 16 GiB of float32 viewed as [S = 16384 slots][4 planes][256^2].
//   lin/k   : one-shot 256-thread workgroups, each one float4 per thread
//             (4 KiB contiguous, the torch fill_ shape), in address order;
//             dynamic LDS caps residency at k workgroups per CU
//   evo/k   : the same 4 KiB pieces in the LDS eval kernel's order (16-slot
//             chunk -> 1024-pixel block -> slot -> plane -> 4 KiB), k per CU
//   item/k  : one workgroup of 256 threads per (1024-px block, 16-slot chunk)
//             writing its 64 pieces (16 slots x 4 planes x 4 KiB), k per CU
//   item16/k: the same item with 1024 threads (the LDS16 kernel's shape)
//   hipMemset for reference
//   hipcc --offload-arch=gfx950 -O3 tools/store_occ.hip -o tools/store_occ
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr long kP = 65536, kS = 16384;
constexpr long kPieces = kS * 4 * kP / 1024;  // 4 KiB pieces (1024 floats)

__device__ __forceinline__ void st(float* p, v4f v) {
  __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
}

// piece index -> float offset, eval order: chunk of 16 slots, 64 pixel
// blocks of 1024 px (XCD-interleaved as the kernel's map: block = x (mod 8)),
// then slot, plane
__device__ __forceinline__ long evo_offset(long k) {
  const long within = k & 63;            // 16 slots x 4 planes
  const long item = k >> 6;              // (chunk, pixel block)
  const long pb = item & 63, sc = item >> 6;
  const long s = sc * 16 + (within >> 2), q = within & 3;
  return (s * 4 + q) * kP + pb * 1024;
}

template <int ORDER>
__global__ __launch_bounds__(256) void one_shot(float* out) {
  extern __shared__ float pad[];
  const long k = blockIdx.x;
  const long base = ORDER == 0 ? k * 1024 : evo_offset(k);
  v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  if (threadIdx.x == 1023) pad[0] = v[0];  // never: keeps the LDS allocation
  st(out + base + threadIdx.x * 4, v);
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void item_kernel(float* out) {
  extern __shared__ float pad[];
  const long item = blockIdx.x;           // (chunk, pixel block)
  const long pb = item & 63, sc = item >> 6;
  v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  if (threadIdx.x == 4095) pad[0] = v[0];
  // 64 pieces of 1024 floats; THREADS / 256 pieces at a time
  for (int j = threadIdx.x / 256; j < 64; j += THREADS / 256) {
    const long s = sc * 16 + (j >> 2), q = j & 3;
    st(out + (s * 4 + q) * kP + pb * 1024 + (threadIdx.x & 255) * 4, v);
  }
}

// the LDS16 eval kernel's store phase: 16 waves, a (16-slot, 1024-px) item
// is 16 slots x 4 planes x 4 KiB.  MODE 0: wave w stores slot w (its 4 planes
// x 4 x 1 KiB) -- the round-2 kernel; MODE 1: slot-major -- for slot j = 0..15
// the 16 waves store its 4 planes x 4 chunks together (one 1 KiB run each)
template <int MODE>
__global__ __launch_bounds__(1024) void item16(float* out, long n_items) {
  extern __shared__ float pad[];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  if (threadIdx.x == 4095) pad[0] = v[0];
  for (long item = blockIdx.x; item < n_items; item += gridDim.x) {
    const long pb = item & 63, sc = item >> 6;
    if (MODE == 0) {
      const long s = sc * 16 + w;
      for (int q = 0; q < 4; ++q)
        for (int c = 0; c < 4; ++c)
          st(out + (s * 4 + q) * kP + pb * 1024 + c * 256 + l * 4, v);
    } else {
      const int q = w >> 2, c = w & 3;
      for (int j = 0; j < 16; ++j) {
        const long s = sc * 16 + j;
        st(out + (s * 4 + q) * kP + pb * 1024 + c * 256 + l * 4, v);
      }
    }
  }
}

int main() {
  float* out;
  const size_t bytes = (size_t)kS * 4 * kP * sizeof(float);
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-28s %7.1f GB/s  (%.3f ms)\n", name, bytes / (best * 1e-3) / 1e9, best);
  };
  const int ks[] = {1, 2, 4, 8};
  for (int k : ks) {
    const size_t lds = 160 * 1024 / k - 256;
    char n0[64], n1[64], n2[64], n3[64];
    snprintf(n0, 64, "lin  one-shot 4KiB, %d/CU", k);
    snprintf(n1, 64, "evo  one-shot 4KiB, %d/CU", k);
    snprintf(n2, 64, "item 256 thr 64 pieces, %d/CU", k);
    snprintf(n3, 64, "item 1024 thr 64 pieces, %d/CU", k);
    time(n0, [&] { hipLaunchKernelGGL(one_shot<0>, dim3(kPieces), dim3(256), lds, 0, out); });
    time(n1, [&] { hipLaunchKernelGGL(one_shot<1>, dim3(kPieces), dim3(256), lds, 0, out); });
    time(n2, [&] { hipLaunchKernelGGL(item_kernel<256>, dim3(kPieces / 64), dim3(256), lds, 0, out); });
    if (k <= 2)
      time(n3, [&] { hipLaunchKernelGGL(item_kernel<1024>, dim3(kPieces / 64), dim3(1024), lds, 0, out); });
  }
  const long n_items = kPieces / 64;
  for (int grid_mul : {0, 1}) {
    // grid_mul 0: one workgroup per item (one-shot); 1: 256 x 1 persistent
    const long grid = grid_mul ? 256 : n_items;
    for (size_t lds : {(size_t)131584, (size_t)65536}) {
      char a[96], b[96];
      snprintf(a, 96, "item16 wave-per-slot %s lds%zuK", grid_mul ? "persist" : "1shot", lds / 1024);
      snprintf(b, 96, "item16 slot-major    %s lds%zuK", grid_mul ? "persist" : "1shot", lds / 1024);
      time(a, [&] { hipLaunchKernelGGL(item16<0>, dim3(grid), dim3(1024), lds, 0, out, n_items); });
      time(b, [&] { hipLaunchKernelGGL(item16<1>, dim3(grid), dim3(1024), lds, 0, out, n_items); });
    }
  }
  time("hipMemset", [&] { (void)hipMemsetAsync(out, 0, bytes, 0); });
  (void)hipFree(out);
  return 0;
}

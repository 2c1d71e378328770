// Store-ceiling probe at 256^2 vs 512^2: does the LDS16 eval kernel's store
// pattern (workgroup of 16 waves per (1024-pixel block, 16*g-slot chunk),
// wave w writes slot w of each 16-slot group: 4 planes x 4 KiB) run slower
// on a 512^2 grid than on a 256^2 one, with no loads or compute at all?
// out = 16 GiB of float32 viewed as [S][4 planes][P].
//   lin      : one-shot 256-thread workgroups, one float4 per thread, in
//              address order (the torch fill_ shape)
//   item g/m : the eval's items, g groups of 16 slots each, XCD map m
//              (0 contiguous pixel blocks per XCD, 1 interleaved), one-shot,
//              131584 B of LDS (one workgroup per CU, as the kernel)
//   hipcc --offload-arch=gfx950 -O3 tools/store_grid.hip -o tools/store_grid
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr long kBytes = 16L << 30;

__device__ __forceinline__ void st(float* p, v4f v) {
  __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
}

__global__ __launch_bounds__(256) void lin(float* out) {
  v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  st(out + (long)blockIdx.x * 1024 + threadIdx.x * 4, v);
}

// item = (pixel block, chunk); blockIdx -> XCD round robin as eval_block
__global__ __launch_bounds__(1024) void item16(float* out, long P, int n_pb,
                                               int groups, int xi) {
  extern __shared__ float pad[];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (threadIdx.x == 4095) pad[0] = 0.f;  // never: keeps the LDS allocation
  const long b = blockIdx.x;
  const int xcd = b & 7;
  const long within = b >> 3;
  const int per = n_pb / 8;
  const int wp = (int)(within % per);
  const long chunk = within / per;
  const int pb = xi ? wp * 8 + xcd : xcd * per + wp;
  v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  for (int g = 0; g < groups; ++g) {
    const long s = (chunk * groups + g) * 16 + w;
    for (int q = 0; q < 4; ++q)
      for (int c = 0; c < 4; ++c)
        st(out + (s * 4 + q) * P + pb * 1024 + c * 256 + l * 4, v);
  }
}

int main() {
  float* out;
  if (hipMalloc(&out, kBytes) != hipSuccess) return 1;
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
    printf("%-34s %7.1f GB/s  (%.3f ms)\n", name, kBytes / (best * 1e-3) / 1e9, best);
  };
  time("lin one-shot 4KiB", [&] {
    hipLaunchKernelGGL(lin, dim3(kBytes / 4096), dim3(256), 0, 0, out);
  });
  for (long P : {65536L, 262144L}) {
    const int n_pb = (int)(P / 1024);
    const long S = kBytes / (16 * P);
    for (int g : {1, 2, 4, 16})
      for (int xi : {0, 1}) {
        const long items = S / (16 * g) * n_pb;
        char name[96];
        snprintf(name, 96, "item16 P=%ld^2 g%d %s", (long)(P == 65536 ? 256 : 512), g,
                 xi ? "interleaved" : "contiguous");
        time(name, [&] {
          hipLaunchKernelGGL(item16, dim3(items), dim3(1024), 131584, 0, out, P, n_pb, g, xi);
        });
      }
  }
  (void)hipFree(out);
  return 0;
}

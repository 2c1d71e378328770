// Store-pattern probe: the eval kernel's output address pattern with no
// compute, versus longer contiguous runs, to see what each candidate mapping
// can reach.  out[S][4][P] float32, P = 256^2, S = 16384 -> 16 GiB.
//   A: current eval mapping -- wave = 64 px x 16 slots; one float4 store
//      instruction covers 4 slots x 256 B (per plane)
//   B: workgroup = 256 px x 16 slots, wave = 4 slots (LDS transpose);
//      one instruction covers 1 slot x 1 KiB
//   D: workgroup = 1024 px x 16 slots: 4 KiB contiguous per (slot, plane)
//   H: workgroup = 4 slots x all P pixels: each wave writes its slot's 1 MiB
//      (4 planes) front to back
//   W: workgroup = 16 slots x 4096 px stripe: 16 KiB per (slot, plane)
//   C: grid-stride fill (upper bound), grid 4096 / 16384 / 65536
//   E: each wave owns one contiguous chunk and streams through it
// Every pattern in a non-temporal and a plain-store flavour.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
// store flavour: 0 plain, 1 nontemporal (builtin), 2 sc1, 3 sc0 sc1, 4 nt sc1
// (2-4: inline-asm vector stores; sc1 drops the line from the XCD L2)
template <int NT>
__device__ __forceinline__ void st(float* p, v4f v) {
  if (NT == 1) __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
  else if (NT == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
  else if (NT == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
  else if (NT == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" :: "v"(p), "v"(v) : "memory");
  else *reinterpret_cast<v4f*>(p) = v;
}

constexpr long P = 65536;

template <int NT>
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
      for (int q = 0; q < 4; ++q) st<NT>(o + q * P, v);
    }
  }
}

// run = contiguous pixels per (slot, plane) owned by one workgroup
template <int NT, int RUN>
__global__ __launch_bounds__(256) void patRun(float* out, long S, long n_pb) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long b = blockIdx.x;
  const long per = n_pb >> 3, x = b & 7, i = b >> 3;
  const long pb = x * per + (i % per), sc = i / per;
  const long p0 = pb * RUN + l * 4;
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
        for (int h = 0; h < RUN / 256; ++h) st<NT>(o + q * P + h * 256, v);
    }
  }
}

template <int NT>
__global__ __launch_bounds__(256) void patH(float* out, long S) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long s = (long)blockIdx.x * 4 + w;
  if (s >= S) return;
  float* o = out + s * 4 * P;
  v4f v = {1.f, 2.f, 3.f, 4.f};
  for (long i = 0; i < 4 * P; i += 256) st<NT>(o + i + l * 4, v);
}

template <int NT>
__global__ __launch_bounds__(256) void patE(float* out, long n4, long per_wave) {
  const int l = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long base = wave * per_wave;
  for (long i = 0; i < per_wave; i += 64) {
    const long k = base + i + l;
    if (k < n4) {
      v4f v = {1.f, 2.f, 3.f, 4.f};
      st<NT>(out + 4 * k, v);
    }
  }
}

template <int NT>
__global__ __launch_bounds__(1024) void patC(float* out, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    v4f v = {1.f, 2.f, 3.f, 4.f};
    st<NT>(out + 4 * i, v);
  }
}

// L: each lane writes U consecutive float4 (16*U contiguous bytes per lane,
// one wave covers 1024*U bytes per U instructions), grid-stride over chunks
template <int NT, int U>
__global__ __launch_bounds__(256) void patL(float* out, long n4) {
  const long stride = (long)gridDim.x * blockDim.x * U;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n4; i += stride) {
    v4f v = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(out + 4 * (i + u), v);
  }
}

// P: persistent pixel-block workgroups -- NB workgroups each own P/NB
// consecutive pixels (RUN = P/NB) and sweep ALL slots in order, so the whole
// chip writes a compact, linearly advancing window (memset-like).
//   MODE 0: per slot, wave w writes plane w (RUN floats)
//   MODE 1: per 16-slot group, wave w writes slots 4w..4w+3, all planes
//   MODE 2: per 16-slot group, slot-major: for slot j, wave w writes plane w
template <int NT, int MODE, int RUN>
__global__ __launch_bounds__(256) void patP(float* out, long S) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long pix0 = (long)blockIdx.x * RUN;
  v4f v = {1.f, 2.f, 3.f, 4.f};
  if (MODE == 0) {
    for (long s = 0; s < S; ++s) {
      float* o = out + (s * 4 + w) * P + pix0;
#pragma unroll
      for (int h = 0; h < RUN / 256; ++h) st<NT>(o + h * 256 + 4 * l, v);
    }
  } else {
    for (long s0 = 0; s0 < S; s0 += 16) {
      if (MODE == 1) {
        for (int j = 0; j < 4; ++j) {
          const long s = s0 + 4 * w + j;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int h = 0; h < RUN / 256; ++h)
              st<NT>(out + (s * 4 + q) * P + pix0 + h * 256 + 4 * l, v);
        }
      } else {
        for (int j = 0; j < 16; ++j) {
          const long s = s0 + j;
#pragma unroll
          for (int h = 0; h < RUN / 256; ++h)
            st<NT>(out + (s * 4 + w) * P + pix0 + h * 256 + 4 * l, v);
        }
      }
    }
  }
}

// X: patC at 256 x 256 with the workgroup -> 4 KiB chunk map rotated by
// SHIFT chunks (SHIFT 0 = patC): tests whether a workgroup's XCD (dealt
// round-robin, g % 8) and the chunk's address matter for write bandwidth
template <int NT, int SHIFT>
__global__ __launch_bounds__(256) void patX(float* out, long n4) {
  const long per_iter = 256L * 256;
  const int g = (blockIdx.x + SHIFT) & 255;
  for (long it = 0; it * per_iter < n4; ++it) {
    const long i = it * per_iter + (long)g * 256 + threadIdx.x;
    v4f v = {1.f, 2.f, 3.f, 4.f};
    if (i < n4) st<NT>(out + 4 * i, v);
  }
}

template <int NT>
static void launch(int k, float* out, long S, size_t bytes) {
  const long n_pb = P / 256, n_sc = S / 256, n4 = (long)(bytes / 16);
  switch (k) {
    case 0: hipLaunchKernelGGL(patA<NT>, dim3(n_pb * n_sc), dim3(256), 0, 0, out, S, n_pb); break;
    case 1: hipLaunchKernelGGL((patRun<NT, 256>), dim3(n_pb * n_sc), dim3(256), 0, 0, out, S, n_pb); break;
    case 2: hipLaunchKernelGGL((patRun<NT, 1024>), dim3(n_pb / 4 * n_sc), dim3(256), 0, 0, out, S, n_pb / 4); break;
    case 3: hipLaunchKernelGGL((patRun<NT, 4096>), dim3(n_pb / 16 * n_sc), dim3(256), 0, 0, out, S, n_pb / 16); break;
    case 4: hipLaunchKernelGGL(patH<NT>, dim3(S / 4), dim3(256), 0, 0, out, S); break;
    case 5: hipLaunchKernelGGL(patC<NT>, dim3(4096), dim3(256), 0, 0, out, n4); break;
    case 6: hipLaunchKernelGGL(patC<NT>, dim3(16384), dim3(256), 0, 0, out, n4); break;
    case 7: hipLaunchKernelGGL(patC<NT>, dim3(65536), dim3(256), 0, 0, out, n4); break;
    case 8: {
      const long waves = 16384L * 4;
      hipLaunchKernelGGL(patE<NT>, dim3(16384), dim3(256), 0, 0, out, n4, (n4 + waves - 1) / waves);
      break;
    }
    case 9: {
      const long waves = 2048L * 4;
      hipLaunchKernelGGL(patE<NT>, dim3(2048), dim3(256), 0, 0, out, n4, (n4 + waves - 1) / waves);
      break;
    }
    case 15: hipLaunchKernelGGL(patC<NT>, dim3(256), dim3(256), 0, 0, out, n4); break;
    case 26: hipLaunchKernelGGL((patX<NT, 0>), dim3(256), dim3(256), 0, 0, out, n4); break;
    case 27: hipLaunchKernelGGL((patX<NT, 1>), dim3(256), dim3(256), 0, 0, out, n4); break;
    case 28: hipLaunchKernelGGL((patX<NT, 4>), dim3(256), dim3(256), 0, 0, out, n4); break;
    case 29: hipLaunchKernelGGL((patX<NT, 8>), dim3(256), dim3(256), 0, 0, out, n4); break;
    case 30: hipLaunchKernelGGL((patX<NT, 64>), dim3(256), dim3(256), 0, 0, out, n4); break;
    case 20: hipLaunchKernelGGL((patP<NT, 0, 256>), dim3(P / 256), dim3(256), 0, 0, out, S); break;
    case 21: hipLaunchKernelGGL((patP<NT, 1, 256>), dim3(P / 256), dim3(256), 0, 0, out, S); break;
    case 22: hipLaunchKernelGGL((patP<NT, 2, 256>), dim3(P / 256), dim3(256), 0, 0, out, S); break;
    case 23: hipLaunchKernelGGL((patP<NT, 0, 512>), dim3(P / 512), dim3(256), 0, 0, out, S); break;
    case 24: hipLaunchKernelGGL((patP<NT, 2, 512>), dim3(P / 512), dim3(256), 0, 0, out, S); break;
    case 25: hipLaunchKernelGGL((patP<NT, 0, 1024>), dim3(P / 1024), dim3(256), 0, 0, out, S); break;
    case 16: hipLaunchKernelGGL(patC<NT>, dim3(512), dim3(256), 0, 0, out, n4); break;
    case 17: hipLaunchKernelGGL(patC<NT>, dim3(1024), dim3(256), 0, 0, out, n4); break;
    case 18: hipLaunchKernelGGL(patC<NT>, dim3(256), dim3(512), 0, 0, out, n4); break;
    case 19: hipLaunchKernelGGL(patC<NT>, dim3(256), dim3(1024), 0, 0, out, n4); break;
    case 10: hipLaunchKernelGGL((patL<NT, 2>), dim3(8192), dim3(256), 0, 0, out, n4); break;
    case 11: hipLaunchKernelGGL((patL<NT, 4>), dim3(4096), dim3(256), 0, 0, out, n4); break;
    case 12: hipLaunchKernelGGL((patL<NT, 4>), dim3(16384), dim3(256), 0, 0, out, n4); break;
    case 13: hipLaunchKernelGGL((patL<NT, 8>), dim3(2048), dim3(256), 0, 0, out, n4); break;
    case 14: hipLaunchKernelGGL((patL<NT, 8>), dim3(8192), dim3(256), 0, 0, out, n4); break;
  }
}

int main() {
  const long S = 16384;
  const size_t bytes = (size_t)S * 4 * P * 4;
  float* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  const char* names[] = {"A  eval 4slot x 256B", "B  1 KiB runs (LDS transpose)",
                         "D  4 KiB runs", "W  16 KiB runs", "H  slot-sequential 1 MiB/wave",
                         "C  grid-stride 4096", "C  grid-stride 16384", "C  grid-stride 65536",
                         "E  wave chunks 16384 wg", "E  wave chunks 2048 wg",
                         "L  32 B/lane grid 8192", "L  64 B/lane grid 4096",
                         "L  64 B/lane grid 16384", "L  128 B/lane grid 2048",
                         "L  128 B/lane grid 8192",
                         "C  grid-stride 256 x 256", "C  grid-stride 512 x 256",
                         "C  grid-stride 1024 x 256", "C  grid-stride 256 x 512",
                         "C  grid-stride 256 x 1024",
                         "P  persistent 256 px, plane/wave", "P  persistent 256 px, 4 slots/wave",
                         "P  persistent 256 px, slot-major", "P  persistent 512 px, plane/wave",
                         "P  persistent 512 px, slot-major", "P  persistent 1024 px, plane/wave",
                         "X  256x256 chunk shift 0", "X  256x256 chunk shift 1",
                         "X  256x256 chunk shift 4", "X  256x256 chunk shift 8",
                         "X  256x256 chunk shift 64"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int nt = 0; nt <= 4; ++nt) {
    for (int k = 0; k < 31; ++k) {
      if (k != 2 && k != 15 && k < 26) continue;
      if (nt >= 1) continue;
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        switch (nt) {
          case 0: launch<0>(k, out, S, bytes); break;
          case 1: launch<1>(k, out, S, bytes); break;
          case 2: launch<2>(k, out, S, bytes); break;
          case 3: launch<3>(k, out, S, bytes); break;
          default: launch<4>(k, out, S, bytes); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      printf("nt=%d %-32s %.1f GB/s (%.3f ms)\n", nt, names[k], bytes / (best * 1e-3) / 1e9, best);
    }
  }
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipMemsetAsync(out, 0, bytes, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  printf("hipMemset %.1f GB/s (%.3f ms)\n", bytes / (best * 1e-3) / 1e9, best);
  return 0;
}

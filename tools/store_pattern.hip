// Store-pattern probe (round 5): which ORDER of the evaluation's output
// stores does HBM take fastest, with no loads and no compute at all?
//
// Round 5's energy variants (SF_EVAL_ENERGY_DIAG, profiles/round5_energy.json)
// showed the register-tile evaluations (config 5, gain) run as fast with the
// contraction and the epilogue removed as with them, at clocks from 2.0 to
// 2.4 GHz: their rate is set by the store stream, not by joules.  This probe
// writes a ring of S slots x 4 planes x P float32 (the eval's [slot][4][y][x]
// layout) in the eval kernels' work-item orders and a few others:
//
//   rows4  the register tile: a wave owns 64 pixels, a store instruction
//          covers 4 slot rows x 256 B (lane l -> slot row (l >> 4) + 4 r),
//          NW waves per workgroup, G 16-slot groups per work item
//   contig the LDS-staged kernels: a workgroup owns RUN pixels, a store
//          instruction covers 1 KiB of one (slot, plane) row
//   lin    one float4 per thread in address order (torch fill_)
//
// Work items map to the XCDs as eval_block (kl_eval_impl.h): contiguous
// pixel blocks per XCD (x0) or interleaved (x1), optionally B pixel bands.
//   hipcc --offload-arch=gfx950 -O3 tools/store_pattern.hip -o tools/store_pattern
//   tools/store_pattern [GiB [1]]   (1: the rhythm sweep -- s_sleep "compute"
//   between store bursts, a barrier per group, LDS-capped occupancy)
//   tools/store_pattern GiB 2 [R]   (2: long launches, R passes of the ring)
//   tools/store_pattern GiB 3 [R]   (3: FMA "compute" vs sleep between bursts)
//   tools/store_pattern GiB 4 [R]   (4, round 6: pitched rings -- the slot
//                                    and plane pitches set off their powers
//                                    of two by 4 KiB or 256 B)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st(float* p, v4f v) {
  __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
}

// eval_block of kl_eval_impl.h (bands: lb = log2 B)
__device__ __forceinline__ void item(long bb, long n_pb, long n_sc, int lb, int xi,
                                     long& pb, long& sc) {
  long band = 0;
  if (lb) {
    n_pb >>= lb;
    const long per_band = n_pb * n_sc;
    band = bb / per_band;
    bb -= band * per_band;
  }
  if ((n_pb & 7) == 0) {
    const long per = n_pb >> 3;
    const long x = bb & 7, i = bb >> 3;
    pb = xi ? (i % per) * 8 + x : x * per + (i % per);
    sc = i / per;
  } else {
    pb = bb % n_pb;
    sc = bb / n_pb;
  }
  pb += band * n_pb;
}

__global__ __launch_bounds__(256) void lin(float* out, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) st(out + 4 * i, v4f{1.f, 2.f, 3.f, (float)threadIdx.x});
}

// register tile: NW waves x 64 pixels per workgroup, G groups of 16 slots
template <int NW>
__global__ __launch_bounds__(64 * NW) void rows4(float* out, long P, long S, long n_pb,
                                                 long n_sc, int G, int lb, int xi,
                                                 long ring) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, lb, xi, pb, sc);
  if (sc >= n_sc) return;
  const long p0 = (pb * NW + w) * 64 + (l & 15) * 4;
  if (p0 >= P) return;
  const v4f v = {1.f, 2.f, 3.f, (float)l};
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + (l >> 4) + 4 * r;
      if (s < S) {
#pragma unroll
        for (int q = 0; q < 4; ++q) st(out + ((s0 % ring + (s - s0)) * 4 + q) * P + p0, v);
      }
    }
  }
}

// LDS-staged pattern: a workgroup of NW waves owns RUN pixels; wave w writes
// slots w * (16 / NW) + j of each group, 1 KiB per store instruction
template <int NW, int RUN, bool VAR = false>
__global__ __launch_bounds__(64 * NW) void contig(float* out, long P, long S, long n_pb,
                                                  long n_sc, int G, int lb, int xi,
                                                  long ring) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, lb, xi, pb, sc);
  if (sc >= n_sc) return;
  const long pix0 = pb * RUN;
  const v4f v = {1.f, 2.f, 3.f, (float)l};
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;
    for (int j = 0; j < 16 / NW; ++j) {
      const long s = s0 + w * (16 / NW) + j;
      if (s >= S) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < RUN / 256; ++c) {
          const long p = pix0 + c * 256 + 4 * l;
          if (p < P) {
            // VAR: values that differ per pixel, slot and plane (the eval's)
            const v4f u = VAR ? v4f{__builtin_sinf((float)(p + s)), __builtin_cosf((float)(p ^ s)),
                                    (float)(q - p), (float)(s * 3 + c)}
                              : v;
            st(out + ((s0 % ring + (s - s0)) * 4 + q) * P + p, u);
          }
        }
    }
  }
}

// the same two patterns with the eval's rhythm: `sl` s_sleep(1) ticks
// (~64 clocks each) of "compute" before each group's stores, a workgroup
// barrier per group (bar), and dynamic LDS to cap workgroups per CU
template <int NW, int RUN, bool VALU = false, int WAIT = 0>
__global__ __launch_bounds__(64 * NW) void contig_t(float* out, long P, long S, long n_pb,
                                                    long n_sc, int G, int xi, int sl, int bar,
                                                    long ring = 0) {
  extern __shared__ float pad[];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (sl < 0) pad[threadIdx.x] = 0.f;  // never: keeps the LDS allocation
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, 0, xi, pb, sc);
  if (sc >= n_sc) return;
  const long pix0 = pb * RUN;
  v4f v = {1.f, 2.f, 3.f, (float)l};
  if (ring == 0) ring = S;
  float x = (float)threadIdx.x;
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;  // uniform per workgroup
    if (VALU) {
      // sl dependent fp32 FMAs of "compute" (kept: folded into the value)
      for (int z = 0; z < sl; ++z) x = __builtin_fmaf(x, 0.999f, 0.5f);
      v[3] = x;
    } else {
      for (int z = 0; z < sl; ++z) __builtin_amdgcn_s_sleep(1);
    }
    if (bar) __syncthreads();
    for (int j = 0; j < 16 / NW; ++j) {
      const long s = s0 + w * (16 / NW) + j;
      if (s >= S) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < RUN / 256; ++c) {
          const long p = pix0 + c * 256 + 4 * l;
          if (p < P) st(out + ((s0 % ring + (s - s0)) * 4 + q) * P + p, v);
        }
    }
    // WAIT 1: every wave waits for its stores of the group to complete
    // before the next group (at most one burst in flight per wave)
    if (WAIT == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (WAIT == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
}

// fill order with "compute": each wave writes `per` consecutive 1 KiB
// float4 rows (a 16 KiB run at per = 16), `work` dependent FMAs before each
__global__ __launch_bounds__(256) void lin_w(float* out, long n4, int per, int work) {
  const long w = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  float x = (float)l;
  for (int k = 0; k < per; ++k) {
    for (int z = 0; z < work; ++z) x = __builtin_fmaf(x, 0.999f, 0.5f);
    const long i = (w * per + k) * 64 + l;
    if (i < n4) st(out + 4 * i, v4f{1.f, 2.f, 3.f, x});
  }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void rows4_t(float* out, long P, long S, long n_pb,
                                                   long n_sc, int G, int lb, int xi, int sl) {
  extern __shared__ float pad[];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (sl < 0) pad[threadIdx.x] = 0.f;
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, lb, xi, pb, sc);
  if (sc >= n_sc) return;
  const long p0 = (pb * NW + w) * 64 + (l & 15) * 4;
  if (p0 >= P) return;
  const v4f v = {1.f, 2.f, 3.f, (float)l};
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;
    for (int z = 0; z < sl; ++z) __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + (l >> 4) + 4 * r;
      if (s < S) {
#pragma unroll
        for (int q = 0; q < 4; ++q) st(out + (s * 4 + q) * P + p0, v);
      }
    }
  }
}

// round 6: the register-tile and LDS-staged orders on a PITCHED ring: plane
// q of ring slot r starts at r * sp + q * qp floats (the eval's layout has
// qp = P, sp = 4 P: every concurrent store stream of the register tile sits
// a power-of-two distance from the next -- 1 MiB at 256^2, 4 MiB at 512^2)
template <int NW>
__global__ __launch_bounds__(64 * NW) void rows4p(float* out, long P, long S, long n_pb,
                                                  long n_sc, int G, int lb, int xi,
                                                  long ring, long qp, long sp) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, lb, xi, pb, sc);
  if (sc >= n_sc) return;
  const long p0 = (pb * NW + w) * 64 + (l & 15) * 4;
  if (p0 >= P) return;
  const v4f v = {1.f, 2.f, 3.f, (float)l};
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long s = s0 + (l >> 4) + 4 * r;
      if (s < S) {
#pragma unroll
        for (int q = 0; q < 4; ++q) st(out + (s0 % ring + (s - s0)) * sp + q * qp + p0, v);
      }
    }
  }
}

template <int NW, int RUN>
__global__ __launch_bounds__(64 * NW) void contigp(float* out, long P, long S, long n_pb,
                                                   long n_sc, int G, int xi, long ring,
                                                   long qp, long sp) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  long pb, sc;
  item(blockIdx.x, n_pb, n_sc, 0, xi, pb, sc);
  if (sc >= n_sc) return;
  const long pix0 = pb * RUN;
  const v4f v = {1.f, 2.f, 3.f, (float)l};
  for (int g = 0; g < G; ++g) {
    const long s0 = (sc * G + g) * 16;
    if (s0 >= S) return;
    for (int j = 0; j < 16 / NW; ++j) {
      const long s = s0 + w * (16 / NW) + j;
      if (s >= S) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < RUN / 256; ++c) {
          const long p = pix0 + c * 256 + 4 * l;
          if (p < P) st(out + (s0 % ring + (s - s0)) * sp + q * qp + p, v);
        }
    }
  }
}

int main(int argc, char** argv) {
  const long gib = argc > 1 ? atol(argv[1]) : 16;
  const long bytes = gib << 30;
  float* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&contig_t<16, 1024>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 131584);
  auto time = [&](const char* name, long wrote, auto launch) {
    launch();
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      printf("%-44s launch failed\n", name);
      return;
    }
    float tot = 0.f, best = 1e30f;
    const int reps = 8;
    for (int r = 0; r < reps; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      tot += ms;
      if (ms < best) best = ms;
    }
    const double gbs = wrote / (tot / reps * 1e-3) / 1e9;
    printf("%-44s %7.1f GB/s  frac %.3f  (mean %.3f ms, best %.3f)\n", name, gbs,
           gbs / 8000.0, tot / reps, best);
    fflush(stdout);
  };
  const long n4 = bytes / 16;
  time("lin (fill_ order)", bytes, [&] {
    hipLaunchKernelGGL(lin, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, out, n4);
  });
  char name[128];
  const bool rhythm = argc > 2 && atoi(argv[2]) == 1;
  if (argc > 2 && atoi(argv[2]) == 3) {
    // round 5: does compute between store bursts (not sleep) speed the
    // store stream?  fill order with FMAs between stores; the LDS16 order
    // (256^2, 2 groups, interleaved map, one workgroup per CU by LDS, a
    // barrier per group) with FMAs vs s_sleep between groups, long launches
    const long n4 = bytes / 16;
    for (int work : {0, 8, 32}) {
      snprintf(name, sizeof name, "lin_w per16 work%-4d", work);
      time(name, bytes, [&] {
        hipLaunchKernelGGL(lin_w, dim3((unsigned)((n4 / 16 + 255) / 256 * 1)), dim3(256), 0, 0,
                           out, n4, 16, work);
      });
    }
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&contig_t<16, 1024, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 131584);
    const long R = argc > 3 ? atol(argv[3]) : 16;
    for (long N : {256L, 512L}) {
      const long P = N * N;
      const long ring = bytes / (16 * P);
      const long S = ring * R;
      const long wrote = S * 16 * P;
      const int G = N == 256 ? 2 : 4;
      const long n_sc = (S + 16 * G - 1) / (16 * G);
      const long n_pb = P / 1024;
      for (int work : {0, 64, 256}) {
        snprintf(name, sizeof name, "lds16-like %ld^2 g%d fma%-5d bar1", N, G, work);
        time(name, wrote, [&] {
          hipLaunchKernelGGL((contig_t<16, 1024, true>), dim3((unsigned)(n_pb * n_sc)),
                             dim3(1024), 131584, 0, out, P, S, n_pb, n_sc, G, 1, work, 1, ring);
        });
      }
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&contig_t<16, 1024, true, 1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 131584);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&contig_t<16, 1024, true, 2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 131584);
      for (int work : {0, 64, 256}) {
        snprintf(name, sizeof name, "lds16-like %ld^2 g%d fma%-5d bar1 wait0", N, G, work);
        time(name, wrote, [&] {
          hipLaunchKernelGGL((contig_t<16, 1024, true, 1>), dim3((unsigned)(n_pb * n_sc)),
                             dim3(1024), 131584, 0, out, P, S, n_pb, n_sc, G, 1, work, 1, ring);
        });
        snprintf(name, sizeof name, "lds16-like %ld^2 g%d fma%-5d bar1 wait8", N, G, work);
        time(name, wrote, [&] {
          hipLaunchKernelGGL((contig_t<16, 1024, true, 2>), dim3((unsigned)(n_pb * n_sc)),
                             dim3(1024), 131584, 0, out, P, S, n_pb, n_sc, G, 1, work, 1, ring);
        });
      }
      for (int sl : {0, 16, 64}) {
        snprintf(name, sizeof name, "lds16-like %ld^2 g%d sleep%-3d bar1", N, G, sl);
        time(name, wrote, [&] {
          hipLaunchKernelGGL((contig_t<16, 1024>), dim3((unsigned)(n_pb * n_sc)), dim3(1024),
                             131584, 0, out, P, S, n_pb, n_sc, G, 1, sl, 1, ring);
        });
      }
    }
    (void)hipFree(out);
    return 0;
  }
  if (argc > 2 && atoi(argv[2]) == 4) {
    // round 6: address interleave.  The register tile's
    // concurrent (slot, plane) streams sit power-of-two pitches apart; are
    // non-power-of-two pitches faster?  Long launches (R passes of the ring)
    const long R = argc > 3 ? atol(argv[3]) : 8;
    for (long N : {256L, 512L}) {
      const long P = N * N;
      // (plane pad, slot pad) in floats: 0, 256 B, 4 KiB
      const long pads[][2] = {{0, 0}, {0, 64}, {0, 1024}, {64, 0}, {1024, 0},
                              {64, 64}, {1024, 1024}, {0, 16384}};
      for (const auto& pd : pads) {
        const long qp = P + pd[0], sp = 4 * qp + pd[1];
        const long ring = (bytes / 4 / sp) / 16 * 16;
        const long S = ring * R;
        const long wrote = S * 16 * P;
        // the register tile as the evaluations run it: 256^2 gain (64
        // groups, contiguous map), 512^2 config 5 (4 groups, 8 bands,
        // interleaved map)
        const int G = N == 256 ? 64 : 4, lb = N == 256 ? 0 : 3, xi = N == 256 ? 0 : 1;
        const long n_pb = P / 256;
        const long n_sc = (S + 16 * G - 1) / (16 * G);
        snprintf(name, sizeof name, "pitch rows4  %ld^2 g%-2d +%ldB plane +%ldB slot", N, G,
                 pd[0] * 4, pd[1] * 4);
        time(name, wrote, [&] {
          hipLaunchKernelGGL(rows4p<4>, dim3((unsigned)(n_pb * n_sc)), dim3(256), 0, 0, out, P,
                             S, n_pb, n_sc, G, lb, xi, ring, qp, sp);
        });
        // the LDS16 order (config 4: 4 KiB runs, 2 groups, interleaved map)
        const int G2 = 2;
        const long n_pb2 = P / 1024, n_sc2 = (S + 16 * G2 - 1) / (16 * G2);
        snprintf(name, sizeof name, "pitch contig %ld^2 g%-2d +%ldB plane +%ldB slot", N, G2,
                 pd[0] * 4, pd[1] * 4);
        time(name, wrote, [&] {
          hipLaunchKernelGGL((contigp<16, 1024>), dim3((unsigned)(n_pb2 * n_sc2)), dim3(1024), 0,
                             0, out, P, S, n_pb2, n_sc2, G2, 1, ring, qp, sp);
        });
      }
    }
    (void)hipFree(out);
    return 0;
  }
  if (argc > 2 && atoi(argv[2]) == 2) {
    // long launches (round 5): the same orders over R passes of the ring in
    // ONE launch (slot s -> s mod ring, as the eval's ring), 40-80 ms per
    // launch instead of 2.5-3.5 ms, so the launch ramp is out of the number
    const long R = argc > 3 ? atol(argv[3]) : 16;
    for (long N : {256L, 512L}) {
      const long P = N * N;
      const long ring = bytes / (16 * P);  // a multiple of 16 slots
      const long S = ring * R;
      const long wrote = S * 16 * P;
      for (int G : {1, 2, 4, 16, 64}) {
        const long n_sc = (S + 16 * G - 1) / (16 * G);
        for (int xi : {0, 1})
          for (int lb : {0, 3}) {
            const long n_pb = P / 256;
            if (lb && (n_pb % (8 << lb))) continue;
            if (N == 256 && lb) continue;
            snprintf(name, sizeof name, "long rows4  %ld^2 nw4 g%-2d x%d b%d", N, G, xi, 1 << lb);
            time(name, wrote, [&] {
              hipLaunchKernelGGL(rows4<4>, dim3((unsigned)(n_pb * n_sc)), dim3(256), 0, 0, out,
                                 P, S, n_pb, n_sc, G, lb, xi, ring);
            });
          }
        if (G == 2 || G == 4)
          for (int xi : {0, 1}) {
            const long n_pb = P / 1024;
            snprintf(name, sizeof name, "long contig %ld^2 run4096 g%-2d x%d VAR", N, G, xi);
            time(name, wrote, [&] {
              hipLaunchKernelGGL((contig<16, 1024, true>), dim3((unsigned)(n_pb * n_sc)),
                                 dim3(1024), 0, 0, out, P, S, n_pb, n_sc, G, 0, xi, ring);
            });
          }
        for (int shape : {0, 2})
          for (int xi : {0, 1}) {
            const int run = 256 << shape;
            const long n_pb = P / run;
            snprintf(name, sizeof name, "long contig %ld^2 run%-4d g%-2d x%d", N, run * 4, G, xi);
            time(name, wrote, [&] {
              const unsigned nb = (unsigned)(n_pb * n_sc);
              if (shape == 0)
                hipLaunchKernelGGL((contig<4, 256>), dim3(nb), dim3(256), 0, 0, out, P, S, n_pb,
                                   n_sc, G, 0, xi, ring);
              else
                hipLaunchKernelGGL((contig<16, 1024>), dim3(nb), dim3(1024), 0, 0, out, P, S,
                                   n_pb, n_sc, G, 0, xi, ring);
            });
          }
      }
    }
    (void)hipFree(out);
    return 0;
  }
  if (rhythm) {
    // the eval's rhythm: compute between store bursts, occupancy caps
    for (long N : {256L, 512L}) {
      const long P = N * N;
      const long S = bytes / (16 * P);
      const long wrote = S * 16 * P;
      for (int G : {4, 64}) {
        const long n_sc = (S + 16 * G - 1) / (16 * G);
        for (int sl : {0, 4, 16, 48, 128})
          for (int bar : {0, 1}) {
            const long n_pb = P / 1024;
            snprintf(name, sizeof name, "lds16-like %ld^2 g%-2d sleep%-3d bar%d", N, G, sl, bar);
            time(name, wrote, [&] {
              hipLaunchKernelGGL((contig_t<16, 1024>), dim3((unsigned)(n_pb * n_sc)), dim3(1024),
                                 131584, 0, out, P, S, n_pb, n_sc, G, 0, sl, bar);
            });
          }
        // register tile at 2 workgroups (8 waves) per CU: ~64 KiB LDS each
        for (int sl : {0, 4, 16, 48, 128})
          for (int lds : {0, 65536}) {
            const long n_pb = P / 256;
            const int lb = N == 512 ? 3 : 0, xi = N == 512 ? 1 : 0;
            snprintf(name, sizeof name, "tile-like  %ld^2 g%-2d sleep%-3d lds%d", N, G, sl, lds);
            time(name, wrote, [&] {
              hipLaunchKernelGGL(rows4_t<4>, dim3((unsigned)(n_pb * n_sc)), dim3(256), lds, 0,
                                 out, P, S, n_pb, n_sc, G, lb, xi, sl);
            });
          }
      }
    }
    (void)hipFree(out);
    return 0;
  }
  for (long N : {256L, 512L}) {
    const long P = N * N;
    const long S = bytes / (16 * P);
    const long wrote = S * 16 * P;
    // the register tile (4 waves; the integer tile also 8) by groups / map / bands
    for (int nw : {4, 8}) {
      const long n_pb = P / (64 * nw);
      for (int G : {1, 4, 16, 64}) {
        const long n_sc = (S + 16 * G - 1) / (16 * G);
        for (int xi : {0, 1})
          for (int lb : {0, 3}) {
            if (lb && (n_pb % (8 << lb))) continue;
            if (N == 256 && lb) continue;
            snprintf(name, sizeof name, "rows4  %ld^2 nw%d g%-2d x%d b%d", N, nw, G, xi, 1 << lb);
            time(name, wrote, [&] {
              if (nw == 4)
                hipLaunchKernelGGL(rows4<4>, dim3((unsigned)(n_pb * n_sc)), dim3(256), 0, 0,
                                   out, P, S, n_pb, n_sc, G, lb, xi, S);
              else
                hipLaunchKernelGGL(rows4<8>, dim3((unsigned)(n_pb * n_sc)), dim3(512), 0, 0,
                                   out, P, S, n_pb, n_sc, G, lb, xi, S);
            });
          }
      }
    }
    // the LDS-staged shapes: 4 waves / 1 KiB, 8 / 2 KiB, 16 / 4 KiB runs
    for (int shape = 0; shape < 3; ++shape) {
      const int run = 256 << shape;
      const long n_pb = P / run;
      for (int G : {1, 4, 16, 64}) {
        const long n_sc = (S + 16 * G - 1) / (16 * G);
        for (int xi : {0, 1}) {
          snprintf(name, sizeof name, "contig %ld^2 run%-4d g%-2d x%d", N, run * 4, G, xi);
          time(name, wrote, [&] {
            const unsigned nb = (unsigned)(n_pb * n_sc);
            if (shape == 0)
              hipLaunchKernelGGL((contig<4, 256>), dim3(nb), dim3(256), 0, 0, out, P, S, n_pb,
                                 n_sc, G, 0, xi, S);
            else if (shape == 1)
              hipLaunchKernelGGL((contig<8, 512>), dim3(nb), dim3(512), 0, 0, out, P, S, n_pb,
                                 n_sc, G, 0, xi, S);
            else
              hipLaunchKernelGGL((contig<16, 1024>), dim3(nb), dim3(1024), 0, 0, out, P, S,
                                 n_pb, n_sc, G, 0, xi, S);
          });
        }
      }
    }
  }
  (void)hipFree(out);
  return 0;
}

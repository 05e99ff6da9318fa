// Microbenchmark of the halo kernel's per-tap inner loop on gfx950: W waves per block, one
// block per CU (LDS padded), per "tap" each wave reads MREP A + NREP B 16-byte fragments from
// LDS (A shifted per tap like the halo, B from a 3-slot ring like the weight slices) and runs
// MREP x NREP v_mfma_f32_16x16x32_bf16, optionally followed by a block barrier.  No global
// memory in the loop.  Prints the MFMA-pipe utilisation per variant.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_lds_bench tools/mfma_lds_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <type_traits>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// MODE 0: all reads, then the MFMAs (hipcc's waits; sched_group_barrier as the halo kernel)
// MODE 1: no LDS reads in the loop (fragments from registers): the MFMA + barrier floor
// MODE 2: all reads, then each column waits for its own B fragment (inline asm, counted)
template <int MREP, int NREP, int MODE, int BARP, int DMA, int NW = 8>
__global__ __launch_bounds__(NW * 64) void loop_kernel(int taps, float* out, const char* wsrc) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  constexpr int AR = NW * 128;  // halo rows: 1024 (8 waves, 64 KiB) / 512 (4 waves, 32 KiB)
  u32x4* A = lds;
  u32x4* B = lds + AR * 4;     // 3 slots x 256 rows x 4 chunks (48 KiB)
  for (int i = tid; i < AR * 4 + 3072; i += NW * 64) lds[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
  __syncthreads();
  f32x4 acc[MREP][NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 ra[MREP], rb[NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m) ra[m] = A[(wave * MREP * 16 + m * 16 + l16) * 4 + g];
#pragma unroll
  for (int n = 0; n < NREP; ++n) rb[n] = B[(n * 16 + l16) * 4 + g];
  // MODE 3: fragments of tap t+1 read (into the other register set) right after the barrier
  // that retired their weights, while tap t's MFMAs run on the set read one iteration earlier
  u32x4 xa[2][MREP], xb[2][NREP];
  auto rd = [&](int t, int set) {
    const int shift = (t % 5) + 68 * ((t / 5) % 5);
#pragma unroll
    for (int m = 0; m < MREP; ++m) {
      const int hp = (wave * MREP * 16 + m * 16 + l16 + shift) & (AR - 1);
      xa[set][m] = A[hp * 4 + (g ^ (((hp >> 2) & 1) << 1))];
    }
#pragma unroll
    for (int n = 0; n < NREP; ++n) {
      const int r = n * 16 + l16;
      xb[set][n] = B[(t % 3) * 1024 + r * 4 + (g ^ (((r >> 2) & 1) << 1))];
    }
  };
  constexpr bool ILV = MODE == 4;
  if constexpr (MODE == 3 || MODE == 4) {
    // two taps per iteration so that the register sets are compile-time indices
    rd(0, 0);
    auto step = [&](int t, auto CUR) {
      constexpr int cur = decltype(CUR)::value;
      if (t + 1 < taps) rd(t + 1, cur ^ 1);
#pragma unroll
      for (int n = 0; n < NREP; ++n)
#pragma unroll
        for (int m = 0; m < MREP; ++m) acc[m][n] = mma(xa[cur][m], xb[cur][n], acc[m][n]);
      if constexpr (ILV) {  // one next-tap read after each column's MFMAs
#pragma unroll
        for (int n = 0; n < NREP; ++n) {
          __builtin_amdgcn_sched_group_barrier(0x008, MREP, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, MREP, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x100, MREP + NREP, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MREP * NREP, 0);
      }
      if constexpr (DMA > 0) {
        char* dst = reinterpret_cast<char*>(B + ((t + 2) % 3) * 1024) + wave * DMA * 1024;
        const char* src = wsrc + ((t * 7) % 64) * 16384 + (wave * DMA * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < DMA; ++j)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j * 1024),
                                           (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, 0, 0);
      }
      if constexpr (DMA == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if constexpr (DMA == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if constexpr (DMA == 1) asm volatile("s_waitcnt vmcnt(1)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    for (int t = 0; t < taps; t += 2) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
    }
    taps = 0;  // (the generic loop below is skipped)
  }
  for (int t = 0; t < taps; ++t) {
    const int shift = (t % 5) + 68 * ((t / 5) % 5);  // 5x5 taps over a 68-wide halo
    const int slot = t % 3;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int n = 0; n < NREP; ++n)
#pragma unroll
        for (int m = 0; m < MREP; ++m) acc[m][n] = mma(ra[m], rb[n], acc[m][n]);
    } else if constexpr (MODE == 0) {
      u32x4 af[MREP], bf[NREP];
#pragma unroll
      for (int m = 0; m < MREP; ++m) {
        const int hp = (wave * MREP * 16 + m * 16 + l16 + shift) & (AR - 1);
        af[m] = A[hp * 4 + (g ^ (((hp >> 2) & 1) << 1))];
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        const int r = n * 16 + l16;
        bf[n] = B[slot * 1024 + r * 4 + (g ^ (((r >> 2) & 1) << 1))];
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n)
#pragma unroll
        for (int m = 0; m < MREP; ++m) acc[m][n] = mma(af[m], bf[n], acc[m][n]);
      __builtin_amdgcn_sched_group_barrier(0x100, MREP + NREP, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MREP * NREP, 0);
    } else {
      u32x4 af[MREP], bf[NREP];
#pragma unroll
      for (int m = 0; m < MREP; ++m) {
        const int hp = (wave * MREP * 16 + m * 16 + l16 + shift) & (AR - 1);
        const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)(A + hp * 4 + (g ^ (((hp >> 2) & 1) << 1)));
        asm volatile("ds_read_b128 %0, %1" : "=v"(af[m]) : "v"(a));
      }
      const unsigned b0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)(B + slot * 1024 + l16 * 4 + (g ^ (((l16 >> 2) & 1) << 1)));
#pragma unroll
      for (int n = 0; n < NREP; ++n) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bf[n]) : "v"(b0), "i"(n * 1024));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        switch (NREP - 1 - n) {
          case 0: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
          case 1: asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory"); break;
          case 2: asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory"); break;
          case 3: asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory"); break;
          case 4: asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); break;
          case 5: asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory"); break;
          case 6: asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory"); break;
          case 7: asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory"); break;
          case 8: asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory"); break;
          case 9: asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory"); break;
          case 10: asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory"); break;
          case 11: asm volatile("s_waitcnt lgkmcnt(11)" ::: "memory"); break;
          default: asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory"); break;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < MREP; ++m) acc[m][n] = mma(af[m], bf[n], acc[m][n]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (DMA > 0) {  // weight-slice pieces for a later tap (1 KiB per wave each), ring as the halo kernel
      char* dst = reinterpret_cast<char*>(B + ((t + 2) % 3) * 1024) + wave * DMA * 1024;
      const char* src = wsrc + ((t * 7) % 64) * 16384 + (wave * DMA * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < DMA; ++j)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j * 1024),
                                         (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, 0, 0);
    }
    if constexpr (BARP > 0) {
      if ((t % BARP) == BARP - 1) {
        if constexpr (DMA == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if constexpr (DMA == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else if constexpr (DMA == 1) asm volatile("s_waitcnt vmcnt(1)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) s += acc[m][n][0];
  out[blockIdx.x * 512 + tid] = s;  // (NW <= 8)
}

template <int MREP, int NREP, int MODE, int BARP, int DMA = 0, int NW = 8, int BPC = 1>
static int run(const char* name, float* out, int taps, hipEvent_t e0, hipEvent_t e1, const char* w) {
  auto k = loop_kernel<MREP, NREP, MODE, BARP, DMA, NW>;
  const int lds = (BPC == 1 ? 150 : 80) * 1024;  // one (or two: 2 x 80 KiB = the CU's 160) blocks per CU
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int blocks = 256 * 4 * BPC;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(NW * 64), lds, 0, taps, out, w);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(NW * 64), lds, 0, taps, out, w);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double flops = 2.0 * 16 * 16 * 32 * MREP * NREP * (double)NW * taps * blocks;
  printf("%-26s %dw x%d bar/%d dma %d MREP %d NREP %2d  %.3f ms  %.0f TF/s  %.1f %% of 2.5 PF\n", name, NW, BPC, BARP, DMA, MREP, NREP, ms, flops / ms / 1e9,
         flops / ms / 1e9 / 25.0);
  return 0;
}

int main() {
  float* out;
  CHECK(hipMalloc(&out, 256 * 4 * 2 * 512 * 4));  // (up to 2 blocks per CU x 512 threads)
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int taps = 2000;
  char* w;
  CHECK(hipMalloc(&w, 64 * 16384 + 65536));
  CHECK(hipMemset(w, 0, 64 * 16384 + 65536));
  // two 4-wave blocks per CU (each with its own barrier) against one 8-wave block
  run<2, 13, 0, 1, 2, 8, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 1, 4, 4, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 1, 0, 4, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 0, 0, 4, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 3, 1, 4, 4, 2>("prefetch next tap", out, taps, e0, e1, w);
  run<2, 13, 4, 1, 4, 4, 2>("prefetch interleaved", out, taps, e0, e1, w);
  run<2, 13, 1, 1, 0, 4, 2>("regs only", out, taps, e0, e1, w);
  run<2, 13, 1, 1>("regs only", out, taps, e0, e1, w);
  run<4, 7, 1, 1, 0, 4>("regs only", out, taps, e0, e1, w);
  run<4, 7, 0, 1, 0, 4>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 7, 0, 1, 4, 4>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 7, 4, 1, 4, 4>("prefetch interleaved", out, taps, e0, e1, w);
  run<4, 13, 0, 1, 4, 4>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 13, 4, 1, 4, 4>("prefetch interleaved", out, taps, e0, e1, w);
  run<2, 13, 4, 1, 2>("prefetch interleaved", out, taps, e0, e1, w);
  run<4, 7, 4, 1, 2>("prefetch interleaved", out, taps, e0, e1, w);
  run<4, 4, 4, 1, 1>("prefetch interleaved", out, taps, e0, e1, w);
  run<2, 13, 4, 1, 0>("prefetch interleaved", out, taps, e0, e1, w);
  run<2, 13, 3, 1, 2>("prefetch next tap", out, taps, e0, e1, w);
  run<4, 7, 3, 1, 2>("prefetch next tap", out, taps, e0, e1, w);
  run<4, 4, 3, 1, 1>("prefetch next tap", out, taps, e0, e1, w);
  run<2, 4, 3, 1, 1>("prefetch next tap", out, taps, e0, e1, w);
  run<2, 13, 0, 0>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 1, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 0, 2, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 13, 2, 1, 2>("lds counted waits", out, taps, e0, e1, w);
  run<4, 7, 0, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 7, 0, 1, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 7, 0, 2, 2>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 4, 0, 1, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  run<4, 4, 0, 2, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  run<2, 4, 0, 1, 1>("lds all-then-mfma", out, taps, e0, e1, w);
  CHECK(hipFree(w));
  CHECK(hipFree(out));
  return 0;
}

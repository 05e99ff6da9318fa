// Pointwise (1x1) convolution for gfx950: Y[p][n] = act(sum_c A[pix(p)][c] Wp[n][c] + bias[n]
// + res_scale * R[p][n]) over the output pixels p, i.e. a plain GEMM whose A rows are pixel rows
// of an NHWC tensor (stride 1 or 2: pix(p) = (n, oy * SH + dymin, ox * SW + dxmin)).
//
// Why not the halo kernel: with one tap, its pipeline step is one 32-channel k-step, and each
// step stages the NEXT k-step's input in registers and writes it to LDS in the same step -- the
// global-load latency is exposed every step (ResNet-50's 1x1 layers of the configs[2] identity
// extractor ran at 1-2.5 % of peak, 11-44 us for 0.3-2 GF; profiles/r04/r50_layers_splits.txt).
// Here both operands arrive by LDS-DMA into a 4-stage ring (three k-steps in flight), one
// counted vmcnt + barrier per k-step, 4 waves on 64/128 x 64/128 tiles (small M x N problems
// get enough blocks without splitting K), and the halo kernel's packed weight image and
// epilogue conventions (bias, residual, activation through LDS; or fp32 partial slices for a
// k split, finished by the split-K epilogue kernel).
//
// LDS rows are 64 bytes (one k-step of one pixel / one output channel); chunk g of row r sits
// at g ^ (((r >> 2) & 1) << 1), the halo kernel's conflict-free image -- the packed weights are
// stored pre-swizzled that way, so their DMA is a straight copy; the A rows are swizzled by
// choosing each lane's SOURCE chunk.
#include "tpg_internal.h"
#include <type_traits>

namespace tpg {

#ifndef PW_NST
#define PW_NST 4  // LDS ring stages (three k-steps in flight)
#endif

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ int pw_swz(int row) { return ((row >> 2) & 1) << 1; }
__device__ u32x4 pw_zero[4];  // the zero line of out-of-grid A rows (64 bytes)

__host__ __device__ constexpr int pw_stage_bytes(int bm, int bn) { return (bm + bn) * 64; }
// the ring (or the epilogue's parked rows, whichever is larger), then the tap table
__host__ __device__ constexpr int pw_lds_bytes(int bm, int bn) {
  return ((PW_NST * pw_stage_bytes(bm, bn) > bm * 16 + 512 * 4 + bm * (bn + 4) * 4)
              ? PW_NST * pw_stage_bytes(bm, bn)
              : bm * 16 + 512 * 4 + bm * (bn + 4) * 4) +
         TPG_MAX_TAPS * 4;
}

template <int N_>
__device__ __forceinline__ void pw_wait_vm() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

TPG_TL_DEFINE(pw)

template <int DT, int BM, int BN>
__global__ __launch_bounds__(256, 2) void pw_kernel(const HaloArgs p) {
  TPG_TL_MARK(0);
  using E = dt_t<DT>;
  static_assert(DT == 1 || DT == 2, "16-bit operands");
  constexpr int KS = 32;                        // channels per k-step (64 bytes)
  constexpr int WTM = BM / 2, WTN = BN / 2;     // 2 x 2 waves
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  constexpr int PA = BM / 64, PB = BN / 64;     // 1 KiB DMA pieces per wave per k-step (4 waves)
  constexpr int STAGE = pw_stage_bytes(BM, BN);
  constexpr int NST = PW_NST;

  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int M = p.N * p.JH * p.JW;
  const int nmt = (M + BM - 1) / BM, nnt = (p.Nout + BN - 1) / BN;
  // 1-D grid over (m-tile, n-tile, k split), m-tiles fastest; each XCD (physical block b on XCD
  // b % 8) gets a contiguous range, i.e. all m-tiles of a few (n-tile, split) pairs, so their
  // weight slices -- the larger operand of these small-map GEMMs (4.7 MB for 512 -> 512 3x3,
  // over one XCD's 4 MB L2) -- are fetched into that XCD's L2 once
  const int per = nmt * nnt, tot = per * (int)(gridDim.x / per);
  const int full = tot & ~7;
  const int b = blockIdx.x;
  const int L = (tot >= 16 && b < full) ? (b & 7) * (full >> 3) + (b >> 3) : b;
  const int mt = L % nmt, rest = L / nmt;
  const int nt = rest % nnt, z = rest / nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ks0 = z * p.kps;
  const int nks = min(p.nks, ks0 + p.kps) - ks0;

  // ---- A: this thread's DMA chunks (piece j of wave w covers 16-byte slots (j*4 + w)*64 + lane
  // of the A image, slot s = row * 4 + physical chunk; the source is the row's logical chunk
  // (s & 3) ^ swz(row)) of the row's pixel shifted by the step's tap; rows outside the grid and
  // taps outside the image read a zero line (LDS-DMA through inline asm, as the halo kernel's
  // weights: the builtin would make the compiler wait for every DMA in flight before each
  // fragment read)
  const int ntaps = p.ntaps, total = nks * ntaps;  // pipeline steps (k-step, tap), tap fastest
  int* s_tap = reinterpret_cast<int*>(lds + pw_lds_bytes(BM, BN) - TPG_MAX_TAPS * 4);
  if (tid < ntaps) {  // (dy - dymin) << 16 | (dx - dxmin) of each tap, from the halo shift table
    const int dyr = p.toff[tid] / p.HW;
    s_tap[tid] = (dyr << 16) | (p.toff[tid] - dyr * p.HW);
  }
  const char* abase[PA];
  int agy[PA], agx[PA];
  const int JHW = p.JH * p.JW;
  const char* Ab = reinterpret_cast<const char*>(p.A);
  const char* zline = reinterpret_cast<const char*>(pw_zero);
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int s = (j * 4 + wave) * 64 + lane;
    const int row = s >> 2, c = (s & 3) ^ pw_swz(row);
    const int q = m0 + row;
    abase[j] = nullptr;
    agy[j] = agx[j] = 0;
    if (q < M) {
      const int nimg = q / JHW, r = q - nimg * JHW;
      const int jy = r / p.JW, ix = r - jy * p.JW;
      agy[j] = jy * p.SH + p.dymin;
      agx[j] = ix * p.SW + p.dxmin;
      abase[j] = Ab + ((int64_t)nimg * p.a_sn + ks0 * KS + c * 8) * (int64_t)sizeof(E);
    }
  }
  // ---- B: the packed image [nks][ntiles][BNL][64 B] of the planner's BN (p.BN >= BN): this
  // tile's BN rows are contiguous
  const int BNLp = (p.BN + 127) / 128 * 128;
  const char* wsrc = reinterpret_cast<const char*>(p.Wp) +
                     (((int64_t)ks0 * ntaps * p.ntiles + n0 / p.BN) * BNLp + (n0 % p.BN)) * 64 + (wave * 1024 + lane * 16);
  const int64_t wstep = (int64_t)p.ntiles * BNLp * 64;
  // (M0 takes a wave-uniform LDS address: the wave index as a scalar)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds)) +
                        (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024;

  const int A_H = p.A_H, A_W = p.A_W, pad_mode = p.pad_mode;
  const int64_t ash = p.a_sh * (int64_t)sizeof(E), asw = p.a_sw * (int64_t)sizeof(E);
  auto issue = [&](int ks, int t, int st) {  // step (ks, t), clamped by the caller
    const uint32_t base = lds0 + (uint32_t)st * STAGE;
    const int tap = s_tap[t];
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      int y = agy[j] + (tap >> 16), x = agx[j] + (tap & 0xffff);
      if (pad_mode) {  // (reflect: the mirrored pixel)
        y = y < 0 ? -y : (y >= A_H ? 2 * A_H - 2 - y : y);
        x = x < 0 ? -x : (x >= A_W ? 2 * A_W - 2 - x : x);
      }
      const bool ok = abase[j] != nullptr && (unsigned)y < (unsigned)A_H && (unsigned)x < (unsigned)A_W;
      lds_dma16(ok ? abase[j] + y * ash + x * asw + ks * (KS * (int)sizeof(E)) : zline, base + j * 4096);
    }
    const char* src = wsrc + (int64_t)(ks * ntaps + t) * wstep;
#pragma unroll
    for (int j = 0; j < PB; ++j) lds_dma16(src + j * 4096, base + BM * 64 + j * 4096);
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int l16 = lane & 15, g = lane >> 4, g16 = g << 4;
  f32x4 acc[MREP][NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the bias of this block's columns, loaded now (its latency under the main loop)
  const float bias_pre = (tid < BN && p.bias && n0 + tid < p.Nout) ? p.bias[n0 + tid] : 0.f;
  __syncthreads();  // (tap table)
  TPG_TL_MARK(1);
  if (total > 0) {
    // issue cursor (iks, it): the step NST - 1 ahead of the one computed, held at the last step
    int iks = 0, it = 0;
    auto advance = [&]() {
      if (iks * ntaps + it + 1 < total) {
        if (++it == ntaps) { it = 0; ++iks; }
      }
    };
#pragma unroll
    for (int s = 0; s < NST - 1; ++s) {
      issue(iks, it, s);
      advance();
    }
    int st = 0;
    for (int ks = 0; ks < total; ++ks) {
      // step ks landed (the NST - 2 younger stages stay in flight); every wave is past step
      // ks - 1, whose stage the next issue overwrites
      pw_wait_vm<(NST - 2) * (PA + PB)>();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const int sti = st == 0 ? NST - 1 : st - 1;  // (ks + NST - 1) % NST
      issue(iks, it, sti);
      advance();
      const char* A = lds + st * STAGE;
      const u32x4* B = reinterpret_cast<const u32x4*>(A + BM * 64);
      u32x4 af[MREP], bf[NREP];
#pragma unroll
      for (int m = 0; m < MREP; ++m) {
        const int r = wm * WTM + m * 16 + l16;
        af[m] = *reinterpret_cast<const u32x4*>(A + (r << 6) + (g16 ^ ((r << 3) & 32)));
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        const int r = wn * WTN + n * 16 + l16;
        bf[n] = B[r * 4 + (g ^ pw_swz(r))];
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n)
#pragma unroll
        for (int m = 0; m < MREP; ++m) acc[m][n] = mfma16x16x32<DT>(af[m], bf[n], acc[m][n]);
      __builtin_amdgcn_sched_group_barrier(0x100, MREP + NREP, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MREP * NREP, 0);
      st = st == NST - 1 ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the clamped tail DMAs)
  }
  TPG_TL_MARK(2);

  // ---- epilogue through LDS (the halo kernel's): rows parked as fp32, then 8-channel groups
  constexpr int LDW = BN + 4, CG = BN / 8, NV = 8 * (int)sizeof(E) / 16;
  __syncthreads();
  int64_t* s_off = reinterpret_cast<int64_t*>(lds);              // [BM][2] out / residual offsets
  float* s_bias = reinterpret_cast<float*>(lds + BM * 16);       // [BN]
  float* s_acc = reinterpret_cast<float*>(lds + BM * 16 + 512 * 4);
  float* Wsk = p.ws ? p.ws + (int64_t)z * M * p.Nout : nullptr;
  for (int q = tid; q < BM; q += 256) {
    const int pix = m0 + q;
    int64_t yo = -1, ro = 0;
    if (pix < M) {
      if (Wsk) {
        yo = (int64_t)pix * p.Nout;
      } else {
        const int nimg = pix / JHW, r = pix - nimg * JHW;
        const int jy = r / p.JW, ix = r - jy * p.JW;
        const int oy = p.oy0 + p.osy * jy, ox = p.ox0 + p.osx * ix;
        yo = (int64_t)nimg * p.y_sn + (int64_t)oy * p.y_sh + (int64_t)ox * p.y_sw;
        ro = (int64_t)nimg * p.r_sn + (int64_t)oy * p.r_sh + (int64_t)ox * p.r_sw;
      }
    }
    s_off[2 * q] = yo;
    s_off[2 * q + 1] = ro;
  }
  if (tid < BN) s_bias[tid] = bias_pre;
  {
    float* base = s_acc + (wm * WTM + 4 * g) * LDW + wn * WTN + l16;
#pragma unroll
    for (int m = 0; m < MREP; ++m)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
#pragma unroll
        for (int n = 0; n < NREP; ++n) base[(m * 16 + reg) * LDW + n * 16] = acc[m][n][reg];
  }
  __syncthreads();
  E* Y = reinterpret_cast<E*>(p.Y);
  const E* R = reinterpret_cast<const E*>(p.R);
  const E* XA = reinterpret_cast<const E*>(p.XA);
  // groups it = tid + 256 k: the residual (or, without one, the producer's x) of every group is
  // loaded first -- one memory latency per thread instead of one per group
  constexpr int IT = BM * CG / 256;
  static_assert(IT * 256 == BM * CG, "whole groups per thread");
  const bool pf_r = R != nullptr;
  const E* PSRC = pf_r ? R : XA;
  const bool pvec = pf_r ? p.rvec : p.yvec;
  u32x4 pv[IT][NV];
  if (!Wsk && PSRC) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int it = tid + 256 * k;
      const int row = it / CG, c0 = (it - row * CG) * 8;
      const int64_t yo = s_off[2 * row];
      const bool ok = pvec && p.Nout - (n0 + c0) >= 8 && yo >= 0;
      const u32x4* src = reinterpret_cast<const u32x4*>(PSRC + (ok ? (pf_r ? s_off[2 * row + 1] : yo) + n0 + c0 : 0));
#pragma unroll
      for (int q = 0; q < NV; ++q) pv[k][q] = src[q];
    }
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int it = tid + 256 * k;
    const int row = it / CG, c0 = (it - row * CG) * 8;
    const int64_t yo = s_off[2 * row];
    const int col0 = n0 + c0;
    const int ncol = min(8, p.Nout - col0);
    if (yo < 0 || ncol <= 0) continue;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0 + 4);
    float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    if (Wsk) {  // fp32 partial slice row
      float* dst = Wsk + yo + col0;
      if (ncol == 8 && p.wvec) {
        *reinterpret_cast<f32x4*>(dst) = a0;
        *reinterpret_cast<f32x4*>(dst + 4) = a1;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < ncol) dst[e] = v[e];
      }
      continue;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += s_bias[c0 + e];
    const bool full = ncol == 8;
    if (R) {
      union { u32x4 u[NV]; E e[8]; } rr;
#pragma unroll
      for (int q = 0; q < NV; ++q) rr.u[q] = pv[k][q];
      if (!(full && p.rvec)) {
        const E* rs = R + s_off[2 * row + 1] + col0;
#pragma unroll
        for (int e = 0; e < 8; ++e) rr.e[e] = e < ncol ? rs[e] : (E)0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.res_scale * (float)rr.e[e];
    }
    union { u32x4 u[NV]; E e[8]; } o;
    if (XA) {  // desc.in_act: v * xa_act'(x), x at the output's offsets
      union { u32x4 u[NV]; E e[8]; } xx;
#pragma unroll
      for (int q = 0; q < NV; ++q) xx.u[q] = pv[k][q];
      if (pf_r && full && p.yvec) {  // (residual prefetched: x loaded here)
        const u32x4* xs = reinterpret_cast<const u32x4*>(XA + yo + col0);
#pragma unroll
        for (int q = 0; q < NV; ++q) xx.u[q] = xs[q];
      } else if (!(full && p.yvec)) {
        const E* xs = XA + yo + col0;
#pragma unroll
        for (int e = 0; e < 8; ++e) xx.e[e] = e < ncol ? xs[e] : (E)0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o.e[e] = (E)tpg_xa_grad(v[e], (float)xx.e[e], p.xa_act, p.xa_slope);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o.e[e] = (E)tpg_act(v[e], p.act, p.slope);
    }
    E* dst = Y + yo + col0;
    if (full && p.yvec) {
#pragma unroll
      for (int q = 0; q < NV; ++q) reinterpret_cast<u32x4*>(dst)[q] = o.u[q];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < ncol) dst[e] = o.e[e];
    }
  }
#ifdef TPG_BLOCK_TIMING
  __syncthreads();
  TPG_TL_MARK(3);
#endif
}

// tile configs {bm, bn}: pw_cfg = 1 + index
static constexpr int PW_BM[4] = {128, 128, 64, 64};
static constexpr int PW_BN[4] = {128, 64, 128, 64};

int pw_tile_bm(int cfg) { return cfg >= 1 && cfg <= 4 ? PW_BM[cfg - 1] : 0; }
int pw_tile_bn(int cfg) { return cfg >= 1 && cfg <= 4 ? PW_BN[cfg - 1] : 0; }

template <int DT, int BM, int BN>
static int launch_pw_t(const HaloArgs& a, hipStream_t s) {
  auto k = pw_kernel<DT, BM, BN>;
  constexpr int lds = pw_lds_bytes(BM, BN);
  static bool once = ((void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds), true);
  (void)once;
  const int M = a.N * a.JH * a.JW;
  const int64_t blocks = (int64_t)((M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN) * a.ksplit;
  if (blocks <= 0 || blocks >= (1ll << 31)) return -1;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}

int launch_pw(const HaloArgs& a, int dtype, hipStream_t s) {
  // the kernel's assumptions (the planner only picks it when they hold): whole
  // 32-channel k-steps, a planner tile at least as wide as this one, 32-bit byte offsets
  if (a.ntaps < 1 || a.ntaps > TPG_MAX_TAPS || a.dil > 1 || a.C % 32 || (dtype != 1 && dtype != 2) || a.pw < 1 ||
      a.pw > 4 || a.HW < 1 || a.HW >= (1 << 16))
    return -1;
  const int bm = PW_BM[a.pw - 1], bn = PW_BN[a.pw - 1];
  if (a.BN < bn || a.BN % bn) return -1;
  const int64_t ext = ((int64_t)(a.N - 1) * a.a_sn + (int64_t)(a.A_H - 1) * a.a_sh + (int64_t)(a.A_W - 1) * a.a_sw + a.C) * 2;
  if (ext >= 0x7FFFFFF0ll || a.a_sn < 0 || a.a_sh < 0 || a.a_sw < 0) return -1;
#define PW_L(BM_, BN_)                                                                          \
  if (bm == BM_ && bn == BN_) return dtype == 1 ? launch_pw_t<1, BM_, BN_>(a, s) : launch_pw_t<2, BM_, BN_>(a, s);
  PW_L(128, 128) PW_L(128, 64) PW_L(64, 128) PW_L(64, 64)
#undef PW_L
  return -1;
}

}  // namespace tpg

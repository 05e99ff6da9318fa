// Halo-tiled direct convolution for gfx950 — the stride-1 / sub-pixel hot path.
//
// Covers every conv whose taps read the A grid with unit stride: Conv2d forward at
// stride 1 (all 3x3 / 5x5 / 7x7 / 2x2-reflect layers of G and D), the Conv2d input
// gradient at any stride and the ConvTranspose2d forward (one launch per parity class,
// SURVEY.md §7 step 5) — and, with SH = SW = 2 (output pixel (y, x) reads halo position
// (2y, 2x) + tap), the stride-2 Conv2d forward and the ConvTranspose2d input gradient.
//
// Block = 256 output (sub-grid) pixels x BN output channels, 8 waves: one TH x TW tile of
// one image, or IMG whole small images (8x8, 10x10, 5x5 ... maps) side by side.  K loop: for each 64-byte channel step (bf16: 32 ch, f32: 16 ch)
//   - the input halo (TH + dy range) x (TW + dx range) pixels x 64 B is gathered ONCE
//     into LDS (zero / reflected outside the image) and reused by all taps;
//   - for each tap the [BN][64 B] weight slice (packed contiguous, pre-swizzled) is staged
//     through a second LDS double buffer, and every wave runs MREP x NREP MFMAs with A
//     fragments read from the halo at the tap's (dy, dx) shift.
// Next step's halo is prefetched into registers and the weights two taps ahead are in
// flight by LDS-DMA while the current tap computes (software pipeline, one barrier per tap).
// Small maps have too few tiles to fill 256 CUs: the k-steps are then split over grid.z and
// each split writes an fp32 partial slice, summed by the epilogue kernel (no atomics).
//
// LDS images use 64-byte pixel rows; the 16-byte chunk g of row p is stored at
// g ^ (((p >> 2) & 1) << 1), which makes the ds_read_b128 fragment reads of both
// operands bank-conflict free for any shift (checked exhaustively over the gfx950
// ds_read_b128 lane groups).
#include "tpg_internal.h"
#include <type_traits>
#include <algorithm>
#include <stdlib.h>
#include <string.h>

// timing ablations (tools only; never in the product build): bit 1 no weight LDS-DMA, 2 no tap
// barrier, 4 no MFMA, 8 no fragment reads, 16 no halo loads / stores
#ifndef TPG_HALO_ABL
#define TPG_HALO_ABL 0
#endif
#if (TPG_HALO_ABL & 2) != 0
#define HALO_BAR ""
#else
#define HALO_BAR "\n\ts_barrier"
#endif

namespace tpg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ int hswz(int row) { return ((row >> 2) & 1) << 1; }

__host__ __device__ constexpr int halo_bnl(int bn) { return (bn + 127) / 128 * 128; }
// epilogue: rows of the tile parked in LDS per pass (fp32, stride BN + 4): 64 on the
// 192..224-wide tiles, whose waves of the later passes still hold all their accumulators while
// a pass is finished (128 rows put the 224 tile with a producer-x epilogue past 256 VGPRs:
// scratch spills, round 5); 256 (two passes) on the 512-row tiles
__host__ __device__ constexpr int halo_epi_rows(int bn, int bm = 256) {
  return bm == 512 ? 256 : bn >= 192 ? 64 : bn >= 80 ? 128 : 256;
}
// (Column-half passes for the 208-wide tile were built in round 5 and removed in round 6: 1.5 %
// faster per launch, but every 416-byte pixel row was written and its residual read in two
// passes: HBM traffic 895 -> 990 MB per enhance_128 launch, gpurun r05ao PMC.)
__host__ __device__ constexpr int halo_epi_acc_bytes(int bn, int bm = 256) {
  return halo_epi_rows(bn, bm) * (bn + 4) * 4;
}
// (row-offset table [BM][2] int64 + bias [256] floats, then the parked accumulators)
__host__ __device__ constexpr int halo_epi_lds(int bn, int bm = 256) { return bm * 16 + 1024 + halo_epi_acc_bytes(bn, bm); }
// 256-row tiles (all small-map and grouped launches): the row-offset table and the bias live in
// their own LDS region past both the main loop's buffers (`main` bytes) and the parked rows, so
// the prologue fills them while its first loads are in flight and the epilogue's residual loads
// can issue before the accumulators are parked
__host__ __device__ constexpr int halo_epi_early_off(int main, int bn) {
  return ((main > halo_epi_acc_bytes(bn) ? main : halo_epi_acc_bytes(bn)) + 15) / 16 * 16;
}

// mask_chunk on a native 4 x u32 vector (first-class value: stays in VGPRs)
template <int EPC>
__device__ __forceinline__ u32x4 mask_chunk4(u32x4 v, int c0, int C) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if constexpr (EPC == 8) {
      const int e = c0 + 2 * d;
      v[d] &= (e + 1 < C) ? 0xFFFFFFFFu : ((e < C) ? 0x0000FFFFu : 0u);
    } else {
      v[d] = (c0 + d < C) ? v[d] : 0u;
    }
  }
  return v;
}

__device__ __forceinline__ float h_act(float v, int act, float slope) { return tpg_act(v, act, slope); }

__device__ __forceinline__ int h_refl(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// g = gy * act'(y) on one 16-byte chunk of each (the masked input-gradient mode)
template <typename E>
__device__ __forceinline__ u32x4 act_mask_chunk(u32x4 g, u32x4 y, int act, float slope) {
  constexpr int N = 16 / sizeof(E);
  union { u32x4 u; E e[N]; } a, b;
  a.u = g;
  b.u = y;
#pragma unroll
  for (int e = 0; e < N; ++e) a.e[e] = (E)tpg_act_grad((float)a.e[e], (float)b.e[e], act, slope);
  return a.u;
}

// (A/B builds: -DTPG_HALO_ROWMAJOR=1 restores the row-major dispatch order of the tiles)
#ifndef TPG_HALO_ROWMAJOR
#define TPG_HALO_ROWMAJOR 0
#endif


TPG_TL_DEFINE(halo)

// workgroup barrier for LDS hand-offs only (no vmcnt drain: vector loads stay in flight)
#define EPI_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

template <int DT, int HL, int BN, int WM, int WN, bool MASK, int BM = 256, int NG = 1>
__global__ __launch_bounds__(512) void halo_kernel(const Grouped<HaloArgs, NG> GA) {
  TPG_TL_MARK(0);
  // block -> (member, x = sub-tile group, y = N-tile, z = k split); a grouped grid is 1-D in
  // the plain grid's dispatch order (x fastest) within each member
  // Small maps (several images per block, or a k split): the dispatch-order block index b runs
  // on XCD b % 8; XCDs are handed contiguous ranges of the logical (x fastest) order, so each
  // XCD runs every sub-tile of a few (N-tile, k split) pairs -- or of one grouped member -- and
  // fetches their weight slices into its own L2 once (a 512-channel 3x3 layer's packed image is
  // 4.7 MB, over one XCD's 4 MB L2, when every XCD streams all of it)
  auto xcd_order = [](int b, int tot) {
    const int full = tot & ~7;
    return (tot >= 16 && b < full) ? (b & 7) * (full >> 3) + (b >> 3) : b;
  };
  int mem = 0, bx, by, bz;
  if constexpr (NG == 1) {
    bx = blockIdx.x; by = blockIdx.y; bz = blockIdx.z;
    const HaloArgs& q = GA.a[0];
    if (!TPG_HALO_ROWMAJOR && !(q.IMG == 1 && gridDim.x >= 64 && (int)gridDim.x == q.N * q.tiles_h * q.tiles_w)) {
      const int gx = gridDim.x, gy = gridDim.y;
      const int L = xcd_order(bx + gx * (by + gy * bz), gx * gy * (int)gridDim.z);
      bx = L % gx;
      const int yz = L / gx;
      by = yz % gy;
      bz = yz / gy;
    }
  } else {
    const int L = TPG_HALO_ROWMAJOR ? (int)blockIdx.x : xcd_order(blockIdx.x, gridDim.x);
    mem = group_member(GA, L);
    const HaloArgs& q = GA.a[mem];
    const int l = L - GA.boff[mem];
    const int gx = (q.N * q.tiles_h * q.tiles_w + q.IMG - 1) / q.IMG;
    const int yz = l / gx;
    bx = l - yz * gx;
    bz = yz / q.ntiles;
    by = yz - bz * q.ntiles;
  }
  const HaloArgs& p = GA.a[mem];
  if constexpr (NG == 1 && !TPG_HALO_ROWMAJOR) {
    // XCD-aware sub-tile order (one image tile per block, >= 64 blocks): physical block b runs on
    // XCD b % 8, so each XCD gets a contiguous range of logical tiles, and logical tiles walk DOWN
    // the tile columns of an image -- vertically adjacent tiles, which share k - 1 rows of their
    // input halo (a third of an 8 x 32 tile's 12 x 36 halo at k = 5), then run together on one
    // XCD and meet in its L2 instead of being re-read from HBM by another XCD
    const int nbx = gridDim.x;
    if (p.IMG == 1 && nbx >= 64 && nbx == p.N * p.tiles_h * p.tiles_w) {
      const int full = nbx & ~7;
      const int L = bx < full ? (bx & 7) * (full >> 3) + (bx >> 3) : bx;
      const int tiles = p.tiles_h * p.tiles_w;
      const int img = L / tiles, r = L - img * tiles;
      const int tx = r / p.tiles_h, ty = r - tx * p.tiles_h;
      bx = img * tiles + ty * p.tiles_w + tx;
    }
  }
  using E = dt_t<DT>;
  constexpr bool BF = DT != 0;  // 16-bit operands (bf16 or fp16)
  constexpr int EPC = 16 / sizeof(E);       // elements per 16-byte chunk
  constexpr int KS = 4 * EPC;                // channels per 64-byte step
  // BM output rows per block (IMG sub-tiles): 256, or 512 for the thin (<= 80-channel) layers
  // of the large maps, which then run 2x the MFMAs per tap barrier
  constexpr int BNL = halo_bnl(BN);          // weight rows per LDS slot (multiple of 128)
  constexpr int GL = BNL / 128;              // 1 KiB LDS-DMA pieces per wave per step
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  static_assert(WM * WN == 8, "8 waves");
  static_assert(MREP * 16 * WM == BM && NREP * 16 * WN == BN, "tile");

  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int hcap = p.hcap;
  constexpr int RS = 3;                                // weight ring slots (one tap slice each)
  u32x4* halo = lds;                                   // [2][hcap][4]
  u32x4* wts = lds + 2 * hcap * 4;                     // [RS][BNL][4] ring
  int* s_toff = reinterpret_cast<int*>(wts + RS * BNL * 4);  // [TPG_MAX_TAPS]
  constexpr bool EARLY = BM == 256;  // (see halo_epi_early_off)
  const int e_base = halo_epi_early_off((2 * p.hcap * 4 + RS * BNL * 4) * 16 + TPG_MAX_TAPS * 4, BN);
  int64_t* s_off = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(lds) + (EARLY ? e_base : 0));  // [BM][2]
  float* s_bias = reinterpret_cast<float*>(s_off + 2 * BM);                                          // [256]

  const int tid = threadIdx.x;
  if (tid < TPG_MAX_TAPS) s_toff[tid] = p.toff[tid];
  const int TH = p.TH, TW = p.TW, IMG = p.IMG, SH = p.SH, SW = p.SW;
  const int THW = TH * TW;
  const int HW = p.HW, HP = p.HH * HW;                 // halo pixels of one sub-tile
  const int tiles = p.tiles_h * p.tiles_w, tiles_w = p.tiles_w;
  const int ntot = p.N * tiles;                        // sub-tiles in the grid
  const int st0 = bx * IMG;
  const int n0 = by * BN;
  const int z = bz;
  const int ks0 = z * p.kps;
  const int nks = min(p.nks, ks0 + p.kps) - ks0;
  const E* Ag = reinterpret_cast<const E*>(p.A);
  const int wave = tid >> 6, lane = tid & 63;
  // packed weights: Wp[step][ntile][BNL][4 chunks]; this wave streams GL KiB of each slice
  const int64_t wstep = (int64_t)p.ntiles * BNL * 64;
  const char* wsrc = reinterpret_cast<const char*>(p.Wp) + (int64_t)ks0 * p.ntaps * wstep +
                     (int64_t)by * BNL * 64 + (wave * GL * 1024 + lane * 16);

  // LDS-DMA of one step's weight slice into ring slot `slot` (GL pieces per wave)
  // (the ring's LDS address and the step offset as 32-bit scalars: the generic-pointer form
  // cost a 64-bit multiply, an address-space null check and two readfirstlanes per step)
  const uint32_t wts_lds = __builtin_amdgcn_readfirstlane(lds_addr(wts)) +
                           (uint32_t)__builtin_amdgcn_readfirstlane(wave) * (GL * 1024);
  const uint32_t wstep32 = (uint32_t)wstep;  // (packed image < 2^31 bytes: planner)
  auto issue_w = [&](int step, int slot) {
    if constexpr ((TPG_HALO_ABL & 1) != 0) return;
    const char* src = wsrc + (uint32_t)step * wstep32;
    const uint32_t d0 = wts_lds + (uint32_t)slot * (BNL * 64);
#pragma unroll
    for (int j = 0; j < GL; ++j) lds_dma16(src + j * 1024, d0 + j * 1024);
  };

  // pipeline steps: ntaps per k-step; with p.half the problem's last k-step (when this block's
  // k range ends there) is paired, ceil(ntaps / 2) steps (see compute)
  const int ntaps = p.ntaps;
  const bool lastp = BF && p.half && ks0 + nks == p.nks && nks > 0;
  const int npair_b = lastp ? (ntaps + 1) >> 1 : 0;
  const int steps_full = (lastp ? nks - 1 : nks) * ntaps;
  // the first two steps' weight DMAs go out before the halo index math (they need none of
  // it), so their latency runs under it
  const int total = steps_full + npair_b;
  if (total > 0) {
    issue_w(0, 0);
    issue_w(min(1, total - 1), 1);
  }

  // ---- per-thread halo slots (fixed across k-steps): element offset from A (absolute,
  // < 2^31 by the planner), negative = outside the image or a dead sub-tile -> zero
  int hoff[HL];
  // mask mode: M / G pixel offset of each slot's pixel (-1 = none) and the slots whose pixel is
  // one of this block's own output pixels (bit q; only the blockIdx.y == 0 blocks store g)
  int mpix[MASK ? HL : 1];
  uint32_t core = 0;
#pragma unroll
  for (int q = 0; q < HL; ++q) {
    const int idx = tid + 512 * q;
    const int hp = idx >> 2, ch = idx & 3;
    hoff[q] = -1;
    if constexpr (MASK) mpix[q] = -1;
    if (hp < IMG * HP) {
      const int sub = (int)p.fd_hp.div(hp), hl = hp - sub * HP;
      const int st = st0 + sub;
      if (st < ntot) {
        const int nimg = (int)p.fd_tiles.div(st), trem = st - nimg * tiles;
        const int ty = (int)p.fd_tilesw.div(trem), tx = trem - ty * tiles_w;
        const int hy = (int)p.fd_hw.div(hl), hx = hl - hy * HW;
        int gy = ty * TH * SH + p.dymin + hy, gx = tx * TW * SW + p.dxmin + hx;
        if (p.pad_mode) { gy = h_refl(gy, p.A_H); gx = h_refl(gx, p.A_W); }
        bool real = true;
        if (p.dil > 1) {  // zero-inserted grid: only multiples of dil are pixels of A
          real = gy >= 0 && gx >= 0 && gy % p.dil == 0 && gx % p.dil == 0;
          gy /= p.dil;
          gx /= p.dil;
        }
        if (real && (unsigned)gy < (unsigned)p.A_H && (unsigned)gx < (unsigned)p.A_W) {
          hoff[q] = (int)((int64_t)nimg * p.a_sn + gy * p.a_sh + gx * p.a_sw) + ch * EPC;
          if constexpr (MASK) {
            mpix[q] = (int)((int64_t)nimg * p.m_sn + gy * p.m_sh + gx * p.m_sw);
            const int cy = gy - ty * TH, cx = gx - tx * TW;  // (SH = SW = 1 in this mode)
            if (by == 0 && (unsigned)cy < (unsigned)TH && (unsigned)cx < (unsigned)TW) core |= 1u << q;
          }
        }
      }
    }
  }
  const int HPT = IMG * HP;

  // Halo chunks are loaded raw (clamped address, unconditional 16-byte load) and masked
  // only when written to LDS a whole k-step later.  (vec-only kernel: the planner sends
  // unaligned tensors to the generic kernel.)
  u32x4 hreg[HL];
  int hc = 0;
  auto load_halo = [&](int ks) {
    if constexpr ((TPG_HALO_ABL & 16) != 0) return;
    const int cbase = (ks0 + ks) * KS;
    hc = cbase + (tid & 3) * EPC;
#pragma unroll
    for (int q = 0; q < HL; ++q) {
      const bool ok = hoff[q] >= 0 && hc < p.C;
      hreg[q] = *reinterpret_cast<const u32x4*>(Ag + (ok ? hoff[q] + cbase : 0));
    }
  };
  int gch = 0;  // mask mode: channel of this thread's chunks in the last stored halo
  auto store_halo = [&](int buf) {
    if constexpr ((TPG_HALO_ABL & 16) != 0) return;
    u32x4* H = halo + buf * hcap * 4;
#pragma unroll
    for (int q = 0; q < HL; ++q) {
      const int idx = tid + 512 * q;
      const int hp = idx >> 2;
      const int pos = hp * 4 + ((idx & 3) ^ hswz(hp));
      u32x4 v = hreg[q];
      if constexpr (MASK) {
        if (hp < HPT) v = act_mask_chunk<E>(v, H[pos], p.mact, p.mslope);  // y chunk, DMA'd in place
      }
      v = mask_chunk4<EPC>(v, hc, p.C);
      if (hoff[q] < 0) v = u32x4{0u, 0u, 0u, 0u};
      if (hp < HPT) H[pos] = v;
      if constexpr (MASK) hreg[q] = v;
    }
    if constexpr (MASK) gch = hc;
  };
  // mask mode: LDS-DMA of y's chunks of k-step ks into halo buffer buf, at the positions the
  // halo chunks will take (lane-linear DMA: the lane landing at position idx fetches pixel
  // idx >> 2, logical chunk (idx & 3) ^ hswz(pixel)); store_halo reads them back, masks and
  // overwrites them.  Invalid pixels fetch element 0 (their g is zeroed anyway).
  const E* Mg = reinterpret_cast<const E*>(p.M);
  auto issue_m = [&](int ks, int buf) {
    if constexpr (MASK) {
      const int cbase = (ks0 + ks) * KS;
      char* dst = reinterpret_cast<char*>(halo + buf * hcap * 4);
#pragma unroll
      for (int q = 0; q < HL; ++q) {
        const int idx = tid + 512 * q;
        const int hp = idx >> 2;
        const int c = cbase + (((idx & 3) ^ hswz(hp)) * EPC);
        const E* src = Mg + ((mpix[q] >= 0 && c < p.C) ? mpix[q] + c : 0);
        if ((512 * q + 64 * wave) / 4 < hcap)  // wave-uniform; hcap % 16 == 0: the instruction stays inside the buffer
          lds_dma16(src, __builtin_amdgcn_readfirstlane(lds_addr(dst + (512 * q + 64 * wave) * 16)));
      }
    }
  };
  // mask mode: the masked chunks of the block's own pixels go to G (issued at the start of the
  // next pipeline step, so the stores are the oldest vector-memory operations of that step)
  E* Gg = reinterpret_cast<E*>(p.G);
  auto store_g = [&]() {
    if constexpr (MASK) {
      if (gch < p.C) {
#pragma unroll
        for (int q = 0; q < HL; ++q)
          if ((core >> q) & 1u) *reinterpret_cast<u32x4*>(Gg + mpix[q] + gch) = hreg[q];
      }
    }
  };
  const int wm = wave / WN, wn = wave % WN;
  const int l16 = lane & 15, g = lane >> 4, g16 = g << 4;
  int hbase[MREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m) {
    const int q = wm * WTM + m * 16 + l16;
    const int sub = (int)p.fd_thw.div(q), rem = q - sub * THW;
    const int ty = (int)p.fd_tw.div(rem), tx = rem - ty * TW;
    hbase[m] = sub < IMG ? sub * HP + ty * SH * HW + tx * SW : 0;  // dead rows read row 0
  }
  f32x4 acc[MREP][NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](u32x4 a, u32x4 b, f32x4 c) -> f32x4 {
    if constexpr ((TPG_HALO_ABL & 4) != 0) {
      c[0] += __builtin_bit_cast(float, a[0] ^ b[1]);
      return c;
    } else if constexpr (BF) {
      return mfma16x16x32<DT>(a, b, c);
    } else {
      const f32x4 a4 = __builtin_bit_cast(f32x4, a);
      const f32x4 b4 = __builtin_bit_cast(f32x4, b);
#pragma unroll
      for (int e = 0; e < 4; ++e) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], c, 0, 0, 0);
      return c;
    }
  };

  // One pipeline step: the A fragments from the halo at tap offset toff (lanes g = 0..3 read
  // chunks g of the 64-byte pixel rows), the B fragments from ring slot wslot.
  // Paired step (p.half: the last k-step holds <= 16 live channels, C % 32 in 1..16): K = 32
  // of one MFMA is channels 0..15 of TWO taps -- lanes g = 0, 1 read chunks 0, 1 at tap offset
  // toff, lanes g = 2, 3 read chunks 0, 1 at toff2 (the packed slice holds the two taps'
  // weights in the same chunk order) -- so that k-step runs ceil(ntaps / 2) steps instead of
  // ntaps half-empty ones (206 channels: 6.9 % fewer MFMAs, 75 / 80: 17 %).
  auto compute = [&](int hbuf, int wslot, int toff, int toff2, bool paired) {
    const u32x4* H = halo + hbuf * hcap * 4;
    const u32x4* Wl = wts + wslot * BNL * 4;
    const int tl = g < 2 ? toff : toff2;
    const int gc = paired ? (g16 & 16) : g16;
    u32x4 af[MREP];
#pragma unroll
    for (int m = 0; m < MREP; ++m) {
      // byte offset hp * 64 + 16 * (chunk ^ hswz(hp)) = (hp << 6) + ((chunk << 4) ^ ((hp << 3) & 32))
      const int hp = hbase[m] + tl;
      af[m] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(H) + (hp << 6) + (gc ^ ((hp << 3) & 32)));
    }
    // all B fragments of the step are read up front into their own registers: reusing one
    // register quad across n made hipcc wait (lgkmcnt(0)) before every B read, exposing
    // the LDS latency 7 times per step on the 224-wide tile
    u32x4 bf[NREP];
#pragma unroll
    for (int n = 0; n < NREP; ++n) {
      const int r = wn * WTN + n * 16 + l16;
      bf[n] = Wl[r * 4 + (g ^ hswz(r))];
    }
#pragma unroll
    for (int n = 0; n < NREP; ++n)
#pragma unroll
      for (int m = 0; m < MREP; ++m) acc[m][n] = mma(af[m], bf[n], acc[m][n]);
    // schedule: every fragment read first, then the MFMAs (counted lgkmcnt waits instead
    // of one full wait per B fragment)
    __builtin_amdgcn_sched_group_barrier(0x100, MREP + NREP, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, MREP * NREP * (BF ? 1 : 4), 0);
  };

  // Software pipeline over steps s = ks*ntaps + t, one barrier per step:
  //   start of s : at t == 0 the halo of k-step ks+1 into registers
  //   body       : MFMAs on ring slot s%3 and halo buffer ks&1, then the LDS-DMA of step s+2's
  //                weights into ring slot (s+2)%3 (unconditional, clamped, so every wave
  //                always has GL DMA pieces per step in flight)
  //   end of s   : at t == ntaps-1 write the next halo to LDS; s_waitcnt vmcnt(GL)
  //                retires step s+1's DMA (issued during s-1) while step s+2's stays in
  //                flight; lgkmcnt(0); s_barrier.  Step s+1 then reads what was retired.
  // epilogue row table: output / residual element offsets of each of the BM rows (-1 = no row),
  // or the split-K slice row; and the bias of this block's columns, loaded into a register
  // here (the 512-row tiles fill their table after the loop, where the load's latency showed)
  float* W = p.ws ? p.ws + (int64_t)z * p.N * p.JH * p.JW * p.Nout : nullptr;
  float bias_pre = 0.f;
  if (tid >= 512 - BN) {
    const int c = n0 + tid - (512 - BN);
    if (p.bias && c < p.Nout) bias_pre = p.bias[c];
  }
  auto epi_table = [&]() {
    for (int q = tid; q < BM; q += 512) {
      const int sub = (int)p.fd_thw.div(q), rem = q - sub * THW;
      const int st = st0 + sub;
      int64_t yo = -1, ro = 0;
      if (sub < IMG && st < ntot) {
        const int nimg = (int)p.fd_tiles.div(st), trem = st - nimg * tiles;
        const int tty = (int)p.fd_tilesw.div(trem), ttx = trem - tty * tiles_w;
        const int ty = (int)p.fd_tw.div(rem), tx = rem - ty * TW;
        const int j = tty * TH + ty, i = ttx * TW + tx;
        if (j < p.JH && i < p.JW) {
          if (W) {
            yo = ((int64_t)(nimg * p.JH + j) * p.JW + i) * p.Nout;
          } else {
            const int oy = p.oy0 + p.osy * j, ox = p.ox0 + p.osx * i;
            yo = (int64_t)nimg * p.y_sn + (int64_t)oy * p.y_sh + (int64_t)ox * p.y_sw;
            ro = (int64_t)nimg * p.r_sn + (int64_t)oy * p.r_sh + (int64_t)ox * p.r_sw;
          }
        }
      }
      s_off[2 * q] = yo;
      s_off[2 * q + 1] = ro;
    }
    if (tid >= 512 - BN) s_bias[tid - (512 - BN)] = bias_pre;  // (the highest threads: BM >= 256 > BN)
  };

  // (the tap table written at entry is read only after the prologue's closing barrier)
  if (total > 0) {
    load_halo(0);
    issue_m(0, 0);
    if constexpr (EARLY) epi_table();  // (while the first halo and weight loads are in flight)
    if constexpr (MASK) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // y chunks landed
    store_halo(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    TPG_TL_MARK(1);
    int ks = 0, t = 0, slot = 0;
    int toff = s_toff[0];
    for (int s = 0; s < steps_full; ++s) {
      const bool more_ks = ks + 1 < nks;
      if (t == 0) {
        store_g();  // g of k-step ks (staged at the end of the previous one)
        if (more_ks) {
          load_halo(ks + 1);
          issue_m(ks + 1, (ks + 1) & 1);  // that buffer was last read in k-step ks - 1
        }
      }
      const int slot2 = slot == 0 ? 2 : slot - 1;  // (s + 2) % 3
      const int toff_next = s_toff[t + 1 == ntaps ? 0 : t + 1];  // read ahead of its use
      compute(ks & 1, slot, toff, toff, false);
      // step s+2's weight DMA behind this step's fragment reads and MFMAs (it has until the end of
      // step s+1): issued ahead of them it delayed the reads the first MFMAs wait on -- 1-3.5 %
      // per layer (r04: enhance_128 fwd 1.153 -> 1.142 ms, add_128 0.416 -> 0.401)
      issue_w(min(s + 2, total - 1), slot2);
      toff = toff_next;
      if (t == ntaps - 1 && more_ks) store_halo((ks + 1) & 1);
      if constexpr (GL == 1) asm volatile("s_waitcnt vmcnt(1)\n\ts_waitcnt lgkmcnt(0)" HALO_BAR ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)" HALO_BAR ::: "memory");
      slot = slot == 2 ? 0 : slot + 1;
      if (++t == ntaps) { t = 0; ++ks; }
    }
    // the paired last k-step (halo staged by the last full step; ks == nks - 1 here)
    for (int j = 0; j < npair_b; ++j) {
      const int s = steps_full + j;
      if (j == 0) store_g();
      const int slot2 = slot == 0 ? 2 : slot - 1;
      compute(ks & 1, slot, s_toff[2 * j], s_toff[min(2 * j + 1, ntaps - 1)], true);
      issue_w(min(s + 2, total - 1), slot2);
      if constexpr (GL == 1) asm volatile("s_waitcnt vmcnt(1)\n\ts_waitcnt lgkmcnt(0)" HALO_BAR ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)" HALO_BAR ::: "memory");
      slot = slot == 2 ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped tail DMA
  } else if constexpr (EARLY) {
    epi_table();
    __syncthreads();
  }
  TPG_TL_MARK(2);

  // ---- epilogue through LDS: the fp32 accumulators of RP rows at a time are parked in LDS,
  // then every thread finishes 8-channel groups of whole pixel rows: bias, residual and
  // activation with 16-byte residual loads / output stores (or an fp32 partial slice row).
  // Row addresses are computed once per block into a table.
  // passes: RP rows of all BN columns (the waves owning them park)
  constexpr int RP = halo_epi_rows(BN, BM);  // rows per pass
  constexpr int NPASS = BM / RP;
  constexpr int LDW = BN + 4;                // padded fp32 row stride
  constexpr int CG0 = BN / 8;                // 8-channel groups per row of a pass
  constexpr int IPT = (RP * CG0 + 511) / 512;  // groups per thread per pass (the last partial)
  constexpr int NV = 8 * (int)sizeof(E) / 16;  // 16-byte vectors per group
  static_assert(RP % WTM == 0, "epilogue tiling");
  static_assert(halo_epi_acc_bytes(BN, BM) == RP * LDW * 4, "epilogue LDS");
  float* s_acc = reinterpret_cast<float*>(lds) + (EARLY ? 0 : BM * 4 + 256);  // [RP][LDW]
  E* Y = reinterpret_cast<E*>(p.Y);
  const E* R = reinterpret_cast<const E*>(p.R);
  const E* XA = reinterpret_cast<const E*>(p.XA);
  // group it of a pass -> (table row, column in the pass) (compile-time divisors)
  auto grp = [&](int pass, int it, int& trow, int& c0) __attribute__((always_inline)) {
    const int row = it / CG0;
    c0 = (it - row * CG0) * 8;
    trow = pass * RP + row;
    return row;
  };
  // residual (or, without one, producer-x) vectors of a pass's groups: bf16 prefetches them,
  // all loads in flight before the first wait; the fp32 parity mode and the rare residual +
  // producer-x case (its x) load in the finishing loop.  One prefetch array: two (round 5's
  // first in_act build) pushed the 208 / 224-wide tiles past 256 VGPRs into ~700 B/lane of
  // scratch spills in the epilogue.
  constexpr int PF = BF ? IPT : 0;
  const bool pf_r = R != nullptr;
  const E* PSRC = pf_r ? R : XA;
  const bool pvec = pf_r ? p.rvec : p.yvec;
  u32x4 pv[IPT][NV];
  auto prefetch = [&](int pass) __attribute__((always_inline)) {
    const int ng = RP * CG0;
    const int cb = 0;
#pragma unroll
    for (int k = 0; k < (PSRC ? PF : 0); ++k) {
      int trow, c0;
      grp(pass, min(tid + 512 * k, ng - 1), trow, c0);  // (clamped past the last group)
      // unconditional (clamped) loads so that all of them issue before the first wait
      const int64_t yo = s_off[2 * trow];
      const int col = n0 + cb + c0;
      const bool ok = pvec && p.Nout - col >= 8 && yo >= 0;
      const u32x4* src = reinterpret_cast<const u32x4*>(PSRC + (ok ? (pf_r ? s_off[2 * trow + 1] : yo) + col : 0));
#pragma unroll
      for (int v = 0; v < NV; ++v) pv[k][v] = src[v];
    }
  };
  if constexpr (EARLY) {
    // (the table is in its own region: pass 0's loads go out before the barrier that frees
    // the halo / ring space for the parked rows)
    if (!W) prefetch(0);
  }
  // (epilogue barriers wait for LDS only: __syncthreads() would also drain vmcnt, i.e. wait for
  // the residual / producer-x loads prefetched just before it -- 2-4 us per pass measured)
  EPI_BARRIER();                             // every wave is done with the halo and the ring
  if constexpr (!EARLY) {
    epi_table();
    EPI_BARRIER();
  }
  TPG_TL_MARK(4);
#pragma unroll 1
  for (int pass = 0; pass < NPASS; ++pass) {
    if (!W && (!EARLY || pass > 0)) prefetch(pass);  // (before the park: latency under the park + barrier)
    if (wm * WTM >= pass * RP && wm * WTM < (pass + 1) * RP) {
      float* base = s_acc + (wm * WTM - pass * RP + 4 * g) * LDW + wn * WTN + l16;  // constant offsets below
#pragma unroll
      for (int m = 0; m < MREP; ++m)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
#pragma unroll
          for (int n = 0; n < NREP; ++n) base[(m * 16 + reg) * LDW + n * 16] = acc[m][n][reg];
    }
    EPI_BARRIER();
    if (pass == 0) TPG_TL_MARK(5);
    const int ng = RP * CG0;
    const int cb = 0;  // first tile column of the pass
    if (W) {  // split-K partial slice rows (fp32, row stride Nout)
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int it = tid + 512 * k;
        if (it >= ng) continue;
        int trow, c0;
        const int row = grp(pass, it, trow, c0);
        const int64_t yo = s_off[2 * trow];
        const int col0 = n0 + cb + c0;
        const int ncol = min(8, p.Nout - col0);
        if (yo < 0 || ncol <= 0) continue;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0 + 4);
        float* dst = W + yo + col0;
        if (ncol == 8 && p.wvec) {
          *reinterpret_cast<f32x4*>(dst) = a0;
          *reinterpret_cast<f32x4*>(dst + 4) = a1;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e < ncol) dst[e] = e < 4 ? a0[e & 3] : a1[e & 3];
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int it = tid + 512 * k;
        if (it >= ng) continue;
        int trow, c0;
        const int row = grp(pass, it, trow, c0);
        const int64_t yo = s_off[2 * trow];
        const int col0 = n0 + cb + c0;
        const int ncol = min(8, p.Nout - col0);
        if (yo < 0 || ncol <= 0) continue;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(s_acc + row * LDW + c0 + 4);
        float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        {
          const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cb + c0);
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cb + c0 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] += b0[e]; v[e + 4] += b1[e]; }
        }
        const bool full = ncol == 8;
        if (R) {
          union { u32x4 u[NV]; E e[8]; } rr;
#pragma unroll
          for (int q = 0; q < NV; ++q) rr.u[q] = pv[k][q];
          if (!(full && p.rvec && BF)) {
            const E* rs = R + s_off[2 * trow + 1] + col0;
#pragma unroll
            for (int e = 0; e < 8; ++e) rr.e[e] = e < ncol ? rs[e] : (E)0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += p.res_scale * (float)rr.e[e];
        }
        union { u32x4 u[NV]; E e[8]; } o;
        if (XA) {  // input gradient for the producer: v * xa_act'(x)
          union { u32x4 u[NV]; E e[8]; } xx;
#pragma unroll
          for (int q = 0; q < NV; ++q) xx.u[q] = pv[k][q];
          if (pf_r && full && p.yvec && BF) {  // (residual prefetched: x loaded here)
            const u32x4* xs = reinterpret_cast<const u32x4*>(XA + yo + col0);
#pragma unroll
            for (int q = 0; q < NV; ++q) xx.u[q] = xs[q];
          } else if (!(full && p.yvec && BF)) {
            const E* xs = XA + yo + col0;
#pragma unroll
            for (int e = 0; e < 8; ++e) xx.e[e] = e < ncol ? xs[e] : (E)0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e)
            o.e[e] = (E)tpg_act_grad(v[e], (float)xx.e[e], p.xa_act, p.xa_slope);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o.e[e] = (E)h_act(v[e], p.act, p.slope);
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
    }
    if (pass + 1 < NPASS) EPI_BARRIER();  // before the next pass overwrites s_acc
    if (pass == 0) TPG_TL_MARK(6);
  }
#ifdef TPG_BLOCK_TIMING
  __syncthreads();
  TPG_TL_MARK(3);
#endif
}

// {id, HL, BN, WM, WN}; id = 8 * (HL - 3) + bn index.  BN 80 serves the 75 / 80-channel layers.  BN 208 (13 fragments on one wave
// column) covers 193..208 output channels (the 206-channel enhance layers) without the 8 %
// of dead MFMA columns a 224 tile carries; BN 192 tiles 384 / 576 / 768 channels exactly with
// 24 MFMAs per wave and barrier (BN 128: 16).  HL = halo chunks per thread:
// the halo buffer holds up to HL*128 pixels.
#define TPG_HALO_BN(X, ID, HL)  \
  X(ID + 0, HL, 32, 8, 1)       \
  X(ID + 1, HL, 64, 8, 1)       \
  X(ID + 2, HL, 96, 8, 1)       \
  X(ID + 3, HL, 128, 4, 2)      \
  X(ID + 4, HL, 224, 4, 2)      \
  X(ID + 5, HL, 208, 8, 1)      \
  X(ID + 6, HL, 192, 4, 2)      \
  X(ID + 7, HL, 80, 8, 1)
#ifndef TPG_HALO_ISA_ONLY
#define TPG_HALO_CFGS(X)        \
  TPG_HALO_BN(X, 0, 3)          \
  TPG_HALO_BN(X, 8, 4)          \
  TPG_HALO_BN(X, 16, 5)
#else  // (ISA inspection builds: the enhance_128 tile only)
#define TPG_HALO_CFGS(X) X(13, 4, 208, 8, 1)
#endif
// 512-row tiles (ids 24, 25): BN 64 / 80 on the large maps, halo up to 1024 pixels (a BN-32
// variant for decoded_img128, D_and_G_model.py:279, measured slower: 47 -> 61 us forward)
#define TPG_HALO_CFGS512(X)     \
  X(24, 8, 64, 8, 1)            \
  X(25, 8, 80, 8, 1)
// stride-2 grids (ids 40..44): halo up to 1024 pixels, so only BN <= 128 fits LDS beside it
#define TPG_HALO_CFGS_S2(X)     \
  X(40, 8, 32, 8, 1)            \
  X(41, 8, 64, 8, 1)            \
  X(42, 8, 96, 8, 1)            \
  X(43, 8, 128, 4, 2)           \
  X(47, 8, 80, 8, 1)

int halo_cfg512(int bn) { return bn == 64 ? 24 : bn == 80 ? 25 : -1; }

int halo_cfg(int hl, int bn) {
  const int bi = bn == 32 ? 0 : bn == 64 ? 1 : bn == 96 ? 2 : bn == 128 ? 3 : bn == 224 ? 4 : bn == 208 ? 5
               : bn == 192 ? 6 : bn == 80 ? 7 : -1;
  if (bi < 0) return -1;
  if (hl >= 6 && hl <= 8) return (bi <= 3 || bi == 7) ? 40 + bi : -1;  // (no mask mode)
  if (hl < 3 || hl > 5) return -1;
  return 8 * (hl - 3) + bi;
}

// Pipeline variants measured and dropped: two taps per barrier with a 6-slot ring (+5 % on
// 7x7 layers alone, -2 % on the train step), a cross-barrier fragment prefetch with a
// 4-slot ring (-2..12 %: the second fragment set pushed the 224-wide tile past 256 VGPRs),
// waves 4-7 at a raised priority (no gain; removed in round 4 with the other variant bits).
size_t halo_lds_bytes(int hcap, int bn, int rs, int bm) {
  const size_t main = (size_t)(2 * hcap * 4 + rs * halo_bnl(bn) * 4) * 16 + TPG_MAX_TAPS * 4;
  if (bm == 256) return (size_t)halo_epi_early_off(main, bn) + bm * 16 + 1024;
  return std::max(main, (size_t)halo_epi_lds(bn, bm));
}

template <int DT, int HL, int BN, int WM, int WN, bool MASK, int BM = 256, int NG = 1>
static int launch_halo_t(const Grouped<HaloArgs, NG>& g, dim3 grid, size_t lds, hipStream_t s) {
  auto k = halo_kernel<DT, HL, BN, WM, WN, MASK, BM, NG>;
  const int maxl = (int)halo_lds_bytes(HL * 128, BN, 3, BM);
  static bool once = ((void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, maxl),
                      true);
  (void)once;
  hipLaunchKernelGGL(k, grid, dim3(512), lds, s, g);
  return (int)hipGetLastError();
}

template <int DT, int HL, int BN, int WM, int WN, bool MASK, int BM = 256>
static int launch_halo_t(const HaloArgs& a, dim3 grid, hipStream_t s) {
  Grouped<HaloArgs, 1> g;
  g.a[0] = a;
  g.boff[0] = 0; g.boff[1] = (int)(grid.x * grid.y * grid.z); g.nm = 1;
  return launch_halo_t<DT, HL, BN, WM, WN, MASK, BM, 1>(g, grid, halo_lds_bytes(a.hcap, a.BN, 3, BM),
                                                        s);
}

#ifdef TPG_HALO_ISA_ONLY
#undef TPG_HALO_CFGS512
#undef TPG_HALO_CFGS_S2
#define TPG_HALO_CFGS512(X)
#define TPG_HALO_CFGS_S2(X)
#endif

int launch_halo(const HaloArgs& a, int dtype, int cfg, hipStream_t s, bool mask) {
  dim3 grid((a.N * a.tiles_h * a.tiles_w + a.IMG - 1) / a.IMG, a.ntiles, a.ksplit);
  // mask mode: one k-step's y chunks must land (LDS-DMA issued at tap 0) before its halo is
  // staged (last tap): at least two taps, the 3-slot ring, whole 16-pixel DMA rows
  if (mask && (a.ntaps < 2 || a.hcap % 16 || a.SH != 1 || a.SW != 1)) return -1;
#define X(id, HL_, BN_, WM_, WN_)                                                          \
  if (cfg == (id)) {                                                                       \
    if (a.hcap > HL_ * 128) return -1;                                                     \
    if (mask) return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, true>(a, grid, s)    \
                   : dtype == 2 ? launch_halo_t<2, HL_, BN_, WM_, WN_, true>(a, grid, s)    \
                                : launch_halo_t<0, HL_, BN_, WM_, WN_, true>(a, grid, s);   \
    return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, false>(a, grid, s)            \
         : dtype == 2 ? launch_halo_t<2, HL_, BN_, WM_, WN_, false>(a, grid, s)            \
                      : launch_halo_t<0, HL_, BN_, WM_, WN_, false>(a, grid, s);           \
  }
  TPG_HALO_CFGS(X)
#undef X
#define X(id, HL_, BN_, WM_, WN_)                                                          \
  if (cfg == (id)) {                                                                       \
    if (a.hcap > HL_ * 128 || mask) return -1;                              \
    return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, false, 512>(a, grid, s)       \
         : dtype == 2 ? launch_halo_t<2, HL_, BN_, WM_, WN_, false, 512>(a, grid, s)       \
                      : launch_halo_t<0, HL_, BN_, WM_, WN_, false, 512>(a, grid, s);      \
  }
  TPG_HALO_CFGS512(X)
#undef X
#define X(id, HL_, BN_, WM_, WN_)                                                          \
  if (cfg == (id)) {                                                                       \
    if (a.hcap > HL_ * 128 || mask) return -1;                              \
    return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, false>(a, grid, s)            \
         : dtype == 2 ? launch_halo_t<2, HL_, BN_, WM_, WN_, false>(a, grid, s)            \
                      : launch_halo_t<0, HL_, BN_, WM_, WN_, false>(a, grid, s);           \
  }
  TPG_HALO_CFGS_S2(X)
#undef X
  return -1;
}

// Grouped builds (16-bit operands, 256-row tiles): the channel widths of the LocalPathway
// layers (32 / 64 / 128-column tiles: 3, 64, 128, 256 and 512 channels) at every halo size,
// and their stride-2 convs.  {id, HL, BN, WM, WN, mask variant}
#define TPG_HALO_GROUP_CFGS(X) \
  X(0, 3, 32, 8, 1, true)      \
  X(1, 3, 64, 8, 1, true)      \
  X(3, 3, 128, 4, 2, true)     \
  X(8, 4, 32, 8, 1, true)      \
  X(9, 4, 64, 8, 1, true)      \
  X(11, 4, 128, 4, 2, true)    \
  X(16, 5, 32, 8, 1, true)     \
  X(17, 5, 64, 8, 1, true)     \
  X(19, 5, 128, 4, 2, true)    \
  X(40, 8, 32, 8, 1, false)    \
  X(41, 8, 64, 8, 1, false)    \
  X(43, 8, 128, 4, 2, false)

#ifdef TPG_HALO_ISA_ONLY
#undef TPG_HALO_GROUP_CFGS
#define TPG_HALO_GROUP_CFGS(X)
#endif

int launch_halo_group(const HaloArgs* a, int n, int dtype, int cfg, hipStream_t s, bool mask) {
  if (n < 2 || n > TPG_GROUP_MAX || (dtype != 1 && dtype != 2)) return -1;
  Grouped<HaloArgs, TPG_GROUP_MAX> g;
  memset(&g, 0, sizeof(g));
  size_t lds = 0;
  int hcap = 0, blocks = 0;
  for (int m = 0; m < n; ++m) {
    const HaloArgs& h = a[m];
    if (h.BN != a[0].BN) return -1;
    if (mask && (h.ntaps < 2 || h.hcap % 16 || h.SH != 1 || h.SW != 1)) return -1;
    g.a[m] = h;
    g.boff[m] = blocks;
    blocks += ((h.N * h.tiles_h * h.tiles_w + h.IMG - 1) / h.IMG) * h.ntiles * h.ksplit;
    hcap = std::max(hcap, h.hcap);
    lds = std::max(lds, halo_lds_bytes(h.hcap, h.BN, 3, 256));
  }
  g.boff[n] = blocks;
  g.nm = n;
  // the halo capacity class every member fits (members differ in map size / tile)
  if (cfg < 24) cfg = halo_cfg(std::max(3, (hcap * 4 + 511) / 512), a[0].BN);
  if (cfg < 0) return -1;
  const dim3 grid(blocks);
#define X(id, HL_, BN_, WM_, WN_, MK_)                                                                  \
  if (cfg == (id)) {                                                                                    \
    if (hcap > HL_ * 128 || (mask && !MK_)) return -1;                                                  \
    if (mask) {                                                                                         \
      if constexpr (MK_)                                                                                \
        return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, MK_, 256, TPG_GROUP_MAX>(g, grid, lds, s) \
                          : launch_halo_t<2, HL_, BN_, WM_, WN_, MK_, 256, TPG_GROUP_MAX>(g, grid, lds, s); \
      return -1;                                                                                        \
    }                                                                                                   \
    return dtype == 1 ? launch_halo_t<1, HL_, BN_, WM_, WN_, false, 256, TPG_GROUP_MAX>(g, grid, lds, s)  \
                      : launch_halo_t<2, HL_, BN_, WM_, WN_, false, 256, TPG_GROUP_MAX>(g, grid, lds, s); \
  }
  TPG_HALO_GROUP_CFGS(X)
#undef X
  return -1;
}

// -------------------------------------------------------------- halo weight packing --
// Wp[ks*ntaps + tap][ntile][BNL rows][4 chunks][EPC]: row r of N-tile nt is output
// n' = nt*BN + r (zero when r >= BN or n' >= Nout); chunk' = chunk ^ hswz(r) holds
// logical channels c = ks*KS + chunk*EPC + e of that tap.  A paired last k-step (half) has
// ceil(ntaps / 2) slices after the full ones (pack_halo_item).
// One thread per 16-byte chunk, 32-bit index math (the packed image is < 2^31 elements).
template <typename E>
__global__ __launch_bounds__(256) void pack_halo_kernel(const PackArgs p, int nks, int bn, int bnl, int ntiles,
                                                        int nchunks) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < nchunks) pack_halo_item<E>(p, bn, bnl, ntiles, idx);
}

size_t halo_wp_bytes(int nks, int ntaps, int bn, int ntiles, int half) {
  return (size_t)halo_steps(nks, ntaps, half) * ntiles * halo_bnl(bn) * 64;
}

int launch_pack_halo(const PackArgs& a, int nks, int bn, int ntiles, hipStream_t s) {
  const int nchunks = halo_steps(nks, a.ntaps, a.half) * ntiles * halo_bnl(bn) * 4;
  const int blocks = (nchunks + 255) / 256;
  if (a.dtype == 2)
    hipLaunchKernelGGL(pack_halo_kernel<_Float16>, dim3(blocks), dim3(256), 0, s, a, nks, bn, halo_bnl(bn), ntiles, nchunks);
  else if (a.dtype == 1)
    hipLaunchKernelGGL(pack_halo_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, a, nks, bn, halo_bnl(bn), ntiles, nchunks);
  else
    hipLaunchKernelGGL(pack_halo_kernel<float>, dim3(blocks), dim3(256), 0, s, a, nks, bn, halo_bnl(bn), ntiles, nchunks);
  return (int)hipGetLastError();
}

}  // namespace tpg

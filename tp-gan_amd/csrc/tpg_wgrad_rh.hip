// Weight gradient of a stride-1 Conv2d by kernel-row halos (gfx950, bf16):
//   dW[a][b][r][s] += sum_{n,py,px} dY[n][py][px][a] * X[n][py + r - pt][px + s - pl][b].
//
// tpg_wgrad2.hip flattens (tap, b) into GEMM columns, so every 64-pixel k-tile DMAs the dY
// tile once per 128-column tile and the X pixels once per TAP: for a 5x5 206-channel layer
// at 128x128 that is ~16 GB of LDS-DMA per call and the kernel runs at the chip's DMA-fill
// rate, not the MFMA rate.  Here a block owns one kernel row r and a group of NT horizontal
// taps s0..s0+NT-1 (GEMM columns = NT x 64 channels), and a k-tile is 64 consecutive
// pixels of ONE image row, so the X operand of all NT taps is a single row segment of
// 64 + NT - 1 halo pixels, loaded once; tap s reads it shifted by s rows in LDS.  Bytes per
// flop drop ~2.4x (dY 16 KB + X 9 KB per 5.2 MFLOP at NT = 5).
//
// Pipeline as in wgrad2: 8 waves, both operands by buffer LDS-DMA (out-of-range offsets read
// zero = padding), 3-stage ring two k-tiles ahead, one counted vmcnt + barrier per k-tile,
// ds_read_b64_tr_b16 fragment reads for v_mfma_f32_16x16x32_bf16, fp32 atomics over the
// pixel splits.  Blocks of one pixel split are adjacent in the XCD-aware order, so the
// tiles that read the same dY / X rows run together on one XCD's L2.
#include "tpg_internal.h"
#include <type_traits>

// timing ablations (tools only; never in the product build): bit 1 no LDS-DMA, 2 no barrier,
// 4 no MFMA, 8 no fragment reads
#ifndef TPG_RH_ABL
#define TPG_RH_ABL 0
#endif

namespace tpg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4r;

__device__ __forceinline__ s16x4 rh_tr_read(const char* p) {
  s16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
// with a constant part of the address in the instruction's offset field (off: a constant once
// the caller's loops are unrolled)
__device__ __forceinline__ s16x4 rh_tr_read_o(const char* base, int off) {
  s16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)base;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(off));
  return v;
}


// chunk swizzles of the LDS rows (256- and 128-byte rows as in tpg_wgrad2.hip; 64-byte rows:
// the g = 0 / 1 row octets of a transposed read use disjoint chunk pairs)
template <int RB>
__device__ __forceinline__ int rh_swz(int row) {
  if constexpr (RB == 256) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  else if constexpr (RB == 128) return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
  else return ((row >> 3) & 1) << 1;
}

__device__ __forceinline__ int rh_refl(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// The tiles held to 128 VGPRs (two 512-thread blocks per CU)
template <int NR, int NT, int BM, int BC>
constexpr bool rh_fits128() {
  return NR == 2 || (NR == 1 && ((BM == 128 && BC == 32 && NT <= 5) || (BM == 64 && BC == 64 && NT <= 4) ||
                                 (BM == 64 && BC == 32)));
}

template <int DT, int NR, int NT, int BM, int BC>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(rh_fits128<NR, NT, BM, BC>() ? 4 : 1)))
void wgrad_rh_kernel(const WgradRHArgs p) {
  // k-tile: 64 pixels = TH x TW (TW = p.tw: a row segment of 64, or TH = 64 / TW whole rows of
  // a narrower map); block taps: NR kernel rows x NT columns (row mode NR = 1, image mode
  // NR = kh), all read from one (TH + NR - 1) x (TW + NT - 1) X halo of the k-tile
  constexpr int KP = 64;
  // BM a (dY channels) x BC b (X channels) per block; GEMM columns: (tap, b)
  constexpr int BN = NR * NT * BC;
  constexpr int WM = (BM == 64 && BC == 64) ? 2 : 4, WN = 8 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  constexpr int RBA = BM * 2, RBB = BC * 2;  // LDS row bytes
  constexpr int BYTES_A = KP * RBA;
  constexpr int GA = BYTES_A / 8192;         // 1 KiB DMA pieces per wave for dY
  constexpr int HROWS = NR == 1 ? 72 : 200;  // >= (TH + NR - 1) * (TW + NT - 1) halo pixels
  constexpr int BYTES_B = HROWS * RBB;
  constexpr int PB = (BYTES_B + 1023) / 1024, GB = (PB + 7) / 8;  // X pieces, per wave
  constexpr int RPP = 1024 / RBA, RPB = 1024 / RBB;              // rows per piece
  constexpr int STAGE = BYTES_A + GB * 8 * 1024;
  static_assert(NR == 1 ? ((NT >= 3 && NT <= 5) || NT == 7) : (NR == NT && NT <= 3), "taps per block");
  static_assert(GA * 8192 == BYTES_A && GA >= 1 && GB <= 2, "dma pieces");
  static_assert(MREP * 16 * WM == BM && NREP * 16 * WN == BN, "waves");

  extern __shared__ __attribute__((aligned(16))) char lds[];  // [3][STAGE]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // XCD-aware block order: physical block b runs on XCD b % 8 and each XCD is handed a
  // contiguous range of logical blocks; logical = split * tiles + tile.
  const int nblk = gridDim.x, full = nblk & ~7, bid = blockIdx.x;
  const int L = bid < full ? (bid & 7) * (full >> 3) + (bid >> 3) : bid;
  const int tile = L % p.tiles, split = L / p.tiles;
  int t = tile;
  const int ta = t % p.nta; t /= p.nta;
  const int tb = t % p.ntb; t /= p.ntb;
  const int r0 = (t % p.nrg) * NR;
  const int s0 = (t / p.nrg) * NT;
  const int a0 = ta * BM, b0 = tb * BC;
  const int kt0 = split * p.kt_per_split;
  const int nkt = min(p.nkt, kt0 + p.kt_per_split) - kt0;
  if (nkt <= 0) return;
  // bias gradient: the blocks of the first b tile, kernel row group and tap group see every
  // dY pixel of their split exactly once; one wave column of them sums the A fragments
  // (k-tile kt of the split is summed by the tile with share index kt % bshare, so the extra
  // MFMAs spread evenly over the a-tile's blocks; bshare = 1 keeps one owner: deterministic)
  const int sid = tb + p.ntb * (t % p.nrg + p.nrg * (t / p.nrg));
  const bool has_bias = p.dbias != nullptr && sid < p.bshare;

  // position of k-tile kt0: (n, py, px0), advanced incrementally (all scalar)
  // TH = floor(64 / TW): pixels TH*TW..63 of a k-tile are dead (zero dY rows), and a last
  // band may run past the map (its rows read zero as well)
  const int TW = p.tw, TH = KP / TW, HW = TW + NT - 1;
  const int segs = p.PW / TW, bands = (p.PH + TH - 1) / TH;
  int n = kt0 / (bands * segs);
  int rem = kt0 - n * bands * segs;
  int py = (rem / segs) * TH;
  int px0 = (rem % segs) * TW;

  const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.P), 0, p.p_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rQ = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Q), 0, p.q_bytes, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;

  // per-lane constants of the DMA pieces
  //   dY piece j of wave w: tile rows (GA*w + j) * RPP .. +RPP-1
  unsigned aoff[GA];
  int ary[GA];  // pixel row of the dY tile row inside the k-tile (large = dead)
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int row = (wave * GA + j) * RPP + lane / (RBA / 16), pc = lane % (RBA / 16);
    const int c = a0 + ((pc ^ rh_swz<RBA>(row)) << 3);
    const bool live = c < p.Ca && row < TH * TW;
    aoff[j] = live ? (unsigned)(((row / TW) * p.p_sh + (row % TW) * p.p_sw + c) * 2) : OOB;
    ary[j] = live ? row / TW : (1 << 28);
  }
  //   X piece j * 8 + w: halo rows (j * 8 + w) * RPB ..; pieces past PB only pad the count
  const int nhalo = (TH + NR - 1) * HW;
  int bhy[GB], bhx[GB], bch[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = (j * 8 + wave) * RPB + lane / (RBB / 16), pc = lane % (RBB / 16);
    const int c = b0 + ((pc ^ rh_swz<RBB>(row)) << 3);
    bhy[j] = row / HW + r0 - p.pt;             // + py  = X row of this halo pixel
    bhx[j] = row % HW + s0 - p.pl;             // + px0 = X column
    bch[j] = (c < p.Cb && row < nhalo && j * 8 + wave < PB) ? c : -1;
  }

  auto issue = [&](int slot, int n_, int py_, int px_) {
    if constexpr ((TPG_RH_ABL & 1) != 0) return;
    char* st = lds + slot * STAGE;
    const int sbase = (n_ * p.p_sn + py_ * p.p_sh + px_ * p.p_sw) * 2;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      // (a local copy: hipcc silently drops the kernel's host stub when the dependent-size
      // array element goes into the builtin directly)
      const unsigned vo = py_ + ary[j] < p.PH ? aoff[j] : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (__attribute__((address_space(3))) void*)(st + (wave * GA + j) * 1024),
                                               16, vo, sbase, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      int qy = py_ + bhy[j], qx = px_ + bhx[j];
      bool ok = bch[j] >= 0;
      if (p.pad_mode) { qy = rh_refl(qy, p.QH); qx = rh_refl(qx, p.QW); }
      else ok = ok && (unsigned)qy < (unsigned)p.QH && (unsigned)qx < (unsigned)p.QW;
      const unsigned off = ok ? (unsigned)((n_ * p.q_sn + qy * p.q_sh + qx * p.q_sw + bch[j]) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (__attribute__((address_space(3))) void*)(st + BYTES_A + (j * 8 + wave) * 1024),
                                               16, off, 0, 0, 0);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  // MFMA blocks of a padded edge tile that hold no real dW element -- 16 rows at or past Ca, or
  // 16 columns whose b channel is at or past Cb or whose tap is past the kernel -- read zeros;
  // their MFMAs are skipped (p.skip; wave-uniform masks, a scalar branch per MFMA).  206
  // channels pad to 256 rows x 224 columns per tap, a quarter of the MFMAs dead.
  unsigned mlive = ~0u, jlive = ~0u;
  if (p.skip) {
    mlive = 0;
    jlive = 0;
#pragma unroll
    for (int m = 0; m < MREP; ++m)
      if (a0 + wm * WTM + m * 16 < p.Ca) mlive |= 1u << m;
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      const int col = wn * WTN + j * 16, tap = col / BC;
      if (b0 + col % BC < p.Cb && r0 + tap / NT < p.kh && s0 + tap % NT < p.kw) jlive |= 1u << j;
    }
    mlive = __builtin_amdgcn_readfirstlane(mlive);
    jlive = __builtin_amdgcn_readfirstlane(jlive);
  }
  const int g = lane >> 4, l16 = lane & 15;
  const int q = l16 >> 2, p4 = l16 & 3;
  const bool bias_wave = has_bias && wn == 0;
  f32x4 acc[MREP][NREP], accb[MREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m) {
    accb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4r{one_pair<DT>(), one_pair<DT>(), one_pair<DT>(), one_pair<DT>()});

  // Fragment reads (transposed, 4 channels x 4 pixels per lane and read): fragment r < 2*MREP
  // is dY (A), the rest X halo rows shifted by the column's tap.  Next substep's reads are
  // issued between this substep's MFMAs (as in wgrad2).
  // Row mode: per-lane LDS byte offsets of the fragment reads.  The chunk swizzles depend on
  // the row only through bits the substep (+32 rows) and, for A, the K half (+4 rows) leave
  // alone, so every read is one of MREP + 2 * NREP lane offsets plus a constant (the
  // instruction's offset field): ~40 % fewer VALU in the k-tile loop.
  constexpr bool IMM = NR == 1;
  int abase[IMM ? MREP : 1], bbase[IMM ? NREP : 1][2];
  if constexpr (IMM) {
#pragma unroll
    for (int m = 0; m < MREP; ++m) {
      const int col = wm * WTM + m * 16 + 4 * p4, row = 8 * g + q;
      abase[m] = row * RBA + (((col >> 3) ^ rh_swz<RBA>(row)) << 4) + (col & 7) * 2;
    }
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int col = wn * WTN + j * 16 + 4 * p4;
        const int tap = col / BC, cb = col % BC;
        const int row = 8 * g + 4 * h + q + tap;  // (row mode: halo row = pixel + tap)
        bbase[j][h] = BYTES_A + row * RBB + (((cb >> 3) ^ rh_swz<RBB>(row)) << 4) + (cb & 7) * 2;
      }
    // opaque to the optimiser: kept as one register each (rematerialised from their parts they
    // cost two VALU per read and k-tile)
#pragma unroll
    for (int m = 0; m < MREP; ++m) asm volatile("" : "+v"(abase[m]));
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      asm volatile("" : "+v"(bbase[j][0]));
      asm volatile("" : "+v"(bbase[j][1]));
    }
  }
  // halo row of this lane's pixel k = ks*32 + 8g + 4h + q for tap (0, 0): (k / TW) * HW + k % TW
  int kbase[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q;
      kbase[ks][h] = (k / TW) * HW + k % TW;
    }
  // BIAS (compile-time): the bias MFMAs sit beside the regular MFMA holding each A fragment
  // (see tpg_wgrad2.hip: no runtime branch inside this hand-scheduled region)
  auto compute = [&](int slot, bool bias_now) {
    const char* A = lds + slot * STAGE;
    const char* B = A + BYTES_A;
    constexpr int NS = KP / 32;
    constexpr int R = 2 * (MREP + NREP), M = MREP * NREP;
    auto addr = [&](int ks, int rr) -> const char* {
      if (rr < 2 * MREP) {
        const int col = wm * WTM + (rr >> 1) * 16 + 4 * p4;
        const int row = ks * 32 + 8 * g + 4 * (rr & 1) + q;
        return A + row * RBA + (((col >> 3) ^ rh_swz<RBA>(row)) << 4) + (col & 7) * 2;
      }
      const int r2 = rr - 2 * MREP;
      const int col = wn * WTN + (r2 >> 1) * 16 + 4 * p4;  // (tap, b) column
      const int tap = col / BC, cb = col % BC;
      const int row = kbase[ks][r2 & 1] + (tap / NT) * HW + tap % NT;
      return B + row * RBB + (((cb >> 3) ^ rh_swz<RBB>(row)) << 4) + (cb & 7) * 2;
    };
    // IMM: lane base + constant offset (asm: a builtin LDS read makes hipcc put vmcnt(0) in
    // front of it for the in-flight LDS-DMA, measured +18 % on the 256 x 32 tile)
    auto rd = [&](int ks, int rr) -> s16x4 {
      if constexpr (IMM) {
        if (rr < 2 * MREP) return rh_tr_read_o(A + abase[rr >> 1], (32 * ks + 4 * (rr & 1)) * RBA);
        const int r2 = rr - 2 * MREP;
        return rh_tr_read_o(A + bbase[r2 >> 1][r2 & 1], 32 * ks * RBB);
      } else {
        return rh_tr_read(addr(ks, rr));
      }
    };
    s16x4 h[2][R];
    // (first-use order, counted waits below: the MFMAs start on their own operands)
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int rr = frag_read_order<MREP, NREP>(k);
      if constexpr ((TPG_RH_ABL & 8) == 0) h[0][rr] = rd(0, rr);
      else h[0][rr] = s16x4{(short)lane, 1, 2, 3};
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < NS; ++ks) {
      const int cur = ks & 1;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int m = i / NREP, j = i % NREP;
        if (ks == 0) {
          wait_lgkm(frag_read_wait<MREP, NREP>(i, i * R / M));
          __builtin_amdgcn_sched_barrier(0);
        }
        const bf16x8 av = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[cur][2 * m], h[cur][2 * m + 1],
                                                                             0, 1, 2, 3, 4, 5, 6, 7));
        const bf16x8 bv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[cur][2 * MREP + 2 * j],
                                                                             h[cur][2 * MREP + 2 * j + 1],
                                                                             0, 1, 2, 3, 4, 5, 6, 7));
        if constexpr ((TPG_RH_ABL & 4) == 0) {
          if ((mlive >> m) & (jlive >> j) & 1u) acc[m][j] = mfma16x16x32<DT>(av, bv, acc[m][j]);
        }
        else acc[m][j][0] += (float)av[0] * (float)bv[1];
        if (ks + 1 < NS) {
#pragma unroll
          for (int rr = i * R / M; rr < (i + 1) * R / M; ++rr) {
            if constexpr ((TPG_RH_ABL & 8) == 0)
              h[cur ^ 1][rr] = rd(ks + 1, rr);
            else h[cur ^ 1][rr] = h[cur][rr];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks + 1 < NS) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // bias (dY row sums) of an owned k-tile, after the hand-scheduled region: the A fragments
    // of both substeps are still in h (substep 1 read into h[1]) and every read has been
    // waited on.  (Bias MFMAs inside the region needed a second, compile-time copy of it,
    // which doubled its hoisted LDS addresses and spilled the wide tiles.)
    static_assert(NS == 2, "h holds both substeps");
    if (bias_now) {
    #pragma unroll
      for (int ks = 0; ks < NS; ++ks)
    #pragma unroll
        for (int m = 0; m < MREP; ++m)
          accb[m] = mfma16x16x32<DT>(__builtin_bit_cast(bf16x8, __builtin_shufflevector(h[ks][2 * m], h[ks][2 * m + 1],
                                                                                       0, 1, 2, 3, 4, 5, 6, 7)),
                                     ones, accb[m]);
    }
  };

  // pipeline: k-tile i in ring slot i % 3, issued two k-tiles ahead (clamped: static vmcnt)
  int in_ = n, iy = py, ix = px0, issued = 0;  // position of the next k-tile to issue
  auto issue_next = [&](int slot) {
    issue(slot, in_, iy, ix);
    if (++issued < nkt) {
      ix += TW;
      if (ix == p.PW) { ix = 0; iy += TH; if (iy >= p.PH) { iy = 0; ++in_; } }  // (partial last band)
    }
  };
#if (TPG_RH_ABL & 2) != 0
#define RH_WAIT_BARRIER() asm volatile("s_waitcnt vmcnt(6)\n\ts_waitcnt lgkmcnt(0)" ::: "memory")
#else
#define RH_WAIT_BARRIER()                                                                          \
  do {                                                                                             \
    if constexpr (GA + GB == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else if constexpr (GA + GB == 3) asm volatile("s_waitcnt vmcnt(3)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else if constexpr (GA + GB == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else if constexpr (GA + GB == 5) asm volatile("s_waitcnt vmcnt(5)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else asm volatile("s_waitcnt vmcnt(6)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");    \
  } while (0)
#endif
  static_assert(GA + GB >= 2 && GA + GB <= 6, "vmcnt");
  issue_next(0);
  issue_next(1);
  RH_WAIT_BARRIER();  // retires k-tile 0
  int slot = 0;
  for (int kt = 0; kt < nkt; ++kt) {
    issue_next(slot == 0 ? 2 : slot - 1);
    compute(slot, bias_wave && (kt0 + kt) % p.bshare == sid);  // (one inlined copy)
    RH_WAIT_BARRIER();  // retires k-tile kt+1, kt+2 stays in flight
    slot = slot == 2 ? 0 : slot + 1;
  }
#undef RH_WAIT_BARRIER
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue through LDS, in row chunks that fit the ring (see tpg_wgrad2.hip): sole owner
  // (ksplit == 1) 16-byte read-add-write of 4 consecutive columns; pixel splits one no-return
  // atomic per lane with 64 lanes on 64 consecutive columns of one dW row (full-rate shape,
  // instead of the MFMA C layout's four 64-byte segments in four rows)
  constexpr int LDC = BN + 4;
  constexpr int RING = 3 * STAGE;
  constexpr int RCH0 = (RING / (LDC * 4)) / WTM * WTM;  // rows per chunk: whole wave rows
  constexpr int RCH = RCH0 < BM ? RCH0 : BM;
  static_assert(RCH >= WTM, "a wave row of the C tile fits in the LDS ring");
  float* Cs = reinterpret_cast<float*>(lds);
  const int amax = min(BM, p.Ca - a0);
  auto col_off = [&](int col) -> int {  // dW element offset of tile column col at a = 0; -1: padding
    const int tap = col / BC;
    const int r = r0 + tap / NT, s = s0 + tap % NT, b = b0 + col % BC;
    if (r >= p.kh || s >= p.kw || b >= p.Cb) return -1;
    return b * p.w_sb + r * p.w_sr + s * p.w_ss;
  };
  constexpr int CG = (BN + 63) / 64;
  int coff[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) coff[c] = (c * 64 + lane < BN) ? col_off(c * 64 + lane) : -1;
  const bool vec_base = p.w_sb == 1 && (p.w_sa & 3) == 0 && ((uintptr_t)p.dW & 15) == 0;
  asm volatile("s_barrier" ::: "memory");  // (every wave's DMAs retired above: the ring is free)
#pragma unroll
  for (int c0 = 0; c0 < BM; c0 += RCH) {
    if (c0 > 0) __syncthreads();  // the previous chunk has been read
    if (wm * WTM >= c0 && wm * WTM < c0 + RCH) {
#pragma unroll
      for (int m = 0; m < MREP; ++m)
#pragma unroll
        for (int j = 0; j < NREP; ++j)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            Cs[(wm * WTM - c0 + m * 16 + 4 * g + reg) * LDC + wn * WTN + j * 16 + l16] = acc[m][j][reg];
    }
    __syncthreads();
    const int rows = min(RCH, amax - c0);
    if (p.ksplit == 1) {
      constexpr int CPR = BN / 4;
      for (int idx = tid; idx < rows * CPR; idx += 512) {
        const int row = idx / CPR, cc = 4 * (idx - row * CPR);
        const float4 v = *reinterpret_cast<const float4*>(Cs + row * LDC + cc);
        float* dst = p.dW + (a0 + c0 + row) * p.w_sa;
        const int o0 = col_off(cc);
        if (vec_base && o0 >= 0 && (o0 & 3) == 0 && col_off(cc + 3) == o0 + 3) {
          float4* d4 = reinterpret_cast<float4*>(dst + o0);
          float4 o = *d4;
          o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
          *d4 = o;
        } else {
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int oe = col_off(cc + e);
            if (oe >= 0) dst[oe] += vv[e];
          }
        }
      }
    } else {
      for (int row = wave; row < rows; row += 8) {
        float* dst = p.dW + (a0 + c0 + row) * p.w_sa;
#pragma unroll
        for (int c = 0; c < CG; ++c)
          if (coff[c] >= 0) atomicAdd(dst + coff[c], Cs[row * LDC + c * 64 + lane]);
      }
    }
  }
  if (bias_wave && l16 == 0) {  // every column of accb holds the row sum
#pragma unroll
    for (int m = 0; m < MREP; ++m)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int a = a0 + wm * WTM + m * 16 + 4 * g + reg;
        if (a >= p.Ca) continue;
        if (p.ksplit == 1 && p.bshare == 1) p.dbias[a] += accb[m][reg];
        else atomicAdd(p.dbias + a, accb[m][reg]);
      }
  }
}

// tile configs {id, BM, BC}; id = desc.algo - 6 (ids 4, 5: image mode, 32-channel b tiles;
// id 6: row mode, 256 dY channels per block, waves 64 x (NT x 32) / 2)
#define TPG_WGRAD_RH_CFGS(X) \
  X(0, 128, 64)              \
  X(1, 128, 32)              \
  X(2, 64, 64)               \
  X(3, 64, 32)               \
  X(4, 128, 32)              \
  X(5, 64, 32)               \
  X(6, 256, 32)

int wgrad_rh_tile(int cfg, int* bm, int* bc) {
#define X(id, BM_, BC_) if (cfg == (id)) { *bm = BM_; *bc = BC_; return 0; }
  TPG_WGRAD_RH_CFGS(X)
#undef X
  return -1;
}

template <int NR, int NT, int BM, int BC>
static int launch_rh_t(const WgradRHArgs& a, hipStream_t s) {
  constexpr int GB = (((NR == 1 ? 72 : 200) * BC * 2 + 1023) / 1024 + 7) / 8;
  const size_t lds = 3 * (64 * BM * 2 + GB * 8 * 1024);
  auto k1 = wgrad_rh_kernel<1, NR, NT, BM, BC>;
  auto k2 = wgrad_rh_kernel<2, NR, NT, BM, BC>;
  static bool once = ((void)hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                      (void)hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                      true);
  (void)once;
  hipLaunchKernelGGL(a.dtype == 2 ? k2 : k1, dim3(a.tiles * a.ksplit), dim3(512), lds, s, a);
  return (int)hipGetLastError();
}

// row-mode configs instantiate the 1 x {3,4,5} tap groups, image-mode ones the 2x2 / 3x3
template <int ID, int BM, int BC>
static int launch_rh_cfg(const WgradRHArgs& a, hipStream_t s) {
  if constexpr (ID < 4 || ID == 6) {
    if (a.nr == 1 && a.nt == 3) return launch_rh_t<1, 3, BM, BC>(a, s);
    if (a.nr == 1 && a.nt == 4) return launch_rh_t<1, 4, BM, BC>(a, s);
    if (a.nr == 1 && a.nt == 5) return launch_rh_t<1, 5, BM, BC>(a, s);
    // a whole 7-tap kernel row per block (7x7 convs): the 4 + 4 grouping computed a dead tap
    // column; only the tiles whose 7 x BC columns keep the fragments within the VGPR budget
    if constexpr (ID >= 1 && ID <= 3)
      if (a.nr == 1 && a.nt == 7) return launch_rh_t<1, 7, BM, BC>(a, s);
  } else {
    if (a.nr == 2 && a.nt == 2) return launch_rh_t<2, 2, BM, BC>(a, s);
    if (a.nr == 3 && a.nt == 3) return launch_rh_t<3, 3, BM, BC>(a, s);
  }
  return -1;
}

int launch_wgrad_rh(const WgradRHArgs& a, hipStream_t s) {
#define X(id, BM_, BC_) \
  if (a.cfg == (id)) return launch_rh_cfg<id, BM_, BC_>(a, s);
  TPG_WGRAD_RH_CFGS(X)
#undef X
  return -1;
}

}  // namespace tpg

// Weight gradient, pipelined (gfx950): dW[a][b][r][s] += sum_p P[p][a] * Q[gather_t(p)][b].
//
// Same problem as tpg_wgrad.hip (P = the pixel-grid operand, Q = the gathered one; see
// there for the Conv2d / ConvTranspose2d role mapping) restructured around the pipeline
// rules that made the halo kernel fast:
//   - 8 waves, block tile BM (a) x BN (b), K = pixels in tiles of KP (bf16: 64, f32: 32);
//   - both operand tiles arrive by buffer LDS-DMA (buffer_load_dwordx4 ... lds) into a
//     3-stage LDS ring, two k-tiles ahead; a pixel outside the image (or past the block's
//     pixel range) gets an offset beyond the buffer's num_records, which the hardware
//     returns as zero: padding costs no instruction;
//   - the LDS image is lane-linear (DMA), so the bank swizzle is applied to the SOURCE
//     address: LDS chunk c of row r holds logical chunk c ^ swz(r), and readers XOR back;
//   - one counted s_waitcnt vmcnt(pieces per k-tile) + lgkmcnt(0) + s_barrier per k-tile.
// Channel tails: a 16-byte chunk that straddles Ca / Cb reads a few channels past the
// tensor's real channels (inside the padded pixel row); they only feed dW rows / columns
// that are never written.
#include "tpg_internal.h"
#include <type_traits>
#include <string.h>

// timing ablations (tools only; never in the product build): bit 1 no LDS-DMA, 2 no barrier,
// 4 no MFMA, 8 no fragment reads, 16 no dW / bias epilogue (accumulators kept live)
#ifndef TPG_W2_ABL
#define TPG_W2_ABL 0
#endif

namespace tpg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4r;

__device__ __forceinline__ int w2_refl(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// ds_read_b64_tr_b16 through inline asm (see compute()) at base + off, off in the
// instruction's offset field (a constant once the caller's loops are unrolled)
__device__ __forceinline__ s16x4 tr_read_o(const char* base, int off) {
  s16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)base;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(off));
  return v;
}

// chunk swizzle of an LDS row of RB bytes (see tpg_wgrad.hip for the tr-read analysis)
template <bool BF, int RB>
__device__ __forceinline__ int w2_swz(int row) {
  if constexpr (BF) {
    if constexpr (RB == 128) return ((((row >> 1) & 1) | (((row >> 3) & 1) << 1))) << 1;
    else return (((row & 3) | (((row >> 3) & 1) << 2))) << 1;
  } else {
    return (row & 1) << 2;
  }
}

// Ring depth: TPG_W2_NST stages (default 3: two k-tiles in flight) where NST stages of the tile
// fit in half the CU's LDS (two blocks per CU), else 3.
#ifndef TPG_W2_NST
#define TPG_W2_NST 3
#endif
__host__ __device__ constexpr int w2_stages(int dt, int bm, int bn) {
  return (TPG_W2_NST * (dt ? 64 * (bm + bn) * 2 : 32 * (bm + bn) * 4) <= 80 * 1024) ? TPG_W2_NST : 3;
}

TPG_TL_DEFINE(wgrad2)

template <int DT, int BM, int BN, int WM, int WN, bool FLAT, int NG = 1>
__global__ __launch_bounds__(512) void wgrad2_kernel(const Grouped<Wgrad2Args, NG> G) {
  TPG_TL_MARK(0);
  // grouped launch: member m owns blocks [boff[m], boff[m + 1]) (its own 1-D grid)
  int mem = 0, bid0 = blockIdx.x, nblk0 = gridDim.x;
  if constexpr (NG > 1) {
    mem = group_member(G, blockIdx.x);
    bid0 = blockIdx.x - G.boff[mem];
    nblk0 = G.boff[mem + 1] - G.boff[mem];
  }
  const Wgrad2Args& p = G.a[mem];
  using E = dt_t<DT>;
  constexpr bool BF = DT != 0;
  constexpr int ES = sizeof(E);
  constexpr int EPC = 16 / ES;
  constexpr int KP = BF ? 64 : 32;            // pixels per k-tile
  constexpr int RBA = BM * ES, RBB = BN * ES;  // LDS row bytes
  constexpr int CPRA = RBA / 16, CPRB = RBB / 16;
  constexpr int BYTES_A = KP * RBA, BYTES_B = KP * RBB;
  constexpr int GA = BYTES_A / 8192, GB = BYTES_B / 8192;  // 1 KiB DMA pieces per wave
  constexpr int STAGE = BYTES_A + BYTES_B;
  constexpr int NST = w2_stages(DT, BM, BN);  // LDS ring depth: NST-1 k-tiles in flight
  static_assert((NST - 2) * (GA + GB) <= 63, "vmcnt field");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  static_assert(GA * 8192 == BYTES_A && GB * 8192 == BYTES_B && GA >= 1 && GB >= 1, "tile bytes");
  static_assert(WM * WN == 8 && MREP * 16 * WM == BM && NREP * 16 * WN == BN, "waves");

  extern __shared__ __attribute__((aligned(16))) char lds[];  // [NST][STAGE]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // 1-D grid, logical block = (tile, tap, split), tile fastest.  Physical block b runs on
  // XCD b % 8; each XCD is handed a contiguous range of logical blocks, so the tiles that
  // share a pixel range (same dY rows, X rows shifted by the taps) meet in one L2.
  const int nta = (p.Ca + BM - 1) / BM;
  const int ntb = ((FLAT ? p.ntaps * p.cbp : p.Cb) + BN - 1) / BN;
  const int nblk = nblk0, full = nblk & ~7;
  const int bid = bid0;
  const int L = bid < full ? (bid & 7) * (full >> 3) + (bid >> 3) : bid;
  const int tile = L % (nta * ntb), rest = L / (nta * ntb);
  const int ta = tile % nta, tb = tile / nta;
  const int a0 = ta * BM, b0 = tb * BN;
  const int tap = FLAT ? 0 : rest % p.ntaps;
  const int pbeg = (FLAT ? rest : rest / p.ntaps) * p.pix_per_split;
  const int pend = min(p.npix, pbeg + p.pix_per_split);
  const int nkt = (pend - pbeg + KP - 1) / KP;
  const int dy = p.dy[tap], dx = p.dx[tap];
  const int PHPW = p.PH * p.PW;
  // kernel arguments used in the DMA address math, hoisted once
  const FastDiv dv_phpw = p.div_phpw, dv_pw = p.div_pw;
  const int PW = p.PW, QH = p.QH, QW = p.QW, qsh = p.qst_h, qsw = p.qst_w, pad_mode = p.pad_mode;
  const int Ca = p.Ca, Cb = p.Cb;
  const int64_t psn = p.p_sn, psh = p.p_sh, psw = p.p_sw, qsn = p.q_sn, qsh_ = p.q_sh, qsw_ = p.q_sw;

  // FLAT: B columns are b' = tap * cbp + b over all taps (a 16-byte chunk never straddles
  // taps since cbp % 8 == 0); each lane's chunk, hence its tap, is fixed per DMA piece.
  int ldy[GB], ldx[GB], lcb[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int o = (wave * GB + j) * 1024 + lane * 16;
    const int row = o / RBB, pc = (o % RBB) / 16;
    const int lc = pc ^ w2_swz<BF, RBB>(row);
    const int col = b0 + lc * EPC;
    if constexpr (FLAT) {
      const int t = col / p.cbp;
      const int tc = t < p.ntaps ? t : 0;
      ldy[j] = p.dy[tc];
      ldx[j] = p.dx[tc];
      lcb[j] = t < p.ntaps ? col - t * p.cbp : (1 << 30);  // past the last tap -> zero
    } else {
      ldy[j] = dy; ldx[j] = dx; lcb[j] = col;
    }
  }
  // Fast address paths (the common case; the generic FastDiv path below is ~4x the VALU
  // and, quarter-rate multiplies included, would outrun the MFMAs it feeds):
  //   P dense  -> byte offset = (pixel * p_sw + c) * ES = scalar(p0) + pconst[j]
  //   Q fast   -> (py, px) of each lane's pixel carried from k-tile to k-tile by
  //               (dpy, dpx) with two conditional wraps; offset = scalar(p0) + qconst[j]
  const bool fastp = p.fastp, fastq = p.fastq;
  const int PH = p.PH, dpy = p.dpy, dpx = p.dpx;
  int pconst[GA], qconst[GB], qpy[GB], qpx[GB], qrow[GB], prow[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int o = (wave * GA + j) * 1024 + lane * 16;
    const int row = o / RBA, pc = (o % RBA) / 16;
    const int lc = pc ^ w2_swz<BF, RBA>(row);
    prow[j] = row;
    pconst[j] = (int)((row * psw + a0 + lc * EPC) * ES);
  }
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int o = (wave * GB + j) * 1024 + lane * 16;
    const int row = o / RBB;
    qrow[j] = row;
    const int pix = pbeg + row;
    const int n = dv_phpw.div(pix), rem = pix - n * PHPW;
    qpy[j] = dv_pw.div(rem);
    qpx[j] = rem - qpy[j] * PW;
    qconst[j] = (int)(((row + ldy[j] * QW + ldx[j]) * qsw_ + lcb[j]) * ES);
    if (lcb[j] >= (FLAT ? p.cbp : Cb)) qpy[j] = -(1 << 28);  // channel past the columns: never valid
  }
  int adv_kt = 0;  // k-tile the (qpy, qpx) state describes
  const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.P), 0, p.p_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rQ = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Q), 0, p.q_bytes, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;

  // DMA of k-tile kt into ring slot `slot` (kt is non-decreasing, +0 or +1 per call)
  auto issue = [&](int kt, int slot) {
    if constexpr ((TPG_W2_ABL & 1) != 0) return;
    char* st = lds + slot * STAGE;
    const int p0 = pbeg + kt * KP;
    if (fastp) {
      const int s0 = p0 * (int)psw * ES;
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const unsigned off = (p0 + prow[j] < pend) ? (unsigned)(s0 + pconst[j]) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (__attribute__((address_space(3))) void*)(st + (wave * GA + j) * 1024),
                                                 16, off, 0, 0, 0);
      }
    } else {
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int o = (wave * GA + j) * 1024 + lane * 16;  // byte offset in the A image
      const int row = o / RBA, pc = (o % RBA) / 16;
      const int lc = pc ^ w2_swz<BF, RBA>(row);
      const int pix = p0 + row;
      const int c = a0 + lc * EPC;
      unsigned off = OOB;
      {
        const int n = dv_phpw.div(pix), rem = pix - n * PHPW;
        const int py = dv_pw.div(rem), px = rem - py * PW;
        const unsigned o2 = (unsigned)((n * psn + py * psh + px * psw + c) * ES);
        off = (pix < pend && c < Ca) ? o2 : OOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (__attribute__((address_space(3))) void*)(st + (wave * GA + j) * 1024),
                                               16, off, 0, 0, 0);
    }
    }
    if (fastq) {
      const bool adv = kt > adv_kt;
      adv_kt = kt;
      const int s0 = p0 * (int)qsw_ * ES;
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        if (adv) {
          int px = qpx[j] + dpx, py = qpy[j] + dpy;
          if (px >= PW) { px -= PW; ++py; }
          if (py >= PH) py -= PH;
          qpx[j] = px; qpy[j] = py;
        }
        const bool ok = (p0 + qrow[j] < pend) && (unsigned)(qpy[j] + ldy[j]) < (unsigned)QH &&
                        (unsigned)(qpx[j] + ldx[j]) < (unsigned)QW;
        const unsigned off = ok ? (unsigned)(s0 + qconst[j]) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rQ, (__attribute__((address_space(3))) void*)(st + BYTES_A + (wave * GB + j) * 1024), 16, off, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int o = (wave * GB + j) * 1024 + lane * 16;
      const int row = o / RBB;
      const int pix = p0 + row;
      const int c = lcb[j];
      unsigned off = OOB;
      {
        const int n = dv_phpw.div(pix), rem = pix - n * PHPW;
        const int py = dv_pw.div(rem), px = rem - py * PW;
        int qy = py * qsh + ldy[j], qx = px * qsw + ldx[j];
        if (pad_mode) { qy = w2_refl(qy, QH); qx = w2_refl(qx, QW); }
        const bool ok = pix < pend && c < (FLAT ? p.cbp : Cb) && (unsigned)qy < (unsigned)QH && (unsigned)qx < (unsigned)QW;
        const unsigned o2 = (unsigned)((n * qsn + qy * qsh_ + qx * qsw_ + c) * ES);
        off = ok ? o2 : OOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rQ, (__attribute__((address_space(3))) void*)(st + BYTES_A + (wave * GB + j) * 1024), 16, off, 0, 0, 0);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, l16 = lane & 15;
  // bias gradient (P = dY): the first column tile (and tap) sees every pixel of the split once
  // (k-tile kt goes to the column tile with share index kt % bshare; bshare = 1: tile 0 only)
  const int sid = tb + ntb * (FLAT ? 0 : tap);
  const bool bias_wave = p.dbias != nullptr && sid < p.bshare && wn == 0;
  const int kt_base = pbeg / KP;
  f32x4 acc[MREP][NREP], accb[MREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m) {
    accb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4r{one_pair<DT>(), one_pair<DT>(), one_pair<DT>(), one_pair<DT>()});
  // per-lane LDS byte offsets of the 16-bit fragment reads (see rd in compute)
  int abase[BF ? MREP : 1], bbase[BF ? NREP : 1];
  if constexpr (BF) {
    const int q = l16 >> 2, p4 = l16 & 3, row = 8 * g + q;
#pragma unroll
    for (int m = 0; m < MREP; ++m) {
      const int col = wm * WTM + m * 16 + 4 * p4;
      abase[m] = row * RBA + (((col >> 3) ^ w2_swz<BF, RBA>(row)) << 4) + (col & 7) * 2;
    }
#pragma unroll
    for (int n = 0; n < NREP; ++n) {
      const int col = wn * WTN + n * 16 + 4 * p4;
      bbase[n] = row * RBB + (((col >> 3) ^ w2_swz<BF, RBB>(row)) << 4) + (col & 7) * 2;
    }
  }

  // BIAS (compile-time): also the bias MFMAs, right beside the regular MFMA that already
  // holds each A fragment (a runtime branch inside this hand-scheduled region let the compiler
  // copy the in-flight ds_read_b64_tr_b16 destinations before their wait: stale fragments)
  auto compute = [&](int slot, bool bias_now) {
    const char* A = lds + slot * STAGE;
    const char* B = A + BYTES_A;
    if constexpr (BF) {
      // Fragments of substep ks+1 are read while substep ks's MFMAs run: one tr read is
      // issued after each MFMA (R reads over M MFMAs), then one counted wait.  The reads
      // are inline asm (hipcc's LDS-DMA alias tracking would put a vmcnt(0) in front of
      // builtin LDS reads); each fragment's two halves are consumed only after the wait,
      // and the ISA is checked to hold them in place (no copies before the wait).
      constexpr int NS = KP / 32;
      constexpr int R = 2 * (MREP + NREP), M = MREP * NREP;
      // read r of substep ks: row ks*32 + 8g + 4(r & 1) + q, whose swizzle depends on the lane
      // alone (bits 0-1 and 3 of the row), so a per-lane base of each fragment plus a constant
      // (lane bases: abase / bbase, computed once per block)
      auto rd = [&](int ks, int r) -> s16x4 {
        if constexpr ((TPG_W2_ABL & 8) != 0) return s16x4{(short)r, (short)ks, 1, 2};
        if (r < 2 * MREP) return tr_read_o(A + abase[r >> 1], (32 * ks + 4 * (r & 1)) * RBA);
        const int rr = r - 2 * MREP;
        return tr_read_o(B + bbase[rr >> 1], (32 * ks + 4 * (rr & 1)) * RBB);
      };
      s16x4 h[2][R];
      // (first-use order, counted waits below: the MFMAs start on their own operands)
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int r = frag_read_order<MREP, NREP>(k);
        h[0][r] = rd(0, r);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < NS; ++ks) {
        const int cur = ks & 1;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const int m = i / NREP, n = i % NREP;
          if (ks == 0) {
            wait_lgkm(frag_read_wait<MREP, NREP>(i, i * R / M));
            __builtin_amdgcn_sched_barrier(0);
          }
          const bf16x8 av = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[cur][2 * m], h[cur][2 * m + 1],
                                                                               0, 1, 2, 3, 4, 5, 6, 7));
          const bf16x8 bv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[cur][2 * MREP + 2 * n],
                                                                               h[cur][2 * MREP + 2 * n + 1],
                                                                               0, 1, 2, 3, 4, 5, 6, 7));
          if constexpr ((TPG_W2_ABL & 4) == 0) acc[m][n] = mfma16x16x32<DT>(av, bv, acc[m][n]);
          else acc[m][n][0] += (float)av[0] * (float)bv[1];
          if (ks + 1 < NS) {
#pragma unroll
            for (int r = i * R / M; r < (i + 1) * R / M; ++r) h[cur ^ 1][r] = rd(ks + 1, r);
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
    } else {
#pragma unroll
      for (int kk = 0; kk < KP / 4; ++kk) {
        const int row = 4 * kk + g;
        float av[MREP], bv[NREP];
#pragma unroll
        for (int m = 0; m < MREP; ++m) {
          const int col = wm * WTM + m * 16 + l16;
          av[m] = *reinterpret_cast<const float*>(A + row * RBA + (((col >> 2) ^ w2_swz<BF, RBA>(row)) << 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int n = 0; n < NREP; ++n) {
          const int col = wn * WTN + n * 16 + l16;
          bv[n] = *reinterpret_cast<const float*>(B + row * RBB + (((col >> 2) ^ w2_swz<BF, RBB>(row)) << 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int m = 0; m < MREP; ++m)
#pragma unroll
          for (int n = 0; n < NREP; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[n], acc[m][n], 0, 0, 0);
        if (bias_now) {
#pragma unroll
          for (int m = 0; m < MREP; ++m) accb[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], 1.0f, accb[m], 0, 0, 0);
        }
      }
    }
  };

// k-tile kt+1 retired, the NST-2 k-tiles after it still in flight
#if (TPG_W2_ABL & 2) != 0
#define W2_WAIT_BARRIER() \
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"i"((NST - 2) * (GA + GB)) : "memory")
#else
#define W2_WAIT_BARRIER() \
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"((NST - 2) * (GA + GB)) : "memory")
#endif

  if (nkt > 0) {
#pragma unroll
    for (int j = 0; j < NST - 1; ++j) issue(min(j, nkt - 1), j);
    W2_WAIT_BARRIER();  // retires k-tile 0
    TPG_TL_MARK(1);
    int slot = 0;
    for (int kt = 0; kt < nkt; ++kt) {
      const int slot2 = slot == 0 ? NST - 1 : slot - 1;
      issue(min(kt + NST - 1, nkt - 1), slot2);  // unconditional (clamped): static vmcnt
      compute(slot, bias_wave && (kt_base + kt) % p.bshare == sid);  // (one inlined copy)
      W2_WAIT_BARRIER();
      slot = slot == NST - 1 ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  TPG_TL_MARK(2);
#undef W2_WAIT_BARRIER

  // ---- epilogue: the fp32 tile goes through LDS so that dW is written in whole rows.
  // The MFMA C layout (col = lane & 15 -> b, row = 4g + reg -> a) made every wave-instruction
  // touch four 64-byte segments in four dW rows; float atomics of that shape ran at about a
  // quarter of the full memory-side rate (ablation, profiles/r04/wgrad2_ablation.txt: without
  // the epilogue enh_8 46 -> 19 us, local_10 40 -> 12 us).  Now:
  //   sole owner (ksplit == 1): 16-byte read-add-write of 4 consecutive columns per thread;
  //   pixel split: one no-return atomic per lane, 64 lanes = 64 consecutive columns of ONE row
  //   (256 contiguous bytes per wave-instruction: the full-rate shape).
  if (nkt <= 0) {  // (an empty pixel split adds nothing; block-uniform)
    TPG_TL_MARK(3);
    return;
  }
  if constexpr ((TPG_W2_ABL & 16) != 0) {
#pragma unroll
    for (int m = 0; m < MREP; ++m) {
      asm volatile("" ::"v"(accb[m]));
#pragma unroll
      for (int n = 0; n < NREP; ++n) asm volatile("" ::"v"(acc[m][n]));
    }
    return;
  }
  constexpr int LDC = BN + 4;  // (+4 floats: the g = 0 / 1 row quads of a C write land on disjoint banks)
  static_assert(BM * LDC * 4 <= NST * STAGE, "C tile fits in the LDS ring");
  float* Cs = reinterpret_cast<float*>(lds);
  // every wave's DMAs have landed (the ring's last clamped re-issues included) before it is overwritten
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        Cs[(wm * WTM + m * 16 + 4 * g + reg) * LDC + wn * WTN + n * 16 + l16] = acc[m][n][reg];
  __syncthreads();
  const int r_tap = p.tr[tap], s_tap = p.ts[tap];
  // element offset in dW of tile column col at a = 0; -1: padding column (past Cb or the last tap)
  auto col_off = [&](int col) -> int {
    const int bq = b0 + col;
    int r = r_tap, s = s_tap, b = bq;
    if constexpr (FLAT) {
      const int t = bq / p.cbp;
      b = bq - t * p.cbp;
      if (t >= p.ntaps || b >= p.Cb) return -1;
      r = p.tr[t];
      s = p.ts[t];
    } else if (bq >= p.Cb) {
      return -1;
    } else if (p.bcomp) {
      const int rs = bq / p.comp_cb;
      b = bq - rs * p.comp_cb;
      r = rs / p.comp_kw;
      s = rs - r * p.comp_kw;
    }
    return b * p.w_sb + r * p.w_sr + s * p.w_ss;
  };
  const int amax = min(BM, p.Ca - a0);
  if (p.ksplit == 1) {
    constexpr int CPR = BN / 4, RPP = 512 / CPR;  // 4-column chunks per row, rows per pass
    constexpr int NIT = (BM + RPP - 1) / RPP;     // passes
    const int ch = tid % CPR, c0 = 4 * ch;
    int off[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) off[e] = col_off(c0 + e);
    const bool vec = p.w_sb == 1 && (p.w_sa & 3) == 0 && ((uintptr_t)p.dW & 15) == 0 && off[0] >= 0 &&
                     (off[0] & 3) == 0 && off[3] == off[0] + 3;
    if (vec) {
      // every pass's dW chunk read first (one memory latency, not one per pass), then add + store
      float4 o[NIT];
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int row = tid / CPR + i * RPP;
        if (row < amax) o[i] = *reinterpret_cast<const float4*>(p.dW + (a0 + row) * p.w_sa + off[0]);
      }
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int row = tid / CPR + i * RPP;
        if (row >= amax) continue;
        const float4 v = *reinterpret_cast<const float4*>(Cs + row * LDC + c0);
        o[i].x += v.x; o[i].y += v.y; o[i].z += v.z; o[i].w += v.w;
        *reinterpret_cast<float4*>(p.dW + (a0 + row) * p.w_sa + off[0]) = o[i];
      }
    }
    for (int row = tid / CPR; !vec && row < amax; row += RPP) {
      const float4 v = *reinterpret_cast<const float4*>(Cs + row * LDC + c0);
      float* dst = p.dW + (a0 + row) * p.w_sa;
      {
        if (off[0] >= 0) dst[off[0]] += v.x;
        if (off[1] >= 0) dst[off[1]] += v.y;
        if (off[2] >= 0) dst[off[2]] += v.z;
        if (off[3] >= 0) dst[off[3]] += v.w;
      }
    }
  } else {
    constexpr int CG = BN / 64;  // 64-column groups of a row
    static_assert(CG * 64 == BN, "row groups");
    int coff[CG];
#pragma unroll
    for (int c = 0; c < CG; ++c) coff[c] = col_off(c * 64 + lane);
    for (int row = wave; row < amax; row += 8) {
      float* dst = p.dW + (a0 + row) * p.w_sa;
#pragma unroll
      for (int c = 0; c < CG; ++c)
        if (coff[c] >= 0) atomicAdd(dst + coff[c], Cs[row * LDC + c * 64 + lane]);
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
#ifdef TPG_BLOCK_TIMING
  __syncthreads();
  TPG_TL_MARK(3);
#endif
}

// {id, BM, BN, WM, WN}
#define TPG_WGRAD2_CFGS(X) \
  X(0, 64, 64, 4, 2)       \
  X(1, 64, 128, 2, 4)      \
  X(2, 128, 64, 4, 2)      \
  X(3, 128, 128, 2, 4)     \
  X(4, 256, 128, 4, 2)

int wgrad2_cfg(int bm, int bn) {
#define X(id, BM_, BN_, WM_, WN_) if (bm == BM_ && bn == BN_) return id;
  TPG_WGRAD2_CFGS(X)
#undef X
  return -1;
}

static int w2_blocks(const Wgrad2Args& a, int bm, int bn) {
  const int ncols = a.bflat ? a.ntaps * a.cbp : a.Cb;
  return ((a.Ca + bm - 1) / bm) * ((ncols + bn - 1) / bn) * (a.bflat ? 1 : a.ntaps) * a.ksplit;
}

template <int DT, int BM, int BN, int WM, int WN, bool FLAT, int NG>
static int launch_w2_k(const Grouped<Wgrad2Args, NG>& g, int blocks, hipStream_t s) {
  auto k = wgrad2_kernel<DT, BM, BN, WM, WN, FLAT, NG>;
  const size_t lds = w2_stages(DT, BM, BN) * (DT ? 64 * (BM + BN) * 2 : 32 * (BM + BN) * 4);
  static bool once = ((void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                      true);
  (void)once;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), lds, s, g);
  return (int)hipGetLastError();
}

template <bool FLAT>
static int launch_wgrad2_t(const Wgrad2Args& a, int dtype, int cfg, int bm, int bn, hipStream_t s) {
  Grouped<Wgrad2Args, 1> g;
  g.a[0] = a;
  g.boff[0] = 0; g.boff[1] = w2_blocks(a, bm, bn); g.nm = 1;
#define X(id, BM_, BN_, WM_, WN_)                                                                       \
  if (cfg == (id)) {                                                                                    \
    if (dtype == 2) return launch_w2_k<2, BM_, BN_, WM_, WN_, FLAT, 1>(g, g.boff[1], s);               \
    if (dtype == 1) return launch_w2_k<1, BM_, BN_, WM_, WN_, FLAT, 1>(g, g.boff[1], s);               \
    return launch_w2_k<0, BM_, BN_, WM_, WN_, FLAT, 1>(g, g.boff[1], s);                               \
  }
  TPG_WGRAD2_CFGS(X)
#undef X
  return -1;
}

int launch_wgrad2(const Wgrad2Args& a, int dtype, int cfg, int bm, int bn, hipStream_t s) {
  return a.bflat ? launch_wgrad2_t<true>(a, dtype, cfg, bm, bn, s) : launch_wgrad2_t<false>(a, dtype, cfg, bm, bn, s);
}

// grouped builds: 16-bit operands, tap-flattened columns, every tile
int launch_wgrad2_group(const Wgrad2Args* a, int n, int dtype, int cfg, int bm, int bn, hipStream_t s) {
  if (n < 2 || n > TPG_GROUP_MAX || (dtype != 1 && dtype != 2)) return -1;
  Grouped<Wgrad2Args, TPG_GROUP_MAX> g;
  memset(&g, 0, sizeof(g));
  int blocks = 0;
  for (int m = 0; m < n; ++m) {
    if (!a[m].bflat) return -1;
    g.a[m] = a[m];
    g.boff[m] = blocks;
    blocks += w2_blocks(a[m], bm, bn);
  }
  g.boff[n] = blocks;
  g.nm = n;
#define X(id, BM_, BN_, WM_, WN_)                                                                       \
  if (cfg == (id)) {                                                                                    \
    if (dtype == 2) return launch_w2_k<2, BM_, BN_, WM_, WN_, true, TPG_GROUP_MAX>(g, blocks, s);      \
    return launch_w2_k<1, BM_, BN_, WM_, WN_, true, TPG_GROUP_MAX>(g, blocks, s);                      \
  }
  TPG_WGRAD2_CFGS(X)
#undef X
  return -1;
}

}  // namespace tpg

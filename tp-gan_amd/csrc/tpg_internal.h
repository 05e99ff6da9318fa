// Internal kernel interfaces of libtpgan_hip.so (gfx950).  The public C-ABI is
// include/tpgan.h; tpg_capi.hip turns a tpg_conv_desc into the problems below.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include "../../include/tpgan.h"

#define TPG_MAX_TAPS 64

namespace tpg {

// ---------------------------------------------------------------- element types ----
// Kernel dtype template parameter DT = tpg_conv_desc.dtype: 0 fp32 (parity mode), 1 bf16,
// 2 fp16.  The two 16-bit types share every layout (8 elements per 16-byte chunk) and differ
// only in the MFMA opcode and in the bits of 1.0.
template <int DT> struct DtT { using E = float; };
template <> struct DtT<1> { using E = __bf16; };
template <> struct DtT<2> { using E = _Float16; };
template <int DT> using dt_t = typename DtT<DT>::E;

typedef __attribute__((ext_vector_type(4))) float mf32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 mbf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 mf16x8;

// v_mfma_f32_16x16x32_bf16 / _f16 on two 16-byte fragments given as any 16-byte bit vector
template <int DT, typename V>
__device__ __forceinline__ mf32x4 mfma16x16x32(V a, V b, mf32x4 c) {
  if constexpr (DT == 2)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(mf16x8, a), __builtin_bit_cast(mf16x8, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(mbf16x8, a), __builtin_bit_cast(mbf16x8, b), c,
                                                   0, 0, 0);
}
// two packed 16-bit ones of DT
template <int DT> __host__ __device__ constexpr uint32_t one_pair() { return DT == 2 ? 0x3C003C00u : 0x3F803F80u; }
__host__ __device__ constexpr int dt_size(int dtype) { return dtype == 0 ? 4 : 2; }

// Activation codes of tpg_conv_desc.act (include/tpgan.h): 0 none, 1 ReLU,
// 2 LeakyReLU(slope), 3 ReLU6 (MobileNetV2.py:104,107 / :150,169).
__device__ __forceinline__ float tpg_act(float v, int act, float slope) {
  if (act == 2) return v > 0.f ? v : v * slope;
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 3) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

// d act / d pre-activation from the saved OUTPUT y (all four are monotone, so the sign
// pattern of y identifies the linear piece; ReLU6 passes gradient only on 0 < y < 6).
__device__ __forceinline__ float tpg_act_grad(float g, float y, int act, float slope) {
  if (act == 2) return y > 0.f ? g : g * slope;
  if (act == 1) return y > 0.f ? g : 0.f;
  if (act == 3) return (y > 0.f && y < 6.f) ? g : 0.f;
  return g;
}

// the input-gradient epilogue's producer act' (desc.in_act)
__device__ __forceinline__ float tpg_xa_grad(float g, float x, int act, float slope) {
  return tpg_act_grad(g, x, act, slope);
}

// Fast unsigned division by a runtime constant for n, d < 2^31 (round-up method):
// s = ceil(log2 d), mul = ceil(2^(31+s) / d) < 2^32, q = umulhi(n, mul) >> (s - 1).
struct FastDiv {
  uint32_t d, mul, shift, dmask;  // dmask = ~0 for d == 1 (q = n), else 0: branch-free
  __host__ void init(uint32_t div) {
    d = div < 1 ? 1 : div;
    if (d == 1) { mul = 0; shift = 0; dmask = 0xFFFFFFFFu; return; }
    uint32_t s = 0;
    while ((1u << s) < d) ++s;
    mul = (uint32_t)(((1ull << (31 + s)) + d - 1) / d);
    shift = s - 1;
    dmask = 0;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (__umulhi(n, mul) + (n & dmask)) >> shift;
  }
};

// LDS-DMA of one 16-byte chunk per lane (global_load_lds_dwordx4): lane i's 16 bytes land at
// LDS byte address lds_base + 16 * i (lds_base wave-uniform).  Inline asm rather than
// __builtin_amdgcn_global_load_lds: the compiler's wait-count pass treats the builtin's LDS write
// as an LGKM event of another kind and then waits lgkmcnt(0) before the first MFMA of every
// pipeline step instead of a counted wait on that step's fragment reads.  Callers order the
// DMA'd bytes themselves (s_waitcnt vmcnt + s_barrier); the pass, not seeing these loads, only
// ever waits for more VMEM operations than it needs (in-order completion), never fewer.
// Per-block timeline (ablation builds only, -DTPG_BLOCK_TIMING; tools/block_timeline.py): thread 0
// of every block stores s_memrealtime (100 MHz) at kernel entry (0), before the main loop (1), after
// it (2) and at the end (3), plus kernel-specific marks 4..7, into the buffer a per-file tpg_abl_tl_<file>() set (vector stores).
#ifdef TPG_BLOCK_TIMING
#define TPG_TL_DEFINE(NAME)                                                                    \
  __device__ unsigned long long* g_tl_buf = nullptr;                                          \
  extern "C" int tpg_abl_tl_##NAME(void* buf) {                                               \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_tl_buf), &buf, sizeof(buf));                   \
  }
#define TPG_TL_MARK(i)                                                                         \
  do {                                                                                         \
    unsigned long long* b_ = g_tl_buf;                                                         \
    if (b_ && threadIdx.x == 0)                                                                \
      b_[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + (i)] =         \
          __builtin_amdgcn_s_memrealtime();                                                    \
  } while (0)
#else
#define TPG_TL_DEFINE(NAME)
#define TPG_TL_MARK(i) do {} while (0)
#endif

__device__ __forceinline__ void lds_dma16(const void* gsrc, uint32_t lds_base) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "{m0}"(lds_base));  // (M0 -> LDS-DMA: 1 wait state)
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// s_waitcnt lgkmcnt(n) for an n that is constant once the caller's loops are unrolled (n > 15:
// the field's maximum, a stricter wait)
__device__ __forceinline__ void wait_lgkm(int n) {
  switch (n < 15 ? (n < 0 ? 0 : n) : 15) {
#define TPG_W(k) case k: asm volatile("s_waitcnt lgkmcnt(" #k ")" ::: "memory"); break;
    TPG_W(0) TPG_W(1) TPG_W(2) TPG_W(3) TPG_W(4) TPG_W(5) TPG_W(6) TPG_W(7)
    TPG_W(8) TPG_W(9) TPG_W(10) TPG_W(11) TPG_W(12) TPG_W(13) TPG_W(14) TPG_W(15)
#undef TPG_W
  }
}

// Weight-gradient kernels' first-substep fragment reads (2 transposed reads per fragment; A
// fragments 0..MREP-1 are reads 0..2*MREP-1, B fragments follow) issued in first-use order of
// the m-major MFMA sequence: A0, B0 .. B(NREP-1), A1 .. A(MREP-1).  frag_read_order(k) is the
// read issued k-th; frag_read_wait(i, ...) the lgkmcnt that lets MFMA i start once its own
// operands have landed, with `later` reads issued after the first substep's.
template <int MREP, int NREP>
__device__ __forceinline__ constexpr int frag_read_order(int k) {
  return k < 2 ? k : k < 2 + 2 * NREP ? 2 * MREP + (k - 2) : 2 + (k - 2 - 2 * NREP);
}
template <int MREP, int NREP>
__device__ __forceinline__ constexpr int frag_read_wait(int i, int later) {
  constexpr int R = 2 * (MREP + NREP);
  const int m = i / NREP, n = i % NREP;
  const int last = m == 0 ? 2 * n + 3 : 2 * NREP + 2 * m + 1;  // position of its last read
  return R - 1 - last + later;
}

// Zero the elements of a 16-byte chunk whose channel index (c0 + e) is >= C.
// Branch-free (selects only) so hipcc keeps loads in flight (no per-element vmcnt(0)).
template <int EPC>
__device__ __forceinline__ uint4 mask_chunk(uint4 v, int c0, int C) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if constexpr (EPC == 8) {  // two bf16 per dword
      const int e = c0 + 2 * d;
      uint32_t m = (e + 1 < C) ? 0xFFFFFFFFu : ((e < C) ? 0x0000FFFFu : 0u);
      w[d] &= m;
    } else {
      w[d] = (c0 + d < C) ? w[d] : 0u;
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------- implicit GEMM ----
// Out[row][n'] = sum_{tap, c} A[pix(row, tap)][c] * Wp[n'][tap][c]   (+ epilogue)
// row enumerates an output sub-grid (n, j, i): output pixel (oy0 + osy*j, ox0 + osx*i);
// A pixel for tap t is (n, j*ist_h + dy[t], i*ist_w + dx[t]) (zero outside, or reflected).
struct IgemmArgs {
  const void* A;
  int64_t a_sn, a_sh, a_sw;   // element strides; channel stride is 1
  int A_H, A_W, C;            // A spatial bounds and real channels per tap
  int upt;                    // 16-channel units per tap
  int ntaps;
  int nunits;                 // packed row length in units (multiple of units-per-k-tile)
  int M, JH, JW;              // rows = N*JH*JW
  int ist_h, ist_w;
  int pad_mode;
  int dil;                    // > 1: A is read on a grid dilated by dil (zeros between real pixels; halo kernel only)
  int vec_ok;                 // A rows 16-byte aligned: vector loads allowed
  const void* Wp;             // packed weights [Npad][nunits*16]
  int Nout;                   // real n'
  void* Y;
  int64_t y_sn, y_sh, y_sw;   // channel stride 1
  int oy0, ox0, osy, osx;
  const float* bias;
  int bias_mod;               // bias index = col % bias_mod when nonzero (composite n')
  const void* R;
  int64_t r_sn, r_sh, r_sw;
  float res_scale;
  int act;
  float slope;
  float* ws;                  // split-K fp32 accumulator [M][Nout]; null when ksplit == 1
  int ksplit, kt_per_split;
  FastDiv div_jw, div_jhjw;
  int8_t dy[TPG_MAX_TAPS], dx[TPG_MAX_TAPS];
};

// ---------------------------------------------------------------- weight gradient ----
// dW[a][b][r][s] += sum_p P[p][a] * Q[gather_t(p)][b]
// p enumerates the P grid (n, py, px); gather_t(p) = (n, py*qst_h + dy[t], px*qst_w + dx[t]).
struct WgradArgs {
  const void* P;
  int64_t p_sn, p_sh, p_sw;
  int PH, PW, Ca;
  const void* Q;
  int64_t q_sn, q_sh, q_sw;
  int QH, QW, Cb;             // Cb = b' extent (composite kh*kw*cb when bcomp)
  int npix;                   // N*PH*PW
  int qst_h, qst_w, pad_mode;
  int vec_p, vec_q;
  int ntaps;
  int bcomp, comp_kw, comp_cb;  // b' = (r*kw + s)*cb + b when bcomp
  float* dW;
  int64_t w_sa, w_sb, w_sr, w_ss;
  int ksplit, pix_per_split;
  FastDiv div_pw, div_phpw;
  int8_t dy[TPG_MAX_TAPS], dx[TPG_MAX_TAPS], tr[TPG_MAX_TAPS], ts[TPG_MAX_TAPS];
  int p_bytes, q_bytes;       // buffer extents for the DMA kernel (out-of-range reads -> 0)
  float* dbias;               // wgrad2 only, P = dY (Conv2d): dbias[a] += sum_p P[p][a] (may be null)
  int bshare;                 // k-tiles' bias sums spread over this many column tiles (1 = tile 0 only)
  int bflat, cbp;             // wgrad2 tap-flattened columns: b' = tap * cbp + b, cbp = rup(Cb, 8)
  int fastp;                  // P dense NHWC: DMA offset = pixel * p_sw + c, no division
  int fastq;                  // Q dense, same grid as P, unit stride, zero pad, image > one k-tile:
  int dpy, dpx;               //   per-lane (py, px) advanced by (dpy, dpx) = divmod(KP, PW) per k-tile
};
typedef WgradArgs Wgrad2Args;

// Stride-1 Conv2d weight gradient by kernel-row halos (tpg_wgrad_rh.hip): P = dY, Q = X,
// both dense channels-last; element strides; byte extents < 2^31.
struct WgradRHArgs {
  int dtype;                  // 1 bf16, 2 fp16
  const void* P;
  int p_sn, p_sh, p_sw, PH, PW, Ca, p_bytes;
  const void* Q;
  int q_sn, q_sh, q_sw, QH, QW, Cb, q_bytes;
  int kh, kw, pt, pl, pad_mode;
  int nr, nt;                 // taps per block: nr kernel rows (1 = row mode, kh = image mode) x nt
  int nrg;                    // kernel-row groups = ceil(kh / nr); tap-column groups = ceil(kw / nt)
  int tw;                     // k-tile width (64 px = (64 / tw) rows of tw)
  int cfg;                    // tile: 0 = 128 x 64, 1 = 128 x 32, 2 = 64 x 64, 3 = 64 x 32 (a x b);
                              // image mode: 4 = 128 x 32, 5 = 64 x 32
  int nta, ntb, tiles;        // tiles = nta * ntb * kh * groups
  int nkt, kt_per_split, ksplit;
  float* dW;
  int64_t w_sa, w_sb, w_sr, w_ss;
  float* dbias;               // dbias[a] += sum_p dY[p][a] (may be null): one MFMA against ones per
                              // A fragment; k-tile kt is summed by tile (kt % bshare) of the a-tile's
                              // (b, row, tap) tiles (bshare = 1: the first one, deterministic)
  int bshare;
  int skip;                   // skip the MFMAs of all-padding 16 x 16 blocks of edge tiles
};

// ---------------------------------------------------------------- weight packing ----
// Wp[n'][unit*16 + e] = W[a][b][r][s] (fp32 master -> compute dtype, zero padded).
// n' and c' = (unit % upt)*16 + e decode by mode: 0 -> a, 1 -> b, 2 -> composite (r,s,b),
// 3 -> composite (r,s,a); tap = unit / upt gives (r, s) when neither is composite.
struct PackArgs {
  const float* W;
  int64_t w_sa, w_sb, w_sr, w_ss;
  void* Wp;
  int Npad, Nreal, nunits, upt, ntaps, Creal;
  int nmode, cmode;
  int comp_kw, comp_c;        // composite decode: idx = (r*kw + s)*comp_c + ch
  int dtype;
  int hnks, half;             // halo layout: k-steps, and whether the last one is paired (HaloArgs.half)
  int8_t tr[TPG_MAX_TAPS], ts[TPG_MAX_TAPS];
};

constexpr int TPG_PACK_GROUPS = 8;  // 256-item groups per block of the batched pack kernel

// Batched weight packing (tpg_pack_run): one job per packed problem.  Jobs start on block
// boundaries (`first_block`, TPG_PACK_GROUPS * 256 items), so every block packs for
// exactly one job.
struct PackJob {
  PackArgs k;
  int kind;                   // 0: implicit-GEMM layout (pack_kernel), 1: halo layout (pack_halo_kernel)
  int nks, bn, bnl, ntiles;   // halo layout
  int items;                  // igemm: Npad * nunits 16-element units; halo: 16-byte chunks
  int first_block;            // set by tpg_pack_prepare (blocks of TPG_PACK_GROUPS * 256 items)
  int nblocks;
};

__device__ __forceinline__ int pack_hswz(int row) { return ((row >> 2) & 1) << 1; }

// igemm layout: item = (n', unit) -> 16 consecutive elements of Wp row n'
template <typename E>
__device__ __forceinline__ void pack_igemm_item(const PackArgs& p, int idx) {
  const int np = idx / p.nunits;
  const int unit = idx - np * p.nunits;
  const int tap = unit / p.upt;
  const int cbase = (unit - tap * p.upt) * 16;
  E out[16];
  const bool ok = np < p.Nreal && tap < p.ntaps;
  int a = 0, b = 0, r = ok ? p.tr[tap] : 0, s = ok ? p.ts[tap] : 0;
  if (p.nmode == 0) a = np;
  else if (p.nmode == 1) b = np;
  else {
    const int rs = np / p.comp_c, ch = np - rs * p.comp_c;
    r = rs / p.comp_kw; s = rs - r * p.comp_kw;
    if (p.nmode == 2) b = ch; else a = ch;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int cp = cbase + e;
    float v = 0.f;
    if (ok && cp < p.Creal) {
      int aa = a, bb = b, rr = r, ss = s;
      if (p.cmode == 0) aa = cp;
      else if (p.cmode == 1) bb = cp;
      else {
        const int rs = cp / p.comp_c, ch = cp - rs * p.comp_c;
        rr = rs / p.comp_kw; ss = rs - rr * p.comp_kw;
        if (p.cmode == 2) bb = ch; else aa = ch;
      }
      v = p.W[(int64_t)aa * p.w_sa + (int64_t)bb * p.w_sb + (int64_t)rr * p.w_sr + (int64_t)ss * p.w_ss];
    }
    out[e] = (E)v;
  }
  uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<E*>(p.Wp) + (int64_t)idx * 16);
  const uint4* src = reinterpret_cast<const uint4*>(out);
#pragma unroll
  for (int q = 0; q < (int)(16 * sizeof(E) / 16); ++q) dst[q] = src[q];
}

// halo layout: Wp[ks*ntaps + tap][ntile][bnl rows][4 chunks][EPC]; item = one 16-byte chunk;
// row r of N-tile nt is n' = nt*bn + r, chunk' = chunk ^ hswz(r)
template <typename E>
__device__ __forceinline__ void pack_halo_item(const PackArgs& p, int bn, int bnl, int ntiles, int idx) {
  constexpr int EPC = 16 / sizeof(E);
  constexpr int ROW = 4 * EPC;
  const int pchunk = idx & 3;
  int rr = idx >> 2;
  const int r = rr % bnl;
  rr /= bnl;
  const int nt = rr % ntiles;
  rr /= ntiles;
  // step rr: k-step rr / ntaps, tap rr % ntaps; past the full k-steps of a paired image (half:
  // the last k-step holds <= 16 live channels) step j carries taps 2j (logical chunks 0, 1) and
  // 2j + 1 (chunks 2, 3), channels 0..15 of that k-step each (tpg_halo.hip compute)
  const int lc = pchunk ^ pack_hswz(r);
  const int nfull = (p.half ? p.hnks - 1 : p.hnks) * p.ntaps;
  int tap, c0;
  bool tap_ok = true;
  if (rr < nfull) {
    tap = rr % p.ntaps;
    c0 = (rr / p.ntaps) * ROW + lc * EPC;
  } else {
    tap = 2 * (rr - nfull) + (lc >> 1);
    c0 = (p.hnks - 1) * ROW + (lc & 1) * EPC;
    tap_ok = tap < p.ntaps;
    if (!tap_ok) tap = 0;
  }
  const int np = nt * bn + r;
  union { uint4 u; E e[EPC]; } o;
  const bool row_ok = r < bn && np < p.Nreal && tap_ok;
  const int tr = p.tr[tap], ts = p.ts[tap];
  const int64_t base = (int64_t)tr * p.w_sr + (int64_t)ts * p.w_ss +
                       (p.nmode == 0 ? (int64_t)np * p.w_sa : (int64_t)np * p.w_sb);
  const int64_t cstride = p.cmode == 0 ? p.w_sa : p.w_sb;
  const float* src = p.W + base + (int64_t)c0 * cstride;
  if (cstride == 1 && row_ok && c0 + EPC <= p.Creal && ((uintptr_t)src % 16) == 0) {
    // contiguous input channels (the forward images of channels-last weights): 16-byte loads
#pragma unroll
    for (int q = 0; q < EPC / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      o.e[4 * q] = (E)v.x; o.e[4 * q + 1] = (E)v.y; o.e[4 * q + 2] = (E)v.z; o.e[4 * q + 3] = (E)v.w;
    }
  } else if (cstride == 1 && row_ok && c0 + EPC <= p.Creal && ((uintptr_t)src % 8) == 0) {
    // (an even channel count that is not a multiple of 4 -- 206 -- leaves every other tap's
    // rows 8-byte aligned only: 8-byte loads instead of 4-byte ones; G's re-pack 0.489 ->
    // 0.470 ms, tools/bench_opt.py, gpurun r06r)
#pragma unroll
    for (int q = 0; q < EPC / 2; ++q) {
      const float2 v = reinterpret_cast<const float2*>(src)[q];
      o.e[2 * q] = (E)v.x; o.e[2 * q + 1] = (E)v.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int c = c0 + e;
      o.e[e] = (E)((row_ok && c < p.Creal) ? p.W[base + (int64_t)c * cstride] : 0.f);
    }
  }
  reinterpret_cast<uint4*>(p.Wp)[idx] = o.u;
}

int launch_pack_many(const PackJob* jobs_dev, int n, int nblocks, hipStream_t s);


struct EpiArgs {               // split-K finalize: Y = act(sum_z ws[z] + bias [+ res])
  const float* ws;
  int nslices;                // number of partial slices (1 for atomically accumulated ws)
  int64_t slice;              // elements per slice (M * Nout)
  int M, Nout, JH, JW;
  void* Y;
  int64_t y_sn, y_sh, y_sw;
  int oy0, ox0, osy, osx;
  const float* bias;
  int bias_mod;
  const void* R;
  int64_t r_sn, r_sh, r_sw;
  float res_scale;
  int act;
  float slope;
  int dtype;
  // input-gradient epilogues (desc.in_act): Y = v * xa_act'(XA), XA read at Y's offsets
  const void* XA;
  int xa_act;
  float xa_slope;
};

// ---------------------------------------------------------------- halo direct conv ----
// (Sub-)grid conv: output (sub-grid) pixel (j, i) reads A at (j*SH + dy[t], i*SW + dx[t]).
// A block owns IMG sub-tiles of TH x TW output pixels (IMG > 1 only for whole-image tiles of
// small maps), i.e. up to 256 rows, and k-steps [z*kps, (z+1)*kps) of its split z.
struct HaloArgs {
  const void* A;
  int64_t a_sn, a_sh, a_sw;
  int A_H, A_W, C;
  int nks;                    // 64-byte channel steps = ceil(C / KS)
  int ntaps;
  int half;                   // 16-bit, C % 32 in 1..16: the last k-step runs two taps per MFMA (paired steps)
  int dymin, dxmin, HH, HW;   // halo of one sub-tile = HH x HW pixels
  int pad_mode, vec_ok;        // vec_ok: 16-byte loads of whole chunks stay inside each pixel row
  int pw;                     // > 0: one-tap problem on the pointwise GEMM kernel, tile config (tpg_pw.hip)
  int N, JH, JW, tiles_h, tiles_w;
  int TH, TW, IMG, SH, SW;    // sub-tile shape, sub-tiles per block, A-grid stride of the taps
  int dil;                    // > 1: halo coordinates are on A dilated by dil (zero between real pixels)
  int hcap;                   // halo pixels per LDS buffer (>= IMG*HH*HW)
  int ksplit, kps;            // split over k-steps (grid.z); > 1 -> fp32 partials into ws
  float* ws;                  // [ksplit][N*JH*JW][Nout] partial slices (class-local rows)
  const void* Wp;             // [nks*ntaps][ntiles][rup(BN,128)][64 B], rows pre-swizzled
  int ntiles, BN, Nout;
  void* Y;
  int64_t y_sn, y_sh, y_sw;
  int oy0, ox0, osy, osx;
  const float* bias;
  const void* R;
  int64_t r_sn, r_sh, r_sw;
  float res_scale;
  int act;
  float slope;
  int yvec, rvec, wvec;       // 16-byte output / residual / partial-slice stores allowed
  // Masked input-gradient mode (launch_halo(..., mask = true); stride-1 "same" Conv2d dgrad):
  // A holds the incoming gradient gy, M the conv's saved output y (same grid); the halo is
  // staged as g = gy * act'(y) (mact / mslope), and every g chunk of the block's own output
  // pixels (blockIdx.y == 0) is also stored to G (G has M's strides), so the weight gradient
  // can read g without a separate activation-backward pass.
  const void* M;
  int64_t m_sn, m_sh, m_sw;
  void* G;
  int mact;
  float mslope;
  // input-gradient epilogue (desc.in_act: the producer of the conv's input x applied act'):
  // the output is v * xa_act'(XA) instead of act(v); XA (= x) is read at Y's element offsets
  const void* XA;
  int xa_act;
  float xa_slope;
  // the prologue's index math by multiply-shift (each runtime division was ~25 VALU; the
  // small-map blocks spent ~1-2 us of a ~5 us prologue on them): HH*HW, HW, tiles_h*tiles_w,
  // tiles_w, TH*TW, TW
  FastDiv fd_hp, fd_hw, fd_tiles, fd_tilesw, fd_thw, fd_tw;
  int toff[TPG_MAX_TAPS];     // per tap: (dy - dymin) * HW + (dx - dxmin), halo pixel shift
};

// ---------------------------------------------------------------- grouped launches ----
// One grid over up to TPG_GROUP_MAX independent problems of the same kernel instance (the
// four LocalPathways' same-shaped layers, tpg_group_begin / tpg_group_end): member m owns
// the 1-D blocks [boff[m], boff[m + 1]) and reads its own argument block a[m].  NG = 1 is the
// plain launch (the kernel keeps its own grid shape).
#define TPG_GROUP_MAX 4
template <typename A, int NG>
struct Grouped {
  A a[NG];
  int boff[NG + 1];
  int nm;
};
template <typename A, int NG>
__device__ __forceinline__ int group_member(const Grouped<A, NG>& G, int bid) {
  int m = 0;
#pragma unroll
  for (int i = 1; i < NG; ++i)
    if (i < G.nm && bid >= G.boff[i]) m = i;
  return m;
}

// g = gy * act'(y) (+ dbias column sums), vector form: pixel-dense channels-last rows, 16-byte
// aligned (tpg_elementwise.hip act_bwd_vec_kernel)
struct ActVecArgs {
  int64_t npix;
  int C, act;
  float slope;
  const void* gy;
  int64_t gps;
  const void* y;
  int64_t yps;
  void* g;
  int64_t gps_out;
  float* dbias;
  int64_t pix_per_block;
  int blocks;
};

// Grouped launchers: return -1 (nothing launched) when the instance has no grouped build or
// the members disagree on it; the caller then launches the members one by one.
int launch_halo_group(const HaloArgs* a, int n, int dtype, int cfg, hipStream_t s, bool mask);
int launch_epilogue_group(const EpiArgs* a, int n, hipStream_t s);
int launch_wgrad2_group(const Wgrad2Args* a, int n, int dtype, int cfg, int bm, int bn, hipStream_t s);
int act_vec_plan(int64_t npix, int c, int dtype, bool dbias, ActVecArgs* out);
int act_vec_args(int n, int c, int h, int w, int act, float slope, const ::tpg_tensor& gy, const ::tpg_tensor& y,
                 const ::tpg_tensor& g, float* dbias, ActVecArgs* a);
int launch_act_vec(const ActVecArgs& a, int dtype, hipStream_t s);
int launch_act_vec_group(const ActVecArgs* a, int n, int dtype, hipStream_t s);

// sets the thread-local message returned by tpg_last_error() (tpg_capi.hip); returns code
int record_error(int code, const char* msg);

// tpg_set_deterministic(): every reduction in a fixed order (no split-K / pixel-split fp32
// atomics, one block per bias-gradient sum); process-wide, for parity and run-to-run tests
int deterministic();

// launchers (return hipError_t as int); cfg selects the tile shape
int launch_igemm(const IgemmArgs& a, int dtype, int cfg, hipStream_t s);
int igemm_cfg_bn(int cfg);
int igemm_cfg_bm(int cfg);
int launch_wgrad(const WgradArgs& a, int dtype, int cfg, hipStream_t s);
int wgrad_cfg_bm(int cfg);
int wgrad_cfg_bn(int cfg);
int launch_pack(const PackArgs& a, hipStream_t s);
int wgrad2_cfg(int bm, int bn);
int launch_wgrad2(const Wgrad2Args& a, int dtype, int cfg, int bm, int bn, hipStream_t s);
int launch_epilogue(const EpiArgs& a, hipStream_t s);
int launch_wgrad_rh(const WgradRHArgs& a, hipStream_t s);
int wgrad_rh_tile(int cfg, int* bm, int* bc);
int halo_cfg(int hl, int bn);
size_t halo_lds_bytes(int hcap, int bn, int rs = 3, int bm = 256);
int halo_cfg512(int bn);
int launch_halo(const HaloArgs& a, int dtype, int cfg, hipStream_t s, bool mask = false);
// pointwise (1x1) GEMM kernel on a one-tap halo plan (a.pw = tile config 1..4: 128x128, 128x64,
// 64x128, 64x64 rows x output channels); same packed weights, epilogue and split-K slices
int launch_pw(const HaloArgs& a, int dtype, hipStream_t s);
// fused G-step losses (tpg_losses.hip): forward when dx / bwd is null / false (partials in part,
// the scalar in out), else the gradient
int launch_image_losses(int n, int c, int h, int w, const tpg_tensor& x, const tpg_tensor& r, float w_pix, float w_sym,
                        float w_tv, float* part, const float* gout, float* out, const tpg_tensor* dx, hipStream_t st);
int launch_l1_set(int nseg, const tpg_l1_seg* segs, float* part, const float* gout, float* out, bool bwd,
                  hipStream_t st);
// SSD landmark head (tpg_ssd.hip): MultiTaskLoss assignment + loss, its backward, the decoder
int launch_ssd_loss_fwd(int B, int n, int C, int k, const float* pred, const float* cls, const float* truth, float width,
                        float height, double ratio_nb, float alpha, float beta, const float* keys, int* labels,
                        unsigned char* sel, float* terms, hipStream_t s);
int launch_ssd_loss_bwd(int B, int n, int C, const float* pred, const float* cls, const float* truth, float width,
                        float height, float alpha, float beta, const int* labels, const unsigned char* sel,
                        const float* terms, const float* gout, float* dloc, float* dcls, hipStream_t s);
int launch_ssd_decode(int B, int n, int C, const float* loc, const float* cls, float conf, float nms_thr, int top_k,
                      int* keep, float* score, hipStream_t s);
int pw_tile_bm(int cfg);
int pw_tile_bn(int cfg);
int launch_pack_halo(const PackArgs& a, int nks, int bn, int ntiles, hipStream_t s);
// pipeline steps of a halo problem (= weight slices of its packed image): ntaps per k-step, the
// last k-step paired (ceil(ntaps / 2)) when half
__host__ __device__ inline int halo_steps(int nks, int ntaps, int half) {
  return half ? (nks - 1) * ntaps + (ntaps + 1) / 2 : nks * ntaps;
}
size_t halo_wp_bytes(int nks, int ntaps, int bn, int ntiles, int half);

}  // namespace tpg

// Weight-gradient kernel for gfx950: dW[a][b][r][s] += sum_p P[p][a] * Q[gather_t(p)][b].
//
//   Conv2d:           P = masked output grad g (output grid), Q = input x gathered at
//                     (oy*stride + r - pad) (zero / reflected outside)
//   ConvTranspose2d:  P = input x (input grid), Q = g gathered at (iy*stride + r - pad)
//   Linear/full conv: one tap, Q channels = flattened (y, x, c) of a dense NHWC image
//
// GEMM over K = pixels (N*H*W, up to 524288 at bs32 / 128^2): grid = (a-tile x b-tile,
// tap, split-K).  Each k-tile is 32 pixels; both operands arrive pixel-major (NHWC rows),
// are staged through LDS in that layout and read transposed:
//   bf16: ds_read_b64_tr_b16 gives a lane 4 consecutive pixels of one channel, two reads
//         form the 8-element k-fragment of v_mfma_f32_16x16x32_bf16
//   f32:  one ds_read_b32 per v_mfma_f32_16x16x4_f32 operand
// Split-K partials are added with no-return fp32 atomics into the caller's fp32 dW
// (lanes 0..15 hit 16 consecutive b, i.e. 64 contiguous bytes on a channels-last weight).
#include "tpg_internal.h"
#include <type_traits>

namespace tpg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ int refl(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// XOR swizzle of the 16-byte chunk index inside an LDS row (see header comment of the
// planner for the conflict analysis): bf16 rows read by ds_read_b64_tr_b16 take 8 rows
// {0..3, 8..11} per 32-lane half; f32 rows read by ds_read_b32 take 2 rows per half.
template <bool BF, int W>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BF) {
    if constexpr (W == 64) return chunk ^ (((((row >> 1) & 1) | (((row >> 3) & 1) << 1))) << 1);
    else return chunk ^ ((((row & 3) | (((row >> 3) & 1) << 2))) << 1);
  } else {
    return chunk ^ ((row & 1) << 2);
  }
}

template <int DT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradArgs p) {
  using E = dt_t<DT>;
  constexpr bool BF = DT != 0;
  constexpr int EPC = 16 / sizeof(E);
  constexpr int KP = 32;                  // pixels per k-tile
  constexpr int CPR_A = BM / EPC;         // 16-byte chunks per LDS row
  constexpr int CPR_B = BN / EPC;
  constexpr int LA = KP * CPR_A / 256;    // chunks staged per thread
  constexpr int LB = KP * CPR_B / 256;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  static_assert(LA >= 1 && LB >= 1, "tile too small");
  static_assert(WM * WN == 4, "4 waves");

  __shared__ __attribute__((aligned(16))) uint4 lds[2 * KP * (CPR_A + CPR_B)];
  __shared__ int8_t s_dy[TPG_MAX_TAPS], s_dx[TPG_MAX_TAPS];
  const int tid = threadIdx.x;
  if (tid < TPG_MAX_TAPS) { s_dy[tid] = p.dy[tid]; s_dx[tid] = p.dx[tid]; }

  const int nta = (p.Ca + BM - 1) / BM;
  const int ta = blockIdx.x % nta, tb = blockIdx.x / nta;
  const int a0 = ta * BM, b0 = tb * BN;
  const int tap = blockIdx.y;
  const int pbeg = blockIdx.z * p.pix_per_split;
  const int pend = min(p.npix, pbeg + p.pix_per_split);
  const E* Pg = reinterpret_cast<const E*>(p.P);
  const E* Qg = reinterpret_cast<const E*>(p.Q);
  const int PHPW = p.PH * p.PW;

  __syncthreads();
  const int dy = s_dy[tap], dx = s_dx[tap];

  uint4 ra[LA], rb[LB];
  uint32_t okA = 0, okB = 0;
  auto load_tile = [&](int p0) {
    okA = 0;
    okB = 0;
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      int idx = tid + 256 * q;
      int row = idx / CPR_A, ch = idx % CPR_A;
      int pix = p0 + row;
      int c = a0 + ch * EPC;
      const bool ok = pix < pend && c < p.Ca;
      int pp = ok ? pix : pbeg;
      int n = p.div_phpw.div(pp);
      int rem = pp - n * PHPW;
      int py = p.div_pw.div(rem);
      int px = rem - py * p.PW;
      const int64_t off = (int64_t)n * p.p_sn + (int64_t)py * p.p_sh + (int64_t)px * p.p_sw + c;
      okA |= (ok ? 1u : 0u) << q;
      if (p.vec_p) {
        ra[q] = *reinterpret_cast<const uint4*>(Pg + (ok ? off : 0));  // masked at store time
      } else {
        union { uint4 u; E e[EPC]; } t;
        t.u = make_uint4(0, 0, 0, 0);
        if (ok)
          for (int e = 0; e < EPC; ++e)
            if (c + e < p.Ca) t.e[e] = Pg[off + e];
        ra[q] = t.u;
      }
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      int idx = tid + 256 * q;
      int row = idx / CPR_B, ch = idx % CPR_B;
      int pix = p0 + row;
      int c = b0 + ch * EPC;
      bool ok = pix < pend && c < p.Cb;
      int pp = ok ? pix : pbeg;
      int n = p.div_phpw.div(pp);
      int rem = pp - n * PHPW;
      int py = p.div_pw.div(rem);
      int px = rem - py * p.PW;
      int qy = py * p.qst_h + dy, qx = px * p.qst_w + dx;
      if (p.pad_mode) { qy = refl(qy, p.QH); qx = refl(qx, p.QW); }
      ok = ok && (unsigned)qy < (unsigned)p.QH && (unsigned)qx < (unsigned)p.QW;
      const int64_t off = (int64_t)n * p.q_sn + (int64_t)qy * p.q_sh + (int64_t)qx * p.q_sw + c;
      okB |= (ok ? 1u : 0u) << q;
      if (p.vec_q) {
        rb[q] = *reinterpret_cast<const uint4*>(Qg + (ok ? off : 0));  // masked at store time
      } else {
        union { uint4 u; E e[EPC]; } t;
        t.u = make_uint4(0, 0, 0, 0);
        if (ok)
          for (int e = 0; e < EPC; ++e)
            if (c + e < p.Cb) t.e[e] = Qg[off + e];
        rb[q] = t.u;
      }
    }
  };

  auto store_tile = [&](int buf) {
    uint4* As = lds + buf * KP * (CPR_A + CPR_B);
    uint4* Bs = As + KP * CPR_A;
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      int idx = tid + 256 * q;
      int row = idx / CPR_A, ch = idx % CPR_A;
      uint4 v = ra[q];
      if (p.vec_p) {
        v = mask_chunk<EPC>(v, a0 + ch * EPC, p.Ca);
        if (!((okA >> q) & 1u)) v = make_uint4(0, 0, 0, 0);
      }
      As[row * CPR_A + swz<BF, BM>(row, ch)] = v;
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      int idx = tid + 256 * q;
      int row = idx / CPR_B, ch = idx % CPR_B;
      uint4 v = rb[q];
      if (p.vec_q) {
        v = mask_chunk<EPC>(v, b0 + ch * EPC, p.Cb);
        if (!((okB >> q) & 1u)) v = make_uint4(0, 0, 0, 0);
      }
      Bs[row * CPR_B + swz<BF, BN>(row, ch)] = v;
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, l16 = lane & 15;
  f32x4 acc[MREP][NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint4* As = lds + buf * KP * (CPR_A + CPR_B);
    const uint4* Bs = As + KP * CPR_A;
    if constexpr (BF) {
      // ds_read_b64_tr_b16: lane 4q+p4 of a 16-lane group addresses row q, columns 4p4..4p4+3
      const int q = l16 >> 2, p4 = l16 & 3;
      bf16x8 af[MREP], bfr[NREP];
#pragma unroll
      for (int m = 0; m < MREP; ++m) {
        const int col = wm * WTM + m * 16 + 4 * p4;
        s16x4 h[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int row = 8 * g + 4 * hh + q;
          const char* base = reinterpret_cast<const char*>(As + row * CPR_A + swz<BF, BM>(row, col >> 3));
          base += (col & 7) * 2;
          h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
        }
        af[m] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[0], h[1], 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        const int col = wn * WTN + n * 16 + 4 * p4;
        s16x4 h[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int row = 8 * g + 4 * hh + q;
          const char* base = reinterpret_cast<const char*>(Bs + row * CPR_B + swz<BF, BN>(row, col >> 3));
          base += (col & 7) * 2;
          h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
        }
        bfr[n] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h[0], h[1], 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int m = 0; m < MREP; ++m)
#pragma unroll
        for (int n = 0; n < NREP; ++n)
          acc[m][n] = mfma16x16x32<DT>(af[m], bfr[n], acc[m][n]);
    } else {
      const float* Af = reinterpret_cast<const float*>(As);
      const float* Bf = reinterpret_cast<const float*>(Bs);
#pragma unroll
      for (int kk = 0; kk < KP / 4; ++kk) {
        const int row = 4 * kk + g;
        float av[MREP], bv[NREP];
#pragma unroll
        for (int m = 0; m < MREP; ++m) {
          const int col = wm * WTM + m * 16 + l16;
          av[m] = Af[row * BM + swz<BF, BM>(row, col >> 2) * 4 + (col & 3)];
        }
#pragma unroll
        for (int n = 0; n < NREP; ++n) {
          const int col = wn * WTN + n * 16 + l16;
          bv[n] = Bf[row * BN + swz<BF, BN>(row, col >> 2) * 4 + (col & 3)];
        }
#pragma unroll
        for (int m = 0; m < MREP; ++m)
#pragma unroll
          for (int n = 0; n < NREP; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[n], acc[m][n], 0, 0, 0);
      }
    }
  };

  if (pbeg < pend) {
    load_tile(pbeg);
    store_tile(0);
    __syncthreads();
    int it = 0;
    for (int p0 = pbeg; p0 < pend; p0 += KP, ++it) {
      const int cur = it & 1;
      const bool more = p0 + KP < pend;
      if (more) load_tile(p0 + KP);
      compute(cur);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: fp32 atomics into dW
  const int r_tap = p.tr[tap], s_tap = p.ts[tap];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int a = a0 + wm * WTM + m * 16 + 4 * g + reg;
      if (a >= p.Ca) continue;
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        const int bq = b0 + wn * WTN + n * 16 + l16;
        if (bq >= p.Cb) continue;
        int r = r_tap, s = s_tap, b = bq;
        if (p.bcomp) {
          int rs = bq / p.comp_cb;
          b = bq - rs * p.comp_cb;
          r = rs / p.comp_kw;
          s = rs - r * p.comp_kw;
        }
        atomicAdd(p.dW + a * p.w_sa + b * p.w_sb + r * p.w_sr + s * p.w_ss, acc[m][n][reg]);
      }
    }
}

#define TPG_WGRAD_CFGS(X) \
  X(0, 64, 64, 2, 2)      \
  X(1, 128, 128, 2, 2)

int wgrad_cfg_bm(int cfg) {
#define X(id, bm, bn, wm, wn) if (cfg == id) return bm;
  TPG_WGRAD_CFGS(X)
#undef X
  return -1;
}
int wgrad_cfg_bn(int cfg) {
#define X(id, bm, bn, wm, wn) if (cfg == id) return bn;
  TPG_WGRAD_CFGS(X)
#undef X
  return -1;
}

int launch_wgrad(const WgradArgs& a, int dtype, int cfg, hipStream_t s) {
  const int bm = wgrad_cfg_bm(cfg), bn = wgrad_cfg_bn(cfg);
  if (bm < 0) return -1;
  dim3 grid(((a.Ca + bm - 1) / bm) * ((a.Cb + bn - 1) / bn), a.ntaps, a.ksplit);
#define X(id, BM_, BN_, WM_, WN_)                                                               \
  if (cfg == id) {                                                                              \
    if (dtype == 1) hipLaunchKernelGGL((wgrad_kernel<1, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a);      \
    else if (dtype == 2) hipLaunchKernelGGL((wgrad_kernel<2, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((wgrad_kernel<0, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a);                 \
  }
  TPG_WGRAD_CFGS(X)
#undef X
  return (int)hipGetLastError();
}

}  // namespace tpg

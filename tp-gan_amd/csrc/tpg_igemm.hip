// Tap-table implicit-GEMM convolution for gfx950 (CDNA4), NHWC activations.
//
// One kernel family covers every conv-shaped op of the TP-GAN hot path
// (SURVEY.md §2 op-class table):
//   Conv2d forward                 rows = output pixels, taps = (r - pad) offsets, input stride s
//   Conv2d input gradient          rows = one parity class of input pixels, taps = the kernel
//                                  positions that reach that class (sub-pixel decomposition)
//   ConvTranspose2d forward        same as the Conv2d input gradient
//   ConvTranspose2d input gradient same as the Conv2d forward
//   Linear / full-kernel conv      one tap, channels = flattened (y, x, c)
//
// GEMM view: Out[row][n'] = sum_{tap, c} A[pix(row, tap)][c] * Wp[n'][tap][c].
// K is walked in 16-channel units of one tap; one k-tile = 128 bytes per row
// (bf16: 4 units = 64 k, f32: 2 units = 32 k).  A rows are gathered from HBM into
// registers (zero outside the image, or reflected), staged through a double-buffered,
// XOR-swizzled LDS image; weights are pre-packed [n'][unit][16] so their tile rows are
// contiguous 128-byte lines.
//
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16; f32 (parity mode) -> v_mfma_f32_16x16x4_f32
// (exact f32 FMA chain).  Both read one 16-byte LDS chunk per lane per operand: lane l
// holds row (l & 15), chunk (4s + (l >> 4)); the f32 form issues 4 MFMAs over the chunk's
// 4 elements, so A and B agree on the k permutation and the sum is over all of K.
//
// Epilogue (fused): + bias, + res_scale * residual, LeakyReLU / ReLU, dtype convert,
// store into any (n, h, w) strided NHWC view (a channel slice implements zero-copy
// output into a concat buffer).  Split-K blocks atomically add fp32 partials into a work
// space instead; tpg_epilogue_kernel finishes them.
#include "tpg_internal.h"
#include <type_traits>
#include <algorithm>
#include <string.h>

namespace tpg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float act_apply(float v, int act, float slope) { return tpg_act(v, act, slope); }

template <typename E>
__device__ __forceinline__ float ld_f(const E* p) { return (float)(*p); }

template <typename E>
__device__ __forceinline__ void st_f(E* p, float v) { *p = (E)v; }

__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

template <int DT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void igemm_kernel(const IgemmArgs p) {
  using E = dt_t<DT>;
  constexpr bool BF = DT != 0;
  constexpr int EPC = 16 / sizeof(E);      // elements per 16-byte chunk
  constexpr int CPU = 16 / EPC;            // chunks per 16-channel unit
  constexpr int UPK = 8 / CPU;             // units per 128-byte k-tile
  constexpr int RA = BM / 32;              // A rows staged per thread
  constexpr int RB = (BN + 31) / 32;       // B rows staged per thread
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MREP = WTM / 16, NREP = WTN / 16;
  static_assert(MREP * 16 * WM == BM && NREP * 16 * WN == BN, "tile");
  static_assert(WM * WN == 4, "4 waves");

  __shared__ __attribute__((aligned(16))) uint4 lds[2 * (BM + BN) * 8];
  __shared__ int8_t s_dy[TPG_MAX_TAPS], s_dx[TPG_MAX_TAPS];

  const int tid = threadIdx.x;
  if (tid < TPG_MAX_TAPS) { s_dy[tid] = p.dy[tid]; s_dx[tid] = p.dx[tid]; }

  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nkt = p.nunits / UPK;
  int kt0 = blockIdx.z * p.kt_per_split;
  int kt1 = min(nkt, kt0 + p.kt_per_split);

  // ---- per-thread staging geometry
  const int chunk = tid & 7;
  const int rsub = tid >> 3;
  const int slot = chunk / CPU;
  const int part = chunk % CPU;
  const E* Ag = reinterpret_cast<const E*>(p.A);
  int64_t a_base[RA];
  int by[RA], bx[RA];
  bool rv[RA];
  const int JHJW = p.JH * p.JW;
#pragma unroll
  for (int q = 0; q < RA; ++q) {
    int row = m0 + rsub + 32 * q;
    rv[q] = row < p.M;
    int rr = rv[q] ? row : 0;
    int n = p.div_jhjw.div(rr);
    int rem = rr - n * JHJW;
    int j = p.div_jw.div(rem);
    int i = rem - j * p.JW;
    a_base[q] = (int64_t)n * p.a_sn;
    by[q] = j * p.ist_h;
    bx[q] = i * p.ist_w;
  }
  const E* Wg = reinterpret_cast<const E*>(p.Wp);
  const int64_t wrow = (int64_t)p.nunits * 16;

  uint4 ra[RA], rb[RB];
  int a_c = 0;
  uint32_t a_ok = 0;
  int tap = 0, cu = 0;
  {
    int u = kt0 * UPK + slot;
    tap = u / p.upt;
    cu = u - tap * p.upt;
  }

  auto load_tile = [&](int kt) {
    // A gather
    const int c = cu * 16 + part * EPC;
    const bool tap_ok = tap < p.ntaps;
    const int dy = tap_ok ? s_dy[tap] : 0;
    const int dx = tap_ok ? s_dx[tap] : 0;
    a_c = c;
    a_ok = 0;
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      int iy = by[q] + dy, ix = bx[q] + dx;
      if (p.pad_mode) { iy = reflect_idx(iy, p.A_H); ix = reflect_idx(ix, p.A_W); }
      const bool ok = tap_ok && rv[q] && (unsigned)iy < (unsigned)p.A_H && (unsigned)ix < (unsigned)p.A_W && c < p.C;
      const int64_t off = a_base[q] + (int64_t)iy * p.a_sh + (int64_t)ix * p.a_sw + c;
      a_ok |= (ok ? 1u : 0u) << q;
      if (p.vec_ok) {
        ra[q] = *reinterpret_cast<const uint4*>(Ag + (ok ? off : 0));  // masked at store time
      } else {
        union { uint4 u; E e[EPC]; } t;
        t.u = make_uint4(0, 0, 0, 0);
        if (ok)
          for (int e = 0; e < EPC; ++e)
            if (c + e < p.C) t.e[e] = Ag[off + e];
        ra[q] = t.u;
      }
    }
    // B (packed weights, always in range)
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      int nr = rsub + 32 * q;
      if (nr < BN) {
        const E* src = Wg + (int64_t)(n0 + nr) * wrow + (int64_t)kt * (UPK * 16) + chunk * EPC;
        rb[q] = *reinterpret_cast<const uint4*>(src);
      }
    }
    // advance unit cursor by one k-tile
    cu += UPK;
    while (cu >= p.upt) { cu -= p.upt; ++tap; }
  };

  auto store_tile = [&](int buf) {
    uint4* As = lds + buf * (BM + BN) * 8;
    uint4* Bs = As + BM * 8;
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      int r = rsub + 32 * q;
      uint4 v = ra[q];
      if (p.vec_ok) {
        v = mask_chunk<EPC>(v, a_c, p.C);
        if (!((a_ok >> q) & 1u)) v = make_uint4(0, 0, 0, 0);
      }
      As[r * 8 + (chunk ^ ((r >> 1) & 7))] = v;
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      int r = rsub + 32 * q;
      if (r < BN) Bs[r * 8 + (chunk ^ ((r >> 1) & 7))] = rb[q];
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, g = lane >> 4;
  f32x4 acc[MREP][NREP];
#pragma unroll
  for (int m = 0; m < MREP; ++m)
#pragma unroll
    for (int n = 0; n < NREP; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint4* As = lds + buf * (BM + BN) * 8;
    const uint4* Bs = As + BM * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 af[MREP], bfr[NREP];
      const int ch = 4 * s + g;
#pragma unroll
      for (int m = 0; m < MREP; ++m) {
        int r = wm * WTM + m * 16 + r16;
        af[m] = As[r * 8 + (ch ^ ((r >> 1) & 7))];
      }
#pragma unroll
      for (int n = 0; n < NREP; ++n) {
        int r = wn * WTN + n * 16 + r16;
        bfr[n] = Bs[r * 8 + (ch ^ ((r >> 1) & 7))];
      }
#pragma unroll
      for (int m = 0; m < MREP; ++m)
#pragma unroll
        for (int n = 0; n < NREP; ++n) {
          if constexpr (BF) {
            acc[m][n] = mfma16x16x32<DT>(af[m], bfr[n], acc[m][n]);
          } else {
            f32x4 a4 = __builtin_bit_cast(f32x4, af[m]);
            f32x4 b4 = __builtin_bit_cast(f32x4, bfr[n]);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], acc[m][n], 0, 0, 0);
          }
        }
    }
  };

  __syncthreads();  // tap table visible
  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      compute(cur);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue
  E* Y = reinterpret_cast<E*>(p.Y);
  const E* R = reinterpret_cast<const E*>(p.R);
#pragma unroll
  for (int m = 0; m < MREP; ++m) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = m0 + wm * WTM + m * 16 + 4 * g + reg;
      if (row >= p.M) continue;
      int n = p.div_jhjw.div(row);
      int rem = row - n * JHJW;
      int j = p.div_jw.div(rem);
      int i = rem - j * p.JW;
      int oy = p.oy0 + p.osy * j, ox = p.ox0 + p.osx * i;
      int64_t yoff = (int64_t)n * p.y_sn + (int64_t)oy * p.y_sh + (int64_t)ox * p.y_sw;
      int64_t roff = (int64_t)n * p.r_sn + (int64_t)oy * p.r_sh + (int64_t)ox * p.r_sw;
#pragma unroll
      for (int nr = 0; nr < NREP; ++nr) {
        const int col = n0 + wn * WTN + nr * 16 + r16;
        if (col >= p.Nout) continue;
        float v = acc[m][nr][reg];
        if (p.ws) {
          atomicAdd(p.ws + (int64_t)row * p.Nout + col, v);
        } else {
          if (p.bias) v += p.bias[p.bias_mod ? col % p.bias_mod : col];
          if (R) v += p.res_scale * ld_f(R + roff + col);
          st_f(Y + yoff + col, act_apply(v, p.act, p.slope));
        }
      }
    }
  }
}

// Split-K finalize: v = sum of the partial slices (+ bias, + residual, activation).
// V columns per thread (4 when Nout % 4 == 0: 16-byte slice reads).
template <typename E, int V, int NG = 1>
__global__ __launch_bounds__(256) void epilogue_kernel(const Grouped<EpiArgs, NG> G) {
  int mem = 0;
  int64_t b0 = blockIdx.x, nb = gridDim.x;
  if constexpr (NG > 1) {  // grouped: member blocks [boff[m], boff[m + 1])
    mem = group_member(G, blockIdx.x);
    b0 = blockIdx.x - G.boff[mem];
    nb = G.boff[mem + 1] - G.boff[mem];
  }
  const EpiArgs& p = G.a[mem];
  const int64_t total = (int64_t)p.M * p.Nout / V;
  const int JHJW = p.JH * p.JW;
  E* Y = reinterpret_cast<E*>(p.Y);
  const E* R = reinterpret_cast<const E*>(p.R);
  const E* XA = reinterpret_cast<const E*>(p.XA);  // (desc.in_act: Y's offsets)
  const bool small = (int64_t)p.M * p.Nout < (1ll << 31);  // 32-bit index math (uniform)
  for (int64_t idx = b0 * blockDim.x + threadIdx.x; idx < total; idx += nb * blockDim.x) {
    const int64_t e0 = idx * V;
    int row, col;
    if (small) {
      row = (int)e0 / p.Nout;
      col = (int)e0 - row * p.Nout;
    } else {
      row = (int)(e0 / p.Nout);
      col = (int)(e0 - (int64_t)row * p.Nout);
    }
    int n = row / JHJW;
    int rem = row - n * JHJW;
    int j = rem / p.JW, i = rem - j * p.JW;
    int oy = p.oy0 + p.osy * j, ox = p.ox0 + p.osx * i;
    float v[V];
    // slices summed in order z = 0, 1, ... (deterministic), their loads issued four at a time:
    // one at a time, every slice exposed a full memory latency (a k split of 8 -> ~8 of them)
    if constexpr (V == 4) {
      const float* src = p.ws + e0;
      float4 a = *reinterpret_cast<const float4*>(src);
      int z = 1;
      for (; z + 3 < p.nslices; z += 4) {
        float4 b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(src + (z + u) * p.slice);
#pragma unroll
        for (int u = 0; u < 4; ++u) { a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w; }
      }
      for (; z < p.nslices; ++z) {
        const float4 b = *reinterpret_cast<const float4*>(src + z * p.slice);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else {
      const float* src = p.ws + e0;
      float a = src[0];
      int z = 1;
      for (; z + 3 < p.nslices; z += 4) {
        float b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = src[(z + u) * p.slice];
#pragma unroll
        for (int u = 0; u < 4; ++u) a += b[u];
      }
      for (; z < p.nslices; ++z) a += src[z * p.slice];
      v[0] = a;
    }
    const int64_t yo = (int64_t)n * p.y_sn + (int64_t)oy * p.y_sh + (int64_t)ox * p.y_sw + col;
    const int64_t ro = (int64_t)n * p.r_sn + (int64_t)oy * p.r_sh + (int64_t)ox * p.r_sw + col;
    if constexpr (V == 4 && sizeof(E) == 2) {
      // four 16-bit outputs as one 8-byte store (and an 8-byte residual load) when aligned
      // (the four halves are taken apart as scalars: this hipcc compiles
      // __builtin_bit_cast(E, vec[u]) of an ext_vector element as element 0 for every u --
      // the parked round-3 version of this path read the first residual four times)
      // (the base pointers too: a channel-offset view through the public C API may start on
      // any 2-byte boundary)
      if (((yo | (R ? ro : 0)) & 3) == 0 && (((uintptr_t)Y | (uintptr_t)R | (uintptr_t)XA) & 7) == 0) {
        uint2 rw = make_uint2(0u, 0u), xw = make_uint2(0u, 0u);
        if (R) rw = *reinterpret_cast<const uint2*>(R + ro);
        if (XA) xw = *reinterpret_cast<const uint2*>(XA + yo);
        uint32_t ow[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t w = h ? rw.y : rw.x;
          const uint32_t xh = h ? xw.y : xw.x;
          uint32_t packed = 0;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int u = 2 * h + e;
            float x = v[u];
            if (p.bias) x += p.bias[p.bias_mod ? (col + u) % p.bias_mod : col + u];
            if (R) {
              const unsigned short r16 = (unsigned short)(e ? (w >> 16) : (w & 0xffffu));
              x += p.res_scale * (float)__builtin_bit_cast(E, r16);
            }
            E o;
            if (XA) {
              const unsigned short x16 = (unsigned short)(e ? (xh >> 16) : (xh & 0xffffu));
              o = (E)tpg_xa_grad(x, (float)__builtin_bit_cast(E, x16), p.xa_act, p.xa_slope);
            } else {
              o = (E)act_apply(x, p.act, p.slope);
            }
            const unsigned short o16 = __builtin_bit_cast(unsigned short, o);
            packed |= (uint32_t)o16 << (16 * e);
          }
          ow[h] = packed;
        }
        *reinterpret_cast<uint2*>(Y + yo) = make_uint2(ow[0], ow[1]);
        continue;
      }
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      float x = v[u];
      if (p.bias) x += p.bias[p.bias_mod ? (col + u) % p.bias_mod : col + u];
      if (R) x += p.res_scale * ld_f(R + ro + u);
      st_f(Y + yo + u, XA ? tpg_xa_grad(x, ld_f(XA + yo + u), p.xa_act, p.xa_slope)
                          : act_apply(x, p.act, p.slope));
    }
  }
}

// tile configurations: {BM, BN, WM, WN}
#define TPG_IGEMM_CFGS(X)   \
  X(0, 128, 16, 4, 1)       \
  X(1, 128, 32, 4, 1)       \
  X(2, 128, 64, 2, 2)       \
  X(3, 128, 96, 4, 1)       \
  X(4, 128, 128, 2, 2)      \
  X(5, 128, 224, 2, 2)

int igemm_cfg_bn(int cfg) {
#define X(id, bm, bn, wm, wn) if (cfg == id) return bn;
  TPG_IGEMM_CFGS(X)
#undef X
  return -1;
}
int igemm_cfg_bm(int cfg) {
#define X(id, bm, bn, wm, wn) if (cfg == id) return bm;
  TPG_IGEMM_CFGS(X)
#undef X
  return -1;
}

int launch_igemm(const IgemmArgs& a, int dtype, int cfg, hipStream_t s) {
  const int bm = igemm_cfg_bm(cfg), bn = igemm_cfg_bn(cfg);
  if (bm < 0) return -1;
  dim3 grid((a.M + bm - 1) / bm, (a.Nout + bn - 1) / bn, a.ksplit);
#define X(id, BM_, BN_, WM_, WN_)                                                              \
  if (cfg == id) {                                                                             \
    if (dtype == 1) hipLaunchKernelGGL((igemm_kernel<1, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a);      \
    else if (dtype == 2) hipLaunchKernelGGL((igemm_kernel<2, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((igemm_kernel<0, BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, a);                 \
  }
  TPG_IGEMM_CFGS(X)
#undef X
  return (int)hipGetLastError();
}

static bool epi_v4(const EpiArgs& a) { return a.Nout % 4 == 0 && ((uintptr_t)a.ws % 16) == 0 && a.slice % 4 == 0; }
static int epi_blocks(const EpiArgs& a, bool v4) {
  const int64_t total = (int64_t)a.M * a.Nout / (v4 ? 4 : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
}

template <typename E, int NG>
static void launch_epi_t(const Grouped<EpiArgs, NG>& g, bool v4, int blocks, hipStream_t s) {
  if (v4) hipLaunchKernelGGL((epilogue_kernel<E, 4, NG>), dim3(blocks), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((epilogue_kernel<E, 1, NG>), dim3(blocks), dim3(256), 0, s, g);
}

int launch_epilogue(const EpiArgs& a, hipStream_t s) {
  const bool v4 = epi_v4(a);
  const int blocks = epi_blocks(a, v4);
  Grouped<EpiArgs, 1> g;
  g.a[0] = a; g.boff[0] = 0; g.boff[1] = blocks; g.nm = 1;
  if (a.dtype == 2) launch_epi_t<_Float16, 1>(g, v4, blocks, s);
  else if (a.dtype == 1) launch_epi_t<__bf16, 1>(g, v4, blocks, s);
  else launch_epi_t<float, 1>(g, v4, blocks, s);
  return (int)hipGetLastError();
}

int launch_epilogue_group(const EpiArgs* a, int n, hipStream_t s) {
  if (n < 2 || n > TPG_GROUP_MAX || (a[0].dtype != 1 && a[0].dtype != 2)) return -1;
  const bool v4 = epi_v4(a[0]);
  Grouped<EpiArgs, TPG_GROUP_MAX> g;
  memset(&g, 0, sizeof(g));
  int blocks = 0;
  for (int m = 0; m < n; ++m) {
    if (a[m].dtype != a[0].dtype || epi_v4(a[m]) != v4) return -1;
    g.a[m] = a[m];
    g.boff[m] = blocks;
    blocks += epi_blocks(a[m], v4);
  }
  g.boff[n] = blocks;
  g.nm = n;
  if (a[0].dtype == 2) launch_epi_t<_Float16, TPG_GROUP_MAX>(g, v4, blocks, s);
  else launch_epi_t<__bf16, TPG_GROUP_MAX>(g, v4, blocks, s);
  return (int)hipGetLastError();
}

}  // namespace tpg

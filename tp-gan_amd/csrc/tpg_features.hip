// Identity-feature extractor kernels (gfx950): the ops MobileNetV2 / ResNet add on top of
// the dense conv family — depthwise 3x3 convolution (MobileNetV2.py:105, groups = C)
// forward / input gradient / weight gradient, MaxPool2d(3, 2, 1) (ResNet.py:33) forward
// and backward with a u8 window argmax, global average pooling (AdaptiveAvgPool2d(1),
// MobileNetV2.py:173 / ResNet.py:45) and the eval-mode BatchNorm fold into the preceding
// conv (MobileNetV2.py:100-112: w' = w * g / sqrt(v + eps), b' = beta - m * g / sqrt(v + eps)).
//
// All of them are HBM-bound (a 3x3 depthwise conv does 9 MACs per 4 bytes moved in bf16):
// channels-last tensors, one thread per 16-byte channel chunk walking a contiguous pixel
// range, so a thread's weights (9 taps x 8 channels) stay in registers and every wave reads
// whole 16-byte chunks of consecutive pixels; neighbouring taps hit L2.
#include "tpg_internal.h"
#include "../../include/tpgan.h"
#include <string.h>
#include <algorithm>

namespace tpg {

template <typename E>
struct Chunk {
  static constexpr int EPC = 16 / sizeof(E);
  union { uint4 u; E e[EPC]; };
};

template <typename E>
__device__ __forceinline__ void load_chunk(const E* p, float* v) {
  Chunk<E> c;
  c.u = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int e = 0; e < Chunk<E>::EPC; ++e) v[e] = (float)c.e[e];
}

template <typename E>
__device__ __forceinline__ void store_chunk(E* p, const float* v) {
  Chunk<E> c;
#pragma unroll
  for (int e = 0; e < Chunk<E>::EPC; ++e) c.e[e] = (E)v[e];
  *reinterpret_cast<uint4*>(p) = c.u;
}

struct DwArgs {
  int N, C, H, W, OH, OW, kh, kw, sh, sw, pt, pl;
  int64_t x_sn, x_sh, x_sw;    // element strides of the input-grid tensor (x or dx)
  int64_t y_sn, y_sh, y_sw;    // element strides of the output-grid tensor (y or g)
  int64_t r_sn, r_sh, r_sw;
  const float* w;              // [C][kh][kw] after the host gathers strides (w_sc, w_sr, w_ss)
  int64_t w_sc, w_sr, w_ss;
  const float* bias;
  int act;
  float slope;
  float res_scale;
  int64_t pix_per_block;
};

// y[n,oy,ox,c] = act(sum_t x[n, oy*sh - pt + r, ox*sw - pl + s, c] * w[c,r,s] + b[c] + res)
template <typename E>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const DwArgs a, const E* __restrict__ x, E* __restrict__ y,
                                                     const E* __restrict__ res) {
  constexpr int EPC = Chunk<E>::EPC;
  const int cg0 = blockIdx.y * 256;                               // first chunk of this channel group
  const int nch = min(256, (a.C + EPC - 1) / EPC - cg0);
  if (nch <= 0) return;  // block-uniform: surplus channel group (grid sized for the fp32 chunk count)
  const int ppi = 256 / nch;
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  if (pl >= ppi) return;
  const int c0 = (cg0 + ch) * EPC;
  const int ntaps = a.kh * a.kw;
  float wr[9][EPC], bv[EPC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int c = c0 + e;
      wr[t][e] = (t < ntaps && c < a.C) ? a.w[c * a.w_sc + (t / a.kw) * a.w_sr + (t % a.kw) * a.w_ss] : 0.f;
    }
#pragma unroll
  for (int e = 0; e < EPC; ++e) bv[e] = (a.bias && c0 + e < a.C) ? a.bias[c0 + e] : 0.f;
  const int64_t npix = (int64_t)a.N * a.OH * a.OW;
  const int64_t p0 = (int64_t)blockIdx.x * a.pix_per_block;
  const int64_t p1 = min(p0 + a.pix_per_block, npix);
  for (int64_t pix = p0 + pl; pix < p1; pix += ppi) {
    const int n = (int)(pix / (a.OH * a.OW));
    const int rem = (int)(pix - (int64_t)n * a.OH * a.OW);
    const int oy = rem / a.OW, ox = rem - oy * a.OW;
    float acc[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = bv[e];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * a.sh - a.pt + t / a.kw, ix = ox * a.sw - a.pl + t % a.kw;
      if (t < ntaps && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
        float v[EPC];
        load_chunk(x + n * a.x_sn + iy * a.x_sh + ix * a.x_sw + c0, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) acc[e] += v[e] * wr[t][e];
      }
    }
    if (res) {
      float rv[EPC];
      load_chunk(res + n * a.r_sn + oy * a.r_sh + ox * a.r_sw + c0, rv);
#pragma unroll
      for (int e = 0; e < EPC; ++e) acc[e] += a.res_scale * rv[e];
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = (c0 + e < a.C) ? tpg_act(acc[e], a.act, a.slope) : 0.f;
    store_chunk(y + n * a.y_sn + oy * a.y_sh + ox * a.y_sw + c0, acc);
  }
}

// dx[n,iy,ix,c] = sum over taps (r,s) with oy = (iy + pt - r) / sh integral and in range
template <typename E>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const DwArgs a, const E* __restrict__ g, E* __restrict__ dx) {
  constexpr int EPC = Chunk<E>::EPC;
  const int cg0 = blockIdx.y * 256;                               // first chunk of this channel group
  const int nch = min(256, (a.C + EPC - 1) / EPC - cg0);
  if (nch <= 0) return;  // block-uniform: surplus channel group (grid sized for the fp32 chunk count)
  const int ppi = 256 / nch;
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  if (pl >= ppi) return;
  const int c0 = (cg0 + ch) * EPC;
  const int ntaps = a.kh * a.kw;
  float wr[9][EPC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int c = c0 + e;
      wr[t][e] = (t < ntaps && c < a.C) ? a.w[c * a.w_sc + (t / a.kw) * a.w_sr + (t % a.kw) * a.w_ss] : 0.f;
    }
  const int64_t npix = (int64_t)a.N * a.H * a.W;
  const int64_t p0 = (int64_t)blockIdx.x * a.pix_per_block;
  const int64_t p1 = min(p0 + a.pix_per_block, npix);
  for (int64_t pix = p0 + pl; pix < p1; pix += ppi) {
    const int n = (int)(pix / (a.H * a.W));
    const int rem = (int)(pix - (int64_t)n * a.H * a.W);
    const int iy = rem / a.W, ix = rem - iy * a.W;
    float acc[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ny = iy + a.pt - t / a.kw, nx = ix + a.pl - t % a.kw;
      const int oy = ny / a.sh, ox = nx / a.sw;
      if (t < ntaps && ny >= 0 && nx >= 0 && ny - oy * a.sh == 0 && nx - ox * a.sw == 0 && oy < a.OH && ox < a.OW) {
        float v[EPC];
        load_chunk(g + n * a.y_sn + oy * a.y_sh + ox * a.y_sw + c0, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) acc[e] += v[e] * wr[t][e];
      }
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = (c0 + e < a.C) ? acc[e] : 0.f;
    store_chunk(dx + n * a.x_sn + iy * a.x_sh + ix * a.x_sw + c0, acc);
  }
}

// dw[c,r,s] += sum over output pixels of g[n,oy,ox,c] * x[n, oy*sh - pt + r, ox*sw - pl + s, c]
// Per-thread partials for all taps in registers, block reduction through LDS one tap at
// a time, one fp32 atomic per (c, tap) per block (<= 256 blocks).
template <typename E>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const DwArgs a, const E* __restrict__ x, const E* __restrict__ g,
                                                       float* __restrict__ dw) {
  constexpr int EPC = Chunk<E>::EPC;
  __shared__ float sb[256 * EPC];
  const int cg0 = blockIdx.y * 256;                               // first chunk of this channel group
  const int nch = min(256, (a.C + EPC - 1) / EPC - cg0);
  if (nch <= 0) return;  // block-uniform: surplus channel group (grid sized for the fp32 chunk count)
  const int ppi = 256 / nch;
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  const bool active = pl < ppi;
  const int c0 = (cg0 + ch) * EPC;
  const int ntaps = a.kh * a.kw;
  float part[9][EPC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < EPC; ++e) part[t][e] = 0.f;
  const int64_t npix = (int64_t)a.N * a.OH * a.OW;
  const int64_t p0 = (int64_t)blockIdx.x * a.pix_per_block;
  const int64_t p1 = min(p0 + a.pix_per_block, npix);
  if (active) {
    for (int64_t pix = p0 + pl; pix < p1; pix += ppi) {
      const int n = (int)(pix / (a.OH * a.OW));
      const int rem = (int)(pix - (int64_t)n * a.OH * a.OW);
      const int oy = rem / a.OW, ox = rem - oy * a.OW;
      float gv[EPC];
      load_chunk(g + n * a.y_sn + oy * a.y_sh + ox * a.y_sw + c0, gv);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = oy * a.sh - a.pt + t / a.kw, ix = ox * a.sw - a.pl + t % a.kw;
        if (t < ntaps && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
          float v[EPC];
          load_chunk(x + n * a.x_sn + iy * a.x_sh + ix * a.x_sw + c0, v);
#pragma unroll
          for (int e = 0; e < EPC; ++e) part[t][e] += v[e] * gv[e];
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    if (t < ntaps) {  // block-uniform
      if (active)
#pragma unroll
        for (int e = 0; e < EPC; ++e) sb[pl * nch * EPC + ch * EPC + e] = part[t][e];
      __syncthreads();
      for (int cl = threadIdx.x; cl < nch * EPC; cl += 256) {
        const int c = cg0 * EPC + cl;
        if (c >= a.C) continue;
        float s = 0.f;
        for (int q = 0; q < ppi; ++q) s += sb[q * nch * EPC + cl];
        atomicAdd(dw + c * a.w_sc + (t / a.kw) * a.w_sr + (t % a.kw) * a.w_ss, s);
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------- MaxPool2d --
// y = max over the k x k window (padding never wins: -inf), argmax = first tap index r*k+s
// attaining it (torch's CPU/GPU kernels also keep the first maximum in scan order).
template <typename E>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int N, int C, int H, int W, int OH, int OW, int k, int s,
                                                          int p, const E* __restrict__ x, int64_t x_sn, int64_t x_sh,
                                                          int64_t x_sw, E* __restrict__ y, int64_t y_sn,
                                                          int64_t y_sh, int64_t y_sw, uint8_t* __restrict__ amax) {
  const int64_t total = (int64_t)N * OH * OW * C;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t pix = idx / C;
    const int ox = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int oy = (int)(t % OH), n = (int)(t / OH);
    float best = -INFINITY;
    int arg = 0;
    for (int r = 0; r < k; ++r)
      for (int q = 0; q < k; ++q) {
        const int iy = oy * s - p + r, ix = ox * s - p + q;
        if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) continue;
        const float v = (float)x[n * x_sn + iy * x_sh + ix * x_sw + c];
        if (v > best || (v != v && best == best)) { best = v; arg = r * k + q; }
      }
    y[n * y_sn + oy * y_sh + ox * y_sw + c] = (E)best;
    amax[idx] = (uint8_t)arg;
  }
}

// gather form: dx[iy,ix,c] = sum of gy over the windows that chose (iy, ix)
template <typename E>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int N, int C, int H, int W, int OH, int OW, int k, int s,
                                                          int p, const E* __restrict__ gy, int64_t g_sn, int64_t g_sh,
                                                          int64_t g_sw, const uint8_t* __restrict__ amax,
                                                          E* __restrict__ dx, int64_t x_sn, int64_t x_sh,
                                                          int64_t x_sw) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t pix = idx / C;
    const int ix = (int)(pix % W);
    const int64_t t = pix / W;
    const int iy = (int)(t % H), n = (int)(t / H);
    float acc = 0.f;
    for (int r = 0; r < k; ++r) {
      const int ny = iy + p - r;
      if (ny < 0 || ny % s) continue;
      const int oy = ny / s;
      if (oy >= OH) continue;
      for (int q = 0; q < k; ++q) {
        const int nx = ix + p - q;
        if (nx < 0 || nx % s) continue;
        const int ox = nx / s;
        if (ox >= OW) continue;
        const int64_t o = (((int64_t)n * OH + oy) * OW + ox) * C + c;
        if (amax[o] == r * k + q) acc += (float)gy[n * g_sn + oy * g_sh + ox * g_sw + c];
      }
    }
    dx[n * x_sn + iy * x_sh + ix * x_sw + c] = (E)acc;
  }
}

// ------------------------------------------------------------ global average pool --
// y[n, c] = mean over H x W (one thread per (n, c), pixels walked in order: deterministic)
template <typename E>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int N, int C, int H, int W, const E* __restrict__ x,
                                                          int64_t x_sn, int64_t x_sh, int64_t x_sw,
                                                          E* __restrict__ y, int64_t y_sn) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= N * C) return;
  const int n = idx / C, c = idx - n * C;
  float s = 0.f;
  for (int iy = 0; iy < H; ++iy)
    for (int ix = 0; ix < W; ++ix) s += (float)x[n * x_sn + iy * x_sh + ix * x_sw + c];
  y[n * y_sn + c] = (E)(s / (float)(H * W));
}

template <typename E>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int N, int C, int H, int W, const E* __restrict__ gy,
                                                          int64_t g_sn, E* __restrict__ dx, int64_t x_sn,
                                                          int64_t x_sh, int64_t x_sw) {
  const int64_t total = (int64_t)N * H * W * C;
  const float inv = 1.f / (float)(H * W);
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t pix = idx / C;
    const int ix = (int)(pix % W);
    const int64_t t = pix / W;
    const int iy = (int)(t % H), n = (int)(t / H);
    dx[n * x_sn + iy * x_sh + ix * x_sw + c] = (E)((float)gy[n * g_sn + c] * inv);
  }
}

// ------------------------------------------------------------------ BatchNorm fold --
// w_out[o][i][r][s] = w[o][i][r][s] * sc[o], b_out[o] = (b0[o] - mean[o]) * sc[o] + beta[o],
// sc[o] = gamma[o] / sqrt(var[o] + eps)  (nn.BatchNorm2d eval: (x - m) / sqrt(v + eps) * g + beta)
__global__ __launch_bounds__(256) void bn_fold_kernel(int O, int I, int KH, int KW, tpg_tensor w, const float* b0,
                                                      const float* gamma, const float* beta, const float* mean,
                                                      const float* var, float eps, tpg_tensor wo, float* bo) {
  const int64_t total = (int64_t)O * I * KH * KW;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(idx % KW);
    int64_t t = idx / KW;
    const int r = (int)(t % KH);
    t /= KH;
    const int i = (int)(t % I);
    const int o = (int)(t / I);
    const float sc = gamma[o] / sqrtf(var[o] + eps);
    const float* wp = reinterpret_cast<const float*>(w.data);
    float* wop = reinterpret_cast<float*>(wo.data);
    wop[o * wo.stride[0] + i * wo.stride[1] + r * wo.stride[2] + s * wo.stride[3]] =
        wp[o * w.stride[0] + i * w.stride[1] + r * w.stride[2] + s * w.stride[3]] * sc;
    if (idx < O) {
      const int oo = (int)idx;
      const float sco = gamma[oo] / sqrtf(var[oo] + eps);
      bo[oo] = ((b0 ? b0[oo] : 0.f) - mean[oo]) * sco + beta[oo];
    }
  }
}


// ----------------------------------------------------------- BatchNorm2d (training) --
// Batch statistics over N*H*W per channel (nn.BatchNorm2d train mode, MobileNetV2.py:
// 101-112): two-pass mean / biased variance for normalisation, unbiased variance into the
// running estimate (momentum), the activation fused into the normalise pass; backward
// recomputes g = act'(y) * dy on the fly.  Per-channel sums: one thread per 16-byte chunk
// walking a contiguous pixel range, block partials combined in LDS, one fp32 atomic per
// channel per block (<= 512 blocks).
struct BnArgs {
  int64_t npix;
  int C, act;
  float slope, eps, momentum;
  const void* x; int64_t x_ps;      // pixel-dense channels-last: element offset = pix * ps + c
  const void* y; int64_t y_ps;
  const void* dy; int64_t dy_ps;
  void* out; int64_t out_ps;         // y (forward) or dx (backward)
  const float* gamma;
  const float* beta;
  float* acc;                         // [2][C] fp32 sums
  float* mean;                        // [C] save_mean
  float* invstd;                      // [C] save_invstd
  float* running_mean;
  float* running_var;
  float* dgamma;
  float* dbeta;
  int64_t pix_per_block;
};

// MODE 0: acc0 += x; 1: acc1 += (x - mean)^2; 2: acc0 += g, acc1 += g * (x - mean)
template <typename E, int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const BnArgs a) {
  constexpr int EPC = Chunk<E>::EPC;
  __shared__ float sb[2][256 * EPC];
  const int cg0 = blockIdx.y * 256;                               // first chunk of this channel group
  const int nch = min(256, (a.C + EPC - 1) / EPC - cg0);
  if (nch <= 0) return;  // block-uniform: surplus channel group (grid sized for the fp32 chunk count)
  const int ppi = 256 / nch;
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  const bool active = pl < ppi;
  const int c0 = (cg0 + ch) * EPC;
  float s0[EPC], s1[EPC], mu[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    s0[e] = 0.f; s1[e] = 0.f;
    mu[e] = (MODE > 0 && active && c0 + e < a.C) ? a.mean[c0 + e] : 0.f;
  }
  const int64_t p0 = (int64_t)blockIdx.x * a.pix_per_block;
  const int64_t p1 = min(p0 + a.pix_per_block, a.npix);
  if (active) {
    for (int64_t pix = p0 + pl; pix < p1; pix += ppi) {
      float xv[EPC];
      load_chunk(reinterpret_cast<const E*>(a.x) + pix * a.x_ps + c0, xv);
      if constexpr (MODE == 2) {
        float gv[EPC], yv[EPC];
        load_chunk(reinterpret_cast<const E*>(a.dy) + pix * a.dy_ps + c0, gv);
        load_chunk(reinterpret_cast<const E*>(a.y) + pix * a.y_ps + c0, yv);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const float g = tpg_act_grad(gv[e], yv[e], a.act, a.slope);
          s0[e] += g;
          s1[e] += g * (xv[e] - mu[e]);
        }
      } else if constexpr (MODE == 1) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) { const float d = xv[e] - mu[e]; s1[e] += d * d; }
      } else {
#pragma unroll
        for (int e = 0; e < EPC; ++e) s0[e] += xv[e];
      }
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      sb[0][pl * nch * EPC + ch * EPC + e] = s0[e];
      sb[1][pl * nch * EPC + ch * EPC + e] = s1[e];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < nch * EPC; cl += 256) {
    const int c = cg0 * EPC + cl;
    if (c >= a.C) continue;
    float t0 = 0.f, t1 = 0.f;
    for (int q = 0; q < ppi; ++q) { t0 += sb[0][q * nch * EPC + cl]; t1 += sb[1][q * nch * EPC + cl]; }
    if (MODE != 1) atomicAdd(a.acc + c, t0);
    if (MODE != 0) atomicAdd(a.acc + a.C + c, t1);
  }
}

// MODE 0: mean = acc0 / M; 1: invstd, running stats; 2: dgamma += acc1 * invstd, dbeta += acc0
template <int MODE>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const BnArgs a) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.C) return;
  const float M = (float)a.npix;
  if (MODE == 0) {
    a.mean[c] = a.acc[c] / M;
  } else if (MODE == 1) {
    const float var = a.acc[a.C + c] / M;
    a.invstd[c] = 1.f / sqrtf(var + a.eps);
    if (a.running_mean) {
      a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * a.mean[c];
      const float unb = a.npix > 1 ? var * M / (M - 1.f) : var;
      a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
    }
  } else {
    if (a.dgamma) a.dgamma[c] += a.acc[a.C + c] * a.invstd[c];
    if (a.dbeta) a.dbeta[c] += a.acc[c];
  }
}

// forward apply: y = act((x - mean) * invstd * gamma + beta)
// backward apply: dx = gamma * invstd * (g - acc0 / M - (x - mean) * invstd^2 * acc1 / M)
template <typename E, bool BWD>
__global__ __launch_bounds__(256) void bn_apply_kernel(const BnArgs a) {
  constexpr int EPC = Chunk<E>::EPC;
  const int cg0 = blockIdx.y * 256;                               // first chunk of this channel group
  const int nch = min(256, (a.C + EPC - 1) / EPC - cg0);
  if (nch <= 0) return;  // block-uniform: surplus channel group (grid sized for the fp32 chunk count)
  const int ppi = 256 / nch;
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  if (pl >= ppi) return;
  const int c0 = (cg0 + ch) * EPC;
  const float M = (float)a.npix;
  float k0[EPC], k1[EPC], k2[EPC], mu[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    const int c = c0 + e;
    const bool ok = c < a.C;
    const float is = ok ? a.invstd[c] : 0.f, gm = ok ? a.gamma[c] : 0.f;
    mu[e] = ok ? a.mean[c] : 0.f;
    if (BWD) {
      k0[e] = gm * is;                                  // scale of g
      k1[e] = ok ? a.acc[c] / M : 0.f;                   // mean(g)
      k2[e] = ok ? is * is * a.acc[a.C + c] / M : 0.f;   // coefficient of (x - mean)
    } else {
      k0[e] = gm * is;
      k1[e] = ok ? a.beta[c] : 0.f;
      k2[e] = 0.f;
    }
  }
  const int64_t p0 = (int64_t)blockIdx.x * a.pix_per_block;
  const int64_t p1 = min(p0 + a.pix_per_block, a.npix);
  for (int64_t pix = p0 + pl; pix < p1; pix += ppi) {
    float xv[EPC], o[EPC];
    load_chunk(reinterpret_cast<const E*>(a.x) + pix * a.x_ps + c0, xv);
    if constexpr (BWD) {
      float gv[EPC], yv[EPC];
      load_chunk(reinterpret_cast<const E*>(a.dy) + pix * a.dy_ps + c0, gv);
      load_chunk(reinterpret_cast<const E*>(a.y) + pix * a.y_ps + c0, yv);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const float g = tpg_act_grad(gv[e], yv[e], a.act, a.slope);
        o[e] = (c0 + e < a.C) ? k0[e] * (g - k1[e] - (xv[e] - mu[e]) * k2[e]) : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < EPC; ++e)
        o[e] = (c0 + e < a.C) ? tpg_act((xv[e] - mu[e]) * k0[e] + k1[e], a.act, a.slope) : 0.f;
    }
    store_chunk(reinterpret_cast<E*>(a.out) + pix * a.out_ps + c0, o);
  }
}

}  // namespace tpg

using namespace tpg;

namespace {

int ffail(int code, const char* msg) { return tpg::record_error(code, msg); }

inline int grid_cap(int64_t total, int cap = 8192) {
  int64_t b = (total + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

bool chunk_ok(const tpg_tensor& t, int C) {
  const int es = t.dtype != TPG_F32 ? 2 : 4, epc = 16 / es;
  if (t.stride[1] != 1 || ((uintptr_t)t.data) % 16) return false;
  for (int i : {0, 2, 3})
    if (t.stride[i] % epc) return false;
  return t.stride[3] >= (C + epc - 1) / epc * epc;
}

int dw_check(const tpg_conv_desc* d) {
  if (!d) return ffail(-1, "null descriptor");
  if (d->in_c != d->out_c || d->transposed || d->pad_mode != TPG_PAD_ZERO)
    return ffail(-2, "depthwise: in_c must equal out_c, zero padding, no transposition");
  if (d->kh * d->kw > 9 || d->kh < 1 || d->kw < 1) return ffail(-4, "depthwise: kernels up to 3x3");
  if (d->dtype != TPG_F32 && d->dtype != TPG_BF16 && d->dtype != TPG_F16) return ffail(-3, "bad dtype");
  const int oh = (d->in_h + d->pad_t + d->pad_b - d->kh) / d->stride_h + 1;
  const int ow = (d->in_w + d->pad_l + d->pad_r - d->kw) / d->stride_w + 1;
  if (oh != d->out_h || ow != d->out_w) return ffail(-6, "depthwise: output size inconsistent with geometry");
  return 0;
}

DwArgs dw_args(const tpg_conv_desc* d, const tpg_tensor& xg, const tpg_tensor& yg, const tpg_tensor& w) {
  DwArgs a;
  memset(&a, 0, sizeof(a));
  a.N = d->n; a.C = d->in_c; a.H = d->in_h; a.W = d->in_w; a.OH = d->out_h; a.OW = d->out_w;
  a.kh = d->kh; a.kw = d->kw; a.sh = d->stride_h; a.sw = d->stride_w; a.pt = d->pad_t; a.pl = d->pad_l;
  a.x_sn = xg.stride[0]; a.x_sh = xg.stride[2]; a.x_sw = xg.stride[3];
  a.y_sn = yg.stride[0]; a.y_sh = yg.stride[2]; a.y_sw = yg.stride[3];
  a.w = reinterpret_cast<const float*>(w.data);
  a.w_sc = w.stride[0]; a.w_sr = w.stride[2]; a.w_ss = w.stride[3];
  a.act = d->act; a.slope = d->slope; a.res_scale = d->res_scale;
  return a;
}

// blocks over the pixel grid: >= `per_lane` pixels per lane, at most `cap` blocks
dim3 dw_grid(DwArgs& a, int64_t npix, int per_lane, int cap) {
  const int epc = 8;  // conservative lanes-per-block estimate for both dtypes
  const int nch = (a.C + epc - 1) / epc;
  const int ppi = std::max(1, 256 / std::max(nch, 1));
  int64_t blocks = (npix + (int64_t)per_lane * ppi - 1) / ((int64_t)per_lane * ppi);
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, cap));
  a.pix_per_block = (npix + blocks - 1) / blocks;
  return dim3((unsigned)blocks, (unsigned)((a.C + 3) / 4 + 255) / 256);  // y: groups of 256 chunks (fp32 bound)
}

}  // namespace

extern "C" int32_t tpg_dwconv2d_fwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, const float* bias,
                                    tpg_tensor residual, tpg_tensor y, tpg_stream_t stream) {
  if (int rc = dw_check(d)) return rc;
  if (!x.data || !y.data || !w.data || w.dtype != TPG_F32) return ffail(-10, "depthwise fwd: NULL / bad tensor");
  if (x.dtype != d->dtype || y.dtype != d->dtype || !chunk_ok(x, d->in_c) || !chunk_ok(y, d->out_c) ||
      (residual.data && (residual.dtype != d->dtype || !chunk_ok(residual, d->out_c))))
    return ffail(-12, "depthwise: tensors must be 16-byte aligned channels-last rows of the compute dtype");
  DwArgs a = dw_args(d, x, y, w);
  a.bias = bias;
  a.r_sn = residual.stride[0]; a.r_sh = residual.stride[2]; a.r_sw = residual.stride[3];
  const dim3 grid = dw_grid(a, (int64_t)a.N * a.OH * a.OW, 4, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == TPG_F16)
    hipLaunchKernelGGL(dw_fwd_kernel<_Float16>, grid, dim3(256), 0, s, a, (const _Float16*)x.data, (_Float16*)y.data,
                       (const _Float16*)residual.data);
  else if (d->dtype == TPG_BF16)
    hipLaunchKernelGGL(dw_fwd_kernel<__bf16>, grid, dim3(256), 0, s, a, (const __bf16*)x.data, (__bf16*)y.data,
                       (const __bf16*)residual.data);
  else
    hipLaunchKernelGGL(dw_fwd_kernel<float>, grid, dim3(256), 0, s, a, (const float*)x.data, (float*)y.data,
                       (const float*)residual.data);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_dwconv2d_bwd_data(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx,
                                         tpg_stream_t stream) {
  if (int rc = dw_check(d)) return rc;
  if (!g.data || !dx.data || !w.data || w.dtype != TPG_F32) return ffail(-10, "depthwise dgrad: NULL / bad tensor");
  if (g.dtype != d->dtype || dx.dtype != d->dtype || !chunk_ok(g, d->out_c) || !chunk_ok(dx, d->in_c))
    return ffail(-12, "depthwise: tensors must be 16-byte aligned channels-last rows of the compute dtype");
  DwArgs a = dw_args(d, dx, g, w);
  const dim3 grid = dw_grid(a, (int64_t)a.N * a.H * a.W, 4, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == TPG_F16)
    hipLaunchKernelGGL(dw_dgrad_kernel<_Float16>, grid, dim3(256), 0, s, a, (const _Float16*)g.data, (_Float16*)dx.data);
  else if (d->dtype == TPG_BF16)
    hipLaunchKernelGGL(dw_dgrad_kernel<__bf16>, grid, dim3(256), 0, s, a, (const __bf16*)g.data, (__bf16*)dx.data);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<float>, grid, dim3(256), 0, s, a, (const float*)g.data, (float*)dx.data);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_dwconv2d_bwd_filter(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor g, tpg_tensor dw,
                                           tpg_stream_t stream) {
  if (int rc = dw_check(d)) return rc;
  if (!g.data || !x.data || !dw.data || dw.dtype != TPG_F32) return ffail(-10, "depthwise wgrad: NULL / bad tensor");
  if (g.dtype != d->dtype || x.dtype != d->dtype || !chunk_ok(g, d->out_c) || !chunk_ok(x, d->in_c))
    return ffail(-12, "depthwise: tensors must be 16-byte aligned channels-last rows of the compute dtype");
  DwArgs a = dw_args(d, x, g, dw);
  a.w = nullptr;
  const dim3 grid = dw_grid(a, (int64_t)a.N * a.OH * a.OW, 16, 256);
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == TPG_F16)
    hipLaunchKernelGGL(dw_wgrad_kernel<_Float16>, grid, dim3(256), 0, s, a, (const _Float16*)x.data,
                       (const _Float16*)g.data, (float*)dw.data);
  else if (d->dtype == TPG_BF16)
    hipLaunchKernelGGL(dw_wgrad_kernel<__bf16>, grid, dim3(256), 0, s, a, (const __bf16*)x.data,
                       (const __bf16*)g.data, (float*)dw.data);
  else
    hipLaunchKernelGGL(dw_wgrad_kernel<float>, grid, dim3(256), 0, s, a, (const float*)x.data, (const float*)g.data,
                       (float*)dw.data);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_maxpool2d_fwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t k, int32_t s, int32_t p,
                                     int32_t oh, int32_t ow, tpg_tensor x, tpg_tensor y, uint8_t* argmax,
                                     tpg_stream_t stream) {
  if (!x.data || !y.data || !argmax) return ffail(-10, "maxpool: NULL tensor");
  if (k < 1 || k * k > 256 || s < 1 || p < 0 || 2 * p > k) return ffail(-2, "maxpool: bad geometry");
  if (oh != (h + 2 * p - k) / s + 1 || ow != (w + 2 * p - k) / s + 1) return ffail(-6, "maxpool: bad output size");
  if (x.dtype != y.dtype || x.stride[1] != 1 || y.stride[1] != 1) return ffail(-12, "maxpool: channels-last, one dtype");
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_cap((int64_t)n * oh * ow * c);
  if (x.dtype == TPG_F16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<_Float16>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const _Float16*)x.data, x.stride[0], x.stride[2], x.stride[3], (_Float16*)y.data, y.stride[0],
                       y.stride[2], y.stride[3], argmax);
  else if (x.dtype == TPG_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<__bf16>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const __bf16*)x.data, x.stride[0], x.stride[2], x.stride[3], (__bf16*)y.data, y.stride[0],
                       y.stride[2], y.stride[3], argmax);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const float*)x.data, x.stride[0], x.stride[2], x.stride[3], (float*)y.data, y.stride[0],
                       y.stride[2], y.stride[3], argmax);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_maxpool2d_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t k, int32_t s, int32_t p,
                                     int32_t oh, int32_t ow, tpg_tensor gy, const uint8_t* argmax, tpg_tensor dx,
                                     tpg_stream_t stream) {
  if (!gy.data || !dx.data || !argmax) return ffail(-10, "maxpool bwd: NULL tensor");
  if (k < 1 || k * k > 256 || s < 1 || p < 0) return ffail(-2, "maxpool: bad geometry");
  if (gy.dtype != dx.dtype || gy.stride[1] != 1 || dx.stride[1] != 1) return ffail(-12, "maxpool: channels-last");
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_cap((int64_t)n * h * w * c);
  if (gy.dtype == TPG_F16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<_Float16>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const _Float16*)gy.data, gy.stride[0], gy.stride[2], gy.stride[3], argmax, (_Float16*)dx.data,
                       dx.stride[0], dx.stride[2], dx.stride[3]);
  else if (gy.dtype == TPG_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<__bf16>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const __bf16*)gy.data, gy.stride[0], gy.stride[2], gy.stride[3], argmax, (__bf16*)dx.data,
                       dx.stride[0], dx.stride[2], dx.stride[3]);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid), dim3(256), 0, st, n, c, h, w, oh, ow, k, s, p,
                       (const float*)gy.data, gy.stride[0], gy.stride[2], gy.stride[3], argmax, (float*)dx.data,
                       dx.stride[0], dx.stride[2], dx.stride[3]);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_avgpool_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor y,
                                   tpg_stream_t stream) {
  if (!x.data || !y.data) return ffail(-10, "avgpool: NULL tensor");
  if (x.dtype != y.dtype || x.stride[1] != 1 || y.stride[1] != 1) return ffail(-12, "avgpool: channels-last");
  hipStream_t st = (hipStream_t)stream;
  const int grid = (n * c + 255) / 256;
  if (x.dtype == TPG_F16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<_Float16>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const _Float16*)x.data,
                       x.stride[0], x.stride[2], x.stride[3], (_Float16*)y.data, y.stride[0]);
  else if (x.dtype == TPG_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<__bf16>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const __bf16*)x.data,
                       x.stride[0], x.stride[2], x.stride[3], (__bf16*)y.data, y.stride[0]);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const float*)x.data,
                       x.stride[0], x.stride[2], x.stride[3], (float*)y.data, y.stride[0]);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_avgpool_bwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor gy, tpg_tensor dx,
                                   tpg_stream_t stream) {
  if (!gy.data || !dx.data) return ffail(-10, "avgpool bwd: NULL tensor");
  if (gy.dtype != dx.dtype || gy.stride[1] != 1 || dx.stride[1] != 1) return ffail(-12, "avgpool: channels-last");
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_cap((int64_t)n * h * w * c);
  if (gy.dtype == TPG_F16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<_Float16>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const _Float16*)gy.data,
                       gy.stride[0], (_Float16*)dx.data, dx.stride[0], dx.stride[2], dx.stride[3]);
  else if (gy.dtype == TPG_BF16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<__bf16>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const __bf16*)gy.data,
                       gy.stride[0], (__bf16*)dx.data, dx.stride[0], dx.stride[2], dx.stride[3]);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, dim3(grid), dim3(256), 0, st, n, c, h, w, (const float*)gy.data,
                       gy.stride[0], (float*)dx.data, dx.stride[0], dx.stride[2], dx.stride[3]);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_bn_fold(int32_t cout, int32_t cin, int32_t kh, int32_t kw, tpg_tensor w, const float* bias,
                               const float* gamma, const float* beta, const float* mean, const float* var, float eps,
                               tpg_tensor w_out, float* b_out, tpg_stream_t stream) {
  if (!w.data || !w_out.data || !b_out || !gamma || !beta || !mean || !var) return ffail(-10, "bn_fold: NULL");
  if (w.dtype != TPG_F32 || w_out.dtype != TPG_F32) return ffail(-13, "bn_fold: weights must be fp32");
  const int grid = grid_cap((int64_t)cout * cin * kh * kw);
  hipLaunchKernelGGL(bn_fold_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, cout, cin, kh, kw, w, bias, gamma,
                     beta, mean, var, eps, w_out, b_out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------- BatchNorm2d training --
namespace {

bool pix_dense(const tpg_tensor& t, int h, int w, int C, int dtype) {
  const int es = dtype != TPG_F32 ? 2 : 4, epc = 16 / es;
  if (t.dtype != dtype || t.stride[1] != 1 || ((uintptr_t)t.data) % 16) return false;
  const int64_t ps = t.stride[3];
  if (ps % epc || ps < (C + epc - 1) / epc * epc) return false;
  return t.stride[2] == ps * w && t.stride[0] == ps * w * h;
}

template <typename E>
int bn_launch_fwd(BnArgs a, int blocks, hipStream_t s) {
  constexpr int EPC = Chunk<E>::EPC;
  const dim3 g(blocks, ((a.C + EPC - 1) / EPC + 255) / 256), b(256), gc((a.C + 255) / 256);
  hipLaunchKernelGGL((bn_reduce_kernel<E, 0>), g, b, 0, s, a);
  hipLaunchKernelGGL((bn_finalize_kernel<0>), gc, b, 0, s, a);
  hipLaunchKernelGGL((bn_reduce_kernel<E, 1>), g, b, 0, s, a);
  hipLaunchKernelGGL((bn_finalize_kernel<1>), gc, b, 0, s, a);
  hipLaunchKernelGGL((bn_apply_kernel<E, false>), g, b, 0, s, a);
  return (int)hipGetLastError();
}

template <typename E>
int bn_launch_bwd(BnArgs a, int blocks, hipStream_t s) {
  constexpr int EPC = Chunk<E>::EPC;
  const dim3 g(blocks, ((a.C + EPC - 1) / EPC + 255) / 256), b(256), gc((a.C + 255) / 256);
  hipLaunchKernelGGL((bn_reduce_kernel<E, 2>), g, b, 0, s, a);
  hipLaunchKernelGGL((bn_finalize_kernel<2>), gc, b, 0, s, a);
  if (a.out) hipLaunchKernelGGL((bn_apply_kernel<E, true>), g, b, 0, s, a);
  return (int)hipGetLastError();
}

int bn_blocks(BnArgs& a) {
  const int nch = (a.C + 7) / 8;
  const int ppi = std::max(1, 256 / nch);
  int64_t blocks = (a.npix + 8LL * ppi - 1) / (8LL * ppi);
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, 512));
  a.pix_per_block = (a.npix + blocks - 1) / blocks;
  return (int)blocks;
}

}  // namespace

extern "C" int32_t tpg_bn_train_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, const float* gamma,
                                    const float* beta, float* running_mean, float* running_var, float momentum,
                                    float eps, int32_t act, float slope, tpg_tensor y, float* save_mean,
                                    float* save_invstd, float* ws, tpg_stream_t stream) {
  if (!x.data || !y.data || !gamma || !beta || !save_mean || !save_invstd || !ws) return ffail(-10, "bn_train_fwd: NULL");
  if ((running_mean == nullptr) != (running_var == nullptr)) return ffail(-10, "bn_train_fwd: running stats pair");
  if (!pix_dense(x, h, w, c, x.dtype) || !pix_dense(y, h, w, c, x.dtype))
    return ffail(-12, "bn_train: pixel-dense 16-byte aligned channels-last tensors");
  BnArgs a;
  memset(&a, 0, sizeof(a));
  a.npix = (int64_t)n * h * w; a.C = c; a.act = act; a.slope = slope; a.eps = eps; a.momentum = momentum;
  a.x = x.data; a.x_ps = x.stride[3]; a.out = y.data; a.out_ps = y.stride[3];
  a.gamma = gamma; a.beta = beta; a.acc = ws; a.mean = save_mean; a.invstd = save_invstd;
  a.running_mean = running_mean; a.running_var = running_var;
  hipStream_t s = (hipStream_t)stream;
  if (hipError_t e = hipMemsetAsync(ws, 0, sizeof(float) * 2 * c, s)) return (int)e;
  const int blocks = bn_blocks(a);
  return x.dtype == TPG_F16 ? bn_launch_fwd<_Float16>(a, blocks, s) : x.dtype == TPG_BF16 ? bn_launch_fwd<__bf16>(a, blocks, s) : bn_launch_fwd<float>(a, blocks, s);
}

extern "C" int32_t tpg_bn_train_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t act, float slope,
                                    tpg_tensor dy, tpg_tensor y, tpg_tensor x, const float* gamma,
                                    const float* save_mean, const float* save_invstd, tpg_tensor dx, float* dgamma,
                                    float* dbeta, float* ws, tpg_stream_t stream) {
  if (!dy.data || !y.data || !x.data || !gamma || !save_mean || !save_invstd || !ws) return ffail(-10, "bn_train_bwd: NULL");
  const int dt = x.dtype;
  if (!pix_dense(x, h, w, c, dt) || !pix_dense(y, h, w, c, dt) || !pix_dense(dy, h, w, c, dt) ||
      (dx.data && !pix_dense(dx, h, w, c, dt)))
    return ffail(-12, "bn_train: pixel-dense 16-byte aligned channels-last tensors");
  BnArgs a;
  memset(&a, 0, sizeof(a));
  a.npix = (int64_t)n * h * w; a.C = c; a.act = act; a.slope = slope;
  a.x = x.data; a.x_ps = x.stride[3]; a.y = y.data; a.y_ps = y.stride[3]; a.dy = dy.data; a.dy_ps = dy.stride[3];
  a.out = dx.data; a.out_ps = dx.stride[3];
  a.gamma = gamma; a.acc = ws; a.mean = const_cast<float*>(save_mean); a.invstd = const_cast<float*>(save_invstd);
  a.dgamma = dgamma; a.dbeta = dbeta;
  hipStream_t s = (hipStream_t)stream;
  if (hipError_t e = hipMemsetAsync(ws, 0, sizeof(float) * 2 * c, s)) return (int)e;
  const int blocks = bn_blocks(a);
  return dt == TPG_F16 ? bn_launch_bwd<_Float16>(a, blocks, s) : dt == TPG_BF16 ? bn_launch_bwd<__bf16>(a, blocks, s) : bn_launch_bwd<float>(a, blocks, s);
}

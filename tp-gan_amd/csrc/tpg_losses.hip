// G-step image losses of the TP-GAN train step (tpgan_train._g_losses; build-defined weights,
// config.py:59-82) as two fused ops instead of ~100 small aten launches on the step's critical
// path between D(fake) and the G backward:
//
//   image losses of the 128 x 128 fake (x) against the frontal target (r):
//     w_pix * mean|x - r|  +  w_sym * mean|x - flip_W(x)|
//       + w_tv * (mean|x[y+1] - x[y]| + mean|x[:, x+1] - x[:, x]|)
//   a set of L1 means (the four local-pathway patches against their frontal crops):
//     sum_i w_i * mean|a_i - b_i|
//
// Forward: one launch of per-block partial sums (fixed grid), one single-block launch summing
// them in block order (deterministic, no atomics) into the fp32 scalar.  Backward: one launch
// writing each element's gradient (sign terms scaled by the incoming scalar gradient), in the
// input's own dtype and strides.  sign(0) = 0 throughout (torch's abs backward).
#include "tpg_internal.h"
#include <algorithm>
#include <string.h>

namespace tpg {

static constexpr int LS_THREADS = 256;
static constexpr int LS_BLOCKS = 512;  // partial-sum blocks (fixed: the final order is fixed)

__device__ __forceinline__ float ls_ld(const tpg_tensor& t, int64_t off) {
  if (t.dtype == TPG_BF16) return (float)reinterpret_cast<const __bf16*>(t.data)[off];
  if (t.dtype == TPG_F16) return (float)reinterpret_cast<const _Float16*>(t.data)[off];
  return reinterpret_cast<const float*>(t.data)[off];
}
__device__ __forceinline__ void ls_st(const tpg_tensor& t, int64_t off, float v) {
  if (t.dtype == TPG_BF16) reinterpret_cast<__bf16*>(t.data)[off] = (__bf16)v;
  else if (t.dtype == TPG_F16) reinterpret_cast<_Float16*>(t.data)[off] = (_Float16)v;
  else reinterpret_cast<float*>(t.data)[off] = v;
}
__device__ __forceinline__ int64_t ls_off(const tpg_tensor& t, int n, int c, int y, int x) {
  return (int64_t)n * t.stride[0] + (int64_t)c * t.stride[1] + (int64_t)y * t.stride[2] + (int64_t)x * t.stride[3];
}
__device__ __forceinline__ float ls_sign(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// block sum of NV values per thread -> thread 0 writes out[0..NV)
template <int NV>
__device__ __forceinline__ void ls_block_sum(float (&v)[NV], float* out) {
  __shared__ float red[LS_THREADS / 64][NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    v[k] = s;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wave][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float s = 0.f;
      for (int w = 0; w < LS_THREADS / 64; ++w) s += red[w][k];
      out[k] = s;
    }
}

struct ImgLossArgs {
  int n, c, h, w;
  tpg_tensor x, r;
  float w_pix, w_sym, w_tv;
};

__global__ __launch_bounds__(LS_THREADS) void img_loss_partial_kernel(const ImgLossArgs a, float* part) {
  const int64_t total = (int64_t)a.n * a.c * a.h * a.w;
  float v[4] = {0.f, 0.f, 0.f, 0.f};  // |x - r|, |x - flip x|, |dy|, |dx|
  for (int64_t i = blockIdx.x * (int64_t)LS_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * LS_THREADS) {
    const int xx = (int)(i % a.w);
    int64_t q = i / a.w;
    const int yy = (int)(q % a.h);
    q /= a.h;
    const int cc = (int)(q % a.c), nn = (int)(q / a.c);
    const float f = ls_ld(a.x, ls_off(a.x, nn, cc, yy, xx));
    v[0] += fabsf(f - ls_ld(a.r, ls_off(a.r, nn, cc, yy, xx)));
    v[1] += fabsf(f - ls_ld(a.x, ls_off(a.x, nn, cc, yy, a.w - 1 - xx)));
    if (yy + 1 < a.h) v[2] += fabsf(ls_ld(a.x, ls_off(a.x, nn, cc, yy + 1, xx)) - f);
    if (xx + 1 < a.w) v[3] += fabsf(ls_ld(a.x, ls_off(a.x, nn, cc, yy, xx + 1)) - f);
  }
  ls_block_sum<4>(v, part + 4 * blockIdx.x);
}

__global__ __launch_bounds__(LS_THREADS) void img_loss_final_kernel(const ImgLossArgs a, const float* part, int nblk,
                                                                   float* out) {
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nblk; b += LS_THREADS)
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += part[4 * b + k];
  __shared__ float s[4];
  ls_block_sum<4>(v, s);
  if (threadIdx.x == 0) {
    const double nc = (double)a.n * a.c;
    const double e = nc * a.h * a.w, ey = nc * (a.h - 1) * a.w, ex = nc * a.h * (a.w - 1);
    out[0] = (float)(a.w_pix * (s[0] / e) + a.w_sym * (s[1] / e) +
                     a.w_tv * ((ey > 0 ? s[2] / ey : 0.0) + (ex > 0 ? s[3] / ex : 0.0)));
  }
}

__global__ __launch_bounds__(LS_THREADS) void img_loss_bwd_kernel(const ImgLossArgs a, const float* gout, tpg_tensor dx) {
  const int64_t total = (int64_t)a.n * a.c * a.h * a.w;
  const float g = gout[0];
  const double nc = (double)a.n * a.c;
  const float ke = (float)(1.0 / (nc * a.h * a.w));
  const float ky = a.h > 1 ? (float)(1.0 / (nc * (a.h - 1) * a.w)) : 0.f;
  const float kx = a.w > 1 ? (float)(1.0 / (nc * a.h * (a.w - 1))) : 0.f;
  for (int64_t i = blockIdx.x * (int64_t)LS_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * LS_THREADS) {
    const int xx = (int)(i % a.w);
    int64_t q = i / a.w;
    const int yy = (int)(q % a.h);
    q /= a.h;
    const int cc = (int)(q % a.c), nn = (int)(q / a.c);
    const float f = ls_ld(a.x, ls_off(a.x, nn, cc, yy, xx));
    // d|x - r|, d|x - flip x| (= 2 sign(x - flip x): x and its mirror both carry the pair),
    // and the two neighbour differences each pixel starts and ends
    float d = a.w_pix * ke * ls_sign(f - ls_ld(a.r, ls_off(a.r, nn, cc, yy, xx)));
    d += a.w_sym * ke * 2.f * ls_sign(f - ls_ld(a.x, ls_off(a.x, nn, cc, yy, a.w - 1 - xx)));
    float t = 0.f;
    if (yy > 0) t += ky * ls_sign(f - ls_ld(a.x, ls_off(a.x, nn, cc, yy - 1, xx)));
    if (yy + 1 < a.h) t -= ky * ls_sign(ls_ld(a.x, ls_off(a.x, nn, cc, yy + 1, xx)) - f);
    if (xx > 0) t += kx * ls_sign(f - ls_ld(a.x, ls_off(a.x, nn, cc, yy, xx - 1)));
    if (xx + 1 < a.w) t -= kx * ls_sign(ls_ld(a.x, ls_off(a.x, nn, cc, yy, xx + 1)) - f);
    ls_st(dx, ls_off(dx, nn, cc, yy, xx), g * (d + a.w_tv * t));
  }
}

struct L1SetArgs {
  int nseg;
  int dims[TPG_L1_MAX_SEGS][4];
  int64_t start[TPG_L1_MAX_SEGS + 1];  // element ranges of the segments in one flat index space
  tpg_tensor a[TPG_L1_MAX_SEGS], b[TPG_L1_MAX_SEGS], da[TPG_L1_MAX_SEGS];
  float wt[TPG_L1_MAX_SEGS];
};

__device__ __forceinline__ int l1_seg(const L1SetArgs& s, int64_t i) {
  int k = 0;
  while (k + 1 < s.nseg && i >= s.start[k + 1]) ++k;
  return k;
}
__device__ __forceinline__ void l1_coords(const L1SetArgs& s, int k, int64_t j, int& n, int& c, int& y, int& x) {
  x = (int)(j % s.dims[k][3]);
  int64_t q = j / s.dims[k][3];
  y = (int)(q % s.dims[k][2]);
  q /= s.dims[k][2];
  c = (int)(q % s.dims[k][1]);
  n = (int)(q / s.dims[k][1]);
}

__global__ __launch_bounds__(LS_THREADS) void l1_set_partial_kernel(const L1SetArgs s, float* part) {
  float v[TPG_L1_MAX_SEGS];
#pragma unroll
  for (int k = 0; k < TPG_L1_MAX_SEGS; ++k) v[k] = 0.f;
  const int64_t total = s.start[s.nseg];
  for (int64_t i = blockIdx.x * (int64_t)LS_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * LS_THREADS) {
    const int k = l1_seg(s, i);
    int n, c, y, x;
    l1_coords(s, k, i - s.start[k], n, c, y, x);
    const float d = fabsf(ls_ld(s.a[k], ls_off(s.a[k], n, c, y, x)) - ls_ld(s.b[k], ls_off(s.b[k], n, c, y, x)));
#pragma unroll
    for (int q = 0; q < TPG_L1_MAX_SEGS; ++q)
      if (q == k) v[q] += d;
  }
  ls_block_sum<TPG_L1_MAX_SEGS>(v, part + TPG_L1_MAX_SEGS * blockIdx.x);
}

__global__ __launch_bounds__(LS_THREADS) void l1_set_final_kernel(const L1SetArgs s, const float* part, int nblk,
                                                                 float* out) {
  float v[TPG_L1_MAX_SEGS];
#pragma unroll
  for (int k = 0; k < TPG_L1_MAX_SEGS; ++k) v[k] = 0.f;
  for (int b = threadIdx.x; b < nblk; b += LS_THREADS)
#pragma unroll
    for (int k = 0; k < TPG_L1_MAX_SEGS; ++k) v[k] += part[TPG_L1_MAX_SEGS * b + k];
  __shared__ float r[TPG_L1_MAX_SEGS];
  ls_block_sum<TPG_L1_MAX_SEGS>(v, r);
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < s.nseg; ++k) {
      const int64_t e = s.start[k + 1] - s.start[k];
      if (e > 0) t += s.wt[k] * (r[k] / (double)e);
    }
    out[0] = (float)t;
  }
}

__global__ __launch_bounds__(LS_THREADS) void l1_set_bwd_kernel(const L1SetArgs s, const float* gout) {
  const float g = gout[0];
  const int64_t total = s.start[s.nseg];
  for (int64_t i = blockIdx.x * (int64_t)LS_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * LS_THREADS) {
    const int k = l1_seg(s, i);
    if (!s.da[k].data) continue;
    int n, c, y, x;
    l1_coords(s, k, i - s.start[k], n, c, y, x);
    const float d = ls_ld(s.a[k], ls_off(s.a[k], n, c, y, x)) - ls_ld(s.b[k], ls_off(s.b[k], n, c, y, x));
    const float ke = (float)(1.0 / (double)(s.start[k + 1] - s.start[k]));
    ls_st(s.da[k], ls_off(s.da[k], n, c, y, x), g * s.wt[k] * ke * ls_sign(d));
  }
}

static int ls_grid(int64_t total) { return (int)std::max<int64_t>(1, std::min<int64_t>(LS_BLOCKS, (total + LS_THREADS - 1) / LS_THREADS)); }

int launch_image_losses(int n, int c, int h, int w, const tpg_tensor& x, const tpg_tensor& r, float w_pix, float w_sym,
                        float w_tv, float* part, const float* gout, float* out, const tpg_tensor* dx, hipStream_t st) {
  ImgLossArgs a;
  a.n = n; a.c = c; a.h = h; a.w = w; a.x = x; a.r = r; a.w_pix = w_pix; a.w_sym = w_sym; a.w_tv = w_tv;
  const int64_t total = (int64_t)n * c * h * w;
  const int blocks = ls_grid(total);
  if (dx) {
    hipLaunchKernelGGL(img_loss_bwd_kernel, dim3(blocks), dim3(LS_THREADS), 0, st, a, gout, *dx);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(img_loss_partial_kernel, dim3(blocks), dim3(LS_THREADS), 0, st, a, part);
  hipLaunchKernelGGL(img_loss_final_kernel, dim3(1), dim3(LS_THREADS), 0, st, a, part, blocks, out);
  return (int)hipGetLastError();
}

int launch_l1_set(int nseg, const tpg_l1_seg* segs, float* part, const float* gout, float* out, bool bwd,
                  hipStream_t st) {
  L1SetArgs s;
  memset(&s, 0, sizeof(s));
  s.nseg = nseg;
  s.start[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    s.dims[k][0] = segs[k].n; s.dims[k][1] = segs[k].c; s.dims[k][2] = segs[k].h; s.dims[k][3] = segs[k].w;
    s.a[k] = segs[k].a; s.b[k] = segs[k].b; s.da[k] = segs[k].da; s.wt[k] = segs[k].weight;
    s.start[k + 1] = s.start[k] + (int64_t)segs[k].n * segs[k].c * segs[k].h * segs[k].w;
  }
  const int blocks = ls_grid(s.start[nseg]);
  if (bwd) {
    hipLaunchKernelGGL(l1_set_bwd_kernel, dim3(blocks), dim3(LS_THREADS), 0, st, s, gout);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(l1_set_partial_kernel, dim3(blocks), dim3(LS_THREADS), 0, st, s, part);
  hipLaunchKernelGGL(l1_set_final_kernel, dim3(1), dim3(LS_THREADS), 0, st, s, part, blocks, out);
  return (int)hipGetLastError();
}

}  // namespace tpg

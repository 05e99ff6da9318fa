// HBM-bound kernels of the TP-GAN hot path (gfx950): weight packing, activation
// backward + bias gradient, strided copy / concat / dtype conversion, LocalFuser,
// maxout, reflection-pad fold and the Adam update.  Each is a grid-stride loop over
// channels-last elements so that consecutive lanes touch consecutive channels.
#include "tpg_internal.h"
#include "../../include/tpgan.h"
#include <stdlib.h>
#include <string.h>
#include <algorithm>

namespace tpg {

__device__ __forceinline__ float ld_any(const void* p, int dtype, int64_t off) {
  return dtype == TPG_BF16 ? (float)reinterpret_cast<const __bf16*>(p)[off]
       : dtype == TPG_F16  ? (float)reinterpret_cast<const _Float16*>(p)[off]
                           : reinterpret_cast<const float*>(p)[off];
}
__device__ __forceinline__ void st_any(void* p, int dtype, int64_t off, float v) {
  if (dtype == TPG_BF16) reinterpret_cast<__bf16*>(p)[off] = (__bf16)v;
  else if (dtype == TPG_F16) reinterpret_cast<_Float16*>(p)[off] = (_Float16)v;
  else reinterpret_cast<float*>(p)[off] = v;
}

static inline int grid_for(int64_t total, int per_block = 256, int cap = 8192) {
  int64_t b = (total + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// ------------------------------------------------------------------ weight packing --
// One thread per 16-channel unit of one packed row, 32-bit index math.
template <typename E>
__global__ __launch_bounds__(256) void pack_kernel(const PackArgs p, int nthreads) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < nthreads) pack_igemm_item<E>(p, idx);
}

// Halo-layout image whose packed rows n' run along the weight's unit-stride channel and whose
// chunks run along a strided one (the input-gradient images of channels-last weights): the
// block's 64 rows x ROW channels are read as unit-stride runs (one 256-byte run per wave and
// load), transposed through LDS and written as the item kernel's 16-byte chunks.
template <typename E>
__device__ __forceinline__ void pack_halo_block_t(const PackArgs& p, int bn, int bnl, int ntiles, int lb) {
  constexpr int EPC = 16 / sizeof(E);
  constexpr int ROW = 4 * EPC;
  __shared__ float tile[ROW][65];
  const int t = threadIdx.x;
  int rr = lb * 64 / bnl;           // (bnl is a multiple of 128: the block's rows share one (ks, tap, nt))
  const int r0 = lb * 64 - rr * bnl;
  const int nt = rr % ntiles;
  rr /= ntiles;
  // step rr as in pack_halo_item: a full k-step's tap, or (paired last k-step) taps 2j (logical
  // channels 0..15 of the row) and 2j + 1 (16..31), channels 0..15 of that k-step each; the
  // thread's quarter of the row (t >> 6) lies in one of the two halves
  const int nfull = (p.half ? p.hnks - 1 : p.hnks) * p.ntaps;
  const bool paired = rr >= nfull;
  const int q = t >> 6;
  int tap, ks, cbase;
  if (!paired) {
    tap = rr % p.ntaps;
    ks = rr / p.ntaps;
    cbase = ks * ROW + q * (ROW / 4);
  } else {
    tap = 2 * (rr - nfull) + (q >> 1);
    ks = p.hnks - 1;
    cbase = ks * ROW + (q & 1) * (ROW / 4);
  }
  const bool tap_ok = tap < p.ntaps;
  const int tp = tap_ok ? tap : 0;
  const int64_t tapoff = (int64_t)p.tr[tp] * p.w_sr + (int64_t)p.ts[tp] * p.w_ss;
  {
    const int rl = t & 63;
    const int r = r0 + rl;
    const int np = nt * bn + r;
    const bool row_ok = r < bn && np < p.Nreal && tap_ok;
    const float* src = p.W + tapoff + np;
#pragma unroll
    for (int e = 0; e < ROW / 4; ++e) {
      const int cl = q * (ROW / 4) + e;
      const int c = cbase + e;
      tile[cl][rl] = (row_ok && c < p.Creal) ? src[(int64_t)c * p.w_sa] : 0.f;
    }
  }
  __syncthreads();
  const int rl = t >> 2, pchunk = t & 3;
  const int cl0 = (pchunk ^ pack_hswz(r0 + rl)) * EPC;
  union { uint4 u; E e[EPC]; } o;
#pragma unroll
  for (int e = 0; e < EPC; ++e) o.e[e] = (E)tile[cl0 + e][rl];
  reinterpret_cast<uint4*>(p.Wp)[(int64_t)lb * 256 + t] = o.u;
}

// Every weight pack of a network in one launch: block b finds its job (binary search over
// first_block), stages the job in LDS and packs TPG_PACK_GROUPS groups of 256 items,
// ((b - first_block)*TPG_PACK_GROUPS + g)*256 + tid (one group per block measured latency-bound
// on the search and the job copy: 150 k blocks for G's images).
__global__ __launch_bounds__(256) void pack_many_kernel(const PackJob* __restrict__ jobs, int n) {
  __shared__ PackJob job;
  __shared__ int jsel;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n - 1;
    const int b = blockIdx.x;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].first_block <= b) lo = mid; else hi = mid - 1;
    }
    jsel = lo;
  }
  __syncthreads();
  {
    const int* src = reinterpret_cast<const int*>(jobs + jsel);
    int* dst = reinterpret_cast<int*>(&job);
    for (int i = threadIdx.x; i < (int)(sizeof(PackJob) / 4); i += 256) dst[i] = src[i];
  }
  __syncthreads();
  const int lb0 = (blockIdx.x - job.first_block) * TPG_PACK_GROUPS;
  if (job.kind == 1 && job.k.cmode == 0 && job.k.nmode == 1 && job.k.w_sb == 1) {
    // (block-uniform: items is a multiple of 256, bnl of 128)
    for (int lb = lb0; lb < lb0 + TPG_PACK_GROUPS && lb * 256 < job.items; ++lb) {
      if (job.k.dtype == TPG_BF16) pack_halo_block_t<__bf16>(job.k, job.bn, job.bnl, job.ntiles, lb);
      else if (job.k.dtype == TPG_F16) pack_halo_block_t<_Float16>(job.k, job.bn, job.bnl, job.ntiles, lb);
      else pack_halo_block_t<float>(job.k, job.bn, job.bnl, job.ntiles, lb);
      __syncthreads();  // (the LDS tile is refilled by the next group)
    }
    return;
  }
#pragma unroll 1
  for (int g = 0; g < TPG_PACK_GROUPS; ++g) {
    const int idx = (lb0 + g) * 256 + threadIdx.x;
    if (idx >= job.items) break;
    if (job.kind == 1) {
      if (job.k.dtype == TPG_BF16) pack_halo_item<__bf16>(job.k, job.bn, job.bnl, job.ntiles, idx);
      else if (job.k.dtype == TPG_F16) pack_halo_item<_Float16>(job.k, job.bn, job.bnl, job.ntiles, idx);
      else pack_halo_item<float>(job.k, job.bn, job.bnl, job.ntiles, idx);
    } else {
      if (job.k.dtype == TPG_BF16) pack_igemm_item<__bf16>(job.k, idx);
      else if (job.k.dtype == TPG_F16) pack_igemm_item<_Float16>(job.k, idx);
      else pack_igemm_item<float>(job.k, idx);
    }
  }
}

int launch_pack_many(const PackJob* jobs_dev, int n, int nblocks, hipStream_t s) {
  if (n <= 0 || nblocks <= 0) return 0;
  hipLaunchKernelGGL(pack_many_kernel, dim3(nblocks), dim3(256), 0, s, jobs_dev, n);
  return (int)hipGetLastError();
}

int launch_pack(const PackArgs& a, hipStream_t s) {
  const int nthreads = a.Npad * a.nunits;
  const int blocks = (nthreads + 255) / 256;
  if (a.dtype == TPG_BF16) hipLaunchKernelGGL(pack_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, a, nthreads);
  else if (a.dtype == TPG_F16) hipLaunchKernelGGL(pack_kernel<_Float16>, dim3(blocks), dim3(256), 0, s, a, nthreads);
  else hipLaunchKernelGGL(pack_kernel<float>, dim3(blocks), dim3(256), 0, s, a, nthreads);
  return (int)hipGetLastError();
}

// --------------------------------------------------- activation backward + bias grad --
// g = gy * act'(y); 64 channels x 4 pixel lanes per block, dbias reduced in LDS and
// added with one atomic per channel per block.
__global__ __launch_bounds__(256) void act_bwd_kernel(int N, int C, int H, int W, int act, float slope,
                                                      tpg_tensor gy, tpg_tensor y, tpg_tensor g, float* dbias) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int64_t npix = (int64_t)N * H * W;
  float sum = 0.f;
  if (c < C) {
    for (int64_t pix = blockIdx.x * 4 + pl; pix < npix; pix += (int64_t)gridDim.x * 4) {
      int n = (int)(pix / ((int64_t)H * W));
      int rem = (int)(pix - (int64_t)n * H * W);
      int h = rem / W, w = rem - (rem / W) * W;
      float v = ld_any(gy.data, gy.dtype, n * gy.stride[0] + c * gy.stride[1] + h * gy.stride[2] + w * gy.stride[3]);
      if (act != TPG_ACT_NONE) {
        float yv = ld_any(y.data, y.dtype, n * y.stride[0] + c * y.stride[1] + h * y.stride[2] + w * y.stride[3]);
        v = tpg_act_grad(v, yv, act, slope);
      }
      st_any(g.data, g.dtype, n * g.stride[0] + c * g.stride[1] + h * g.stride[2] + w * g.stride[3], v);
      sum += v;
    }
  }
  red[pl][cl] = sum;
  __syncthreads();
  if (pl == 0 && c < C && dbias) {
    float s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    atomicAdd(dbias + c, s);
  }
}

// Row form for pixel-dense channels-last tensors of any alignment, pixel stride and dtype
// mix (channel slices of concat buffers, fp32 incoming gradients), C <= 256: lane = channel,
// 256 / C pixel lanes per block, eight pixels per iteration with every load issued first; no
// index division.  dbias as in the vector form (up to 4096 blocks).
__global__ __launch_bounds__(256) void act_bwd_rows_kernel(int64_t npix, int C, int act, float slope, tpg_tensor gy,
                                                           tpg_tensor y, tpg_tensor g, float* dbias,
                                                           int64_t pix_per_block) {
  constexpr int U = 8;  // 2- or 4-byte lanes: more pixels in flight than the vector form
  __shared__ float sb[256];
  const int ppi = 256 / C;
  const int c = threadIdx.x % C, pl = threadIdx.x / C;
  const bool active = pl < ppi;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block;
  if (p0 >= npix) return;  // (uniform) the grid may overshoot by a block
  const int64_t p1 = p0 + pix_per_block < npix ? p0 + pix_per_block : npix;
  const bool has_act = act != TPG_ACT_NONE;
  const int64_t gs = gy.stride[3], ys = y.stride[3], os = g.stride[3];
  float part = 0.f;
  if (active) {
    for (int64_t pb = p0 + pl; pb < p1; pb += (int64_t)U * ppi) {
      float vg[U], vy[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pix = pb + (int64_t)u * ppi;
        const int64_t pc = pix < p1 ? pix : p0;  // clamped: every load issues before any use
        vg[u] = ld_any(gy.data, gy.dtype, pc * gs + c);
        vy[u] = has_act ? ld_any(y.data, y.dtype, pc * ys + c) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pix = pb + (int64_t)u * ppi;
        if (pix < p1) {
          const float v = has_act ? tpg_act_grad(vg[u], vy[u], act, slope) : vg[u];
          st_any(g.data, g.dtype, pix * os + c, v);
          part += v;
        }
      }
    }
  }
  if (!dbias) return;
  sb[threadIdx.x] = active ? part : 0.f;
  __syncthreads();
  if (threadIdx.x < C) {
    float sum = 0.f;
    for (int q = 0; q < ppi; ++q) sum += sb[q * C + threadIdx.x];
    atomicAdd(dbias + threadIdx.x, sum);
  }
}

// Vector form for channels-last tensors with pixel-dense, 16-byte aligned rows: a thread
// owns one 16-byte channel chunk and walks a contiguous pixel range of its block, four
// pixels per iteration with all loads issued before any use (HBM latency hiding).  Its
// dbias partials stay in registers; the block combines them through LDS (no LDS atomics)
// and adds one global atomic per channel, with at most 1024 blocks per launch.
template <typename E, int NG = 1>
__global__ __launch_bounds__(256) void act_bwd_vec_kernel(const Grouped<ActVecArgs, NG> G) {
  int mem = 0, bid = blockIdx.x;
  if constexpr (NG > 1) {  // grouped: member blocks [boff[m], boff[m + 1])
    mem = group_member(G, blockIdx.x);
    bid = blockIdx.x - G.boff[mem];
  }
  const ActVecArgs& a = G.a[mem];
  const int64_t npix = a.npix, pix_per_block = a.pix_per_block;
  const int C = a.C, act = a.act;
  const float slope = a.slope;
  const E* gy = reinterpret_cast<const E*>(a.gy);
  const E* y = reinterpret_cast<const E*>(a.y);
  E* g = reinterpret_cast<E*>(a.g);
  const int64_t gps = a.gps, yps = a.yps, gps_out = a.gps_out;
  float* dbias = a.dbias;
  constexpr int EPC = 16 / sizeof(E);
  constexpr int U = 4;
  __shared__ float sb[256 * EPC];
  const int nch = (C + EPC - 1) / EPC;
  const int ppi = 256 / nch;                      // pixel lanes per block
  const int ch = threadIdx.x % nch, pl = threadIdx.x / nch;
  const bool active = pl < ppi;
  float part[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) part[e] = 0.f;
  const int c0 = ch * EPC;
  const int64_t p0 = (int64_t)bid * pix_per_block;
  const int64_t p1 = p0 + pix_per_block < npix ? p0 + pix_per_block : npix;
  const bool has_act = act != TPG_ACT_NONE;
  if (active) {
    for (int64_t pb = p0 + pl; pb < p1; pb += (int64_t)U * ppi) {
      union V { uint4 u; E e[EPC]; };
      V vg[U], vy[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pix = pb + (int64_t)u * ppi;
        if (pix < p1) {
          vg[u].u = *reinterpret_cast<const uint4*>(gy + pix * gps + c0);
          if (has_act) vy[u].u = *reinterpret_cast<const uint4*>(y + pix * yps + c0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pix = pb + (int64_t)u * ppi;
        if (pix < p1) {
          V vo;
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            float v = (float)vg[u].e[e];
            if (has_act) v = tpg_act_grad(v, (float)vy[u].e[e], act, slope);
            if (c0 + e >= C) v = 0.f;
            vo.e[e] = (E)v;
            part[e] += v;
          }
          if (g) *reinterpret_cast<uint4*>(g + pix * gps_out + c0) = vo.u;  // (null: column sums only)
        }
      }
    }
  }
  if (!dbias) return;
  // LDS layout [pixel lane][channel]: sb[pl * nch * EPC + c]
#pragma unroll
  for (int e = 0; e < EPC; ++e)
    if (active) sb[pl * nch * EPC + c0 + e] = part[e];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int q = 0; q < ppi; ++q) s += sb[q * nch * EPC + c];
    atomicAdd(dbias + c, s);
  }
}

// Column sums: dbias[c] += sum over pixels of g (the bias gradient where no other launch of
// the fused backward summed it).  64 channels x 4 pixel lanes per block, any strides.
__global__ __launch_bounds__(256) void colsum_kernel(int N, int C, int H, int W, tpg_tensor g, float* dbias) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int64_t npix = (int64_t)N * H * W;
  float sum = 0.f;
  if (c < C) {
    for (int64_t pix = blockIdx.x * 4 + pl; pix < npix; pix += (int64_t)gridDim.x * 4) {
      const int n = (int)(pix / ((int64_t)H * W));
      const int rem = (int)(pix - (int64_t)n * H * W);
      const int h = rem / W, w = rem - h * W;
      sum += ld_any(g.data, g.dtype, n * g.stride[0] + c * g.stride[1] + h * g.stride[2] + w * g.stride[3]);
    }
  }
  red[pl][cl] = sum;
  __syncthreads();
  if (pl == 0 && c < C) atomicAdd(dbias + c, red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]);
}

// ------------------------------------------------------------ strided 4-D copy --
__global__ __launch_bounds__(256) void copy4d_kernel(int N, int C, int H, int W, tpg_tensor in, tpg_tensor out) {
  const int64_t total = (int64_t)N * C * H * W;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    // channel fastest (channels-last order)
    int c = (int)(idx % C);
    int64_t pix = idx / C;
    int w = (int)(pix % W);
    int64_t t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float v = ld_any(in.data, in.dtype, n * in.stride[0] + c * in.stride[1] + h * in.stride[2] + w * in.stride[3]);
    st_any(out.data, out.dtype, n * out.stride[0] + c * out.stride[1] + h * out.stride[2] + w * out.stride[3], v);
  }
}

// Pixel-group copy: one thread per (pixel, 8 consecutive channels), offsets computed once
// per thread (not per element).  Any input layout (NCHW images read coalesced along w) into
// a channels-last output; 16-byte loads / stores where both rows hold the whole group at
// 16-byte alignment and the dtypes are 16-bit.  (Concats into channel slices, to_cl.)
__global__ __launch_bounds__(256) void copy4d_grp_kernel(int N, int C, int H, int W, int G, tpg_tensor in,
                                                         tpg_tensor out, int vin, int vout) {
  const int total = N * H * W * G;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int gi = idx % G;
  const int pix = idx / G;
  const int w = pix % W, t = pix / W;
  const int h = t % H, n = t / H;
  const int c0 = gi * 8;
  const int nc = min(8, C - c0);
  const int64_t io = n * in.stride[0] + (int64_t)c0 * in.stride[1] + h * in.stride[2] + w * in.stride[3];
  const int64_t oo = n * out.stride[0] + (int64_t)c0 * out.stride[1] + h * out.stride[2] + w * out.stride[3];
  float v[8];
  if (vin && nc == 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(in.data) + io);
    const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint16_t b = (uint16_t)(q[e >> 1] >> (16 * (e & 1)));
      v[e] = in.dtype == TPG_BF16 ? __uint_as_float((uint32_t)b << 16) : (float)__builtin_bit_cast(_Float16, b);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < nc ? ld_any(in.data, in.dtype, io + e * in.stride[1]) : 0.f;
  }
  if (vout && nc == 8) {
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t lo, hi;
      if (out.dtype == TPG_BF16) {
        lo = __builtin_bit_cast(uint16_t, (__bf16)v[2 * e]);
        hi = __builtin_bit_cast(uint16_t, (__bf16)v[2 * e + 1]);
      } else {
        lo = __builtin_bit_cast(uint16_t, (_Float16)v[2 * e]);
        hi = __builtin_bit_cast(uint16_t, (_Float16)v[2 * e + 1]);
      }
      q[e] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out.data) + oo) = uint4{q[0], q[1], q[2], q[3]};
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e < nc) st_any(out.data, out.dtype, oo + e * out.stride[1], v[e]);
  }
}

// ------------------------------------------------------------------ tap folding --
// Thin-input convs (3-channel images): the taps of an FH x FW window are folded into the
// channel dimension, y[n][y'][x'][(fy*FW + fx)*C + c] = x[n][y'*sh + fy - pt][x'*sw + fx - pl][c]
// (zero outside), so the conv that follows reads 16-27 live channels per 32-channel MFMA
// k-step instead of 3 (the weights are a strided view of the same memory).  One thread per
// output (pixel, folded channel); the backward gathers dx from every folded copy.
__global__ __launch_bounds__(256) void fold_taps_kernel(int N, int C, int H, int W, int FH, int FW, int sh, int sw,
                                                        int pt, int pl, int OH, int OW, tpg_tensor x, tpg_tensor y) {
  const int CF = FH * FW * C;
  const int64_t total = (int64_t)N * OH * OW * CF;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int cf = (int)(idx % CF);
    const int64_t pix = idx / CF;
    const int ox = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int oy = (int)(t % OH), n = (int)(t / OH);
    const int tap = cf / C, c = cf - tap * C;
    const int iy = oy * sh + tap / FW - pt, ix = ox * sw + tap % FW - pl;
    float v = 0.f;
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      v = ld_any(x.data, x.dtype, n * x.stride[0] + c * x.stride[1] + iy * x.stride[2] + ix * x.stride[3]);
    st_any(y.data, y.dtype, n * y.stride[0] + cf * y.stride[1] + oy * y.stride[2] + ox * y.stride[3], v);
  }
}

__global__ __launch_bounds__(256) void unfold_taps_kernel(int N, int C, int H, int W, int FH, int FW, int sh, int sw,
                                                          int pt, int pl, int OH, int OW, tpg_tensor gy, tpg_tensor dx) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t pix = idx / C;
    const int ix = (int)(pix % W);
    const int64_t t = pix / W;
    const int iy = (int)(t % H), n = (int)(t / H);
    float acc = 0.f;
    for (int fy = 0; fy < FH; ++fy) {
      const int ny = iy + pt - fy;
      if (ny < 0 || ny % sh) continue;
      const int oy = ny / sh;
      if (oy >= OH) continue;
      for (int fx = 0; fx < FW; ++fx) {
        const int nx = ix + pl - fx;
        if (nx < 0 || nx % sw) continue;
        const int ox = nx / sw;
        if (ox >= OW) continue;
        const int cf = (fy * FW + fx) * C + c;
        acc += ld_any(gy.data, gy.dtype, n * gy.stride[0] + cf * gy.stride[1] + oy * gy.stride[2] + ox * gy.stride[3]);
      }
    }
    st_any(dx.data, dx.dtype, n * dx.stride[0] + c * dx.stride[1] + iy * dx.stride[2] + ix * dx.stride[3], acc);
  }
}

extern "C" int32_t tpg_fold_taps_impl(int32_t n, int32_t c, int32_t h, int32_t w, int32_t fh, int32_t fw, int32_t sh,
                                      int32_t sw, int32_t pt, int32_t pl, int32_t oh, int32_t ow, tpg_tensor x,
                                      tpg_tensor y, int32_t backward, hipStream_t s) {
  if (backward)
    hipLaunchKernelGGL(unfold_taps_kernel, dim3(grid_for((int64_t)n * h * w * c)), dim3(256), 0, s, n, c, h, w, fh, fw,
                       sh, sw, pt, pl, oh, ow, y, x);
  else
    hipLaunchKernelGGL(fold_taps_kernel, dim3(grid_for((int64_t)n * oh * ow * fh * fw * c)), dim3(256), 0, s, n, c, h,
                       w, fh, fw, sh, sw, pt, pl, oh, ow, x, y);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ LocalFuser --
struct FuseGeom {
  tpg_tensor part[4];
  int ph[4], pw[4], top[4], left[4];
};

__global__ __launch_bounds__(256) void fuse_fwd_kernel(int N, int C, int OH, int OW, FuseGeom g, tpg_tensor y,
                                                       uint8_t* amax) {
  const int64_t total = (int64_t)N * OH * OW * C;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(idx % C);
    int64_t pix = idx / C;
    int x = (int)(pix % OW);
    int64_t t = pix / OW;
    int yy = (int)(t % OH);
    int n = (int)(t / OH);
    float best = 0.f;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int py = yy - g.top[k], px = x - g.left[k];
      float v = 0.f;
      if ((unsigned)py < (unsigned)g.ph[k] && (unsigned)px < (unsigned)g.pw[k]) {
        const tpg_tensor& P = g.part[k];
        v = ld_any(P.data, P.dtype, n * P.stride[0] + c * P.stride[1] + py * P.stride[2] + px * P.stride[3]);
      }
      if (k == 0 || v > best || (v != v && best == best)) { best = v; arg = k; }
    }
    st_any(y.data, y.dtype, n * y.stride[0] + c * y.stride[1] + yy * y.stride[2] + x * y.stride[3], best);
    if (amax) amax[idx] = (uint8_t)arg;
  }
}

__global__ __launch_bounds__(256) void fuse_bwd_kernel(int N, int C, int OH, int OW, int k, tpg_tensor gy,
                                                       const uint8_t* amax, tpg_tensor dpart, int ph, int pw, int top,
                                                       int left) {
  const int64_t total = (int64_t)N * ph * pw * C;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(idx % C);
    int64_t pix = idx / C;
    int px = (int)(pix % pw);
    int64_t t = pix / pw;
    int py = (int)(t % ph);
    int n = (int)(t / ph);
    int yy = py + top, x = px + left;
    float v = 0.f;
    if ((unsigned)yy < (unsigned)OH && (unsigned)x < (unsigned)OW) {
      int64_t cidx = (((int64_t)n * OH + yy) * OW + x) * C + c;
      if (amax[cidx] == k)
        v = ld_any(gy.data, gy.dtype, n * gy.stride[0] + c * gy.stride[1] + yy * gy.stride[2] + x * gy.stride[3]);
    }
    st_any(dpart.data, dpart.dtype,
           n * dpart.stride[0] + c * dpart.stride[1] + py * dpart.stride[2] + px * dpart.stride[3], v);
  }
}

// ---------------------------------------------------------------------- maxout --
__global__ __launch_bounds__(256) void maxout_fwd_kernel(int B, int M, tpg_tensor x, tpg_tensor y, uint8_t* amax) {
  const int64_t total = (int64_t)B * M;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int b = (int)(idx / M), j = (int)(idx % M);
    float v0 = ld_any(x.data, x.dtype, b * x.stride[0] + (2 * j) * x.stride[1]);
    float v1 = ld_any(x.data, x.dtype, b * x.stride[0] + (2 * j + 1) * x.stride[1]);
    bool second = (v1 > v0) || (v1 != v1 && v0 == v0);
    st_any(y.data, y.dtype, b * y.stride[0] + j * y.stride[1], second ? v1 : v0);
    if (amax) amax[idx] = second ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void maxout_bwd_kernel(int B, int M, tpg_tensor gy, const uint8_t* amax,
                                                         tpg_tensor dx) {
  const int64_t total = (int64_t)B * 2 * M;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int b = (int)(idx / (2 * M)), i = (int)(idx % (2 * M));
    int j = i >> 1;
    float v = 0.f;
    if (amax[(int64_t)b * M + j] == (i & 1)) v = ld_any(gy.data, gy.dtype, b * gy.stride[0] + j * gy.stride[1]);
    st_any(dx.data, dx.dtype, b * dx.stride[0] + i * dx.stride[1], v);
  }
}

// -------------------------------------------------- reflection-pad gradient fold --
// dx[n, iy, ix, c] = sum of dpad at every padded position that reads (iy, ix).
__global__ __launch_bounds__(256) void reflect_fold_kernel(int N, int C, int H, int W, int pt, int pb, int pl, int pr,
                                                           tpg_tensor dpad, tpg_tensor dx) {
  const int64_t total = (int64_t)N * H * W * C;
  const int PH = H + pt + pb, PW = W + pl + pr;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(idx % C);
    int64_t pix = idx / C;
    int ix = (int)(pix % W);
    int64_t t = pix / W;
    int iy = (int)(t % H);
    int n = (int)(t / H);
    int ys[3], xs[3], ny = 0, nx = 0;
    ys[ny++] = iy + pt;
    if (iy >= 1 && iy <= pt) ys[ny++] = pt - iy;
    if (iy <= H - 2 && iy >= H - 1 - pb) { int q = 2 * H - 2 - iy + pt; if (q < PH) ys[ny++] = q; }
    xs[nx++] = ix + pl;
    if (ix >= 1 && ix <= pl) xs[nx++] = pl - ix;
    if (ix <= W - 2 && ix >= W - 1 - pr) { int q = 2 * W - 2 - ix + pl; if (q < PW) xs[nx++] = q; }
    float v = 0.f;
    for (int a = 0; a < ny; ++a)
      for (int b = 0; b < nx; ++b)
        v += ld_any(dpad.data, dpad.dtype,
                    n * dpad.stride[0] + c * dpad.stride[1] + ys[a] * dpad.stride[2] + xs[b] * dpad.stride[3]);
    st_any(dx.data, dx.dtype, n * dx.stride[0] + c * dx.stride[1] + iy * dx.stride[2] + ix * dx.stride[3], v);
  }
}

int launch_reflect_fold(int N, int C, int H, int W, int pt, int pb, int pl, int pr, const tpg_tensor& dpad,
                        const tpg_tensor& dx, hipStream_t s) {
  hipLaunchKernelGGL(reflect_fold_kernel, dim3(grid_for((int64_t)N * H * W * C)), dim3(256), 0, s, N, C, H, W, pt,
                     pb, pl, pr, dpad, dx);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------- Adam --
// torch.optim.Adam (amsgrad=False, maximize=False): g += wd * p; m = b1 m + (1-b1) g;
// v = b2 v + (1-b2) g^2; p -= lr / (1-b1^t) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
// The bias corrections come from a device state {step, 1-b1^t, sqrt(1-b2^t)} that
// adam_sched_kernel advances, so a captured hipGraph replays correct steps.
// st[3] != 0 (set by grad_finite_kernel for this step's gradients): the step is skipped --
// counter, moments and parameters stay as they are (torch.cuda.amp.GradScaler's skip).
__global__ void adam_sched_kernel(float* st, float b1, float b2, int32_t host_step) {
  if (st[3] != 0.f) return;
  const float t = host_step > 0 ? (float)host_step : st[0] + 1.f;
  st[0] = t;
  st[1] = 1.f - powf(b1, t);
  st[2] = sqrtf(1.f - powf(b2, t));
}

// (no FP contraction: the compiler fused differently in the scalar head, the unrolled body and
// the remainder loop, so an element's update depended by an ulp on where its bucket slice started)
__device__ __forceinline__ void adam_one(float& pv, float g, float gscale, float& mv, float& vv, float lr_bc1, float b1,
                                         float b2, float eps, float wd, float bc2s) {
#pragma clang fp contract(off)
  g *= gscale;
  if (wd != 0.f) g += wd * pv;
  mv = b1 * mv + (1.f - b1) * g;
  vv = b2 * vv + (1.f - b2) * g * g;
  pv = pv - lr_bc1 * mv / (sqrtf(vv) / bc2s + eps);
}

typedef float tpg_f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ tpg_f4 adam_ld(const float* p, int64_t i) {
  const tpg_f4* q = reinterpret_cast<const tpg_f4*>(p) + i;
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void adam_st(float* p, int64_t i, tpg_f4 v) {
  tpg_f4* q = reinterpret_cast<tpg_f4*>(p) + i;
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// head: elements before the first 16-byte boundary (a bucket slice of the flat buffers starts
// wherever its first parameter does; all four buffers share the misalignment), updated one per
// thread by block 0; the rest from p + head on in float4s (U of each operand in flight per thread)
template <bool NT, int U>
__global__ __launch_bounds__(256) void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ gr,
                                                   float* __restrict__ m, float* __restrict__ v, float lr, float b1,
                                                   float b2, float eps, float wd, const float* __restrict__ st,
                                                   float gscale, int head) {
  if (st[3] != 0.f) return;  // non-finite gradients this step (grad_finite_kernel)
  const float lr_bc1 = lr / st[1], bc2s = st[2];
  if (head > 0) {
    if (blockIdx.x == 0 && (int)threadIdx.x < head)
      adam_one(p[threadIdx.x], gr[threadIdx.x], gscale, m[threadIdx.x], v[threadIdx.x], lr_bc1, b1, b2, eps, wd, bc2s);
    p += head; gr += head; m += head; v += head; n -= head;
  }
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    tpg_f4 pv[U], g[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pv[u] = adam_ld<NT>(p, i + u * stride);
      g[u] = adam_ld<NT>(gr, i + u * stride);
      mv[u] = adam_ld<NT>(m, i + u * stride);
      vv[u] = adam_ld<NT>(v, i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = pv[u][e], me = mv[u][e], ve = vv[u][e];
        adam_one(pe, g[u][e], gscale, me, ve, lr_bc1, b1, b2, eps, wd, bc2s);
        pv[u][e] = pe; mv[u][e] = me; vv[u][e] = ve;
      }
      adam_st<NT>(p, i + u * stride, pv[u]);
      adam_st<NT>(m, i + u * stride, mv[u]);
      adam_st<NT>(v, i + u * stride, vv[u]);
    }
  }
  for (; i < n4; i += stride) {
    tpg_f4 pv = adam_ld<NT>(p, i), g = adam_ld<NT>(gr, i), mv = adam_ld<NT>(m, i), vv = adam_ld<NT>(v, i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], me = mv[e], ve = vv[e];
      adam_one(pe, g[e], gscale, me, ve, lr_bc1, b1, b2, eps, wd, bc2s);
      pv[e] = pe; mv[e] = me; vv[e] = ve;
    }
    adam_st<NT>(p, i, pv);
    adam_st<NT>(m, i, mv);
    adam_st<NT>(v, i, vv);
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    adam_one(p[i], gr[i], gscale, m[i], v[i], lr_bc1, b1, b2, eps, wd, bc2s);
}


// st[3] := 1 when any gradient element is inf / NaN (st[3] zeroed by a memset node first; every
// writer stores the same value, so the race is benign).  HBM-bound: 4 B per element.
__global__ __launch_bounds__(256) void grad_finite_kernel(int64_t n, const float* __restrict__ gr, float* st) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 g = reinterpret_cast<const float4*>(gr)[i];
    bad |= !(isfinite(g.x) && isfinite(g.y) && isfinite(g.z) && isfinite(g.w));
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) bad |= !isfinite(gr[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) st[3] = 1.f;
}

}  // namespace tpg

using namespace tpg;

// pixel-dense channels-last rows (channel stride 1, any pixel stride / alignment)
static bool pix_dense_any(const tpg_tensor& t, int h, int w) {
  return t.stride[1] == 1 && t.stride[2] == t.stride[3] * w && t.stride[0] == t.stride[2] * h;
}

// act_bwd grid shaping: pixels per lane, block cap
static int act_ppl() { return 4; }
static int act_cap() { return 1024; }


static bool pix_dense_vec(const tpg_tensor& t, int h, int w, int dtype, int c) {
  const int es = dtype != TPG_F32 ? 2 : 4, epc = 16 / es;
  if (t.dtype != dtype || t.stride[1] != 1) return false;
  const int64_t ps = t.stride[3];
  if (ps % epc || ps < (c + epc - 1) / epc * epc) return false;
  if (t.stride[2] != ps * w || t.stride[0] != ps * w * h) return false;
  return ((uintptr_t)t.data % 16) == 0;
}

namespace tpg {
// vector form plan: >= 4 pixels per lane (one unrolled iteration: small maps get enough
// blocks to hide the load latency), <= 1024 blocks (bounds the dbias atomics per channel);
// deterministic mode with a bias gradient: one block, so every dbias element gets ONE atomic
// add (a fixed-order sum)
int act_vec_plan(int64_t npix, int c, int dtype, bool dbias, ActVecArgs* a) {
  memset(a, 0, sizeof(*a));
  const int epc = dtype != TPG_F32 ? 8 : 4;
  const int ppi = 256 / ((c + epc - 1) / epc);
  const int64_t blocks = (dbias && deterministic()) ? 1 :
      std::max<int64_t>(1, std::min<int64_t>((npix + act_ppl() * ppi - 1) / (act_ppl() * ppi), act_cap()));
  a->npix = npix;
  a->C = c;
  a->pix_per_block = (npix + blocks - 1) / blocks;
  a->blocks = (int)blocks;
  return 0;
}

// the vector form's arguments when it applies (0), else 1
int act_vec_args(int n, int c, int h, int w, int act, float slope, const tpg_tensor& gy, const tpg_tensor& y,
                 const tpg_tensor& g, float* dbias, ActVecArgs* a) {
  const int dt = g.dtype;
  const int epc = dt != TPG_F32 ? 8 : 4;
  if (!(c <= 1024 && (c + epc - 1) / epc <= 256 && pix_dense_vec(gy, h, w, dt, c) && pix_dense_vec(g, h, w, dt, c) &&
        (act == TPG_ACT_NONE || pix_dense_vec(y, h, w, dt, c))))
    return 1;
  act_vec_plan((int64_t)n * h * w, c, dt, dbias != nullptr, a);
  a->act = act; a->slope = slope;
  a->gy = gy.data; a->gps = gy.stride[3]; a->y = y.data; a->yps = y.stride[3]; a->g = g.data; a->gps_out = g.stride[3];
  a->dbias = dbias;
  return 0;
}

template <int NG>
static void launch_act_vec_t(const Grouped<ActVecArgs, NG>& g, int blocks, int dtype, hipStream_t s) {
  if (dtype == TPG_F16) hipLaunchKernelGGL((act_bwd_vec_kernel<_Float16, NG>), dim3(blocks), dim3(256), 0, s, g);
  else if (dtype == TPG_BF16) hipLaunchKernelGGL((act_bwd_vec_kernel<__bf16, NG>), dim3(blocks), dim3(256), 0, s, g);
  else if constexpr (NG == 1) hipLaunchKernelGGL((act_bwd_vec_kernel<float, NG>), dim3(blocks), dim3(256), 0, s, g);
}

int launch_act_vec(const ActVecArgs& a, int dtype, hipStream_t s) {
  Grouped<ActVecArgs, 1> g;
  g.a[0] = a; g.boff[0] = 0; g.boff[1] = a.blocks; g.nm = 1;
  launch_act_vec_t<1>(g, a.blocks, dtype, s);
  return (int)hipGetLastError();
}

int launch_act_vec_group(const ActVecArgs* a, int n, int dtype, hipStream_t s) {
  if (n < 2 || n > TPG_GROUP_MAX || (dtype != TPG_BF16 && dtype != TPG_F16)) return -1;
  Grouped<ActVecArgs, TPG_GROUP_MAX> g;
  memset(&g, 0, sizeof(g));
  int blocks = 0;
  for (int m = 0; m < n; ++m) {
    g.a[m] = a[m];
    g.boff[m] = blocks;
    blocks += a[m].blocks;
  }
  g.boff[n] = blocks;
  g.nm = n;
  launch_act_vec_t<TPG_GROUP_MAX>(g, blocks, dtype, s);
  return (int)hipGetLastError();
}
}  // namespace tpg

extern "C" int32_t tpg_act_bwd_impl(int32_t n, int32_t c, int32_t h, int32_t w, int32_t act, float slope,
                                     tpg_tensor gy, tpg_tensor y, tpg_tensor g, float* dbias, hipStream_t s) {
  const int dt = g.dtype;
  ActVecArgs a;
  if (act_vec_args(n, c, h, w, act, slope, gy, y, g, dbias, &a) == 0) return launch_act_vec(a, dt, s);
  int64_t npix = (int64_t)n * h * w;
  if (c <= 256 && pix_dense_any(gy, h, w) && pix_dense_any(g, h, w) &&
      (act == TPG_ACT_NONE || pix_dense_any(y, h, w))) {
    const int ppi = 256 / c;
    const int64_t blocks = (dbias && deterministic()) ? 1 :
        std::max<int64_t>(1, std::min<int64_t>((npix + 8 * ppi - 1) / (8 * ppi), 4 * act_cap()));
    const int64_t ppb = (npix + blocks - 1) / blocks;
    hipLaunchKernelGGL(act_bwd_rows_kernel, dim3((int)blocks), dim3(256), 0, s, npix, c, act, slope, gy, y, g, dbias,
                       ppb);
    return (int)hipGetLastError();
  }
  int gx = (int)std::min<int64_t>((npix + 63) / 64, 2048);
  if (gx < 1 || (dbias && deterministic())) gx = 1;
  dim3 grid(gx, (c + 63) / 64);
  hipLaunchKernelGGL(act_bwd_kernel, grid, dim3(256), 0, s, n, c, h, w, act, slope, gy, y, g, dbias);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_colsum_impl(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor g, float* dbias,
                                    hipStream_t s) {
  const int64_t npix = (int64_t)n * h * w;
  // pixel-dense 16-bit rows: the activation-backward vector kernel with no output (16-byte loads,
  // several pixels in flight per lane; the generic loop below divided 64-bit pixel indices per
  // element and ran at ~2 TB/s -- 30 us per ConvTranspose2d bias once its gradient arrived masked)
  if (g.dtype != TPG_F32 && c <= 1024 && (c + 7) / 8 <= 256 && pix_dense_vec(g, h, w, g.dtype, c)) {
    ActVecArgs a;
    memset(&a, 0, sizeof(a));
    act_vec_plan(npix, c, g.dtype, true, &a);
    a.act = TPG_ACT_NONE; a.slope = 0.f;
    a.gy = g.data; a.gps = g.stride[3]; a.y = g.data; a.yps = g.stride[3];
    a.g = nullptr; a.gps_out = 0;
    a.dbias = dbias;
    return launch_act_vec(a, g.dtype, s);
  }
  int gx = (int)std::min<int64_t>((npix + 63) / 64, 1024);
  if (gx < 1 || deterministic()) gx = 1;
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, (c + 63) / 64), dim3(256), 0, s, n, c, h, w, g, dbias);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_copy4d_impl(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor in, tpg_tensor out,
                                    hipStream_t s) {
  const int G = (c + 7) / 8;
  if ((int64_t)n * h * w * G < (1ll << 31) - 256) {
    // 16-byte groups: 16-bit dtype, channel stride 1, every group start 16-byte aligned
    auto vec = [&](const tpg_tensor& t) {
      return (t.dtype == TPG_BF16 || t.dtype == TPG_F16) && t.stride[1] == 1 && t.stride[0] % 8 == 0 &&
             t.stride[2] % 8 == 0 && t.stride[3] % 8 == 0 && ((uintptr_t)t.data & 15) == 0;
    };
    const int total = n * h * w * G;
    hipLaunchKernelGGL(copy4d_grp_kernel, dim3((total + 255) / 256), dim3(256), 0, s, n, c, h, w, G, in, out,
                       (int)vec(in), (int)vec(out));
  } else {
    hipLaunchKernelGGL(copy4d_kernel, dim3(grid_for((int64_t)n * c * h * w)), dim3(256), 0, s, n, c, h, w, in, out);
  }
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_fuse_fwd_impl(int32_t n, int32_t c, int32_t oh, int32_t ow, const tpg_tensor* parts,
                                      const int32_t* ph, const int32_t* pw, const int32_t* top, const int32_t* left,
                                      tpg_tensor y, uint8_t* amax, hipStream_t s) {
  FuseGeom g;
  for (int k = 0; k < 4; ++k) {
    g.part[k] = parts[k]; g.ph[k] = ph[k]; g.pw[k] = pw[k]; g.top[k] = top[k]; g.left[k] = left[k];
  }
  hipLaunchKernelGGL(fuse_fwd_kernel, dim3(grid_for((int64_t)n * oh * ow * c)), dim3(256), 0, s, n, c, oh, ow, g, y,
                     amax);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_fuse_bwd_impl(int32_t n, int32_t c, int32_t oh, int32_t ow, tpg_tensor gy, const uint8_t* amax,
                                      const tpg_tensor* dparts, const int32_t* ph, const int32_t* pw,
                                      const int32_t* top, const int32_t* left, hipStream_t s) {
  for (int k = 0; k < 4; ++k) {
    if (!dparts[k].data) continue;
    hipLaunchKernelGGL(fuse_bwd_kernel, dim3(grid_for((int64_t)n * ph[k] * pw[k] * c)), dim3(256), 0, s, n, c, oh,
                       ow, k, gy, amax, dparts[k], ph[k], pw[k], top[k], left[k]);
  }
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_maxout_fwd_impl(int32_t b, int32_t m, tpg_tensor x, tpg_tensor y, uint8_t* amax, hipStream_t s) {
  hipLaunchKernelGGL(maxout_fwd_kernel, dim3(grid_for((int64_t)b * m)), dim3(256), 0, s, b, m, x, y, amax);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_maxout_bwd_impl(int32_t b, int32_t m, tpg_tensor gy, const uint8_t* amax, tpg_tensor dx,
                                        hipStream_t s) {
  hipLaunchKernelGGL(maxout_bwd_kernel, dim3(grid_for((int64_t)b * 2 * m)), dim3(256), 0, s, b, m, gy, amax, dx);
  return (int)hipGetLastError();
}

// state: device float[4] {step, 1-b1^t, sqrt(1-b2^t), -}; host_step > 0 sets the step
// explicitly, 0 advances the device counter (graph replay).
extern "C" int32_t tpg_adam_impl(int64_t numel, float* param, const float* grad, float* m, float* v, float lr,
                                  float b1, float b2, float eps, float wd, int32_t host_step, float gscale,
                                  float* state, hipStream_t s) {
  // argument checks before any launch: an error must not advance the device step counter
  // the four buffers must share their offset inside a 16-byte chunk (elements of one flat layout)
  const uintptr_t mis = (uintptr_t)param % 16;
  if ((uintptr_t)param % 4 || (uintptr_t)grad % 16 != mis || (uintptr_t)m % 16 != mis || (uintptr_t)v % 16 != mis)
    return -1;
  if (host_step >= 0) hipLaunchKernelGGL(adam_sched_kernel, dim3(1), dim3(1), 0, s, state, b1, b2, host_step);
  if (numel <= 0) return (int)hipGetLastError();
  const int head = (int)std::min<int64_t>(numel, mis ? (int64_t)((16 - mis) / 4) : 0);
  // (nontemporal loads / stores, up to 64 Ki blocks: 0.85 -> 0.71 ms for G's 138 M parameters,
  // 4.5 -> 5.4 TB/s; the step 32.44 -> 32.34 ms, profiles/r04/ab_adam_pack.txt)
  int blocks = (int)std::min<int64_t>(((numel - head) / 4 + 255) / 256, 65536);
  if (blocks < 1) blocks = 1;
  auto k = adam_kernel<true, 2>;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, s, numel, param, grad, m, v, lr, b1, b2, eps, wd, state,
                     gscale, head);
  return (int)hipGetLastError();
}

extern "C" int32_t tpg_grad_check_impl(int64_t numel, const float* grad, float* state, hipStream_t s) {
  if (((uintptr_t)grad) % 16) return -1;
  hipError_t e = hipMemsetAsync(state + 3, 0, sizeof(float), s);
  if (e) return (int)e;
  if (numel <= 0) return 0;
  int blocks = (int)std::min<int64_t>((numel / 4 + 255) / 256, 2048);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(grad_finite_kernel, dim3(blocks), dim3(256), 0, s, numel, grad, state);
  return (int)hipGetLastError();
}

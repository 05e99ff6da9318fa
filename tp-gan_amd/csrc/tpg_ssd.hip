// SSD landmark head of the MobileNetV2 pretraining: the target assignment +
// loss of MultiTaskLoss (MobileNetV2.py:342-534) and the confidence filter + greedy NMS of
// MultiTaskDecoder (:536-649), batched over images (the reference takes batch 1 and loops over
// points with .item(); tp-gan_amd/MobileNetV2.py keeps that CPU semantics and calls these for
// device tensors).
//
// ssd_loss_fwd: one block per image, everything in LDS (n <= TPG_SSD_MAXN anchors):
//   d[l][i]  = ||pred_i - true_l||  (four landmarks)
//   thr[l]   = k-th smallest d[l][:], k = int(ratio * n)     (topk(k, largest=False)[0].max())
//   label[i] = argmin over {l : d[l][i] <= thr[l]} of d[l][i] (first landmark on ties), else -1
//   background: the -1 anchors, or -- when there are more than int(#positives * ratio_nb) of
//     them -- the ones holding the smallest of the caller's uniform keys (a draw without
//     replacement; the keys come from the caller so the RNG stays torch's)
//   terms: per landmark the location MSE (clamped to [0, 1] by the image size) and the class
//     CE of its positives, the background CE, and alpha * loc + beta * cls (fixed-order block
//     sums: deterministic).
// ssd_loss_bwd: one thread per (image, anchor): the gradients of mean_b(total_b) w.r.t. the
//   predicted locations (through the clamp) and the class logits.
// ssd_decode: one block per (image, class): softmax confidence > threshold, sorted by score
//   (then index), greedy suppression of the points within nms_thr (<=) of each kept one, the
//   first top_k kept.
#include "tpg_internal.h"
#include <math.h>

namespace tpg {

static constexpr int SSD_T = 256;

__device__ __forceinline__ int ssd_pow2(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

// ascending bitonic sort of (key, idx) pairs by key, then idx (n2 a power of two)
__device__ void ssd_sort(float* key, int* idx, int n2) {
  for (int k = 2; k <= n2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n2; i += SSD_T) {
        const int p = i ^ j;
        if (p > i) {
          const float a = key[i], b = key[p];
          const int ia = idx[i], ib = idx[p];
          const bool gt = a > b || (a == b && ia > ib);
          if (gt == ((i & k) == 0)) {
            key[i] = b; key[p] = a;
            idx[i] = ib; idx[p] = ia;
          }
        }
      }
      __syncthreads();
    }
}

// fixed-order block sum of NV floats per thread (result valid in thread 0)
template <int NV>
__device__ void ssd_bsum(float (&v)[NV], float* red) {
  for (int q = 0; q < NV; ++q) red[q * SSD_T + threadIdx.x] = v[q];
  __syncthreads();
  for (int s = SSD_T / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int q = 0; q < NV; ++q) red[q * SSD_T + threadIdx.x] += red[q * SSD_T + threadIdx.x + s];
    __syncthreads();
  }
  for (int q = 0; q < NV; ++q) v[q] = red[q * SSD_T];
  __syncthreads();
}

__device__ __forceinline__ float ssd_lse(const float* x, int C) {
  float m = x[0];
  for (int c = 1; c < C; ++c) m = fmaxf(m, x[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += expf(x[c] - m);
  return m + logf(s);
}

struct SsdArgs {
  int B, n, C, k;
  const float* pred;   // (B, n, 2)
  const float* cls;    // (B, n, C)
  const float* truth;  // (B, 8)
  float w, h;  // image width / height (locations are divided by them, as MobileNetV2.py:472-473)
  double ratio_nb;
  float alpha, beta;
  const float* keys;   // (B, n) uniform [0, 1)
  int* labels;         // (B, n)
  unsigned char* sel;  // (B, n) background drawn
  float* terms;        // (B, TPG_SSD_TERMS)
};

__global__ __launch_bounds__(SSD_T) void ssd_loss_fwd_kernel(const SsdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, n = a.n, tid = threadIdx.x;
  const int n2 = ssd_pow2(n);
  float* d = smem;                                      // [4][n]
  float* key = d + 4 * n;                               // [n2]
  int* idx = reinterpret_cast<int*>(key + n2);          // [n2]
  int* lab = idx + n2;                                  // [n]
  float* red = reinterpret_cast<float*>(lab + n);       // [11][SSD_T]
  __shared__ float thr[4];
  __shared__ int cnt[5];
  const float* P = a.pred + (int64_t)b * n * 2;
  const float* T = a.truth + (int64_t)b * 8;
  for (int i = tid; i < n; i += SSD_T) {
    const float px = P[2 * i], py = P[2 * i + 1];
    for (int l = 0; l < 4; ++l) {
      const float dx = px - T[2 * l], dy = py - T[2 * l + 1];
      d[l * n + i] = sqrtf(dx * dx + dy * dy);
    }
  }
  if (tid < 5) cnt[tid] = 0;
  __syncthreads();
  for (int l = 0; l < 4; ++l) {
    for (int i = tid; i < n2; i += SSD_T) {
      key[i] = i < n ? d[l * n + i] : INFINITY;
      idx[i] = i;
    }
    __syncthreads();
    ssd_sort(key, idx, n2);
    if (tid == 0) thr[l] = key[a.k - 1];
    __syncthreads();
  }
  int* L = a.labels + (int64_t)b * n;
  for (int i = tid; i < n; i += SSD_T) {
    int best = -1;
    float bd = INFINITY;
    for (int l = 0; l < 4; ++l) {
      const float v = d[l * n + i];
      if (v <= thr[l] && v < bd) { best = l; bd = v; }
    }
    lab[i] = best;
    L[i] = best;
    atomicAdd(&cnt[best < 0 ? 4 : best], 1);  // (integer counts: order-free)
  }
  __syncthreads();
  // background draw
  const int nbg = cnt[4];
  const int cap = (int)floor((double)(n - nbg) * a.ratio_nb);
  const bool all_bg = nbg <= cap;
  unsigned char* S = a.sel + (int64_t)b * n;
  if (!all_bg) {
    const float* K = a.keys + (int64_t)b * n;
    for (int i = tid; i < n2; i += SSD_T) {
      key[i] = i < n ? (lab[i] < 0 ? K[i] : 2.f) : 3.f;
      idx[i] = i;
    }
    __syncthreads();
    ssd_sort(key, idx, n2);
    for (int i = tid; i < n; i += SSD_T) S[i] = 0;
    __syncthreads();
    for (int r = tid; r < cap; r += SSD_T) S[idx[r]] = 1;  // (the cap smallest keys: all background)
  } else {
    for (int i = tid; i < n; i += SSD_T) S[i] = lab[i] < 0 ? 1 : 0;
  }
  __syncthreads();
  // loss partials: se[4], ce[4], bg ce, nsel
  const float tcx[4] = {fminf(fmaxf(T[0] / a.w, 0.f), 1.f), fminf(fmaxf(T[2] / a.w, 0.f), 1.f),
                        fminf(fmaxf(T[4] / a.w, 0.f), 1.f), fminf(fmaxf(T[6] / a.w, 0.f), 1.f)};
  const float tcy[4] = {fminf(fmaxf(T[1] / a.h, 0.f), 1.f), fminf(fmaxf(T[3] / a.h, 0.f), 1.f),
                        fminf(fmaxf(T[5] / a.h, 0.f), 1.f), fminf(fmaxf(T[7] / a.h, 0.f), 1.f)};
  float v[10];
  for (int q = 0; q < 10; ++q) v[q] = 0.f;
  const float* X = a.cls + (int64_t)b * n * a.C;
  for (int i = tid; i < n; i += SSD_T) {
    const int l = lab[i];
    const bool s = S[i] != 0;
    if (l < 0 && !s) continue;
    const float* x = X + (int64_t)i * a.C;
    const float lse = ssd_lse(x, a.C);
    if (l >= 0) {
      const float pcx = fminf(fmaxf(P[2 * i] / a.w, 0.f), 1.f), pcy = fminf(fmaxf(P[2 * i + 1] / a.h, 0.f), 1.f);
      const float ex = pcx - tcx[l], ey = pcy - tcy[l];
      for (int q = 0; q < 4; ++q)
        if (q == l) { v[q] += ex * ex + ey * ey; v[4 + q] += lse - x[q]; }
    } else {
      v[8] += lse - x[4];
      v[9] += 1.f;
    }
  }
  ssd_bsum<10>(v, red);
  if (tid == 0) {
    float* o = a.terms + (int64_t)b * TPG_SSD_TERMS;
    float loc = 0.f, cls = 0.f;
    for (int l = 0; l < 4; ++l) {
      const float c = (float)cnt[l];
      const float ll = c > 0 ? v[l] / (2.f * c) : 0.f, cl = c > 0 ? v[4 + l] / c : 0.f;
      o[1 + l] = ll;
      o[5 + l] = cl;
      o[11 + l] = c;
      loc += ll;
      cls += cl;
    }
    const float cb = v[9] > 0 ? v[8] / v[9] : 0.f;
    o[9] = cb;
    o[10] = v[9];
    o[0] = a.alpha * loc + a.beta * (cb + cls);
  }
}

__global__ __launch_bounds__(SSD_T) void ssd_loss_bwd_kernel(const SsdArgs a, const float* __restrict__ gout,
                                                             float* __restrict__ dloc, float* __restrict__ dcls) {
  const int64_t t = (int64_t)blockIdx.x * SSD_T + threadIdx.x;
  if (t >= (int64_t)a.B * a.n) return;
  const int b = (int)(t / a.n);
  const int l = a.labels[t];
  const bool s = a.sel[t] != 0;
  const float* o = a.terms + (int64_t)b * TPG_SSD_TERMS;
  const float g = gout[0] / (float)a.B;  // d mean_b / d total_b
  const float* P = a.pred + t * 2;
  const float* T = a.truth + (int64_t)b * 8;
  float gx = 0.f, gy = 0.f;
  if (l >= 0) {
    const float c = o[11 + l];
    const float ux = P[0] / a.w, uy = P[1] / a.h;
    const float pcx = fminf(fmaxf(ux, 0.f), 1.f), pcy = fminf(fmaxf(uy, 0.f), 1.f);
    const float tcx = fminf(fmaxf(T[2 * l] / a.w, 0.f), 1.f), tcy = fminf(fmaxf(T[2 * l + 1] / a.h, 0.f), 1.f);
    // d(se / 2c)/d pc = (pc - tc) / c; clamp passes the gradient on [0, 1] (inclusive, as torch)
    if (ux >= 0.f && ux <= 1.f) gx = g * a.alpha * (pcx - tcx) / c / a.w;
    if (uy >= 0.f && uy <= 1.f) gy = g * a.alpha * (pcy - tcy) / c / a.h;
  }
  dloc[t * 2] = gx;
  dloc[t * 2 + 1] = gy;
  const float* x = a.cls + t * a.C;
  float* dx = dcls + t * a.C;
  if (l < 0 && !s) {
    for (int c = 0; c < a.C; ++c) dx[c] = 0.f;
    return;
  }
  const int tgt = l >= 0 ? l : 4;
  const float cntv = l >= 0 ? o[11 + l] : o[10];
  const float scale = g * a.beta / cntv;
  const float lse = ssd_lse(x, a.C);
  for (int c = 0; c < a.C; ++c) dx[c] = scale * (expf(x[c] - lse) - (c == tgt ? 1.f : 0.f));
}

struct SsdDecArgs {
  int B, n, C, top_k;
  const float* loc;  // (B, n, 2)
  const float* cls;  // (B, n, C)
  float conf, nms2;  // confidence threshold, squared NMS distance
  int* keep;         // (B, C, top_k) anchor index or -1
  float* score;      // (B, C, top_k)
};

__global__ __launch_bounds__(SSD_T) void ssd_decode_kernel(const SsdDecArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, c = blockIdx.y, n = a.n, tid = threadIdx.x;
  const int n2 = ssd_pow2(n);
  float* key = smem;                                    // [n2] -score
  int* idx = reinterpret_cast<int*>(key + n2);          // [n2]
  int* alive = idx + n2;                                // [n2] sorted position alive
  __shared__ int pick;
  const float* X = a.cls + (int64_t)b * n * a.C;
  for (int i = tid; i < n2; i += SSD_T) {
    float k = INFINITY;
    if (i < n) {
      const float* x = X + (int64_t)i * a.C;
      const float s = expf(x[c] - ssd_lse(x, a.C));
      if (s > a.conf) k = -s;
    }
    key[i] = k;
    idx[i] = i;
  }
  __syncthreads();
  ssd_sort(key, idx, n2);
  for (int i = tid; i < n2; i += SSD_T) alive[i] = key[i] < INFINITY;
  __syncthreads();
  const float* Lc = a.loc + (int64_t)b * n * 2;
  int* K = a.keep + ((int64_t)b * a.C + c) * a.top_k;
  float* S = a.score + ((int64_t)b * a.C + c) * a.top_k;
  for (int r = 0; r < a.top_k; ++r) {
    if (tid == 0) {
      int p = -1;
      for (int i = 0; i < n2 && p < 0; ++i)
        if (alive[i]) p = i;  // (the highest remaining score: sorted order)
      pick = p;
      K[r] = p < 0 ? -1 : idx[p];
      S[r] = p < 0 ? 0.f : -key[p];
    }
    __syncthreads();
    const int p = pick;
    if (p < 0) break;
    const float qx = Lc[2 * idx[p]], qy = Lc[2 * idx[p] + 1];
    for (int i = tid; i < n2; i += SSD_T) {
      if (!alive[i]) continue;
      const float dx = Lc[2 * idx[i]] - qx, dy = Lc[2 * idx[i] + 1] - qy;
      if (i == p || dx * dx + dy * dy <= a.nms2) alive[i] = 0;
    }
    __syncthreads();
  }
}

static size_t ssd_fwd_lds(int n) {
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  return (size_t)4 * n * 4 + (size_t)n2 * 8 + (size_t)n * 4 + (size_t)10 * SSD_T * 4;
}

int launch_ssd_loss_fwd(int B, int n, int C, int k, const float* pred, const float* cls, const float* truth, float width,
                        float height, double ratio_nb, float alpha, float beta, const float* keys, int* labels,
                        unsigned char* sel, float* terms, hipStream_t s) {
  SsdArgs a{B, n, C, k, pred, cls, truth, width, height, ratio_nb, alpha, beta, keys, labels, sel, terms};
  const size_t lds = ssd_fwd_lds(n);
  // (the largest dynamic size any n <= TPG_SSD_MAXN needs: the whole 160 KiB would leave no room
  // for the kernel's static LDS, and the failed attribute call makes the launch report an error)
  static bool once = ((void)hipFuncSetAttribute((const void*)ssd_loss_fwd_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                (int)ssd_fwd_lds(TPG_SSD_MAXN)), true);
  (void)once;
  hipLaunchKernelGGL(ssd_loss_fwd_kernel, dim3(B), dim3(SSD_T), lds, s, a);
  return (int)hipGetLastError();
}

int launch_ssd_loss_bwd(int B, int n, int C, const float* pred, const float* cls, const float* truth, float width,
                        float height, float alpha, float beta, const int* labels, const unsigned char* sel,
                        const float* terms, const float* gout, float* dloc, float* dcls, hipStream_t s) {
  SsdArgs a{B, n, C, 0, pred, cls, truth, width, height, 0.0, alpha, beta, nullptr,
            const_cast<int*>(labels), const_cast<unsigned char*>(sel), const_cast<float*>(terms)};
  const int64_t tot = (int64_t)B * n;
  hipLaunchKernelGGL(ssd_loss_bwd_kernel, dim3((unsigned)((tot + SSD_T - 1) / SSD_T)), dim3(SSD_T), 0, s, a, gout,
                     dloc, dcls);
  return (int)hipGetLastError();
}

int launch_ssd_decode(int B, int n, int C, const float* loc, const float* cls, float conf, float nms_thr, int top_k,
                      int* keep, float* score, hipStream_t s) {
  SsdDecArgs a{B, n, C, top_k, loc, cls, conf, nms_thr * nms_thr, keep, score};
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  const size_t lds = (size_t)n2 * 12;
  static bool once = ((void)hipFuncSetAttribute((const void*)ssd_decode_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, TPG_SSD_MAXN * 12), true);
  (void)once;
  hipLaunchKernelGGL(ssd_decode_kernel, dim3(B, C), dim3(SSD_T), lds, s, a);
  return (int)hipGetLastError();
}

}  // namespace tpg

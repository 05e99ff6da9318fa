// C-ABI of libtpgan_hip.so (include/tpgan.h): turns a tpg_conv_desc into implicit-GEMM
// problems (tpg_igemm.hip) and weight-gradient problems (tpg_wgrad.hip).
//
//  op          Conv2d                                  ConvTranspose2d
//  forward     direct form: rows = output pixels,      sub-pixel form: one launch per output
//              A = x gathered at oy*s + r - pad        parity class, taps that reach it
//  bwd_data    sub-pixel form over the input grid,     direct form over the input grid,
//              A = g                                   A = g gathered at iy*s + r - pad
//  bwd_filter  P = g (output grid), Q = x gathered     P = x (input grid), Q = g gathered
//
// A full-kernel conv (Linear fc1 as a 8x8 conv on an 8x8 map) and a transposed conv of a
// 1x1 map (deconv_8) become plain GEMMs over flattened (y, x, c) channels when the
// tensors are dense NHWC ("composite" channels).
#include "tpg_internal.h"
#include "../../include/tpgan.h"
#include <stdarg.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include <string>
#include <vector>
#include <algorithm>

extern "C" int32_t tpg_act_bwd_impl(int32_t, int32_t, int32_t, int32_t, int32_t, float, tpg_tensor, tpg_tensor,
                                     tpg_tensor, float*, hipStream_t);
extern "C" int32_t tpg_copy4d_impl(int32_t, int32_t, int32_t, int32_t, tpg_tensor, tpg_tensor, hipStream_t);
extern "C" int32_t tpg_fold_taps_impl(int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t,
                                      int32_t, int32_t, int32_t, tpg_tensor, tpg_tensor, int32_t, hipStream_t);
extern "C" int32_t tpg_fuse_fwd_impl(int32_t, int32_t, int32_t, int32_t, const tpg_tensor*, const int32_t*,
                                      const int32_t*, const int32_t*, const int32_t*, tpg_tensor, uint8_t*, hipStream_t);
extern "C" int32_t tpg_fuse_bwd_impl(int32_t, int32_t, int32_t, int32_t, tpg_tensor, const uint8_t*, const tpg_tensor*,
                                      const int32_t*, const int32_t*, const int32_t*, const int32_t*, hipStream_t);
extern "C" int32_t tpg_maxout_fwd_impl(int32_t, int32_t, tpg_tensor, tpg_tensor, uint8_t*, hipStream_t);
extern "C" int32_t tpg_maxout_bwd_impl(int32_t, int32_t, tpg_tensor, const uint8_t*, tpg_tensor, hipStream_t);
extern "C" int32_t tpg_adam_impl(int64_t, float*, const float*, float*, float*, float, float, float, float, float,
                                  int32_t, float, float*, hipStream_t);

namespace tpg {
int launch_reflect_fold(int N, int C, int H, int W, int pt, int pb, int pl, int pr, const tpg_tensor& dpad,
                        const tpg_tensor& dx, hipStream_t s);
}

using namespace tpg;

static thread_local std::string g_err;
static int g_det = 0;  // tpg_set_deterministic

// Share of the chip an op plans its grid for: 1, or 4 when desc.flags has TPG_FLAG_CONCURRENT
// (the op runs beside other streams' work, e.g. the four local pathways: fewer K / pixel
// splits, since the other streams fill the CUs a split would).  Set per entry point.
static thread_local int g_share = 1;
// small-map convs with several taps on the pointwise kernel (tpg_pw.hip; 0: the halo kernel, A/B)
#ifndef TPG_PW_TAPS
#define TPG_PW_TAPS 1
#endif
// forced k-step split of the forward / input-gradient launches (desc.data_ksplit; 0 = planner)
static thread_local int g_data_ks = 0;
// paired last k-step in the halo kernel (HaloArgs.half); TPG_HALO_PAIR=0 (read once at load, so
// every packed image and plan of the process agree) turns it off for same-box A/B runs
static const int g_halo_pair = [] {
  const char* e = getenv("TPG_HALO_PAIR");
  return (e && e[0] == '0') ? 0 : 1;
}();
// wgrad_rh: MFMAs of all-padding blocks of edge tiles skipped (WgradRHArgs.skip); TPG_RH_SKIP=0
// (read once at load) runs them, for same-box A/B runs
static const int g_rh_skip = [] {
  const char* e = getenv("TPG_RH_SKIP");
  return (e && e[0] == '0') ? 0 : 1;
}();
// kernel of the small-map multi-tap forward / input-gradient plans (desc.data_algo; 0 = rule)
static thread_local int g_data_algo = 0;
struct ShareScope {
  int prev, prev_ks, prev_algo;
  explicit ShareScope(const tpg_conv_desc* d) : prev(g_share), prev_ks(g_data_ks), prev_algo(g_data_algo) {
    g_data_ks = (d && d->data_ksplit > 0) ? d->data_ksplit : 0;
    g_data_algo = (d && (d->data_algo == 1 || d->data_algo == 2)) ? d->data_algo : 0;
    // (1/2 .. 1/8 measured within run-to-run spread, profiles/r02c/share)
    g_share = (d && (d->flags & TPG_FLAG_CONCURRENT)) ? 4 : 1;
  }
  ~ShareScope() { g_share = prev; g_data_ks = prev_ks; g_data_algo = prev_algo; }
};

int tpg::deterministic() { return __atomic_load_n(&g_det, __ATOMIC_RELAXED); }

static int32_t fail(int32_t code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int tpg::record_error(int code, const char* msg) {
  g_err = msg;
  return code;
}

static int32_t hip_check(int e, const char* what) {
  if (e == 0) return 0;
  return fail(e > 0 ? e : -100, "%s failed: %s", what, e > 0 ? hipGetErrorString((hipError_t)e) : "bad config");
}

// ------------------------------------------------------------------ launch groups --
// Between tpg_group_begin and tpg_group_end the halo conv, its split-K epilogue, the
// tap-flattened weight gradient and the vector activation backward are recorded instead of
// launched, tagged with the member (tpg_group_member) whose call issued them.  At the end,
// when every member issued the same sequence of kernel instances, position j of all members
// runs as ONE grouped launch (tpg_internal.h Grouped); otherwise, and for anything a member
// launches outside those four kernels (which first flushes the record), the launches run
// one by one in their original order.  Members must be independent of each other.
struct GLaunch {
  int kind;  // 1 halo, 2 epilogue, 3 wgrad2, 4 act_bwd (vector form)
  int member;
  hipStream_t s;
  int dtype, cfg, bm, bn;
  bool mask;
  HaloArgs h;
  EpiArgs e;
  Wgrad2Args w;
  ActVecArgs v;
};
struct GroupRec {
  bool active = false;
  int member = 0;
  std::vector<GLaunch> q;
};
static thread_local GroupRec g_grp;

static int run_one(const GLaunch& L) {
  switch (L.kind) {
    case 1: return launch_halo(L.h, L.dtype, L.cfg, L.s, L.mask);
    case 2: return launch_epilogue(L.e, L.s);
    case 3: return launch_wgrad2(L.w, L.dtype, L.cfg, L.bm, L.bn, L.s);
    default: return launch_act_vec(L.v, L.dtype, L.s);
  }
}

// run the recorded launches one by one, in order (the record stays active)
static int group_flush() {
  if (!g_grp.active || g_grp.q.empty()) return 0;
  int rc = 0;
  for (const GLaunch& L : g_grp.q)
    if (!rc) rc = run_one(L);
  g_grp.q.clear();
  return rc;
}

// same kernel instance up to what a grouped launch adapts per member (the halo kernel's halo
// capacity class: the grouped launch takes the largest the members need)
static bool same_instance(const GLaunch& a, const GLaunch& b) {
  if (a.kind != b.kind || a.s != b.s || a.dtype != b.dtype || a.mask != b.mask) return false;
  if (a.kind == 1) return (a.cfg >= 40) == (b.cfg >= 40) && (a.cfg >= 40 ? a.cfg == b.cfg : a.cfg % 8 == b.cfg % 8);
  return a.cfg == b.cfg && a.bm == b.bm && a.bn == b.bn;
}

// Members run their own launches in order; across members any interleaving is valid.  Each
// round takes the first unfinished member's next launch and groups it with every other
// member whose next launch is the same instance.
static int group_run_merged() {
  std::vector<std::vector<const GLaunch*>> by(std::max(g_grp.member, 0) + 1);
  for (const GLaunch& L : g_grp.q) by[L.member].push_back(&L);
  by.erase(std::remove_if(by.begin(), by.end(), [](const std::vector<const GLaunch*>& v) { return v.empty(); }),
           by.end());
  const int nmem = (int)by.size();
  std::vector<size_t> head(nmem, 0);
  int rc = 0;
  for (;;) {
    int lead = -1;
    for (int m = 0; m < nmem && lead < 0; ++m)
      if (head[m] < by[m].size()) lead = m;
    if (lead < 0) break;
    const GLaunch& L0 = *by[lead][head[lead]];
    std::vector<int> mem;
    for (int m = lead; m < nmem && (int)mem.size() < TPG_GROUP_MAX; ++m)
      if (head[m] < by[m].size() && same_instance(*by[m][head[m]], L0)) mem.push_back(m);
    const int n = (int)mem.size();
    int r = -1;
    if (n >= 2) {
      if (L0.kind == 1) {
        HaloArgs a[TPG_GROUP_MAX];
        for (int k = 0; k < n; ++k) a[k] = by[mem[k]][head[mem[k]]]->h;
        r = launch_halo_group(a, n, L0.dtype, L0.cfg, L0.s, L0.mask);
      } else if (L0.kind == 2) {
        EpiArgs a[TPG_GROUP_MAX];
        for (int k = 0; k < n; ++k) a[k] = by[mem[k]][head[mem[k]]]->e;
        r = launch_epilogue_group(a, n, L0.s);
      } else if (L0.kind == 3) {
        Wgrad2Args a[TPG_GROUP_MAX];
        for (int k = 0; k < n; ++k) a[k] = by[mem[k]][head[mem[k]]]->w;
        r = launch_wgrad2_group(a, n, L0.dtype, L0.cfg, L0.bm, L0.bn, L0.s);
      } else {
        ActVecArgs a[TPG_GROUP_MAX];
        for (int k = 0; k < n; ++k) a[k] = by[mem[k]][head[mem[k]]]->v;
        r = launch_act_vec_group(a, n, L0.dtype, L0.s);
      }
    }
    if (r == -1) {  // a single member, or no grouped build of this instance: one by one
      r = 0;
      for (int k = 0; k < n && !r; ++k) r = run_one(*by[mem[k]][head[mem[k]]]);
    }
    if (r && !rc) rc = r;
    for (int k = 0; k < n; ++k) ++head[mem[k]];
  }
  g_grp.q.clear();
  return rc;
}

static GLaunch& grec(int kind, hipStream_t s, int dtype) {
  g_grp.q.emplace_back();
  GLaunch& L = g_grp.q.back();
  L.kind = kind; L.member = std::max(g_grp.member, 0); L.s = s; L.dtype = dtype;
  L.cfg = L.bm = L.bn = 0; L.mask = false;
  return L;
}

static int do_halo(const HaloArgs& h, int dtype, int cfg, hipStream_t s, bool mask) {
  if (h.pw > 0 && !mask) {  // (not a launch-group kernel: the recorded launches go first)
    const int rc = group_flush();
    if (rc) return rc;
    const int e = launch_pw(h, dtype, s);
    if (e != -1) return e;
    // the pointwise kernel refused the plan (its 32-bit byte-extent / stride conditions are
    // stricter than the planner's element-count checks): the halo kernel of the same plan and
    // packed weight image takes it
    HaloArgs h2 = h;
    h2.pw = 0;
    return launch_halo(h2, dtype, cfg, s, false);
  }
  if (!g_grp.active) return launch_halo(h, dtype, cfg, s, mask);
  GLaunch& L = grec(1, s, dtype);
  L.h = h; L.cfg = cfg; L.mask = mask;
  return 0;
}
static int do_epilogue(const EpiArgs& e, hipStream_t s) {
  if (!g_grp.active) return launch_epilogue(e, s);
  GLaunch& L = grec(2, s, e.dtype);
  L.e = e;
  return 0;
}
static int do_wgrad2(const Wgrad2Args& w, int dtype, int cfg, int bm, int bn, hipStream_t s) {
  if (!g_grp.active || !w.bflat) {
    const int rc = group_flush();
    return rc ? rc : launch_wgrad2(w, dtype, cfg, bm, bn, s);
  }
  GLaunch& L = grec(3, s, dtype);
  L.w = w; L.cfg = cfg; L.bm = bm; L.bn = bn;
  return 0;
}

// any other launch: the recorded ones go first
#define TPG_GROUP_SYNC()             \
  do {                               \
    const int grc_ = group_flush();  \
    if (grc_) return hip_check(grc_, "group flush"); \
  } while (0)

static int do_act_bwd(int n, int c, int h, int w, int act, float slope, const tpg_tensor& gy, const tpg_tensor& y,
                      const tpg_tensor& g, float* dbias, hipStream_t s) {
  if (g_grp.active) {
    ActVecArgs v;
    if (act_vec_args(n, c, h, w, act, slope, gy, y, g, dbias, &v) == 0) {
      GLaunch& L = grec(4, s, g.dtype);
      L.v = v;
      return 0;
    }
    const int rc = group_flush();
    if (rc) return rc;
  }
  return tpg_act_bwd_impl(n, c, h, w, act, slope, gy, y, g, dbias, s);
}

extern "C" void tpg_group_begin(void) {
  group_flush();
  g_grp.active = true;
  g_grp.member = -1;
  g_grp.q.clear();
}

extern "C" void tpg_group_member(void) {
  if (g_grp.active) ++g_grp.member;
}

extern "C" int32_t tpg_group_end(void) {
  if (!g_grp.active) return 0;
  const int rc = g_grp.q.empty() ? 0 : group_run_merged();
  g_grp.active = false;
  g_grp.q.clear();
  return hip_check(rc, "grouped launch");
}

static inline int esize(int dtype) { return dtype == TPG_F32 ? 4 : 2; }
static inline bool half16(int dtype) { return dtype == TPG_BF16 || dtype == TPG_F16; }  // 16-bit MFMA operands
static inline int64_t rup(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int pmod(int a, int m) { return ((a % m) + m) % m; }

// ------------------------------------------------------------------ problem plans --
struct Prob {
  IgemmArgs a;
  PackArgs pk;
  int cfg = 0;
  size_t wp_bytes = 0, sk_bytes = 0;
  bool halo = false;          // run on the halo-tiled direct-conv kernel
  HaloArgs h;
  int hcfg = -1;
  size_t g_wp = 0, g_sk = 0;  // generic-kernel sizes, kept for the run-time fallback
};

static int choose_cfg(int nout) {
  if (nout <= 16) return 0;
  if (nout <= 32) return 1;
  if (nout <= 64) return 2;
  if (nout <= 96) return 3;
  if (nout <= 128) return 4;
  if (nout > 192 && nout <= 224) return 5;
  return 4;
}

// fill unit / tile / split-K bookkeeping once geometry, C, Nout and taps are known
static void finish(Prob& P, int dtype, int M) {
  IgemmArgs& a = P.a;
  const int upk = half16(dtype) ? 4 : 2;
  a.upt = cdiv(std::max(a.C, 1), 16);
  a.nunits = a.ntaps > 0 ? (int)rup((int64_t)a.ntaps * a.upt, upk) : 0;
  a.M = M;
  P.cfg = choose_cfg(a.Nout);
  const int bn = igemm_cfg_bn(P.cfg), bm = igemm_cfg_bm(P.cfg);
  const int npad = (int)rup(a.Nout, bn);
  P.wp_bytes = (size_t)rup((int64_t)npad * a.nunits * 16 * esize(dtype), 256);
  const int nkt = a.nunits / upk;
  const int blocks = cdiv(M, bm) * (npad / bn);
  a.ksplit = 1;
  a.kt_per_split = std::max(nkt, 1);
  if (!deterministic() && (g_data_ks > 0 || (blocks < 480 / g_share && nkt >= 8))) {
    int ks = g_data_ks > 0 ? std::min(g_data_ks, std::max(nkt, 1))  // (an autotuner's pick)
                           : std::min(cdiv(960 / g_share, blocks), nkt / 4);
    if (ks > 1) {
      a.kt_per_split = cdiv(nkt, ks);
      a.ksplit = cdiv(nkt, a.kt_per_split);
    }
  }
  P.sk_bytes = a.ksplit > 1 ? (size_t)rup((int64_t)M * a.Nout * 4, 256) : 0;
  a.div_jw.init(a.JW);
  a.div_jhjw.init(a.JH * a.JW);
  PackArgs& k = P.pk;
  k.Npad = npad;
  k.Nreal = a.Nout;
  k.nunits = a.nunits;
  k.upt = a.upt;
  k.ntaps = a.ntaps;
  k.Creal = a.C;
  k.dtype = dtype;
}

// direct form: output grid OH x OW (one class), A pixel = o*s + (r - pad)
static Prob direct_prob(int N, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  Prob P;
  memset(&P.a, 0, sizeof(P.a));
  memset(&P.pk, 0, sizeof(P.pk));
  IgemmArgs& a = P.a;
  a.JH = OH; a.JW = OW; a.oy0 = 0; a.ox0 = 0; a.osy = 1; a.osx = 1; a.ist_h = sh; a.ist_w = sw;
  a.ntaps = kh * kw;
  for (int r = 0; r < kh; ++r)
    for (int s = 0; s < kw; ++s) {
      int t = r * kw + s;
      a.dy[t] = (int8_t)(r - pt); a.dx[t] = (int8_t)(s - pl);
      P.pk.tr[t] = (int8_t)r; P.pk.ts[t] = (int8_t)s;
    }
  (void)N;
  return P;
}

// sub-pixel form: out grid OH x OW, class (py, px); A pixel = j + (p + pad - r)/s
static std::vector<Prob> subpixel_probs(int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  std::vector<Prob> v;
  for (int py = 0; py < sh; ++py)
    for (int px = 0; px < sw; ++px) {
      if (py >= OH || px >= OW) continue;
      Prob P;
      memset(&P.a, 0, sizeof(P.a));
      memset(&P.pk, 0, sizeof(P.pk));
      IgemmArgs& a = P.a;
      a.JH = cdiv(OH - py, sh); a.JW = cdiv(OW - px, sw);
      a.oy0 = py; a.ox0 = px; a.osy = sh; a.osx = sw; a.ist_h = 1; a.ist_w = 1;
      int t = 0;
      for (int r = 0; r < kh; ++r) {
        if (pmod(py + pt - r, sh) != 0) continue;
        for (int s = 0; s < kw; ++s) {
          if (pmod(px + pl - s, sw) != 0) continue;
          a.dy[t] = (int8_t)((py + pt - r) / sh);
          a.dx[t] = (int8_t)((px + pl - s) / sw);
          P.pk.tr[t] = (int8_t)r; P.pk.ts[t] = (int8_t)s;
          ++t;
        }
      }
      a.ntaps = t;
      v.push_back(P);
    }
  return v;
}

// stride 2 on maps of <= 64 x 64 outputs (64x64: conv2
// s2 dgrad 0.096 -> 0.039 ms, step -0.3 ms); stride 4 likewise (deconv_32, D_and_G_model.py:220:
// sixteen parity classes, four of them without a tap: 0.138 -> 0.023 ms).  (Thin layers on
// larger maps stay in class form: deconv_128, 16 -> 8 channels at 128x128, measured 54 -> 63 us
// in the zero-insertion form.)
static bool use_dilated(int OH, int OW, int kh, int kw, int sh, int sw, int pad_mode) {
  return sh == sw && (sh == 2 || sh == 4) && pad_mode == TPG_PAD_ZERO && kh <= 5 && kw <= 5 &&
         OH * OW <= 64 * 64;
}

// zero-insertion form of the same problem (stride-2, small maps): ONE unit-stride problem
// over the whole OH x OW grid reading A dilated by s (A pixel (y + pt - r) / s when
// divisible, else zero), all taps; 4x the MACs of the class form, one launch instead of
// four on maps where each class launch is mostly fixed cost
static Prob dilated_prob(int OH, int OW, int kh, int kw, int s, int pt, int pl) {
  Prob P;
  memset(&P.a, 0, sizeof(P.a));
  memset(&P.pk, 0, sizeof(P.pk));
  IgemmArgs& a = P.a;
  a.JH = OH; a.JW = OW; a.oy0 = 0; a.ox0 = 0; a.osy = 1; a.osx = 1; a.ist_h = 1; a.ist_w = 1;
  a.dil = s;
  int t = 0;
  for (int r = 0; r < kh; ++r)
    for (int c = 0; c < kw; ++c) {
      a.dy[t] = (int8_t)(pt - r);
      a.dx[t] = (int8_t)(pl - c);
      P.pk.tr[t] = (int8_t)r; P.pk.ts[t] = (int8_t)c;
      ++t;
    }
  a.ntaps = t;
  return P;
}

static bool dense_nhwc(const tpg_tensor& t, int C, int H, int W) {
  return t.stride[1] == 1 && t.stride[3] == C && t.stride[2] == (int64_t)W * C;
}

static bool vec_ok(const tpg_tensor& t, int dtype) {
  const int es = esize(dtype);
  if (t.stride[1] != 1) return false;
  if (((uintptr_t)t.data) % 16) return false;
  for (int i : {0, 2, 3})
    if ((t.stride[i] * es) % 16) return false;
  return true;
}

// geometry of a full-kernel conv (kernel = input map, 1x1 output) or a transposed conv of a
// 1x1 map (output = kernel), no padding: the composite-channel GEMM forms
static bool gemm_form(const tpg_conv_desc* d) {
  if (d->pad_t || d->pad_b || d->pad_l || d->pad_r || d->pad_mode) return false;
  if (!d->transposed) return d->in_h == d->kh && d->in_w == d->kw && d->out_h == 1 && d->out_w == 1;
  return d->in_h == 1 && d->in_w == 1 && d->out_h == d->kh && d->out_w == d->kw;
}
static bool big_taps(const tpg_conv_desc* d) { return d->kh * d->kw > TPG_MAX_TAPS; }

static int32_t check_desc(const tpg_conv_desc* d) {
  if (!d) return fail(-1, "null descriptor");
  if (d->n <= 0 || d->in_c <= 0 || d->out_c <= 0 || d->kh <= 0 || d->kw <= 0) return fail(-2, "bad sizes");
  if (d->stride_h <= 0 || d->stride_w <= 0) return fail(-2, "bad stride");
  // empty maps, and (Conv2d) a kernel larger than the padded input, which C's truncating
  // division would otherwise turn into a 0- or 1-pixel output (torch rejects both)
  if (d->in_h <= 0 || d->in_w <= 0 || d->out_h <= 0 || d->out_w <= 0) return fail(-2, "empty spatial map");
  if (!d->transposed && (d->in_h + d->pad_t + d->pad_b < d->kh || d->in_w + d->pad_l + d->pad_r < d->kw))
    return fail(-6, "kernel %dx%d larger than the padded input", d->kh, d->kw);
  if (d->dtype != TPG_F32 && d->dtype != TPG_BF16 && d->dtype != TPG_F16) return fail(-3, "bad dtype %d", d->dtype);
  // more taps than the tap tables hold: only the full-kernel GEMM forms (fc1 / deconv_8 at
  // 256x256: 16x16 kernels on a 16x16 map or from a 1x1 map), which need no tap table
  if (d->kh * d->kw > TPG_MAX_TAPS && !gemm_form(d))
    return fail(-4, "kernel %dx%d has more than %d taps", d->kh, d->kw, TPG_MAX_TAPS);
  if (d->transposed) {
    if (d->pad_mode != TPG_PAD_ZERO) return fail(-5, "reflect padding is only defined for Conv2d");
    int nh = (d->in_h - 1) * d->stride_h - d->pad_t - d->pad_b + d->kh;
    int nw = (d->in_w - 1) * d->stride_w - d->pad_l - d->pad_r + d->kw;
    if (d->out_h < nh || d->out_w < nw || d->out_h >= nh + d->stride_h || d->out_w >= nw + d->stride_w)
      return fail(-6, "ConvTranspose2d output %dx%d inconsistent with geometry (natural %dx%d)", d->out_h, d->out_w, nh, nw);
  } else {
    int oh = (d->in_h + d->pad_t + d->pad_b - d->kh) / d->stride_h + 1;
    int ow = (d->in_w + d->pad_l + d->pad_r - d->kw) / d->stride_w + 1;
    if (oh != d->out_h || ow != d->out_w) return fail(-6, "Conv2d output %dx%d != %dx%d", d->out_h, d->out_w, oh, ow);
    if (d->pad_mode == TPG_PAD_REFLECT &&
        (d->pad_t >= d->in_h || d->pad_b >= d->in_h || d->pad_l >= d->in_w || d->pad_r >= d->in_w))
      return fail(-7, "reflection padding must be smaller than the input");
  }
  if (std::max(std::abs(d->pad_t), std::abs(d->pad_l)) > 100 || d->kh > 64 || d->kw > 64) return fail(-8, "geometry out of range");
  return 0;
}

// Route a unit-stride (sub-)grid problem to the halo kernel.  Tile choice: a TH x TW tile
// of one image (large maps) or IMG whole images per 256-row block (small maps), minimising
// computed rows x taps plus staged halo pixels; then a split over k-steps when the grid
// has too few blocks to fill the chip (fp32 partial slices, summed by the epilogue).
static void maybe_halo(Prob& P, int dtype, int N) {
  IgemmArgs& a = P.a;
  // unit-stride grids, and stride 2 in both directions (halo (2·th + k − 2) x (2·tw + k − 2))
  const int S = a.ist_h;
  if (a.ntaps < 1 || a.C < 1 || a.ist_h != a.ist_w || (S != 1 && S != 2)) return;
  int dymin = 127, dymax = -128, dxmin = 127, dxmax = -128;
  for (int t = 0; t < a.ntaps; ++t) {
    dymin = std::min<int>(dymin, a.dy[t]); dymax = std::max<int>(dymax, a.dy[t]);
    dxmin = std::min<int>(dxmin, a.dx[t]); dxmax = std::max<int>(dxmax, a.dx[t]);
  }
  const int sy = dymax - dymin + 1, sx = dxmax - dxmin + 1;
  if (sy > 7 || sx > 7) return;
  const int JH = a.JH, JW = a.JW;
  // output channels per block first: the 512-row tile (halo up to 1024 pixels) serves the
  // thin layers (BN 64 / 80) of the large maps, where 256 rows run only 8-10 MFMAs per wave
  // between tap barriers; it needs >= 512 blocks (two rounds of the chip) without a k split
  int bn;
  if (a.Nout <= 32) bn = 32;
  else if (a.Nout <= 64) bn = 64;
  else if (a.Nout <= 80) bn = 80;
  else if (a.Nout <= 96) bn = 96;
  else if (a.Nout <= 128) bn = 128;
  else if (a.Nout > 192 && a.Nout <= 208) bn = 208;  // (BN 224 on 4 x 2 waves measured 2 % slower, r04)
  else {
    // fewest padded columns among the 128 / 192 / 224 tiles, the wider tile on ties
    // (measured: enhance_16 768->768 at 16x16 -24 %, the 8x8 576-channel layers +6 µs)
    int64_t best = -1;
    for (int c : {224, 192, 128}) {
      const int64_t pad = rup(a.Nout, c);
      if (best < 0 || pad < best) { best = pad; bn = c; }
    }
  }
  // (not for deep inputs: conv5_0's 206 -> 64 forward measured 0.43 -> 0.46 ms with it, against
  // add_128 0.59 -> 0.49 and conv0_res 0.35 -> 0.27)
  if (S == 2 && bn > 128) bn = 128;  // (the 1024-pixel halo leaves LDS for 128-row weight slices)
  const int bm = (S == 1 && halo_cfg512(bn) >= 0 && dtype != TPG_F32 && (int64_t)N * JH * JW >= 512 * 512 &&
                  JW >= 64 && cdiv(a.Nout, bn) == 1 && a.C <= 128) ? 512 : 256;
  const int HCAP = (bm == 512 || S == 2) ? 1024 : 5 * 128;
  int bth = 0, btw = 0, bimg = 0;
  int64_t bcost = -1;
  auto consider = [&](int th, int tw, int img) {
    if (th < 1 || tw < 1 || img < 1 || th * tw * img > bm) return;
    const int hpi = ((th - 1) * S + sy) * ((tw - 1) * S + sx);
    if ((int64_t)img * hpi > HCAP) return;
    const int64_t nsub = (int64_t)N * cdiv(JH, th) * cdiv(JW, tw);
    const int64_t blocks = (nsub + img - 1) / img;
    const int64_t cost = blocks * ((int64_t)bm * a.ntaps + (int64_t)img * hpi);
    if (bcost < 0 || cost < bcost) { bcost = cost; bth = th; btw = tw; bimg = img; }
  };
  if (JH * JW <= bm)
    for (int img = std::min(bm / (JH * JW), N); img >= 1; --img) consider(JH, JW, img);
  for (int tw : {JW, 64, 48, 40, 32, 24, 16, 8}) {
    if (tw > JW || tw > bm) continue;
    const int thmax = std::min(JH, bm / tw);
    if (thmax < 1) continue;
    consider(cdiv(JH, cdiv(JH, thmax)), tw, 1);
    // (stride 2: the tallest tile's halo may not fit; shorter ones, whole rows per block)
    if (S > 1)
      for (int th = thmax - 1; th >= 1 && th * tw * 2 >= bm / 2; --th) consider(th, tw, 1);
  }
  if (bcost < 0) return;
  if (a.Nout <= 32) bn = 32;
  else if (a.Nout <= 64) bn = 64;
  // (whole 16-pixel rows: the masked-gradient mode DMAs y into the halo buffer 16 pixels per
  // wave instruction)
  const int hcap = (int)rup((int64_t)bimg * ((bth - 1) * S + sy) * ((btw - 1) * S + sx), 16);
  const int hl = std::max(3, cdiv(hcap * 4, 512));
  const int cfg = bm == 512 ? halo_cfg512(bn) : halo_cfg(S == 2 ? 8 : hl, bn);
  if (cfg < 0) return;
  HaloArgs& h = P.h;
  memset(&h, 0, sizeof(h));
  const int ks_elems = half16(dtype) ? 32 : 16;
  h.A_H = a.A_H; h.A_W = a.A_W; h.C = a.C;
  h.nks = cdiv(a.C, ks_elems);
  h.ntaps = a.ntaps;
  // (16-bit: a last k-step with <= 16 live channels runs two taps per MFMA; never on the
  // pointwise kernel, which needs C % 32 == 0)
  h.half = (half16(dtype) && g_halo_pair && a.C % 32 != 0 && a.C % 32 <= 16) ? 1 : 0;
  h.dymin = dymin; h.dxmin = dxmin;
  h.TH = bth; h.TW = btw; h.IMG = bimg; h.SH = S; h.SW = S; h.dil = a.dil;
  h.HH = (bth - 1) * S + sy; h.HW = (btw - 1) * S + sx;
  h.hcap = hcap;
  for (int t = 0; t < a.ntaps; ++t) h.toff[t] = (a.dy[t] - dymin) * h.HW + (a.dx[t] - dxmin);
  h.pad_mode = a.pad_mode;
  h.N = N; h.JH = JH; h.JW = JW;
  h.tiles_h = cdiv(JH, bth); h.tiles_w = cdiv(JW, btw);
  h.fd_hp.init(h.HH * h.HW); h.fd_hw.init(h.HW);
  h.fd_tiles.init(h.tiles_h * h.tiles_w); h.fd_tilesw.init(h.tiles_w);
  h.fd_thw.init(bth * btw); h.fd_tw.init(btw);
  h.BN = bn; h.ntiles = cdiv(a.Nout, bn); h.Nout = a.Nout;
  h.oy0 = a.oy0; h.ox0 = a.ox0; h.osy = a.osy; h.osx = a.osx;
  // split over k-steps until the grid covers the chip (each split >= 4 pipeline steps)
  const int64_t base = (((int64_t)N * h.tiles_h * h.tiles_w + bimg - 1) / bimg) * h.ntiles;
  int ks = 1;
  constexpr int split_below = 256, split_to = 256, split_steps = 4;  // (swept in round 2: best)
  // (deterministic mode: no k-split at all, so a sample's outputs are summed in the same
  // order whatever the batch size — the DP run then matches the 1-GPU run at its global batch)
  if (base < split_below / g_share && !deterministic()) {
    const int kps_min = cdiv(split_steps, a.ntaps);
    ks = (int)std::min<int64_t>(cdiv(split_to / g_share, (int)base), std::max(1, h.nks / kps_min));
  }
  if (g_data_ks > 0 && !deterministic()) ks = std::min(g_data_ks, h.nks);  // (an autotuner's pick)
  // one tap (1x1 convs, stride 1 or 2) on whole 32-channel k-steps: the pointwise GEMM kernel,
  // whose 4-stage DMA ring hides the loads this kernel exposes every k-step when there is only
  // one tap per step; the largest of its tiles that still gives a chip's worth of blocks, and a
  // k split only for the few-block problems
  // Several taps: the same kernel (tap-shifted A rows by DMA, no reuse of a halo across taps)
  // where the halo grid is too small for the chip and would split K and the input is at most 256
  // channels deep (measured: local_20 128 ch 0.034 -> 0.021 ms, ResNet-50 l2 3x3 0.028 -> 0.018;
  // 512 / 768-channel maps slower, they keep the halo); desc.data_algo overrides (autotuner)
  const bool small_map = a.ntaps > 1 && (g_data_algo == 2 || (g_data_algo == 0 && TPG_PW_TAPS &&
                                                              base < split_below / g_share && a.C <= 256));
  h.pw = 0;
  if ((a.ntaps == 1 || small_map) && a.dil <= 1 && half16(dtype) && a.C % 32 == 0 && bn % 64 == 0 && bn <= 192) {
    const int64_t M = (int64_t)N * JH * JW;
    int64_t bb = 0;
    for (int c = 1; c <= 4; ++c) {
      if (pw_tile_bn(c) > bn || bn % pw_tile_bn(c)) continue;
      const int64_t blocks = cdiv(M, pw_tile_bm(c)) * (int64_t)cdiv(a.Nout, pw_tile_bn(c));
      if (blocks > bb) { h.pw = c; bb = blocks; }
      if (blocks >= 240 / g_share) { h.pw = c; bb = blocks; break; }
    }
    ks = 1;
    if (bb < 128 / g_share && !deterministic()) ks = (int)std::min<int64_t>(cdiv(256 / g_share, (int)bb), h.nks / 8);
    if (g_data_ks > 0 && !deterministic()) ks = std::min(g_data_ks, h.nks);
  }
  h.kps = cdiv(h.nks, std::max(ks, 1));
  h.ksplit = cdiv(h.nks, h.kps);
  P.halo = true;
  P.hcfg = cfg;
  P.g_wp = P.wp_bytes;
  P.g_sk = P.sk_bytes;
  P.wp_bytes = (size_t)rup((int64_t)halo_wp_bytes(h.nks, h.ntaps, bn, h.ntiles, h.half), 256);
  P.pk.hnks = h.nks;
  P.pk.half = h.half;
  P.sk_bytes = h.ksplit > 1 ? (size_t)rup((int64_t)h.ksplit * a.M * a.Nout * 4, 256) : 0;
}

// ---- forward plans
static std::vector<Prob> plan_fwd(const tpg_conv_desc* d, bool composite) {
  std::vector<Prob> v;
  if (!d->transposed) {
    if (composite) {
      Prob P = direct_prob(d->n, 1, 1, 1, 1, 1, 1, 0, 0);
      P.a.C = d->kh * d->kw * d->in_c;
      P.a.A_H = 1; P.a.A_W = 1;
      P.pk.cmode = 2; P.pk.nmode = 0; P.pk.comp_kw = d->kw; P.pk.comp_c = d->in_c;
      P.a.Nout = d->out_c;
      finish(P, d->dtype, d->n);
      v.push_back(P);
    } else {
      Prob P = direct_prob(d->n, d->out_h, d->out_w, d->kh, d->kw, d->stride_h, d->stride_w, d->pad_t, d->pad_l);
      P.a.C = d->in_c; P.a.A_H = d->in_h; P.a.A_W = d->in_w; P.a.Nout = d->out_c;
      P.a.pad_mode = d->pad_mode;
      P.pk.nmode = 0; P.pk.cmode = 1;
      finish(P, d->dtype, d->n * d->out_h * d->out_w);
      maybe_halo(P, d->dtype, d->n);
      v.push_back(P);
    }
  } else {
    if (composite) {
      Prob P = direct_prob(d->n, 1, 1, 1, 1, 1, 1, 0, 0);
      P.a.C = d->in_c; P.a.A_H = 1; P.a.A_W = 1;
      P.a.Nout = d->kh * d->kw * d->out_c;
      P.pk.nmode = 2; P.pk.cmode = 0; P.pk.comp_kw = d->kw; P.pk.comp_c = d->out_c;
      finish(P, d->dtype, d->n);
      v.push_back(P);
    } else {
      if (use_dilated(d->out_h, d->out_w, d->kh, d->kw, d->stride_h, d->stride_w, d->pad_mode)) {
        Prob P = dilated_prob(d->out_h, d->out_w, d->kh, d->kw, d->stride_h, d->pad_t, d->pad_l);
        P.a.C = d->in_c; P.a.A_H = d->in_h; P.a.A_W = d->in_w; P.a.Nout = d->out_c;
        P.pk.nmode = 1; P.pk.cmode = 0;
        finish(P, d->dtype, d->n * P.a.JH * P.a.JW);
        maybe_halo(P, d->dtype, d->n);
        if (P.halo) {
          v.push_back(P);
          return v;
        }
      }
      for (Prob& P : subpixel_probs(d->out_h, d->out_w, d->kh, d->kw, d->stride_h, d->stride_w, d->pad_t, d->pad_l)) {
        P.a.C = d->in_c; P.a.A_H = d->in_h; P.a.A_W = d->in_w; P.a.Nout = d->out_c;
        P.pk.nmode = 1; P.pk.cmode = 0;
        finish(P, d->dtype, d->n * P.a.JH * P.a.JW);
        maybe_halo(P, d->dtype, d->n);
        v.push_back(P);
      }
    }
  }
  return v;
}

static bool fwd_composite(const tpg_conv_desc* d, const tpg_tensor* x, const tpg_tensor* y) {
  if (!d->transposed) {
    if (d->in_h != d->kh || d->in_w != d->kw || d->out_h != 1 || d->out_w != 1) return false;
    if (d->pad_t || d->pad_b || d->pad_l || d->pad_r || d->pad_mode) return false;
    if (d->kh == 1 && d->kw == 1) return false;
    return !x || dense_nhwc(*x, d->in_c, d->in_h, d->in_w);
  }
  if (d->in_h != 1 || d->in_w != 1 || d->out_h != d->kh || d->out_w != d->kw) return false;
  if (d->pad_t || d->pad_b || d->pad_l || d->pad_r) return false;
  if (d->kh == 1 && d->kw == 1) return false;
  return !y || dense_nhwc(*y, d->out_c, d->out_h, d->out_w);
}

// ---- input-gradient plans (geometry of the op's forward; for reflect, the padded input)
static std::vector<Prob> plan_bwd_data(const tpg_conv_desc* d, bool composite) {
  std::vector<Prob> v;
  if (!d->transposed) {
    if (composite) {  // dX[n][(y,x,ci)] = sum_co g[n][co] W[co][ci][y][x]
      Prob P = direct_prob(d->n, 1, 1, 1, 1, 1, 1, 0, 0);
      P.a.C = d->out_c; P.a.A_H = 1; P.a.A_W = 1;
      P.a.Nout = d->kh * d->kw * d->in_c;
      P.pk.nmode = 2; P.pk.cmode = 0; P.pk.comp_kw = d->kw; P.pk.comp_c = d->in_c;
      finish(P, d->dtype, d->n);
      v.push_back(P);
    } else {
      const bool refl = d->pad_mode == TPG_PAD_REFLECT;
      const int IH = refl ? d->in_h + d->pad_t + d->pad_b : d->in_h;
      const int IW = refl ? d->in_w + d->pad_l + d->pad_r : d->in_w;
      const int pt = refl ? 0 : d->pad_t, pl = refl ? 0 : d->pad_l;
      if (use_dilated(IH, IW, d->kh, d->kw, d->stride_h, d->stride_w, 0)) {
        Prob P = dilated_prob(IH, IW, d->kh, d->kw, d->stride_h, pt, pl);
        P.a.C = d->out_c; P.a.A_H = d->out_h; P.a.A_W = d->out_w; P.a.Nout = d->in_c;
        P.pk.nmode = 1; P.pk.cmode = 0;
        finish(P, d->dtype, d->n * P.a.JH * P.a.JW);
        maybe_halo(P, d->dtype, d->n);
        if (P.halo) {
          v.push_back(P);
          return v;
        }
      }
      for (Prob& P : subpixel_probs(IH, IW, d->kh, d->kw, d->stride_h, d->stride_w, pt, pl)) {
        P.a.C = d->out_c; P.a.A_H = d->out_h; P.a.A_W = d->out_w; P.a.Nout = d->in_c;
        P.pk.nmode = 1; P.pk.cmode = 0;
        finish(P, d->dtype, d->n * P.a.JH * P.a.JW);
        maybe_halo(P, d->dtype, d->n);
        v.push_back(P);
      }
    }
  } else {
    if (composite) {  // dx[n][ci] = sum_{y,x,co} g[n][(y,x,co)] W[ci][co][y][x]
      Prob P = direct_prob(d->n, 1, 1, 1, 1, 1, 1, 0, 0);
      P.a.C = d->kh * d->kw * d->out_c; P.a.A_H = 1; P.a.A_W = 1;
      P.a.Nout = d->in_c;
      P.pk.nmode = 0; P.pk.cmode = 2; P.pk.comp_kw = d->kw; P.pk.comp_c = d->out_c;
      finish(P, d->dtype, d->n);
      v.push_back(P);
    } else {
      Prob P = direct_prob(d->n, d->in_h, d->in_w, d->kh, d->kw, d->stride_h, d->stride_w, d->pad_t, d->pad_l);
      P.a.C = d->out_c; P.a.A_H = d->out_h; P.a.A_W = d->out_w; P.a.Nout = d->in_c;
      P.pk.nmode = 0; P.pk.cmode = 1;
      finish(P, d->dtype, d->n * d->in_h * d->in_w);
      maybe_halo(P, d->dtype, d->n);
      v.push_back(P);
    }
  }
  return v;
}

static bool bwd_data_composite(const tpg_conv_desc* d, const tpg_tensor* g, const tpg_tensor* dx) {
  if (!d->transposed) {
    if (d->in_h != d->kh || d->in_w != d->kw || d->out_h != 1 || d->out_w != 1) return false;
    if (d->pad_t || d->pad_b || d->pad_l || d->pad_r || d->pad_mode) return false;
    if (d->kh == 1 && d->kw == 1) return false;
    return !dx || dense_nhwc(*dx, d->in_c, d->in_h, d->in_w);
  }
  if (d->in_h != 1 || d->in_w != 1 || d->out_h != d->kh || d->out_w != d->kw) return false;
  if (d->pad_t || d->pad_b || d->pad_l || d->pad_r) return false;
  if (d->kh == 1 && d->kw == 1) return false;
  return !g || dense_nhwc(*g, d->out_c, d->out_h, d->out_w);
}

static size_t probs_ws(const std::vector<Prob>& v) {
  size_t wp = 0, sk = 0;
  for (const Prob& P : v) {
    wp += std::max(P.wp_bytes, P.g_wp);
    sk = std::max(sk, std::max(P.sk_bytes, P.g_sk));
  }
  return wp + sk;
}

static size_t reflect_tmp_bytes(const tpg_conv_desc* d) {
  if (d->transposed || d->pad_mode != TPG_PAD_REFLECT) return 0;
  return (size_t)rup((int64_t)d->n * (d->in_h + d->pad_t + d->pad_b) * (d->in_w + d->pad_l + d->pad_r) *
                         rup(d->in_c, 8) * esize(d->dtype), 256);
}

extern "C" size_t tpg_conv2d_workspace(const tpg_conv_desc* d, int32_t op) {
  ShareScope share_scope(d);
  if (check_desc(d)) return 0;
  if (op == TPG_OP_FWD) {
    size_t a = big_taps(d) ? 0 : probs_ws(plan_fwd(d, false));
    if (fwd_composite(d, nullptr, nullptr)) a = std::max(a, probs_ws(plan_fwd(d, true)));
    return a + 256;
  }
  if (op == TPG_OP_BWD_DATA) {
    size_t a = big_taps(d) ? 0 : probs_ws(plan_bwd_data(d, false)) + reflect_tmp_bytes(d);
    if (bwd_data_composite(d, nullptr, nullptr)) a = std::max(a, probs_ws(plan_bwd_data(d, true)));
    return a + 256;
  }
  return 256;  // bwd_filter accumulates straight into dw
}

// run a list of problems: pack -> [zero split-K] -> igemm -> [finalize]
// Masked input-gradient mode of the halo kernel (tpg_conv2d_bwd): A = gy, M = the saved
// output y, G = where g = gy * act'(y) goes (M's strides).
struct HaloMask {
  tpg_tensor M, G;
  int act;
  float slope;
};

// desc.in_act: the input gradient's epilogue multiplies by act'(X) (X = the conv's input x, the
// producer's activated output, read at the output's offsets); `applied` reports whether the
// launched plan did (every problem on the halo / pointwise kernels, X laid out like Y)
struct HaloXA {
  tpg_tensor X;
  int act;
  float slope;
  bool applied;
};

static int32_t run_probs(std::vector<Prob>& v, int dtype, const tpg_tensor& A, const tpg_tensor& W, const float* bias,
                         int bias_mod, const tpg_tensor& R, float res_scale, const tpg_tensor& Y, int act, float slope,
                         char* ws, size_t ws_bytes, hipStream_t s, const char* packed = nullptr,
                         const HaloMask* mk = nullptr, HaloXA* xa = nullptr) {
  size_t need = probs_ws(v);
  if (need > ws_bytes) return fail(-20, "workspace too small: %zu < %zu", ws_bytes, need);
  const bool vA = vec_ok(A, dtype);
  if (mk) {  // the mask mode has no generic-kernel fallback: decide before launching anything
    // (the 512-row and stride-2 halo configs, ids >= 24, have no masked variant)
    if (v.size() != 1 || !v[0].halo || v[0].hcfg >= 24 || v[0].h.ntaps < 2 || !vA) return -31;
    const int64_t ext = (int64_t)(v[0].h.N - 1) * std::abs(A.stride[0]) + (int64_t)(v[0].h.A_H - 1) * std::abs(A.stride[2]) +
                        (int64_t)(v[0].h.A_W - 1) * std::abs(A.stride[3]) + v[0].h.C + 64;
    const int64_t extm = (int64_t)(v[0].h.N - 1) * mk->M.stride[0] + (int64_t)(v[0].h.A_H - 1) * mk->M.stride[2] +
                         (int64_t)(v[0].h.A_W - 1) * mk->M.stride[3] + v[0].h.C + 64;
    if (ext >= (1ll << 31) || extm >= (1ll << 31)) return -31;
  }
  for (Prob& P : v) {
    if (!P.halo) continue;
    // the halo kernel takes 16-byte aligned channels-last rows and keeps 32-bit element
    // offsets into A
    const int64_t ext = (int64_t)(P.h.N - 1) * std::abs(A.stride[0]) + (int64_t)(P.h.A_H - 1) * std::abs(A.stride[2]) +
                        (int64_t)(P.h.A_W - 1) * std::abs(A.stride[3]) + P.h.C + 64;
    if (!vA || ext >= (1ll << 31)) {
      if (packed) return fail(-21, "pre-packed weights assume the halo kernel; these tensors need the generic one");
      P.halo = false;
      P.wp_bytes = P.g_wp;
      P.sk_bytes = P.g_sk;
    }
  }
  // the producer's act' in the epilogues: all or nothing (a partial application could not be
  // completed by the caller's separate pass without applying it twice)
  const void* XA = nullptr;
  if (xa) {
    xa->applied = false;
    bool ok = xa->X.data && xa->X.dtype == Y.dtype && xa->X.stride[0] == Y.stride[0] && xa->X.stride[2] == Y.stride[2] &&
              xa->X.stride[3] == Y.stride[3] && xa->X.stride[1] == 1 && vec_ok(xa->X, dtype) == vec_ok(Y, dtype);
    for (const Prob& P : v) ok = ok && P.halo;
    if (ok) {
      XA = xa->X.data;
      xa->applied = true;
    }
  }
  size_t off = 0;
  std::vector<char*> wps;
  for (Prob& P : v) {
    wps.push_back((packed ? const_cast<char*>(packed) : ws) + off);
    off += std::max(P.wp_bytes, P.g_wp);
  }
  char* sk = ws + (packed ? 0 : off);
  for (size_t i = 0; i < v.size(); ++i) {
    Prob& P = v[i];
    IgemmArgs& a = P.a;
    PackArgs& k = P.pk;
    k.W = reinterpret_cast<const float*>(W.data);
    k.w_sa = W.stride[0]; k.w_sb = W.stride[1]; k.w_sr = W.stride[2]; k.w_ss = W.stride[3];
    k.Wp = wps[i];
    if (P.halo) {
      HaloArgs& h = P.h;
      if (h.ntaps > 0 && !packed) {
        TPG_GROUP_SYNC();
        int e = launch_pack_halo(k, h.nks, h.BN, h.ntiles, s);
        if (e) return hip_check(e, "pack_halo");
      }
      h.A = A.data; h.a_sn = A.stride[0]; h.a_sh = A.stride[2]; h.a_sw = A.stride[3];
      h.vec_ok = vA;
      h.Wp = wps[i];
      h.Y = Y.data; h.y_sn = Y.stride[0]; h.y_sh = Y.stride[2]; h.y_sw = Y.stride[3];
      h.bias = bias;
      h.R = R.data; h.r_sn = R.stride[0]; h.r_sh = R.stride[2]; h.r_sw = R.stride[3];
      h.res_scale = res_scale; h.act = act; h.slope = slope;
      h.ws = h.ksplit > 1 ? reinterpret_cast<float*>(sk) : nullptr;
      h.yvec = vec_ok(Y, dtype);
      h.rvec = R.data ? vec_ok(R, dtype) : 0;
      h.wvec = a.Nout % 4 == 0;
      if (mk) {
        h.M = mk->M.data; h.m_sn = mk->M.stride[0]; h.m_sh = mk->M.stride[2]; h.m_sw = mk->M.stride[3];
        h.G = mk->G.data; h.mact = mk->act; h.mslope = mk->slope;
      }
      h.XA = XA; h.xa_act = XA ? xa->act : 0; h.xa_slope = XA ? xa->slope : 0.f;
      int e = do_halo(h, dtype, P.hcfg, s, mk != nullptr);
      if (e) return hip_check(e, "halo conv");
      if (h.ksplit > 1) {
        EpiArgs ep;
        memset(&ep, 0, sizeof(ep));
        ep.ws = h.ws; ep.nslices = h.ksplit; ep.slice = (int64_t)a.M * a.Nout;
        ep.M = a.M; ep.Nout = a.Nout; ep.JH = a.JH; ep.JW = a.JW;
        ep.Y = Y.data; ep.y_sn = Y.stride[0]; ep.y_sh = Y.stride[2]; ep.y_sw = Y.stride[3];
        ep.oy0 = a.oy0; ep.ox0 = a.ox0; ep.osy = a.osy; ep.osx = a.osx;
        ep.bias = bias; ep.bias_mod = 0;
        ep.R = R.data; ep.r_sn = R.stride[0]; ep.r_sh = R.stride[2]; ep.r_sw = R.stride[3];
        ep.res_scale = res_scale; ep.act = act; ep.slope = slope; ep.dtype = dtype;
        ep.XA = XA; ep.xa_act = XA ? xa->act : 0; ep.xa_slope = XA ? xa->slope : 0.f;
        e = do_epilogue(ep, s);
        if (e) return hip_check(e, "halo epilogue");
      }
      continue;
    }
    TPG_GROUP_SYNC();
    if (a.nunits > 0 && !packed) {
      int e = launch_pack(k, s);
      if (e) return hip_check(e, "pack");
    }
    a.A = A.data; a.a_sn = A.stride[0]; a.a_sh = A.stride[2]; a.a_sw = A.stride[3];
    a.vec_ok = vA;
    a.Wp = wps[i];
    a.Y = Y.data; a.y_sn = Y.stride[0]; a.y_sh = Y.stride[2]; a.y_sw = Y.stride[3];
    a.bias = bias; a.bias_mod = bias_mod;
    a.R = R.data; a.r_sn = R.stride[0]; a.r_sh = R.stride[2]; a.r_sw = R.stride[3];
    a.res_scale = res_scale; a.act = act; a.slope = slope;
    a.ws = nullptr;
    if (a.ksplit > 1) {
      a.ws = reinterpret_cast<float*>(sk);
      hipError_t e = hipMemsetAsync(sk, 0, (size_t)a.M * a.Nout * 4, s);
      if (e) return hip_check((int)e, "hipMemsetAsync");
    }
    int e = launch_igemm(a, dtype, P.cfg, s);
    if (e) return hip_check(e, "igemm");
    if (a.ksplit > 1) {
      EpiArgs ep;
      memset(&ep, 0, sizeof(ep));
      ep.ws = a.ws; ep.nslices = 1; ep.slice = 0; ep.M = a.M; ep.Nout = a.Nout; ep.JH = a.JH; ep.JW = a.JW;
      ep.Y = a.Y; ep.y_sn = a.y_sn; ep.y_sh = a.y_sh; ep.y_sw = a.y_sw;
      ep.oy0 = a.oy0; ep.ox0 = a.ox0; ep.osy = a.osy; ep.osx = a.osx;
      ep.bias = bias; ep.bias_mod = bias_mod;
      ep.R = a.R; ep.r_sn = a.r_sn; ep.r_sh = a.r_sh; ep.r_sw = a.r_sw;
      ep.res_scale = res_scale; ep.act = act; ep.slope = slope; ep.dtype = dtype;
      e = launch_epilogue(ep, s);
      if (e) return hip_check(e, "epilogue");
    }
  }
  return 0;
}

static int32_t check_tensor(const tpg_tensor& t, int dtype, const char* name) {
  if (!t.data) return fail(-10, "%s is NULL", name);
  if (t.dtype != dtype) return fail(-11, "%s dtype %d != %d", name, t.dtype, dtype);
  if (t.stride[1] != 1) return fail(-12, "%s must be channels-last (channel stride 1), got %lld", name,
                                    (long long)t.stride[1]);
  return 0;
}

// ------------------------------------------------------------ pre-packed weights --
// The packed image of (d, op) is the weight part of the op's workspace for the plan the
// op picks on 16-byte aligned channels-last tensors: one region per problem, in plan order.
static std::vector<Prob> pack_plan(const tpg_conv_desc* d, int32_t op) {
  if (op == TPG_OP_FWD) return plan_fwd(d, fwd_composite(d, nullptr, nullptr));
  return plan_bwd_data(d, bwd_data_composite(d, nullptr, nullptr));
}

extern "C" size_t tpg_conv2d_packed_bytes(const tpg_conv_desc* d, int32_t op) {
  ShareScope share_scope(d);
  if (check_desc(d) || (op != TPG_OP_FWD && op != TPG_OP_BWD_DATA)) return 0;
  size_t b = 0;
  for (const Prob& P : pack_plan(d, op)) b += std::max(P.wp_bytes, P.g_wp);
  return b;
}

extern "C" size_t tpg_pack_job_bytes(void) { return sizeof(PackJob); }

extern "C" int32_t tpg_conv2d_pack_jobs(const tpg_conv_desc* d, int32_t op, tpg_tensor w, void* wp, void* jobs,
                                        int32_t max_jobs) {
  ShareScope share_scope(d);
  int32_t rc = check_desc(d);
  if (rc) return rc;
  if (op != TPG_OP_FWD && op != TPG_OP_BWD_DATA) return fail(-2, "pack: op must be fwd or bwd_data");
  if (!w.data || w.dtype != TPG_F32 || !wp || !jobs) return fail(-10, "pack: NULL / non-fp32 weight");
  std::vector<Prob> v = pack_plan(d, op);
  PackJob* out = reinterpret_cast<PackJob*>(jobs);
  int n = 0;
  size_t off = 0;
  for (Prob& P : v) {
    const size_t region = std::max(P.wp_bytes, P.g_wp);
    const bool has = P.halo ? P.h.ntaps > 0 : P.a.nunits > 0;
    if (has) {
      if (n >= max_jobs) return fail(-22, "pack: more than %d jobs", max_jobs);
      PackJob& j = out[n++];
      memset(&j, 0, sizeof(j));
      j.k = P.pk;
      j.k.W = reinterpret_cast<const float*>(w.data);
      j.k.w_sa = w.stride[0]; j.k.w_sb = w.stride[1]; j.k.w_sr = w.stride[2]; j.k.w_ss = w.stride[3];
      j.k.Wp = reinterpret_cast<char*>(wp) + off;
      if (P.halo) {
        j.kind = 1;
        j.nks = P.h.nks; j.bn = P.h.BN; j.bnl = (P.h.BN + 127) / 128 * 128; j.ntiles = P.h.ntiles;
        j.items = halo_steps(j.nks, j.k.ntaps, P.h.half) * j.ntiles * j.bnl * 4;
      } else {
        j.kind = 0;
        j.items = j.k.Npad * j.k.nunits;
      }
      j.nblocks = cdiv(j.items, 256 * TPG_PACK_GROUPS);
    }
    off += region;
  }
  return n;
}

extern "C" int64_t tpg_pack_prepare(void* jobs, int32_t n) {
  PackJob* j = reinterpret_cast<PackJob*>(jobs);
  int64_t b = 0;
  for (int i = 0; i < n; ++i) {
    j[i].first_block = (int)b;
    b += j[i].nblocks;
  }
  return b;
}

extern "C" int32_t tpg_pack_run(const void* jobs_dev, int32_t n, int64_t nblocks, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (n <= 0) return 0;
  if (!jobs_dev || nblocks <= 0 || nblocks >= (1ll << 31)) return fail(-2, "pack_run: bad batch");
  return hip_check(launch_pack_many(reinterpret_cast<const PackJob*>(jobs_dev), n, (int)nblocks, (hipStream_t)stream),
                   "pack_run");
}

extern "C" int32_t tpg_conv2d_fwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, const float* bias,
                                  tpg_tensor residual, tpg_tensor y, void* ws, size_t ws_bytes, tpg_stream_t stream) {
  ShareScope share_scope(d);
  int32_t rc = check_desc(d);
  if (rc) return rc;
  if ((rc = check_tensor(x, d->dtype, "x")) || (rc = check_tensor(y, d->dtype, "y"))) return rc;
  if (!w.data || (w.dtype != TPG_F32 && !(d->flags & TPG_FLAG_WPACKED))) return fail(-13, "weight must be fp32");
  if (residual.data && (rc = check_tensor(residual, d->dtype, "residual"))) return rc;
  const bool comp = fwd_composite(d, &x, &y);
  const bool packed = d->flags & TPG_FLAG_WPACKED;
  if (!comp && big_taps(d)) return fail(-4, "%dx%d kernel: only the dense NHWC GEMM form is supported", d->kh, d->kw);
  if (packed && comp != fwd_composite(d, nullptr, nullptr))
    return fail(-21, "pre-packed weights assume a full-kernel GEMM; these tensors are not dense NHWC");
  std::vector<Prob> v = plan_fwd(d, comp);
  int bias_mod = (comp && d->transposed) ? d->out_c : 0;
  if (comp && residual.data) return fail(-14, "residual not supported on a full-kernel conv");
  return run_probs(v, d->dtype, x, w, bias, bias_mod, residual, d->res_scale, y, d->act, d->slope,
                   reinterpret_cast<char*>(ws), ws_bytes, (hipStream_t)stream,
                   packed ? reinterpret_cast<const char*>(w.data) : nullptr);
}

static int32_t bwd_data_impl(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx, void* ws,
                             size_t ws_bytes, tpg_stream_t stream, HaloXA* xa);

extern "C" int32_t tpg_conv2d_bwd_data(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx, void* ws,
                                       size_t ws_bytes, tpg_stream_t stream) {
  ShareScope share_scope(d);
  int32_t rc = check_desc(d);
  if (rc) return rc;
  if (d->in_act != TPG_ACT_NONE) return fail(-33, "bwd_data: desc.in_act needs x (tpg_conv2d_bwd)");
  return bwd_data_impl(d, g, w, dx, ws, ws_bytes, stream, nullptr);
}

static int32_t bwd_data_impl(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx, void* ws,
                             size_t ws_bytes, tpg_stream_t stream, HaloXA* xa) {
  int32_t rc;
  if ((rc = check_tensor(g, d->dtype, "g")) || (rc = check_tensor(dx, d->dtype, "dx"))) return rc;
  const bool packed = d->flags & TPG_FLAG_WPACKED;
  if (!w.data || (w.dtype != TPG_F32 && !packed)) return fail(-13, "weight must be fp32");
  hipStream_t s = (hipStream_t)stream;
  const bool comp = bwd_data_composite(d, &g, &dx);
  if (!comp && big_taps(d)) return fail(-4, "%dx%d kernel: only the dense NHWC GEMM form is supported", d->kh, d->kw);
  if (packed && comp != bwd_data_composite(d, nullptr, nullptr))
    return fail(-21, "pre-packed weights assume a full-kernel GEMM; these tensors are not dense NHWC");
  const char* pk = packed ? reinterpret_cast<const char*>(w.data) : nullptr;
  std::vector<Prob> v = plan_bwd_data(d, comp);
  tpg_tensor none;
  memset(&none, 0, sizeof(none));
  const bool refl = !comp && !d->transposed && d->pad_mode == TPG_PAD_REFLECT;
  // DX_ACCUM: dx's entry values ride in as the epilogue's residual (read, then overwritten by
  // the same thread): dx = dgrad + dx
  const bool acc = d->flags & TPG_FLAG_DX_ACCUM;
  if (acc && (comp || refl)) return fail(-32, "dx accumulation: zero-padded, non-GEMM-form geometries only");
  if (!refl)
    return run_probs(v, d->dtype, g, w, nullptr, 0, acc ? dx : none, acc ? 1.f : 0.f, dx, TPG_ACT_NONE, 0.f,
                     reinterpret_cast<char*>(ws), ws_bytes, s, pk, nullptr, xa);
  // reflect: gradient of the padded input into a dense NHWC temp, then fold onto dx
  const size_t tmpb = reflect_tmp_bytes(d);
  if (ws_bytes < tmpb) return fail(-20, "workspace too small");
  const int PH = d->in_h + d->pad_t + d->pad_b, PW = d->in_w + d->pad_l + d->pad_r, Cp = (int)rup(d->in_c, 8);
  tpg_tensor tmp;
  memset(&tmp, 0, sizeof(tmp));
  tmp.data = ws; tmp.dtype = d->dtype;
  tmp.stride[0] = (int64_t)PH * PW * Cp; tmp.stride[1] = 1; tmp.stride[2] = (int64_t)PW * Cp; tmp.stride[3] = Cp;
  rc = run_probs(v, d->dtype, g, w, nullptr, 0, none, 0.f, tmp, TPG_ACT_NONE, 0.f, reinterpret_cast<char*>(ws) + tmpb,
                 ws_bytes - tmpb, s, pk);
  if (rc) return rc;
  TPG_GROUP_SYNC();
  return hip_check(launch_reflect_fold(d->n, d->in_c, d->in_h, d->in_w, d->pad_t, d->pad_b, d->pad_l, d->pad_r, tmp, dx, s),
                   "reflect_fold");
}

// Row-halo weight gradient (tpg_wgrad_rh.hip) for a stride-1 Conv2d: returns 1 when the
// shape is not covered (caller falls back), else the launch status.
static int32_t wgrad_rh(const tpg_conv_desc* d, const tpg_tensor& x, const tpg_tensor& g, const tpg_tensor& dw,
                        float* dbias, hipStream_t stream) {
  if (!half16(d->dtype) || d->stride_h != 1 || d->stride_w != 1) return 1;
  const int PH = d->out_h, PW = d->out_w, QH = d->in_h, QW = d->in_w;
  // row mode: one kernel row, 3/5/7 taps, 64-pixel row segments; image mode (algos 10, 11 and
  // the default below 64 pixels of width): all taps of a 2x2 / 3x3 kernel from one halo of
  // (64 / tw) whole rows of width tw
  const bool row_ok = PW % 64 == 0 && (d->kw == 3 || d->kw == 5 || d->kw == 7);
  // image mode k-tile: th = floor(64 / tw) rows of tw = min(PW, 64); the fragment reads reach
  // halo row (63 / tw + kh - 1) * (tw + kw - 1) + tw + kw - 2, inside the 200-row LDS image
  const int tw = std::min(PW, 64);
  const bool img_ok = d->kh == d->kw && (d->kw == 2 || d->kw == 3) && PW % tw == 0 && tw >= 4 &&
                      (63 / tw + d->kh - 1) * (tw + d->kw - 1) + tw + d->kw - 2 < 200;
  // (untuned default only for full 64-pixel k-tiles: 40-wide maps measured slower than wgrad2)
  const bool img = d->algo == 10 || d->algo == 11 || (d->algo == 0 && !row_ok && 64 % tw == 0);
  if (img ? !img_ok : !row_ok) return 1;
  if (d->pad_t >= QH || d->pad_l >= QW || !vec_ok(g, d->dtype) || !vec_ok(x, d->dtype)) return 1;
  if (g.stride[2] != (int64_t)PW * g.stride[3] || g.stride[0] != (int64_t)PH * g.stride[2]) return 1;
  if (x.stride[2] != (int64_t)QW * x.stride[3] || x.stride[0] != (int64_t)QH * x.stride[2]) return 1;
  // extents cover the last pixel's whole 16-byte chunks (vec_ok: pixel stride >= ceil8(C))
  const int64_t pb = ((int64_t)(d->n - 1) * g.stride[0] + (int64_t)(PH - 1) * g.stride[2] +
                      (int64_t)(PW - 1) * g.stride[3] + rup(d->out_c, 8)) * 2;
  const int64_t qb = ((int64_t)(d->n - 1) * x.stride[0] + (int64_t)(QH - 1) * x.stride[2] +
                      (int64_t)(QW - 1) * x.stride[3] + rup(d->in_c, 8)) * 2;
  if (pb >= (1ll << 31) || qb >= (1ll << 31)) return 1;
  WgradRHArgs a;
  memset(&a, 0, sizeof(a));
  a.dtype = d->dtype;
  a.P = g.data; a.p_sn = (int)g.stride[0]; a.p_sh = (int)g.stride[2]; a.p_sw = (int)g.stride[3];
  a.PH = PH; a.PW = PW; a.Ca = d->out_c; a.p_bytes = (int)pb;
  a.Q = x.data; a.q_sn = (int)x.stride[0]; a.q_sh = (int)x.stride[2]; a.q_sw = (int)x.stride[3];
  a.QH = QH; a.QW = QW; a.Cb = d->in_c; a.q_bytes = (int)qb;
  a.kh = d->kh; a.kw = d->kw; a.pt = d->pad_t; a.pl = d->pad_l; a.pad_mode = d->pad_mode;
  a.nr = img ? d->kh : 1;
  a.nrg = cdiv(a.kh, a.nr);
  a.tw = img ? tw : 64;
  // tile: fewest padded MACs, the 128 x 64 tile (best operand reuse) on ties
  int bm = 128, bc = 64;
  if (d->algo >= 6 && d->algo <= 12) {
    a.cfg = d->algo - 6;
    wgrad_rh_tile(a.cfg, &bm, &bc);
  } else {
    int64_t best = -1;
    for (int c = img ? 4 : 0; c < (img ? 6 : 4); ++c) {
      int m, b;
      wgrad_rh_tile(c, &m, &b);
      const int64_t cost = rup(a.Ca, m) * rup(a.Cb, b) * (100 + (m == 64 ? 8 : 0) + (b == 32 ? 8 : 0));
      if (best < 0 || cost < best) { best = cost; a.cfg = c; bm = m; bc = b; }
    }
  }
  // taps per block: a whole kernel row, except 7-wide rows on the 128 x 64 / 256 x 32 tiles
  // (7 x BC columns there exceed the VGPR budget: 4 + 4 taps, one of them dead)
  a.nt = img ? d->kw : (d->kw == 7 && (a.cfg == 0 || a.cfg == 6)) ? 4 : d->kw;
  a.nta = cdiv(a.Ca, bm); a.ntb = cdiv(a.Cb, bc);
  a.tiles = a.nta * a.ntb * a.nrg * cdiv(a.kw, a.nt);
  a.nkt = d->n * cdiv(PH, 64 / a.tw) * (PW / a.tw);
  int ks = 1;
  if (d->algo >= 6 && d->ksplit >= 1) {
    ks = d->ksplit;
  } else {
    // pixel splits: whole rounds of resident blocks (one per CU, two for the <= 128-VGPR
    // tiles) against the fp32 atomics every extra split adds (~1.3 TB/s of added bytes)
    const int resident = (img || a.cfg == 6 ? 256 : (a.cfg == 3 || (a.cfg != 0 && a.nt <= 4)) ? 512 : 256) / g_share;
    const int taps = a.nr * a.nt;
    const double flops = 2.0 * a.tiles * bm * taps * bc * 64.0 * a.nkt;
    double best = -1;
    for (int k = 1; k <= 64 && k <= a.nkt; ++k) {
      const int64_t blocks = (int64_t)a.tiles * k;
      const double rounds = (double)((blocks + resident - 1) / resident);
      const double t = rounds * flops / blocks / (4.5e12 * 256 / resident) +
                       (k > 1 ? k * (double)a.tiles * bm * taps * bc * 4 / 1.3e12 : 0.0);
      if (best < 0 || t < best) { best = t; ks = k; }
    }
  }
  ks = std::max(1, std::min(ks, a.nkt));
  if (deterministic()) ks = 1;  // one block adds each dW element once
  a.kt_per_split = cdiv(a.nkt, ks);
  a.ksplit = cdiv(a.nkt, a.kt_per_split);
  a.dW = reinterpret_cast<float*>(dw.data);
  a.w_sa = dw.stride[0]; a.w_sb = dw.stride[1]; a.w_sr = dw.stride[2]; a.w_ss = dw.stride[3];
  a.dbias = dbias;
  // bias MFMAs spread over up to 16 / ksplit tiles: same-address atomics serialise (~50 ns
  // each), so blocks x splits adding into one dbias row must stay few
  a.bshare = deterministic() ? 1 : std::max(1, std::min(a.ntb * a.nrg * cdiv(a.kw, a.nt), 16 / a.ksplit));
  a.skip = g_rh_skip;
  TPG_GROUP_SYNC();
  return hip_check(launch_wgrad_rh(a, stream), "wgrad_rh");
}

// Weight gradient; with dbias (Conv2d only: the pixel-grid operand is g) the bias gradient is
// summed by the same launch where the kernel supports it (*bias_done), else left to the caller.
static int32_t bwd_filter_impl(const tpg_conv_desc* d, const tpg_tensor& x, const tpg_tensor& g, const tpg_tensor& dw,
                               float* dbias, bool* bias_done, tpg_stream_t stream) {
  ShareScope share_scope(d);
  *bias_done = false;
  if (d->transposed) dbias = nullptr;
  int32_t rc = check_desc(d);
  if (rc) return rc;
  if ((rc = check_tensor(x, d->dtype, "x")) || (rc = check_tensor(g, d->dtype, "g"))) return rc;
  if (!dw.data || dw.dtype != TPG_F32) return fail(-13, "dw must be fp32");
  WgradArgs a;
  memset(&a, 0, sizeof(a));
  const tpg_tensor& P = d->transposed ? x : g;  // iteration grid operand
  const tpg_tensor& Q = d->transposed ? g : x;  // gathered operand
  const int PH = d->transposed ? d->in_h : d->out_h, PW = d->transposed ? d->in_w : d->out_w;
  const int QH = d->transposed ? d->out_h : d->in_h, QW = d->transposed ? d->out_w : d->in_w;
  const int Ca = d->transposed ? d->in_c : d->out_c, cb = d->transposed ? d->out_c : d->in_c;
  const bool comp = d->transposed ? bwd_data_composite(d, &g, nullptr) : fwd_composite(d, &x, nullptr);
  if (!comp && big_taps(d)) return fail(-4, "%dx%d kernel: only the dense NHWC GEMM form is supported", d->kh, d->kw);
  a.P = P.data; a.p_sn = P.stride[0]; a.p_sh = P.stride[2]; a.p_sw = P.stride[3];
  a.Q = Q.data; a.q_sn = Q.stride[0]; a.q_sh = Q.stride[2]; a.q_sw = Q.stride[3];
  a.Ca = Ca;
  a.vec_p = vec_ok(P, d->dtype);
  a.vec_q = vec_ok(Q, d->dtype);
  if (comp) {
    a.PH = 1; a.PW = 1; a.QH = 1; a.QW = 1;
    a.Cb = d->kh * d->kw * cb;
    a.bcomp = 1; a.comp_kw = d->kw; a.comp_cb = cb;
    a.ntaps = 1; a.dy[0] = 0; a.dx[0] = 0; a.tr[0] = 0; a.ts[0] = 0;
    a.qst_h = 1; a.qst_w = 1;
  } else {
    a.PH = PH; a.PW = PW; a.QH = QH; a.QW = QW; a.Cb = cb;
    a.qst_h = d->stride_h; a.qst_w = d->stride_w;
    a.pad_mode = d->transposed ? 0 : d->pad_mode;
    a.ntaps = d->kh * d->kw;
    for (int r = 0; r < d->kh; ++r)
      for (int s = 0; s < d->kw; ++s) {
        int t = r * d->kw + s;
        a.dy[t] = (int8_t)(r - d->pad_t); a.dx[t] = (int8_t)(s - d->pad_l);
        a.tr[t] = (int8_t)r; a.ts[t] = (int8_t)s;
      }
  }
  a.npix = d->n * a.PH * a.PW;
  a.dW = reinterpret_cast<float*>(dw.data);
  a.w_sa = dw.stride[0]; a.w_sb = dw.stride[1]; a.w_sr = dw.stride[2]; a.w_ss = dw.stride[3];
  a.div_pw.init(a.PW);
  a.div_phpw.init(a.PH * a.PW);
  // kernel-row halo kernel (stride-1 Conv2d, bf16, 64-pixel row segments): algo 6, and the
  // default for untuned calls when it applies
  const bool rh_algo = d->algo >= 6 && d->algo <= 12;
  if ((d->algo == 0 || rh_algo) && !comp && !d->transposed) {
    const int rc = wgrad_rh(d, x, g, dw, dbias, (hipStream_t)stream);
    if (rc != 1) {
      *bias_done = rc == 0 && dbias != nullptr;
      return rc;
    }
  }
  if (rh_algo) return fail(-30, "wgrad: row-halo kernel does not apply to this shape");
  // pipelined DMA kernel when both operands are 16-byte aligned channels-last rows
  if (a.vec_p && a.vec_q) {
    // non-composite: columns flattened over taps (b' = tap * rup(Cb, 8) + b), so channel
    // counts like 75 / 206 waste at most 7 columns per tap instead of a tile remainder
    a.bflat = comp ? 0 : 1;
    a.cbp = (int)rup(a.Cb, 8);
    const int64_t ncols = a.bflat ? (int64_t)a.ntaps * a.cbp : a.Cb;
    const int ngrid = a.bflat ? 1 : a.ntaps;
    // Default tile / pixel-split choice (padded MACs, 64-wide tiles charged 15% for their
    // lower operand reuse; about 2048 blocks).  Callers that autotune pass their choice in
    // the descriptor: algo = tile index + 1 into cand[], ksplit = pixel splits.
    static const int cand[5][2] = {{256, 128}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
    const int kp = half16(d->dtype) ? 64 : 32;
    const int nkt = cdiv(a.npix, kp);
    int bm = 0, bn = 0, bks = 1;
    {
      int64_t best = -1;
      for (auto& c : cand) {
        const int64_t cost = (int64_t)rup(a.Ca, c[0]) * rup(ncols, c[1]) * ngrid * ((c[0] == 64 || c[1] == 64) ? 115 : 100);
        if (best < 0 || cost < best) { best = cost; bm = c[0]; bn = c[1]; }
      }
      const int tiles = cdiv(a.Ca, bm) * (int)((ncols + bn - 1) / bn) * ngrid;
      bks = std::max(1, cdiv(2048 / g_share, tiles));
      bks = std::min(bks, std::max(1, a.npix / (kp * 8)));
    }
    if (d->algo >= 1 && d->algo <= 5 && d->ksplit >= 1) {
      bm = cand[d->algo - 1][0]; bn = cand[d->algo - 1][1];
      bks = std::min(d->ksplit, nkt);
    }
    if (deterministic()) bks = 1;
    a.pix_per_split = (int)rup(cdiv(a.npix, bks), kp);
    a.ksplit = cdiv(a.npix, a.pix_per_split);
    const int es = esize(d->dtype);
    // byte extent up to the end of the last pixel's last 16-byte chunk (a chunk straddling C
    // must not count as out of range: vec_ok rows are padded to whole chunks)
    auto extent = [&](const tpg_tensor& t, int n, int h, int w, int c) -> int64_t {
      return ((int64_t)(n - 1) * t.stride[0] + (int64_t)(h - 1) * t.stride[2] + (int64_t)(w - 1) * t.stride[3] +
              rup(c, 16 / es)) * es;
    };
    const int64_t pb = extent(P, d->n, a.PH == 1 && comp ? 1 : PH, a.PW == 1 && comp ? 1 : PW, a.Ca);
    const int64_t qb = comp ? extent(Q, d->n, 1, 1, a.Cb) : extent(Q, d->n, QH, QW, cb);
    if (pb < (1ll << 31) && qb < (1ll << 31)) {
      a.p_bytes = (int)pb;
      a.q_bytes = (int)qb;
      // division-free DMA addressing (see tpg_wgrad2.hip)
      a.fastp = !comp && P.stride[2] == (int64_t)PW * P.stride[3] && P.stride[0] == (int64_t)PH * P.stride[2];
      a.fastq = a.bflat && a.qst_h == 1 && a.qst_w == 1 && a.pad_mode == 0 && QH == PH && QW == PW &&
                Q.stride[2] == (int64_t)QW * Q.stride[3] && Q.stride[0] == (int64_t)QH * Q.stride[2] &&
                (int64_t)PH * PW > kp;
      a.dpy = kp / a.PW;
      a.dpx = kp % a.PW;
      a.dbias = dbias;
      a.bshare = deterministic() ? 1 : std::max(1, std::min((int)((ncols + bn - 1) / bn) * ngrid, 16 / a.ksplit));
      const int32_t r2 = hip_check(do_wgrad2(a, d->dtype, wgrad2_cfg(bm, bn), bm, bn, (hipStream_t)stream), "wgrad2");
      *bias_done = r2 == 0 && dbias != nullptr;
      return r2;
    }
  }
  const int cfg = (a.Ca >= 128 && a.Cb >= 128) ? 1 : 0;
  const int bm = wgrad_cfg_bm(cfg), bn = wgrad_cfg_bn(cfg);
  const int tiles = cdiv(a.Ca, bm) * cdiv(a.Cb, bn) * a.ntaps;
  int ks = std::max(1, cdiv(1536, tiles));
  ks = std::min(ks, std::max(1, a.npix / (32 * 16)));
  if (deterministic()) ks = 1;
  a.pix_per_split = (int)rup(cdiv(a.npix, ks), 32);
  a.ksplit = cdiv(a.npix, a.pix_per_split);
  TPG_GROUP_SYNC();
  return hip_check(launch_wgrad(a, d->dtype, cfg, (hipStream_t)stream), "wgrad");
}

extern "C" int32_t tpg_conv2d_bwd_filter(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor g, tpg_tensor dw, void* ws,
                                         size_t ws_bytes, tpg_stream_t stream) {
  (void)ws; (void)ws_bytes;
  bool bias_done;
  return bwd_filter_impl(d, x, g, dw, nullptr, &bias_done, stream);
}

extern "C" int32_t tpg_colsum_impl(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor g, float* dbias,
                                    hipStream_t s);

// Fused per-layer backward (SURVEY.md §8b tpg_conv2d_bwd): g = gy * act'(y), dx, dw, dbias.
extern "C" int32_t tpg_conv2d_bwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, tpg_tensor y, tpg_tensor gy,
                                  tpg_tensor g, tpg_tensor dx, tpg_tensor dw, float* dbias, void* ws, size_t ws_bytes,
                                  tpg_stream_t stream) {
  ShareScope share_scope(d);
  int32_t rc = check_desc(d);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (!gy.data) return fail(-10, "conv2d_bwd: gy is NULL");
  const bool has_act = d->act != TPG_ACT_NONE;
  if (has_act && !y.data) return fail(-10, "conv2d_bwd: y is NULL with an activation");
  // without an activation g IS gy (when it already has the compute dtype)
  // (16-byte aligned channels-last rows: the weight-gradient DMA kernels read g as it is)
  const bool g_is_gy = !has_act && gy.dtype == d->dtype && vec_ok(gy, d->dtype);
  if (!g_is_gy && (rc = check_tensor(g, d->dtype, "g"))) return rc;
  const tpg_tensor& G = g_is_gy ? gy : g;
  bool have_g = g_is_gy, bias_done = false, dx_done = false;
  const bool acc = dx.data && (d->flags & TPG_FLAG_DX_ACCUM);
  // desc.in_act: dx leaves as dx * in_act'(x) (the producer's activation backward)
  HaloXA xa;
  memset(&xa, 0, sizeof(xa));
  const bool xact = dx.data && d->in_act != TPG_ACT_NONE;
  if (xact) {
    if (d->in_act < TPG_ACT_NONE || d->in_act > TPG_ACT_RELU6) return fail(-2, "conv2d_bwd: bad in_act %d", d->in_act);
    if ((rc = check_tensor(x, d->dtype, "x")) || (rc = check_tensor(dx, d->dtype, "dx"))) return rc;
    xa.X = x; xa.act = d->in_act; xa.slope = d->in_slope;
  }
  if (acc && (bwd_data_composite(d, nullptr, nullptr) || (!d->transposed && d->pad_mode == TPG_PAD_REFLECT)))
    return fail(-32, "dx accumulation: zero-padded, non-GEMM-form geometries only");
  // pre-packed weights that the input-gradient plan of these tensors cannot use: report it
  // (-21) before anything is launched, so the caller's retry with fp32 weights adds nothing twice
  if ((d->flags & TPG_FLAG_WPACKED) && dx.data &&
      (!vec_ok(G, d->dtype) || bwd_data_composite(d, &G, &dx) != bwd_data_composite(d, nullptr, nullptr)))
    return fail(-21, "pre-packed weights assume the halo kernel / dense NHWC; these tensors need another plan");
  // 1. the input gradient with the activation' applied while its halo is staged (writes g)
  // (round 1 measured 42.1 ms/step with maps up to 64 x 64, 42.5 with every map, 43.0 with
  // none; after the 512-row and stride-2 tiles -- which have no masked variant and now fall
  // back to the separate pass -- every map measured 37.39 vs 37.54 / 37.56 at 64 x 64)
  if (!have_g && dx.data && !d->transposed && d->stride_h == 1 && d->stride_w == 1 && d->pad_mode == TPG_PAD_ZERO &&
      d->in_h == d->out_h && d->in_w == d->out_w && gy.dtype == d->dtype && y.dtype == d->dtype &&
      dx.dtype == d->dtype && vec_ok(gy, d->dtype) && vec_ok(y, d->dtype) && vec_ok(g, d->dtype) &&
      y.stride[0] == g.stride[0] && y.stride[2] == g.stride[2] && y.stride[3] == g.stride[3]) {
    const bool packed = d->flags & TPG_FLAG_WPACKED;
    if (w.data && (w.dtype == TPG_F32 || packed) && !bwd_data_composite(d, &gy, &dx)) {
      std::vector<Prob> v = plan_bwd_data(d, false);
      HaloMask mk;
      mk.M = y; mk.G = g; mk.act = d->act; mk.slope = d->slope;
      tpg_tensor none;
      memset(&none, 0, sizeof(none));
      rc = run_probs(v, d->dtype, gy, w, nullptr, 0, acc ? dx : none, acc ? 1.f : 0.f, dx, TPG_ACT_NONE, 0.f,
                     reinterpret_cast<char*>(ws), ws_bytes, s, packed ? reinterpret_cast<const char*>(w.data) : nullptr,
                     &mk, xact ? &xa : nullptr);
      if (rc == 0) have_g = dx_done = true;
      else if (rc != -31) return rc;
    }
  }
  // 2. otherwise the activation backward pass materialises g (and sums the bias when there is
  // no weight gradient: with one, the weight-gradient launch sums it, the same order whether
  // the caller runs the weight gradient here or as a second call on another stream)
  if (!have_g) {
    // (ConvTranspose2d: its weight-gradient kernels never take the bias -- it would cost a
    // separate column-sum launch, so this pass keeps it)
    float* db = (dw.data && !d->transposed) ? nullptr : dbias;
    rc = hip_check(do_act_bwd(d->n, d->out_c, d->out_h, d->out_w, d->act, d->slope, gy, y, g, db, s),
                   "act_bwd");
    if (rc) return rc;
    have_g = true;
    bias_done = db != nullptr;
  }
  if (dx.data && !dx_done) {
    xa.applied = false;
    if ((rc = bwd_data_impl(d, G, w, dx, ws, ws_bytes, stream, xact ? &xa : nullptr))) return rc;
  }
  if (xact && !xa.applied) {  // (plans whose epilogue cannot take it: one in-place pass over dx)
    rc = hip_check(do_act_bwd(d->n, d->in_c, d->in_h, d->in_w, d->in_act, d->in_slope, dx, x, dx, nullptr, s),
                   "act_bwd (in_act)");
    if (rc) return rc;
  }
  // 3. the weight gradient, summing the bias gradient in the same launch where it can
  if (dw.data) {
    bool b = false;
    if ((rc = bwd_filter_impl(d, x, G, dw, bias_done ? nullptr : dbias, &b, stream))) return rc;
    bias_done = bias_done || b;
  }
  if (dbias && !bias_done) {
    TPG_GROUP_SYNC();
    return hip_check(tpg_colsum_impl(d->n, d->out_c, d->out_h, d->out_w, G, dbias, s), "colsum");
  }
  return 0;
}

// ------------------------------------------------------------------ fused G losses --
static constexpr size_t LOSS_WS = 512 * TPG_L1_MAX_SEGS * sizeof(float);  // (tpg_losses.hip LS_BLOCKS)
extern "C" size_t tpg_loss_workspace(void) { return LOSS_WS; }

static int32_t check_loss_tensor(const tpg_tensor& t, const char* what) {
  if (!t.data) return fail(-10, "%s is NULL", what);
  if (t.dtype != TPG_F32 && t.dtype != TPG_BF16 && t.dtype != TPG_F16) return fail(-11, "%s: bad dtype %d", what, t.dtype);
  return 0;
}

extern "C" int32_t tpg_image_losses_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor r,
                                        float w_pix, float w_sym, float w_tv, float* ws, size_t ws_bytes, float* out,
                                        tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc;
  if (n < 1 || c < 1 || h < 1 || w < 1) return fail(-2, "image_losses: empty shape");
  if ((rc = check_loss_tensor(x, "x")) || (rc = check_loss_tensor(r, "r"))) return rc;
  if (!ws || ws_bytes < LOSS_WS || !out) return fail(-20, "image_losses: workspace / out");
  return hip_check(launch_image_losses(n, c, h, w, x, r, w_pix, w_sym, w_tv, ws, nullptr, out, nullptr,
                                       (hipStream_t)stream), "image_losses");
}

extern "C" int32_t tpg_image_losses_bwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor r,
                                        float w_pix, float w_sym, float w_tv, const float* gout, tpg_tensor dx,
                                        tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc;
  if (n < 1 || c < 1 || h < 1 || w < 1) return fail(-2, "image_losses: empty shape");
  if ((rc = check_loss_tensor(x, "x")) || (rc = check_loss_tensor(r, "r")) || (rc = check_loss_tensor(dx, "dx")))
    return rc;
  if (!gout) return fail(-10, "image_losses: gout is NULL");
  return hip_check(launch_image_losses(n, c, h, w, x, r, w_pix, w_sym, w_tv, nullptr, gout, nullptr, &dx,
                                       (hipStream_t)stream), "image_losses_bwd");
}

static int32_t check_l1_segs(int32_t nseg, const tpg_l1_seg* segs, bool bwd) {
  if (nseg < 1 || nseg > TPG_L1_MAX_SEGS || !segs) return fail(-2, "l1_set: 1..%d segments", TPG_L1_MAX_SEGS);
  for (int k = 0; k < nseg; ++k) {
    const tpg_l1_seg& s = segs[k];
    int32_t rc;
    if (s.n < 1 || s.c < 1 || s.h < 1 || s.w < 1) return fail(-2, "l1_set: segment %d empty", k);
    if ((rc = check_loss_tensor(s.a, "a")) || (rc = check_loss_tensor(s.b, "b"))) return rc;
    if (bwd && s.da.data && (rc = check_loss_tensor(s.da, "da"))) return rc;
  }
  return 0;
}

extern "C" int32_t tpg_l1_set_fwd(int32_t nseg, const tpg_l1_seg* segs, float* ws, size_t ws_bytes, float* out,
                                  tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc = check_l1_segs(nseg, segs, false);
  if (rc) return rc;
  if (!ws || ws_bytes < LOSS_WS || !out) return fail(-20, "l1_set: workspace / out");
  return hip_check(launch_l1_set(nseg, segs, ws, nullptr, out, false, (hipStream_t)stream), "l1_set");
}

extern "C" int32_t tpg_l1_set_bwd(int32_t nseg, const tpg_l1_seg* segs, const float* gout, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc = check_l1_segs(nseg, segs, true);
  if (rc) return rc;
  if (!gout) return fail(-10, "l1_set: gout is NULL");
  return hip_check(launch_l1_set(nseg, segs, nullptr, gout, nullptr, true, (hipStream_t)stream), "l1_set_bwd");
}

extern "C" int32_t tpg_act_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t act, float slope, tpg_tensor gy,
                               tpg_tensor y, tpg_tensor g, float* dbias, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (!gy.data || !g.data || (act != TPG_ACT_NONE && !y.data)) return fail(-10, "act_bwd: NULL tensor");
  return hip_check(tpg_act_bwd_impl(n, c, h, w, act, slope, gy, y, g, dbias, (hipStream_t)stream), "act_bwd");
}

extern "C" int32_t tpg_copy4d(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor in, tpg_tensor out,
                              tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (!in.data || !out.data) return fail(-10, "copy4d: NULL tensor");
  if ((int64_t)n * c * h * w == 0) return 0;
  return hip_check(tpg_copy4d_impl(n, c, h, w, in, out, (hipStream_t)stream), "copy4d");
}

extern "C" int32_t tpg_fold_taps(int32_t n, int32_t c, int32_t h, int32_t w, int32_t fh, int32_t fw, int32_t sh,
                                 int32_t sw, int32_t pt, int32_t pl, int32_t oh, int32_t ow, tpg_tensor x, tpg_tensor y,
                                 int32_t backward, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (!x.data || !y.data) return fail(-10, "fold_taps: NULL tensor");
  if (fh < 1 || fw < 1 || sh < 1 || sw < 1 || n < 0 || c < 1 || (int64_t)fh * fw * c > 4096)
    return fail(-2, "fold_taps: bad geometry");
  if ((int64_t)n * (backward ? (int64_t)h * w * c : (int64_t)oh * ow * fh * fw * c) == 0) return 0;
  return hip_check(tpg_fold_taps_impl(n, c, h, w, fh, fw, sh, sw, pt, pl, oh, ow, x, y, backward, (hipStream_t)stream),
                   "fold_taps");
}

extern "C" int32_t tpg_local_fuse_fwd(int32_t n, int32_t c, int32_t out_h, int32_t out_w, const tpg_tensor* parts,
                                      const int32_t* ph, const int32_t* pw, const int32_t* top, const int32_t* left,
                                      tpg_tensor y, uint8_t* argmax, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  for (int k = 0; k < 4; ++k)
    if (!parts[k].data) return fail(-10, "local_fuse: part %d NULL", k);
  return hip_check(tpg_fuse_fwd_impl(n, c, out_h, out_w, parts, ph, pw, top, left, y, argmax, (hipStream_t)stream),
                   "local_fuse_fwd");
}

extern "C" int32_t tpg_local_fuse_bwd(int32_t n, int32_t c, int32_t out_h, int32_t out_w, tpg_tensor gy,
                                      const uint8_t* argmax, const tpg_tensor* dparts, const int32_t* ph,
                                      const int32_t* pw, const int32_t* top, const int32_t* left, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (!argmax || !gy.data) return fail(-10, "local_fuse_bwd: NULL");
  return hip_check(tpg_fuse_bwd_impl(n, c, out_h, out_w, gy, argmax, dparts, ph, pw, top, left, (hipStream_t)stream),
                   "local_fuse_bwd");
}

extern "C" int32_t tpg_maxout2_fwd(int32_t b, int32_t m, tpg_tensor x, tpg_tensor y, uint8_t* argmax,
                                   tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  return hip_check(tpg_maxout_fwd_impl(b, m, x, y, argmax, (hipStream_t)stream), "maxout_fwd");
}

extern "C" int32_t tpg_maxout2_bwd(int32_t b, int32_t m, tpg_tensor gy, const uint8_t* argmax, tpg_tensor dx,
                                   tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  return hip_check(tpg_maxout_bwd_impl(b, m, gy, argmax, dx, (hipStream_t)stream), "maxout_bwd");
}

extern "C" int32_t tpg_adam(int64_t numel, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                            float lr, float beta1, float beta2, float eps, float weight_decay, int32_t step,
                            float grad_scale, float* state, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (numel < 0) return fail(-2, "adam: numel must be >= 0");
  if (numel == 0 && step < 0) return 0;
  if (!state) return fail(-10, "adam: NULL state");
  if (numel > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)) return fail(-10, "adam: NULL pointer");
  const int rc = tpg_adam_impl(numel, param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step,
                               grad_scale, state, (hipStream_t)stream);
  if (rc == -1) return fail(-15, "adam: buffers must be 4-byte aligned, at one offset inside 16 bytes");
  return hip_check(rc, "adam");
}

extern "C" int32_t tpg_grad_check_impl(int64_t, const float*, float*, hipStream_t);

extern "C" int32_t tpg_grad_check(int64_t numel, const float* grad, float* state, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  if (!grad || !state) return fail(-10, "grad_check: NULL pointer");
  const int rc = tpg_grad_check_impl(numel, grad, state, (hipStream_t)stream);
  if (rc == -1) return fail(-15, "grad_check: gradient buffer must be 16-byte aligned");
  return hip_check(rc, "grad_check");
}

extern "C" void tpg_set_deterministic(int32_t on) { __atomic_store_n(&g_det, on ? 1 : 0, __ATOMIC_RELAXED); }
extern "C" int32_t tpg_get_deterministic(void) { return tpg::deterministic(); }

extern "C" const char* tpg_version(void) { return "tpgan_hip 0.1 gfx950"; }
extern "C" const char* tpg_last_error(void) { return g_err.c_str(); }

// ---- SSD landmark head (MobileNetV2.py:342-649; tpg_ssd.hip)
static int32_t check_ssd(int32_t B, int32_t n, int32_t C, const void* pred, const void* cls, const char* who) {
  if (B < 1 || n < 1 || n > TPG_SSD_MAXN || C < 5) return fail(-2, "%s: B %d, n %d (1..%d), C %d (>= 5)", who, B, n,
                                                              TPG_SSD_MAXN, C);
  if (!pred || !cls) return fail(-10, "%s: NULL input", who);
  if (((uintptr_t)pred | (uintptr_t)cls) % 4) return fail(-15, "%s: inputs must be 4-byte aligned", who);
  return 0;
}

extern "C" int32_t tpg_ssd_loss_fwd(int32_t B, int32_t n, int32_t C, const float* pred, const float* cls,
                                    const float* truth, float width, float height, int32_t k, double ratio_nb,
                                    float alpha, float beta, const float* keys, int32_t* labels, uint8_t* sel,
                                    float* terms, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc = check_ssd(B, n, C, pred, cls, "ssd_loss_fwd");
  if (rc) return rc;
  if (!truth || !keys || !labels || !sel || !terms) return fail(-10, "ssd_loss_fwd: NULL buffer");
  if (!(width > 0.f) || !(height > 0.f)) return fail(-2, "ssd_loss_fwd: image size must be positive");
  if (k < 1 || k > n) return fail(-2, "ssd_loss_fwd: k = %d outside 1..%d", k, n);
  return hip_check(launch_ssd_loss_fwd(B, n, C, k, pred, cls, truth, width, height, ratio_nb, alpha, beta, keys, labels,
                                       sel, terms, (hipStream_t)stream), "ssd_loss_fwd");
}

extern "C" int32_t tpg_ssd_loss_bwd(int32_t B, int32_t n, int32_t C, const float* pred, const float* cls,
                                    const float* truth, float width, float height, float alpha, float beta,
                                    const int32_t* labels, const uint8_t* sel, const float* terms, const float* gout,
                                    float* dloc, float* dcls, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc = check_ssd(B, n, C, pred, cls, "ssd_loss_bwd");
  if (rc) return rc;
  if (!truth || !labels || !sel || !terms || !gout || !dloc || !dcls) return fail(-10, "ssd_loss_bwd: NULL buffer");
  if (!(width > 0.f) || !(height > 0.f)) return fail(-2, "ssd_loss_bwd: image size must be positive");
  return hip_check(launch_ssd_loss_bwd(B, n, C, pred, cls, truth, width, height, alpha, beta, labels, sel, terms, gout,
                                       dloc, dcls, (hipStream_t)stream), "ssd_loss_bwd");
}

extern "C" int32_t tpg_ssd_decode(int32_t B, int32_t n, int32_t C, const float* loc, const float* cls, float conf,
                                  float nms_thr, int32_t top_k, int32_t* keep, float* score, tpg_stream_t stream) {
  TPG_GROUP_SYNC();
  int32_t rc = check_ssd(B, n, C, loc, cls, "ssd_decode");
  if (rc) return rc;
  if (top_k < 1 || top_k > 64) return fail(-2, "ssd_decode: top_k %d outside 1..64", top_k);
  if (!keep || !score) return fail(-10, "ssd_decode: NULL output");
  return hip_check(launch_ssd_decode(B, n, C, loc, cls, conf, nms_thr, top_k, keep, score, (hipStream_t)stream),
                   "ssd_decode");
}

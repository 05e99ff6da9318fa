// Host-side AddressSanitizer sweep of the convolution planner (tpg_capi.hip).
//
// The planner (check_desc -> plan_fwd / plan_bwd_data / maybe_halo / wgrad tile choice ->
// workspace and pre-pack sizing) is pure host code: it runs before any launch and sizes the
// buffers every kernel later indexes, so an out-of-range tap table, a vector overrun or a
// wrong region size shows up here first.  This driver feeds it a deterministic sweep of
// valid geometries (TP-GAN's layer shapes plus a random walk over kernel / stride / pad /
// channel / dtype / transposed / flags combinations) and of malformed descriptors, through
// every entry point that does no device work:
//   tpg_conv2d_workspace (all three ops and out-of-range op codes),
//   tpg_conv2d_packed_bytes, tpg_conv2d_pack_jobs (host job table only), tpg_pack_prepare,
//   and the launch entry points with descriptors check_desc rejects (validation path only).
// Built with `make -C tp-gan_amd asan` (planner object compiled with -fsanitize=address on
// the host side only; the kernels are the product's) and run by tests/test_host_logic.py.
// Exit status: 0 clean, 1 a consistency check failed; ASan aborts on a memory error.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/tpgan.h"

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
  return (uint32_t)(g_rng >> 11);
}
static int pick(const int* v, int n) { return v[rnd() % n]; }

static int g_fail = 0;
static long g_valid = 0, g_rejected = 0, g_jobs = 0;

static void run_one(const tpg_conv_desc& d0, bool expect_valid) {
  // the descriptor is copied to a heap block of exactly its size so a read past it is caught
  tpg_conv_desc* d = (tpg_conv_desc*)malloc(sizeof(tpg_conv_desc));
  memcpy(d, &d0, sizeof(*d));
  size_t ws[3];
  for (int op = 0; op < 3; ++op) ws[op] = tpg_conv2d_workspace(d, op);
  (void)tpg_conv2d_workspace(d, -1);
  (void)tpg_conv2d_workspace(d, 3);
  const bool ok = ws[0] != 0;  // 0 = rejected by check_desc; a valid plan needs >= 256
  if (ok) ++g_valid; else ++g_rejected;
  if (expect_valid && !ok) {
    fprintf(stderr, "valid descriptor rejected: n=%d c=%d->%d %dx%d->%dx%d k=%dx%d s=%d pad=%d,%d,%d,%d T=%d dt=%d: %s\n",
            d->n, d->in_c, d->out_c, d->in_h, d->in_w, d->out_h, d->out_w, d->kh, d->kw, d->stride_h, d->pad_t,
            d->pad_b, d->pad_l, d->pad_r, d->transposed, d->dtype, tpg_last_error());
    g_fail = 1;
  }
  for (int op = 0; op < 3; ++op)
    if ((ws[op] != 0) != ok) { fprintf(stderr, "workspace(op=%d) disagrees with check_desc\n", op); g_fail = 1; }
  for (int op = 0; op < 2; ++op) {
    const size_t pb = tpg_conv2d_packed_bytes(d, op);
    if (ok && pb + 256 > ws[op] && !(d->flags & TPG_FLAG_WPACKED)) {
      // the pre-packed image is the weight part of the op's workspace
      fprintf(stderr, "packed_bytes(op=%d)=%zu exceeds workspace %zu\n", op, pb, ws[op]);
      g_fail = 1;
    }
    // host job table: an exact-size heap block, a short table, and a table of zero entries
    const size_t jb = tpg_pack_job_bytes();
    const int cap = 1 + (int)(rnd() % 8);
    void* jobs = malloc(jb * cap);
    std::vector<float> w(16, 0.f);
    tpg_tensor wt;
    memset(&wt, 0, sizeof(wt));
    wt.data = w.data();
    wt.dtype = TPG_F32;
    char* wp = (char*)0x10000;  // only offset, never dereferenced on the host
    const int n = tpg_conv2d_pack_jobs(d, op, wt, wp, jobs, cap);
    if (n > 0) {
      g_jobs += n;
      const int64_t nb = tpg_pack_prepare(jobs, n);
      if (nb <= 0) { fprintf(stderr, "pack_prepare returned %lld for %d jobs\n", (long long)nb, n); g_fail = 1; }
    }
    (void)tpg_conv2d_pack_jobs(d, op, wt, wp, jobs, 0);
    free(jobs);
  }
  if (!ok) {  // launch entry points must stop at validation (no device work happens)
    tpg_tensor z;
    memset(&z, 0, sizeof(z));
    if (tpg_conv2d_fwd(d, z, z, nullptr, z, z, nullptr, 0, nullptr) == 0 ||
        tpg_conv2d_bwd_data(d, z, z, z, nullptr, 0, nullptr) == 0 ||
        tpg_conv2d_bwd_filter(d, z, z, z, nullptr, 0, nullptr) == 0) {
      fprintf(stderr, "launch entry accepted a rejected descriptor\n");
      g_fail = 1;
    }
  }
  free(d);
}

static tpg_conv_desc conv(int n, int ci, int h, int w, int co, int k, int s, int p, int dt, bool T = false,
                          int op_pad = 0, int pm = TPG_PAD_ZERO) {
  tpg_conv_desc d;
  memset(&d, 0, sizeof(d));
  d.n = n; d.in_c = ci; d.in_h = h; d.in_w = w; d.out_c = co;
  d.kh = d.kw = k; d.stride_h = d.stride_w = s;
  d.pad_t = d.pad_b = d.pad_l = d.pad_r = p;
  d.pad_mode = pm; d.transposed = T ? 1 : 0; d.dtype = dt;
  d.slope = 0.2f; d.res_scale = 1.f;
  if (T) {
    d.out_h = (h - 1) * s - 2 * p + k + op_pad;
    d.out_w = (w - 1) * s - 2 * p + k + op_pad;
  } else {
    d.out_h = (h + 2 * p - k) / s + 1;
    d.out_w = (w + 2 * p - k) / s + 1;
  }
  return d;
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 4000;
  const int dts[3] = {TPG_F32, TPG_BF16, TPG_F16};
  // TP-GAN's own layer shapes (global generator, local pathways, discriminator) at 128x128
  // and bs32, every dtype, plus the full-kernel GEMM forms (fc1, deconv from a 1x1 map)
  for (int dt : dts) {
    const int B = 32;
    run_one(conv(B, 3, 128, 128, 64, 7, 1, 3, dt), true);
    run_one(conv(B, 64, 128, 128, 64, 5, 2, 2, dt), true);
    run_one(conv(B, 64, 64, 64, 128, 3, 2, 1, dt), true);
    run_one(conv(B, 128, 32, 32, 256, 3, 2, 1, dt), true);
    run_one(conv(B, 256, 16, 16, 512, 3, 2, 1, dt), true);
    run_one(conv(B, 512, 8, 8, 512, 3, 1, 1, dt), true);
    run_one(conv(B, 64, 128, 128, 64, 3, 1, 1, dt, false, 0, TPG_PAD_REFLECT), true);
    run_one(conv(B, 64, 1, 1, 64, 8, 1, 0, dt, true), true);
    run_one(conv(B, 512, 8, 8, 256, 3, 2, 1, dt, true, 1), true);
    run_one(conv(B, 256, 16, 16, 128, 3, 2, 1, dt, true, 1), true);
    run_one(conv(B, 128, 32, 32, 64, 3, 2, 1, dt, true, 1), true);
    run_one(conv(B, 96, 128, 128, 64, 5, 1, 2, dt), true);
    run_one(conv(B, 64, 128, 128, 3, 3, 1, 1, dt), true);
    run_one(conv(B, 3, 40, 48, 64, 3, 1, 1, dt), true);
    run_one(conv(B, 64, 20, 24, 128, 3, 2, 1, dt), true);
    run_one(conv(B, 128, 10, 12, 64, 3, 2, 1, dt, true, 1), true);
    run_one(conv(B, 256, 16, 16, 1, 16, 1, 0, dt), true);  // a full-kernel GEMM form
  }
  const int chans[] = {1, 2, 3, 4, 7, 8, 12, 16, 32, 48, 64, 96, 128, 192, 256, 320, 512};
  const int sizes[] = {1, 2, 3, 4, 5, 7, 8, 10, 12, 16, 20, 24, 31, 32, 40, 48, 64, 96, 128, 256};
  const int batches[] = {1, 2, 3, 4, 8, 16, 32};
  for (long it = 0; it < iters; ++it) {
    tpg_conv_desc d;
    memset(&d, 0, sizeof(d));
    d.n = pick(batches, 7);
    d.in_c = pick(chans, 17);
    d.out_c = pick(chans, 17);
    d.in_h = pick(sizes, 20);
    d.in_w = rnd() % 4 ? d.in_h : pick(sizes, 20);
    d.kh = 1 + rnd() % 7;
    d.kw = rnd() % 4 ? d.kh : 1 + rnd() % 7;
    if (rnd() % 40 == 0) d.kh = d.kw = 8 + rnd() % 9;  // large kernels: GEMM form or rejected
    d.stride_h = 1 + rnd() % 4;
    d.stride_w = rnd() % 4 ? d.stride_h : 1 + rnd() % 4;
    d.transposed = rnd() % 4 == 0;
    d.dtype = pick(dts, 3);
    d.pad_t = rnd() % d.kh; d.pad_b = rnd() % 3 ? d.pad_t : rnd() % d.kh;
    d.pad_l = rnd() % d.kw; d.pad_r = rnd() % 3 ? d.pad_l : rnd() % d.kw;
    d.pad_mode = (!d.transposed && rnd() % 5 == 0) ? TPG_PAD_REFLECT : TPG_PAD_ZERO;
    d.act = rnd() % 4; d.slope = 0.2f; d.res_scale = 1.f;
    d.ksplit = rnd() % 3 ? 0 : 1 + rnd() % 16;
    d.data_ksplit = rnd() % 3 ? 0 : 1 + rnd() % 64;
    d.data_algo = rnd() % 3 ? 0 : (int)(rnd() % 4) - 1;
    d.algo = rnd() % 3 ? 0 : (int)(rnd() % 14) - 1;
    d.flags = rnd() % 8;
    if (d.transposed) {
      d.out_h = (d.in_h - 1) * d.stride_h - d.pad_t - d.pad_b + d.kh + (int)(rnd() % d.stride_h);
      d.out_w = (d.in_w - 1) * d.stride_w - d.pad_l - d.pad_r + d.kw + (int)(rnd() % d.stride_w);
    } else {
      d.out_h = (d.in_h + d.pad_t + d.pad_b - d.kh) / d.stride_h + 1;
      d.out_w = (d.in_w + d.pad_l + d.pad_r - d.kw) / d.stride_w + 1;
    }
    // geometries with an empty output or padding the reflect rule forbids are expected to be
    // rejected; everything else must plan
    bool valid = d.out_h > 0 && d.out_w > 0 && (d.in_h + d.pad_t + d.pad_b >= d.kh || d.transposed) &&
                 (d.in_w + d.pad_l + d.pad_r >= d.kw || d.transposed) && d.kh * d.kw <= 49;
    if (d.pad_mode == TPG_PAD_REFLECT &&
        (d.pad_t >= d.in_h || d.pad_b >= d.in_h || d.pad_l >= d.in_w || d.pad_r >= d.in_w))
      valid = false;
    // malformed descriptors: one field corrupted
    if (rnd() % 6 == 0) {
      valid = false;
      switch (rnd() % 9) {
        case 0: d.n = -(int)(rnd() % 3); break;
        case 1: d.in_c = 0; break;
        case 2: d.out_c = -1; break;
        case 3: d.kh = 0; break;
        case 4: d.stride_w = 0; break;
        case 5: d.dtype = 3 + rnd() % 5; break;
        case 6: d.out_h += 1 + d.stride_h; break;
        case 7: d.out_w = d.transposed ? d.out_w - 1 : d.out_w + 1; break;
        case 8: d.pad_t = d.pad_l = 200; break;
      }
    }
    // the random walk only asserts on rejection of shapes the planner documents as covered
    run_one(d, valid && d.kh <= 7 && d.kw <= 7 && d.out_h > 0 && d.out_w > 0 && d.in_h > 0);
  }
  (void)tpg_conv2d_workspace(nullptr, TPG_OP_FWD);
  printf("planner_asan: %ld valid, %ld rejected descriptors, %ld pack jobs, %s\n", g_valid, g_rejected, g_jobs,
         g_fail ? "FAILED" : "ok");
  return g_fail;
}

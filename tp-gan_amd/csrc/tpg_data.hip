// Device-side data path: landmarks -> 5 points -> integer crop boxes ->
// [-1, 1] patches, the work DataAndDataset.py does per sample on the host.
//
//  landmark_boxes_kernel  get_5_landmarks_pixal_position (UtilityMethods.py:148-164), the
//                         TestDataset 128/size rescale (DataAndDataset.py:243-246) and the
//                         crop boxes of process() (DataAndDataset.py:42-54); one thread per face.
//  crop_norm_kernel       PIL crop (zero outside the image) + ToTensor + x*2-1
//                         (DataAndDataset.py:51-54, 216-220, 252-255) for up to 8 jobs
//                         (4 patches + whole images) of a batch in one launch.
//
// Arithmetic follows the reference bit for bit: float32 row sums in index order divided by
// the count (numpy's mean over axis 0 of a (k, 2) float32 array), float32 rescale and mouth
// midpoint, floor to int; u8 / 255 (IEEE division) * 2 - 1 in float32.  Contraction into
// FMA is switched off in both kernels so the rounding sequence is the reference's.
// HBM-bound byte work: each output element is one u8 read (cached across neighbouring
// threads of a row) and one 2- or 4-byte write.
#include "tpg_internal.h"
#include "../../include/tpgan.h"

namespace tpg {
namespace {

struct LmArgs {
  int32_t lo[5], hi[5];  // inclusive landmark index ranges (five_pts_idx)
  int32_t pw[4], ph[4];  // patch (width, height): left_eye, right_eye, nose, mouth
};

__global__ void landmark_boxes_kernel(int n, int npts, const float* __restrict__ lm, const float* __restrict__ scale,
                                      LmArgs a, float* __restrict__ lm5, int32_t* __restrict__ boxes,
                                      int32_t* __restrict__ status) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const float* p = lm + (int64_t)b * npts * 2;
  float pt[5][2];
  for (int j = 0; j < 5; ++j) {
    // numpy slice x[lo:hi+1] clipped to the array, then a sequential float32 sum
    const int s0 = a.lo[j] < 0 ? 0 : (a.lo[j] > npts ? npts : a.lo[j]);
    const int s1 = a.hi[j] + 1 > npts ? npts : a.hi[j] + 1;
    const int cnt = s1 > s0 ? s1 - s0 : 0;
    for (int d = 0; d < 2; ++d) {
      float acc = 0.f;
      for (int i = s0; i < s1; ++i) acc = acc + p[2 * i + d];
      pt[j][d] = cnt > 0 ? acc / (float)cnt : __builtin_nanf("");  // mean of an empty slice: NaN
    }
  }
  if (scale) {
    const float sx = scale[2 * b], sy = scale[2 * b + 1];
    for (int j = 0; j < 5; ++j) {
      pt[j][0] = pt[j][0] * sx;
      pt[j][1] = pt[j][1] * sy;
    }
  }
  for (int j = 0; j < 5; ++j) {
    lm5[(int64_t)b * 10 + 2 * j] = pt[j][0];
    lm5[(int64_t)b * 10 + 2 * j + 1] = pt[j][1];
  }
  // process(): the mouth centre replaces point 3 (DataAndDataset.py:42-43)
  pt[3][0] = (pt[3][0] + pt[4][0]) / 2.0f;
  pt[3][1] = (pt[3][1] + pt[4][1]) / 2.0f;
  int st = 0;
  for (int i = 0; i < 4; ++i) {
    int xy[2];
    for (int d = 0; d < 2; ++d) {
      const float v = pt[i][d];
      if (!(v == v) || fabsf(v) > 1.0e9f) {  // math.floor raises on NaN / inf (ValueError / OverflowError)
        st = 1;
        xy[d] = 0;
      } else {
        xy[d] = (int)floorf(v);
      }
    }
    int32_t* o = boxes + (int64_t)b * 16 + 4 * i;
    o[0] = xy[0] - a.pw[i] / 2 + 1;
    o[1] = xy[1] - a.ph[i] / 2 + 1;
    o[2] = xy[0] + a.pw[i] / 2 + 1;
    o[3] = xy[1] + a.ph[i] / 2 + 1;
  }
  status[b] = st;
}

constexpr int MAX_JOBS = 8;

struct CropJob {
  tpg_tensor out;   // logical [n, c, h, w] (f32 or bf16)
  int32_t h, w;     // output size
  int32_t slot;     // box row slot (left = boxes[b*box_stride + 4*slot], upper = +1); -1: origin
};

struct CropArgs {
  const uint8_t* img;
  int64_t is[4];    // element strides of the logical (n, c, h, w) u8 view
  int32_t c, in_h, in_w, njobs, box_stride;
  const int32_t* boxes;
  CropJob job[MAX_JOBS];
};

__global__ void crop_norm_kernel(CropArgs a) {
#pragma clang fp contract(off)
  const CropJob& j = a.job[blockIdx.y];
  const int b = blockIdx.z;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= j.h * j.w) return;
  const int y = pix / j.w, x = pix - y * j.w;
  int left = 0, upper = 0;
  if (j.slot >= 0) {
    left = a.boxes[(int64_t)b * a.box_stride + 4 * j.slot];
    upper = a.boxes[(int64_t)b * a.box_stride + 4 * j.slot + 1];
  }
  const int sy = upper + y, sx = left + x;
  const bool in = sy >= 0 && sy < a.in_h && sx >= 0 && sx < a.in_w;
  const uint8_t* src = a.img + b * a.is[0] + (int64_t)(in ? sy : 0) * a.is[2] + (int64_t)(in ? sx : 0) * a.is[3];
  char* dst = (char*)j.out.data;
  const int es = j.out.dtype == TPG_BF16 ? 2 : 4;
  const int64_t o = b * j.out.stride[0] + (int64_t)y * j.out.stride[2] + (int64_t)x * j.out.stride[3];
  for (int c = 0; c < a.c; ++c) {
    const float u = in ? (float)src[c * a.is[1]] : 0.f;
    const float v = (u / 255.0f) * 2.0f - 1.0f;
    const int64_t e = o + c * j.out.stride[1];
    if (es == 2)
      reinterpret_cast<__hip_bfloat16*>(dst)[e] = __float2bfloat16(v);
    else
      reinterpret_cast<float*>(dst)[e] = v;
  }
}

}  // namespace
}  // namespace tpg

using namespace tpg;

extern "C" int32_t tpg_landmark_boxes(int32_t n, int32_t npts, const float* lm, const float* scale,
                                      const int32_t* pts_idx, const int32_t* patch_wh, float* lm5, int32_t* boxes,
                                      int32_t* status, tpg_stream_t stream) {
  if (n == 0) return 0;
  if (n < 0 || npts <= 0) return record_error(-2, "landmark_boxes: bad sizes");
  if (!lm || !pts_idx || !patch_wh || !lm5 || !boxes || !status) return record_error(-10, "landmark_boxes: NULL pointer");
  LmArgs a;
  for (int j = 0; j < 5; ++j) {
    a.lo[j] = pts_idx[2 * j];
    a.hi[j] = pts_idx[2 * j + 1];
  }
  for (int i = 0; i < 4; ++i) {
    a.pw[i] = patch_wh[2 * i];
    a.ph[i] = patch_wh[2 * i + 1];
    if (a.pw[i] <= 0 || a.ph[i] <= 0) return record_error(-2, "landmark_boxes: bad patch size");
  }
  hipLaunchKernelGGL(landmark_boxes_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, npts, lm, scale,
                     a, lm5, boxes, status);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : record_error((int)e, hipGetErrorString(e));
}

extern "C" int32_t tpg_crop_normalize(int32_t n, int32_t c, int32_t in_h, int32_t in_w, const uint8_t* img,
                                      const int64_t* img_stride, int32_t njobs, const tpg_tensor* outs,
                                      const int32_t* out_hw, const int32_t* slots, const int32_t* boxes,
                                      int32_t box_stride, tpg_stream_t stream) {
  if (n == 0 || njobs == 0) return 0;
  if (n < 0 || c <= 0 || in_h <= 0 || in_w <= 0 || njobs < 0) return record_error(-2, "crop_normalize: bad sizes");
  if (njobs > MAX_JOBS) return record_error(-2, "crop_normalize: at most 8 jobs per launch");
  if (!img || !img_stride || !outs || !out_hw || !slots) return record_error(-10, "crop_normalize: NULL pointer");
  CropArgs a;
  a.img = img;
  for (int i = 0; i < 4; ++i) a.is[i] = img_stride[i];
  a.c = c;
  a.in_h = in_h;
  a.in_w = in_w;
  a.njobs = njobs;
  a.box_stride = box_stride;
  a.boxes = boxes;
  int maxpix = 1;
  for (int k = 0; k < njobs; ++k) {
    CropJob& j = a.job[k];
    j.out = outs[k];
    j.h = out_hw[2 * k];
    j.w = out_hw[2 * k + 1];
    j.slot = slots[k];
    if (!j.out.data) return record_error(-10, "crop_normalize: output NULL");
    if (j.out.dtype != TPG_F32 && j.out.dtype != TPG_BF16) return record_error(-3, "crop_normalize: bad dtype");
    if (j.h <= 0 || j.w <= 0) return record_error(-2, "crop_normalize: bad output size");
    if (j.slot >= 0 && (!boxes || 4 * j.slot + 2 > box_stride)) return record_error(-2, "crop_normalize: bad box slot");
    if (j.h * j.w > maxpix) maxpix = j.h * j.w;
  }
  hipLaunchKernelGGL(crop_norm_kernel, dim3((maxpix + 255) / 256, njobs, n), dim3(256), 0, (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : record_error((int)e, hipGetErrorString(e));
}

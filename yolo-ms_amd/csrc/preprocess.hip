// Input pipeline on the GPU: the dataset's per-image Resize -> Normalize ->
// ToTensorV2 (yolov8/tools/dataset.py:132-134, applied per sample in __getitem__ :176) and the
// collate's torch.stack (:260) as ONE batched kernel over variable-size uint8 RGB images that were
// copied to the device as decoded (1 byte per channel: a quarter of the PCIe bytes of the
// reference's fp32 CHW tensors), plus the optional horizontal / vertical flips of the training
// transform (:124-127).
//
// Resize follows cv2.resize(INTER_LINEAR) coordinate semantics: half-pixel centres
// (src = (dst + 0.5) * in / out - 0.5), the weight of a coordinate below 0 or at/after the last
// pixel clamped to the edge pixel (fx = 0).  cv2 evaluates uint8 images with 11-bit fixed-point
// weights; here the weights and the blend are fp32 (cv2 is not installed, so its integer
// rounding is not reproduced: parity with it is unpinned, within one intensity level).
// Normalize: (v / 255 - mean_c) / std_c (albumentations' max_pixel_value 255).
#include "yms_common.hpp"

namespace yms {

struct PrepImage {
  const unsigned char* src;   // HWC uint8, rows of `pitch` bytes
  int h, w, pitch, flags;     // flags: bit 0 horizontal flip, bit 1 vertical flip
};

__device__ __forceinline__ void lin_coord(int d, float scale, int n, int& i0, int& i1, float& f) {
  float x = ((float)d + 0.5f) * scale - 0.5f;
  int s = (int)floorf(x);
  f = x - (float)s;
  if (s < 0) { s = 0; f = 0.f; }
  if (s >= n - 1) { s = n - 1; f = 0.f; }
  i0 = s;
  i1 = s + 1 < n ? s + 1 : n - 1;
}

// one thread per output pixel of one image (blockIdx.y = image); output NCHW [n][3][H][W]
template <typename T>
__global__ __launch_bounds__(256) void resize_normalize_kernel(const PrepImage* imgs, int H, int W, float s0, float s1,
                                                               float s2, float b0, float b1, float b2, T* out) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const PrepImage im = imgs[b];
  int oy = p / W, ox = p - oy * W;
  // flips act on the source image before the resize (the transform order of dataset.py)
  const float scy = (float)im.h / (float)H, scx = (float)im.w / (float)W;
  int y0, y1, x0, x1;
  float fy, fx;
  lin_coord(oy, scy, im.h, y0, y1, fy);
  lin_coord(ox, scx, im.w, x0, x1, fx);
  if (im.flags & 1) { x0 = im.w - 1 - x0; x1 = im.w - 1 - x1; }
  if (im.flags & 2) { y0 = im.h - 1 - y0; y1 = im.h - 1 - y1; }
  const unsigned char* r0 = im.src + (long)y0 * im.pitch;
  const unsigned char* r1 = im.src + (long)y1 * im.pitch;
  const float s[3] = {s0, s1, s2}, bb[3] = {b0, b1, b2};
  T* o = out + (long)b * 3 * H * W + p;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v00 = r0[3 * x0 + c], v01 = r0[3 * x1 + c];
    const float v10 = r1[3 * x0 + c], v11 = r1[3 * x1 + c];
    const float top = v00 + fx * (v01 - v00);
    const float bot = v10 + fx * (v11 - v10);
    const float v = top + fy * (bot - top);
    o[(long)c * H * W] = (T)(v * s[c] + bb[c]);
  }
}

// ------------------------------------------------------------------------------------------
// Training augmentation (dataset.py:84-131): the albumentations chain HueSaturationValue ->
// Rotate -> ShiftScaleRotate(shift) -> RandomScale -> Affine(shear) -> Perspective -> flips ->
// Resize -> Normalize, with each image's transforms sampled on the host (yms/data.py) and handed
// over as a chain of stages.  Stage k maps its OUTPUT pixel-index coordinates to its INPUT frame
// (in_w x in_h) through the 3x3 matrix m (homogeneous; affine stages have a last row 0 0 1), then
// applies that input frame's border rule:
//   AUG_REFLECT101 -- cv2.BORDER_REFLECT_101 (Rotate, ShiftScaleRotate): reflected into the frame;
//   AUG_CLAMP      -- resize semantics (RandomScale, flips, the final Resize): clamped to the edge;
//   AUG_CONSTANT   -- cv2.BORDER_CONSTANT 0 (Affine, Perspective): a coordinate more than half a
//                     pixel outside the frame makes the pixel 0 before Normalize.
// One thread per output pixel walks the chain from the last stage back to the source image and
// samples it ONCE, bilinearly (albumentations resamples after every geometric transform; here the
// coordinates are composed exactly and only the final sample interpolates -- parity with the
// sequential resampling is unpinned, and so is cv2's fixed-point rounding).  The HSV shift is
// applied to each of the four source taps before the blend, in cv2's 8-bit HSV encoding (H in
// [0, 180), S and V in [0, 255]) with albumentations' LUT semantics: hue (h + dh) mod 180, S and V
// clipped to [0, 255], each truncated to an integer, as on uint8 images (restated; unpinned).
enum { AUG_REFLECT101 = 0, AUG_CLAMP = 1, AUG_CONSTANT = 2 };
constexpr int AUG_MAX_STAGES = 8;

struct AugStage {
  float m[9];
  int in_w, in_h, border, pad_;
};
struct AugImage {
  const unsigned char* src;
  int h, w, pitch, nst;
  float hsv[3];       // hue, saturation, value shifts (LUT units)
  int do_hsv;
  AugStage st[AUG_MAX_STAGES];
};

__device__ __forceinline__ float reflect101(float x, int n) {
#pragma clang fp contract(off)
  if (n <= 1) return 0.f;
  const float L = (float)(n - 1);
  const float period = 2.f * L;
  x = fabsf(x);
  x = x - period * floorf(x / period);
  if (x > L) x = period - x;
  return x;
}

// cv2 COLOR_RGB2HSV / COLOR_HSV2RGB for 8-bit images, restated in fp32 (values rounded to the
// nearest integer like cv2's saturate_cast; no FMA contraction, so the host restatement in
// oracle/preprocess_ref.py evaluates the same fp32 operations)
__device__ __forceinline__ void rgb2hsv8(float r, float g, float b, float& h, float& s, float& v) {
#pragma clang fp contract(off)
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b));
  const float d = mx - mn;
  v = mx;
  s = mx > 0.f ? rintf(255.f * d / mx) : 0.f;
  float hd = 0.f;
  if (d > 0.f) {
    if (mx == r) hd = 60.f * (g - b) / d;
    else if (mx == g) hd = 120.f + 60.f * (b - r) / d;
    else hd = 240.f + 60.f * (r - g) / d;
    if (hd < 0.f) hd += 360.f;
  }
  h = rintf(hd * 0.5f);
  if (h >= 180.f) h -= 180.f;
}
__device__ __forceinline__ void hsv2rgb8(float h, float s, float v, float& r, float& g, float& b) {
#pragma clang fp contract(off)
  const float sf = s * (1.f / 255.f);
  float hh = h * 2.f / 60.f;                   // sector in [0, 6)
  const int i = (int)floorf(hh);
  const float f = hh - (float)i;
  const float p = v * (1.f - sf), q = v * (1.f - sf * f), t = v * (1.f - sf * (1.f - f));
  switch (((i % 6) + 6) % 6) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
  r = fminf(fmaxf(rintf(r), 0.f), 255.f);
  g = fminf(fmaxf(rintf(g), 0.f), 255.f);
  b = fminf(fmaxf(rintf(b), 0.f), 255.f);
}
__device__ __forceinline__ void hsv_shift8(const float (&sh)[3], float& r, float& g, float& b) {
#pragma clang fp contract(off)
  float h, s, v;
  rgb2hsv8(r, g, b, h, s, v);
  h = h + sh[0];
  h = h - 180.f * floorf(h / 180.f);
  h = floorf(h);
  s = floorf(fminf(fmaxf(s + sh[1], 0.f), 255.f));
  v = floorf(fminf(fmaxf(v + sh[2], 0.f), 255.f));
  hsv2rgb8(h, s, v, r, g, b);
}

template <typename T>
__global__ __launch_bounds__(256) void augment_normalize_kernel(const AugImage* imgs, int H, int W, float s0, float s1,
                                                                float s2, float b0, float b1, float b2, T* out) {
#pragma clang fp contract(off)   // plain fp32 operations in source order: oracle/preprocess_ref.py replays them
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const AugImage& im = imgs[b];
  const int oy = p / W, ox = p - oy * W;
  float x = (float)ox, y = (float)oy;
  bool blank = false;
  for (int k = im.nst - 1; k >= 0; --k) {
    const AugStage& s = im.st[k];
    const float X = s.m[0] * x + s.m[1] * y + s.m[2];
    const float Y = s.m[3] * x + s.m[4] * y + s.m[5];
    const float Z = s.m[6] * x + s.m[7] * y + s.m[8];
    x = X / Z;
    y = Y / Z;
    if (!(fabsf(x) < 1e7f && fabsf(y) < 1e7f)) { blank = true; break; }
    if (s.border == AUG_REFLECT101) {
      x = reflect101(x, s.in_w);
      y = reflect101(y, s.in_h);
    } else if (s.border == AUG_CONSTANT) {
      if (x < -0.5f || y < -0.5f || x > (float)s.in_w - 0.5f || y > (float)s.in_h - 0.5f) { blank = true; break; }
      x = fminf(fmaxf(x, 0.f), (float)(s.in_w - 1));
      y = fminf(fmaxf(y, 0.f), (float)(s.in_h - 1));
    } else {
      x = fminf(fmaxf(x, 0.f), (float)(s.in_w - 1));
      y = fminf(fmaxf(y, 0.f), (float)(s.in_h - 1));
    }
  }
  const float sc[3] = {s0, s1, s2}, bb[3] = {b0, b1, b2};
  T* o = out + (long)b * 3 * H * W + p;
  float v[3] = {0.f, 0.f, 0.f};
  if (!blank) {
    const int x0 = min((int)floorf(x), im.w - 1), y0 = min((int)floorf(y), im.h - 1);
    const float fx = x - (float)x0, fy = y - (float)y0;
    const int x1 = min(x0 + 1, im.w - 1), y1 = min(y0 + 1, im.h - 1);
    float t[4][3];
    const int xs[4] = {x0, x1, x0, x1}, ys[4] = {y0, y0, y1, y1};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned char* px = im.src + (long)ys[q] * im.pitch + 3 * xs[q];
      t[q][0] = px[0];
      t[q][1] = px[1];
      t[q][2] = px[2];
      if (im.do_hsv) hsv_shift8(im.hsv, t[q][0], t[q][1], t[q][2]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float top = t[0][c] + fx * (t[1][c] - t[0][c]);
      const float bot = t[2][c] + fx * (t[3][c] - t[2][c]);
      v[c] = top + fy * (bot - top);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) o[(long)c * H * W] = (T)(v[c] * sc[c] + bb[c]);
}

}  // namespace yms

using namespace yms;

extern "C" {

yms_status yms_resize_normalize(int dtype, int n, const void* images, int out_h, int out_w, const float* mean,
                                const float* std, void* out, void* stream) {
  if (n <= 0) return YMS_OK;
  if (!images || !out || !mean || !std || out_h <= 0 || out_w <= 0) return YMS_ERR_INVALID;
  for (int c = 0; c < 3; ++c)
    if (!(std[c] > 0.f)) return YMS_ERR_INVALID;
  // v / 255 - mean) / std = v * s + b
  const float s0 = 1.f / (255.f * std[0]), s1 = 1.f / (255.f * std[1]), s2 = 1.f / (255.f * std[2]);
  const float b0 = -mean[0] / std[0], b1 = -mean[1] / std[1], b2 = -mean[2] / std[2];
  const dim3 grid((unsigned)cdiv((long)out_h * out_w, 256), (unsigned)n);
  const PrepImage* im = (const PrepImage*)images;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case YMS_F32:
      hipLaunchKernelGGL(resize_normalize_kernel<float>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0, b1,
                         b2, (float*)out);
      break;
    case YMS_BF16:
      hipLaunchKernelGGL(resize_normalize_kernel<bf16>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0, b1,
                         b2, (bf16*)out);
      break;
    case YMS_F16:
      hipLaunchKernelGGL(resize_normalize_kernel<f16>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0, b1,
                         b2, (f16*)out);
      break;
    default:
      return YMS_ERR_INVALID;
  }
  return launch_status();
}

size_t yms_augment_image_bytes(void) { return sizeof(AugImage); }

yms_status yms_augment_normalize(int dtype, int n, const void* images, int out_h, int out_w, const float* mean,
                                 const float* std, void* out, void* stream) {
  if (n <= 0) return YMS_OK;
  if (!images || !out || !mean || !std || out_h <= 0 || out_w <= 0) return YMS_ERR_INVALID;
  for (int c = 0; c < 3; ++c)
    if (!(std[c] > 0.f)) return YMS_ERR_INVALID;
  const float s0 = 1.f / (255.f * std[0]), s1 = 1.f / (255.f * std[1]), s2 = 1.f / (255.f * std[2]);
  const float b0 = -mean[0] / std[0], b1 = -mean[1] / std[1], b2 = -mean[2] / std[2];
  const dim3 grid((unsigned)cdiv((long)out_h * out_w, 256), (unsigned)n);
  const AugImage* im = (const AugImage*)images;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case YMS_F32:
      hipLaunchKernelGGL(augment_normalize_kernel<float>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0,
                         b1, b2, (float*)out);
      break;
    case YMS_BF16:
      hipLaunchKernelGGL(augment_normalize_kernel<bf16>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0,
                         b1, b2, (bf16*)out);
      break;
    case YMS_F16:
      hipLaunchKernelGGL(augment_normalize_kernel<f16>, grid, dim3(256), 0, st, im, out_h, out_w, s0, s1, s2, b0,
                         b1, b2, (f16*)out);
      break;
    default:
      return YMS_ERR_INVALID;
  }
  return launch_status();
}

}  // extern "C"

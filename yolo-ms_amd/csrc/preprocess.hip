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

}  // extern "C"

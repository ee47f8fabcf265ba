// Detection loss and target assignment on gfx950: the semantics of the
// reference's ComputeLoss (yolov8/tools/loss.py:94-677, restated in oracle/loss_ref.py), fused
// with its analytic gradient so one forward launch sequence yields the three loss terms and
// d(total)/d(head maps) in the head maps' own NHWC layout:
//
//   decode_kernel   per anchor: softmax over each side's 16 DFL bins, expected offsets (grid
//                   units, loss.py:127-206), decoded (cx, cy, w, h) in pixels
//   topk_kernel     per target row: plain IoU of every decoded box with the GT (loss.py:252),
//                   k = min(10, #IoU > 0.1) best anchors (ties -> lower index)  (loss.py:312-315)
//   assign_kernel   per image, GTs in target order: fg mask, target box / l-t-r-b OVERWRITTEN by
//                   later GTs, class bits accumulated (loss.py:297-365)
//   cls_kernel      BCE-with-logits over every anchor x class: per-image sums + gradient
//                   (the mean is added twice when the image has foreground, loss.py:530/551)
//   box_kernel      per foreground anchor: 1 - CIoU (or IoU / GIoU / DIoU) and the two-bin DFL
//                   cross entropy, per-image sums and NaN flags (loss.py:553-648)
//   boxgrad_kernel  their gradient into the 64 DFL logits (zeros for background anchors,
//                   no box gradient for an image whose box loss was NaN)
//   finalize_kernel per-image means -> batch means -> 7.5 box + 0.5 cls + 1.5 dfl
//
// Reductions are deterministic (fixed-order block partials, fp64 finals).  HBM-bound: the head
// maps are read twice (cls + box) and the gradient written once.
#include <algorithm>
#include <cmath>

#include "yms_common.hpp"

namespace yms {

constexpr int DL_DFL = 16;              // bins per side (the head's reg_max)
constexpr int DL_TOPK = 10;
constexpr float DL_IOU_MIN = 0.1f;
constexpr float DL_EPS = 1e-7f;
constexpr int DL_MAXL = 4;
constexpr int DL_ASSIGN_LDS = 4096;     // target rows staged per image in assign_kernel

struct LossLevels {
  const void* x[DL_MAXL];   // head maps, NHWC with channel stride ld
  void* g[DL_MAXL];         // gradients (same layout), may be null
  int h[DL_MAXL], w[DL_MAXL], off[DL_MAXL + 1];
  float stride[DL_MAXL];
  int nl, ld;
};

__device__ __forceinline__ int level_of(const LossLevels& L, int a) {
  int l = 0;
  while (l + 1 < L.nl && a >= L.off[l + 1]) ++l;
  return l;
}
// anchor a of image b -> element offset of its row, level, and pixel centre (loss.py:424-431)
__device__ __forceinline__ long anchor_row(const LossLevels& L, int b, int a, int& l, float& ax, float& ay) {
  l = level_of(L, a);
  const int r = a - L.off[l], hy = r / L.w[l], wx = r - hy * L.w[l];
  ax = ((float)wx + 0.5f) * L.stride[l];
  ay = ((float)hy + 0.5f) * L.stride[l];
  return (((long)b * L.h[l] + hy) * L.w[l] + wx) * L.ld;
}

template <typename T>
__device__ __forceinline__ void load_dist(const T* row, float (&v)[4 * DL_DFL]) {
#pragma unroll
  for (int k = 0; k < 4 * DL_DFL / 8; ++k) {
    float t[8];
    Vec8<T>::load(row + 8 * k, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[8 * k + i] = t[i];
  }
}

// softmax of each side's bins in place (v -> probabilities), expected bin index e[s], and the
// log-sum-exp of each side's logits (log-probabilities as logit - lse, as log_softmax)
__device__ __forceinline__ void dfl_softmax(float (&v)[4 * DL_DFL], float (&e)[4], float (&lse)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float m = v[s * DL_DFL];
#pragma unroll
    for (int i = 1; i < DL_DFL; ++i) m = fmaxf(m, v[s * DL_DFL + i]);
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < DL_DFL; ++i) {
      const float q = expf(v[s * DL_DFL + i] - m);
      v[s * DL_DFL + i] = q;
      z += q;
    }
    lse[s] = m + logf(z);
    const float iz = 1.0f / z;
    float ex = 0.f;
#pragma unroll
    for (int i = 0; i < DL_DFL; ++i) {
      v[s * DL_DFL + i] *= iz;
      ex += v[s * DL_DFL + i] * (float)i;
    }
    e[s] = ex;
  }
}

// (cx, cy, w, h) -> x1 y1 x2 y2 as bbox_iou converts (loss.py:26-29)
__device__ __forceinline__ void cxcywh_to_xyxy(const float* c, float (&b)[4]) {
  b[0] = c[0] - c[2] / 2;
  b[1] = c[1] - c[3] / 2;
  b[2] = c[0] + c[2] / 2;
  b[3] = c[1] + c[3] / 2;
}

__device__ __forceinline__ float plain_iou(const float (&p)[4], const float (&g)[4]) {
  const float iw = fmaxf(fminf(p[2], g[2]) - fmaxf(p[0], g[0]), 0.f);
  const float ih = fmaxf(fminf(p[3], g[3]) - fmaxf(p[1], g[1]), 0.f);
  const float inter = iw * ih;
  const float un = (p[2] - p[0]) * (p[3] - p[1]) + (g[2] - g[0]) * (g[3] - g[1]) - inter + DL_EPS;
  return inter / un;
}

// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void decode_kernel(LossLevels L, int A, float* pbox) {
  const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (a >= A) return;
  int l;
  float ax, ay;
  const long row = anchor_row(L, b, a, l, ax, ay);
  float v[4 * DL_DFL], e[4], lse[4];
  load_dist(reinterpret_cast<const T*>(L.x[l]) + row, v);
  dfl_softmax(v, e, lse);
  const float x1 = ax - e[0], y1 = ay - e[1], x2 = ax + e[2], y2 = ay + e[3];
  float4 o = make_float4((x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1);
  reinterpret_cast<float4*>(pbox)[(long)b * A + a] = o;
}

// per target row j: top-k anchors by IoU (value desc, index asc)
__global__ __launch_bounds__(256) void topk_kernel(const float* tg, int B, int A, float img_w, float img_h,
                                                   const float* pbox, int* kcnt, int* kidx) {
  const int j = blockIdx.x, tid = threadIdx.x;
  const float* t = tg + (long)j * 6;
  const int b = (int)t[0];
  if (!(t[0] >= 0.f) || b >= B) {   // not an image of this batch: never assigned
    if (tid == 0) kcnt[j] = 0;
    return;
  }
  const float gc[4] = {t[2] * img_w, t[3] * img_h, t[4] * img_w, t[5] * img_h};
  float g[4];
  cxcywh_to_xyxy(gc, g);
  // thread-local top-k, sorted descending (value desc, index asc)
  float bv[DL_TOPK];
  int bi[DL_TOPK];
#pragma unroll
  for (int q = 0; q < DL_TOPK; ++q) { bv[q] = -1.f; bi[q] = 0x7fffffff; }
  int cnt = 0;
  const float4* pb = reinterpret_cast<const float4*>(pbox) + (long)b * A;
  for (int a = tid; a < A; a += 256) {
    const float4 c4 = pb[a];
    const float c[4] = {c4.x, c4.y, c4.z, c4.w};
    float p[4];
    cxcywh_to_xyxy(c, p);
    const float iou = plain_iou(p, g);
    cnt += iou > DL_IOU_MIN ? 1 : 0;
    if (iou > bv[DL_TOPK - 1]) {     // strictly greater: an equal later index ranks after
      float cv = iou;
      int ci = a;
#pragma unroll
      for (int q = 0; q < DL_TOPK; ++q) {
        if (cv > bv[q]) {
          const float tv = bv[q];
          const int ti = bi[q];
          bv[q] = cv; bi[q] = ci;
          cv = tv; ci = ti;
        }
      }
    }
  }
  __shared__ int scnt[4];
  __shared__ float rv[4];
  __shared__ int ri[4], rt[4];
  int c = cnt;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  if ((tid & 63) == 0) scnt[tid >> 6] = c;
  __syncthreads();
  const int total = (scnt[0] + scnt[1]) + (scnt[2] + scnt[3]);
  const int k = total < DL_TOPK ? total : DL_TOPK;
  // k rounds of block argmax over each thread's current head (value desc, index asc)
  int head = 0;
  for (int r = 0; r < k; ++r) {
    float v = head < DL_TOPK ? bv[0] : -1.f;
    int ix = head < DL_TOPK ? bi[0] : 0x7fffffff;
    int owner = tid;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float ov = __shfl_xor(v, m);
      const int oi = __shfl_xor(ix, m), oo = __shfl_xor(owner, m);
      if (ov > v || (ov == v && oi < ix)) { v = ov; ix = oi; owner = oo; }
    }
    if ((tid & 63) == 0) { rv[tid >> 6] = v; ri[tid >> 6] = ix; rt[tid >> 6] = owner; }
    __syncthreads();
    float wv = rv[0];
    int wi = ri[0], wo = rt[0];
    for (int q = 1; q < 4; ++q)
      if (rv[q] > wv || (rv[q] == wv && ri[q] < wi)) { wv = rv[q]; wi = ri[q]; wo = rt[q]; }
    if (tid == 0) kidx[(long)j * DL_TOPK + r] = wi;
    if (tid == wo) {                  // pop the winner's head
#pragma unroll
      for (int q = 0; q < DL_TOPK - 1; ++q) { bv[q] = bv[q + 1]; bi[q] = bi[q + 1]; }
      bv[DL_TOPK - 1] = -1.f;
      bi[DL_TOPK - 1] = 0x7fffffff;
      ++head;
    }
    __syncthreads();
  }
  if (tid == 0) kcnt[j] = k;
}

// per image: apply the GTs in target order
__global__ __launch_bounds__(256) void assign_kernel(const float* tg, int M, int A, int nc, int nw, float img_w,
                                                     float img_h, LossLevels L, const int* kcnt, const int* kidx,
                                                     unsigned char* fg, float* tbox, float* tltrb,
                                                     unsigned* cbits, int* nfg) {
  const int b = blockIdx.x, tid = threadIdx.x;
  unsigned char* f = fg + (long)b * A;
  unsigned* bits = cbits + (long)b * A * nw;
  for (int a = tid; a < A; a += 256) f[a] = 0;
  for (long i = tid; i < (long)A * nw; i += 256) bits[i] = 0u;
  // this image's target rows, in target order (one scan of the image column)
  __shared__ int mine[DL_ASSIGN_LDS];
  __shared__ int nmine;
  if (tid == 0) nmine = 0;
  __syncthreads();
  const bool staged = M <= DL_ASSIGN_LDS;
  if (staged) {
    for (int j0 = 0; j0 < M; j0 += 256) {
      const int j = j0 + tid;
      const bool hit = j < M && tg[(long)j * 6] >= 0.f && (int)tg[(long)j * 6] == b;
      const unsigned long long bal = __ballot(hit);
      __shared__ int wcnt[4];
      if ((tid & 63) == 0) wcnt[tid >> 6] = __popcll(bal);
      __syncthreads();
      int base = nmine;
      for (int q = 0; q < (tid >> 6); ++q) base += wcnt[q];
      if (hit) mine[base + __popcll(bal & ((1ull << (tid & 63)) - 1ull))] = j;
      __syncthreads();
      if (tid == 0) nmine += (wcnt[0] + wcnt[1]) + (wcnt[2] + wcnt[3]);
      __syncthreads();
    }
  }
  const int nj = staged ? nmine : M;
  for (int jj = 0; jj < nj; ++jj) {
    const int j = staged ? mine[jj] : jj;
    const float* t = tg + (long)j * 6;
    if (!staged && (!(t[0] >= 0.f) || (int)t[0] != b)) continue;    // block-uniform
    const int k = kcnt[j];
    const int lab = (int)t[1];
    if (tid < k) {
      const int a = kidx[(long)j * DL_TOPK + tid];
      const float gc[4] = {t[2] * img_w, t[3] * img_h, t[4] * img_w, t[5] * img_h};
      f[a] = 1;
      float4* tb = reinterpret_cast<float4*>(tbox) + (long)b * A + a;
      *tb = make_float4(gc[0], gc[1], gc[2], gc[3]);
      // l-t-r-b distances of the anchor centre to the GT sides (loss.py:327-353)
      const float x1 = gc[0] - gc[2] / 2, y1 = gc[1] - gc[3] / 2;
      const float x2 = gc[0] + gc[2] / 2, y2 = gc[1] + gc[3] / 2;
      int l;
      float ax, ay;
      (void)anchor_row(L, 0, a, l, ax, ay);
      reinterpret_cast<float4*>(tltrb)[(long)b * A + a] = make_float4(ax - x1, ay - y1, x2 - ax, y2 - ay);
      if (lab >= 0 && lab < nc) bits[(long)a * nw + (lab >> 5)] |= 1u << (lab & 31);
    }
    __syncthreads();
  }
  int c = 0;
  for (int a = tid; a < A; a += 256) c += f[a];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  __shared__ int sc[4];
  if ((tid & 63) == 0) sc[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) nfg[b] = (sc[0] + sc[1]) + (sc[2] + sc[3]);
}

// BCEWithLogits value (1 - t) x + (1 + (pw - 1) t) softplus(-x) and its derivative
// sigmoid(x) (1 + (pw - 1) t) - pw t, from one exponential and one logarithm
__device__ __forceinline__ float bce_logits(float x, float t, float pw, float& dx) {
  const float e = __expf(-fabsf(x));
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  const float sig = x >= 0.f ? r : e * r;
  const float lw = 1.f + (pw - 1.f) * t;
  dx = sig * lw - pw * t;
  // log(1 + e) by the hardware logarithm: absolute error ~1e-7 (also where e < eps and log1p
  // would keep more relative digits of a ~1e-7 term), well inside the loss tolerance
  return (1.f - t) * x + lw * (fmaxf(-x, 0.f) + __logf(1.f + e));
}

// block partial sums (fixed order) of one float per thread -> part[slot]
__device__ __forceinline__ void block_sum_store(float v, float* part, long slot) {
  __shared__ float s[4];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[slot] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
}

// BCE over anchors x classes: thread = (anchor, 8-class chunk)
template <typename T>
__global__ __launch_bounds__(256) void cls_kernel(LossLevels L, int A, int nc, int nw, const unsigned* cbits,
                                                  const int* nfg, const float* pos_weight, float gscale,
                                                  float* part) {
  const int b = blockIdx.y;
  const int G = (nc + 7) / 8;
  const int i = blockIdx.x * 256 + threadIdx.x;       // A * G < 2^31 (host-checked): 32-bit division
  float acc = 0.f;
  if (i < A * G) {
    const int a = i / G, q = i - a * G;
    const int c0 = q * 8, nv = min(8, nc - c0);
    int l;
    float ax, ay;
    const long row = anchor_row(L, b, a, l, ax, ay) + 4 * DL_DFL + c0;
    float x[8];
    load8(reinterpret_cast<const T*>(L.x[l]) + row, nv, x);
    const unsigned* bits = cbits + ((long)b * A + a) * nw;
    const float f = nfg[b] > 0 ? 2.f : 1.f;      // loss.py:530 + :551
    float gr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      gr[k] = 0.f;
      if (k < nv) {
        const int c = c0 + k;
        const float t = (bits[c >> 5] >> (c & 31)) & 1u ? 1.f : 0.f;
        const float pw = pos_weight ? pos_weight[c] : 1.f;
        float dx;
        acc += bce_logits(x[k], t, pw, dx);
        gr[k] = dx * f * gscale;
      }
    }
    if (L.g[l]) store8(reinterpret_cast<T*>(L.g[l]) + row, nv, gr);
  }
  block_sum_store(acc, part, (long)b * gridDim.x + blockIdx.x);
}

// box + DFL value of one foreground anchor (and, GRAD, d/d logits scaled by sb, sd)
template <bool GRAD>
__device__ __forceinline__ void box_dfl(float (&v)[4 * DL_DFL], float ax, float ay, float stride,
                                        const float4 tb4, const float4 tl4, int iou_type, float sb, float sd,
                                        float& lbox, float& ldfl) {
  // DFL targets in stride units and their two bins (loss.py:602-630), read before the softmax
  const float tl[4] = {tl4.x / stride, tl4.y / stride, tl4.z / stride, tl4.w / stride};
  int li[4], ri[4];
  float wl[4], wr[4], xl[4], xr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float fl = floorf(tl[s]);
    const float fr = floorf(tl[s] + 1.0f);
    wr[s] = tl[s] - fl;
    wl[s] = 1.0f - wr[s];
    li[s] = (int)fminf(fmaxf(fl, 0.f), (float)(DL_DFL - 1));
    ri[s] = (int)fminf(fmaxf(fr, 0.f), (float)(DL_DFL - 1));
    xl[s] = v[s * DL_DFL + li[s]];
    xr[s] = v[s * DL_DFL + ri[s]];
  }
  float e[4], lse[4];
  dfl_softmax(v, e, lse);     // v: probabilities
  // decoded box, converted (cx, cy, w, h) -> xyxy exactly as the reference's chain does
  const float x1 = ax - e[0], y1 = ay - e[1], x2 = ax + e[2], y2 = ay + e[3];
  const float pc[4] = {(x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1};
  const float tc[4] = {tb4.x, tb4.y, tb4.z, tb4.w};
  float p[4], g[4];
  cxcywh_to_xyxy(pc, p);
  cxcywh_to_xyxy(tc, g);
  // IoU terms
  const float iwr = fminf(p[2], g[2]) - fmaxf(p[0], g[0]);
  const float ihr = fminf(p[3], g[3]) - fmaxf(p[1], g[1]);
  const float iw = fmaxf(iwr, 0.f), ih = fmaxf(ihr, 0.f);
  const float inter = iw * ih;
  const float w1 = p[2] - p[0], h1 = p[3] - p[1], w2 = g[2] - g[0], h2 = g[3] - g[1];
  const float un = w1 * h1 + w2 * h2 - inter + DL_EPS;
  const float iou = inter / un;
  float val = iou;
  // d(val)/d(p0..p3)
  float dp[4] = {0.f, 0.f, 0.f, 0.f};
  if (GRAD) {
    // d iou = (d inter * un - inter * d un) / un^2,  d un = d(w1 h1) - d inter
    float di[4] = {0.f, 0.f, 0.f, 0.f};
    if (iwr >= 0.f) {         // clamp(min=0) passes the gradient at 0 (torch semantics)
      if (p[2] < g[2]) di[2] += ih;
      if (p[0] > g[0]) di[0] -= ih;
    }
    if (ihr >= 0.f) {
      if (p[3] < g[3]) di[3] += iw;
      if (p[1] > g[1]) di[1] -= iw;
    }
    const float da[4] = {-h1, -w1, h1, w1};
    const float iu2 = 1.f / (un * un);
#pragma unroll
    for (int k = 0; k < 4; ++k) dp[k] = (di[k] * un - inter * (da[k] - di[k])) * iu2;
  }
  if (iou_type != 0) {
    const float cwr = fmaxf(p[2], g[2]) - fminf(p[0], g[0]);
    const float chr = fmaxf(p[3], g[3]) - fminf(p[1], g[1]);
    const float cw = fmaxf(cwr, 0.f), ch = fmaxf(chr, 0.f);
    if (iou_type == 1) {       // GIoU
      const float ca = cw * ch + DL_EPS;
      val = iou - (ca - un) / ca;
      if (GRAD) {
        // d[-(ca - un)/ca] = -(d ca * un ... ) : -(1 - un/ca) -> d = (d un * ca - un * d ca) / ca^2
        float dca[4] = {0.f, 0.f, 0.f, 0.f};
        if (cwr >= 0.f) {
          if (p[2] > g[2]) dca[2] += ch;
          if (p[0] < g[0]) dca[0] -= ch;
        }
        if (chr >= 0.f) {
          if (p[3] > g[3]) dca[3] += cw;
          if (p[1] < g[1]) dca[1] -= cw;
        }
        // un' = d(w1 h1) - d inter: recompute d inter from dp is messy; rebuild it
        float di[4] = {0.f, 0.f, 0.f, 0.f};
        if (iwr >= 0.f) { if (p[2] < g[2]) di[2] += ih; if (p[0] > g[0]) di[0] -= ih; }
        if (ihr >= 0.f) { if (p[3] < g[3]) di[3] += iw; if (p[1] > g[1]) di[1] -= iw; }
        const float da[4] = {-h1, -w1, h1, w1};
#pragma unroll
        for (int k = 0; k < 4; ++k) dp[k] += ((da[k] - di[k]) * ca - un * dca[k]) / (ca * ca);
      }
    } else {                   // DIoU / CIoU
      const float rx = (p[0] + p[2]) / 2 - (g[0] + g[2]) / 2;
      const float ry = (p[1] + p[3]) / 2 - (g[1] + g[3]) / 2;
      const float rho2 = rx * rx + ry * ry;
      const float c2 = cw * cw + ch * ch;
      const float dterm = rho2 / c2;
      val = iou - dterm;
      if (GRAD) {
        // d(rho2/c2) = (d rho2 c2 - rho2 d c2) / c2^2
        const float drho[4] = {rx, ry, rx, ry};            // d rho2 / d p_k = 2 r * 1/2
        float dc2[4] = {0.f, 0.f, 0.f, 0.f};
        if (cwr >= 0.f) {
          if (p[2] > g[2]) dc2[2] += 2.f * cw;
          if (p[0] < g[0]) dc2[0] -= 2.f * cw;
        }
        if (chr >= 0.f) {
          if (p[3] > g[3]) dc2[3] += 2.f * ch;
          if (p[1] < g[1]) dc2[1] -= 2.f * ch;
        }
        const float ic = 1.f / (c2 * c2);
#pragma unroll
        for (int k = 0; k < 4; ++k) dp[k] -= (drho[k] * c2 - rho2 * dc2[k]) * ic;
      }
      if (iou_type == 3) {     // CIoU: - alpha v, alpha detached
        const float at = atanf(w2 / (h2 + DL_EPS)) - atanf(w1 / (h1 + DL_EPS));
        const float k4 = 4.f / (float)(M_PI * M_PI);
        const float vv = k4 * at * at;
        const float alpha = vv / (1.f - iou + vv + DL_EPS);
        val -= alpha * vv;
        if (GRAD) {
          // d v / d(w1, h1): v = k4 at^2, at = atan(w2/(h2+eps)) - atan(w1/(h1+eps))
          const float hh = h1 + DL_EPS;
          const float q = w1 / hh;
          const float den = 1.f / (1.f + q * q);
          const float dat_dw1 = -den / hh, dat_dh1 = den * w1 / (hh * hh);
          const float dv_dw1 = 2.f * k4 * at * dat_dw1, dv_dh1 = 2.f * k4 * at * dat_dh1;
          // w1 = p2 - p0, h1 = p3 - p1
          dp[0] += alpha * dv_dw1;
          dp[2] -= alpha * dv_dw1;
          dp[1] += alpha * dv_dh1;
          dp[3] -= alpha * dv_dh1;
        }
      }
    }
  }
  lbox = 1.f - val;
  // DFL: two-bin cross entropy, -log_softmax at the two bins (loss.py:644-645)
  float dfl = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) dfl += (lse[s] - xl[s]) * wl[s] + (lse[s] - xr[s]) * wr[s];
  ldfl = dfl;
  if (GRAD) {
    // box: loss 1 - val -> d/dp = -dp; p0 = ax - e0 (d/de0 = -1), p1 = ay - e1, p2 = ax + e2, p3 = ay + e3
    const float ge[4] = {dp[0] * sb, dp[1] * sb, -dp[2] * sb, -dp[3] * sb};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < DL_DFL; ++i) {
        const float pr = v[s * DL_DFL + i];
        float gi = ge[s] * pr * ((float)i - e[s]);      // d e_s / d logit_i = p_i (i - e_s)
        gi += sd * (pr - (i == li[s] ? wl[s] : 0.f) - (i == ri[s] ? wr[s] : 0.f));
        v[s * DL_DFL + i] = gi;
      }
  }
}

// per foreground anchor: box and DFL sums, NaN flags
template <typename T>
__global__ __launch_bounds__(256) void box_kernel(LossLevels L, int A, const unsigned char* fg, const float* tbox,
                                                  const float* tltrb, int iou_type, float* part) {
  const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  float lb = 0.f, ld = 0.f, nb = 0.f, nd = 0.f;
  if (a < A && fg[(long)b * A + a]) {
    int l;
    float ax, ay;
    const long row = anchor_row(L, b, a, l, ax, ay);
    float v[4 * DL_DFL];
    load_dist(reinterpret_cast<const T*>(L.x[l]) + row, v);
    const float4 tb = reinterpret_cast<const float4*>(tbox)[(long)b * A + a];
    const float4 tl = reinterpret_cast<const float4*>(tltrb)[(long)b * A + a];
    box_dfl<false>(v, ax, ay, L.stride[l], tb, tl, iou_type, 0.f, 0.f, lb, ld);
    if (isnan(lb)) { nb = 1.f; lb = 0.f; }
    if (isnan(ld)) { nd = 1.f; ld = 0.f; }
  }
  const long slot = ((long)b * gridDim.x + blockIdx.x) * 4;
  block_sum_store(lb, part, slot + 0);
  block_sum_store(ld, part, slot + 1);
  block_sum_store(nb, part, slot + 2);
  block_sum_store(nd, part, slot + 3);
}

// gradient of the box + DFL terms into the 64 DFL logits of every anchor
template <typename T>
__global__ __launch_bounds__(256) void boxgrad_kernel(LossLevels L, int A, const unsigned char* fg,
                                                      const float* tbox, const float* tltrb, int iou_type,
                                                      const float* img_flags, float lam_box, float lam_dfl,
                                                      int B, const int* nfg) {
  const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (a >= A) return;
  int l;
  float ax, ay;
  const long row = anchor_row(L, b, a, l, ax, ay);
  if (!L.g[l]) return;
  T* gp = reinterpret_cast<T*>(L.g[l]) + row;
  float v[4 * DL_DFL];
  if (fg[(long)b * A + a]) {
    load_dist(reinterpret_cast<const T*>(L.x[l]) + row, v);
    const float n = (float)nfg[b];
    // no gradient from a term that was NaN for this image (the reference replaces it by 0)
    const float sb = img_flags[2 * b] != 0.f ? 0.f : lam_box / ((float)B * n);
    const float sd = img_flags[2 * b + 1] != 0.f ? 0.f : lam_dfl / ((float)B * 4.f * n);
    const float4 tb = reinterpret_cast<const float4*>(tbox)[(long)b * A + a];
    const float4 tl = reinterpret_cast<const float4*>(tltrb)[(long)b * A + a];
    float lb, ld;
    box_dfl<true>(v, ax, ay, L.stride[l], tb, tl, iou_type, sb, sd, lb, ld);
  } else {
#pragma unroll
    for (int i = 0; i < 4 * DL_DFL; ++i) v[i] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4 * DL_DFL / 8; ++k) {
    float t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = v[8 * k + i];
    Vec8<T>::store(gp + 8 * k, t);
  }
}

// per-image NaN flags from the box partials (needed before the gradient pass)
__global__ void flags_kernel(int B, int gx, const float* part, float* flags) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float nb = 0.f, nd = 0.f;
  for (int k = 0; k < gx; ++k) {
    nb += part[((long)b * gx + k) * 4 + 2];
    nd += part[((long)b * gx + k) * 4 + 3];
  }
  flags[2 * b] = nb;
  flags[2 * b + 1] = nd;
}

// per-image sums in fixed order (one thread per image), then thread 0 combines the images
__global__ __launch_bounds__(256) void finalize_kernel(int B, int A, int nc, int gxc, const float* pcls, int gxb,
                                                       const float* pbox, const int* nfg, float lam_box,
                                                       float lam_cls, float lam_dfl, double* img, float* out) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    const float* pc = pcls + (long)b * gxc;
    int k = 0;
    for (; k + 3 < gxc; k += 4) { s0 += pc[k]; s1 += pc[k + 1]; s2 += pc[k + 2]; s3 += pc[k + 3]; }
    for (; k < gxc; ++k) s0 += pc[k];
    const double mean = ((s0 + s1) + (s2 + s3)) / ((double)A * (double)nc);
    double cls = mean, box = 0.0, dfl = 0.0;
    if (nfg[b] > 0) {
      cls = 2.0 * mean;                                  // loss.py:530 + :551
      double sb = 0.0, sd = 0.0, fb = 0.0, fd = 0.0;
      for (int q = 0; q < gxb; ++q) {
        const float* p = pbox + ((long)b * gxb + q) * 4;
        sb += p[0]; sd += p[1]; fb += p[2]; fd += p[3];
      }
      if (fb == 0.0) box = sb / (double)nfg[b];
      if (fd == 0.0) dfl = sd / (4.0 * (double)nfg[b]);
    }
    img[3 * b] = cls;
    img[3 * b + 1] = box;
    img[3 * b + 2] = dfl;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double lcls = 0.0, lbox = 0.0, ldfl = 0.0;
  for (int b = 0; b < B; ++b) { lcls += img[3 * b]; lbox += img[3 * b + 1]; ldfl += img[3 * b + 2]; }
  lbox /= B; lcls /= B; ldfl /= B;
  out[0] = (float)(lam_box * lbox + lam_cls * lcls + lam_dfl * ldfl);
  out[1] = (float)lbox;
  out[2] = (float)lcls;
  out[3] = (float)ldfl;
}

// workspace layout (bytes, 256-aligned pieces)
struct LossWs {
  size_t pbox, kcnt, kidx, fg, tbox, tltrb, cbits, nfg, pcls, pboxp, flags, img, total;
};
static LossWs loss_ws(int B, int A, int nc, int M) {
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  const int nw = (nc + 31) / 32;
  const int gxc = cdiv((long)A * ((nc + 7) / 8), 256), gxb = cdiv(A, 256);
  LossWs w{};
  size_t o = 0;
  w.pbox = o; o += al((size_t)B * A * 16);
  w.kcnt = o; o += al((size_t)(M > 0 ? M : 1) * 4);
  w.kidx = o; o += al((size_t)(M > 0 ? M : 1) * DL_TOPK * 4);
  w.fg = o; o += al((size_t)B * A);
  w.tbox = o; o += al((size_t)B * A * 16);
  w.tltrb = o; o += al((size_t)B * A * 16);
  w.cbits = o; o += al((size_t)B * A * nw * 4);
  w.nfg = o; o += al((size_t)B * 4);
  w.pcls = o; o += al((size_t)B * gxc * 4);
  w.pboxp = o; o += al((size_t)B * gxb * 16);
  w.flags = o; o += al((size_t)B * 8);
  w.img = o; o += al((size_t)B * 24);
  w.total = o;
  return w;
}

// d(total)/d(maps) times the incoming loss gradient g (a device scalar), in place.  The fused loss
// writes its map gradients in the forward, before g exists; in the training loop g is the 1.0 seed
// of loss.backward(), so every block reads g and leaves at once -- one short launch instead of an
// elementwise pass over the 155 MB of head gradients (configs[2]).  Otherwise v = T(float(v) *
// float(T(g))): torch's `grad * g.to(grad.dtype)`.
struct ScaleBufs {
  void* p[4];
  long n[4];
};

template <typename T>
__global__ __launch_bounds__(256) void scale_by_dev_kernel(ScaleBufs b, const float* g) {
  const float gv = *g;
  if (gv == 1.0f) return;
  const float s = to_f(from_f<T>(gv));
  T* p = (T*)b.p[blockIdx.y];
  const long n = b.n[blockIdx.y];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = from_f<T>(to_f(p[i]) * s);
}

}  // namespace yms

using namespace yms;

extern "C" {

size_t yms_det_loss_ws_bytes(int batch, int anchors, int nc, int n_targets) {
  if (batch <= 0 || anchors <= 0 || nc <= 0 || n_targets < 0) return 0;
  return loss_ws(batch, anchors, nc, n_targets).total;
}

yms_status yms_det_loss(int dtype, int batch, int nc, int nlevels, const void* const* maps, void* const* grads,
                        const int* hs, const int* ws_, const float* strides, int ld, const float* targets,
                        int n_targets, float img_w, float img_h, int iou_type, const float* pos_weight,
                        const float* lambdas, void* ws, size_t ws_bytes, float* out, void* stream) {
  if (batch <= 0 || nc <= 0 || nlevels <= 0 || nlevels > DL_MAXL || !maps || !hs || !ws_ || !strides || !out ||
      !lambdas || n_targets < 0 || (n_targets > 0 && !targets) || iou_type < 0 || iou_type > 3)
    return YMS_ERR_INVALID;
  if (ld < 4 * DL_DFL + nc || ld % 8) return YMS_ERR_INVALID;
  long a_total = 0;
  for (int l = 0; l < nlevels; ++l) a_total += (long)hs[l] * ws_[l];
  if (a_total * ((nc + 7) / 8) >= (1l << 31) - 256) return YMS_ERR_UNSUPPORTED;
  LossLevels L{};
  L.nl = nlevels;
  L.ld = ld;
  int A = 0;
  for (int l = 0; l < nlevels; ++l) {
    if (!maps[l] || hs[l] <= 0 || ws_[l] <= 0) return YMS_ERR_INVALID;
    L.x[l] = maps[l];
    L.g[l] = grads ? grads[l] : nullptr;
    L.h[l] = hs[l];
    L.w[l] = ws_[l];
    L.stride[l] = strides[l];
    L.off[l] = A;
    A += hs[l] * ws_[l];
  }
  L.off[nlevels] = A;
  const LossWs w = loss_ws(batch, A, nc, n_targets);
  if (!ws || ws_bytes < w.total) return YMS_ERR_INVALID;
  char* base = (char*)ws;
  float* pbox = (float*)(base + w.pbox);
  int* kcnt = (int*)(base + w.kcnt);
  int* kidx = (int*)(base + w.kidx);
  unsigned char* fg = (unsigned char*)(base + w.fg);
  float* tbox = (float*)(base + w.tbox);
  float* tltrb = (float*)(base + w.tltrb);
  unsigned* cbits = (unsigned*)(base + w.cbits);
  int* nfg = (int*)(base + w.nfg);
  float* pcls = (float*)(base + w.pcls);
  float* pboxp = (float*)(base + w.pboxp);
  float* flags = (float*)(base + w.flags);
  double* img = (double*)(base + w.img);
  const int nw = (nc + 31) / 32;
  const int gxc = cdiv((long)A * ((nc + 7) / 8), 256), gxb = cdiv(A, 256);
  hipStream_t st = (hipStream_t)stream;
  const float gscale = lambdas[1] / ((float)batch * (float)A * (float)nc);
#define YMS_LOSS_CASE(T)                                                                                        \
  hipLaunchKernelGGL(decode_kernel<T>, dim3(gxb, batch), dim3(256), 0, st, L, A, pbox);                        \
  if (n_targets > 0)                                                                                           \
    hipLaunchKernelGGL(topk_kernel, dim3(n_targets), dim3(256), 0, st, targets, batch, A, img_w, img_h, pbox,  \
                       kcnt, kidx);                                                                            \
  hipLaunchKernelGGL(assign_kernel, dim3(batch), dim3(256), 0, st, targets, n_targets, A, nc, nw, img_w, img_h, \
                     L, kcnt, kidx, fg, tbox, tltrb, cbits, nfg);                                              \
  hipLaunchKernelGGL(cls_kernel<T>, dim3(gxc, batch), dim3(256), 0, st, L, A, nc, nw, cbits, nfg, pos_weight,  \
                     gscale, pcls);                                                                            \
  hipLaunchKernelGGL(box_kernel<T>, dim3(gxb, batch), dim3(256), 0, st, L, A, fg, tbox, tltrb, iou_type,        \
                     pboxp);                                                                                   \
  hipLaunchKernelGGL(flags_kernel, dim3(cdiv(batch, 64)), dim3(64), 0, st, batch, gxb, pboxp, flags);           \
  if (grads)                                                                                                   \
    hipLaunchKernelGGL(boxgrad_kernel<T>, dim3(gxb, batch), dim3(256), 0, st, L, A, fg, tbox, tltrb, iou_type,  \
                       flags, lambdas[0], lambdas[2], batch, nfg);                                             \
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, st, batch, A, nc, gxc, pcls, gxb, pboxp, nfg,      \
                     lambdas[0], lambdas[1], lambdas[2], img, out);
  switch (dtype) {
    case YMS_F32: { YMS_LOSS_CASE(float) break; }
    case YMS_BF16: { YMS_LOSS_CASE(bf16) break; }
    case YMS_F16: { YMS_LOSS_CASE(f16) break; }
    default: return YMS_ERR_INVALID;
  }
#undef YMS_LOSS_CASE
  return launch_status();
}

yms_status yms_scale_by_device_scalar(int dtype, int nbuf, void* const* bufs, const long* counts, const float* g,
                                      void* stream) {
  if (nbuf < 1 || nbuf > 4 || !bufs || !counts || !g) return YMS_ERR_INVALID;
  ScaleBufs b{};
  long mx = 0;
  for (int i = 0; i < nbuf; ++i) {
    if (!bufs[i] || counts[i] < 0) return YMS_ERR_INVALID;
    b.p[i] = bufs[i];
    b.n[i] = counts[i];
    mx = std::max(mx, counts[i]);
  }
  const dim3 grid((unsigned)std::max<long>(1, std::min<long>(1024, cdiv(mx, 256))), (unsigned)nbuf);
  switch (dtype) {
    case YMS_F32: hipLaunchKernelGGL(scale_by_dev_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, b, g); break;
    case YMS_BF16: hipLaunchKernelGGL(scale_by_dev_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, b, g); break;
    case YMS_F16: hipLaunchKernelGGL(scale_by_dev_kernel<f16>, grid, dim3(256), 0, (hipStream_t)stream, b, g); break;
    default: return YMS_ERR_INVALID;
  }
  return launch_status();
}

}  // extern "C"

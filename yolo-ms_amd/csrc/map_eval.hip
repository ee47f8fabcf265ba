// mAP@0.5 evaluation: GPU per-image detection <-> ground-truth matching and the
// host-side per-class precision/recall accumulation, replacing the reference's
// torchmetrics.MeanAveragePrecision(iou_thresholds=[0.5]) call in validate_epoch
// (yolov8/tools/train.py:41-47, 146, 152-153).  The semantics are the published COCOeval
// algorithm at that setting (oracle/map_ref.py restates it; torchmetrics / pycocotools are not
// installed here, so parity is against that restatement):
//   per (image, class): detections stably sorted by score (descending), the first 100 kept;
//   greedy matching in that order at IoU >= 0.5 (double precision, xywh areas, no +1), each
//   detection taking the unmatched ground truth of highest IoU (ties -> the later one);
//   per class: kept detections ordered by (score desc, image, input index), tp/fp cumsums,
//   precision made monotone, 101-point interpolation; mAP = mean over classes with ground truth.
#include <algorithm>
#include <cmath>
#include <vector>

#include "yms_common.hpp"

namespace yms {

constexpr int MAP_MAXDET = 100;
constexpr int MAP_MAX_GT = 2048;      // ground truths per image (LDS)

// one wave per image
__global__ __launch_bounds__(64) void map_match_kernel(const float* dbox, const float* dscore, const int* dlabel,
                                                       const int* doff, const float* gbox, const int* glabel,
                                                       const int* goff, uint8_t* tp, uint8_t* kept, int* rank_out) {
  __shared__ double gb[MAP_MAX_GT][4];
  __shared__ int gl[MAP_MAX_GT];
  __shared__ uint8_t gm[MAP_MAX_GT];
  const int img = blockIdx.x, lane = threadIdx.x;
  const int d0 = doff[img], nd = doff[img + 1] - d0;
  const int g0 = goff[img], ng = goff[img + 1] - g0;
  for (int j = lane; j < ng; j += 64) {
    const float* q = gbox + (long)(g0 + j) * 4;
    gb[j][0] = (double)q[0];
    gb[j][1] = (double)q[1];
    gb[j][2] = (double)(q[2] - q[0]);     // width / height in fp32, as box_convert
    gb[j][3] = (double)(q[3] - q[1]);
    gl[j] = glabel[g0 + j];
    gm[j] = 0;
  }
  // rank of every detection within its class: stable descending score order
  for (int d = lane; d < nd; d += 64) {
    const int lab = dlabel[d0 + d];
    const float sc = dscore[d0 + d];
    int r = 0;
    for (int j = 0; j < nd; ++j) {
      if (dlabel[d0 + j] != lab) continue;
      const float sj = dscore[d0 + j];
      r += (sj > sc || (sj == sc && j < d)) ? 1 : 0;
    }
    rank_out[d0 + d] = r;
    kept[d0 + d] = r < MAP_MAXDET ? 1 : 0;
    tp[d0 + d] = 0;
  }
  __syncthreads();
  // greedy matching per ground-truth class, detections in rank order
  for (int gi = 0; gi < ng; ++gi) {
    const int c = gl[gi];
    bool first = true;                     // process each class once: at its first ground truth
    for (int j = 0; j < gi; ++j)
      if (gl[j] == c) { first = false; break; }
    if (!first) continue;
    for (int r = 0; r < MAP_MAXDET; ++r) {
      // the class-c detection of rank r (at most one)
      int found = -1;
      for (int d = lane; d < nd; d += 64)
        if (dlabel[d0 + d] == c && rank_out[d0 + d] == r) found = d;
      unsigned long long any = __ballot(found >= 0);
      if (!any) break;                    // fewer than r + 1 detections of this class
      const int src = __ffsll((long long)any) - 1;
      const int d = __shfl(found, src);
      // xyxy -> xywh in fp32 (torchvision box_convert on the fp32 tensors), IoU in double
      const float* bp = dbox + (long)(d0 + d) * 4;
      const double b[2] = {(double)bp[0], (double)bp[1]};
      const double bw = (double)(bp[2] - bp[0]), bh = (double)(bp[3] - bp[1]);
      // best unmatched ground truth: max IoU >= 0.5, the later index on ties
      double best = -1.0;
      int bj = -1;
      for (int j = lane; j < ng; j += 64) {
        if (gl[j] != c || gm[j]) continue;
        const double gw = gb[j][2], gh = gb[j][3];
        const double w = fmin(b[0] + bw, gb[j][0] + gw) - fmax(b[0], gb[j][0]);
        const double h = fmin(b[1] + bh, gb[j][1] + gh) - fmax(b[1], gb[j][1]);
        double iou = 0.0;
        if (w > 0.0 && h > 0.0) {
          const double inter = w * h;
          iou = inter / (bw * bh + gw * gh - inter);
        }
        if (iou >= fmin(0.5, 1.0 - 1e-10) && (iou > best || (iou == best && j > bj))) {
          best = iou;
          bj = j;
        }
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
        const double ob = __shfl_xor(best, m);
        const int oj = __shfl_xor(bj, m);
        if (ob > best || (ob == best && oj > bj)) {
          best = ob;
          bj = oj;
        }
      }
      if (bj >= 0) {
        if (lane == 0) {
          gm[bj] = 1;
          tp[d0 + d] = 1;
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace yms

using namespace yms;

// numpy's pairwise summation (np.mean / np.sum over float64 arrays), so the host AP matches the
// COCOeval restatement bit for bit
static double np_pairwise_sum(const double* a, long n) {
  if (n < 8) {
    double r = 0.0;
    for (long i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    long i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  long n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_sum(a, n2) + np_pairwise_sum(a + n2, n - n2);
}

extern "C" {

yms_status yms_map_match(int n_images, const float* det_boxes, const float* det_scores, const int* det_labels,
                         const int* det_off, const float* gt_boxes, const int* gt_labels, const int* gt_off,
                         uint8_t* tp, uint8_t* kept, int* rank_ws, int max_gt_per_image, void* stream) {
  if (n_images <= 0) return YMS_OK;
  if (!det_off || !gt_off || !tp || !kept || !rank_ws) return YMS_ERR_INVALID;
  if (max_gt_per_image > MAP_MAX_GT) return YMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(map_match_kernel, dim3((unsigned)n_images), dim3(64), 0, (hipStream_t)stream, det_boxes,
                     det_scores, det_labels, det_off, gt_boxes, gt_labels, gt_off, tp, kept, rank_ws);
  return launch_status();
}

// host: per-class precision / recall over the whole evaluation set (COCOeval.accumulate at one
// IoU threshold, area 'all', maxDets 100).  Inputs are host arrays in evaluation order.
yms_status yms_map_accumulate(int n_det, const float* scores, const int* labels, const int* image,
                              const uint8_t* tp, const uint8_t* kept, int n_classes, const int* n_gt,
                              double* ap, double* map) {
  if (n_det < 0 || n_classes <= 0 || !n_gt || !ap || !map) return YMS_ERR_INVALID;
  if (n_det > 0 && (!scores || !labels || !image || !tp || !kept)) return YMS_ERR_INVALID;
  std::vector<std::vector<int>> by(n_classes);
  for (int i = 0; i < n_det; ++i)
    if (kept[i] && labels[i] >= 0 && labels[i] < n_classes) by[labels[i]].push_back(i);
  const double eps = std::nextafter(1.0, 2.0) - 1.0;   // np.spacing(1)
  std::vector<double> aps;
  for (int c = 0; c < n_classes; ++c) {
    ap[c] = -1.0;
    if (n_gt[c] <= 0) continue;
    std::vector<int>& v = by[c];
    std::stable_sort(v.begin(), v.end(), [&](int a, int b) {
      if (scores[a] != scores[b]) return scores[a] > scores[b];
      if (image[a] != image[b]) return image[a] < image[b];
      return a < b;
    });
    const int nd = (int)v.size();
    std::vector<double> rc(nd), pr(nd);
    double tps = 0.0, fps = 0.0;
    for (int k = 0; k < nd; ++k) {
      if (tp[v[k]]) tps += 1.0; else fps += 1.0;
      rc[k] = tps / (double)n_gt[c];
      pr[k] = tps / (fps + tps + eps);
    }
    for (int k = nd - 1; k > 0; --k)
      if (pr[k] > pr[k - 1]) pr[k - 1] = pr[k];
    double q[101];
    for (int t = 0; t <= 100; ++t) {
      const double thr = (double)t * 0.01;      // np.linspace(0, 1, 101) = arange(101) * 0.01
      const int pi = (int)(std::lower_bound(rc.begin(), rc.end(), thr) - rc.begin());
      q[t] = pi < nd ? pr[pi] : 0.0;
    }
    ap[c] = np_pairwise_sum(q, 101) / 101.0;
    aps.push_back(ap[c]);
  }
  *map = aps.empty() ? -1.0 : np_pairwise_sum(aps.data(), (long)aps.size()) / (double)aps.size();
  return YMS_OK;
}

}  // extern "C"

/* CPU restatement of the reference's post-process + class-wise NMS.
 * TEST INFRASTRUCTURE ONLY (parity oracle / CPU baseline) -- never linked into the product.
 *
 * Reference call sites (paths relative to /root/reference):
 *   yolov8/tools/train.py:63-113   validate_epoch post-process + per-class torchvision.ops.nms
 *   yolov8/tools/test.py:166-218   identical block in the inference CLI
 *
 * The NMS arithmetic itself lives in third-party torchvision (requirements.txt:2,
 * "torchvision>=0.15.0", unpinned), which is absent from /root/reference and from this
 * image.  Its published CPU algorithm (torchvision/csrc/ops/cpu/nms_kernel.cpp) is
 * restated here:
 *   order  = scores.sort(stable=true, descending=true)
 *   area_i = (x2-x1)*(y2-y1)                      (fp32, no +1)
 *   greedily keep i; suppress j if inter/(area_i+area_j-inter) > iou_threshold,
 *   inter = max(0,xx2-xx1)*max(0,yy2-yy1), the fp32 ratio promoted to double for the
 *   compare (iou_threshold is a double in the CPU kernel).
 *   max / min are std::max / std::min, restated literally: std::max(a, b) = (a < b) ? b : a,
 *   std::min(a, b) = (b < a) ? b : a -- on a NaN operand they return the FIRST argument, where
 *   C's fmaxf / fminf (and the GPU's v_max_f32 / v_min_f32) return the non-NaN one.  The
 *   suppression decisions cannot differ: a NaN coordinate of box i (j) makes area_i (area_j)
 *   NaN, so the ratio is NaN under either semantics and NaN > iou is false
 *   (tests/test_nms_gpu.py's NaN-coordinate case checks the GPU against this literal form).
 * PARITY UNPINNED for NMS: no reference test or fixture pins NMS output; the oracle is
 * checked by known-answer tests (tests/test_nms_oracle.py).
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off -fPIC -shared)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float s; int64_t i; } sk_t;

static inline float std_max(float a, float b) { return (a < b) ? b : a; }
static inline float std_min(float a, float b) { return (b < a) ? b : a; }

static int cmp_desc_stable(const void* a, const void* b) {
  const sk_t* x = (const sk_t*)a;
  const sk_t* y = (const sk_t*)b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return (x->i < y->i) ? -1 : (x->i > y->i);   /* ties: original order (stable) */
}

/* torchvision::ops::nms(boxes[n,4] xyxy, scores[n], iou) -> keep (indices into 0..n-1) */
int64_t yms_ref_nms(const float* boxes, const float* scores, int64_t n, double iou_thr,
                    int64_t* keep) {
  if (n <= 0) return 0;
  sk_t* order = (sk_t*)malloc(sizeof(sk_t) * (size_t)n);
  float* areas = (float*)malloc(sizeof(float) * (size_t)n);
  unsigned char* sup = (unsigned char*)calloc((size_t)n, 1);
  for (int64_t i = 0; i < n; ++i) {
    order[i].s = scores[i];
    order[i].i = i;
    const float* b = boxes + 4 * i;
    areas[i] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  qsort(order, (size_t)n, sizeof(sk_t), cmp_desc_stable);
  int64_t nk = 0;
  for (int64_t _i = 0; _i < n; ++_i) {
    int64_t i = order[_i].i;
    if (sup[i]) continue;
    keep[nk++] = i;
    const float ix1 = boxes[4 * i], iy1 = boxes[4 * i + 1], ix2 = boxes[4 * i + 2], iy2 = boxes[4 * i + 3];
    const float iarea = areas[i];
    for (int64_t _j = _i + 1; _j < n; ++_j) {
      int64_t j = order[_j].i;
      if (sup[j]) continue;
      const float xx1 = std_max(ix1, boxes[4 * j]);
      const float yy1 = std_max(iy1, boxes[4 * j + 1]);
      const float xx2 = std_min(ix2, boxes[4 * j + 2]);
      const float yy2 = std_min(iy2, boxes[4 * j + 3]);
      const float w = std_max(0.0f, xx2 - xx1);
      const float h = std_max(0.0f, yy2 - yy1);
      const float inter = w * h;
      const float ovr = inter / (iarea + areas[j] - inter);
      if ((double)ovr > iou_thr) sup[j] = 1;
    }
  }
  free(order);
  free(areas);
  free(sup);
  return nk;
}

/* Post-process of ONE image (train.py:63-101):
 *   pred [A, 4+nc] = (cx, cy, w, h, p_0..p_{nc-1})
 *   xyxy = (cx - w/2, cy - h/2, cx + w/2, cy + h/2)
 *   score, label = max / first-argmax over classes
 *   keep score > conf, then NMS per label ascending, segments concatenated.
 * Outputs: keep_idx = anchor indices, keep_lbl = labels; returns the count.
 * boxes_out (optional, [A,4]) receives the xyxy boxes of every anchor. */
int64_t yms_ref_postprocess(const float* pred, int64_t A, int nc, float conf, double iou_thr,
                            int64_t* keep_idx, int32_t* keep_lbl, float* boxes_out) {
  const int no = 4 + nc;
  float* boxes = (float*)malloc(sizeof(float) * 4 * (size_t)(A > 0 ? A : 1));
  float* score = (float*)malloc(sizeof(float) * (size_t)(A > 0 ? A : 1));
  int32_t* label = (int32_t*)malloc(sizeof(int32_t) * (size_t)(A > 0 ? A : 1));
  int64_t* counts = (int64_t*)calloc((size_t)nc + 1, sizeof(int64_t));
  for (int64_t a = 0; a < A; ++a) {
    const float* p = pred + a * no;
    const float cx = p[0], cy = p[1], w = p[2], h = p[3];
    boxes[4 * a + 0] = cx - w / 2;
    boxes[4 * a + 1] = cy - h / 2;
    boxes[4 * a + 2] = cx + w / 2;
    boxes[4 * a + 3] = cy + h / 2;
    float best = p[4];
    int bl = 0;
    for (int c = 1; c < nc; ++c) {
      if (p[4 + c] > best) { best = p[4 + c]; bl = c; }
    }
    score[a] = best;
    label[a] = (best > conf) ? bl : -1;
    if (label[a] >= 0) counts[bl]++;
  }
  if (boxes_out) memcpy(boxes_out, boxes, sizeof(float) * 4 * (size_t)A);
  int64_t total = 0;
  int64_t maxc = 0;
  for (int c = 0; c < nc; ++c) if (counts[c] > maxc) maxc = counts[c];
  float* cb = (float*)malloc(sizeof(float) * 4 * (size_t)(maxc > 0 ? maxc : 1));
  float* cs = (float*)malloc(sizeof(float) * (size_t)(maxc > 0 ? maxc : 1));
  int64_t* ci = (int64_t*)malloc(sizeof(int64_t) * (size_t)(maxc > 0 ? maxc : 1));
  int64_t* kk = (int64_t*)malloc(sizeof(int64_t) * (size_t)(maxc > 0 ? maxc : 1));
  for (int c = 0; c < nc; ++c) {
    if (!counts[c]) continue;
    int64_t m = 0;
    for (int64_t a = 0; a < A; ++a) {
      if (label[a] != c) continue;
      memcpy(cb + 4 * m, boxes + 4 * a, sizeof(float) * 4);
      cs[m] = score[a];
      ci[m] = a;
      ++m;
    }
    int64_t nk = yms_ref_nms(cb, cs, m, iou_thr, kk);
    for (int64_t t = 0; t < nk; ++t) {
      keep_idx[total] = ci[kk[t]];
      keep_lbl[total] = c;
      ++total;
    }
  }
  free(cb); free(cs); free(ci); free(kk);
  free(boxes); free(score); free(label); free(counts);
  return total;
}

// BatchNorm / SiLU / residual, SPPF pooling, nearest-x2 upsample and layout kernels for the
// YOLOv8 hot path on gfx950.  All are HBM-bound streaming kernels: 16-B vectorised NHWC
// accesses (8 channels per item), grid-stride loops, fp32 math, deterministic reductions
// (per-block partial rows reduced in a fixed order, fp64 final sums).
//
// Reference semantics (paths relative to rafaelghiorzi/YOLO-MS):
//   nn.BatchNorm2d(eps=1e-3, momentum=0.03) + nn.SiLU   yolov8/model/components.py:72-77
//   Bottleneck residual (always on)                     yolov8/model/components.py:87-93
//   SPPF: three chained MaxPool2d(5, 1, 2) + cat        yolov8/model/components.py:136-146
//   Upsample nearest x2                                 yolov8/model/components.py:159-160
#include <cstdlib>
#include <algorithm>

#include "yms_common.hpp"

namespace yms {

static inline unsigned grid_for(long items, int block = 256, long cap = 16384) {
  long g = (items + block - 1) / block;
  if (g < 1) g = 1;
  return (unsigned)std::min(g, cap);
}

// ------------------------------------------------------------------------------------------
// BN fold (eval) and finalize (train)
// ------------------------------------------------------------------------------------------
__global__ void bn_fold_kernel(int c, const float* g, const float* b, const float* rm,
                               const float* rv, float eps, float* scale, float* shift) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  if (!g) {  // bias-only (plain nn.Conv2d)
    scale[i] = 1.0f;
    shift[i] = b ? b[i] : 0.0f;
    return;
  }
  const float sc = g[i] / sqrtf(rv[i] + eps);
  scale[i] = sc;
  shift[i] = b[i] - rm[i] * sc;
}

// Statistics rows (conv_common.hpp contract): row r = (sum z, sum (z - mean_r)^2) over n_r
// pixels, n_r = counts[r] (the producers write the count table right after the rows; rows with
// n_r = 0 are skipped).  Rows are merged in ONE pass in fp64 with the shifted-data form of
// Chan's update: with K = the first row's mean (a sample of the data, so |mean - K| is of the
// order of the spread),  M2 = sum_r [M2_r + n_r (m_r - K)^2] - (sum_r n_r (m_r - K))^2 / N,
// free of the sum z^2 - n mean^2 cancellation.  Row means m_r are formed in fp32 (the
// producers' own precision).
struct Moments {           // n, sum n_r (m_r - K), sum [M2_r + n_r (m_r - K)^2] about the shift K
  double n = 0.0, d1 = 0.0, d2 = 0.0, K = 0.0;
  __device__ void add_row(float s1, float m2, float nr) {
    if (!(nr > 0.f)) return;
    const float mr = s1 / nr;
    if (n == 0.0) K = (double)mr;
    const double d = (double)mr - K;
    n += nr;
    d1 += nr * d;
    d2 += (double)m2 + nr * d * d;
  }
  __device__ void merge(const Moments& o) {      // re-centre o on this K, then add
    if (o.n == 0.0) return;
    if (n == 0.0) { *this = o; return; }
    const double e = o.K - K;
    n += o.n;
    d1 += o.d1 + o.n * e;
    d2 += o.d2 + 2.0 * e * o.d1 + o.n * e * e;
  }
  __device__ double sum() const { return d1 + n * K; }
  __device__ double m2() const { return n > 0.0 ? d2 - d1 * d1 / n : 0.0; }
  __device__ void store(double (*red)[4], int i) const { red[i][0] = n; red[i][1] = d1; red[i][2] = d2; red[i][3] = K; }
  __device__ static Moments load(const double (*red)[4], int i) {
    Moments m;
    m.n = red[i][0]; m.d1 = red[i][1]; m.d2 = red[i][2]; m.K = red[i][3];
    return m;
  }
};

// Pre-reduction for long statistics tables: block (cb, s) merges rows [s*R, (s+1)*R) of
// channels [64cb, 64cb+64) and stores the merged (sum, M2) over row s*R -- the first row of its
// own range, so no block reads a row another block writes (the count table is left as it is:
// the finalize sums the counts of each merged range).  256 threads = 64 channels x 4 lanes, two
// rows in flight per lane.
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(int c, float* stats, int rows, int ld, int R) {
  __shared__ double red[4 * 64][4];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * R, r1 = min(rows, r0 + R);
  const float* cnt = stats + (long)rows * 2 * ld;
  const float* s1p = stats + ch;
  const float* m2p = stats + ld + ch;
  const long rs = 2l * ld;
  Moments a, b;
  if (ch < c) {
    int r = r0 + ty;
    for (; r + 4 < r1; r += 8) {
      a.add_row(s1p[r * rs], m2p[r * rs], cnt[r]);
      b.add_row(s1p[(r + 4) * rs], m2p[(r + 4) * rs], cnt[r + 4]);
    }
    if (r < r1) a.add_row(s1p[r * rs], m2p[r * rs], cnt[r]);
    a.merge(b);
  }
  a.store(red, ty * 64 + tx);
  __syncthreads();
  if (ty == 0 && ch < c) {
    Moments t = Moments::load(red, tx);
    for (int k = 1; k < 4; ++k) t.merge(Moments::load(red, k * 64 + tx));
    stats[(long)r0 * rs + ch] = (float)t.sum();
    stats[(long)r0 * rs + ld + ch] = (float)t.m2();
  }
}

// rows are read at stride rs (rs > 1 after bn_stats_partial_kernel; merged row k covers original
// rows [k*rs, min(rows_total, (k+1)*rs)), its count the sum of theirs); FIN_CW channels x FIN_RL
// row lanes per block (1024 threads: short tables are latency-bound, so many lanes with few
// rows each), one shifted pass per lane, fixed-order tree combine
constexpr int FIN_CW = 8, FIN_RL = 1024 / FIN_CW;
__global__ __launch_bounds__(1024) void bn_finalize_kernel(int c, const float* stats, int rows, int ld, int rs,
                                                           int rows_total, long count, const float* g,
                                                           const float* b, float* rm, float* rv, float momentum,
                                                           float eps, float* mi, int mi_ld, float* scale,
                                                           float* shift) {
  __shared__ double red[FIN_RL * (FIN_CW + 1)][4];
  const int tx = threadIdx.x % FIN_CW, ty = threadIdx.x / FIN_CW;
  const int ch = blockIdx.x * FIN_CW + tx;
  const float* cnt = stats + (long)rows_total * 2 * ld;
  Moments a;
  if (ch < c) {
    if (rs == 1) {
      // four rows per iteration, every load issued before the first use
      int r = ty;
      for (; r + 3 * FIN_RL < rows; r += 4 * FIN_RL) {
        float s1[4], m2[4], n[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s1[u] = stats[(long)(r + FIN_RL * u) * 2 * ld + ch];
          m2[u] = stats[(long)(r + FIN_RL * u) * 2 * ld + ld + ch];
          n[u] = cnt[r + FIN_RL * u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) a.add_row(s1[u], m2[u], n[u]);
      }
      for (; r < rows; r += FIN_RL) a.add_row(stats[(long)r * 2 * ld + ch], stats[(long)r * 2 * ld + ld + ch], cnt[r]);
    } else {
      for (int r = ty; r < rows; r += FIN_RL) {
        float n = 0.f;   // integer-valued: exact in fp32 below 2^24 pixels per merged row
        for (int q = r * rs, e = min(rows_total, (r + 1) * rs); q < e; ++q) n += cnt[q];
        a.add_row(stats[(long)r * rs * 2 * ld + ch], stats[(long)r * rs * 2 * ld + ld + ch], n);
      }
    }
  }
  // fixed-order tree over the row lanes: lane ty absorbs lane ty + h
  for (int h = FIN_RL / 2; h >= 1; h >>= 1) {
    if (ty >= h && ty < 2 * h) a.store(red, ty * (FIN_CW + 1) + tx);
    __syncthreads();
    if (ty < h) a.merge(Moments::load(red, (ty + h) * (FIN_CW + 1) + tx));
    __syncthreads();
  }
  if (ty == 0 && ch < c) {
    const double mean = a.n > 0.0 ? a.sum() / a.n : 0.0;
    const double var = fmax(a.m2(), 0.0) / (double)count;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const double uvar = count > 1 ? var * (double)count / (double)(count - 1) : var;
    if (rm) rm[ch] = (float)((1.0 - momentum) * (double)rm[ch] + momentum * mean);
    if (rv) rv[ch] = (float)((1.0 - momentum) * (double)rv[ch] + momentum * uvar);
    mi[ch] = (float)mean;
    mi[mi_ld + ch] = invstd;
    const float sc = g[ch] * invstd;
    scale[ch] = sc;
    shift[ch] = b[ch] - (float)mean * sc;
  }
}

// Forward finalize for tables of <= 1024 rows (rs == 1), latency-shaped: 8 channels x 32 row
// lanes (256 threads), each lane issues the loads of up to 8 rows at a time (24 in flight) and
// folds them with the same shifted fp64 update; a 5-level fixed-order tree over the lanes (the
// 1024-thread kernel above runs a 7-level tree with two barriers per level).  In the forward no
// side-stream work competes for CU slots, so the finalize's latency is the step's.  Measured
// step-neutral to slightly faster (YOLOv8-s 18.71 / 18.71 -> 18.67 / 18.74 ms, YOLO-MS-S 37.29 /
// 37.37 -> 37.24 / 37.26 ms, profiles/r03u_bn_finalize_small_ab.txt).
constexpr int FIN3_RL = 32;
__global__ __launch_bounds__(256) void bn_finalize_small_kernel(int c, const float* stats, int rows, int ld,
                                                                long count, const float* g, const float* b, float* rm,
                                                                float* rv, float momentum, float eps, float* mi,
                                                                int mi_ld, float* scale, float* shift) {
  __shared__ double red[FIN3_RL * 9][4];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int ch = blockIdx.x * 8 + tx;
  const float* cnt = stats + (long)rows * 2 * ld;
  Moments a;
  if (ch < c) {
    for (int r0 = ty; r0 < rows; r0 += FIN3_RL * 8) {
      float s1[8], m2[8], n[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + FIN3_RL * u;
        const bool ok = r < rows;
        s1[u] = ok ? stats[(long)r * 2 * ld + ch] : 0.f;
        m2[u] = ok ? stats[(long)r * 2 * ld + ld + ch] : 0.f;
        n[u] = ok ? cnt[r] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a.add_row(s1[u], m2[u], n[u]);
    }
  }
  for (int h = FIN3_RL / 2; h >= 1; h >>= 1) {
    if (ty >= h && ty < 2 * h) a.store(red, ty * 9 + tx);
    __syncthreads();
    if (ty < h) a.merge(Moments::load(red, (ty + h) * 9 + tx));
    __syncthreads();
  }
  if (ty == 0 && ch < c) {
    const double mean = a.n > 0.0 ? a.sum() / a.n : 0.0;
    const double var = fmax(a.m2(), 0.0) / (double)count;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const double uvar = count > 1 ? var * (double)count / (double)(count - 1) : var;
    if (rm) rm[ch] = (float)((1.0 - momentum) * (double)rm[ch] + momentum * mean);
    if (rv) rv[ch] = (float)((1.0 - momentum) * (double)rv[ch] + momentum * uvar);
    mi[ch] = (float)mean;
    mi[mi_ld + ch] = invstd;
    const float sc = g[ch] * invstd;
    scale[ch] = sc;
    shift[ch] = b[ch] - (float)mean * sc;
  }
}

// ------------------------------------------------------------------------------------------
// Channel-stationary mapping for the per-channel elementwise / reduction kernels:
// G = ceil(C/8) 16-B channel groups, thread (py, g) = (tid / G, tid % G) keeps the same
// 8 channels (and their BN parameters, in registers) for every pixel it visits; the
// PY = 256 / G pixel lanes of a block walk a contiguous pixel range.  One wave-row of a
// pixel is a fully coalesced 16*G-byte segment.  Requires G <= 256 (C <= 2048).
// ------------------------------------------------------------------------------------------
struct ChanMap {
  int G, PY, g, py;
  bool active;
  __device__ ChanMap(int c) {
    G = (c + 7) >> 3;
    PY = 256 / G;
    g = threadIdx.x % G;
    py = threadIdx.x / G;
    active = py < PY;
  }
};

__device__ __forceinline__ void load_params8(const float* p, int c0, int c, float (&v)[8], float dflt) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (p && c0 + i < c) ? p[c0 + i] : dflt;
}

// U pixels per thread per iteration: all U loads issue before any use (memory-level
// parallelism; these kernels are HBM-bound).
constexpr int BN_U = 4;
// the backward reduce / apply passes (8 measured slower: the YOLOv8-s step went 17.80 -> 17.90 ms
// (reduce) and -> 19.43 ms (apply), profiles/r05u_bn_unroll_ab.txt)
constexpr int BN_UR = 4, BN_UA = 4;

// Pixel-range order of the elementwise passes over a tensor: blocks are dispatched in index order,
// so block b taking range nblocks - 1 - b walks the tensor from its end.  A pass that follows one
// which walked the same tensor forward then reads the most recently touched bytes first -- the
// ones still held by the 256 MB memory-side cache -- instead of the ones it evicted first.
// Interleaved A/B (YOLOv8-s B=64 step, 3 reps, profiles/r05r_bn_order_ab.txt): the forward affine
// pass reversed (after the conv that wrote z) 18.22 -> 18.17 ms; also reversing the backward
// reduce or apply gave no more.
constexpr bool BN_REV_AFFINE = true, BN_REV_RED = false, BN_REV_APPLY = false;
// Non-temporal loads where a pass reads a tensor for the last time while the weight gradients run
// beside it (the backward apply's gy and z, the forward affine's z; the reduce's reads stay cached:
// the apply re-reads the same bytes next).  Interleaved A/B (profiles/r06s_bn_nt_ab.txt): YOLOv8-s
// 17.72 -> 17.64 ms/step, YOLO-MS-S 35.56 -> 35.38 ms (each alone gives part of it).
template <bool REV> __device__ __forceinline__ long block_range() {
  return REV ? (long)(gridDim.x - 1 - blockIdx.x) : (long)blockIdx.x;
}

// PIPE (the default): software-pipelined (c % 8 == 0) like the backward passes: the next U pixels' loads
// (clamped to the block's last pixel, masked) are in flight while this U is computed and stored.
template <typename T, bool PIPE = false>
__global__ __launch_bounds__(256) void affine_act_kernel(long npix, int c, const T* z, int z_ld, int z_off,
                                                         const float* scale, const float* shift, int act,
                                                         const T* res, int res_ld, int res_off, T* y,
                                                         int y_ld, int y_off, long ppb) {
  ChanMap m(c);
  if (!m.active) return;
  const int c0 = m.g * 8, nv = min(8, c - c0);
  float sc[8], sh[8];
  load_params8(scale, c0, c, sc, 1.0f);
  load_params8(shift, c0, c, sh, 0.0f);
  const long p0 = block_range<BN_REV_AFFINE>() * ppb, p1 = min(npix, p0 + ppb);
  auto emit = [&](long pix, const Raw8<T>& zz, const Raw8<T>& rres, int valid) {
    float v[8], r[8];
    unpack8(zz, v);
    if (res) unpack8(rres, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float a = v[i] * sc[i] + sh[i];
      if (act == YMS_ACT_SILU) a = silu_f(a);
      if (res) a += r[i];
      v[i] = a;
    }
    store8(y + pix * y_ld + y_off + c0, valid, v);
  };
  const long step = (long)m.PY * BN_U;
  if (PIPE && c % 8 == 0) {
    auto issue = [&](long b, Raw8<T> (&zz)[BN_U], Raw8<T> (&rres)[BN_U]) {
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long pix = min(b + (long)u * m.PY, p1 - 1);
        load_raw8_nt(z + pix * z_ld + z_off + c0, zz[u]);       // z's last read until the backward
        if (res) load_raw8(res + pix * res_ld + res_off + c0, 8, rres[u]);
      }
    };
    auto consume = [&](long b, const Raw8<T> (&zz)[BN_U], const Raw8<T> (&rres)[BN_U]) {
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long pix = b + (long)u * m.PY;
        if (pix < p1) emit(pix, zz[u], rres[u], 8);
      }
    };
    long base = p0 + m.py;
    if (base < p1) {
      Raw8<T> za[BN_U], ra[BN_U], zb[BN_U], rb[BN_U];
      issue(base, za, ra);
      while (true) {
        issue(base + step, zb, rb);
        consume(base, za, ra);
        base += step;
        if (base >= p1) break;
        issue(base + step, za, ra);
        consume(base, zb, rb);
        base += step;
        if (base >= p1) break;
      }
    }
  } else {
    for (long base = p0 + m.py; base < p1; base += step) {
      Raw8<T> zr[BN_U], rr[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long pix = base + (long)u * m.PY;
        if (pix < p1) {
          load_raw8(z + pix * z_ld + z_off + c0, nv, zr[u]);
          if (res) load_raw8(res + pix * res_ld + res_off + c0, nv, rr[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long pix = base + (long)u * m.PY;
        if (pix < p1) emit(pix, zr[u], rr[u], nv);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// BN + SiLU backward.  Each block owns a contiguous pixel range and writes one partial row
// [2][c] (sum da, sum da*xhat) -- deterministic, no atomics.
// ------------------------------------------------------------------------------------------
struct BwdFin {          // fused finalize (FIN): the last reduce block to finish sums every partial row
  unsigned* cnt;        // arrival counter, zero on entry (the plan zeroes one per layer per backward)
  float *dgamma, *dbeta, *coef;
  long count;
};

// PIPE = false: the serial loop for every c (c % 8 != 0 tails; the host launches PIPE = true)
template <typename T, bool HAS_Z, bool FIN = false, bool PIPE = true>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(long npix, int c, const T* z, int z_ld,
                                                            int z_off, const T* gy, int gy_ld, int gy_off,
                                                            const float* scale, const float* shift,
                                                            const float* mi, int act, float* ws, long ppb,
                                                            BwdFin fin = BwdFin{}) {
  __shared__ float red[2][2048 + 64];
  ChanMap m(c);
  const int c0 = m.g * 8, nv = min(8, c - c0);
  float a1[8], a2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a1[i] = 0.f; a2[i] = 0.f; }
  if (m.active) {
    float sc[8], sh[8], mu[8], is[8];
    if (HAS_Z) {
      load_params8(scale, c0, c, sc, 0.f);
      load_params8(shift, c0, c, sh, 0.f);
      load_params8(mi, c0, c, mu, 0.f);
      load_params8(mi + c, c0, c, is, 0.f);
    }
    const long p0 = block_range<BN_REV_RED>() * ppb, p1 = min(npix, p0 + ppb);
    auto accum = [&](const Raw8<T>& g, const Raw8<T>& zz) {
      float gv[8], zv[8];
      unpack8(g, gv);
      if (HAS_Z) unpack8(zz, zv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float da = gv[i], xh = 0.f;
        if (HAS_Z) {
          const float a = zv[i] * sc[i] + sh[i];
          if (act == YMS_ACT_SILU) da = gv[i] * dsilu_f(a);
          xh = (zv[i] - mu[i]) * is[i];
        }
        a1[i] += da;
        a2[i] += da * xh;
      }
    };
    const long step = (long)m.PY * BN_UR;
    if (PIPE && c % 8 == 0) {
      // software-pipelined: the next U pixels' loads are in flight while this U's math runs
      // (2 blocks per CU leave too few waves to hide HBM latency otherwise).  Loads are
      // unconditional -- pixels past the range re-read the last one and are masked out of the
      // sums -- so no branch separates a load from its wait and vmcnt can count.
      auto issue = [&](long b, Raw8<T> (&g)[BN_UR], Raw8<T> (&zz)[BN_UR]) {
#pragma unroll
        for (int u = 0; u < BN_UR; ++u) {
          const long pix = min(b + (long)u * m.PY, p1 - 1);
          load_raw8(gy + pix * gy_ld + gy_off + c0, 8, g[u]);
          if (HAS_Z) load_raw8(z + pix * z_ld + z_off + c0, 8, zz[u]);
        }
      };
      auto consume = [&](long b, const Raw8<T> (&g)[BN_UR], const Raw8<T> (&zz)[BN_UR]) {
#pragma unroll
        for (int u = 0; u < BN_UR; ++u)
          if (b + (long)u * m.PY < p1) accum(g[u], zz[u]);
      };
      long base = p0 + m.py;
      if (base < p1) {
        Raw8<T> ga[BN_UR], za[BN_UR], gb[BN_UR], zb[BN_UR];
        issue(base, ga, za);
        while (true) {
          issue(base + step, gb, zb);
          consume(base, ga, za);
          base += step;
          if (base >= p1) break;
          issue(base + step, ga, za);
          consume(base, gb, zb);
          base += step;
          if (base >= p1) break;
        }
      }
    } else {
      for (long base = p0 + m.py; base < p1; base += step) {
        Raw8<T> gr[BN_UR], zr[BN_UR];
#pragma unroll
        for (int u = 0; u < BN_UR; ++u) {
          const long pix = base + (long)u * m.PY;
          if (pix < p1) {
            load_raw8(gy + pix * gy_ld + gy_off + c0, nv, gr[u]);
            if (HAS_Z) load_raw8(z + pix * z_ld + z_off + c0, nv, zr[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < BN_UR; ++u)
          if (base + (long)u * m.PY < p1) accum(gr[u], zr[u]);
      }
    }
  }
  // reduce over the PY pixel lanes in a fixed order: red[k][py*8G + g*8 + i]
  const int W = m.G * 8;
  for (int lane0 = 0; lane0 < m.PY; lane0 += 2048 / W) {
    const int lanes = min(m.PY - lane0, 2048 / W);
    if (m.active && m.py >= lane0 && m.py < lane0 + lanes) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[0][(m.py - lane0) * W + c0 + i] = a1[i];
        red[1][(m.py - lane0) * W + c0 + i] = a2[i];
      }
    }
    __syncthreads();
    for (int ch = threadIdx.x; ch < c; ch += 256) {
      float t1 = 0.f, t2 = 0.f;
      for (int l = 0; l < lanes; ++l) { t1 += red[0][l * W + ch]; t2 += red[1][l * W + ch]; }
      if (lane0 == 0) {
        ws[block_range<BN_REV_RED>() * 2 * c + ch] = t1;          // row = the block's pixel range
        ws[block_range<BN_REV_RED>() * 2 * c + c + ch] = t2;
      } else {
        ws[block_range<BN_REV_RED>() * 2 * c + ch] += t1;
        ws[block_range<BN_REV_RED>() * 2 * c + c + ch] += t2;
      }
    }
    __syncthreads();
  }
  if constexpr (FIN) {
    // in-launch finalize (cdna_hip_programming.md G16 counter hand-off): every wave drains its
    // partial-row stores, one agent-scope release + ticket; the block drawing the last ticket
    // acquires and sums all rows in a fixed order (deterministic whichever block is last)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(&red[0][0]);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(fin.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = (t == gridDim.x - 1) ? 1u : 0u;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (flag[0] == 0) return;
    __syncthreads();
    const int rows = gridDim.x, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    double* dred = reinterpret_cast<double*>(&red[0][0]);     // [2][8][33] doubles
    for (int cb = 0; cb < c; cb += 32) {
      const int ch = cb + tx;
      double b1[4] = {0, 0, 0, 0}, b2[4] = {0, 0, 0, 0};
      if (ch < c) {
        int r = ty;
        for (; r + 24 < rows; r += 32) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            b1[u] += ws[(long)(r + 8 * u) * 2 * c + ch];
            b2[u] += ws[(long)(r + 8 * u) * 2 * c + c + ch];
          }
        }
        for (; r < rows; r += 8) {
          b1[0] += ws[(long)r * 2 * c + ch];
          b2[0] += ws[(long)r * 2 * c + c + ch];
        }
      }
      dred[(0 * 8 + ty) * 33 + tx] = (b1[0] + b1[1]) + (b1[2] + b1[3]);
      dred[(1 * 8 + ty) * 33 + tx] = (b2[0] + b2[1]) + (b2[2] + b2[3]);
      __syncthreads();
      if (ty == 0 && ch < c) {
        double t1 = 0.0, t2 = 0.0;
        for (int k = 0; k < 8; ++k) { t1 += dred[(0 * 8 + k) * 33 + tx]; t2 += dred[(1 * 8 + k) * 33 + tx]; }
        if (fin.dbeta) fin.dbeta[ch] = (float)t1;
        if (fin.dgamma) fin.dgamma[ch] = (float)t2;
        if (fin.coef) {
          fin.coef[ch] = (float)(t1 / (double)fin.count);
          fin.coef[c + ch] = (float)(t2 / (double)fin.count);
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(fin.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// 32 channels x TY row lanes per block.  TY = 8 (256 threads) by default: with the weight
// gradients running on the side stream, a 1024-thread block waits for a whole CU to drain,
// which puts that wait on the main stream's critical path.
template <int TY>
__global__ __launch_bounds__(32 * TY) void bn_bwd_finalize_kernel(int c, const float* ws, int rows, long count,
                                                                  float* dgamma, float* dbeta, float* coef) {
  __shared__ double red[2][TY][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int ch = blockIdx.x * 32 + tx;
  double a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
  if (ch < c) {
    int r = ty;
    for (; r + 3 * TY < rows; r += 4 * TY) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a1[u] += ws[(long)(r + TY * u) * 2 * c + ch];
        a2[u] += ws[(long)(r + TY * u) * 2 * c + c + ch];
      }
    }
    for (; r < rows; r += TY) {
      a1[0] += ws[(long)r * 2 * c + ch];
      a2[0] += ws[(long)r * 2 * c + c + ch];
    }
  }
  red[0][ty][tx] = (a1[0] + a1[1]) + (a1[2] + a1[3]);
  red[1][ty][tx] = (a2[0] + a2[1]) + (a2[2] + a2[3]);
  __syncthreads();
  if (ty == 0 && ch < c) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < TY; ++k) { t1 += red[0][k][tx]; t2 += red[1][k][tx]; }
    if (dbeta) dbeta[ch] = (float)t1;
    if (dgamma) dgamma[ch] = (float)t2;
    if (coef) {
      coef[ch] = (float)(t1 / (double)count);
      coef[c + ch] = (float)(t2 / (double)count);
    }
  }
}


// PIPE (the default): software-pipelined like the reduce (c % 8 == 0): the next U pixels' loads (clamped to
// the block's last pixel, masked) are in flight while this U is computed and stored.  Stores stay
// masked: dz may overwrite z in place and gres may accumulate, so a duplicate pixel must not be
// written twice.
template <typename T, bool PIPE = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(long npix, int c, const T* z, int z_ld, int z_off,
                                                           const T* gy, int gy_ld, int gy_off, const float* scale,
                                                           const float* shift, const float* mi,
                                                           const float* coef, int act, T* dz, int dz_ld,
                                                           int dz_off, T* gres, int gres_ld, int gres_off,
                                                           int gres_acc, long ppb) {
  ChanMap m(c);
  if (!m.active) return;
  const int c0 = m.g * 8, nv = min(8, c - c0);
  // dz = sc*(da - k0 - (z-mu)*is*k1) = sc*da + A + B*z
  float sc[8], sh[8], A[8], Bz[8];
  {
    float mu[8], is[8], k0[8], k1[8];
    load_params8(scale, c0, c, sc, 0.f);
    load_params8(shift, c0, c, sh, 0.f);
    load_params8(mi, c0, c, mu, 0.f);
    load_params8(mi + c, c0, c, is, 0.f);
    load_params8(coef, c0, c, k0, 0.f);
    load_params8(coef + c, c0, c, k1, 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      Bz[i] = -sc[i] * k1[i] * is[i];
      A[i] = -sc[i] * k0[i] - Bz[i] * mu[i];
    }
  }
  const long p0 = block_range<BN_REV_APPLY>() * ppb, p1 = min(npix, p0 + ppb);
  const bool racc = gres && gres_acc;
  auto emit = [&](long pix, const Raw8<T>& g, const Raw8<T>& zz, const Raw8<T>& rres, int valid) {
    float gv[8], zv[8], out[8];
    unpack8(g, gv);
    unpack8(zz, zv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float da = gv[i];
      if (act == YMS_ACT_SILU) da *= dsilu_f(zv[i] * sc[i] + sh[i]);
      out[i] = sc[i] * da + A[i] + Bz[i] * zv[i];
    }
    if (gres) {
      float r[8];
      if (gres_acc) {
        unpack8(rres, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] += gv[i];
        store8(gres + pix * gres_ld + gres_off + c0, valid, r);
      } else {
        store8(gres + pix * gres_ld + gres_off + c0, valid, gv);
      }
    }
    store8(dz + pix * dz_ld + dz_off + c0, valid, out);
  };
  const long step = (long)m.PY * BN_UA;
  if (PIPE && c % 8 == 0) {
    auto issue = [&](long b, Raw8<T> (&g)[BN_UA], Raw8<T> (&zz)[BN_UA], Raw8<T> (&rres)[BN_UA]) {
#pragma unroll
      for (int u = 0; u < BN_UA; ++u) {
        const long pix = min(b + (long)u * m.PY, p1 - 1);
        load_raw8_nt(gy + pix * gy_ld + gy_off + c0, g[u]);     // the last reads of gy and z
        load_raw8_nt(z + pix * z_ld + z_off + c0, zz[u]);
        if (racc) load_raw8(gres + pix * gres_ld + gres_off + c0, 8, rres[u]);
      }
    };
    auto consume = [&](long b, const Raw8<T> (&g)[BN_UA], const Raw8<T> (&zz)[BN_UA], const Raw8<T> (&rres)[BN_UA]) {
#pragma unroll
      for (int u = 0; u < BN_UA; ++u) {
        const long pix = b + (long)u * m.PY;
        if (pix < p1) emit(pix, g[u], zz[u], rres[u], 8);
      }
    };
    long base = p0 + m.py;
    if (base < p1) {
      Raw8<T> ga[BN_UA], za[BN_UA], ra[BN_UA], gb[BN_UA], zb[BN_UA], rb[BN_UA];
      issue(base, ga, za, ra);
      // the next group's loads go out before this group's stores.  Every pixel is loaded and
      // stored by one thread (in-place dz over z is per pixel and per thread); a clamped load of
      // another thread's pixel may see its dz, but that value is masked and never stored
      while (true) {
        issue(base + step, gb, zb, rb);
        consume(base, ga, za, ra);
        base += step;
        if (base >= p1) break;
        issue(base + step, ga, za, ra);
        consume(base, gb, zb, rb);
        base += step;
        if (base >= p1) break;
      }
    }
  } else {
    for (long base = p0 + m.py; base < p1; base += step) {
      Raw8<T> gr[BN_UA], zr[BN_UA], rr[BN_UA];
#pragma unroll
      for (int u = 0; u < BN_UA; ++u) {
        const long pix = base + (long)u * m.PY;
        if (pix < p1) {
          load_raw8(gy + pix * gy_ld + gy_off + c0, nv, gr[u]);
          load_raw8(z + pix * z_ld + z_off + c0, nv, zr[u]);
          if (racc) load_raw8(gres + pix * gres_ld + gres_off + c0, nv, rr[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < BN_UA; ++u) {
        const long pix = base + (long)u * m.PY;
        if (pix < p1) emit(pix, gr[u], zr[u], rr[u], nv);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// SPPF pools: slot k = clipped (4k+1)x(4k+1) window max of slot 0 (== k chained MaxPool5).
// ------------------------------------------------------------------------------------------
// One MaxPool2d(5, 1, 2) of the SPPF chain: slot `out` = pool5(slot `in`) (-inf padding).
// The chain p1 = pool(x), p2 = pool(p1), p3 = pool(p2) runs as three launches (75 loads per
// output group instead of the 169 of a direct 13x13 window); max is exact and a NaN in the window
// wins (torch's `val > max || isnan(val)`), so the result is bit-identical to the reference's chained
// pools.
template <typename T>
__global__ __launch_bounds__(256) void pool5_fwd_kernel(int n, int h, int w, int c, T* buf, int ld, int in_off,
                                                        int out_off) {
  const int G = c >> 3;
  const uint32_t total = (uint32_t)n * h * w * G;
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
    const uint32_t g = t % G, pix = t / G;
    const uint32_t x = pix % w, r = pix / w;
    const uint32_t y = r % h, b = r / h;
    float m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = -INFINITY;
    const int y0 = max((int)y - 2, 0), y1 = min((int)y + 2, h - 1);
    const int x0 = max((int)x - 2, 0), x1 = min((int)x + 2, w - 1);
    for (int yy = y0; yy <= y1; ++yy) {
      const T* row = buf + ((long)(b * h + yy) * w) * ld + in_off + g * 8;
      for (int xx = x0; xx <= x1; ++xx) {
        float v[8];
        Vec8<T>::load(row + (long)xx * ld, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = (v[i] > m[i] || v[i] != v[i]) ? v[i] : m[i];   // NaN propagates (torch)
      }
    }
    Vec8<T>::store(buf + (long)pix * ld + out_off + g * 8, m);
  }
}

// argmax of a 5x5 (pad 2, -inf) window over input slot `in`, PyTorch scan order, first max.
template <typename T>
__global__ void pool5_argmax_kernel(int n, int h, int w, int c, const T* buf, int ld, int in_off,
                                    uint8_t* arg) {
  const int G = (c + 7) >> 3;
  const uint32_t total = (uint32_t)n * h * w * G;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    uint32_t r = t / G;
    const int x = (int)(r % w);
    r /= w;
    const int y = (int)(r % h);
    const int b = (int)(r / h);
    const int c0 = g * 8, nv = min(8, c - c0);
    float best[8];
    uint8_t idx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; idx[i] = 255; }
    for (int ky = 0; ky < 5; ++ky) {
      const int yy = y - 2 + ky;
      if (yy < 0 || yy >= h) continue;
      for (int kx = 0; kx < 5; ++kx) {
        const int xx = x - 2 + kx;
        if (xx < 0 || xx >= w) continue;
        float v[8];
        load8(buf + (((long)b * h + yy) * w + xx) * ld + in_off + c0, nv, v);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (idx[i] == 255 || v[i] > best[i] || v[i] != v[i]) {  // (val > maxval) || isnan(val)
            best[i] = v[i];
            idx[i] = (uint8_t)(ky * 5 + kx);
          }
      }
    }
    uint8_t* a = arg + ((((long)b * h + y) * w + x) * G + g) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = idx[i];
  }
}

// g[in slot] += sum over the 25 outputs o whose argmax points at this position of g[out slot]
template <typename T>
__global__ void pool5_gather_kernel(int n, int h, int w, int c, const uint8_t* arg, T* g, int ld,
                                    int in_off, int out_off) {
  const int G = (c + 7) >> 3;
  const uint32_t total = (uint32_t)n * h * w * G;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int gg = (int)(t % G);
    uint32_t r = t / G;
    const int x = (int)(r % w);
    r /= w;
    const int y = (int)(r % h);
    const int b = (int)(r / h);
    const int c0 = gg * 8, nv = min(8, c - c0);
    float acc[8];
    load8(g + (((long)b * h + y) * w + x) * ld + in_off + c0, nv, acc);
    // output o = (y - ky + 2, x - kx + 2) sees this input at window offset (ky, kx)
    for (int ky = 0; ky < 5; ++ky) {
      const int oy = y - ky + 2;
      if (oy < 0 || oy >= h) continue;
      for (int kx = 0; kx < 5; ++kx) {
        const int ox = x - kx + 2;
        if (ox < 0 || ox >= w) continue;
        const long o = ((long)b * h + oy) * w + ox;
        const uint8_t* a = arg + (o * G + gg) * 8;
        const uint2 av = *reinterpret_cast<const uint2*>(a);
        const uint8_t want = (uint8_t)(ky * 5 + kx);
        float gv[8];
        load8(g + o * ld + out_off + c0, nv, gv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint8_t ai = (uint8_t)(((i < 4 ? av.x : av.y) >> (8 * (i & 3))) & 0xff);
          if (ai == want) acc[i] += gv[i];
        }
      }
    }
    store8(g + (((long)b * h + y) * w + x) * ld + in_off + c0, nv, acc);
  }
}


// ------------------------------------------------------------------------------------------
// nearest x2 upsample
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void upsample_fwd_kernel(int n, int h, int w, int c, const T* x, int x_ld, int x_off,
                                    T* y, int y_ld, int y_off) {
  const int G = (c + 7) >> 3;
  const int H2 = 2 * h, W2 = 2 * w;
  const long total = (long)n * H2 * W2 * G;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    long r = t / G;
    const int X = (int)(r % W2);
    r /= W2;
    const int Y = (int)(r % H2);
    const int b = (int)(r / H2);
    const int c0 = g * 8, nv = min(8, c - c0);
    float v[8];
    load8(x + (((long)b * h + (Y >> 1)) * w + (X >> 1)) * x_ld + x_off + c0, nv, v);
    store8(y + (((long)b * H2 + Y) * W2 + X) * y_ld + y_off + c0, nv, v);
  }
}

template <typename T>
__global__ void upsample_bwd_kernel(int n, int h, int w, int c, const T* gy, int gy_ld, int gy_off,
                                    T* gx, int gx_ld, int gx_off, int accumulate) {
  const int G = (c + 7) >> 3;
  const int W2 = 2 * w;
  const long total = (long)n * h * w * G;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    long r = t / G;
    const int x = (int)(r % w);
    r /= w;
    const int y = (int)(r % h);
    const int b = (int)(r / h);
    const int c0 = g * 8, nv = min(8, c - c0);
    float s[8];
    T* dst = gx + (((long)b * h + y) * w + x) * gx_ld + gx_off + c0;
    if (accumulate) load8(dst, nv, s);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = 0.f;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float v[8];
      const int Y = 2 * y + (d >> 1), X = 2 * x + (d & 1);
      load8(gy + (((long)b * 2 * h + Y) * W2 + X) * gy_ld + gy_off + c0, nv, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += v[i];
    }
    store8(dst, nv, s);
  }
}

// ------------------------------------------------------------------------------------------
// layout / cast
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void pack_input_kernel(int n, int c, int h, int w, const float* x, T* y, int ld) {
  const long npix = (long)n * h * w;
  const long hw = (long)h * w;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < npix; t += (long)gridDim.x * blockDim.x) {
    const long b = t / hw, s = t - b * hw;
    for (int c0 = 0; c0 < ld; c0 += 8) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (c0 + i < c) ? x[(b * c + c0 + i) * hw + s] : 0.0f;
      Vec8<T>::store(y + t * ld + c0, v);
    }
  }
}

// NHWC view -> NCHW contiguous, 64x64 (pixel x channel) tiles through LDS.
template <typename TI, typename TO>
__global__ void nhwc_to_nchw_kernel(int n, long hw, int c, const TI* x, int ld, int off, TO* y) {
  __shared__ float tile[64][65];
  const long pt = (long)blockIdx.x * 64;
  const int ct = blockIdx.y * 64;
  const int b = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const long p = pt + r;
    const int ch = ct + tx;
    tile[r][tx] = (p < hw && ch < c) ? (float)x[((long)b * hw + p) * ld + off + ch] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int ch = ct + r;
    const long p = pt + tx;
    if (p < hw && ch < c) y[((long)b * c + ch) * hw + p] = (TO)tile[tx][r];
  }
}

template <typename TI, typename TO>
__global__ void nchw_to_nhwc_kernel(int n, long hw, int c, const TI* x, TO* y, int ld, int off,
                                    int accumulate) {
  __shared__ float tile[64][65];
  const long pt = (long)blockIdx.x * 64;
  const int ct = blockIdx.y * 64;
  const int b = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int ch = ct + r;
    const long p = pt + tx;
    tile[r][tx] = (p < hw && ch < c) ? (float)x[((long)b * c + ch) * hw + p] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const long p = pt + r;
    const int ch = ct + tx;
    if (p < hw && ch < c) {
      TO* d = y + ((long)b * hw + p) * ld + off + ch;
      float v = tile[tx][r];
      if (accumulate) v += (float)*d;
      *d = (TO)v;
    }
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(long count, const TI* x, TO* y) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < count; t += (long)gridDim.x * blockDim.x)
    y[t] = (TO)(float)x[t];
}

}  // namespace yms

using namespace yms;

#define YMS_DT_DISPATCH(dt, T, ...)                 \
  do {                                              \
    if ((dt) == YMS_BF16) { typedef bf16 T; __VA_ARGS__; } \
    else if ((dt) == YMS_F16) { typedef f16 T; __VA_ARGS__; } \
    else if ((dt) == YMS_F32) { typedef float T; __VA_ARGS__; } \
    else return YMS_ERR_INVALID;                    \
  } while (0)

static bool vok(int ld, int off, int c) { return c > 0 && ld % 8 == 0 && off % 8 == 0 && off + c <= ld; }

extern "C" {

yms_status yms_bn_fold(int c, const float* gamma, const float* beta, const float* rmean,
                       const float* rvar, float eps, float* scale, float* shift, void* stream) {
  if (c <= 0 || !scale || !shift) return YMS_ERR_INVALID;
  if (gamma && (!beta || !rmean || !rvar)) return YMS_ERR_INVALID;
  hipLaunchKernelGGL(bn_fold_kernel, dim3(cdiv(c, 256)), dim3(256), 0, (hipStream_t)stream, c, gamma,
                     beta, rmean, rvar, eps, scale, shift);
  return launch_status();
}

yms_status yms_bn_finalize_ld(int c, float* stats, int rows, int stats_ld, long count,
                              const float* gamma, const float* beta, float* rmean, float* rvar,
                              float momentum, float eps, float* mean_invstd, int mi_ld, float* scale,
                              float* shift, void* stream) {
  if (c <= 0 || !stats || rows <= 0 || count <= 0 || !gamma || !beta || !mean_invstd || !scale || !shift)
    return YMS_ERR_INVALID;
  if (stats_ld < c || mi_ld < c) return YMS_ERR_INVALID;
  int rs = 1, nrows = rows;
  if (rows > 1024) {   // long tables: pre-reduce in parallel (in place), then finalize the partial rows
    const int S = std::min(256, cdiv(rows, 64));
    rs = cdiv(rows, S);
    nrows = cdiv(rows, rs);
    hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(cdiv(c, 64), nrows), dim3(256), 0, (hipStream_t)stream, c,
                       stats, rows, stats_ld, rs);
  }
  if (rs == 1) {
    hipLaunchKernelGGL(bn_finalize_small_kernel, dim3(cdiv(c, 8)), dim3(256), 0, (hipStream_t)stream, c,
                       (const float*)stats, rows, stats_ld, count, gamma, beta, rmean, rvar, momentum, eps,
                       mean_invstd, mi_ld, scale, shift);
    return launch_status();
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(c, FIN_CW)), dim3(1024), 0, (hipStream_t)stream, c,
                     (const float*)stats, nrows, stats_ld, rs, rows, count, gamma, beta, rmean, rvar, momentum,
                     eps, mean_invstd, mi_ld, scale, shift);
  return launch_status();
}

yms_status yms_bn_finalize(int c, float* stats, int rows, int stats_ld, long count,
                           const float* gamma, const float* beta, float* rmean, float* rvar,
                           float momentum, float eps, float* mean_invstd, float* scale,
                           float* shift, void* stream) {
  return yms_bn_finalize_ld(c, stats, rows, stats_ld, count, gamma, beta, rmean, rvar, momentum, eps,
                            mean_invstd, c, scale, shift, stream);
}

// pixels per block for the channel-stationary kernels: about four U-pixel iterations per
// thread (amortises the per-channel parameter loads; measured best of 1/2/4/8), at most 8192
// blocks
static long elem_ppb(long npix, int c, int iters = 4) {
  const long py = 256 / ((c + 7) / 8);
  long blocks = std::min<long>(std::max<long>(cdiv(npix, py * BN_U * iters), 1), 8192);
  // (round 3: a floor of 1024-2048 blocks for the small 20^2 / 40^2 layers made the step slower,
  // profiles/r03s_bn_minblocks_ab.txt: the extra blocks wait for CU slots the side stream holds)
  return (npix + blocks - 1) / blocks;
}

yms_status yms_affine_act(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                          const float* scale, const float* shift, int act,
                          const void* res, int res_ld, int res_off,
                          void* y, int y_ld, int y_off, void* stream) {
  if (npix <= 0 || !z || !y || !vok(z_ld, z_off, c) || !vok(y_ld, y_off, c)) return YMS_ERR_INVALID;
  if (res && !vok(res_ld, res_off, c)) return YMS_ERR_INVALID;
  if (c > 2048) return YMS_ERR_UNSUPPORTED;
  // two U-pixel iterations per thread: the forward affine pass (no side-stream work beside it) took
  // 1.73 / 1.74 ms per YOLOv8-s step against 1.80 / 1.80 at four, 3.66-3.68 vs 3.70-3.73 ms on
  // YOLO-MS-S (interleaved, profiles/r03y_affine_iters_ab.txt)
  // software-pipelined loop: affine 1.72 -> 1.70 ms per YOLOv8-s step, 3.68 -> 3.57 ms on YOLO-MS-S,
  // steps 18.20 -> 18.13 ms and 37.24 -> 37.12 ms over the serial loop (interleaved pairs; pipelined
  // at 4 / 8 iterations slower, profiles/r03zg_affine_pipe_ab.txt)
  const long ppb = elem_ppb(npix, c, 2);
  const unsigned blocks = (unsigned)((npix + ppb - 1) / ppb);
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL((affine_act_kernel<T, true>), dim3(blocks), dim3(256), 0,
                                               (hipStream_t)stream, npix, c, (const T*)z, z_ld, z_off,
                                               scale, shift, act, (const T*)res, res_ld, res_off, (T*)y,
                                               y_ld, y_off, ppb));
  return launch_status();
}

// pixels per BN-backward reduce block.  Partial-sum rows = reduce blocks, at most 256 with the
// pipelined reduce loop (one block per CU; cap 128 / 256 / 384 / 512: 18.64 / 18.28 / 18.52 /
// 18.74 ms per YOLOv8-s step, interleaved, profiles/r03ze_bn_reduce_pipe_cap_ab.txt).  With the
// serial loop 512 was best (round 2: 1024 19.82 ms, 512 19.50, 256 19.53, 2048 20.33).  The fused
// reduce + finalize (one last block sums the whole table) also keeps rows <= 32768 / c (table
// <= 256 KB); the two-kernel path does not: that cap left 64-128 reduce blocks on 256 CUs for
// the 256/512-channel layers (interleaved A/B: YOLOv8-s 19.51 -> 19.26 ms, -l 61.7 -> 60.9 ms).
static long bwd_pix_per_block(long npix, int c, bool fused) {
  constexpr long cap = 256, cprod = 32768;
  const long ccap = fused ? std::max(32l, cprod / std::max(c, 1)) : cap;
  const long rows = std::max(1l, std::min(std::min(cap, ccap), (npix + 63) / 64));
  return (npix + rows - 1) / rows;
}

// the number of partial rows the reduce WRITES = its launched block count ceil(npix / ppb).
// Once a cap applies this can be below the cap (npix = 44801, c = 64: ppb 176, 255 blocks), so the
// scratch size, the launch and the finalize all use this one function.
int yms_bn_bwd_rows(long npix, int c) {
  if (npix <= 0 || c <= 0) return 0;
  const long ppb = bwd_pix_per_block(npix, c, false);   // >= the fused path's rows: sizes both
  return (int)((npix + ppb - 1) / ppb);
}

yms_status yms_bn_act_bwd_reduce(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                 const void* gy, int gy_ld, int gy_off, const float* scale,
                                 const float* shift, const float* mean_invstd, int act,
                                 float* ws, void* stream) {
  if (npix <= 0 || !gy || !ws || !vok(gy_ld, gy_off, c)) return YMS_ERR_INVALID;
  if (z && (!vok(z_ld, z_off, c) || !scale || !shift || !mean_invstd)) return YMS_ERR_INVALID;
  if (c > 2048) return YMS_ERR_UNSUPPORTED;
  const long ppb = bwd_pix_per_block(npix, c, false);
  const unsigned rows = (unsigned)((npix + ppb - 1) / ppb);
  // software-pipelined loop (c % 8 == 0).  At 512 rows it was step-neutral over the serial loop
  // (the reduce -10%, the apply after it +5%, profiles/r03zb_bn_reduce_pipe_ab.txt); with the
  // latency hidden inside each block, half the blocks (256 rows, bwd_pix_per_block) win: YOLOv8-s
  // 18.63 -> 18.32 ms/step, YOLO-MS-S 37.42 -> 37.28 ms (means of four interleaved runs each,
  // profiles/r03zd_*, r03ze_*); serial at 256 rows is slower.
#define YMS_RED(HZ)                                                                                      \
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, HZ, false, true>), dim3(rows), dim3(256), 0, \
                                               (hipStream_t)stream, npix, c, HZ ? (const T*)z : (const T*)nullptr, \
                                               HZ ? z_ld : 0, HZ ? z_off : 0, (const T*)gy, gy_ld, gy_off, scale,  \
                                               shift, mean_invstd, act, ws, ppb))
  if (z) YMS_RED(true);
  else YMS_RED(false);
#undef YMS_RED
  return launch_status();
}

yms_status yms_bn_act_bwd_finalize(int c, const float* ws, int rows, long count, float* dgamma,
                                   float* dbeta, float* coef, void* stream) {
  if (c <= 0 || !ws || rows <= 0 || count <= 0) return YMS_ERR_INVALID;
  // (tried and dropped: float4 channel quads x 32 row lanes with every load of a lane in flight --
  // 19.42 -> 19.65 ms; a latency-shaped 8-channel x 32-lane variant with 4x the blocks -- +0.15-0.3
  // ms, profiles/r03q_bn_finalize_ab.txt: inside the step the finalize waits for CU slots, not loads)
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<8>, dim3(cdiv(c, 32)), dim3(256), 0, (hipStream_t)stream, c, ws,
                     rows, count, dgamma, dbeta, coef);
  return launch_status();
}

yms_status yms_bn_act_bwd_apply(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                const void* gy, int gy_ld, int gy_off, const float* scale,
                                const float* shift, const float* mean_invstd, const float* coef,
                                int act, void* dz, int dz_ld, int dz_off,
                                void* gres, int gres_ld, int gres_off, int gres_acc, void* stream) {
  if (npix <= 0 || !z || !gy || !dz || !scale || !shift || !mean_invstd || !coef) return YMS_ERR_INVALID;
  if (!vok(z_ld, z_off, c) || !vok(gy_ld, gy_off, c) || !vok(dz_ld, dz_off, c)) return YMS_ERR_INVALID;
  if (gres && !vok(gres_ld, gres_off, c)) return YMS_ERR_INVALID;
  if (c > 2048) return YMS_ERR_UNSUPPORTED;
  // software-pipelined loop at eight U-pixel iterations per thread (half the blocks of the serial
  // loop's best, four): YOLO-MS-S 37.27 -> 37.11 ms/step, YOLOv8-s 18.53 -> 18.49 ms (means of
  // two interleaved runs; 4 / 16 iterations pipelined are slower, profiles/r03zf_bn_apply_pipe_ab.txt)
  const long ppb = elem_ppb(npix, c, 8 * BN_U / BN_UA);    // the same pixels per block at any U
  const unsigned blocks = (unsigned)((npix + ppb - 1) / ppb);
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true>), dim3(blocks), dim3(256), 0,
                                               (hipStream_t)stream, npix, c, (const T*)z, z_ld, z_off,
                                               (const T*)gy, gy_ld, gy_off, scale, shift, mean_invstd, coef,
                                               act, (T*)dz, dz_ld, dz_off, (T*)gres, gres_ld, gres_off, gres_acc, ppb));
  return launch_status();
}

yms_status yms_bn_act_bwd_reduce_finalize(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                          const void* gy, int gy_ld, int gy_off, const float* scale,
                                          const float* shift, const float* mean_invstd, int act, float* ws,
                                          unsigned* counter, float* dgamma, float* dbeta, float* coef,
                                          void* stream) {
  if (npix <= 0 || !gy || !ws || !counter || !vok(gy_ld, gy_off, c)) return YMS_ERR_INVALID;
  if (z && (!vok(z_ld, z_off, c) || !scale || !shift || !mean_invstd)) return YMS_ERR_INVALID;
  if (c > 2048) return YMS_ERR_UNSUPPORTED;
  const long ppb = bwd_pix_per_block(npix, c, true);
  const unsigned rows = (unsigned)((npix + ppb - 1) / ppb);
  const BwdFin fin{counter, dgamma, dbeta, coef, npix};
  if (z) {
    YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, true>), dim3(rows), dim3(256), 0,
                                                 (hipStream_t)stream, npix, c, (const T*)z, z_ld, z_off,
                                                 (const T*)gy, gy_ld, gy_off, scale, shift, mean_invstd,
                                                 act, ws, ppb, fin));
  } else {
    YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false, true>), dim3(rows), dim3(256), 0,
                                                 (hipStream_t)stream, npix, c, (const T*)nullptr, 0, 0,
                                                 (const T*)gy, gy_ld, gy_off, scale, shift, mean_invstd,
                                                 act, ws, ppb, fin));
  }
  return launch_status();
}

yms_status yms_bias_bwd(int dtype, long npix, int c, const void* gy, int gy_ld, int gy_off,
                        float* ws, unsigned* counter, float* dbias, void* stream) {
  return yms_bn_act_bwd_reduce_finalize(dtype, npix, c, nullptr, 0, 0, gy, gy_ld, gy_off, nullptr, nullptr,
                                        nullptr, YMS_ACT_NONE, ws, counter, nullptr, dbias, nullptr, stream);
}

size_t yms_sppf_ws_bytes(int n, int h, int w, int c) {
  return (size_t)n * h * w * ((c + 7) / 8) * 8;
}

yms_status yms_sppf_pool_fwd(int dtype, int n, int h, int w, int c, void* buf, int ld, int off,
                             void* stream) {
  if (n <= 0 || h <= 0 || w <= 0 || !buf || !vok(ld, off, 4 * c) || c % 8 != 0) return YMS_ERR_INVALID;
  const long items = (long)n * h * w * ((c + 7) / 8);
  if (items >= (1l << 31)) return YMS_ERR_UNSUPPORTED;
  for (int k = 1; k <= 3; ++k)
    YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL(pool5_fwd_kernel<T>, dim3(grid_for(items)), dim3(256), 0,
                                                 (hipStream_t)stream, n, h, w, c, (T*)buf, ld,
                                                 off + (k - 1) * c, off + k * c));
  return launch_status();
}

yms_status yms_sppf_pool_bwd(int dtype, int n, int h, int w, int c, const void* buf, int ld,
                             int off, void* gbuf, int gld, int goff, void* ws, void* stream) {
  if (n <= 0 || !buf || !gbuf || !ws || !vok(ld, off, 4 * c) || !vok(gld, goff, 4 * c) || c % 8 != 0)
    return YMS_ERR_INVALID;
  if (ld != gld) return YMS_ERR_UNSUPPORTED;
  const long items = (long)n * h * w * ((c + 7) / 8);
  if (items >= (1l << 31)) return YMS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  // (round 3: a bit-identical whole-map fused backward, one launch per pool with the argmax and the
  // gather in LDS, was slower inside the overlapped step -- 18.37-18.47 -> 18.51-18.57 ms,
  // profiles/r03v_sppf_fused_ab.txt: its 64 KB-LDS blocks waited for the side stream's LDS)
  for (int k = 3; k >= 1; --k) {
    // pool k reads slot k-1 (value buf) and produced slot k; push grad of slot k into slot k-1
    YMS_DT_DISPATCH(dtype, T, {
      hipLaunchKernelGGL(pool5_argmax_kernel<T>, dim3(grid_for(items)), dim3(256), 0, st, n, h, w, c,
                         (const T*)buf, ld, off + (k - 1) * c, (uint8_t*)ws);
      hipLaunchKernelGGL(pool5_gather_kernel<T>, dim3(grid_for(items)), dim3(256), 0, st, n, h, w, c,
                         (const uint8_t*)ws, (T*)gbuf, gld, goff + (k - 1) * c, goff + k * c);
    });
  }
  return launch_status();
}

yms_status yms_upsample2x_fwd(int dtype, int n, int h, int w, int c, const void* x, int x_ld,
                              int x_off, void* y, int y_ld, int y_off, void* stream) {
  if (n <= 0 || !x || !y || !vok(x_ld, x_off, c) || !vok(y_ld, y_off, c)) return YMS_ERR_INVALID;
  const long items = (long)n * 4 * h * w * ((c + 7) / 8);
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL(upsample_fwd_kernel<T>, dim3(grid_for(items)), dim3(256), 0,
                                               (hipStream_t)stream, n, h, w, c, (const T*)x, x_ld, x_off,
                                               (T*)y, y_ld, y_off));
  return launch_status();
}

yms_status yms_upsample2x_bwd(int dtype, int n, int h, int w, int c, const void* gy, int gy_ld,
                              int gy_off, void* gx, int gx_ld, int gx_off, int accumulate,
                              void* stream) {
  if (n <= 0 || !gy || !gx || !vok(gy_ld, gy_off, c) || !vok(gx_ld, gx_off, c)) return YMS_ERR_INVALID;
  const long items = (long)n * h * w * ((c + 7) / 8);
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL(upsample_bwd_kernel<T>, dim3(grid_for(items)), dim3(256), 0,
                                               (hipStream_t)stream, n, h, w, c, (const T*)gy, gy_ld, gy_off,
                                               (T*)gx, gx_ld, gx_off, accumulate));
  return launch_status();
}

yms_status yms_pack_input(int dtype, int n, int c, int h, int w, const float* x, void* y, int ld,
                          void* stream) {
  if (n <= 0 || c <= 0 || !x || !y || ld % 8 != 0 || ld < c) return YMS_ERR_INVALID;
  const long npix = (long)n * h * w;
  YMS_DT_DISPATCH(dtype, T, hipLaunchKernelGGL(pack_input_kernel<T>, dim3(grid_for(npix)), dim3(256), 0,
                                               (hipStream_t)stream, n, c, h, w, x, (T*)y, ld));
  return launch_status();
}

#define YMS_DT2(d1, d2, T1, T2, ...)                                          \
  YMS_DT_DISPATCH(d1, T1, { YMS_DT_DISPATCH(d2, T2, __VA_ARGS__); })

yms_status yms_nhwc_to_nchw(int dtype, int dtype_nchw, int n, int h, int w, int c, const void* x,
                            int ld, int off, void* y, void* stream) {
  if (n <= 0 || !x || !y || ld < off + c) return YMS_ERR_INVALID;
  const long hw = (long)h * w;
  dim3 grid((unsigned)cdiv(hw, 64), (unsigned)cdiv(c, 64), (unsigned)n);
  YMS_DT2(dtype, dtype_nchw, TI, TO, hipLaunchKernelGGL((nhwc_to_nchw_kernel<TI, TO>), grid, dim3(256), 0,
                                                        (hipStream_t)stream, n, hw, c, (const TI*)x, ld, off,
                                                        (TO*)y));
  return launch_status();
}

yms_status yms_nchw_to_nhwc(int dtype_nchw, int dtype, int n, int h, int w, int c, const void* x,
                            void* y, int ld, int off, int accumulate, void* stream) {
  if (n <= 0 || !x || !y || ld < off + c) return YMS_ERR_INVALID;
  const long hw = (long)h * w;
  dim3 grid((unsigned)cdiv(hw, 64), (unsigned)cdiv(c, 64), (unsigned)n);
  YMS_DT2(dtype_nchw, dtype, TI, TO, hipLaunchKernelGGL((nchw_to_nhwc_kernel<TI, TO>), grid, dim3(256), 0,
                                                        (hipStream_t)stream, n, hw, c, (const TI*)x, (TO*)y,
                                                        ld, off, accumulate));
  return launch_status();
}

yms_status yms_cast(int dtype_in, int dtype_out, long count, const void* x, void* y, void* stream) {
  if (count <= 0 || !x || !y) return YMS_ERR_INVALID;
  YMS_DT2(dtype_in, dtype_out, TI, TO, hipLaunchKernelGGL((cast_kernel<TI, TO>), dim3(grid_for(count)),
                                                          dim3(256), 0, (hipStream_t)stream, count,
                                                          (const TI*)x, (TO*)y));
  return launch_status();
}

}  // extern "C"

extern "C" yms_status yms_zero(void* p, size_t bytes, void* stream) {
  if (!p) return YMS_ERR_INVALID;
  if (bytes == 0) return YMS_OK;
  return hipMemsetAsync(p, 0, bytes, (hipStream_t)stream) == hipSuccess ? YMS_OK : YMS_ERR_LAUNCH;
}

extern "C" yms_status yms_copy(void* dst, const void* src, size_t bytes, void* stream) {
  if (!dst || !src) return YMS_ERR_INVALID;
  if (bytes == 0) return YMS_OK;
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess
             ? YMS_OK : YMS_ERR_LAUNCH;
}

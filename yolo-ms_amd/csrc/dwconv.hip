// Depthwise k x k convolution (groups = channels, stride 1, pad k/2, k = 3/5/7/9) for gfx950,
// NHWC, the large-kernel mid conv of the YOLO-MS MS-Block inverted bottleneck (SURVEY 7.4:
// IB_k = 1x1 expand -> depthwise k x k -> 1x1 project; heterogeneous kernel sizes 3/5/7/9 per
// backbone stage, the "HKS" of the paper; the reference holds the MS-Block only as a diagram,
// annotations.md:66-133).  Not a dense contraction: VALU + LDS, bounded by HBM (k = 3, 5) or
// by the VALU FMA rate (k = 7, 9), never MFMA.
//
// Mapping: a 256-thread block owns a TY x TX = 8 x 32 output tile of one image and 32 channels;
// wave w owns 8 channels (one 16-B NHWC chunk), lane (ty, qx) = (lane / 8, lane % 8) owns the
// RX = 4 consecutive pixels (ty, 4 qx .. 4 qx + 3).  The (8 + k - 1) x (32 + k - 1) input halo of
// the block's channels is staged once in LDS (planar per wave, zero outside the image) with the
// block's k x k x 32 weights; per kernel row a lane slides an (RX + k - 1)-pixel window over its
// row and accumulates RX outputs in fp32 registers.
//   forward: y = act(conv * scale + shift) (eval, BN folded) | z + per-tile BN partial sums (train)
//   dgrad  : dx (+)= conv(dz, rot180(w))
//   wgrad  : dw[c][t] = sum_p x[p + d_t][c] dz[p][c]: per-lane (kernel row, tile row, column
//            segment) register partials across all of a block's tiles, one fixed-order LDS
//            reduction per block, per-block rows + fixed-order reduce
#include <algorithm>
#include <cstdlib>

#include "yms_common.hpp"

namespace yms {

constexpr int DW_TY = 8, DW_TX = 32, DW_RX = 4, DW_G = 4, DW_CB = DW_G * 8;   // 32 channels per block
enum { DW_FWD_AFFINE = 0, DW_FWD_STATS = 1, DW_DGRAD = 2 };

struct DwParams {
  const char* src;
  int src_ld, src_off;
  const float* w;        // [C][k][k] fp32 (nn.Conv2d(groups=C) weight)
  char* dst;
  int dst_ld, dst_off;
  const float* scale;
  const float* shift;
  int act;
  float* stats;
  int stats_ld;
  float* stats_cnt;      // per-tile pixel counts, right after the rows
  int accumulate;
  int N, H, W, C;
  int tiles_x, tiles_y;  // spatial tiles per image
};

// stage the (TY + K - 1) x (TX + K - 1) halo of 32 channels (zero outside the image / past C)
template <typename T, int K, int NT = 256>
__device__ __forceinline__ void dw_stage_halo(const DwParams& p, Raw8<T>* lds, int n, int y0, int x0, int c0) {
  constexpr int HH = DW_TY + K - 1, HW = DW_TX + K - 1, P = K / 2;
  const T* src = reinterpret_cast<const T*>(p.src);
  for (int it = threadIdx.x; it < DW_G * HH * HW; it += NT) {
    const int g = it / (HH * HW), r = it - g * (HH * HW);
    const int hy = r / HW, hx = r - hy * HW;
    const int y = y0 + hy - P, x = x0 + hx - P, c = c0 + 8 * g;
    Raw8<T> v;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 2); ++k) v.v[k] = u32x4{0u, 0u, 0u, 0u};
    if (y >= 0 && y < p.H && x >= 0 && x < p.W && c < p.C)
      load_raw8(src + (((long)n * p.H + y) * p.W + x) * p.src_ld + p.src_off + c, min(8, p.C - c), v);
    lds[it] = v;
  }
}

template <typename T, int K, int MODE>
__global__ __launch_bounds__(256) void dwconv_kernel(DwParams p) {
  constexpr int HH = DW_TY + K - 1, HW = DW_TX + K - 1;
  __shared__ Raw8<T> halo[DW_G * HH * HW];
  __shared__ __attribute__((aligned(16))) float wl[DW_G][K * K][8];
  const int tile = blockIdx.x;
  const int per_img = p.tiles_x * p.tiles_y;
  const int n = tile / per_img, rem = tile - n * per_img;
  const int y0 = (rem / p.tiles_x) * DW_TY, x0 = (rem % p.tiles_x) * DW_TX;
  const int c0 = blockIdx.y * DW_CB;
  dw_stage_halo<T, K>(p, halo, n, y0, x0, c0);
  for (int it = threadIdx.x; it < DW_G * K * K * 8; it += 256) {
    const int g = it / (K * K * 8), r = it - g * (K * K * 8);
    const int t = r / 8, i = r - t * 8;
    const int c = c0 + 8 * g + i;
    // dgrad correlates with the kernel rotated by 180 degrees
    const int tw = MODE == DW_DGRAD ? K * K - 1 - t : t;
    wl[g][t][i] = c < p.C ? p.w[(long)c * K * K + tw] : 0.0f;
  }
  __syncthreads();
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ty = lane >> 3, qx = lane & 7;
  const Raw8<T>* hp = halo + g * HH * HW;
  float acc[DW_RX][8];
#pragma unroll
  for (int i = 0; i < DW_RX; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[i][c] = 0.0f;
  // one kernel row at a time (not unrolled): the row's k x 8 weights live in registers
#pragma unroll 1
  for (int dy = 0; dy < K; ++dy) {
    float wr[K][8];
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&wl[g][dy * K + dx][0]);
      const f32x4 b = *reinterpret_cast<const f32x4*>(&wl[g][dy * K + dx][4]);
#pragma unroll
      for (int c = 0; c < 4; ++c) { wr[dx][c] = a[c]; wr[dx][4 + c] = b[c]; }
    }
    const Raw8<T>* row = hp + (ty + dy) * HW + 4 * qx;
#pragma unroll
    for (int q = 0; q < DW_RX + K - 1; ++q) {
      float v[8];
      unpack8(row[q], v);
#pragma unroll
      for (int i = 0; i < DW_RX; ++i) {
        const int dx = q - i;
        if (dx >= 0 && dx < K) {
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[i][c] += v[c] * wr[dx][c];
        }
      }
    }
  }
  const int c = c0 + 8 * g, nv = min(8, p.C - c);
  const int y = y0 + ty;
  float sc[8], sh[8];
  if (MODE == DW_FWD_AFFINE) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = (p.scale && c + k < p.C) ? p.scale[c + k] : 1.0f;
      sh[k] = (p.shift && c + k < p.C) ? p.shift[c + k] : 0.0f;
    }
  }
  if (nv > 0 && y < p.H) {
    T* dst = reinterpret_cast<T*>(p.dst);
#pragma unroll
    for (int i = 0; i < DW_RX; ++i) {
      const int x = x0 + 4 * qx + i;
      if (x >= p.W) continue;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = acc[i][k];
        if (MODE == DW_FWD_AFFINE) {
          v = v * sc[k] + sh[k];
          if (p.act == YMS_ACT_SILU) v = silu_f(v);
        }
        o[k] = v;
      }
      T* d = dst + (((long)n * p.H + y) * p.W + x) * p.dst_ld + p.dst_off + c;
      if (MODE == DW_DGRAD && p.accumulate) {
        float r[8];
        load8(d, nv, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += r[k];
      }
      store8(d, nv, o);
    }
  }
  if (MODE == DW_FWD_STATS) {
    // one statistics row per spatial tile (conv_common.hpp contract; its pixel count goes to the
    // count table after the rows): sum and centred M2 over the tile's valid pixels, two passes
    // over the fp32 accumulators, wave butterflies in a fixed order
    const int vy = min(DW_TY, p.H - y0), vx = min(DW_TX, p.W - x0);
    const float inv_n = 1.0f / (float)(vy * vx);
    float s1[8], m2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s = 0.f;
      if (y < p.H) {
#pragma unroll
        for (int i = 0; i < DW_RX; ++i)
          if (x0 + 4 * qx + i < p.W) s += acc[i][k];
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) s += __shfl_xor(s, m);
      const float mu = s * inv_n;
      float q = 0.f;
      if (y < p.H) {
#pragma unroll
        for (int i = 0; i < DW_RX; ++i)
          if (x0 + 4 * qx + i < p.W) {
            const float d = acc[i][k] - mu;
            q += d * d;
          }
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) q += __shfl_xor(q, m);
      s1[k] = s;
      m2[k] = q;
    }
    if (lane < 8 && c + lane < p.C) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k == lane) { a = s1[k]; b = m2[k]; }
      float* so = p.stats + (long)tile * 2 * p.stats_ld;
      so[c + lane] = a;
      so[p.stats_ld + c + lane] = b;
    }
    if (blockIdx.y == 0 && threadIdx.x == 0) p.stats_cnt[tile] = (float)(vy * vx);
  }
}

// wgrad: a 512-thread block owns 32 channels (4 groups of 8, 128 lanes each) and walks the
// spatial tiles blockIdx.x, blockIdx.x + gridDim.x, ...; per tile the x halo and the dz tile are
// staged in LDS.  Lane (dy, ty, s) of a group owns kernel row dy, tile row ty and column segment s
// (S segments of SL = 32 / S columns, K * 8 * S <= 128 lanes active) and keeps the K x 8 partial
// taps dw[dy][0..K)[8 channels] in registers across ALL its tiles: per 4 columns it reads the 4 dz
// values and the 4 + K - 1 halo values once and does 4 K 8 FMAs.  One fixed-order LDS reduction
// over (ty, s) at the end writes ws[blockIdx.x][tap][c]; dwconv_wgrad_reduce_kernel sums the blocks.
template <int K>
struct DwWg {
  static constexpr int S = K == 3 ? 4 : (K == 9 ? 1 : 2);
  static constexpr int SL = DW_TX / S;
  static constexpr int NA = K * DW_TY * S;   // active lanes per channel group
};
constexpr int DW_WG_NT = 512, DW_WG_LPG = DW_WG_NT / DW_G;

template <typename T, int K>
__global__ __launch_bounds__(DW_WG_NT) void dwconv_wgrad_kernel(DwParams p, const char* dz, int dz_ld, int dz_off,
                                                                 float* ws) {
  constexpr int HH = DW_TY + K - 1, HW = DW_TX + K - 1;
  constexpr int S = DwWg<K>::S, SL = DwWg<K>::SL, NA = DwWg<K>::NA;
  static_assert(NA <= DW_WG_LPG && SL % 4 == 0, "dw wgrad lane mapping");
  constexpr int HALO = DW_G * HH * HW, DZN = DW_G * DW_TY * DW_TX;
  constexpr int STAGE_B = (HALO + DZN) * (int)sizeof(Raw8<T>);
  constexpr int RED_B = NA * K * 8 * (int)sizeof(float);
  __shared__ __attribute__((aligned(16))) char smem[STAGE_B > RED_B ? STAGE_B : RED_B];
  Raw8<T>* halo = reinterpret_cast<Raw8<T>*>(smem);
  Raw8<T>* dzl = halo + HALO;
  float* red = reinterpret_cast<float*>(smem);
  const int c0 = blockIdx.y * DW_CB;
  const int g = threadIdx.x / DW_WG_LPG, l = threadIdx.x % DW_WG_LPG;
  const bool active = l < NA;
  const int ll = active ? l : 0;
  const int dy = ll / (DW_TY * S), r = ll % (DW_TY * S);
  const int ty = r / S, sx = (r % S) * SL;
  float part[K][8];
#pragma unroll
  for (int dx = 0; dx < K; ++dx)
#pragma unroll
    for (int k = 0; k < 8; ++k) part[dx][k] = 0.0f;
  const int per_img = p.tiles_x * p.tiles_y, ntiles = p.N * per_img;
  const T* dzp = reinterpret_cast<const T*>(dz);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / per_img, rem = tile - n * per_img;
    const int y0 = (rem / p.tiles_x) * DW_TY, x0 = (rem % p.tiles_x) * DW_TX;
    __syncthreads();      // previous tile's LDS reads are done
    dw_stage_halo<T, K, DW_WG_NT>(p, halo, n, y0, x0, c0);
    for (int it = threadIdx.x; it < DZN; it += DW_WG_NT) {
      const int g2 = it / (DW_TY * DW_TX), r2 = it - g2 * (DW_TY * DW_TX);
      const int y = y0 + r2 / DW_TX, x = x0 + r2 % DW_TX, c = c0 + 8 * g2;
      Raw8<T> v;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(T) / 2); ++k) v.v[k] = u32x4{0u, 0u, 0u, 0u};
      if (y < p.H && x < p.W && c < p.C)
        load_raw8(dzp + (((long)n * p.H + y) * p.W + x) * dz_ld + dz_off + c, min(8, p.C - c), v);
      dzl[it] = v;
    }
    __syncthreads();
    if (active) {
      const Raw8<T>* hrow = halo + g * HH * HW + (ty + dy) * HW + sx;
      const Raw8<T>* drow = dzl + g * DW_TY * DW_TX + ty * DW_TX + sx;
#pragma unroll 2
      for (int x4 = 0; x4 < SL; x4 += 4) {
        float d[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i) unpack8(drow[x4 + i], d[i]);
#pragma unroll
        for (int q = 0; q < 4 + K - 1; ++q) {
          float v[8];
          unpack8(hrow[x4 + q], v);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int dx = q - i;
            if (dx >= 0 && dx < K) {
#pragma unroll
              for (int k = 0; k < 8; ++k) part[dx][k] += v[k] * d[i][k];
            }
          }
        }
      }
    }
  }
  // fixed-order reduction over the (ty, s) lanes of each kernel row, one channel group at a time
  for (int gg = 0; gg < DW_G; ++gg) {
    __syncthreads();
    if (g == gg && active) {
      float* rp = red + l * K * 8;
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        *reinterpret_cast<f32x4*>(rp + dx * 8) = f32x4{part[dx][0], part[dx][1], part[dx][2], part[dx][3]};
        *reinterpret_cast<f32x4*>(rp + dx * 8 + 4) = f32x4{part[dx][4], part[dx][5], part[dx][6], part[dx][7]};
      }
    }
    __syncthreads();
    for (int it = threadIdx.x; it < K * K * 8; it += DW_WG_NT) {
      const int t = it / 8, k = it - t * 8;
      const int ddy = t / K, ddx = t - ddy * K;
      float s = 0.f;
      for (int rr = 0; rr < DW_TY * S; ++rr) s += red[((ddy * DW_TY * S + rr) * K + ddx) * 8 + k];
      const int cc = c0 + 8 * gg + k;
      if (cc < p.C) ws[((long)blockIdx.x * K * K + t) * p.C + cc] = s;
    }
  }
}

// dw[c][t] (+)= sum_b ws[b][t][c]: 64 outputs per block, wave w sums blocks b = w (mod 4) in order,
// the four partials are added in a fixed order
__global__ __launch_bounds__(256) void dwconv_wgrad_reduce_kernel(const float* ws, int blocks, int C, int KK, float* dw,
                                                                  int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const long stride = (long)C * KK;
  float s = 0.f;
  if (j < stride)
    for (int b = w; b < blocks; b += 4) s += ws[(long)b * stride + j];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && j < stride) {
    s = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    const int t = j / C, c = j - t * C;
    float* o = dw + (long)c * KK + t;
    *o = accumulate ? *o + s : s;
  }
}

static int dw_tiles(const yms_dw_shape* s, int& tx, int& ty) {
  tx = (s->w + DW_TX - 1) / DW_TX;
  ty = (s->h + DW_TY - 1) / DW_TY;
  return s->n * tx * ty;
}

static bool dw_shape_ok(const yms_dw_shape* s) {
  return s && s->n > 0 && s->h > 0 && s->w > 0 && s->c > 0 && s->c % 8 == 0 && (s->k == 3 || s->k == 5 || s->k == 7 || s->k == 9) &&
         s->dtype >= 0 && s->dtype <= 2 && (long)s->n * s->h * s->w < (1l << 31);
}
static bool dw_view_ok(int ld, int off, int c) { return ld % 8 == 0 && off % 8 == 0 && off + c <= ld; }

// spatial partitions of the wgrad grid: about 1024 blocks in total over the channel groups (two
// 512-thread blocks fit a CU), each walking several tiles so the ws rows stay few
static int dw_wgrad_blocks(const yms_dw_shape* s) {
  int tx, ty;
  const int t = dw_tiles(s, tx, ty);
  const int cg = (s->c + DW_CB - 1) / DW_CB;
  return std::max(1, std::min(t, std::max(1, 1024 / cg)));
}

#define YMS_DW_K(K, ...)                                        \
  switch (K) {                                                  \
    case 3: { constexpr int KK = 3; __VA_ARGS__; } break;       \
    case 5: { constexpr int KK = 5; __VA_ARGS__; } break;       \
    case 7: { constexpr int KK = 7; __VA_ARGS__; } break;       \
    default: { constexpr int KK = 9; __VA_ARGS__; } break;      \
  }
#define YMS_DW_T(dt, ...)                                       \
  do {                                                          \
    if ((dt) == YMS_BF16) { typedef bf16 TT; __VA_ARGS__; }     \
    else if ((dt) == YMS_F16) { typedef f16 TT; __VA_ARGS__; }  \
    else { typedef float TT; __VA_ARGS__; }                     \
  } while (0)

// y (+)= a + b over npix x c (b may be NULL): the MS-Block branch sum (X_i + Y_{i-1}) and, with
// b = NULL, its backward (each addend's gradient (+)= the sum's gradient)
template <typename T>
__global__ __launch_bounds__(256) void add_views_kernel(long items, int cg, const T* a, int a_ld, int a_off,
                                                        const T* b, int b_ld, int b_off, T* y, int y_ld, int y_off,
                                                        int accumulate) {
  for (long it = blockIdx.x * 256l + threadIdx.x; it < items; it += (long)gridDim.x * 256) {
    const long pix = it / cg;
    const int c = (int)(it - pix * cg) * 8;
    float va[8], vb[8], vy[8];
    Vec8<T>::load(a + pix * a_ld + a_off + c, va);
    if (b) Vec8<T>::load(b + pix * b_ld + b_off + c, vb);
    if (accumulate) Vec8<T>::load(y + pix * y_ld + y_off + c, vy);
#pragma unroll
    for (int k = 0; k < 8; ++k) va[k] = (b ? va[k] + vb[k] : va[k]) + (accumulate ? vy[k] : 0.0f);
    Vec8<T>::store(y + pix * y_ld + y_off + c, va);
  }
}

}  // namespace yms

using namespace yms;

extern "C" {

int yms_dwconv_stats_rows(const yms_dw_shape* s) {
  if (!dw_shape_ok(s)) return 0;
  int tx, ty;
  return dw_tiles(s, tx, ty);
}

yms_status yms_dwconv_fwd(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const float* w, void* y,
                          int y_ld, int y_off, const float* scale, const float* shift, int act, float* stats,
                          int stats_ld, void* stream) {
  if (!dw_shape_ok(s) || !x || !w || !y || !dw_view_ok(x_ld, x_off, s->c) || !dw_view_ok(y_ld, y_off, s->c))
    return YMS_ERR_INVALID;
  if (stats && stats_ld < s->c) return YMS_ERR_INVALID;
  DwParams p{};
  p.src = (const char*)x; p.src_ld = x_ld; p.src_off = x_off; p.w = w;
  p.dst = (char*)y; p.dst_ld = y_ld; p.dst_off = y_off;
  p.scale = scale; p.shift = shift; p.act = act; p.stats = stats; p.stats_ld = stats_ld;
  if (stats) p.stats_cnt = stats + (long)yms_dwconv_stats_rows(s) * 2 * stats_ld;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  const int tiles = dw_tiles(s, p.tiles_x, p.tiles_y);
  dim3 grid((unsigned)tiles, (unsigned)((s->c + DW_CB - 1) / DW_CB));
  hipStream_t st = (hipStream_t)stream;
  YMS_DW_T(s->dtype, YMS_DW_K(s->k, {
    if (stats) hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_FWD_STATS>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_FWD_AFFINE>), grid, dim3(256), 0, st, p);
  }));
  return launch_status();
}

yms_status yms_dwconv_dgrad(const yms_dw_shape* s, const void* dz, int dz_ld, int dz_off, const float* w, void* dx,
                            int dx_ld, int dx_off, int accumulate, void* stream) {
  if (!dw_shape_ok(s) || !dz || !w || !dx || !dw_view_ok(dz_ld, dz_off, s->c) || !dw_view_ok(dx_ld, dx_off, s->c))
    return YMS_ERR_INVALID;
  DwParams p{};
  p.src = (const char*)dz; p.src_ld = dz_ld; p.src_off = dz_off; p.w = w;
  p.dst = (char*)dx; p.dst_ld = dx_ld; p.dst_off = dx_off; p.accumulate = accumulate;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  const int tiles = dw_tiles(s, p.tiles_x, p.tiles_y);
  dim3 grid((unsigned)tiles, (unsigned)((s->c + DW_CB - 1) / DW_CB));
  hipStream_t st = (hipStream_t)stream;
  YMS_DW_T(s->dtype, YMS_DW_K(s->k, hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_DGRAD>), grid, dim3(256), 0, st, p)));
  return launch_status();
}

size_t yms_dwconv_wgrad_ws_bytes(const yms_dw_shape* s) {
  if (!dw_shape_ok(s)) return 0;
  return (size_t)dw_wgrad_blocks(s) * s->k * s->k * s->c * sizeof(float);
}

yms_status yms_dwconv_wgrad(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const void* dz, int dz_ld,
                            int dz_off, float* ws, size_t ws_bytes, float* dw, int accumulate, void* stream) {
  if (!dw_shape_ok(s) || !x || !dz || !ws || !dw || !dw_view_ok(x_ld, x_off, s->c) || !dw_view_ok(dz_ld, dz_off, s->c))
    return YMS_ERR_INVALID;
  if (ws_bytes < yms_dwconv_wgrad_ws_bytes(s)) return YMS_ERR_INVALID;
  DwParams p{};
  p.src = (const char*)x; p.src_ld = x_ld; p.src_off = x_off;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  dw_tiles(s, p.tiles_x, p.tiles_y);
  const int blocks = dw_wgrad_blocks(s);
  dim3 grid((unsigned)blocks, (unsigned)((s->c + DW_CB - 1) / DW_CB));
  hipStream_t st = (hipStream_t)stream;
  YMS_DW_T(s->dtype, YMS_DW_K(s->k, hipLaunchKernelGGL((dwconv_wgrad_kernel<TT, KK>), grid, dim3(DW_WG_NT), 0, st, p,
                                                      (const char*)dz, dz_ld, dz_off, ws)));
  yms_status e = launch_status();
  if (e != YMS_OK) return e;
  const int KK2 = s->k * s->k;
  hipLaunchKernelGGL(dwconv_wgrad_reduce_kernel, dim3((unsigned)((s->c * KK2 + 63) / 64)), dim3(256), 0, st, ws,
                     blocks, s->c, KK2, dw, accumulate);
  return launch_status();
}

yms_status yms_add_views(int dtype, long npix, int c, const void* a, int a_ld, int a_off, const void* b, int b_ld,
                         int b_off, void* y, int y_ld, int y_off, int accumulate, void* stream) {
  if (npix <= 0 || c <= 0 || c % 8 || !a || !y || !dw_view_ok(a_ld, a_off, c) || !dw_view_ok(y_ld, y_off, c))
    return YMS_ERR_INVALID;
  if (b && !dw_view_ok(b_ld, b_off, c)) return YMS_ERR_INVALID;
  const long items = npix * (c / 8);
  const unsigned grid = (unsigned)std::min<long>((items + 255) / 256, 16384);
  YMS_DW_T(dtype, hipLaunchKernelGGL(add_views_kernel<TT>, dim3(grid), dim3(256), 0, (hipStream_t)stream, items, c / 8,
                                     (const TT*)a, a_ld, a_off, (const TT*)b, b_ld, b_off, (TT*)y, y_ld, y_off,
                                     accumulate));
  return launch_status();
}

}  // extern "C"

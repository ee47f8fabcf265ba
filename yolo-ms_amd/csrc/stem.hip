// Stem convolution for gfx950: Conv2d(cin <= 3, cout, k=3, stride 2, pad 1) read straight from
// the model's NCHW fp32 input, the first layer of every YOLOv8 / YOLO-MS backbone
// (yolov8/model/yolov8_backbone.py:30-40, Conv(in_channels, int(64*w), 3, 2, 1) -> BN -> SiLU,
// components.py:69-77).
//
// The generic path packs the input to NHWC (8 channels, 5 of them zero padding) in one HBM pass
// and then runs the implicit-GEMM kernel on a K of 27 padded to two 64-wide k-tiles: about 3x the
// algorithmic bytes and half of every MFMA wasted.  Here one 256-thread block owns an 8 x 32 tile
// of output pixels and all output channels:
//   - the block's (2*8+1) x (2*32+1) x cin input footprint is read once from the NCHW planes
//     (coalesced rows of 65 floats, zero outside the image) into LDS as fp32;
//   - wave w builds the im2col A fragments of its two 32-pixel rows directly from LDS (K = 27 in
//     two 16-wide k-steps, k = ci*9 + kh*3 + kw, the nn.Conv2d weight order), rounding to the
//     compute dtype the way the packing kernel does (round-to-nearest-even);
//   - the B fragments come from the fp32 weight [cout][cin][3][3] itself (no packed copy),
//     rounded the same way; v_mfma_f32_32x32x16_{bf16,f16}, fp32 accumulation;
//   - epilogue: eval = folded BN scale/shift + SiLU, train = z plus one BN statistics row per
//     block (sum and centred M2 over the block's valid pixels, waves merged with Chan's update;
//     conv_common.hpp contract, counts after the rows), staged through LDS so every lane writes
//     whole 16-B NHWC chunks.
#include <algorithm>
#include <cstdlib>

#include "conv_common.hpp"

namespace yms {

constexpr int ST_TH = 8, ST_TW = 32;                    // output tile (rows x cols)
constexpr int ST_IH = 2 * ST_TH + 1;
// LDS footprint rows: input column 2*ox0 - 1 + c at index c + 3, so the 64 aligned columns
// 2*ox0 .. 2*ox0 + 63 start at a 16-B boundary (float4 loads and LDS stores)
constexpr int ST_IW = 2 * ST_TW + 4;
constexpr int ST_IN = 3 * ST_IH * ST_IW;                // fp32 input footprint, cin <= 3

struct StemParams {
  const float* x;        // [N][CI][H][W] fp32
  const float* w;        // [CO][CI][3][3] fp32
  char* y;
  int y_ld, y_off;
  const float* scale;
  const float* shift;
  int act;
  float* stats;
  int stats_ld;
  float* stats_cnt;
  int N, CI, H, W, CO, Ho, Wo, tiles_x, tiles_y;
  int vec4;              // W % 4 == 0 and 16-B aligned planes: float4 input loads
  int ysplit, tps;       // strips per image column of tiles, tiles per strip
};

template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const T ta = (T)a, tb = (T)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ta) | ((uint32_t)__builtin_bit_cast(uint16_t, tb) << 16);
}

// NT = 32-channel output tiles (cout <= 32 * NT), STATS = training epilogue.  A block walks a
// vertical strip of p.tps tiles (same columns, consecutive tile rows); the footprint of tile t + 1
// is loaded into registers while tile t computes and stores (software pipeline, one barrier
// pair per tile; the input and output LDS regions are disjoint).
template <typename T, int NT, bool STATS>
__global__ __launch_bounds__(256) void conv_stem_kernel(StemParams p) {
  constexpr int CP = NT * 32;                  // padded channels per pixel in the LDS out tile
  constexpr int OP = CP * (int)sizeof(T) + 16; // LDS out row pitch (bytes), 16-B skew per pixel
  constexpr int OUT_B = 4 * 64 * OP;
  constexpr int IN_B = ST_IN * 4;
  constexpr int RED_B = 4 * 3 * CP * 4;
  __shared__ __attribute__((aligned(16))) char smem[IN_B + OUT_B + RED_B];
  float* xin = reinterpret_cast<float*>(smem);
  float* red = reinterpret_cast<float*>(smem + IN_B + OUT_B);

  const int per_col = p.tiles_x * p.ysplit;
  const int n = blockIdx.x / per_col, rem = blockIdx.x - n * per_col;
  const int tx = rem % p.tiles_x, ty0 = (rem / p.tiles_x) * p.tps, ty1 = min(p.tiles_y, ty0 + p.tps);
  const int ox0 = tx * ST_TW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const float* xn = p.x + (long)n * p.CI * p.H * p.W;
  const int ix0 = 2 * ox0;

  // footprint of tile row ty: per row (ci, hy) 16 float4 of the aligned columns 2*ox0 .. +63
  constexpr int NV = 3 * ST_IH * 16, NVI = (NV + 255) / 256;
  f32x4 v[NVI];
  float hcol = 0.f;                              // left halo column 2*ox0 - 1 (threads < 3*ST_IH)
  auto load_tile = [&](int ty) {
    const int iy0 = 2 * ty * ST_TH - 1;
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int it = tid + 256 * j;
      const int row = it >> 4, q = it & 15;      // row = ci * ST_IH + hy
      const int ci = row / ST_IH, iy = iy0 + row - ci * ST_IH, ix = ix0 + 4 * q;
      v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (it < NV && ci < p.CI && iy >= 0 && iy < p.H) {
        const float* src = xn + ((long)ci * p.H + iy) * p.W + ix;
        if (p.vec4) {
          if (ix < p.W) v[j] = *reinterpret_cast<const f32x4*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[j][e] = ix + e < p.W ? src[e] : 0.f;
        }
      }
    }
    if (tid < 3 * ST_IH) {
      const int ci = tid / ST_IH, iy = iy0 + tid - ci * ST_IH;
      hcol = (ci < p.CI && iy >= 0 && iy < p.H && ix0 >= 1) ? xn[((long)ci * p.H + iy) * p.W + ix0 - 1] : 0.f;
    }
  };

  // weight fragments: lane holds B[k = 16 s + 8 lh + j][co = 32 b + lr]
  const int K = p.CI * 9;
  u32x4 bfr[NT][2];
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int co = 32 * b + lr;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float wv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * lh + j;
        wv[j] = (co < p.CO && k < K) ? p.w[(long)co * K + k] : 0.0f;
      }
      bfr[b][s] = u32x4{pack2<T>(wv[0], wv[1]), pack2<T>(wv[2], wv[3]), pack2<T>(wv[4], wv[5]),
                        pack2<T>(wv[6], wv[7])};
    }
  }
  // im2col LDS offsets of this lane's 16 k values (k = ci*9 + kh*3 + kw; -1 = zero pad)
  int koff[2][8];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * lh + j;
      const int ci = k / 9, t = k - ci * 9, kh = t / 3, kw = t - kh * 3;
      koff[s][j] = k < K ? (ci * ST_IH + kh) * ST_IW + kw + 3 : -1;
    }
  float sc[NT], sh[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int co = 32 * b + lr;
    sc[b] = (!STATS && co < p.CO && p.scale) ? p.scale[co] : 1.0f;
    sh[b] = (!STATS && co < p.CO && p.shift) ? p.shift[co] : 0.0f;
  }
  auto prow = [&](int i) { return (i & 3) + 8 * (i >> 2) + 4 * lh; };
  const int vx = min(ST_TW, p.Wo - ox0);         // valid columns of the strip's tiles
  const int cch = p.CO / 8;
  T* y = reinterpret_cast<T*>(p.y);
  char* ot = smem + IN_B + wave * 64 * OP;

  load_tile(ty0);
  for (int ty = ty0; ty < ty1; ++ty) {
    const int oy0 = ty * ST_TH;
    // (a) registers -> LDS footprint (the previous tile's reads of xin ended before its barrier B2)
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int it = tid + 256 * j;
      if (it < NV) *reinterpret_cast<f32x4*>(xin + (it >> 4) * ST_IW + 4 + 4 * (it & 15)) = v[j];
    }
    if (tid < 3 * ST_IH) xin[tid * ST_IW + 3] = hcol;
    __syncthreads();                                                   // B1
    if (ty + 1 < ty1) load_tile(ty + 1);                               // in flight during (b)-(e)
    // (b) two 32-pixel rows per wave: output row oy0 + 2 wave + a, pixel lr of the row
    f32x16 acc[2][NT];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int b = 0; b < NT; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;
      const int base = 2 * (2 * wave + a) * ST_IW + 2 * lr;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float av[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = koff[s][j] >= 0 ? xin[base + koff[s][j]] : 0.0f;
        const u32x4 af = u32x4{pack2<T>(av[0], av[1]), pack2<T>(av[2], av[3]), pack2<T>(av[4], av[5]),
                               pack2<T>(av[6], av[7])};
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = Mfma<T>::mma(af, bfr[b][s], acc[a][b]);
      }
    }
    bool rowok[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) rowok[a] = oy0 + 2 * wave + a < p.Ho;
    // (c) statistics: per-wave moments of each channel over its valid pixels
    if constexpr (STATS) {
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        float s = 0.f, cntv = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (rowok[a] && prow(i) < vx) { s += acc[a][b][i]; cntv += 1.f; }
        s += __shfl_xor(s, 32);
        cntv += __shfl_xor(cntv, 32);
        const float mu = cntv > 0.f ? s / cntv : 0.f;
        float q = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (rowok[a] && prow(i) < vx) {
              const float d = acc[a][b][i] - mu;
              q += d * d;
            }
        q += __shfl_xor(q, 32);
        if (lh == 0) {
          red[(wave * 3 + 0) * CP + 32 * b + lr] = cntv;
          red[(wave * 3 + 1) * CP + 32 * b + lr] = s;
          red[(wave * 3 + 2) * CP + 32 * b + lr] = q;
        }
      }
    }
    // (d) epilogue values -> the wave's LDS out tile [64 pixels][CP channels] in T (the wave's
    //     own region: its previous global stores read it before B1)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int co = 32 * b + lr;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float val = acc[a][b][i];
          if (!STATS) {
            val = val * sc[b] + sh[b];
            if (p.act == YMS_ACT_SILU) val = silu_f(val);
          }
          *reinterpret_cast<T*>(ot + (a * 32 + prow(i)) * OP + co * (int)sizeof(T)) = (T)val;
        }
    }
    __syncthreads();                                                   // B2
    // (e) Chan's merge of the four waves -> the tile's statistics row; out tile -> NHWC
    if constexpr (STATS) {
      const int tile = (n * p.tiles_y + ty) * p.tiles_x + tx;
      if (tid < p.CO) {
        float nt = 0.f, st = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) { nt += red[(w * 3 + 0) * CP + tid]; st += red[(w * 3 + 1) * CP + tid]; }
        const float mean = nt > 0.f ? st / nt : 0.f;
        float m2 = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float nw = red[(w * 3 + 0) * CP + tid];
          if (nw > 0.f) {
            const float d = red[(w * 3 + 1) * CP + tid] / nw - mean;
            m2 += red[(w * 3 + 2) * CP + tid] + nw * d * d;
          }
        }
        float* so = p.stats + (long)tile * 2 * p.stats_ld;
        so[tid] = st;
        so[p.stats_ld + tid] = m2;
        if (tid == 0) p.stats_cnt[tile] = nt;
      }
    }
    for (int it = lane; it < 64 * cch; it += 64) {
      const int px = it / cch, ch = it - px * cch;
      const int a = px >> 5, ox = ox0 + (px & 31), oy = oy0 + 2 * wave + a;
      if (oy < p.Ho && ox < p.Wo) {
        const u32x4 val = *reinterpret_cast<const u32x4*>(ot + px * OP + ch * 16);
        *reinterpret_cast<u32x4*>(y + (((long)n * p.Ho + oy) * p.Wo + ox) * p.y_ld + p.y_off + 8 * ch) = val;
      }
    }
  }
}

static bool stem_shape_ok(const yms_conv_shape* s) {
  return s && s->n > 0 && s->h > 0 && s->w > 0 && s->cin >= 1 && s->cin <= 3 && s->cout >= 8 && s->cout % 8 == 0 &&
         s->cout <= 96 && s->k == 3 && s->stride == 2 && s->pad == 1 && s->ho == (s->h - 1) / 2 + 1 &&
         s->wo == (s->w - 1) / 2 + 1 && (s->dtype == YMS_BF16 || s->dtype == YMS_F16);
}

static int stem_tiles(const yms_conv_shape* s, int& tx, int& ty) {
  tx = (s->wo + ST_TW - 1) / ST_TW;
  ty = (s->ho + ST_TH - 1) / ST_TH;
  return s->n * tx * ty;
}

}  // namespace yms

using namespace yms;

extern "C" {

int yms_conv_stem_supported(const yms_conv_shape* s) { return stem_shape_ok(s) ? 1 : 0; }

int yms_conv_stem_stats_rows(const yms_conv_shape* s) {
  if (!stem_shape_ok(s)) return 0;
  int tx, ty;
  return stem_tiles(s, tx, ty);
}

yms_status yms_conv_stem_fwd(const yms_conv_shape* s, const float* x, const float* w, void* y, int y_ld, int y_off,
                             const float* scale, const float* shift, int act, float* stats, int stats_ld,
                             void* stream) {
  if (!s || !x || !w || !y) return YMS_ERR_INVALID;
  if (!stem_shape_ok(s)) return YMS_ERR_UNSUPPORTED;
  if (y_ld % 8 || y_off % 8 || y_off + s->cout > y_ld) return YMS_ERR_INVALID;
  if (stats && stats_ld < s->cout) return YMS_ERR_INVALID;
  if ((long)s->n * s->cin * s->h * s->w >= (1l << 31)) return YMS_ERR_UNSUPPORTED;
  StemParams p{};
  p.x = x; p.w = w; p.y = (char*)y; p.y_ld = y_ld; p.y_off = y_off;
  p.scale = scale; p.shift = shift; p.act = act;
  p.stats = stats; p.stats_ld = stats_ld;
  p.N = s->n; p.CI = s->cin; p.H = s->h; p.W = s->w; p.CO = s->cout; p.Ho = s->ho; p.Wo = s->wo;
  const int tiles = stem_tiles(s, p.tiles_x, p.tiles_y);
  p.vec4 = (s->w % 4 == 0 && ((uintptr_t)x & 15) == 0) ? 1 : 0;
  if (stats) p.stats_cnt = stats + (long)tiles * 2 * stats_ld;
  // strips of tps tiles: about 1024 blocks (4 per CU), so each block pipelines several tiles
  static const long target = getenv("YMS_STEM_BLOCKS") ? std::max(1, atoi(getenv("YMS_STEM_BLOCKS"))) : 1024;
  const long cols = (long)s->n * p.tiles_x;
  const int want = (int)std::max(1l, std::min<long>(p.tiles_y, (target + cols - 1) / cols));
  p.tps = (p.tiles_y + want - 1) / want;
  p.ysplit = (p.tiles_y + p.tps - 1) / p.tps;
  const unsigned blocks = (unsigned)(cols * p.ysplit);
  hipStream_t st = (hipStream_t)stream;
  const int nt = (s->cout + 31) / 32;
#define YMS_STEM(TT)                                                                                         \
  do {                                                                                                       \
    if (stats) {                                                                                             \
      if (nt == 1) hipLaunchKernelGGL((conv_stem_kernel<TT, 1, true>), dim3(blocks), dim3(256), 0, st, p);    \
      else if (nt == 2) hipLaunchKernelGGL((conv_stem_kernel<TT, 2, true>), dim3(blocks), dim3(256), 0, st, p); \
      else hipLaunchKernelGGL((conv_stem_kernel<TT, 3, true>), dim3(blocks), dim3(256), 0, st, p);            \
    } else {                                                                                                 \
      if (nt == 1) hipLaunchKernelGGL((conv_stem_kernel<TT, 1, false>), dim3(blocks), dim3(256), 0, st, p);   \
      else if (nt == 2) hipLaunchKernelGGL((conv_stem_kernel<TT, 2, false>), dim3(blocks), dim3(256), 0, st, p); \
      else hipLaunchKernelGGL((conv_stem_kernel<TT, 3, false>), dim3(blocks), dim3(256), 0, st, p);           \
    }                                                                                                        \
  } while (0)
  if (s->dtype == YMS_BF16) YMS_STEM(bf16);
  else YMS_STEM(f16);
#undef YMS_STEM
  return launch_status();
}

}  // extern "C"

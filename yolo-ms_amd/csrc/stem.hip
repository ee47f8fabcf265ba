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

// ------------------------------------------------------------------------------------------
// Stem weight gradient with the BN + SiLU backward apply fused into its operand loads:
//   dz = scale * (da - k0 - (z - mean) * invstd * k1),  da = gy * SiLU'(z * scale + shift)
//   dW[co][k] = sum_pixels dz[pixel][co] * im2col(x)[pixel][k]     (k = ci*9 + kh*3 + kw)
// The stem's input never needs a gradient, so its dz has no other consumer: the generic path's
// full-tensor apply pass (read gy, z; write dz) and the NHWC input pack disappear; dz is rounded
// to the compute dtype as the apply pass would store it.  Per tile (8 x 32 output pixels): dz
// goes to LDS transposed ([channel][pixel]), the fp32 input footprint as in the forward; wave w
// owns pixel rows 2w, 2w+1: A = dz^T (32 channels x 16 pixels per k-step), B = im2col (16 pixels
// x 32 taps), accumulated over the block's whole strip; the 4 waves' tiles are summed in LDS
// into one partial [cout][27] row per block, reduced in a fixed order by stem_wgrad_reduce.
template <typename T, int NT>
__global__ __launch_bounds__(256) void conv_stem_wgrad_kernel(StemParams p, const T* gy, int gy_ld, int gy_off,
                                                              const T* z, int z_ld, int z_off, const float* mi,
                                                              const float* coef, float* ws) {
  constexpr int CP = NT * 32;
  constexpr int DP = 256 + 8;                       // dz^T row pitch (elements): 16-B aligned, skewed
  constexpr int IN_B = ST_IN * 4;
  constexpr int DZ_B = CP * DP * (int)sizeof(T);
  constexpr int RED_B = 4 * CP * 32 * 4;
  constexpr int MAIN_B = (IN_B + DZ_B) > RED_B ? (IN_B + DZ_B) : RED_B;
  __shared__ __attribute__((aligned(16))) char smem[MAIN_B + 4 * CP * 4];
  float* xin = reinterpret_cast<float*>(smem);
  T* dzt = reinterpret_cast<T*>(smem + IN_B);
  float* red = reinterpret_cast<float*>(smem);
  float (*prm)[CP] = reinterpret_cast<float (*)[CP]>(smem + MAIN_B);   // scale, shift, a0, bz per channel

  const int per_col = p.tiles_x * p.ysplit;
  const int n = blockIdx.x / per_col, rem = blockIdx.x - n * per_col;
  const int tx = rem % p.tiles_x, ty0 = (rem / p.tiles_x) * p.tps, ty1 = min(p.tiles_y, ty0 + p.tps);
  const int ox0 = tx * ST_TW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const float* xn = p.x + (long)n * p.CI * p.H * p.W;
  const int ix0 = 2 * ox0, K = p.CI * 9, cch = p.CO / 8;

  // dz items: (pixel pair, 8-channel group), tid, tid + 256, ...: two adjacent pixels of one row
  constexpr int NPAIR = 128 * CP / 8, NDZ = (NPAIR + 255) / 256;
  // per-channel apply coefficients: dz = scale * da + a0 + bz * z (bn_bwd_apply_kernel's form)
  for (int c = tid; c < CP; c += 256) {
    float sc = 0.f, sh = 0.f, a0 = 0.f, bz = 0.f;
    if (c < p.CO) {
      sc = p.scale[c];
      sh = p.shift[c];
      const float mu = mi[c], is = mi[p.CO + c];
      bz = -sc * coef[p.CO + c] * is;
      a0 = -sc * coef[c] - bz * mu;
    }
    prm[0][c] = sc; prm[1][c] = sh; prm[2][c] = a0; prm[3][c] = bz;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[b][i] = 0.0f;
  // this lane's B column: tap k = lr (zero past K)
  const int kk = lr;
  const int kci = kk / 9, kt = kk - kci * 9, kkh = kt / 3, kkw = kt - kkh * 3;
  const bool kok = kk < K;

  // registers of the tile in flight: input footprint rows, left halo column, raw gy / z chunks
  constexpr int NV = 3 * ST_IH * 16, NVI = (NV + 255) / 256;
  f32x4 xv[NVI];
  float hcol = 0.f;
  Raw8<T> graw[NDZ][2], zraw[NDZ][2];
  auto load_tile = [&](int ty) {
    const int oy0 = ty * ST_TH, iy0 = 2 * oy0 - 1;
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int it = tid + 256 * j;
      const int row = it >> 4, q = it & 15;
      const int ci = row / ST_IH, iy = iy0 + row - ci * ST_IH, ix = ix0 + 4 * q;
      xv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (it < NV && ci < p.CI && iy >= 0 && iy < p.H) {
        const float* src = xn + ((long)ci * p.H + iy) * p.W + ix;
        if (p.vec4) {
          if (ix < p.W) xv[j] = *reinterpret_cast<const f32x4*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[j][e] = ix + e < p.W ? src[e] : 0.f;
        }
      }
    }
    if (tid < 3 * ST_IH) {
      const int ci = tid / ST_IH, iy = iy0 + tid - ci * ST_IH;
      hcol = (ci < p.CI && iy >= 0 && iy < p.H && ix0 >= 1) ? xn[((long)ci * p.H + iy) * p.W + ix0 - 1] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NDZ; ++j) {
      const int it = tid + 256 * j;
      const int pp = it / (CP / 8), g = it - pp * (CP / 8);
      const int oy = oy0 + (pp >> 4), c0 = 8 * g;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ox = ox0 + 2 * (pp & 15) + h;
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 2); ++k) { graw[j][h].v[k] = u32x4{0u, 0u, 0u, 0u}; zraw[j][h].v[k] = graw[j][h].v[k]; }
        if (it < NPAIR && g < cch && oy < p.Ho && ox < p.Wo) {
          const long pix = ((long)n * p.Ho + oy) * p.Wo + ox;
          load_raw8(gy + pix * gy_ld + gy_off + c0, 8, graw[j][h]);
          load_raw8(z + pix * z_ld + z_off + c0, 8, zraw[j][h]);
        }
      }
    }
  };

  load_tile(ty0);
  for (int ty = ty0; ty < ty1; ++ty) {
    __syncthreads();                                   // previous tile's LDS reads are done
    // (a) footprint registers -> LDS
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int it = tid + 256 * j;
      if (it < NV) *reinterpret_cast<f32x4*>(xin + (it >> 4) * ST_IW + 4 + 4 * (it & 15)) = xv[j];
    }
    if (tid < 3 * ST_IH) xin[tid * ST_IW + 3] = hcol;
    // (b) dz = BN+SiLU backward of (gy, z), dtype-rounded, two pixels per 32-bit LDS store into
    //     the transposed tile [channel][pixel] (invalid pixels / padded channels are zeros)
#pragma unroll
    for (int j = 0; j < NDZ; ++j) {
      const int it = tid + 256 * j;
      if (it < NPAIR) {
        const int pp = it / (CP / 8), g = it - pp * (CP / 8), c0 = 8 * g;
        const int oy = ty * ST_TH + (pp >> 4);
        float o[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bool valid = g < cch && oy < p.Ho && ox0 + 2 * (pp & 15) + h < p.Wo;
          float gv[8], zv[8];
          unpack8(graw[j][h], gv);
          unpack8(zraw[j][h], zv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int c = c0 + e;
            const float sc = prm[0][c], sh = prm[1][c], a0 = prm[2][c], bz = prm[3][c];
            float da = gv[e];
            if (p.act == YMS_ACT_SILU) da *= dsilu_f(zv[e] * sc + sh);
            o[h][e] = valid ? sc * da + a0 + bz * zv[e] : 0.f;   // no pixel / channel: no dz
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          *reinterpret_cast<uint32_t*>(dzt + (c0 + e) * DP + 2 * pp) = pack2<T>(o[0][e], o[1][e]);
      }
    }
    __syncthreads();
    if (ty + 1 < ty1) load_tile(ty + 1);               // in flight during the MFMAs
    // (c) MFMAs: wave w, pixel rows a = 0, 1 (pixels 64 w + 32 a + 0..31), 2 k-steps of 16 pixels
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int prow = 2 * wave + a;                   // tile row of these 32 pixels
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int p0 = 16 * s2 + 8 * lh;               // pixel column of element j = 0
        float bv[8];
        const int base = (kci * ST_IH + 2 * prow + kkh) * ST_IW + kkw + 3 + 2 * p0;
#pragma unroll
        for (int j = 0; j < 8; ++j) bv[j] = kok ? xin[base + 2 * j] : 0.f;
        const u32x4 bf = u32x4{pack2<T>(bv[0], bv[1]), pack2<T>(bv[2], bv[3]), pack2<T>(bv[4], bv[5]),
                               pack2<T>(bv[6], bv[7])};
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const u32x4 af = *reinterpret_cast<const u32x4*>(dzt + (32 * b + lr) * DP + 64 * wave + 32 * a + p0);
          acc[b] = Mfma<T>::mma(af, bf, acc[b]);
        }
      }
    }
  }
  // (d) sum the 4 waves' [co][k] tiles in LDS (fixed order), one partial row per block
  __syncthreads();
#pragma unroll
  for (int b = 0; b < NT; ++b)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = 32 * b + (i & 3) + 8 * (i >> 2) + 4 * lh;
      red[(wave * CP + co) * 32 + lr] = acc[b][i];
    }
  __syncthreads();
  for (int it = tid; it < p.CO * K; it += 256) {
    const int co = it / K, k = it - co * K;
    const float v = ((red[(0 * CP + co) * 32 + k] + red[(1 * CP + co) * 32 + k]) + red[(2 * CP + co) * 32 + k]) +
                    red[(3 * CP + co) * 32 + k];
    ws[(long)blockIdx.x * p.CO * K + it] = v;
  }
}

// dw[co][k] (+)= sum_b ws[b][co][k] in a fixed order: 64 outputs per block, 16 waves; wave w sums
// rows w, w + 16, ... into 4 independent partials (4 loads in flight per lane: the row count is
// ~1000, a single dependent chain per lane made this reduce latency-bound), then a fixed-order
// tree over the waves
__global__ __launch_bounds__(1024) void stem_wgrad_reduce_kernel(const float* ws, int blocks, int items, float* dw,
                                                                 int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < items) {
    int b = w;
    for (; b + 48 < blocks; b += 64) {
      s0 += ws[(long)b * items + j];
      s1 += ws[(long)(b + 16) * items + j];
      s2 += ws[(long)(b + 32) * items + j];
      s3 += ws[(long)(b + 48) * items + j];
    }
    for (; b < blocks; b += 16) s0 += ws[(long)b * items + j];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int h = 8; h >= 1; h >>= 1) {
    if (w < h) red[w][lane] += red[w + h][lane];
    __syncthreads();
  }
  if (w == 0 && j < items) dw[j] = accumulate ? dw[j] + red[0][lane] : red[0][lane];
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

// strips of tps tiles: about `target` blocks, so each block walks several tiles
static unsigned stem_strips(const yms_conv_shape* s, StemParams& p, long target) {
  const long cols = (long)s->n * p.tiles_x;
  const int want = (int)std::max(1l, std::min<long>(p.tiles_y, (target + cols - 1) / cols));
  p.tps = (p.tiles_y + want - 1) / want;
  p.ysplit = (p.tiles_y + p.tps - 1) / p.tps;
  return (unsigned)(cols * p.ysplit);
}

constexpr long STEM_WG_BLOCKS = 1024;

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
  const unsigned blocks = stem_strips(s, p, 1024);
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

size_t yms_conv_stem_wgrad_ws_bytes(const yms_conv_shape* s) {
  if (!stem_shape_ok(s)) return 0;
  StemParams p{};
  stem_tiles(s, p.tiles_x, p.tiles_y);
  return (size_t)stem_strips(s, p, STEM_WG_BLOCKS) * s->cout * s->cin * 9 * sizeof(float);
}

yms_status yms_conv_stem_wgrad(const yms_conv_shape* s, const float* x, const void* gy, int gy_ld, int gy_off,
                               const void* z, int z_ld, int z_off, const float* scale, const float* shift,
                               const float* mean_invstd, const float* coef, int act, float* ws, size_t ws_bytes,
                               float* dw, int accumulate, void* stream) {
  if (!s || !x || !gy || !z || !scale || !shift || !mean_invstd || !coef || !ws || !dw) return YMS_ERR_INVALID;
  if (!stem_shape_ok(s)) return YMS_ERR_UNSUPPORTED;
  if (gy_ld % 8 || gy_off % 8 || gy_off + s->cout > gy_ld || z_ld % 8 || z_off % 8 || z_off + s->cout > z_ld)
    return YMS_ERR_INVALID;
  if (ws_bytes < yms_conv_stem_wgrad_ws_bytes(s)) return YMS_ERR_INVALID;
  if ((long)s->n * s->cin * s->h * s->w >= (1l << 31)) return YMS_ERR_UNSUPPORTED;
  StemParams p{};
  p.x = x; p.scale = scale; p.shift = shift; p.act = act;
  p.N = s->n; p.CI = s->cin; p.H = s->h; p.W = s->w; p.CO = s->cout; p.Ho = s->ho; p.Wo = s->wo;
  stem_tiles(s, p.tiles_x, p.tiles_y);
  p.vec4 = (s->w % 4 == 0 && ((uintptr_t)x & 15) == 0) ? 1 : 0;
  const unsigned blocks = stem_strips(s, p, STEM_WG_BLOCKS);
  hipStream_t st = (hipStream_t)stream;
  const int nt = (s->cout + 31) / 32;
#define YMS_STEM_WG(TT)                                                                                        \
  do {                                                                                                         \
    const TT* g_ = (const TT*)gy; const TT* z_ = (const TT*)z;                                                 \
    if (nt == 1) hipLaunchKernelGGL((conv_stem_wgrad_kernel<TT, 1>), dim3(blocks), dim3(256), 0, st, p, g_, gy_ld, \
                                    gy_off, z_, z_ld, z_off, mean_invstd, coef, ws);                          \
    else if (nt == 2) hipLaunchKernelGGL((conv_stem_wgrad_kernel<TT, 2>), dim3(blocks), dim3(256), 0, st, p, g_, \
                                         gy_ld, gy_off, z_, z_ld, z_off, mean_invstd, coef, ws);              \
    else hipLaunchKernelGGL((conv_stem_wgrad_kernel<TT, 3>), dim3(blocks), dim3(256), 0, st, p, g_, gy_ld,    \
                            gy_off, z_, z_ld, z_off, mean_invstd, coef, ws);                                  \
  } while (0)
  if (s->dtype == YMS_BF16) YMS_STEM_WG(bf16);
  else YMS_STEM_WG(f16);
#undef YMS_STEM_WG
  yms_status e = launch_status();
  if (e != YMS_OK) return e;
  const int items = s->cout * s->cin * 9;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((items + 63) / 64), dim3(1024), 0, st, ws, (int)blocks, items, dw,
                     accumulate);
  return launch_status();
}

}  // extern "C"

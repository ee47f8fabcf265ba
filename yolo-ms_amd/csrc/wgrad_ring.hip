// Weight gradient of a k x k convolution (1x1 / 3x3, any stride) as a TT GEMM over pixels on
// MFMA, with BOTH operands streamed global -> LDS by raw-buffer LDS-DMA into an ST-deep ring.
//
//   dW[co][tap * cin8 + ci] = sum_p dz[p][co] * x[src(p, tap)][ci]    (components.py:72 backward)
//
// The register-staged TT kernel (conv_igemm.hip, conv_wgrad_kernel) keeps one 32-pixel k-tile
// per block in flight and round-trips it through VGPRs; it measured 0.08 of the bf16 MFMA peak
// inside the training step.  Here:
//   * a block owns a BM (output channels) x BN (im2col columns) tile and a contiguous pixel range
//     (split-K); k-tiles of KP pixels go to LDS as 128-B rows: column block cb (64 columns) of
//     pixel row r lives at cb * KP * 128 + r * 128, with its 16-B chunk c stored at c ^ 4((r>>1)&1)
//     (the two rows k and k + 2 that one transposed read pairs would otherwise share banks);
//   * 8 waves; wave w issues the wave-instructions of pixel rows 8 (w % (KP/8)) .. + 7 for every
//     column block it covers, so ONE pixel decomposition per lane per k-tile serves its dz and
//     im2col loads; out-of-image / out-of-range / past-the-end lanes get voffset = NT_OOB and the
//     hardware writes zeros (no exec-masked branches);
//   * the MFMA operands are read with ds_read_b64_tr_b16 (8 consecutive pixels along K per lane),
//     v_mfma_f32_32x32x16_{bf16,f16}; the wait for k-tile g is a counted vmcnt that leaves ST-2
//     later k-tiles in flight across a raw s_barrier (conv_common.hpp);
//   * blocks of one pixel split are consecutive logical ids (XCD-remapped: they share dz rows and
//     im2col pixels in one L2) and write one fp32 partial slab each, summed in a fixed order by
//     wgrad_reduce_kernel (deterministic).
#include "conv_common.hpp"
#include "wgrad_ring.hpp"

#include <algorithm>
#include <cstdlib>

namespace yms {

struct WRParams {
  const char* x;
  const char* dz;
  float* slab;
  int x_ld, x_off, dz_ld, dz_off;   // elements
  uint32_t x_bytes, dz_bytes;       // raw-buffer extents (< 2^31)
  int SH, SW, stride, pad;
  int cout8, cpt, Kc, M, nkt, kt_per_split;
  int tiles_n, tiles_mn, slab_rows, slab_ld;
  FastDiv div_ow, div_ohw;
};

template <typename T, int KS, int BM, int BN, int KP, int ST, int OCC>
__global__ __launch_bounds__(512, OCC) void conv_wgrad_ring_kernel(WRParams p) {
  constexpr int NW = 8;
  constexpr int WGN = BN / 32 < 4 ? BN / 32 : 4, WGM = NW / WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int ES = (int)sizeof(T);
  constexpr int RG = KP / 8;                                   // 8-row groups per column block
  constexpr int A_INS = (BM / 64) * RG, B_INS = (BN / 64) * RG; // 1-KB wave-instructions per k-tile
  constexpr int A_PW = A_INS / NW, B_PW = B_INS / NW;
  constexpr int A_BYTES = BM * KP * 2, STAGE = (BM + BN) * KP * 2;
  constexpr int NG = A_PW + B_PW;
  static_assert(ES == 2 && TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wgrad ring tile");
  static_assert(A_INS % NW == 0 && B_INS % NW == 0 && (RG % NW == 0 || NW % RG == 0), "wgrad ring loads");
  __shared__ __attribute__((aligned(1024))) char smem[ST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WGN, wn = wv % WGN;
  const int tmn = p.tiles_mn;
  const int lid = tmn >= 4 ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int wg = lid % tmn;
  const int tile_n = wg % p.tiles_n, tile_m = wg / p.tiles_n;
  const int split = lid / tmn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(p.nkt, kt0 + p.kt_per_split);
  const int total = kt1 - kt0;

  const __amdgpu_buffer_rsrc_t rs_a =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dz, (short)0, (int)p.dz_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_b =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, NT_RSRC3);

  // ---- loader geometry (fixed per lane) ----
  const int prow = 8 * (wv % RG) + (lane >> 3);                // pixel row within the k-tile
  const int lc = (lane & 7) ^ (((lane >> 4) & 1) << 2);        // logical chunk of this lane's LDS slot
  const uint32_t dz_row = (uint32_t)(p.dz_ld * ES);
  uint32_t a_col[A_PW];                                        // byte offset within a dz row, or NT_OOB
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int cb = (wv + NW * j) / RG;
    const int ch = m0 + cb * 64 + lc * 8;
    a_col[j] = ch < p.cout8 ? (uint32_t)((p.dz_off + ch) * ES) : NT_OOB;
  }
  int b_kh[B_PW], b_kw[B_PW], b_cc[B_PW];
  bool b_ok[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int cb = (wv + NW * j) / RG;
    const int kc = n0 / 8 + cb * 8 + lc;
    b_ok[j] = kc < p.Kc;
    const int t = kc / p.cpt;
    b_cc[j] = (kc - t * p.cpt) * 16;
    b_kh[j] = t / KS;
    b_kw[j] = t - b_kh[j] * KS;
  }
  auto issue = [&](int stage, int kt) {
    char* sa = smem + stage * STAGE;
    char* sb = sa + A_BYTES;
    const int q = kt * KP + prow;
    const bool qok = q < p.M;
    const uint32_t mm = qok ? (uint32_t)q : 0u;
    const uint32_t n = fdiv(mm, p.div_ohw);
    const uint32_t rem = mm - n * p.div_ohw.d;
    const uint32_t oy = fdiv(rem, p.div_ow);
    const uint32_t ox = rem - oy * p.div_ow.d;
#pragma unroll
    for (int j = 0; j < A_PW; ++j) {
      const uint32_t vo = (qok && a_col[j] != NT_OOB) ? mm * dz_row + a_col[j] : NT_OOB;
      blds16(rs_a, sa + (wv + NW * j) * 1024, vo);
    }
    const int y0 = (int)oy * p.stride - p.pad, x0 = (int)ox * p.stride - p.pad;
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int iy = y0 + b_kh[j], ix = x0 + b_kw[j];
      const bool ok = qok && b_ok[j] && iy >= 0 && iy < p.SH && ix >= 0 && ix < p.SW;
      const uint32_t e = (uint32_t)((((int)n * p.SH + iy) * p.SW + ix) * p.x_ld + p.x_off);
      blds16(rs_b, sb + (wv + NW * j) * 1024, ok ? e * ES + (uint32_t)b_cc[j] : NT_OOB);
    }
  };

  // ---- compute geometry: transposed reads of pixel rows 16 s + 8 th + qq (+4) ----
  const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
  const int th = g >> 1, tcb = 16 * (g & 1);
  const int lr = lane & 31, lh = lane >> 5;
  const int swz = ((qq >> 1) & 1) << 2;                        // same for rows k and k + 4
  auto col_off = [&](int col) {                                // byte offset of logical column col
    return (col >> 6) * (KP * 128) + ((((col & 63) >> 3) ^ swz) << 4) + ((col >> 2) & 1) * 8;
  };
  int a_in[TM], b_in[TN];
#pragma unroll
  for (int a = 0; a < TM; ++a) a_in[a] = col_off(wm * WTM + a * 32 + tcb + 4 * pp) + (8 * th + qq) * 128;
#pragma unroll
  for (int b = 0; b < TN; ++b) b_in[b] = col_off(wn * WTN + b * 32 + tcb + 4 * pp) + (8 * th + qq) * 128;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  auto compute = [&](int stage) {
    const char* A = smem + stage * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int s = 0; s < KP / 16; ++s) {
      u32x4 af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const char* pa = A + a_in[a] + s * 16 * 128;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)pa);
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(pa + 4 * 128));
        const uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
        af[a] = u32x4{u0.x, u0.y, u1.x, u1.y};
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const char* pb = B + b_in[b] + s * 16 * 128;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)pb);
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(pb + 4 * 128));
        const uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
        bfr[b] = u32x4{u0.x, u0.y, u1.x, u1.y};
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = Mfma<T>::mma(af[a], bfr[b], acc[a][b]);
    }
  };

  // ---- ring: k-tile g lands, k-tile g + ST - 1 issues into the stage g - 1 left, g computes ----
#pragma unroll
  for (int s0 = 0; s0 < ST - 1; ++s0)
    if (s0 < total) issue(s0, kt0 + s0);
  int stage = 0;
  for (int gg = 0; gg < total; ++gg) {
    wait_tiles<NG, ST - 2>(total - 1 - gg);
    raw_barrier();
    if (gg + ST - 1 < total) {
      int ns = stage + ST - 1;
      if (ns >= ST) ns -= ST;
      issue(ns, kt0 + gg + ST - 1);
    }
    compute(stage);
    if (++stage == ST) stage = 0;
  }

  // ---- partial slab: rows co, columns tap * cin8 + ci ----
  float* slab = p.slab + (long)split * p.slab_rows * p.slab_ld;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        const int col = n0 + wn * WTN + b * 32 + lr;
        slab[(long)row * p.slab_ld + col] = acc[a][b][i];
      }
}

static int env_int_wr(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// 64-pixel k-tiles, 2 stages, 2 blocks per CU (round 4, measured and dropped: 32-pixel k-tiles with
// 2 / 4 stages, 3 stages at 1 block per CU, and the 64 x 64 GEMMs on zero-filled 64 x 128 tiles)
bool wgrad_ring_plan(const yms_conv_shape* s, WRPlan* w) {
  const int on = env_int_wr("YMS_WG_RING", 1);   // read per call: tests switch it at run time
  if (!on || s->dtype == YMS_F32 || (s->k != 1 && s->k != 3)) return false;
  WRPlan q{};
  q.cin8 = (int)rup(s->cin, 8);
  q.cpt = q.cin8 / 8;
  const int kf = s->k * s->k * q.cin8;
  q.kc = kf / 8;
  // 64-row tiles for <= 64 output channels; <= 32 channels and 64-column-only GEMMs stay on the
  // register-staged kernel (its 32-row / 64-column tiles) unless YMS_WG_RING=2
  q.bm = s->cout <= 64 ? 64 : 128;
  q.bn = kf <= 64 ? 64 : 128;
  if (q.bm == 64 && q.bn == 64) return false;
  if (on != 2 && s->cout <= 32) return false;
  q.kp = 64;
  q.tiles_m = cdiv(s->cout, q.bm);
  q.tiles_n = cdiv(kf, q.bn);
  q.slab_rows = q.tiles_m * q.bm;
  q.slab_ld = q.tiles_n * q.bn;
  const long M = (long)s->n * s->ho * s->wo;
  if (M >= (1l << 30)) return false;
  q.nkt = cdiv(M, q.kp);
  const int blocks = q.tiles_m * q.tiles_n;
  // about 4 blocks per CU, at least 8 k-tiles per split; the slab round trip capped at a fraction
  // of the layer's own x + dz bytes (keeping >= 256 blocks), as for the register-staged kernel
  int splits = std::max(1, std::min(cdiv(q.nkt, 8), cdiv(4l * conv_cu_count(), blocks)));
  const double data = (double)M * (double)(rup(s->cout, 8) + q.cin8) * 2.0;
  const double slab_rt = 2.0 * 4.0 * (double)q.slab_rows * (double)q.slab_ld;
  const double ratio = getenv("YMS_WG_SLAB_RATIO") ? atof(getenv("YMS_WG_SLAB_RATIO")) : 0.05;   // see conv_igemm.hip
  const int cap = std::max((int)(ratio * data / slab_rt), cdiv(256, blocks));
  splits = std::max(1, std::min(splits, cap));
  q.kt_per_split = cdiv(q.nkt, splits);
  q.splits = cdiv(q.nkt, q.kt_per_split);
  *w = q;
  return true;
}

template <typename T, int KS, int BM, int BN>
static void launch_wr_t(const WRPlan&, const WRParams& p, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((conv_wgrad_ring_kernel<T, KS, BM, BN, 64, 2, 2>), grid, dim3(512), 0, st, p);
}

template <typename T, int KS>
static void launch_wr_k(const WRPlan& w, const WRParams& p, dim3 grid, hipStream_t st) {
  if (w.bm == 128 && w.bn == 128) launch_wr_t<T, KS, 128, 128>(w, p, grid, st);
  else if (w.bm == 64) launch_wr_t<T, KS, 64, 128>(w, p, grid, st);
  else launch_wr_t<T, KS, 128, 64>(w, p, grid, st);
}

yms_status wgrad_ring_launch(const yms_conv_shape* s, const WRPlan& w, const void* x, int x_ld, int x_off,
                             const void* dz, int dz_ld, int dz_off, float* slab, hipStream_t st) {
  WRParams p{};
  p.x = (const char*)x;
  p.dz = (const char*)dz;
  p.slab = slab;
  p.x_ld = x_ld; p.x_off = x_off; p.dz_ld = dz_ld; p.dz_off = dz_off;
  const long es = 2;
  const long M = (long)s->n * s->ho * s->wo;
  const long dzb = M * dz_ld * es, xb = (long)s->n * s->h * s->w * x_ld * es;
  if (dzb >= (1l << 31) - (1l << 20) || xb >= (1l << 31) - (1l << 20)) return YMS_ERR_UNSUPPORTED;
  p.dz_bytes = (uint32_t)dzb;
  p.x_bytes = (uint32_t)xb;
  p.SH = s->h; p.SW = s->w; p.stride = s->stride; p.pad = s->pad;
  p.cout8 = (int)rup(s->cout, 8);
  p.cpt = w.cpt; p.Kc = w.kc; p.M = (int)M;
  p.nkt = w.nkt; p.kt_per_split = w.kt_per_split;
  p.tiles_n = w.tiles_n; p.tiles_mn = w.tiles_m * w.tiles_n;
  p.slab_rows = w.slab_rows; p.slab_ld = w.slab_ld;
  p.div_ow = make_fastdiv(s->wo);
  p.div_ohw = make_fastdiv(s->ho * s->wo);
  const dim3 grid((unsigned)(w.tiles_m * w.tiles_n * w.splits));
  if (s->dtype == YMS_BF16) {
    if (s->k == 1) launch_wr_k<bf16, 1>(w, p, grid, st); else launch_wr_k<bf16, 3>(w, p, grid, st);
  } else {
    if (s->k == 1) launch_wr_k<f16, 1>(w, p, grid, st); else launch_wr_k<f16, 3>(w, p, grid, st);
  }
  return launch_status();
}

}  // namespace yms

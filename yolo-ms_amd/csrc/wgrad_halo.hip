// Weight gradient of a 3x3 convolution (stride 1 or 2) on MFMA with the input staged ONCE per
// spatial patch for all nine taps.
//
//   dW[co][tap][ci] = sum_p dz[p][co] * x[src(p, tap)][ci]     (yolov8/model/components.py:72 backward)
//
// The im2col TT kernel (conv_igemm.hip) gathers every input pixel nine times through L2 (once
// per tap) and re-reads dz once per tap-column tile; with two register-staged k-tiles of 32
// pixels in flight it also leaves the streaming layers (160^2 / 320^2 maps, 32-64 channels)
// at 0.6-1.4 TB/s.  Here a block owns (32*MB output channels) x (all 9 taps x 32*NB input
// channels) and walks output-pixel PATCHES (R rows x TW columns of one image):
//   * per patch, the dz tile [KP pixels][BM] and the input halo [HR x HC pixels][BC] go global
//     -> LDS by raw-buffer LDS-DMA (out-of-image / out-of-range lanes load zeros) into an NS-deep
//     ring that prefetches the next patch while the current one computes;
//   * the MFMA operands are read with ds_read_b64_tr_b16 (pixels along K): every lane supplies
//     the LDS row of its own pixel, so the B operand of tap (dy, dx) is simply the halo row of
//     (r*S + dy, c*S + dx) -- the nine taps share one staged halo;
//   * each wave owns one 32-channel co block, three (tap, ci-block) columns and every WK-th
//     16-pixel k-step of the patch: one A fragment per k-step feeds three MFMAs
//     (v_mfma_f32_32x32x16_{bf16,f16}); the WK wave groups write separate partial slabs, so a
//     block keeps 3 * MB * NB * WK waves busy without a second staged patch;
//   * blocks of one pixel split are consecutive logical ids (XCD-remapped, shared L2) and write
//     one fp32 partial slab each, reduced in a fixed order by wgrad_reduce_kernel.
#include "conv_common.hpp"
#include "wgrad_halo.hpp"

#include <algorithm>
#include <cstdlib>

namespace yms {

struct WHParams {
  const char* x;
  const char* dz;
  float* slab;
  int x_ld, x_off, dz_ld, dz_off;   // elements
  uint32_t x_bytes, dz_bytes;       // raw-buffer extents (< 2^31)
  int H, W, OH, OW, pad;
  int cin8, cout8;
  int TW, R, HC, HPX, RTW;          // patch R x TW, halo width HC, halo pixels, R*TW
  int ptx, pty, npatch, pps;
  int tiles_co, tiles_ci, slab_rows, slab_ld;
  FastDiv div_tw, div_hc, div_ptx, div_pp;
};

template <typename T, int S, int MB, int NB, int WK, int KP, int HB, int NS>
__global__ __launch_bounds__(WK * MB * NB * 3 * 64, KP * 3 * MB * NB * WK <= 384 * 6 ? 2 : 1)
void conv_wgrad_halo_kernel(WHParams p) {
  constexpr int NWV = WK * MB * NB * 3;     // waves: (k-step group) x co block x three (tap, ci-block) columns
  constexpr int NSTEP = KP / 16 / WK;       // k-steps of one wave per patch
  constexpr int ES = (int)sizeof(T);
  constexpr int BM = 32 * MB, BC = 32 * NB;
  constexpr int CA = BM * ES / 16, CB = BC * ES / 16;   // 16-B chunks per LDS row (8 / 4 for 16-bit)
  constexpr int PA = CA * 16, PB = CB * 16;
  constexpr int A_INS = KP * CA / 64, B_INS = HB * CB / 64;   // wave-instructions (1 KB) per stage
  constexpr int A_PW = (A_INS + NWV - 1) / NWV, B_PW = (B_INS + NWV - 1) / NWV;
  constexpr int A_BYTES = A_PW * NWV * 1024, B_BYTES = B_PW * NWV * 1024;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int Q = A_PW + B_PW;             // DMA instructions per wave per stage (uniform)
  static_assert(KP % (16 * WK) == 0 && (KP * CA) % 64 == 0 && (HB * CB) % 64 == 0, "tile");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int tiles = p.tiles_co * p.tiles_ci;
  const int lid = tiles >= 4 ? xcd_remap(blockIdx.x, G) : (int)blockIdx.x;
  const int tile = lid % tiles, split = lid / tiles;
  const int co_t = tile % p.tiles_co, ci_t = tile / p.tiles_co;
  const int co_base = co_t * BM, ci_base = ci_t * BC;
  const int pa0 = split * p.pps, pa1 = min(p.npatch, pa0 + p.pps);
  const int np = pa1 - pa0;
  if (np <= 0) return;

  const __amdgpu_buffer_rsrc_t rs_a =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dz, (short)0, (int)p.dz_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_b =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, NT_RSRC3);

  // XOR swizzle of the 16-B chunk within an A row (MB = 2: 8 chunks per 128-B row): rows k and
  // k + 2 of one transposed read would otherwise hit the same banks (pitch 32 dwords).
  auto swz_a = [](int k) { return CA == 8 ? ((k & 2) << 1) : 0; };

  // ---- loader: one patch into ring stage `stage` ----
  auto issue = [&](int stage, int pi) {
    const uint32_t n = fdiv((uint32_t)pi, p.div_pp);
    const uint32_t rem = (uint32_t)pi - n * p.div_pp.d;
    const uint32_t py = fdiv(rem, p.div_ptx);
    const uint32_t px = rem - py * p.div_ptx.d;
    const int oy0 = (int)py * p.R, ox0 = (int)px * p.TW;
    const int iy0 = oy0 * S - p.pad, ix0 = ox0 * S - p.pad;
    char* sa = smem + stage * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int j = 0; j < A_PW; ++j) {
      const int ins = j * NWV + wv;
      const int li = ins * 64 + lane;
      const int k = li / CA, ch = (li % CA) ^ swz_a(k);
      uint32_t vo = NT_OOB;
      if (ins < A_INS && k < p.RTW) {
        const uint32_t r = fdiv((uint32_t)k, p.div_tw);
        const int oy = oy0 + (int)r, ox = ox0 + (k - (int)r * p.TW);
        const int c = co_base + ch * (16 / ES);
        if (oy < p.OH && ox < p.OW && c < p.cout8)
          vo = (uint32_t)(((((int)n * p.OH + oy) * p.OW + ox) * p.dz_ld + p.dz_off + c) * ES);
      }
      blds16(rs_a, sa + ins * 1024, vo);
    }
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      const int ins = j * NWV + wv;
      const int li = ins * 64 + lane;
      const int h = li / CB, ch = li % CB;
      uint32_t vo = NT_OOB;
      if (ins < B_INS && h < p.HPX) {
        const uint32_t hy = fdiv((uint32_t)h, p.div_hc);
        const int iy = iy0 + (int)hy, ix = ix0 + (h - (int)hy * p.HC);
        const int c = ci_base + ch * (16 / ES);
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && c < p.cin8)
          vo = (uint32_t)(((((int)n * p.H + iy) * p.W + ix) * p.x_ld + p.x_off + c) * ES);
      }
      blds16(rs_b, sb + ins * 1024, vo);
    }
  };

  // ---- compute ----
  const int wk = wv / (MB * 3 * NB), wr = wv % (MB * 3 * NB);
  const int cb = wr % MB, cg = wr / MB;     // co block, column group (three columns)
  const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
  const int th = g >> 1, tcb = 16 * (g & 1);
  const int lr = lane & 31, lh = lane >> 5;
  // A read: logical column cb*32 + tcb + 4pp of pixel rows k = 16 s + 8 th + qq (+4); the row
  // swizzle depends on k & 2 = qq & 2 only, so the in-row byte offset is fixed per lane
  const int a_col = cb * 32 + tcb + 4 * pp;
  const int a_in = (((a_col >> 3) ^ swz_a(qq)) << 4) + ((a_col >> 2) & 1) * 8;
  int b_off[3];       // byte offset of (tap, ci block) column j within a halo row + tap row/col shift
  int b_tap[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = cg * 3 + j;
    const int tap = c / NB, nb = c % NB;
    const int col = nb * 32 + tcb + 4 * pp;
    b_off[j] = (col >> 3) * 16 + ((col >> 2) & 1) * 8;
    b_tap[j] = (tap / 3) * p.HC + (tap % 3);
  }
  f32x16 acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.0f;

  // halo row (tap 0,0) of this lane's two pixels in each of its k-steps: patch-independent
  auto hbase = [&](int k) -> int {
    if (k >= p.RTW) return 0;                 // padding pixel: dz row is zero, any staged row
    const uint32_t r = fdiv((uint32_t)k, p.div_tw);
    return (int)r * S * p.HC + (k - (int)r * p.TW) * S;
  };
  int hb1[NSTEP], hb2[NSTEP];
#pragma unroll
  for (int t = 0; t < NSTEP; ++t) {
    const int k1 = 16 * (wk + t * WK) + 8 * th + qq;
    hb1[t] = hbase(k1) * PB;
    hb2[t] = hbase(k1 + 4) * PB;
  }
  auto compute = [&](int stage) {
    const char* A = smem + stage * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
      const int k1 = 16 * (wk + t * WK) + 8 * th + qq;
      const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(A + k1 * PA + a_in));
      const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(A + (k1 + 4) * PA + a_in));
      const uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
      const u32x4 af = u32x4{u0.x, u0.y, u1.x, u1.y};
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const s16x4 w0 =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(B + hb1[t] + b_tap[j] * PB + b_off[j]));
        const s16x4 w1 =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)(B + hb2[t] + b_tap[j] * PB + b_off[j]));
        const uint2 x0 = __builtin_bit_cast(uint2, w0), x1 = __builtin_bit_cast(uint2, w1);
        acc[j] = Mfma<T>::mma(af, u32x4{x0.x, x0.y, x1.x, x1.y}, acc[j]);
      }
    }
  };

  // ---- ring: stage g lands, the next patch's DMA issues, stage g computes ----
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < np) issue(s0, pa0 + s0);
  int stage = 0;
  for (int gi2 = 0; gi2 < np; ++gi2) {
    wait_tiles<Q, NS - 2>(np - 1 - gi2);
    raw_barrier();
    if (gi2 + NS - 1 < np) {
      int ns = stage + NS - 1;
      if (ns >= NS) ns -= NS;
      issue(ns, pa0 + gi2 + NS - 1);
    }
    compute(stage);
    if (++stage == NS) stage = 0;
  }

  // ---- partial slab: rows co, columns tap * cin8 + ci ----
  float* slab = p.slab + (long)(split * WK + wk) * p.slab_rows * p.slab_ld;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = cg * 3 + j;
    const int tap = c / NB, nb = c % NB;
    const int ci = ci_base + nb * 32 + lr;
    if (ci < p.cin8) {
      const int col = tap * p.cin8 + ci;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = co_base + cb * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        slab[(long)co * p.slab_ld + col] = acc[j][i];
      }
    }
  }
}

static int env_int_wh(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// patch width: the whole output row when it is narrow, else a divisor of it near 32
static int pick_tw(int ow) {
  if (ow <= 40) return ow;
  for (int t : {32, 40, 36, 28, 24, 20, 16})
    if (ow % t == 0) return t;
  return 32;
}

bool wgrad_halo_plan(const yms_conv_shape* s, WHPlan* w) {
  const int on = env_int_wh("YMS_WG_HALO", 1);   // read per call: tests switch it at run time
  if (!on || s->k != 3 || s->pad != 1 || s->dtype == YMS_F32) return false;
  // measured on every 3x3 layer of YOLOv8-s at B=64 (profiles/r03_wgrad_halo_micro.txt): the halo
  // kernel wins where the output channels fill its 32 / 64-channel blocks exactly (160^2
  // 32->32: 143 -> 92 us, 80^2 128->64: 156 -> 107 us, 20^2 512->64: 52 -> 38 us, 320^2 32->64
  // stride 2: 264 -> 194 us); for 80 / 128+ output channels (tile quantisation, dz re-read per
  // 32-channel input block) and 3-channel inputs the im2col kernel stays ahead.  YMS_WG_HALO=2
  // forces the halo kernel on every 3x3 shape (tests / A/B).
  if (on != 2 && !((s->cout == 32 || s->cout == 64) && s->cin >= 16)) return false;
  WHPlan q{};
  q.S = s->stride;
  q.mb = s->cout <= 32 ? 1 : 2;
  q.nb = 1;
  // <= 64 KB of LDS per block, so the side-stream weight gradients fit on a CU beside the main
  // stream's conv blocks (round 3, measured and dropped: 256 / 128-pixel patches in 112-150 KB,
  // faster in isolation, but such a block waits for a whole CU to drain: in the training step that
  // cost more than the nine-fold input re-read it removes)
  q.wk = q.mb == 1 ? 2 : 1;
  q.kp = q.S == 1 ? 128 : 64;
  q.hb = q.S == 1 ? 256 : 384;
  q.TW = std::min(pick_tw(s->wo), q.kp);
  // 64 -> 64 stride-1 layers (the 80^2 C2f bottlenecks): with 32-channel input blocks every dz
  // patch is read twice, once per block (PMC: 2.44x the algorithmic bytes on the YOLOv8-s step's
  // seven such layers, profiles/r06_wgrad_pmc_layers.txt); one block covering all 64 input
  // channels (12 waves) reads dz once, on 64-pixel patches of 4 x 16 (halo 6 x 18 = 1.69x)
  if (q.S == 1 && q.mb == 2 && rup(s->cin, 8) == 64 && s->wo % 16 == 0 && s->ho >= 4 &&
      env_int_wh("YMS_WG_HALO_NB2", 1)) {
    q.nb = 2;
    q.kp = 64;
    q.hb = 128;
    q.TW = 16;
  }
  q.R = std::max(1, std::min(s->ho, q.kp / q.TW));
  for (;;) {
    q.HR = (q.R - 1) * q.S + 3;
    q.HC = (q.TW - 1) * q.S + 3;
    if (q.HR * q.HC <= q.hb || q.R == 1) break;
    --q.R;
  }
  if (q.HR * q.HC > q.hb) return false;
  q.ptx = cdiv(s->wo, q.TW);
  q.pty = cdiv(s->ho, q.R);
  const long npatch = (long)s->n * q.ptx * q.pty;
  if (npatch >= (1l << 30)) return false;
  q.npatch = (int)npatch;
  const int cin8 = (int)rup(s->cin, 8);
  q.tiles_co = cdiv(s->cout, 32 * q.mb);
  q.tiles_ci = cdiv(cin8, 32 * q.nb);
  q.slab_rows = q.tiles_co * 32 * q.mb;
  q.slab_ld = 9 * cin8;
  const int tiles = q.tiles_co * q.tiles_ci;
  // about two blocks per CU in all; each split writes (and the reduce re-reads) one fp32 slab, so
  // cap the slab round trip at the layer's own x + dz bytes (keeping >= 256 blocks)
  int splits = std::max(1, std::min(q.npatch, cdiv(2l * conv_cu_count(), tiles)));
  const double data = (double)s->n * s->ho * s->wo * rup(s->cout, 8) * 2.0 + (double)s->n * s->h * s->w * cin8 * 2.0;
  const double slab_rt = 2.0 * 4.0 * (double)q.slab_rows * q.slab_ld * q.wk;
  const double ratio = getenv("YMS_WG_SLAB_RATIO") ? atof(getenv("YMS_WG_SLAB_RATIO")) : 0.05;   // see conv_igemm.hip
  const int cap = std::max((int)(ratio * data / slab_rt), cdiv(256, tiles));
  splits = std::max(1, std::min(splits, cap));
  q.pps = cdiv(q.npatch, splits);
  q.splits = cdiv(q.npatch, q.pps);
  *w = q;
  return true;
}

template <typename T, int S, int MB, int NB, int WK, int KP, int HB, int NS>
static void launch_wh(const WHParams& p, int blocks, hipStream_t st) {
  hipLaunchKernelGGL((conv_wgrad_halo_kernel<T, S, MB, NB, WK, KP, HB, NS>), dim3(blocks),
                     dim3(WK * MB * NB * 3 * 64), 0, st, p);
}

template <typename T>
static void dispatch_wh(const WHPlan& w, const WHParams& p, int blocks, hipStream_t st) {
  if (w.S == 1) {
    if (w.mb == 1) launch_wh<T, 1, 1, 1, 2, 128, 256, 2>(p, blocks, st);
    else if (w.nb == 2) launch_wh<T, 1, 2, 2, 1, 64, 128, 2>(p, blocks, st);
    else launch_wh<T, 1, 2, 1, 1, 128, 256, 2>(p, blocks, st);
  } else {
    if (w.mb == 1) launch_wh<T, 2, 1, 1, 2, 64, 384, 2>(p, blocks, st);
    else launch_wh<T, 2, 2, 1, 1, 64, 384, 2>(p, blocks, st);
  }
}

yms_status wgrad_halo_launch(const yms_conv_shape* s, const WHPlan& w, const void* x, int x_ld, int x_off,
                             const void* dz, int dz_ld, int dz_off, float* slab, hipStream_t st) {
  WHParams p{};
  p.x = (const char*)x;
  p.dz = (const char*)dz;
  p.slab = slab;
  p.x_ld = x_ld; p.x_off = x_off; p.dz_ld = dz_ld; p.dz_off = dz_off;
  const long es = 2;
  const long dzb = (long)s->n * s->ho * s->wo * dz_ld * es, xb = (long)s->n * s->h * s->w * x_ld * es;
  if (dzb >= (1l << 31) - (1l << 20) || xb >= (1l << 31) - (1l << 20)) return YMS_ERR_UNSUPPORTED;
  p.dz_bytes = (uint32_t)dzb;
  p.x_bytes = (uint32_t)xb;
  p.H = s->h; p.W = s->w; p.OH = s->ho; p.OW = s->wo; p.pad = s->pad;
  p.cin8 = (int)rup(s->cin, 8);
  p.cout8 = (int)rup(s->cout, 8);
  p.TW = w.TW; p.R = w.R; p.HC = w.HC; p.HPX = w.HR * w.HC; p.RTW = w.R * w.TW;
  p.ptx = w.ptx; p.pty = w.pty; p.npatch = w.npatch; p.pps = w.pps;
  p.tiles_co = w.tiles_co; p.tiles_ci = w.tiles_ci; p.slab_rows = w.slab_rows; p.slab_ld = w.slab_ld;
  p.div_tw = make_fastdiv(w.TW);
  p.div_hc = make_fastdiv(w.HC);
  p.div_ptx = make_fastdiv(w.ptx);
  p.div_pp = make_fastdiv(w.ptx * w.pty);
  const int blocks = w.tiles_co * w.tiles_ci * w.splits;
  if (s->dtype == YMS_BF16) dispatch_wh<bf16>(w, p, blocks, st);
  else dispatch_wh<f16>(w, p, blocks, st);
  return launch_status();
}

}  // namespace yms

// Halo-tiled 3x3 stride-1 convolution for gfx950 (16-bit types): the forward of the reference's
// 3x3 Conv blocks (yolov8/model/components.py:69-77 -- every Bottleneck conv, :80-93, and the
// head's 3x3 branch convs, yolov8_head.py:83-110) and their stride-1 input gradient.
//
// The im2col NT kernel (conv_igemm.hip) streams one (tap, 64-channel) k-tile of A per step, so
// every input pixel crosses L2 -> LDS nine times per channel chunk.  Here an output tile is a
// TH x TW block of the batch laid out as one tall "virtual" image -- image n occupies virtual rows
// n*(H+1) .. n*(H+1)+H-1 and virtual row n*(H+1)+H is a zero separator -- so the 3x3 neighbourhood
// of every tile pixel lies inside ONE (TH+2) x (TW+2) halo of the virtual image, whatever images
// the tile spans.  Per 64-channel chunk group the halo is staged ONCE (raw-buffer LDS-DMA,
// out-of-image / separator pixels read as zeros) and the nine taps read shifted windows of it:
// A-operand LDS fill drops from 9 x 256 to (TH+2)(TW+2) ~ 330 pixel rows per chunk group, and
// the per-k-tile fill is the 16 KB weight tile plus 1/9 of the halo.
//
// Pipeline (one 512-thread block per CU, persistent over output tiles): a 3-deep ring of weight
// k-tiles (tap t, chunk group cg) and a double-buffered halo.  The halo of chunk-step j+1 is
// issued in pieces alongside the weight loads of taps 0..HS-1 of chunk-step j, so every wave
// issues a fixed, tap-determined number of DMAs per step and waits with a counted vmcnt.
// Separator / padding / dead rows of a tile are not stored.  Training-forward convolutions with BN
// statistics always take the NT kernels (their per-128-pixel statistics rows, conv_common.hpp).
#include <algorithm>
#include <cstdlib>

#include "conv_common.hpp"
#include "conv_halo.hpp"

namespace yms {

constexpr int HL_BM = 256;                 // output pixels per tile (TH * TW <= 256)
constexpr int HL_HPX = 384;                // halo pixel capacity per buffer
constexpr int HL_HBUF = HL_HPX * 128;      // bytes per halo buffer
constexpr int HL_ST = 3;                   // weight k-tile ring depth
constexpr int HL_MAX_AFFINE = 512;

struct HaloParams {
  const char* src;
  const char* wp;
  char* dst;
  int src_ld, src_off, dst_ld, dst_off;
  const float* scale;
  const float* shift;
  int act;
  const char* res;
  int res_ld, res_off;
  int N, H, W;
  int TW, TH, ntx, tiles_m, tiles_n;
  int Ncols;          // valid output channels
  int nkc;            // 64-channel chunk groups along the reduction dimension
  int hp;             // halo pixels of a tile = (TH+2) * (TW+2)
  int hs;             // halo pieces = ceil(hp / (threads / 8)) (a piece = one DMA per lane)
  int vrows;          // N * (H + 1) virtual rows
  uint32_t src_bytes;
  FastDiv div_tw, div_tw2, div_h1;
};

template <typename T, int MODE, int EPI, int BN, int WGM, int WGN>
__global__ __launch_bounds__(WGM * WGN * 64, 1) void conv_halo_kernel(HaloParams p) {
  constexpr int BM = HL_BM, NTHR = WGM * WGN * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int RPP = NTHR / NT_KCH;                 // weight rows (and halo pixels) per load pass
  constexpr bool B_PART = BN < RPP;                  // only the first BN/8 waves load weights
  constexpr int B_SLOTS = B_PART ? 1 : BN / RPP;
  constexpr int HS_MAX = HL_HPX / RPP;
  constexpr int BSTAGE = BN * 128;
  constexpr int PRM = (EPI == EPI_AFFINE) ? 2 * HL_MAX_AFFINE * 4 : 0;
  constexpr int NH = (BM * BN * (int)sizeof(T) > HL_HBUF) ? 2 : 1;
  constexpr int HR = BM / NH;
  static_assert(TM >= 1 && TN >= 1 && HR * BN * (int)sizeof(T) <= HL_HBUF && HR % WTM == 0, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * HL_HBUF + HL_ST * BSTAGE + PRM];
  char* const bring = smem + 2 * HL_HBUF;
  float* prm = reinterpret_cast<float*>(smem + 2 * HL_HBUF + HL_ST * BSTAGE);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int lr = lane & 31, lh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int ntiles = p.tiles_m * p.tiles_n;
  if (lb >= ntiles) return;
  const int my_tiles = (ntiles - lb + G - 1) / G;
  const int nkt = 9 * p.nkc;
  const int total = my_tiles * nkt;
  const int J = my_tiles * p.nkc;                      // chunk-steps of this block
  if constexpr (EPI == EPI_AFFINE) {
    for (int c = tid; c < p.Ncols; c += NTHR) {
      prm[c] = p.scale ? p.scale[c] : 1.0f;
      prm[HL_MAX_AFFINE + c] = p.shift ? p.shift[c] : 0.0f;
    }
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t rs_a =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, (int)p.src_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_b = __builtin_amdgcn_make_buffer_rsrc((void*)p.wp, (short)0, 0x7fffffff, NT_RSRC3);
  constexpr int ES = (int)sizeof(T);
  const int TW2 = p.TW + 2;

  // ---- halo loader: lane fills LDS slot (tid & 7) of halo pixel s*64 + tid/8 ----
  int hsrc[HS_MAX];          // byte offset of the lane's source chunk (chunk group 0), or -1
  auto setup_halo = [&](int t) {
    const int tm = t / p.tiles_n;
    const int tyb = tm / p.ntx, txb = tm - (tm / p.ntx) * p.ntx;
    const int V0 = tyb * p.TH, x0 = txb * p.TW;
#pragma unroll
    for (int s = 0; s < HS_MAX; ++s) {
      const int hp = s * RPP + (tid >> 3);
      const uint32_t hv = fdiv((uint32_t)hp, p.div_tw2);
      const int hx = hp - (int)hv * TW2;
      const int V = V0 - 1 + (int)hv, x = x0 - 1 + hx;
      bool ok = hp < p.hp && V >= 0 && V < p.vrows && x >= 0 && x < p.W;
      const uint32_t Vu = ok ? (uint32_t)V : 0u;
      const uint32_t n = fdiv(Vu, p.div_h1);
      const int y = (int)Vu - (int)n * (p.H + 1);
      ok = ok && y < p.H;
      const int q = (tid & 7) ^ ((hp >> 1) & 7);
      hsrc[s] = ok ? (((((int)n * p.H + y) * p.W + x) * p.src_ld + p.src_off) * ES + q * 16) : -1;
    }
  };
  auto issue_halo_piece = [&](int s, int cg, int hb) {
    const uint32_t vo = hsrc[s] >= 0 ? (uint32_t)(hsrc[s] + cg * 128) : NT_OOB;
    blds16(rs_a, smem + hb * HL_HBUF + s * (RPP * 128) + wv * 1024, vo);
  };
  // ---- weight loader: incremental (tile, chunk group, tap) position, all wave-uniform ----
  const int qb = (tid & 7) ^ ((tid >> 4) & 7), rb = tid >> 3;
  const int prow_bytes = nkt * NT_KCH * 16;            // bytes per packed weight row
  int b_tap = 0, b_cg = 0, b_tile = lb;
  int b_n0 = (lb % p.tiles_n) * BN;
  const int my_b = B_PART ? (wv * 8 < BN ? 1 : 0) : B_SLOTS;   // weight DMAs per k-tile of this wave
  auto issue_b = [&](int stage) {
    const int kb = b_tap * p.nkc + b_cg;               // packed K order: (tap, chunk group)
    if (!B_PART || wv * 8 < BN) {
#pragma unroll
      for (int j = 0; j < B_SLOTS; ++j)
        blds16(rs_b, bring + stage * BSTAGE + j * (RPP * 128) + wv * 1024,
               (uint32_t)((b_n0 + j * RPP + rb) * prow_bytes + kb * 128 + qb * 16));
    }
    if (++b_tap == 9) {
      b_tap = 0;
      if (++b_cg == p.nkc) {
        b_cg = 0;
        b_tile += G;
        b_n0 = (b_tile % p.tiles_n) * BN;
      }
    }
  };

  // ---- A fragment addressing: lane rows are tile-independent ----
  int hpb[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int r = wm * WTM + a * 32 + lr;
    const int ty = (int)fdiv((uint32_t)r, p.div_tw), tx = r - ty * p.TW;
    hpb[a] = ty * TW2 + tx;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;
  const int swz = (lr >> 1) & 7;
  auto compute = [&](int hb, int stage, int tap) {
    const char* Hb = smem + hb * HL_HBUF;
    const char* B = bring + stage * BSTAGE;
    const int dy = tap / 3, dx = tap - (tap / 3) * 3;
    const int toff = MODE == MODE_FWD ? dy * TW2 + dx : (2 - dy) * TW2 + (2 - dx);
    int aad[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int hp = hpb[a] + toff;
      aad[a] = hp * 128 + ((lh ^ ((hp >> 1) & 7)) << 4);
    }
    u32x4 af[2][TM], bfr[2][TN];
    auto frags = [&](int s, int slot) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af[slot][a] = *reinterpret_cast<const u32x4*>(Hb + (aad[a] ^ (s << 5)));
      const int co = ((2 * s + lh) ^ swz) * 16;
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bfr[slot][b] = *reinterpret_cast<const u32x4*>(B + (wn * WTN + b * 32 + lr) * 128 + co);
    };
    frags(0, 0);
#pragma unroll
    for (int s = 0; s < NT_KCH / 2; ++s) {
      if (s + 1 < NT_KCH / 2) frags(s + 1, (s + 1) & 1);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = Mfma<T>::mma(af[s & 1][a], bfr[s & 1][b], acc[a][b]);
    }
  };

  auto lds_barrier = [&]() {
    __builtin_amdgcn_s_waitcnt((0xF) | (3 << 14) | (0x7 << 4) | (0 << 8));   // lgkmcnt(0) only
    raw_barrier();
  };
  // virtual row V of the tall image -> (is a real pixel row, row base = n*H + y)
  auto vrow = [&](int V, int& rbase) {
    if (V < 0 || V >= p.vrows) return false;
    const uint32_t n = fdiv((uint32_t)V, p.div_h1);
    const int y = V - (int)n * (p.H + 1);
    rbase = (int)n * p.H + y;
    return y < p.H;
  };
  auto epilogue = [&](int t, char* stg_base) {
    const int tm = t / p.tiles_n, n0 = (t % p.tiles_n) * BN;
    const int tyb = tm / p.ntx, txb = tm - (tm / p.ntx) * p.ntx;
    const int V0 = tyb * p.TH, x0 = txb * p.TW;
    // rows outside the image set (separator rows, rows past the batch, dead rows ty >= TH)
    // contribute nothing: zero their accumulators before statistics and staging
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        const int ty = (int)fdiv((uint32_t)r, p.div_tw);
        int rbase;
        const bool ok = ty < p.TH && vrow(V0 + ty, rbase);
        if (!ok) {
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b][i] = 0.0f;
        }
      }
    if constexpr (EPI == EPI_AFFINE) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n0 + wn * WTN + b * 32 + lr;
        const bool cv = col < p.Ncols;
        const float sc = cv ? prm[col] : 1.0f;
        const float sh = cv ? prm[HL_MAX_AFFINE + col] : 0.0f;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = acc[a][b][i] * sc + sh;
            if (p.act == YMS_ACT_SILU) v = silu_f(v);
            acc[a][b][i] = v;
          }
      }
    }
    T* stg = reinterpret_cast<T*>(stg_base);
    constexpr int CH = BN / 8;
    constexpr int RS = NTHR / CH;
    const int ch = tid % CH, rr = tid / CH;
    const int col0 = n0 + ch * 8;
    const int nv = p.Ncols - col0;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      lds_barrier();
      if (NH == 1 || (wm * WTM) / HR == h) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int rl = wm * WTM - h * HR + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
              stg[rl * BN + wn * WTN + b * 32 + lr] = (T)acc[a][b][i];
              acc[a][b][i] = 0.0f;
            }
      }
      lds_barrier();
#pragma unroll
      for (int j = 0; j < HR / RS; ++j) {
        const int rl = rr + RS * j;
        const int r = h * HR + rl;
        const int ty = (int)fdiv((uint32_t)r, p.div_tw), tx = r - ty * p.TW;
        int rbase;
        if (ty >= p.TH || !vrow(V0 + ty, rbase) || nv <= 0) continue;
        const long pix = (long)rbase * p.W + x0 + tx;
        float v[8];
        unpack8(*reinterpret_cast<const Raw8<T>*>(stg + rl * BN + ch * 8), v);
        T* dst = reinterpret_cast<T*>(p.dst) + pix * p.dst_ld + p.dst_off + col0;
        if (EPI == EPI_AFFINE && p.res) {
          float rv[8];
          load8(reinterpret_cast<const T*>(p.res) + pix * p.res_ld + p.res_off + col0, nv, rv);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += rv[i];
        } else if (EPI == EPI_ACCUM) {
          float rv[8];
          load8(dst, nv, rv);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += rv[i];
        }
        store8(dst, nv, v);
      }
    }
  };

  // ---- the flattened (tile, chunk group, tap) stream ----
  // issue group I_g = weight k-tile g+ST-1 (+ halo piece `tap` of chunk-step j+1 when tap < hs);
  // iteration g waits until at most the loads of I_{g-1} are in flight
  setup_halo(lb);
  for (int s = 0; s < p.hs; ++s) issue_halo_piece(s, 0, 0);
#pragma unroll
  for (int s0 = 0; s0 < HL_ST - 1; ++s0)
    if (s0 < total) issue_b(s0);
  int stage = 0, tap = 0, j = 0, cg = 0, tile = lb;
  int prev_loads = total > 1 ? my_b : 0;               // loads issued after k-tile 0's weights
  for (int g = 0; g < total; ++g) {
    switch (prev_loads) {
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<1>(); break;
      case 2: wait_vmcnt<2>(); break;
      default: wait_vmcnt<3>(); break;
    }
    raw_barrier();
    int loads = 0;
    if (g + HL_ST - 1 < total) {
      int ns = stage + HL_ST - 1;
      if (ns >= HL_ST) ns -= HL_ST;
      issue_b(ns);
      loads = my_b;
    }
    if (tap < p.hs && j + 1 < J) {
      const int cgn = cg + 1 == p.nkc ? 0 : cg + 1;
      if (cgn == 0 && tap == 0) setup_halo(tile + G);
      issue_halo_piece(tap, cgn, (j + 1) & 1);
      ++loads;
    }
    prev_loads = loads;
    compute(j & 1, stage, tap);
    if (++stage == HL_ST) stage = 0;
    if (++tap == 9) {
      tap = 0;
      if (cg + 1 == p.nkc) epilogue(tile, smem + (j & 1) * HL_HBUF);
      ++j;
      if (++cg == p.nkc) {
        cg = 0;
        tile += G;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// Opt-in (YMS_HALO=1): on MI355X the im2col NT kernel is faster on every S / L layer but one
// (profiles/r02_halo_micro.txt: 128->128 @40^2 501 vs 547 TF/s, 256->256 @20^2 658 vs 764,
// 64->64 @80^2 340 vs 469; only 256->64 @40^2 wins, 482 vs 398).  The halo cuts the A-operand
// L2->LDS fill ~3x, but its two halo buffers hold the CU to ONE block, so every per-k-tile
// barrier stalls all 16 waves at once, where the NT kernel runs 2-3 independent blocks per CU.
static bool halo_geometry(const yms_conv_shape* s, int mode, HaloGeo* g) {
  static const int enabled = getenv("YMS_HALO") ? atoi(getenv("YMS_HALO")) : 0;
  if (!enabled || !s || s->dtype == YMS_F32) return false;
  if (s->k != 3 || s->stride != 1 || s->pad != 1 || s->ho != s->h || s->wo != s->w) return false;
  const int kred = mode == 0 ? s->cin : s->cout;     // reduction channels
  const int ncols = mode == 0 ? s->cout : s->cin;    // output channels
  if (kred % 64 != 0 || ncols <= 0) return false;
  int TW, TH;
  if (s->w >= 64 && s->w % 16 == 0) {
    TW = 16;
    TH = 16;
  } else if (s->w < 64) {
    TW = s->w;
    TH = std::min(HL_BM / TW, 32);
    while (TH > 1 && (TH + 2) * (TW + 2) > HL_HPX) --TH;
    if (TH < 2) return false;
  } else {
    return false;
  }
  g->TW = TW;
  g->TH = TH;
  g->ntx = s->w / TW;
  const long vrows = (long)s->n * (s->h + 1);
  g->nty = (int)((vrows + TH - 1) / TH);
  g->tiles_m = g->ntx * g->nty;
  g->bn = ncols <= 64 ? 64 : 128;
  g->tiles_n = (ncols + g->bn - 1) / g->bn;
  g->hp = (TH + 2) * (TW + 2);
  g->nkc = kred / 64;
  if (vrows >= (1l << 30) || (long)g->tiles_m * g->tiles_n >= (1l << 30)) return false;
  return true;
}

bool conv_halo_geometry(const yms_conv_shape* s, int mode, HaloGeo* g) { return halo_geometry(s, mode, g); }

// 16 waves per block (4 per SIMD) by default; YMS_HALO_WAVES=8 selects 8 (dev A/B)
static int halo_waves() {
  static const int w = getenv("YMS_HALO_WAVES") ? atoi(getenv("YMS_HALO_WAVES")) : 16;
  return w == 8 ? 8 : 16;
}

template <typename T, int MODE, int EPI>
static void launch_halo(HaloParams p, int bn, hipStream_t st) {
  const long ntiles = (long)p.tiles_m * p.tiles_n;
  const unsigned grid = (unsigned)std::max<long>(1, std::min<long>(ntiles, conv_cu_count()));
  const int waves = halo_waves();
  p.hs = (p.hp + waves * 8 - 1) / (waves * 8);
  if (waves == 8) {
    if (bn == 64)
      hipLaunchKernelGGL((conv_halo_kernel<T, MODE, EPI, 64, 4, 2>), dim3(grid), dim3(512), 0, st, p);
    else
      hipLaunchKernelGGL((conv_halo_kernel<T, MODE, EPI, 128, 4, 2>), dim3(grid), dim3(512), 0, st, p);
  } else {
    if (bn == 64)
      hipLaunchKernelGGL((conv_halo_kernel<T, MODE, EPI, 64, 8, 2>), dim3(grid), dim3(1024), 0, st, p);
    else
      hipLaunchKernelGGL((conv_halo_kernel<T, MODE, EPI, 128, 8, 2>), dim3(grid), dim3(1024), 0, st, p);
  }
}

yms_status conv_halo_launch(const yms_conv_shape* s, int mode, const HaloGeo& g, const void* src, int src_ld,
                            int src_off, const void* wpacked, void* dst, int dst_ld, int dst_off, const float* scale,
                            const float* shift, int act, const void* res, int res_ld, int res_off, float* stats,
                            int accumulate, hipStream_t st) {
  HaloParams p{};
  p.src = (const char*)src;
  p.wp = (const char*)wpacked;
  p.dst = (char*)dst;
  p.src_ld = src_ld; p.src_off = src_off; p.dst_ld = dst_ld; p.dst_off = dst_off;
  p.scale = scale; p.shift = shift; p.act = act;
  p.res = (const char*)res; p.res_ld = res_ld; p.res_off = res_off;
  p.N = s->n; p.H = s->h; p.W = s->w;
  p.TW = g.TW; p.TH = g.TH; p.ntx = g.ntx; p.tiles_m = g.tiles_m; p.tiles_n = g.tiles_n;
  p.Ncols = mode == 0 ? s->cout : s->cin;
  p.nkc = g.nkc;
  p.hp = g.hp;
  p.vrows = s->n * (s->h + 1);
  const long es = 2;
  const long bytes = (long)s->n * s->h * s->w * src_ld * es;
  if (bytes >= (1l << 31) - (1l << 20)) return YMS_ERR_UNSUPPORTED;
  if (g.hp > HL_HPX) return YMS_ERR_UNSUPPORTED;
  p.src_bytes = (uint32_t)bytes;
  p.div_tw = make_fastdiv(g.TW);
  p.div_tw2 = make_fastdiv(g.TW + 2);
  p.div_h1 = make_fastdiv(s->h + 1);
  if (stats || (mode == 0 && p.Ncols > HL_MAX_AFFINE)) return YMS_ERR_UNSUPPORTED;
#define YMS_HALO_CASE(T)                                                                   \
  if (mode == 0) {                                                                         \
    launch_halo<T, MODE_FWD, EPI_AFFINE>(p, g.bn, st);                                     \
  } else {                                                                                 \
    if (accumulate) launch_halo<T, MODE_DGRAD, EPI_ACCUM>(p, g.bn, st);                    \
    else launch_halo<T, MODE_DGRAD, EPI_STORE>(p, g.bn, st);                               \
  }
  if (s->dtype == YMS_BF16) { YMS_HALO_CASE(bf16) }
  else { YMS_HALO_CASE(f16) }
#undef YMS_HALO_CASE
  return launch_status();
}

}  // namespace yms

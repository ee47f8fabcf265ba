// Direct 3x3 convolution for small channel counts on gfx950 (MI355X): the forward of the
// reference's 3x3 Conv blocks (yolov8/model/components.py:69-77) where the reduction has 32 or 64
// channels and the output at most 64 -- the Bottleneck convs of the 160^2 / 80^2 C2f stages
// (components.py:80-122) and the 80^2 head branches (yolov8_head.py:83-110) -- and the stride-1
// input gradient of the same layers.
//
// Why not the implicit GEMM (conv_igemm.hip): these layers are HBM-bound (a 64->64 3x3 conv moves
// 2 B per output element per channel and does 2*576 FLOP per output element: 288 FLOP/B, under the
// 312 FLOP/B ridge), yet the im2col k-tiles bring every input pixel nine times across L2 -> LDS and
// a 32- or 64-column tile pays a full k-tile of A per MFMA column block.  Here:
//   * the block's whole packed weight matrix (<= 72 KB: 64 x 9 x 64 bf16) sits in LDS for the
//     life of the persistent block (loaded once by LDS-DMA);
//   * an output tile of TH x TW = 256 pixels (TW = 32 or 16) needs one (TH+2) x (TW+2) halo of the
//     input (340 / 324 pixels: 1.3x the tile), staged ONCE by raw-buffer LDS-DMA (out-of-image
//     pixels read as zeros through the buffer range check), double-buffered so the next tile's halo
//     lands while this one computes;
//   * the nine taps read shifted windows of the halo as MFMA A fragments (v_mfma_f32_32x32x16,
//     rows = pixels, K = channels of one tap), B fragments from the resident weights: no k-tile
//     pipeline, ONE barrier per tile;
//   * the epilogue stages the tile through the halo buffer just consumed and writes 16-B rows with
//     raw-buffer stores (rows past the map are dropped by the range check, so every lane issues the
//     same loads / stores and the waits are counted): BN+SiLU(+residual) in eval, z plus per-block
//     centred BN statistics in training (conv_common.hpp contract, one row per block), store or
//     accumulate for the input gradient.
// Input gradient (stride 1, pad 1): dx(y, x) = sum_t dz(y + 1 - dy_t, x + 1 - dx_t) W_t^T, i.e. the
// same halo with the taps mirrored and the transposed packing of yms_conv_pack_weight(for_dgrad=1).
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "conv_common.hpp"
#include "conv_direct.hpp"


namespace yms {

struct DirectParams {
  const char* src;
  const char* wp;
  char* dst;
  const char* res;
  int src_ld, src_off, dst_ld, dst_off, res_ld, res_off;
  const float* scale;
  const float* shift;
  int act;
  float* stats;
  int stats_ld;
  float* stats_cnt;
  int H, W;                    // source map (stride 1: also the output map)
  int OH, OW;                  // output map
  int tiles_x, tiles_y, ntiles;
  int Ncols;                   // valid output channels (multiple of 8)
  int nkt;                     // packed weight k-tiles per row (row pitch nkt * 128 B)
  int wrows;                   // packed weight rows (128-padded): the stride-2 class blocks' pitch
  uint32_t src_bytes, dst_bytes, res_bytes;
  // input gradient with the producer's BN + act backward reduce fused (BNR): the producer's pre-BN
  // z (a view of the dx pixels' channels), its scale / shift / [mean | invstd] and act; partial rows
  // bws[block][2][Ncols] = (sum da, sum da * xhat) over the block's final dx values
  const char* bz;
  int bz_ld, bz_off;
  uint32_t bz_bytes;
  const float* bsc;
  const float* bsh;
  const float* bmi;
  int bact;
  float* bws;
};

// BN + act backward partial sums (bn_pool.hip bn_bwd_reduce_kernel's formula) of one 16-B chunk of
// the FINAL input gradient g (channels c0 .. c0 + 7, the values as stored) against the producer's z:
// da = g * act'(z * scale + shift), xhat = (z - mean) * invstd; s1 += da, s2 += da * xhat.
// bnp: [4][COP] floats in LDS (scale, shift, mean, invstd).
template <typename T>
__device__ __forceinline__ void cd_bnred(const float (&g)[8], const u32x4& zraw, const float* bnp, int cop, int c0,
                                         int act, float* s1, float* s2) {
  float zv[8];
  unpack8(*reinterpret_cast<const Raw8<T>*>(&zraw), zv);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 sc = *reinterpret_cast<const float4*>(bnp + c0 + 4 * h);
    const float4 sh = *reinterpret_cast<const float4*>(bnp + cop + c0 + 4 * h);
    const float4 mu = *reinterpret_cast<const float4*>(bnp + 2 * cop + c0 + 4 * h);
    const float4 is = *reinterpret_cast<const float4*>(bnp + 3 * cop + c0 + 4 * h);
    const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
    const float muv[4] = {mu.x, mu.y, mu.z, mu.w}, isv[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * h + j;
      float da = g[i];
      if (act == YMS_ACT_SILU) da = g[i] * dsilu_f(zv[i] * scv[j] + shv[j]);
      s1[i] += da;
      s2[i] += da * ((zv[i] - muv[j]) * isv[j]);
    }
  }
}

// Block merge of the per-lane BN-reduce sums: lane (wave, lr, lh) holds channels cf*32 + 16pp + 8lh +
// (0..7) of its pixels; the 256 lanes of each channel (8 waves x 32) are summed in a fixed order
// through LDS (scratch: 2 x 16 x 256 floats) and written as row `row` of bws ([rows][2][Ncols]).
template <int NCF>
__device__ __forceinline__ void cd_bnred_store(float (&s1)[NCF][16], float (&s2)[NCF][16], char* scratch,
                                               float* bws, int row, int ncols) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
  float* const t = reinterpret_cast<float*>(scratch);     // [2][16][256]
  const int u = tid >> 5, k = tid & 31;                    // thread: channel u of the pass, lane group k
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (lh == h) {
        const int j = wave * 32 + lr;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          t[i * 256 + j] = s1[cf][i];
          t[(16 + i) * 256 + j] = s2[cf][i];
        }
      }
      __syncthreads();
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a += t[u * 256 + 8 * k + e];
        b += t[(16 + u) * 256 + 8 * k + e];
      }
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
      }
      if (k == 0) {                                        // register u = 8pp + jj: channel 16pp + 8h + jj

        const int pp = u >> 3, jj = u & 7;
        const int c = cf * 32 + 16 * pp + 8 * h + jj;
        if (c < ncols) {
          bws[(long)row * 2 * ncols + c] = a;
          bws[(long)row * 2 * ncols + ncols + c] = b;
        }
      }
      __syncthreads();
    }
}

template <int TW, int CP, int NCF> struct DirGeo {
  static constexpr int NTHR = 512, NW = 8, BM = 256, TH = BM / TW;
  static constexpr int HWD = TW + 2, HP = (TH + 2) * HWD;   // halo width, pixels
  static constexpr int PITCH = CP * 16;                     // LDS bytes per halo pixel
  static constexpr int HGR = HP * CP;                        // halo 16-B granules
  static constexpr int NP = (HGR + NTHR - 1) / NTHR;         // halo LDS-DMA passes
  static constexpr int COP = 32 * NCF;                       // output columns (padded)
  static constexpr int NKT = (9 * CP + 7) / 8;               // packed k-tiles (8 chunks each)
  static constexpr int WBYTES = NKT * COP * 128;
  static constexpr int BUF = HP * PITCH;
  static constexpr int LDS = WBYTES + 2 * BUF + 4 * COP * 4; // + affine [2][COP] / BN-reduce [4][COP]
  static constexpr int OCC = LDS <= 80 * 1024 ? 2 : 1;       // resident blocks per CU
  static constexpr int SS = CP == 8 ? 1 : 2;                 // halo swizzle: chunk ^ ((p >> SS) & (CP-1))
  static constexpr int NST = 2 * NCF;                        // 16-B stores (and operand loads) per lane per tile
  static_assert(CP == 4 || CP == 8, "reduction of 32 or 64 channels");
  static_assert(BM % TW == 0 && LDS <= 160 * 1024 && (2 * 16 * 256 + 256) * 4 <= LDS, "tile");
};

__device__ __forceinline__ u32x4 cd_ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
#else
  (void)r; (void)voff;
  return u32x4{0u, 0u, 0u, 0u};
#endif
}
__device__ __forceinline__ void cd_st16(__amdgpu_buffer_rsrc_t r, uint32_t voff, const u32x4& v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 0);
#else
  (void)r; (void)voff; (void)v;
#endif
}
// two 16-bit values packed into one dword (low = a)
template <typename T> __device__ __forceinline__ uint32_t cd_pack2(float a, float b) {
  T t[2] = {(T)a, (T)b};
  uint32_t u;
  __builtin_memcpy(&u, t, 4);
  return u;
}
// lanes 32-63 of `lo` trade places with lanes 0-31 of `hi` (v_permlane32_swap_b32)
__device__ __forceinline__ void cd_swap(uint32_t& lo, uint32_t& hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
  lo = r[0];
  hi = r[1];
#else
  (void)lo; (void)hi;
#endif
}
// Chan merge of (n, mean, M2) with (nb, mb, qb)
__device__ __forceinline__ void cd_chan(float& n, float& m, float& q, float nb, float mb, float qb) {
  const float nn = n + nb;
  if (nn > 0.f) {
    const float d = mb - m, f = nb / nn;
    m += d * f;
    q += qb + d * d * (n * f);
    n = nn;
  }
}

// Transposed MFMA: A = weights (rows = output channels), B = pixels, so lane (lr, lh) ends a tile
// holding, per 32-channel fragment, channels 8g + 4lh + (0..3) (g = 0..3) of tile pixel 32*wave + lr.
// After packing to 16 bits, one v_permlane32_swap per dword pair gives every lane 8 consecutive
// channels of its pixel (lanes 0-31: 16p..16p+7, lanes 32-63: 16p+8..16p+15, for pair p = g/2): the
// epilogue writes 16-B NHWC chunks straight from registers -- no LDS staging, no barrier -- so one
// wave's epilogue (VALU, stores) overlaps the other waves' MFMAs of the next tile.  BN statistics are
// per-lane Welford moments over the block's tiles (each lane sees one pixel per tile), merged across
// lanes and waves (Chan) once at the end.
// BNR variants run one block per CU (2 waves per SIMD: up to 256 VGPRs, so the per-lane sums never
// spill -- scratch traffic would also break the counted vmcnt waits)
template <typename T, int TW, int CP, int NCF, int MODE, int EPI, bool BNR = false>
__global__ __launch_bounds__(512, (BNR ? 2 : 2 * DirGeo<TW, CP, NCF>::OCC)) void conv_direct_kernel(DirectParams p) {
  static_assert(!BNR || MODE == MODE_DGRAD, "the BN-reduce epilogue belongs to the input gradient");
  using G = DirGeo<TW, CP, NCF>;
  constexpr int NTHR = G::NTHR, TH = G::TH, HWD = G::HWD, PITCH = G::PITCH, COP = G::COP, BUF = G::BUF;
  constexpr int ES = (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wts = smem;
  char* const bufs = smem + G::WBYTES;
  float* const prm = reinterpret_cast<float*>(smem + G::WBYTES + 2 * BUF);   // [2][COP]: scale, shift

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int Gn = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, Gn);
  if (lb >= p.ntiles) return;   // (the host grid never exceeds the tile count)

  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, (int)p.src_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc((void*)p.dst, (short)0, (int)p.dst_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_res = __builtin_amdgcn_make_buffer_rsrc((void*)p.res, (short)0, (int)p.res_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_bz = __builtin_amdgcn_make_buffer_rsrc((void*)p.bz, (short)0, (int)p.bz_bytes, NT_RSRC3);

  // ---- resident weights: [kt][COP rows][128 B], chunk c of row r at slot c ^ ((r >> 1) & 7) ----
  {
    const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)p.wp, (short)0, 0x7fffffff, NT_RSRC3);
    constexpr int WGR = G::NKT * COP * 8, WPASS = (WGR + NTHR - 1) / NTHR;
#pragma unroll
    for (int j = 0; j < WPASS; ++j) {
      const int g = j * NTHR + tid;
      if (WGR % NTHR == 0 || g < WGR) {
        const int kt = g / (COP * 8), r = (g >> 3) % COP, slot = g & 7;
        const int c = slot ^ ((r >> 1) & 7);
        blds16(rs_w, wts + j * NTHR * 16 + wv * 1024, (uint32_t)((r * p.nkt * 8 + kt * 8 + c) * 16));
      }
    }
  }
  if constexpr (EPI == EPI_AFFINE) {
    if (tid < COP) {
      const bool cv = tid < p.Ncols;
      prm[tid] = (cv && p.scale) ? p.scale[tid] : 1.0f;
      prm[COP + tid] = (cv && p.shift) ? p.shift[tid] : 0.0f;
    }
  }
  if constexpr (BNR) {
    // the producer's BN parameters [scale | shift | mean | invstd] of the dx channels
    if (tid < COP) {
      const bool cv = tid < p.Ncols;
      prm[tid] = cv ? p.bsc[tid] : 0.0f;
      prm[COP + tid] = cv ? p.bsh[tid] : 0.0f;
      prm[2 * COP + tid] = cv ? p.bmi[tid] : 0.0f;
      prm[3 * COP + tid] = cv ? p.bmi[p.Ncols + tid] : 0.0f;
    }
  }

  auto tile_pos = [&](int t, int& n, int& tyi, int& txi) {
    txi = t % p.tiles_x;
    const int r = t / p.tiles_x;
    tyi = r % p.tiles_y;
    n = r / p.tiles_y;
  };

  // ---- halo loader: granule g = j*NTHR + tid of the halo image -> pixel g / CP, slot g % CP ----
  int hl_hy[G::NP], hl_hx[G::NP], hl_c[G::NP];
#pragma unroll
  for (int j = 0; j < G::NP; ++j) {
    const int g = j * NTHR + tid;
    const int px = g / CP, slot = g % CP;
    hl_hy[j] = px / HWD;
    hl_hx[j] = px - (px / HWD) * HWD;
    hl_c[j] = (slot ^ ((px >> G::SS) & (CP - 1))) * 16;
  }
  auto issue_halo = [&](int t, int b) {
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
    const int y0 = tyi * TH - 1, x0 = txi * TW - 1;
    const int pix0 = (n * p.H + y0) * p.W + x0;
    char* base = bufs + b * BUF + wv * 1024;
#pragma unroll
    for (int j = 0; j < G::NP; ++j) {
      const int iy = y0 + hl_hy[j], ix = x0 + hl_hx[j];
      const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const uint32_t vo =
          ok ? (uint32_t)(((pix0 + hl_hy[j] * p.W + hl_hx[j]) * p.src_ld + p.src_off) * ES + hl_c[j]) : NT_OOB;
      if (G::HGR % NTHR == 0 || j + 1 < G::NP || j * NTHR + tid < G::HGR)
        blds16(rs_src, base + j * NTHR * 16, vo);
    }
  };

  // ---- this lane's output pixel (tile row 32*wave + lr) and its 16-B chunks (frag cf, pair pp) ----
  const int hr = wave * 32 + lr;
  const int oty = hr / TW, otx = hr - (hr / TW) * TW;
  auto out_off = [&](int n, int tyi, int txi, int cf, int pp, int ld, int off, bool& ok) -> uint32_t {
    const int oy = tyi * TH + oty;
    const int c0 = cf * 32 + 16 * pp + 8 * lh;
    ok = oy < p.H && c0 < p.Ncols;
    return (uint32_t)((((n * p.H + oy) * p.W + txi * TW + otx) * ld + off + c0) * ES);
  };

  // ---- MFMA fragment addressing (tile-independent) ----
  const int hp0 = oty * HWD + otx;                       // this lane's halo pixel at tap (0, 0)
  int bb[NCF];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) {
    const int col = cf * 32 + lr;
    bb[cf] = col * 128 + ((lh ^ ((col >> 1) & 7)) << 4);
  }

  // per-lane Welford moments of this lane's channels (training forward)
  float wn = 0.f;
  float wm[NCF][16], wq[NCF][16];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      wm[cf][i] = 0.f;
      wq[cf][i] = 0.f;
    }

  const int my_tiles = (p.ntiles - lb + Gn - 1) / Gn;
  const bool has_rv = (EPI == EPI_AFFINE && p.res != nullptr) || EPI == EPI_ACCUM;
  const bool has_ops = has_rv || BNR;
  u32x4 rv[NCF][2];      // residual / accumulate operands of the next epilogue
  u32x4 zv[BNR ? NCF : 1][2];   // BNR: the producer's z at the next epilogue's dx chunks
  float bs1[BNR ? NCF : 1][16], bs2[BNR ? NCF : 1][16];   // BNR: per-lane sums of da, da * xhat
  if constexpr (BNR) {
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        bs1[cf][i] = 0.f;
        bs2[cf][i] = 0.f;
      }
  }
  auto load_ops = [&](int t) {
    if (!has_ops) return;
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        bool ok;
        if (has_rv) {
          const uint32_t o = EPI == EPI_ACCUM ? out_off(n, tyi, txi, cf, pp, p.dst_ld, p.dst_off, ok)
                                              : out_off(n, tyi, txi, cf, pp, p.res_ld, p.res_off, ok);
          rv[cf][pp] = cd_ld16(EPI == EPI_ACCUM ? rs_dst : rs_res, ok ? o : NT_OOB);
        }
        if constexpr (BNR) {
          const uint32_t o = out_off(n, tyi, txi, cf, pp, p.bz_ld, p.bz_off, ok);
          zv[cf][pp] = cd_ld16(rs_bz, ok ? o : NT_OOB);
        }
      }
  };

  f32x16 acc[NCF];
  // k-steps in groups of KG (a whole tap, or half a tap where the statistics moments need the
  // registers); group g + 1's fragments are read while group g's MFMAs run
  constexpr int KS = 9 * CP / 2, KG = (CP == 8 && NCF == 2) ? 2 : CP / 2, NG = KS / KG;
  auto compute = [&](int b) {
    const char* Hb = bufs + b * BUF;
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[cf][i] = 0.0f;
    u32x4 af[2][KG], bf[2][KG][NCF];
    auto frags = [&](int grp, int slot) {
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        const int ks = grp * KG + j, tap = ks / (CP / 2), kc = ks % (CP / 2);
        const int dy = tap / 3, dx = tap % 3;
        const int toff = MODE == MODE_FWD ? dy * HWD + dx : (2 - dy) * HWD + (2 - dx);
        const int hp = hp0 + toff;
        const int ab = hp * PITCH + ((lh ^ ((hp >> G::SS) & (CP - 1))) << 4);
        af[slot][j] = *reinterpret_cast<const u32x4*>(Hb + (ab ^ (kc << 5)));
        const int q0 = tap * CP + 2 * kc, kt = q0 >> 3, cw0 = q0 & 7;
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
          bf[slot][j][cf] = *reinterpret_cast<const u32x4*>(wts + kt * COP * 128 + (bb[cf] ^ (cw0 << 4)));
      }
    };
    frags(0, 0);
#pragma unroll
    for (int grp = 0; grp < NG; ++grp) {
      // scheduling fences: the compiler would otherwise sink each read next to its MFMA (and wait
      // out the LDS latency there)
      __builtin_amdgcn_sched_barrier(0);
      if (grp + 1 < NG) frags(grp + 1, (grp + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < KG; ++j)
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
          acc[cf] = Mfma<T>::mma(bf[grp & 1][j][cf], af[grp & 1][j], acc[cf]);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // epilogue of tile t from the accumulators (operands in rv, waited for by the caller)
  auto epilogue = [&](int t) {
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
    const bool pix_ok = tyi * TH + oty < p.H;
    if constexpr (EPI == EPI_STATS) {
      if (pix_ok) {
        wn += 1.f;
        const float inv = 1.0f / wn;
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float x = acc[cf][i];
            const float d = x - wm[cf][i];
            wm[cf][i] += d * inv;
            wq[cf][i] += d * (x - wm[cf][i]);
          }
      }
    }
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf) {
      float sc[16], sh[16];
      if constexpr (EPI == EPI_AFFINE) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 a = *reinterpret_cast<const float4*>(prm + cf * 32 + 8 * g + 4 * lh);
          const float4 c = *reinterpret_cast<const float4*>(prm + COP + cf * 32 + 8 * g + 4 * lh);
          sc[4 * g] = a.x; sc[4 * g + 1] = a.y; sc[4 * g + 2] = a.z; sc[4 * g + 3] = a.w;
          sh[4 * g] = c.x; sh[4 * g + 1] = c.y; sh[4 * g + 2] = c.z; sh[4 * g + 3] = c.w;
        }
      }
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        float v[8];   // groups 2pp (v[0..3]) and 2pp+1 (v[4..7]) of this lane
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * pp + j;
          float x = acc[cf][i];
          if constexpr (EPI == EPI_AFFINE) {
            x = x * sc[i] + sh[i];
            if (p.act == YMS_ACT_SILU) x = silu_f(x);
          }
          v[j] = x;
        }
        uint32_t a0 = cd_pack2<T>(v[0], v[1]), a1 = cd_pack2<T>(v[2], v[3]);
        uint32_t b0 = cd_pack2<T>(v[4], v[5]), b1 = cd_pack2<T>(v[6], v[7]);
        cd_swap(a0, b0);
        cd_swap(a1, b1);
        u32x4 ov = {a0, a1, b0, b1};     // channels cf*32 + 16pp + 8lh + (0..7)
        if (has_rv) {
          float f[8], r[8];
          unpack8(*reinterpret_cast<const Raw8<T>*>(&ov), f);
          unpack8(*reinterpret_cast<const Raw8<T>*>(&rv[cf][pp]), r);
          ov = u32x4{cd_pack2<T>(f[0] + r[0], f[1] + r[1]), cd_pack2<T>(f[2] + r[2], f[3] + r[3]),
                     cd_pack2<T>(f[4] + r[4], f[5] + r[5]), cd_pack2<T>(f[6] + r[6], f[7] + r[7])};
        }
        bool ok;
        const uint32_t off = out_off(n, tyi, txi, cf, pp, p.dst_ld, p.dst_off, ok);
        cd_st16(rs_dst, ok ? off : NT_OOB, ov);
        if constexpr (BNR) {
          if (ok) {     // the stored (rounded) gradient, as the separate reduce pass would read it
            float g[8];
            unpack8(*reinterpret_cast<const Raw8<T>*>(&ov), g);
            cd_bnred<T>(g, zv[cf][pp], prm, COP, cf * 32 + 16 * pp + 8 * lh, p.bact, &bs1[cf][8 * pp],
                        &bs2[cf][8 * pp]);
          }
        }
      }
    }
  };

  // vector-memory order per wave (the counted waits below rely on it):
  //   prologue: halo(lb) (drained), ops(lb), halo(lb + G);
  //   tile t: [barrier] halo(t + G), compute, wait(ops(t)), epilogue(t) stores, ops(t + G)
  // (measured: running waves 4-7's epilogue one tile late, so that one wave's VALU epilogue issues
  // beside its SIMD partner's MFMAs, was neutral to -8 %: the layers are bound by the halo and
  // output bytes per CU in flight, not by the epilogue)
  issue_halo(lb, 0);
  wait_vmcnt<0>();
  __syncthreads();                               // weights, halo(lb), affine parameters visible
  load_ops(lb);
  if (my_tiles > 1) issue_halo(lb + Gn, 1);

  for (int it = 0, t = lb; it < my_tiles; ++it, t += Gn) {
    const int b = it & 1;
    const bool has_next = it + 1 < my_tiles;
    if (it > 0) {
      // this wave's halo(t) DMAs have landed: younger are the last epilogue's stores and the next
      // epilogue's operand loads (residual / accumulate operand, BNR: the producer's z)
      if (has_rv && BNR) wait_vmcnt<3 * G::NST>();
      else if (has_ops) wait_vmcnt<2 * G::NST>();
      else wait_vmcnt<G::NST>();
      __builtin_amdgcn_s_waitcnt((0xF) | (3 << 14) | (0x7 << 4) | (0 << 8));   // lgkmcnt(0)
      raw_barrier();     // halo(t) visible everywhere; every wave is done reading buffer b ^ 1
      if (has_next) issue_halo(t + Gn, b ^ 1);
    }
    compute(b);
    if (has_ops) {
      if (has_next) wait_vmcnt<G::NP - 1>();   // ops(t); halo(t + G) may stay in flight
      else wait_vmcnt<0>();
    }
    epilogue(t);
    if (has_next) load_ops(t + Gn);
  }

  if constexpr (BNR) {
    __syncthreads();                                    // weights and halo buffers are free now
    cd_bnred_store<NCF>(bs1, bs2, smem, p.bws, lb, p.Ncols);
  }
  if constexpr (EPI == EPI_STATS) {
    // Merge the 256 per-lane moment sets of each channel (8 waves x 32 lanes of one half) in LDS,
    // 16 channels (one fragment half) per pass, all 512 threads: thread (u, k) sums contributors
    // 8k..8k+7 of channel u, then 32-lane shuffles -- first the count and sum, then the M2 about
    // the merged mean (sum of q_j + n_j (m_j - M)^2): no divisions per contributor.
    __syncthreads();                                    // weights and halo buffers are free now
    float* const mq = reinterpret_cast<float*>(smem);   // [16][256] means, [16][256] M2s, [256] counts
    float* const nl = mq + 2 * 16 * 256;
    const int u = tid >> 5, k = tid & 31;
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (lh == h) {
          const int j = wave * 32 + lr;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            mq[i * 256 + j] = wm[cf][i];
            mq[(16 + i) * 256 + j] = wq[cf][i];
          }
          nl[j] = wn;
        }
        __syncthreads();
        float n = 0.f, sm = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float nj = nl[8 * k + e];
          n += nj;
          sm += nj * mq[u * 256 + 8 * k + e];
        }
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          n += __shfl_xor(n, o);
          sm += __shfl_xor(sm, o);
        }
        const float mean = n > 0.f ? sm / n : 0.f;
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = mq[u * 256 + 8 * k + e] - mean;
          q += mq[(16 + u) * 256 + 8 * k + e] + nl[8 * k + e] * d * d;
        }
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o);
        if (k == 0) {
          const int c = cf * 32 + 8 * (u >> 2) + 4 * h + (u & 3);
          float* so = p.stats + (long)lb * 2 * p.stats_ld;
          so[c] = sm;
          so[p.stats_ld + c] = q;
          if (c == 0) p.stats_cnt[lb] = n;
        }
        __syncthreads();                                  // before the next pass overwrites mq
      }
  }
}

// ------------------------------------------------------------------------------------------
// Stride-2 input gradient (pad 1, k 3) by output parity class, for the same channel range.  For
// dx pixel (2a + ry, 2b + rx) only the taps kh = kh0 + 2jy, kw = kw0 + 2jx contribute (kh0 = 1 - ry,
// jy < 1 + ry; likewise for x), reading dz(a + ry - jy, b + rx - jx): tiles of 256 class positions
// (a, b) need one (TH+1) x (TW+1) halo of dz, and the four classes (1, 2, 2, 4 taps: 9 in all, the
// stride-1 kernel's MFMA work per 256 positions) run one after the other on it, each writing its
// 256 dx pixels.  Weights: the parity-class packing of yms_conv_pack_weight(for_dgrad=1, stride 2).
// ------------------------------------------------------------------------------------------
template <int TW, int CP, int NCF> struct DirGeo2 {
  static constexpr int NTHR = 512, NW = 8, BM = 256, TH = BM / TW;
  static constexpr int HWD = TW + 1, HP = (TH + 1) * HWD;
  static constexpr int PITCH = CP * 16, HGR = HP * CP, NP = (HGR + NTHR - 1) / NTHR;
  static constexpr int COP = 32 * NCF;
  static constexpr int taps(int c) { return (1 + (c >> 1)) * (1 + (c & 1)); }
  static constexpr int nkt(int c) { return (taps(c) * CP + 7) / 8; }
  static constexpr int cumk(int c) { return c == 0 ? 0 : cumk(c - 1) + nkt(c - 1); }
  static constexpr int NKT = cumk(4);
  static constexpr int WBYTES = NKT * COP * 128;
  static constexpr int BUF = HP * PITCH;
  static constexpr int LDS = WBYTES + 2 * BUF + 4 * COP * 4;   // + BN-reduce parameters [4][COP]
  static constexpr int OCC = LDS <= 80 * 1024 ? 2 : 1;
  static constexpr int SS = CP == 8 ? 1 : 2;
  static constexpr int NST = 2 * NCF;                  // 16-B stores per lane per class
  static_assert((CP == 4 || CP == 8) && BM % TW == 0 && LDS <= 160 * 1024, "tile");
};

template <typename T, int TW, int CP, int NCF, int EPI, bool BNR = false>
__global__ __launch_bounds__(512, (BNR ? 2 : 2 * DirGeo2<TW, CP, NCF>::OCC)) void conv_direct_dgrad2_kernel(DirectParams p) {
  using G = DirGeo2<TW, CP, NCF>;
  constexpr int NTHR = G::NTHR, TH = G::TH, HWD = G::HWD, PITCH = G::PITCH, COP = G::COP, BUF = G::BUF;
  constexpr int ES = (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wts = smem;
  char* const bufs = smem + G::WBYTES;
  float* const bnp = reinterpret_cast<float*>(smem + G::WBYTES + 2 * BUF);   // BNR: [4][COP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int Gn = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, Gn);
  if (lb >= p.ntiles) return;

  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, (int)p.src_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc((void*)p.dst, (short)0, (int)p.dst_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_bz = __builtin_amdgcn_make_buffer_rsrc((void*)p.bz, (short)0, (int)p.bz_bytes, NT_RSRC3);
  if constexpr (BNR) {
    if (tid < COP) {
      const bool cv = tid < p.Ncols;
      bnp[tid] = cv ? p.bsc[tid] : 0.0f;
      bnp[COP + tid] = cv ? p.bsh[tid] : 0.0f;
      bnp[2 * COP + tid] = cv ? p.bmi[tid] : 0.0f;
      bnp[3 * COP + tid] = cv ? p.bmi[p.Ncols + tid] : 0.0f;
    }
  }

  // ---- resident weights: class blocks [kt][COP][128 B] (swizzled as in the stride-1 kernel) ----
  {
    const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)p.wp, (short)0, 0x7fffffff, NT_RSRC3);
    constexpr int WGR = G::NKT * COP * 8, WPASS = (WGR + NTHR - 1) / NTHR;
#pragma unroll
    for (int j = 0; j < WPASS; ++j) {
      const int g = j * NTHR + tid;
      if (WGR % NTHR == 0 || g < WGR) {
        const int K = g / (COP * 8), r = (g >> 3) % COP, slot = g & 7;
        const int c = K >= G::cumk(3) ? 3 : K >= G::cumk(2) ? 2 : K >= G::cumk(1) ? 1 : 0;
        const int ktl = K - G::cumk(c);
        const int nk = G::nkt(c);
        const int ch = slot ^ ((r >> 1) & 7);
        const long el = (long)p.wrows * 64 * G::cumk(c) + (long)r * nk * 64;
        blds16(rs_w, wts + j * NTHR * 16 + wv * 1024, (uint32_t)(el * 2 + (ktl * 8 + ch) * 16));
      }
    }
  }
  auto tile_pos = [&](int t, int& n, int& tyi, int& txi) {
    txi = t % p.tiles_x;
    const int r = t / p.tiles_x;
    tyi = r % p.tiles_y;
    n = r / p.tiles_y;
  };
  // ---- dz halo rows a0 .. a0 + TH, columns b0 .. b0 + TW ----
  int hl_hy[G::NP], hl_hx[G::NP], hl_c[G::NP];
#pragma unroll
  for (int j = 0; j < G::NP; ++j) {
    const int g = j * NTHR + tid;
    const int px = g / CP, slot = g % CP;
    hl_hy[j] = px / HWD;
    hl_hx[j] = px - (px / HWD) * HWD;
    hl_c[j] = (slot ^ ((px >> G::SS) & (CP - 1))) * 16;
  }
  auto issue_halo = [&](int t, int b) {
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
    const int y0 = tyi * TH, x0 = txi * TW;
    const int pix0 = (n * p.H + y0) * p.W + x0;      // p.H x p.W: the dz map
    char* base = bufs + b * BUF + wv * 1024;
#pragma unroll
    for (int j = 0; j < G::NP; ++j) {
      const int iy = y0 + hl_hy[j], ix = x0 + hl_hx[j];
      const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const uint32_t vo =
          ok ? (uint32_t)(((pix0 + hl_hy[j] * p.W + hl_hx[j]) * p.src_ld + p.src_off) * ES + hl_c[j]) : NT_OOB;
      if (G::HGR % NTHR == 0 || j + 1 < G::NP || j * NTHR + tid < G::HGR)
        blds16(rs_src, base + j * NTHR * 16, vo);
    }
  };
  const int hr = wave * 32 + lr;
  const int oty = hr / TW, otx = hr - (hr / TW) * TW;
  // dx pixel (2a + ry, 2b + rx) of this lane's position, chunk (cf, pp)
  auto out_off = [&](int n, int tyi, int txi, int cls, int cf, int pp, bool& ok, int ld, int off) -> uint32_t {
    const int oy = 2 * (tyi * TH + oty) + (cls >> 1), ox = 2 * (txi * TW + otx) + (cls & 1);
    const int c0 = cf * 32 + 16 * pp + 8 * lh;
    ok = oy < p.OH && ox < p.OW && c0 < p.Ncols;
    return (uint32_t)((((n * p.OH + oy) * p.OW + ox) * ld + off + c0) * ES);
  };
  int bb[NCF];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) {
    const int col = cf * 32 + lr;
    bb[cf] = col * 128 + ((lh ^ ((col >> 1) & 7)) << 4);
  }

  const int my_tiles = (p.ntiles - lb + Gn - 1) / Gn;
  constexpr bool ACC = EPI == EPI_ACCUM;
  u32x4 rv[ACC ? 4 : 1][NCF][2];
  u32x4 zv[BNR ? 4 : 1][NCF][2];   // BNR: the producer's z at the next tile's dx chunks
  float bs1[BNR ? NCF : 1][16], bs2[BNR ? NCF : 1][16];
  if constexpr (BNR) {
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        bs1[cf][i] = 0.f;
        bs2[cf][i] = 0.f;
      }
  }
  auto load_ops = [&](int t) {
    if constexpr (!ACC && !BNR) return;
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          bool ok;
          if constexpr (ACC) {
            const uint32_t o = out_off(n, tyi, txi, c, cf, pp, ok, p.dst_ld, p.dst_off);
            rv[c][cf][pp] = cd_ld16(rs_dst, ok ? o : NT_OOB);
          }
          if constexpr (BNR) {
            const uint32_t o = out_off(n, tyi, txi, c, cf, pp, ok, p.bz_ld, p.bz_off);
            zv[c][cf][pp] = cd_ld16(rs_bz, ok ? o : NT_OOB);
          }
        }
  };

  f32x16 acc[NCF];
  auto compute = [&](int b, auto cls_c) {
    constexpr int c = decltype(cls_c)::value;
    constexpr int ry = c >> 1, rx = c & 1, ntx = 1 + rx, taps = G::taps(c);
    constexpr int KS = taps * CP / 2, KG = CP / 2, NG = KS / KG;
    const char* Hb = bufs + b * BUF;
    const char* Wc = wts + G::cumk(c) * COP * 128;
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[cf][i] = 0.0f;
    u32x4 af[2][KG], bf[2][KG][NCF];
    auto frags = [&](int grp, int slot) {
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        const int ks = grp * KG + j, tl = ks / (CP / 2), kc = ks % (CP / 2);
        const int jy = tl / ntx, jx = tl % ntx;
        const int hp = (oty + ry - jy) * HWD + (otx + rx - jx);
        const int ab = hp * PITCH + ((lh ^ ((hp >> G::SS) & (CP - 1))) << 4);
        af[slot][j] = *reinterpret_cast<const u32x4*>(Hb + (ab ^ (kc << 5)));
        const int q0 = tl * CP + 2 * kc, kt = q0 >> 3, cw0 = q0 & 7;
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
          bf[slot][j][cf] = *reinterpret_cast<const u32x4*>(Wc + kt * COP * 128 + (bb[cf] ^ (cw0 << 4)));
      }
    };
    frags(0, 0);
#pragma unroll
    for (int grp = 0; grp < NG; ++grp) {
      __builtin_amdgcn_sched_barrier(0);
      if (grp + 1 < NG) frags(grp + 1, (grp + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < KG; ++j)
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf) acc[cf] = Mfma<T>::mma(bf[grp & 1][j][cf], af[grp & 1][j], acc[cf]);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto epilogue = [&](int t, int c) {
    int n, tyi, txi;
    tile_pos(t, n, tyi, txi);
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int i0 = 8 * pp;
        uint32_t a0 = cd_pack2<T>(acc[cf][i0], acc[cf][i0 + 1]), a1 = cd_pack2<T>(acc[cf][i0 + 2], acc[cf][i0 + 3]);
        uint32_t b0 = cd_pack2<T>(acc[cf][i0 + 4], acc[cf][i0 + 5]), b1 = cd_pack2<T>(acc[cf][i0 + 6], acc[cf][i0 + 7]);
        cd_swap(a0, b0);
        cd_swap(a1, b1);
        u32x4 ov = {a0, a1, b0, b1};
        if constexpr (ACC) {
          float f[8], r[8];
          unpack8(*reinterpret_cast<const Raw8<T>*>(&ov), f);
          unpack8(*reinterpret_cast<const Raw8<T>*>(&rv[c][cf][pp]), r);
          ov = u32x4{cd_pack2<T>(f[0] + r[0], f[1] + r[1]), cd_pack2<T>(f[2] + r[2], f[3] + r[3]),
                     cd_pack2<T>(f[4] + r[4], f[5] + r[5]), cd_pack2<T>(f[6] + r[6], f[7] + r[7])};
        }
        bool ok;
        const uint32_t off = out_off(n, tyi, txi, c, cf, pp, ok, p.dst_ld, p.dst_off);
        cd_st16(rs_dst, ok ? off : NT_OOB, ov);
        if constexpr (BNR) {
          if (ok) {
            float g[8];
            unpack8(*reinterpret_cast<const Raw8<T>*>(&ov), g);
            cd_bnred<T>(g, zv[c][cf][pp], bnp, COP, cf * 32 + 16 * pp + 8 * lh, p.bact, &bs1[cf][8 * pp],
                        &bs2[cf][8 * pp]);
          }
        }
      }
  };

  // vector-memory order per wave: prologue halo(lb) (drained), ops(lb), halo(lb + G); tile t:
  // [barrier] halo(t + G), 4 x (compute, epilogue stores), ops(t + G)
  issue_halo(lb, 0);
  wait_vmcnt<0>();
  __syncthreads();
  load_ops(lb);
  if (my_tiles > 1) issue_halo(lb + Gn, 1);
  for (int it = 0, t = lb; it < my_tiles; ++it, t += Gn) {
    const int b = it & 1;
    const bool has_next = it + 1 < my_tiles;
    if (it > 0) {
      // younger than halo(t): 4 classes' stores (+ ops(t): accumulate operands, BNR z)
      wait_vmcnt<(4 + (ACC ? 4 : 0) + (BNR ? 4 : 0)) * G::NST>();
      __builtin_amdgcn_s_waitcnt((0xF) | (3 << 14) | (0x7 << 4) | (0 << 8));   // lgkmcnt(0)
      raw_barrier();
      if (has_next) issue_halo(t + Gn, b ^ 1);
    }
    compute(b, std::integral_constant<int, 0>{});
    if constexpr (ACC || BNR) {
      if (has_next) wait_vmcnt<G::NP - 1>();     // ops(t); halo(t + G) may stay in flight
      else wait_vmcnt<0>();
    }
    epilogue(t, 0);
    compute(b, std::integral_constant<int, 1>{});
    epilogue(t, 1);
    compute(b, std::integral_constant<int, 2>{});
    epilogue(t, 2);
    compute(b, std::integral_constant<int, 3>{});
    epilogue(t, 3);
    if (has_next) load_ops(t + Gn);
  }
  if constexpr (BNR) {
    __syncthreads();
    cd_bnred_store<NCF>(bs1, bs2, smem, p.bws, lb, p.Ncols);
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
template <template <int, int, int> class GEO>
static int direct_occ(int tw, int cp, int ncf) {
  if (tw == 32) {
    if (cp == 8) return ncf == 2 ? GEO<32, 8, 2>::OCC : GEO<32, 8, 1>::OCC;
    return ncf == 2 ? GEO<32, 4, 2>::OCC : GEO<32, 4, 1>::OCC;
  }
  if (cp == 8) return ncf == 2 ? GEO<16, 8, 2>::OCC : GEO<16, 8, 1>::OCC;
  return ncf == 2 ? GEO<16, 4, 2>::OCC : GEO<16, 4, 1>::OCC;   // (constants only: nothing launched)
}

// Route switch, read ONCE per process from YMS_DIRECT (0 = off) and changed only through
// yms_conv_direct_set: the route decides how many statistics rows a forward writes
// (yms_conv_stats_rows), which a plan sizes when it is built, so it must not flip under a plan.
static int& direct_route() {
  static int on = [] {
    const char* e = getenv("YMS_DIRECT");
    return (e && atoi(e) == 0) ? 0 : 1;
  }();
  return on;
}

bool conv_direct_geometry(const yms_conv_shape* s, int mode, DirectGeo* g, bool bnred) {
  if (!direct_route()) return false;
  if (!s || s->dtype == YMS_F32 || s->k != 3 || s->pad != 1) return false;
  const bool s2 = s->stride == 2;
  if (s2 ? (mode != 1 || s->ho != (s->h + 1) / 2 || s->wo != (s->w + 1) / 2)
         : (s->stride != 1 || s->ho != s->h || s->wo != s->w))
    return false;
  const int cr = mode == 0 ? s->cin : s->cout;      // reduction channels
  const int co = mode == 0 ? s->cout : s->cin;      // output channels
  const int cr8 = (int)rup(cr, 8);
  if (!(cr8 == 32 || cr8 == 64) || co % 8 != 0 || co > 64) return false;
  DirectGeo q{};
  const int gw = s->wo, gh = s->ho;                 // tile grid: output map, or the class positions
  if (gw % 32 == 0) q.TW = 32;
  else if (gw % 16 == 0) q.TW = 16;
  else return false;
  q.TH = 256 / q.TW;
  q.CP = cr8 / 8;
  q.NCF = co <= 32 ? 1 : 2;
  q.S2 = s2;
  if (s2 && q.CP == 4 && q.NCF == 2) return false;   // not instantiated (launch_dgrad2_t)
  q.tiles_x = gw / q.TW;
  q.tiles_y = cdiv(gh, q.TH);
  q.ntiles = (long)s->n * q.tiles_x * q.tiles_y;
  if (q.ntiles >= (1l << 30)) return false;
  // the BN-reduce epilogue: 32-channel output fragments only (two fragments' sums, operands and
  // fragments exceed 256 VGPRs), one block per CU
  if (bnred && (mode != 1 || q.NCF != 1)) return false;
  const int occ = bnred ? 1 : s2 ? direct_occ<DirGeo2>(q.TW, q.CP, q.NCF) : direct_occ<DirGeo>(q.TW, q.CP, q.NCF);
  q.grid = (int)std::max<long>(1, std::min<long>(q.ntiles, (long)occ * conv_cu_count()));
  *g = q;
  return true;
}

template <typename T, int TW, int CP, int NCF, int MODE, int EPI, bool BNR = false>
static void launch_direct(const DirectParams& p, int grid, hipStream_t st) {
  using G = DirGeo<TW, CP, NCF>;
  auto k = conv_direct_kernel<T, TW, CP, NCF, MODE, EPI, BNR>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(G::NTHR), G::LDS, st, p);
}

template <typename T, int TW, int CP, int NCF>
static void launch_direct_epi(const DirectParams& p, int mode, int epi, int grid, hipStream_t st) {
  if (mode == 0) {
    if (epi == EPI_STATS) launch_direct<T, TW, CP, NCF, MODE_FWD, EPI_STATS>(p, grid, st);
    else launch_direct<T, TW, CP, NCF, MODE_FWD, EPI_AFFINE>(p, grid, st);
  } else if (p.bws) {
    if constexpr (NCF == 1) {     // (conv_direct_geometry admits the BN-reduce epilogue on NCF = 1 only)
      if (epi == EPI_ACCUM) launch_direct<T, TW, CP, NCF, MODE_DGRAD, EPI_ACCUM, true>(p, grid, st);
      else launch_direct<T, TW, CP, NCF, MODE_DGRAD, EPI_STORE, true>(p, grid, st);
    }
  } else {
    if (epi == EPI_ACCUM) launch_direct<T, TW, CP, NCF, MODE_DGRAD, EPI_ACCUM>(p, grid, st);
    else launch_direct<T, TW, CP, NCF, MODE_DGRAD, EPI_STORE>(p, grid, st);
  }
}

template <typename T, int TW, int CP, int NCF, int EPI, bool BNR>
static void launch_dgrad2_k(const DirectParams& p, int grid, hipStream_t st) {
  using G = DirGeo2<TW, CP, NCF>;
  auto k = conv_direct_dgrad2_kernel<T, TW, CP, NCF, EPI, BNR>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(G::NTHR), G::LDS, st, p);
}

template <typename T, int TW, int CP, int NCF>
static void launch_dgrad2(const DirectParams& p, int epi, int grid, hipStream_t st) {
  if (p.bws) {
    if constexpr (NCF == 1) {
      if (epi == EPI_ACCUM) launch_dgrad2_k<T, TW, CP, NCF, EPI_ACCUM, true>(p, grid, st);
      else launch_dgrad2_k<T, TW, CP, NCF, EPI_STORE, true>(p, grid, st);
    }
  } else {
    if (epi == EPI_ACCUM) launch_dgrad2_k<T, TW, CP, NCF, EPI_ACCUM, false>(p, grid, st);
    else launch_dgrad2_k<T, TW, CP, NCF, EPI_STORE, false>(p, grid, st);
  }
}

// (32 reduction channels with 33..64 outputs is not instantiated: at two blocks per CU its four
// classes' accumulate operands do not fit the registers; conv_direct_geometry routes it to the NT kernel)
template <typename T>
static void launch_dgrad2_t(const DirectGeo& g, const DirectParams& p, int epi, hipStream_t st) {
  if (g.TW == 32) {
    if (g.CP == 8) {
      if (g.NCF == 2) launch_dgrad2<T, 32, 8, 2>(p, epi, g.grid, st);
      else launch_dgrad2<T, 32, 8, 1>(p, epi, g.grid, st);
    } else {
      launch_dgrad2<T, 32, 4, 1>(p, epi, g.grid, st);
    }
  } else {
    if (g.CP == 8) {
      if (g.NCF == 2) launch_dgrad2<T, 16, 8, 2>(p, epi, g.grid, st);
      else launch_dgrad2<T, 16, 8, 1>(p, epi, g.grid, st);
    } else {
      launch_dgrad2<T, 16, 4, 1>(p, epi, g.grid, st);
    }
  }
}

template <typename T>
static void launch_direct_t(const DirectGeo& g, const DirectParams& p, int mode, int epi, hipStream_t st) {
  if (g.S2) {
    launch_dgrad2_t<T>(g, p, epi, st);
    return;
  }
  if (g.TW == 32) {
    if (g.CP == 8) {
      if (g.NCF == 2) launch_direct_epi<T, 32, 8, 2>(p, mode, epi, g.grid, st);
      else launch_direct_epi<T, 32, 8, 1>(p, mode, epi, g.grid, st);
    } else {
      if (g.NCF == 2) launch_direct_epi<T, 32, 4, 2>(p, mode, epi, g.grid, st);
      else launch_direct_epi<T, 32, 4, 1>(p, mode, epi, g.grid, st);
    }
  } else {
    if (g.CP == 8) {
      if (g.NCF == 2) launch_direct_epi<T, 16, 8, 2>(p, mode, epi, g.grid, st);
      else launch_direct_epi<T, 16, 8, 1>(p, mode, epi, g.grid, st);
    } else {
      if (g.NCF == 2) launch_direct_epi<T, 16, 4, 2>(p, mode, epi, g.grid, st);
      else launch_direct_epi<T, 16, 4, 1>(p, mode, epi, g.grid, st);
    }
  }
}

yms_status conv_direct_launch(const yms_conv_shape* s, int mode, const DirectGeo& g, const void* src, int src_ld,
                              int src_off, const void* wpacked, void* dst, int dst_ld, int dst_off,
                              const float* scale, const float* shift, int act, const void* res, int res_ld,
                              int res_off, float* stats, int accumulate, hipStream_t st, const DirectBnRed* bnr) {
  DirectParams p{};
  if (bnr) {
    if (mode != 1 || !bnr->z || !bnr->scale || !bnr->shift || !bnr->mean_invstd || !bnr->ws) return YMS_ERR_INVALID;
    const long zb = (long)s->n * s->h * s->w * bnr->z_ld * 2;
    if (zb >= (1l << 31) - (1l << 20)) return YMS_ERR_UNSUPPORTED;
    p.bz = (const char*)bnr->z;
    p.bz_ld = bnr->z_ld;
    p.bz_off = bnr->z_off;
    p.bz_bytes = (uint32_t)zb;
    p.bsc = bnr->scale;
    p.bsh = bnr->shift;
    p.bmi = bnr->mean_invstd;
    p.bact = bnr->act;
    p.bws = bnr->ws;
  }
  p.src = (const char*)src;
  p.wp = (const char*)wpacked;
  p.dst = (char*)dst;
  p.res = (const char*)res;
  p.src_ld = src_ld; p.src_off = src_off; p.dst_ld = dst_ld; p.dst_off = dst_off;
  p.res_ld = res_ld; p.res_off = res_off;
  p.scale = scale; p.shift = shift; p.act = act;
  // source map: x (forward) or dz (input gradient); output map: y or dx
  p.H = mode == 0 ? s->h : s->ho; p.W = mode == 0 ? s->w : s->wo;
  p.OH = mode == 0 ? s->ho : s->h; p.OW = mode == 0 ? s->wo : s->w;
  p.tiles_x = g.tiles_x; p.tiles_y = g.tiles_y; p.ntiles = (int)g.ntiles;
  p.Ncols = mode == 0 ? s->cout : s->cin;
  p.nkt = (9 * g.CP + 7) / 8;      // the packed row pitch of yms_conv_pack_weight (fwd and stride-1 dgrad)
  p.wrows = (int)rup(p.Ncols, 128);  // rows of the stride-2 class blocks (yms_conv_pack_weight, dg2_geo)
  const long spix = (long)s->n * p.H * p.W, opix = (long)s->n * p.OH * p.OW;
  const long sb = spix * src_ld * 2, db = opix * dst_ld * 2, rb = res ? opix * res_ld * 2 : 0;
  const long lim = (1l << 31) - (1l << 20);
  if (sb >= lim || db >= lim || rb >= lim) return YMS_ERR_UNSUPPORTED;
  p.src_bytes = (uint32_t)sb;
  p.dst_bytes = (uint32_t)db;
  p.res_bytes = (uint32_t)rb;
  int epi;
  if (mode == 0) {
    epi = stats ? EPI_STATS : EPI_AFFINE;
    if (stats) {
      p.stats = stats;
      p.stats_ld = (int)rup(s->cout, 128);
      p.stats_cnt = stats + (long)g.grid * 2 * p.stats_ld;
    }
  } else {
    epi = accumulate ? EPI_ACCUM : EPI_STORE;
  }
  if (s->dtype == YMS_BF16) launch_direct_t<bf16>(g, p, mode, epi, st);
  else launch_direct_t<f16>(g, p, mode, epi, st);
  return launch_status();
}

}  // namespace yms

extern "C" int yms_conv_direct_set(int on) {
  const int prev = yms::direct_route();
  if (on >= 0) yms::direct_route() = on ? 1 : 0;
  return prev;
}

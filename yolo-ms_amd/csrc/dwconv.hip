// Depthwise k x k convolution (groups = channels, stride 1, pad k/2, k = 3/5/7/9) for gfx950,
// NHWC, the large-kernel mid conv of the YOLO-MS MS-Block inverted bottleneck (SURVEY 7.4:
// IB_k = 1x1 expand -> depthwise k x k -> 1x1 project; heterogeneous kernel sizes 3/5/7/9 per
// backbone stage, the "HKS" of the paper; the reference holds the MS-Block only as a diagram,
// annotations.md:66-133).  Forward / dgrad: VALU + LDS, bounded by HBM (k = 3, 5) or by the VALU
// FMA rate (k = 7, 9); the k = 5 / 7 / 9 weight gradient on maps up to 64 (k = 5: 96) wide runs on MFMA as a
// band-diagonal product (dwconv_wgrad_mfma_kernel).
//
// Mapping: a 256-thread block owns a TY x TX = 8 x 32 output tile of one image and 32 channels;
// wave w owns 8 channels (one 16-B NHWC chunk), lane (ty, qx) = (lane / 8, lane % 8) owns the
// RX = 4 consecutive pixels (ty, 4 qx .. 4 qx + 3).  Forward and dgrad blocks walk a vertical
// strip of such tiles; the input rows (32 + k - 1 wide, zero outside the image) live in an LDS
// ring, and the rows of the next tile are loaded while the current one computes.  Per kernel row a
// lane slides an (RX + k - 1)-pixel window over its row and accumulates RX outputs in fp32.
//   forward: y = act(conv * scale + shift) (eval, BN folded) | z + per-tile BN partial sums (train)
//   dgrad  : dx (+)= conv(dz, rot180(w))
//   wgrad  : dw[c][t] = sum_p x[p + d_t][c] dz[p][c]: per-lane (kernel row, tile row, column
//            segment) register partials across all of a block's tiles, one fixed-order LDS
//            reduction per block, per-block rows + fixed-order reduce
#include <algorithm>
#include <cstdlib>

#include "conv_common.hpp"

namespace yms {

constexpr int DW_TY = 8, DW_TX = 32, DW_RX = 4, DW_G = 4, DW_CB = DW_G * 8;   // 32 channels per block
constexpr int DW_FEW_ROWS = 32;   // weight-gradient partial rows summed by the one-pass reduce
constexpr int DW_WGM_CG = 16;     // channels per dwconv_wgrad_mfma_kernel block
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
  int ysplit, tps;       // forward / dgrad: strips per image column of tiles, tiles per strip
  int ncg, nlog;         // strip kernels: channel groups, logical blocks (see dw_block)
};

// logical (spatial block bx, channel group by) of a strip kernel's 1-D launch: channel groups
// fastest and the grid padded to a multiple of 8 so consecutive logical blocks run on one XCD
// (block i runs on XCD i % 8) -- the channel groups of one tile read the same 128-B lines of each
// NHWC pixel through one L2, instead of each group streaming the whole map separately (a map larger
// than the 256-MB Infinity Cache was then fetched from HBM once per group)
__device__ __forceinline__ bool dw_block(const DwParams& p, int& bx, int& by) {
  const int l = (int)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
  if (l >= p.nlog) return false;
  by = l % p.ncg;
  bx = l / p.ncg;
  return true;
}

// LDS row stride (16-B chunks) for rows of n chunks: one chunk of padding when n is a multiple
// of 4 (a 64-B multiple: rows read by one wave's lanes would start in the same banks); other
// widths already stagger (k = 3 and 7 halos), and the k = 3 ring must stay at 4 blocks per CU
constexpr int dw_rs(int n) { return n % 4 == 0 ? n + 1 : n; }

// stage the (TY + K - 1) x (TX + K - 1) halo of 32 channels (zero outside the image / past C)
// into rows of dw_rs(HW) chunks
template <typename T, int K, int NT = 256>
__device__ __forceinline__ void dw_stage_halo(const DwParams& p, Raw8<T>* lds, int n, int y0, int x0, int c0) {
  constexpr int HH = DW_TY + K - 1, HW = DW_TX + K - 1, P = K / 2, RS = dw_rs(HW);
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
    lds[(g * HH + hy) * RS + hx] = v;
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// one input row (image row y, halo columns x0 - P .. x0 + TX - 1 + P, the wave's 8 channels c) into
// an LDS ring row (wave-uniform LDS byte address lds_row) by LDS-DMA, 16 B per lane, no registers;
// out-of-image columns / rows and channels past C read as zeros through the buffer range check.
// Inline asm on purpose: hipcc treats its own LDS-DMA as a pending write to the whole LDS object
// and waits vmcnt(0) before the next ds_read, which would serialise this prefetch with the FMAs of
// the current tile (the ring slots written and read are disjoint by construction); completion is
// counted by hand (wait_vmcnt<0> + barrier at the end of each tile).  M0 is saved and restored in
// the same statement (it is compiler-reserved).
template <typename T, int K, int TX = DW_TX>
__device__ __forceinline__ void dw_row_dma(i32x4 rs, uint32_t lds_row, int y, int x0, int c, int H, int W, int C,
                                           int ld, int lane) {
  constexpr int CPE = (int)sizeof(T) / 2, NCH = (TX + K - 1) * CPE;
#pragma unroll
  for (int j0 = 0; j0 < NCH; j0 += 64) {
    const int j = j0 + lane;
    if (j < NCH) {
      const int hx = j / CPE, part = j - hx * CPE;
      const int x = x0 + hx - K / 2;
      uint32_t vo = NT_OOB;
      if (y >= 0 && y < H && x >= 0 && x < W && c < C)
        vo = ((uint32_t)(y * W + x) * (uint32_t)ld + (uint32_t)c) * (uint32_t)sizeof(T) + 16u * part;
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(vo), "s"(rs), "s"(lds_row + 16u * j0)
                   : "memory");
    }
  }
}

// forward / dgrad: a block walks a vertical strip of tiles (p.tps tiles of one image column tile
// and 32 channels), keeping the input rows in an LDS ring of RB = 2 TY + K - 1 rows: tile t reads
// rows y0 - P .. y0 + TY - 1 + P while the TY rows the next tile adds stream into the other ring
// slots by LDS-DMA (issued before the tile's FMAs, waited for at the tile's end), so each input
// row crosses HBM once per strip and the loads overlap the arithmetic.  Row y lives in ring slot
// (y + P) % RB; wave g loads the rows of its own channel group.
// blocks per CU the forward / dgrad registers are budgeted for (LDS ring: 40 / 49 / 60 / 72 KB bf16)
// (fp32 rings are twice as large: 1-2 blocks)
template <typename T, int K> struct DwOcc {
  static constexpr int v = sizeof(T) == 4 ? (K == 3 ? 2 : 1) : (K == 3 ? 4 : (K == 5 ? 3 : 2));
};

// forward / dgrad tile widths: TX = 32 (8 rows), 40 (6 rows) or 20 (12 rows) output pixels, RX = 4
// per lane, so the lanes of a wave cover TY rows x TX / 4 column groups (64 / 60 / 60 lanes) and a
// 20-, 40- or 80-wide map wastes no columns (a 32-wide tile used 62.5 % of its lanes at 40^2 and
// 52 % at 20^2, where the k = 7 / 9 layers of the MS-Blocks sit)
template <int TX> struct DwTy { static constexpr int v = TX == 32 ? 8 : (TX == 40 ? 6 : 12); };

// raw-buffer 16-B store; an offset at or past num_records is dropped by the hardware, so every
// lane of every wave issues the same store instructions (the end-of-tile wait counts them)
__device__ __forceinline__ void dw_bst16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, const u32x4& v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, 0, 0);
#else
  (void)rs; (void)voff; (void)v;
#endif
}
__device__ __forceinline__ void dw_bst4(__amdgpu_buffer_rsrc_t rs, uint32_t voff, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, 0, 0);
#else
  (void)rs; (void)voff; (void)v;
#endif
}
template <typename T>
__device__ __forceinline__ Raw8<T> pack_raw8(const float (&v)[8]) {
  T t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = (T)v[i];
  Raw8<T> r;
  __builtin_memcpy(&r, t, sizeof(t));
  return r;
}

template <typename T, int K, int MODE, int TX = DW_TX, int G = DW_G>
__global__ __launch_bounds__(G * 64, (G >= 7 ? 2 : DwOcc<T, K>::v))
void dwconv_kernel(DwParams p) {
  constexpr int CB = G * 8, NT = G * 64;
  constexpr int TY = DwTy<TX>::v, CGX = TX / DW_RX;
  constexpr int P = K / 2, HW = TX + K - 1, RB = 2 * TY + K - 1;
  // ONE __shared__ object: a second one beside the LDS-DMA target makes hipcc wait vmcnt(0) before
  // the first ds_read of every kernel row (cdna_hip_programming.md, .s-level trap (a))
  constexpr int RS = dw_rs(HW);   // ring row stride (chunks)
  constexpr int RING_B = G * RB * RS * (int)sizeof(Raw8<T>);
  constexpr int WL_B = G * K * K * 8 * (int)sizeof(float);
  constexpr bool STATS = MODE == DW_FWD_STATS;
  __shared__ __attribute__((aligned(16))) char smem[RING_B + WL_B + G * 16 * (int)sizeof(float)];
  Raw8<T>* ring = reinterpret_cast<Raw8<T>*>(smem);
  float (*wl)[K * K][8] = reinterpret_cast<float (*)[K * K][8]>(smem + RING_B);
  float (*scl)[16] = reinterpret_cast<float (*)[16]>(smem + RING_B + WL_B);   // eval scale | shift (LDS:
                                                                                // not live across the FMAs)
  int bx, by;
  if (!dw_block(p, bx, by)) return;
  const int per_img = p.tiles_x * p.ysplit;
  const int n = bx / per_img, sidx = bx - n * per_img;
  const int tx = sidx % p.tiles_x, t0 = (sidx / p.tiles_x) * p.tps, t1 = min(p.tiles_y, t0 + p.tps);
  const int x0 = tx * TX;
  const int c0 = by * CB;
  {
    // the block's 32 x K x K weights are one contiguous range of p.w: coalesced loads, all issued
    // before the LDS stores (dgrad correlates with the kernel rotated by 180 degrees)
    constexpr int NWL = (CB * K * K + NT - 1) / NT;
    const int nvalid = min(CB, p.C - c0) * K * K;
    float wv[NWL];
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int it = threadIdx.x + NT * j;
      wv[j] = it < nvalid ? p.w[(long)c0 * K * K + it] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int it = threadIdx.x + NT * j;
      if (it < CB * K * K) {
        const int cl = it / (K * K), t = it - cl * (K * K);
        const int tw = MODE == DW_DGRAD ? K * K - 1 - t : t;
        wl[cl >> 3][tw][cl & 7] = wv[j];
      }
    }
  }
  if (MODE == DW_FWD_AFFINE && threadIdx.x < G * 16) {
    const int gg = threadIdx.x >> 4, k = threadIdx.x & 7, c = c0 + 8 * gg + k;
    scl[gg][threadIdx.x & 15] = (threadIdx.x & 8) ? ((p.shift && c < p.C) ? p.shift[c] : 0.0f)
                                                  : ((p.scale && c < p.C) ? p.scale[c] : 1.0f);
  }
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ty = lane / CGX, qx = lane - ty * CGX;   // ty >= TY: idle lane (60 of 64 used at TX 20 / 40)
  const int c = c0 + 8 * g, nv = min(8, p.C - c);
  // raw buffer resource over image n's rows (32-bit offsets: checked on the host)
  const uintptr_t ib = reinterpret_cast<uintptr_t>(reinterpret_cast<const T*>(p.src) +
                                                   (long)n * p.H * p.W * p.src_ld + p.src_off);
  const i32x4 rs = {(int)(uint32_t)ib, (int)(uint32_t)(ib >> 32) & 0xffff,
                    (int)((long)p.H * p.W * p.src_ld * (long)sizeof(T)), NT_RSRC3};
  const uint32_t myring = __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>(ring + g * RB * RS));   // LDS byte address (wave-uniform)
  constexpr uint32_t ROWB = RS * (uint32_t)sizeof(Raw8<T>);
  // destination resource over image n (32-bit offsets, checked on the host); stores go through it
  // so every wave issues the same, unconditional store instructions (out-of-tile lanes: NT_OOB)
  const uintptr_t db = reinterpret_cast<uintptr_t>(reinterpret_cast<T*>(p.dst) + (long)n * p.H * p.W * p.dst_ld +
                                                   p.dst_off);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)db, (short)0, (int)((long)p.H * p.W * p.dst_ld * (long)sizeof(T)), NT_RSRC3);
  const long srows = (long)p.N * p.tiles_y * p.tiles_x;
  const __amdgpu_buffer_rsrc_t rstat = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.stats, (short)0, STATS ? (int)(srows * 2 * p.stats_ld * 4) : 0, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rcnt = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.stats_cnt, (short)0, STATS ? (int)(srows * 4) : 0, NT_RSRC3);
  // prologue: the first tile's TY + K - 1 rows
  for (int hy = 0; hy < TY + K - 1; ++hy)
    dw_row_dma<T, K, TX>(rs, myring + ((t0 * TY + hy) % RB) * ROWB, t0 * TY - P + hy, x0, c, p.H, p.W, p.C,
                         p.src_ld, lane);
  wait_vmcnt<0>();
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    const int y0 = t * TY;
    const bool more = t + 1 < t1;
    // the next tile's TY new rows y0 + TY + P .. y0 + 2 TY - 1 + P go to slots this tile does not read
    if (more) {
      int sl = (y0 + TY + 2 * P) % RB;
      for (int hy = 0; hy < TY; ++hy) {
        dw_row_dma<T, K, TX>(rs, myring + sl * ROWB, y0 + TY + P + hy, x0, c, p.H, p.W, p.C, p.src_ld, lane);
        sl = sl + 1 == RB ? 0 : sl + 1;
      }
    }
    const Raw8<T>* hp = ring + g * RB * RS + 4 * (ty < TY ? qx : 0);
    float acc[DW_RX][8];
#pragma unroll
    for (int i = 0; i < DW_RX; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[i][k] = 0.0f;
    // one kernel row at a time (not unrolled): the row's k x 8 weights live in registers
    int slot = (y0 + ty) % RB;   // ring slot of input row y0 + ty - P
#pragma unroll 1
    for (int dy = 0; dy < K; ++dy) {
      float wr[K][8];
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&wl[g][dy * K + dx][0]);
        const f32x4 b = *reinterpret_cast<const f32x4*>(&wl[g][dy * K + dx][4]);
#pragma unroll
        for (int k = 0; k < 4; ++k) { wr[dx][k] = a[k]; wr[dx][4 + k] = b[k]; }
      }
      const Raw8<T>* row = hp + slot * RS;
#pragma unroll
      for (int q = 0; q < DW_RX + K - 1; ++q) {
        float v[8];
        unpack8(row[q], v);
#pragma unroll
        for (int i = 0; i < DW_RX; ++i) {
          const int dx = q - i;
          if (dx >= 0 && dx < K) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[i][k] += v[k] * wr[dx][k];
          }
        }
      }
      slot = slot + 1 == RB ? 0 : slot + 1;
    }
    const int tile = (n * p.tiles_y + t) * p.tiles_x + tx;   // statistics row (image-major tiles)
    const int y = y0 + ty;
    const bool yok = ty < TY && y < p.H;
    // every wave issues exactly NST vector-memory instructions after its last DMA of this tile (the
    // stores below; statistics: two row stores and the count): the end-of-tile wait leaves them in
    // flight and waits for the next tile's rows only (vmcnt retires in issue order on gfx9)
    constexpr int NST = DW_RX * (int)(sizeof(T) / 2) + (STATS ? 3 : 0);
#pragma unroll
    for (int i = 0; i < DW_RX; ++i) {
      const int x = x0 + 4 * qx + i;
      const bool ok = nv > 0 && yok && x < p.W;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = acc[i][k];
        if (MODE == DW_FWD_AFFINE) {
          v = v * scl[g][k] + scl[g][8 + k];
          if (p.act == YMS_ACT_SILU) v = silu_f(v);
        }
        o[k] = v;
      }
      const uint32_t e = ok ? (uint32_t)((y * p.W + x) * p.dst_ld + c) : 0u;
      if (MODE == DW_DGRAD && p.accumulate) {
        // (this load retires the tile's DMA with it: accumulation is the rare case)
        float r[8];
        if (ok) load8(reinterpret_cast<const T*>(db) + e, nv, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += ok ? r[k] : 0.0f;
      }
      const Raw8<T> rv = pack_raw8<T>(o);
#pragma unroll
      for (int h = 0; h < (int)(sizeof(T) / 2); ++h)
        dw_bst16(rd, ok ? e * (uint32_t)sizeof(T) + 16u * h : NT_OOB, rv.v[h]);
    }
    if (STATS) {
      // one statistics row per spatial tile (conv_common.hpp contract; its pixel count goes to the
      // count table after the rows): sum and centred M2 over the tile's valid pixels, two passes
      // over the fp32 accumulators, wave butterflies in a fixed order
      const int vy = min(TY, p.H - y0), vx = min(TX, p.W - x0);
      const float inv_n = 1.0f / (float)(vy * vx);
      float s1[8], m2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s = 0.f;
        if (yok) {
#pragma unroll
          for (int i = 0; i < DW_RX; ++i)
            if (x0 + 4 * qx + i < p.W) s += acc[i][k];
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) s += __shfl_xor(s, m);
        const float mu = s * inv_n;
        float q = 0.f;
        if (yok) {
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
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k == lane) { a = s1[k]; b = m2[k]; }
      const bool sok = lane < 8 && c + lane < p.C;
      const uint32_t so = (uint32_t)(((long)tile * 2 * p.stats_ld + c + lane) * 4);
      dw_bst4(rstat, sok ? so : NT_OOB, a);
      dw_bst4(rstat, sok ? so + (uint32_t)p.stats_ld * 4u : NT_OOB, b);
      dw_bst4(rcnt, (by == 0 && threadIdx.x == 0) ? (uint32_t)tile * 4u : NT_OOB, (float)(vy * vx));
    }
    wait_vmcnt<NST>();
    __syncthreads();
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
  constexpr int HRS = dw_rs(HW), DRS = dw_rs(DW_TX);   // padded LDS row strides (chunks)
  constexpr int HALO = DW_G * HH * HRS, DZN = DW_G * DW_TY * DW_TX;
  constexpr int DZL = DW_G * DW_TY * DRS;
  constexpr int STAGE_B = (HALO + DZL) * (int)sizeof(Raw8<T>);
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
      dzl[(g2 * DW_TY + r2 / DW_TX) * DRS + r2 % DW_TX] = v;
    }
    __syncthreads();
    if (active) {
      const Raw8<T>* hrow = halo + (g * HH + ty + dy) * HRS + sx;
      const Raw8<T>* drow = dzl + (g * DW_TY + ty) * DRS + sx;
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

// wgrad, k = 5 / 7 / 9, 16-bit types (fp32 keeps the kernel above): the same lane
// work as dwconv_wgrad_kernel -- lane (dy, ty, s) of a channel group keeps the K x 8 partial taps of
// kernel row dy for its tile row and column segment in registers across all of the block's tiles --
// on tiles shaped for the map and the kernel: TX = the forward's width (20 / 40 / 32: no idle
// columns on the 20 / 40 / 80-wide maps) and TY rows such that K TY S of the 128 lanes of a group
// are busy (the 8 x 32 tile kept 56-88 % of them busy and wasted 3/8 of its columns on 20-wide
// maps), and with the NEXT tile's halo and dz chunks fetched into registers while the current tile
// computes (the tile kernel staged each tile synchronously).  Same fixed-order reductions.
template <int K, int TX>
struct DwWg2 {
  static constexpr int S = TX == 20 ? 1 : 2;
  static constexpr int TY = TX == 20 ? (K == 5 ? 20 : 10) : (K == 5 ? 12 : (K == 7 ? 9 : 7));
  static constexpr int SL = TX / S;
  static constexpr int NA = K * TY * S;
};

template <typename T, int K, int TX>
__global__ __launch_bounds__(DW_WG_NT) void dwconv_wgrad2_kernel(DwParams p, const char* dz, int dz_ld, int dz_off,
                                                                  float* ws) {
  using W = DwWg2<K, TX>;
  constexpr int TY = W::TY, S = W::S, SL = W::SL, NA = W::NA;
  static_assert(NA <= DW_WG_LPG && SL % 4 == 0 && sizeof(T) == 2, "dw wgrad2 lane mapping");
  constexpr int HH = TY + K - 1, HW = TX + K - 1, P = K / 2;
  constexpr int HRS = dw_rs(HW), DRS = dw_rs(TX);
  constexpr int HALO_N = DW_G * HH * HW, DZ_N = DW_G * TY * TX;          // 16-B items per tile
  constexpr int ITEMS = (HALO_N + DZ_N + DW_WG_NT - 1) / DW_WG_NT;
  constexpr int HALO = DW_G * HH * HRS, DZL = DW_G * TY * DRS;
  constexpr int STAGE_B = (HALO + DZL) * (int)sizeof(Raw8<T>);
  constexpr int RED_B = NA * K * 8 * (int)sizeof(float);
  __shared__ __attribute__((aligned(16))) char smem[STAGE_B > RED_B ? STAGE_B : RED_B];
  Raw8<T>* halo = reinterpret_cast<Raw8<T>*>(smem);
  Raw8<T>* dzl = halo + HALO;
  float* red = reinterpret_cast<float*>(smem);
  const int c0 = blockIdx.y * DW_CB;
  const int tid = threadIdx.x;
  const int g = tid / DW_WG_LPG, l = tid % DW_WG_LPG;
  const bool active = l < NA;
  const int ll = active ? l : 0;
  const int dy = ll / (TY * S), r = ll % (TY * S);
  const int ty = r / S, sx = (r % S) * SL;
  const int tiles_x = (p.W + TX - 1) / TX, tiles_y = (p.H + TY - 1) / TY;
  const int per_img = tiles_x * tiles_y, ntiles = p.N * per_img;
  const T* src = reinterpret_cast<const T*>(p.src);
  const T* dzp = reinterpret_cast<const T*>(dz);
  // item it of a tile: halo chunk (g, hy, hx) for it < HALO_N, else dz chunk (g, ty, tx)
  auto fetch = [&](int tile, Raw8<T> (&buf)[ITEMS]) {
    const int n = tile / per_img, rem = tile - n * per_img;
    const int y0 = (rem / tiles_x) * TY, x0 = (rem % tiles_x) * TX;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int it = tid + j * DW_WG_NT;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(T) / 2); ++k) buf[j].v[k] = u32x4{0u, 0u, 0u, 0u};
      int y, x, c;
      const T* base;
      long ld, off;
      if (it < HALO_N) {
        const int gg = it / (HH * HW), rr = it - gg * (HH * HW);
        y = y0 + rr / HW - P; x = x0 + rr % HW - P; c = c0 + 8 * gg;
        base = src; ld = p.src_ld; off = p.src_off;
      } else if (it < HALO_N + DZ_N) {
        const int i2 = it - HALO_N, gg = i2 / (TY * TX), rr = i2 - gg * (TY * TX);
        y = y0 + rr / TX; x = x0 + rr % TX; c = c0 + 8 * gg;
        base = dzp; ld = dz_ld; off = dz_off;
      } else {
        continue;
      }
      if (y >= 0 && y < p.H && x >= 0 && x < p.W && c < p.C)
        load_raw8(base + (((long)n * p.H + y) * p.W + x) * ld + off + c, min(8, p.C - c), buf[j]);
    }
  };
  auto store = [&](const Raw8<T> (&buf)[ITEMS]) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int it = tid + j * DW_WG_NT;
      if (it < HALO_N) {
        const int gg = it / (HH * HW), rr = it - gg * (HH * HW);
        halo[(gg * HH + rr / HW) * HRS + rr % HW] = buf[j];
      } else if (it < HALO_N + DZ_N) {
        const int i2 = it - HALO_N, gg = i2 / (TY * TX), rr = i2 - gg * (TY * TX);
        dzl[(gg * TY + rr / TX) * DRS + rr % TX] = buf[j];
      }
    }
  };
  float part[K][8];
#pragma unroll
  for (int dx = 0; dx < K; ++dx)
#pragma unroll
    for (int k = 0; k < 8; ++k) part[dx][k] = 0.0f;
  Raw8<T> buf[ITEMS];
  if ((int)blockIdx.x < ntiles) fetch(blockIdx.x, buf);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();      // the previous tile's LDS reads are done
    store(buf);
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x, buf);   // in flight during the FMAs
    if (active) {
      const Raw8<T>* hrow = halo + (g * HH + ty + dy) * HRS + sx;
      const Raw8<T>* drow = dzl + (g * TY + ty) * DRS + sx;
#pragma unroll 1
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
    for (int it = tid; it < K * K * 8; it += DW_WG_NT) {
      const int t = it / 8, k = it - t * 8;
      const int ddy = t / K, ddx = t - ddy * K;
      float s = 0.f;
      for (int rr = 0; rr < TY * S; ++rr) s += red[((ddy * TY * S + rr) * K + ddx) * 8 + k];
      const int cc = c0 + 8 * gg + k;
      if (cc < p.C) ws[((long)blockIdx.x * K * K + t) * p.C + cc] = s;
    }
  }
}

// wgrad, k = 3: the forward's strip walker (TY x TX tiles, RX = 4 pixels per lane, the input rows
// in an LDS-DMA ring, the next tile's rows and dz chunks in flight while the current tile
// computes).  Every lane keeps the 3 x 3 x 8 partial taps of its pixels in registers across the
// whole strip: per kernel row it reads RX + 2 ring chunks and does 3 RX 8 FMAs against its RX dz
// chunks.  At the end the 72 partials are summed over the wave's lanes by a fixed butterfly and
// lane 0 writes ws[block][tap][c] (dwconv_wgrad_reduce_kernel sums the strips in a fixed order).
// Replaces the 8 x 32-tile kernel above for k = 3, which staged each tile synchronously.
template <typename T, int TX, int G>
__global__ __launch_bounds__(G * 64, 2) void dwconv_wgrad3_kernel(DwParams p, const char* dz, int dz_ld, int dz_off,
                                                                  float* ws) {
  constexpr int K = 3, P = 1;
  constexpr int CB = G * 8, TY = DwTy<TX>::v, CGX = TX / DW_RX;
  constexpr int HW = TX + K - 1, RB = 2 * TY + K - 1, RS = dw_rs(HW);
  constexpr int RING_B = G * RB * RS * (int)sizeof(Raw8<T>);
  __shared__ __attribute__((aligned(16))) char smem[RING_B];
  Raw8<T>* ring = reinterpret_cast<Raw8<T>*>(smem);
  int bx, by;
  if (!dw_block(p, bx, by)) return;
  const int per_img = p.tiles_x * p.ysplit;
  const int n = bx / per_img, sidx = bx - n * per_img;
  const int tx = sidx % p.tiles_x, t0 = (sidx / p.tiles_x) * p.tps, t1 = min(p.tiles_y, t0 + p.tps);
  const int x0 = tx * TX;
  const int c0 = by * CB;
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ty = lane / CGX, qx = lane - ty * CGX;
  const int c = c0 + 8 * g, nv = min(8, p.C - c);
  const uintptr_t ib = reinterpret_cast<uintptr_t>(reinterpret_cast<const T*>(p.src) +
                                                   (long)n * p.H * p.W * p.src_ld + p.src_off);
  const i32x4 rs = {(int)(uint32_t)ib, (int)(uint32_t)(ib >> 32) & 0xffff,
                    (int)((long)p.H * p.W * p.src_ld * (long)sizeof(T)), NT_RSRC3};
  const uint32_t myring = __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>(ring + g * RB * RS));
  constexpr uint32_t ROWB = RS * (uint32_t)sizeof(Raw8<T>);
  const T* dzp = reinterpret_cast<const T*>(dz) + (long)n * p.H * p.W * dz_ld + dz_off;
  // this lane's RX dz chunks of tile t (zeros outside the image / past C / idle lanes)
  auto load_dz = [&](int t, Raw8<T> (&d)[DW_RX]) {
    const int y = t * TY + ty;
#pragma unroll
    for (int i = 0; i < DW_RX; ++i) {
      const int x = x0 + 4 * qx + i;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(T) / 2); ++k) d[i].v[k] = u32x4{0u, 0u, 0u, 0u};
      if (ty < TY && y < p.H && x < p.W && nv > 0) load_raw8(dzp + ((long)y * p.W + x) * dz_ld + c, 8, d[i]);
    }
  };
  float part[K][K][8];
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b)
#pragma unroll
      for (int k = 0; k < 8; ++k) part[a][b][k] = 0.0f;
  Raw8<T> dzc[DW_RX], dzn[DW_RX];
  for (int hy = 0; hy < TY + K - 1; ++hy)
    dw_row_dma<T, K, TX>(rs, myring + ((t0 * TY + hy) % RB) * ROWB, t0 * TY - P + hy, x0, c, p.H, p.W, p.C,
                         p.src_ld, lane);
  load_dz(t0, dzc);
  wait_vmcnt<0>();
  __syncthreads();
  const Raw8<T>* hp = ring + g * RB * RS + 4 * (ty < TY ? qx : 0);
  for (int t = t0; t < t1; ++t) {
    const int y0 = t * TY;
    const bool more = t + 1 < t1;
    if (more) {
      int sl = (y0 + TY + 2 * P) % RB;
      for (int hy = 0; hy < TY; ++hy) {
        dw_row_dma<T, K, TX>(rs, myring + sl * ROWB, y0 + TY + P + hy, x0, c, p.H, p.W, p.C, p.src_ld, lane);
        sl = sl + 1 == RB ? 0 : sl + 1;
      }
      load_dz(t + 1, dzn);
    }
    float d[DW_RX][8];
#pragma unroll
    for (int i = 0; i < DW_RX; ++i) unpack8(dzc[i], d[i]);
    // idle lanes (ty >= TY) read row 0's slots: their dz is zero, but a slot of a later row may be
    // unwritten LDS (NaN patterns) or landing now
    int slot = (y0 + (ty < TY ? ty : 0)) % RB;
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
      const Raw8<T>* row = hp + slot * RS;
#pragma unroll
      for (int q = 0; q < DW_RX + K - 1; ++q) {
        float v[8];
        unpack8(row[q], v);
#pragma unroll
        for (int i = 0; i < DW_RX; ++i) {
          const int dx = q - i;
          if (dx >= 0 && dx < K) {
#pragma unroll
            for (int k = 0; k < 8; ++k) part[dy][dx][k] += v[k] * d[i][k];
          }
        }
      }
      slot = slot + 1 == RB ? 0 : slot + 1;
    }
    wait_vmcnt<0>();
    __syncthreads();
    if (more) {
#pragma unroll
      for (int i = 0; i < DW_RX; ++i) dzc[i] = dzn[i];
    }
  }
  // fixed-order butterfly over the wave's 64 lanes, lane 0 writes the block's 9 x 8 partial taps
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = part[a][b][k];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
        part[a][b][k] = v;
      }
  if (lane == 0 && nv > 0) {
#pragma unroll
    for (int t = 0; t < K * K; ++t) {
      float* o = ws + ((long)bx * K * K + t) * p.C + c;
      *reinterpret_cast<f32x4*>(o) = f32x4{part[t / K][t % K][0], part[t / K][t % K][1], part[t / K][t % K][2],
                                           part[t / K][t % K][3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{part[t / K][t % K][4], part[t / K][t % K][5],
                                               part[t / K][t % K][6], part[t / K][t % K][7]};
    }
  }
}

// wgrad, k = 5 / 7 / 9 on maps at most 64 wide (k = 5: 96), 16-bit types: the per-channel correlation
// on MFMA.
// For one channel, rows a of the padded input and rows b of dz,
//   G_dx[a][b] = sum_x Xp[a][x + dx] D[b][x],   dw[dy][dx] = sum_b G_dx[b + dy][b]
// i.e. per kernel column dx one product (a x x) . (x x b) whose band diagonals a - b = 0 .. K-1 are
// the weight gradient.  A unit = (image, 16 dz rows b0 .. b0 + 15): the band a - b in [0, K) lies in
// two 16 x 16 blocks, the diagonal one (a in b0 .. b0 + 15) and the one below it (a in b0 + 16 ..
// b0 + 31, skipped when those rows are all padding), each accumulated over 32-column chunks by
// mfma_f32_16x16x32 into per-(block, dx) accumulators that stay in registers across all of a thread
// block's units (the diagonals are relative to b0).  Of the lower block only rows a < b0 + 16 + K - 1
// reach the band: the rest of its rows are whatever LDS holds there, and their products land in
// entries a - b >= K that are never read.  The dz fragment (lane: row b, 8 columns) is read once per
// chunk and reused by 2 K products; the input fragment (lane: row a, 16 columns) once per block and
// chunk, the K column windows dx = 0 .. K-1 cut from registers (dword selects / v_alignbit).  At the
// end each wave sums the 16 entries of every diagonal through LDS in a fixed order and writes
// ws[group][t][c]; a reduce kernel sums the groups.  A block is 16 channels (512 threads, two
// channels per wave; neighbouring lanes load the two 16-B halves of a pixel's 32 B).  LDS holds a unit
// channel-major (16 NB + K - 1 input rows, 16 NB dz rows; image column x of the input at x + 4), rows
// 96 / 160 / 224 B apart: the 16 rows one ds_read_b128 lane group touches (two column slots) fall in
// distinct banks.  NB = 2 for maps of 17-32 rows (one staging for both dz blocks).  Staging items
// are 4 pixels x 8 channels of one row: four 16-B loads (rows outside the image load as zeros,
// columns past the map are never loaded), re-paired per channel with v_perm into eight 8-B LDS
// writes; the next unit's items are loaded into registers while the current one computes.
template <int K, int NCH, int CG, int NB>
struct DwWgM {
  // NB 16-row dz blocks per unit (2: a 20- or 32-row map is one unit, staged once)
  static constexpr int P = K / 2, PA = 4, SH = PA - P, DR = 16 * NB, XR = DR + K - 1, NT = 32 * CG, NW = CG / 2;
  static constexpr int H2 = CG / 8;
  static constexpr int XL = NCH == 1 ? 48 : (NCH == 2 ? 80 : 112);   // row stride (elements), both operands'
  static constexpr int XE = CG * XR * XL, LDS_EL = XE + CG * DR * XL;
  static constexpr int NIX = (XR * 8 * NCH * H2 + NT - 1) / NT, NID = (DR * 8 * NCH * H2 + NT - 1) / NT;
  static_assert(XL >= 32 * NCH + 8, "row holds the chunks and the window overhang");
  static_assert(LDS_EL * 2 <= (CG == 8 ? 80 : 160) * 1024 && NW * 512 * 4 <= LDS_EL * 2, "LDS");
};

template <typename T> __device__ __forceinline__ f32x4 mfma16x16x32(const u32x4& a, const u32x4& b, f32x4 c);
template <> __device__ __forceinline__ f32x4 mfma16x16x32<bf16>(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                 0);
}
template <> __device__ __forceinline__ f32x4 mfma16x16x32<f16>(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// 8 consecutive 16-bit values starting at element s of a 16-element register row
__device__ __forceinline__ u32x4 dw_window(const unsigned (&v)[8], int s) {
  const int m = s >> 1;
  if (!(s & 1)) return u32x4{v[m], v[m + 1], v[m + 2], v[m + 3]};
  return u32x4{__builtin_amdgcn_alignbit(v[m + 1], v[m], 16), __builtin_amdgcn_alignbit(v[m + 2], v[m + 1], 16),
               __builtin_amdgcn_alignbit(v[m + 3], v[m + 2], 16), __builtin_amdgcn_alignbit(v[m + 4], v[m + 3], 16)};
}
template <typename T, int K, int NCH, int CG, int NB>
__global__ __launch_bounds__(32 * CG, CG == 8 ? 2 : 1) void dwconv_wgrad_mfma_kernel(DwParams p, const char* dz,
                                                                                   int dz_ld, int dz_off, float* ws,
                                                                                   int nj, int upb, int ncg, int ngrp) {
  using G = DwWgM<K, NCH, CG, NB>;
  constexpr int P = G::P, PA = G::PA, SH = G::SH, XR = G::XR, XL = G::XL, NT = G::NT, NW = G::NW, H2 = G::H2;
  constexpr int DR = G::DR;
  constexpr int NIX = G::NIX, NID = G::NID;
  __shared__ __attribute__((aligned(16))) unsigned short lds[G::LDS_EL];
  unsigned short* xs = lds;
  unsigned short* ds = lds + G::XE;
  // block -> (unit group, channel group), channel group fastest.  The grid is padded to a multiple
  // of 8 and block i runs on XCD i % 8: consecutive logical blocks (the channel groups of the same
  // pixels, 2 CG B of each 128-B line apiece) run on one XCD and share its L2
  const int b = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (b >= ncg * ngrp) return;
  const int cgi = b % ncg, grp = b / ncg;
  const int c0 = cgi * CG;
  const int u0 = grp * upb, u1 = min(p.N * nj, u0 + upb);
  const int tid = threadIdx.x;
  // staging items: (row, group of 4 columns, 8-channel half), halves fastest (neighbouring lanes
  // load the two 16-B halves of one pixel's 32 B).  Per item: LDS offset of its first channel's row
  // segment, byte offset of its first pixel in image row 0 (-1: no item / channels past C), the
  // staged row, and how many of its 4 pixels lie inside the map
  const int ng = (p.W + 3) >> 2;
  const uint32_t xrow = (uint32_t)p.W * p.src_ld * 2, drow = (uint32_t)p.W * dz_ld * 2;
  int xslot[NIX], xoff[NIX], xr_[NIX], xm[NIX], dslot[NID], doff[NID], dr_[NID], dm[NID];
#pragma unroll
  for (int i = 0; i < NIX; ++i) {
    const int it = tid + NT * i, h = it % H2, rm = it / H2, r = rm / ng, m = rm - r * ng;
    const bool ok = r < XR && c0 + 8 * h < p.C;
    xslot[i] = (8 * h * XR + r) * XL + 4 * m + PA;
    xoff[i] = ok ? (int)((((uint32_t)r * p.W + 4 * m) * p.src_ld + 8 * h) * 2) : -1;
    xr_[i] = r;
    xm[i] = ok ? min(4, p.W - 4 * m) : 0;
  }
#pragma unroll
  for (int i = 0; i < NID; ++i) {
    const int it = tid + NT * i, h = it % H2, rm = it / H2, r = rm / ng, m = rm - r * ng;
    const bool ok = r < DR && c0 + 8 * h < p.C;
    dslot[i] = (8 * h * DR + r) * XL + 4 * m;
    doff[i] = ok ? (int)((((uint32_t)r * p.W + 4 * m) * dz_ld + 8 * h) * 2) : -1;
    dr_[i] = r;
    dm[i] = ok ? min(4, p.W - 4 * m) : 0;
  }
  // columns outside the image, past the map width and channels past C stay zero for every unit
  for (int i = tid; i < G::LDS_EL / 8; i += NT) reinterpret_cast<u32x4*>(lds)[i] = u32x4{0u, 0u, 0u, 0u};
  const char* xsrc = reinterpret_cast<const char*>(reinterpret_cast<const T*>(p.src) + p.src_off + c0);
  const char* dsrc = reinterpret_cast<const char*>(reinterpret_cast<const T*>(dz) + dz_off + c0);
  const long ximg = (long)p.H * p.W * p.src_ld * 2, dimg = (long)p.H * p.W * dz_ld * 2;
  u32x4 xv[NIX][4], dv[NID][4];
  // rows outside the image load as zeros (the LDS rows vary per unit); pixels past the map width
  // are never loaded (their LDS columns stay zero)
  auto load = [&](int unit) {
    const int n = unit / nj, j = unit - n * nj;
    const char* xi = xsrc + n * ximg;
    const char* di = dsrc + n * dimg;
    const int yx = DR * j - P, yd = DR * j;   // image row of staged row 0
#pragma unroll
    for (int i = 0; i < NIX; ++i) {
      const int y = yx + xr_[i];
      const bool ok = xoff[i] >= 0 && y >= 0 && y < p.H;
      const uint32_t o = (uint32_t)xoff[i] + (uint32_t)yx * xrow;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xv[i][k] = u32x4{0u, 0u, 0u, 0u};
        if (ok && k < xm[i]) xv[i][k] = *reinterpret_cast<const u32x4*>(xi + o + k * p.src_ld * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < NID; ++i) {
      const int y = yd + dr_[i];
      const bool ok = doff[i] >= 0 && y < p.H;
      const uint32_t o = (uint32_t)doff[i] + (uint32_t)yd * drow;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dv[i][k] = u32x4{0u, 0u, 0u, 0u};
        if (ok && k < dm[i]) dv[i][k] = *reinterpret_cast<const u32x4*>(di + o + k * dz_ld * 2);
      }
    }
  };
  // 4 pixels x 8 channels -> 8 channel rows of 4 columns (one 8-B write each)
  auto put = [&](unsigned short* d0, int cs, const u32x4 (&v)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const unsigned lo01 = __builtin_amdgcn_perm(v[1][d], v[0][d], 0x05040100u);
      const unsigned lo23 = __builtin_amdgcn_perm(v[3][d], v[2][d], 0x05040100u);
      const unsigned hi01 = __builtin_amdgcn_perm(v[1][d], v[0][d], 0x07060302u);
      const unsigned hi23 = __builtin_amdgcn_perm(v[3][d], v[2][d], 0x07060302u);
      *reinterpret_cast<uint2*>(d0 + (2 * d) * cs) = make_uint2(lo01, lo23);
      *reinterpret_cast<uint2*>(d0 + (2 * d + 1) * cs) = make_uint2(hi01, hi23);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < NIX; ++i)
      if (xoff[i] >= 0) put(xs + xslot[i], XR * XL, xv[i]);
#pragma unroll
    for (int i = 0; i < NID; ++i)
      if (doff[i] >= 0) put(ds + dslot[i], DR * XL, dv[i]);
  };
  const int lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  f32x4 acc[2][2][K];   // [channel of the wave][diagonal / lower block][dx]
#pragma unroll
  for (int cl = 0; cl < 2; ++cl)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dx = 0; dx < K; ++dx) acc[cl][s][dx] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int unit) {
    const int j = unit % nj;
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      const int b0 = DR * j + 16 * jj;               // image row of this dz block's first row
      if (b0 >= p.H) break;
      const bool lower = b0 + 16 - P < p.H;          // the lower block's input rows are not all padding
#pragma unroll
      for (int cl = 0; cl < 2; ++cl) {
        const int ch = w + NW * cl;
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
          const u32x4 bw = *reinterpret_cast<const u32x4*>(ds + (ch * DR + 16 * jj + r16) * XL + 32 * q + 8 * g);
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            if (s == 1 && !lower) break;
            const unsigned short* xr = xs + (ch * XR + 16 * (jj + s) + r16) * XL + 32 * q + 8 * g;
            const u32x4 v0 = *reinterpret_cast<const u32x4*>(xr), v1 = *reinterpret_cast<const u32x4*>(xr + 8);
            const unsigned v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
            for (int dx = 0; dx < K; ++dx)
              acc[cl][s][dx] = mfma16x16x32<T>(dw_window(v, dx + SH), bw, acc[cl][s][dx]);
          }
        }
      }
    }
  };
  // LDS-only barriers: __syncthreads() would drain the next unit's loads (vmcnt(0)) right after
  // issuing them
  if (u0 < u1) load(u0);
  for (int unit = u0; unit < u1; ++unit) {
    lds_barrier();   // zero fill done / the previous unit's reads done
    store();
    if (unit + 1 < u1) load(unit + 1);
    lds_barrier();
    compute(unit);
  }
  // diagonal sums: lane (b = lane & 15, a = 4 (lane >> 4) + i) holds G[a][b] (diagonal block) and
  // G[a + 16][b] (lower block); dw[dy][dx] = sum over b of G[b + dy][b], 16 terms in a fixed order
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds) + w * 512;
#pragma unroll
  for (int cl = 0; cl < 2; ++cl) {
    const int c = c0 + w + NW * cl;
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(4 * g + i) * 16 + r16] = acc[cl][0][dx][i];
        red[256 + (4 * g + i) * 16 + r16] = acc[cl][1][dx][i];
      }
      __syncthreads();
      // lane (dy = lane & 15, quarter h = lane >> 4) sums b = 4 h .. 4 h + 3, then the quarters pair up
      const int dy = r16;
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bb = 4 * g + k;
        sum += bb + dy < 16 ? red[(bb + dy) * 16 + bb] : red[256 + ((bb + dy) & 15) * 16 + bb];
      }
      sum += __shfl_xor(sum, 16);
      sum += __shfl_xor(sum, 32);
      if (g == 0 && dy < K && c < p.C) ws[((long)grp * K * K + dy * K + dx) * p.C + c] = sum;
      __syncthreads();
    }
  }
}

// forward / dgrad, 16-bit types, on MFMA (selected for k = 7 on maps up to 48 wide: dw_fm): per
// channel a Toeplitz product per kernel row.  For a block of 16 output rows y0 .. y0 + 15 and 16 output columns x0 .. x0 + 15,
//   Y[m][n] = sum_dy sum_k A_dy[m][k] B_dy[k][n],  A_dy[m][k] = X[y0 + m + dy - P][x0 + k - 4],
//   B_dy[k][n] = w[dy][k - n - SH]  (zero outside 0 .. K-1; SH = 4 - P)
// one mfma_f32_16x16x32 per kernel row over 32 staged columns (the 16 + K - 1 the outputs reach sit
// inside them).  The weights enter as two bf16 / f16 parts (w = hi + lo, residual 2^-16 |w|), so the
// products match the fp32-weight VALU kernels to fp32 rounding: two MFMAs per kernel row, still far
// under the HBM time.  B_dy (per channel, lane: 8 rows k of column n) is built once per block in
// registers; the input fragment is one ds_read_b128 per (row block, column block, dy).  A block is
// (image, 16 output rows, 8 channels): the 16 + K - 1 input rows staged channel-major as the
// MFMA weight gradient stages them (4 pixels x 8 channels per item, v_perm, 8-B LDS writes), 2
// channels per wave with all ceil(W / 16) column blocks' accumulators in registers; the epilogue
// (folded BN + SiLU | statistics of the tile | dgrad accumulate) goes back to NHWC through LDS as
// 16-B pixel chunks.  Statistics rows: one per (image, 16-row block) -- yms_dwconv_stats_rows.
constexpr int dw_fm_xl(int ncb) {   // row stride: >= 16 ncb + 16 elements, (16-B units) = 2 mod 4
  int t = (16 * ncb + 16 + 7) / 8;
  while (t % 4 != 2) ++t;
  return 8 * t;
}
template <int K, int NCB>
struct DwFm {
  static constexpr int P = K / 2, SH = 4 - P, XR = 16 + K - 1, XL = dw_fm_xl(NCB), WMAX = 16 * NCB;
  static constexpr int XE = 8 * XR * XL;                                   // staged input (elements)
  static constexpr int NI = (XR * (WMAX / 4) + 255) / 256;                 // 4-pixel items per thread
  static_assert(XE * 2 + 8 * K * K * 4 <= 80 * 1024, "two blocks per CU");
  static_assert(16 * WMAX * 8 <= XE, "output tile fits the staging area");
};

template <typename T, int K, int NCB, int MODE>
__global__ __launch_bounds__(256, 2) void dwconv_mfma_kernel(DwParams p, int upb) {
  using G = DwFm<K, NCB>;
  constexpr int P = G::P, SH = G::SH, XR = G::XR, XL = G::XL, NI = G::NI;
  constexpr bool STATS = MODE == DW_FWD_STATS;
  __shared__ __attribute__((aligned(16))) unsigned short xs[G::XE];
  __shared__ float wl[8][K * K];
  int grp, by;
  if (!dw_block(p, grp, by)) return;
  const int nj = (p.H + 15) >> 4;
  const int u0 = grp * upb, u1 = min(p.N * nj, u0 + upb);
  const int c0 = 8 * by;
  const bool cok = c0 < p.C;
  const int tid = threadIdx.x;
  // input items: (staged row r, 4-pixel group m), fixed per thread; rows outside the image load as
  // zeros.  The next unit's items are loaded into registers while the current one computes.
  const int ng = (p.W + 3) >> 2;
  const char* src = reinterpret_cast<const char*>(reinterpret_cast<const T*>(p.src) + p.src_off + c0);
  const long img = (long)p.H * p.W * p.src_ld * 2;
  int ir[NI], im[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    ir[i] = it / ng;
    im[i] = it - ir[i] * ng;
  }
  u32x4 v[NI][4];
  auto load = [&](int unit) {
    const int n = unit / nj, y0 = 16 * (unit - n * nj);
    const char* si = src + n * img;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int y = y0 - P + ir[i];
      const bool ok = ir[i] < XR && y >= 0 && y < p.H && cok;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[i][k] = u32x4{0u, 0u, 0u, 0u};
        if (ok && 4 * im[i] + k < p.W)
          v[i][k] = *reinterpret_cast<const u32x4*>(si + ((long)(y * p.W + 4 * im[i] + k) * p.src_ld) * 2);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if (ir[i] < XR) {
        unsigned short* d0 = xs + ir[i] * XL + 4 * im[i] + 4;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const unsigned lo01 = __builtin_amdgcn_perm(v[i][1][d], v[i][0][d], 0x05040100u);
          const unsigned lo23 = __builtin_amdgcn_perm(v[i][3][d], v[i][2][d], 0x05040100u);
          const unsigned hi01 = __builtin_amdgcn_perm(v[i][1][d], v[i][0][d], 0x07060302u);
          const unsigned hi23 = __builtin_amdgcn_perm(v[i][3][d], v[i][2][d], 0x07060302u);
          *reinterpret_cast<uint2*>(d0 + (2 * d) * XR * XL) = make_uint2(lo01, lo23);
          *reinterpret_cast<uint2*>(d0 + (2 * d + 1) * XR * XL) = make_uint2(hi01, hi23);
        }
      }
  };
  if (u0 < u1) load(u0);
  // weights (dgrad: rotated by 180 degrees), channels past C zero
  for (int it = tid; it < 8 * K * K; it += 256) {
    const int cl = it / (K * K), t = it - cl * (K * K);
    const int tw = MODE == DW_DGRAD ? K * K - 1 - t : t;
    wl[cl][tw] = c0 + cl < p.C ? p.w[(long)(c0 + cl) * K * K + t] : 0.0f;
  }
  __syncthreads();
  const int lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  // B_dy fragments of the wave's two channels (rows k = 8 g .. 8 g + 7 of column n = lane & 15), hi
  // and lo parts, built once for all the block's units
  u32x4 bh[2][K], bl[2][K];
  float sc[2], sf[2];
#pragma unroll
  for (int cl = 0; cl < 2; ++cl) {
    const int ch = w + 4 * cl, c = c0 + ch;
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
      T hv[8], lv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int dx = 8 * g + e - r16 - SH;
        const float wv = dx >= 0 && dx < K ? wl[ch][dy * K + dx] : 0.0f;
        hv[e] = (T)wv;
        lv[e] = (T)(wv - (float)hv[e]);
      }
      __builtin_memcpy(&bh[cl][dy], hv, 16);
      __builtin_memcpy(&bl[cl][dy], lv, 16);
    }
    sc[cl] = 1.f;
    sf[cl] = 0.f;
    if (MODE == DW_FWD_AFFINE && c < p.C) {
      if (p.scale) sc[cl] = p.scale[c];
      if (p.shift) sf[cl] = p.shift[c];
    }
  }
  // columns outside the image and past the map width stay zero for every unit
  for (int i = tid; i < G::XE / 8; i += 256) reinterpret_cast<u32x4*>(xs)[i] = u32x4{0u, 0u, 0u, 0u};
  T* ys = reinterpret_cast<T*>(xs);
  for (int unit = u0; unit < u1; ++unit) {
    const int n = unit / nj, y0 = 16 * (unit - n * nj);
    const int vy = min(16, p.H - y0);
    lds_barrier();   // zero fill / the previous unit's output stores read
    if (unit > u0) {
      // the output tile overwrote the staging area: restore the zero columns
      for (int i = tid; i < 16 * p.W; i += 256) reinterpret_cast<u32x4*>(xs)[i] = u32x4{0u, 0u, 0u, 0u};
      lds_barrier();
    }
    store();
    if (unit + 1 < u1) load(unit + 1);
    lds_barrier();
    f32x4 acc[2][NCB];
#pragma unroll
    for (int cl = 0; cl < 2; ++cl) {
      const int ch = w + 4 * cl;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (16 * cb < p.W) {
          const unsigned short* xr = xs + (ch * XR + r16) * XL + 16 * cb + 8 * g;
#pragma unroll
          for (int dy = 0; dy < K; ++dy) {
            const u32x4 av = *reinterpret_cast<const u32x4*>(xr + dy * XL);
            a4 = mfma16x16x32<T>(av, bh[cl][dy], a4);
            a4 = mfma16x16x32<T>(av, bl[cl][dy], a4);
          }
        }
        acc[cl][cb] = a4;
      }
    }
    // epilogue.  Lane (column n = lane & 15, rows 4 (lane >> 4) + i) of column block cb holds output
    // pixel (y0 + 4 g + i, 16 cb + n) of channel c0 + w + 4 cl.
    lds_barrier();   // staging reads done: the area becomes the [row][column][8 channels] output tile
#pragma unroll
    for (int cl = 0; cl < 2; ++cl) {
      const int chl = w + 4 * cl, c = c0 + chl;
      if (STATS) {
        float s = 0.f;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (4 * g + i < vy && 16 * cb + r16 < p.W) s += acc[cl][cb][i];
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) s += __shfl_xor(s, m);
        const float mu = s / (float)(vy * p.W);
        float q = 0.f;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (4 * g + i < vy && 16 * cb + r16 < p.W) {
              const float d = acc[cl][cb][i] - mu;
              q += d * d;
            }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) q += __shfl_xor(q, m);
        if (lane == 0 && c < p.C) {
          p.stats[(long)unit * 2 * p.stats_ld + c] = s;
          p.stats[(long)unit * 2 * p.stats_ld + p.stats_ld + c] = q;
        }
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i, x = 16 * cb + r16;
          if (r < vy && x < p.W) {
            float o = acc[cl][cb][i];
            if (MODE == DW_FWD_AFFINE) {
              o = o * sc[cl] + sf[cl];
              if (p.act == YMS_ACT_SILU) o = silu_f(o);
            }
            ys[(r * p.W + x) * 8 + chl] = (T)o;
          }
        }
    }
    if (STATS && by == 0 && tid == 0) p.stats_cnt[unit] = (float)(vy * p.W);
    lds_barrier();
    // 16-B NHWC stores (dgrad accumulate: + the destination's values in fp32)
    if (cok) {
      T* dst = reinterpret_cast<T*>(p.dst) + p.dst_off + c0 + ((long)n * p.H + y0) * p.W * p.dst_ld;
      for (int it = tid; it < vy * p.W; it += 256) {
        T* o = dst + (long)it * p.dst_ld;
        const u32x4 val = *reinterpret_cast<const u32x4*>(ys + it * 8);
        if (MODE == DW_DGRAD && p.accumulate) {
          float a[8], b8[8];
          Vec8<T>::load(o, a);
          T t8[8];
          __builtin_memcpy(t8, &val, 16);
#pragma unroll
          for (int e = 0; e < 8; ++e) b8[e] = (float)t8[e] + a[e];
          Vec8<T>::store(o, b8);
        } else {
          *reinterpret_cast<u32x4*>(o) = val;
        }
      }
    }
  }
}

// dw[c][t] (+)= sum_b ws[b][t][c] for few rows (the MFMA kernel's unit groups): one output per
// thread, rows summed in order with all loads in flight
__global__ __launch_bounds__(256) void dwconv_wgrad_reduce_few_kernel(const float* ws, int blocks, int C, int KK,
                                                                      float* dw, int accumulate) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const long stride = (long)C * KK;
  if (j >= stride) return;
  float v[DW_FEW_ROWS];
#pragma unroll
  for (int b = 0; b < DW_FEW_ROWS; ++b) v[b] = b < blocks ? ws[(long)b * stride + j] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int b = 0; b < DW_FEW_ROWS; ++b) s += v[b];
  const int t = j / C, c = j - t * C;
  float* o = dw + (long)c * KK + t;
  *o = accumulate ? *o + s : s;
}

// dw[c][t] (+)= sum_b ws[b][t][c]: 64 outputs per block, 16 waves; wave w sums blocks
// b = w (mod 16) into 4 independent partials (4 loads in flight per lane; one dependent chain
// over ~500 rows made the reduce latency-bound), then a fixed-order tree over the waves
__global__ __launch_bounds__(1024) void dwconv_wgrad_reduce_kernel(const float* ws, int blocks, int C, int KK, float* dw,
                                                                   int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const long stride = (long)C * KK;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < stride) {
    int b = w;
    for (; b + 48 < blocks; b += 64) {
      s0 += ws[(long)b * stride + j];
      s1 += ws[(long)(b + 16) * stride + j];
      s2 += ws[(long)(b + 32) * stride + j];
      s3 += ws[(long)(b + 48) * stride + j];
    }
    for (; b < blocks; b += 16) s0 += ws[(long)b * stride + j];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int h = 8; h >= 1; h >>= 1) {
    if (w < h) red[w][lane] += red[w + h][lane];
    __syncthreads();
  }
  if (w == 0 && j < stride) {
    const float s = red[0][lane];
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

// forward / dgrad tile width (DwTy): whole tiles across the 20 / 40 / 80-wide maps of a 640 input,
// 32 where it divides the width
static int dw_fwd_tx(const yms_dw_shape* s) {
  if (s->w % 32 == 0) return 32;
  if (s->w % 40 == 0) return 40;
  if (s->w <= 20) return 20;
  if (s->w <= 40) return 40;
  return 32;
}
static int dw_fwd_ty(int tx) { return tx == 32 ? 8 : (tx == 40 ? 6 : 12); }
static int dw_fwd_tiles(const yms_dw_shape* s, int& tx, int& ty) {
  const int TX = dw_fwd_tx(s), TY = dw_fwd_ty(TX);
  tx = (s->w + TX - 1) / TX;
  ty = (s->h + TY - 1) / TY;
  return s->n * tx * ty;
}
static int dw_occ(const yms_dw_shape* s) {
  if (s->dtype == YMS_F32) return s->k == 3 ? 2 : 1;
  return s->k == 3 ? 4 : (s->k == 5 ? 3 : 2);
}

// channel groups of 8 per forward / dgrad block: 8 (64 channels = one 128-B line of an NHWC pixel
// per block, 512 threads) for k = 3 when C is a multiple of 64, 7 (56 channels) for k = 3 when C is a
// multiple of 56 but not of 32, else 4 (32 channels: the other part of each line is read and written
// by the neighbouring blocks, on the same XCD).
static int dw_fwd_g(const yms_dw_shape* s) {
  if (s->k != 3 || s->dtype == YMS_F32) return 4;
  if (s->c % 64 == 0) return 8;
  // 56-channel blocks (448 threads) where 32-channel blocks would leave lanes idle: C = 112, 168, ...
  // (k3@160 c112 fwd 306 -> 282 us, dgrad 289 -> 253 us; profiles/r05ze_dw_g7_ab.txt)
  return s->c % 32 != 0 && s->c % 56 == 0 ? 7 : 4;
}

// forward / dgrad grid: image column tiles split into strips of tps tiles.  The strip length is
// chosen so the blocks fill whole rounds of the resident slots (occupancy x CUs): a block walks its
// strip serially, so a last round of a few blocks costs a full strip time, while shorter strips
// re-read K - 1 halo rows each (cost model: rounds x (tps TY + K - 1) rows).
static dim3 dw_strip_grid(const yms_dw_shape* s, DwParams& p) {
  dw_fwd_tiles(s, p.tiles_x, p.tiles_y);
  const int TY = dw_fwd_ty(dw_fwd_tx(s)), G = dw_fwd_g(s);
  const long cg = (s->c + 8 * G - 1) / (8 * G);
  const long base = (long)s->n * p.tiles_x * cg;
  const long slots = (long)(G >= 7 ? 2 : dw_occ(s)) * conv_cu_count();
  double best = 1e30;
  int best_tps = p.tiles_y;
  for (int tps = p.tiles_y; tps >= 1; --tps) {
    const long ys = (p.tiles_y + tps - 1) / tps;
    const long rounds = (base * ys + slots - 1) / slots;
    const double cost = (double)rounds * (tps * TY + s->k - 1);
    if (cost < best * 0.999) { best = cost; best_tps = tps; }
  }
  p.tps = best_tps;
  p.ysplit = (p.tiles_y + p.tps - 1) / p.tps;
  return dim3((unsigned)((long)s->n * p.tiles_x * p.ysplit), (unsigned)cg);
}

// the 1-D launch of a strip kernel's (spatial blocks x channel groups) grid (dw_block)
static dim3 dw_launch(dim3 g, DwParams& p) {
  p.ncg = (int)g.y;
  p.nlog = (int)(g.x * g.y);
  return dim3((unsigned)((p.nlog + 7) / 8 * 8));
}

// forward / dgrad on MFMA (dwconv_mfma_kernel): k = 7, 16-bit types, maps up to 48 wide (two or
// three 16-column blocks).  Measured against the VALU strip kernels on the YOLO-MS shapes
// (profiles/r05x_dw_fm_ab.txt): k = 7 1.0-1.3x faster (forward with statistics 1.3x); k = 3 / 5 / 9
// slower or even (per-unit staging and epilogue through LDS bound it, not the MFMAs), so they stay
// on the VALU kernels.
static bool dw_fm(const yms_dw_shape* s) { return s->k == 7 && s->dtype != YMS_F32 && s->w <= 48; }
static int dw_fm_ncb(const yms_dw_shape* s) { return s->w <= 32 ? 2 : 3; }
// grid: (unit groups, 8-channel groups); units (image, 16 output rows) per block: about two rounds
// of two resident blocks per CU (the weight fragments are built once per block)
static dim3 dw_fm_grid(const yms_dw_shape* s, int& upb) {
  const long units = (long)s->n * ((s->h + 15) / 16), ncg = (s->c + 7) / 8;
  upb = (int)std::max(1l, (units * ncg + 4l * conv_cu_count() - 1) / (4l * conv_cu_count()));
  return dim3((unsigned)((units + upb - 1) / upb), (unsigned)ncg);
}

static bool dw_shape_ok(const yms_dw_shape* s) {
  return s && s->n > 0 && s->h > 0 && s->w > 0 && s->c > 0 && s->c % 8 == 0 && (s->k == 3 || s->k == 5 || s->k == 7 || s->k == 9) &&
         s->dtype >= 0 && s->dtype <= 2 && (long)s->n * s->h * s->w < (1l << 31);
}
static bool dw_view_ok(int ld, int off, int c) { return ld % 8 == 0 && off % 8 == 0 && off + c <= ld; }
// forward / dgrad read one image through a raw buffer resource: 32-bit byte offsets below the
// out-of-range marker NT_OOB
static bool dw_image_fits(const yms_dw_shape* s, int ld) {
  const long esz = s->dtype == YMS_F32 ? 4 : 2;
  return (long)s->h * s->w * ld * esz < (long)NT_OOB;
}

// k = 3 weight gradient on the strip walker (16-bit types; fp32 keeps the tile kernel)
static bool dw_wg3(const yms_dw_shape* s) { return s->k == 3 && s->dtype != YMS_F32; }
// its grid: the forward's tiles, 32-channel blocks (two 256-thread blocks per CU at ~230 VGPRs);
// strips as long as whole rounds of the resident blocks allow (cost model as dw_strip_grid, plus
// the per-strip butterfly and partial row ~ 3 tiles)
static dim3 dw_wg3_grid(const yms_dw_shape* s, DwParams& p) {
  dw_fwd_tiles(s, p.tiles_x, p.tiles_y);
  const int TY = dw_fwd_ty(dw_fwd_tx(s));
  const long cg = (s->c + 31) / 32;
  const long base = (long)s->n * p.tiles_x * cg;
  const long slots = 2l * conv_cu_count();
  double best = 1e30;
  int best_tps = p.tiles_y;
  for (int tps = p.tiles_y; tps >= 1; --tps) {
    const long ys = (p.tiles_y + tps - 1) / tps;
    const long rounds = (base * ys + slots - 1) / slots;
    const double cost = (double)rounds * (tps * TY + s->k - 1 + 3 * TY);
    if (cost < best * 0.999) { best = cost; best_tps = tps; }
  }
  p.tps = best_tps;
  p.ysplit = (p.tiles_y + p.tps - 1) / p.tps;
  return dim3((unsigned)((long)s->n * p.tiles_x * p.ysplit), (unsigned)cg);
}

// k = 5 / 7 / 9 weight gradient on map-shaped tiles with register prefetch (16-bit types)
static bool dw_wg2(const yms_dw_shape* s) { return s->k >= 5 && s->dtype != YMS_F32; }
static void dw_wg2_tile(const yms_dw_shape* s, int& tx, int& ty) {
  tx = dw_fwd_tx(s);    // DwWg2<K, TX>::TY
  ty = tx == 20 ? (s->k == 5 ? 20 : 10) : (s->k == 5 ? 12 : (s->k == 7 ? 9 : 7));
}
// dwconv_wgrad2_kernel grid: tiles of one channel group per block, about two blocks per CU in total
static int dw_wg2_blocks(const yms_dw_shape* s) {
  int tx, ty;
  dw_wg2_tile(s, tx, ty);
  const long tiles = (long)s->n * ((s->w + tx - 1) / tx) * ((s->h + ty - 1) / ty);
  const int cg = (s->c + DW_CB - 1) / DW_CB;
  return (int)std::max(1l, std::min(tiles, std::max(1l, (long)(2 * conv_cu_count()) / cg)));
}

// k = 5 / 7 / 9 weight gradient on MFMA (dwconv_wgrad_mfma_kernel): 16-bit types, maps at most 64
// wide (one or two 32-column chunks per staged row), k = 5 also up to 96 (three chunks: the 2 x 2 x 5
// accumulators leave registers for them; k = 7 / 9 would spill)
static bool dw_wgm(const yms_dw_shape* s) {
  return s->k >= 5 && s->dtype != YMS_F32 && (s->w <= 64 || (s->w <= 96 && s->k == 5));
}
struct DwWgmCfg {
  int nch, nb, nj, ncg, upb, groups;
};
// units = (image, 16 dz rows; 32 for maps of 17-32 rows and one column chunk); 16 channels per block (512 threads, one block per CU: 8 waves of
// ~220 VGPRs; 32-B pixel pieces per block, measured 4-8 % faster on k = 7 than 8-channel blocks at
// two per CU, equal on k = 9); units per block: the fewest that keep the grid within one round of
// the resident blocks; each unit group adds one ws row per tap and channel
static DwWgmCfg dw_wgm_cfg(const yms_dw_shape* s) {
  DwWgmCfg c;
  c.nch = (s->w + 31) / 32;
  // maps of 17-32 rows and one column chunk: both 16-row dz blocks in one unit (one staging)
  c.nb = c.nch == 1 && s->h > 16 && s->h <= 32 ? 2 : 1;
  c.nj = (s->h + 16 * c.nb - 1) / (16 * c.nb);
  c.ncg = (s->c + DW_WGM_CG - 1) / DW_WGM_CG;
  const long units = (long)s->n * c.nj, slots = (DW_WGM_CG == 8 ? 2l : 1l) * conv_cu_count();
  c.upb = (int)std::max(1l, (units * c.ncg + slots - 1) / slots);
  while (c.upb < units && (long)c.ncg * ((units + c.upb - 1) / c.upb) > slots) ++c.upb;
  c.groups = (int)((units + c.upb - 1) / c.upb);
  return c;
}

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
#define YMS_DW_TXS(TXV, ...)                                    \
  do {                                                          \
    if ((TXV) == 40) { constexpr int TXX = 40; __VA_ARGS__; }   \
    else if ((TXV) == 20) { constexpr int TXX = 20; __VA_ARGS__; } \
    else { constexpr int TXX = 32; __VA_ARGS__; }               \
  } while (0)
#define YMS_DW_NCB(V, ...)                                      \
  do {                                                          \
    if ((V) == 2) { constexpr int NCBB = 2; __VA_ARGS__; }      \
    else { constexpr int NCBB = 3; __VA_ARGS__; }               \
  } while (0)
#define YMS_DW_T16(dt, ...)                                     \
  do {                                                          \
    if ((dt) == YMS_BF16) { typedef bf16 TT; __VA_ARGS__; }     \
    else { typedef f16 TT; __VA_ARGS__; }                       \
  } while (0)
#define YMS_DW_T(dt, ...)                                       \
  do {                                                          \
    if ((dt) == YMS_BF16) { typedef bf16 TT; __VA_ARGS__; }     \
    else if ((dt) == YMS_F16) { typedef f16 TT; __VA_ARGS__; }  \
    else { typedef float TT; __VA_ARGS__; }                     \
  } while (0)

// y (+)= a + b over npix x c (b may be NULL): the MS-Block branch sum (X_i + Y_{i-1}) and, with
// b = NULL, its backward (each addend's gradient (+)= the sum's gradient); grid-stride over 16-B items.
// The 16-bit loads of a / b here and of g in add_grad2 are the tensors' last reads and carry the
// non-temporal hint (YOLO-MS-S 34.22 -> 34.06 ms/step interleaved, profiles/r06w_add_nt_ab.txt).
template <typename T>
__global__ __launch_bounds__(256) void add_views_kernel(long items, int cg, const T* a, int a_ld, int a_off,
                                                        const T* b, int b_ld, int b_off, T* y, int y_ld, int y_off,
                                                        int accumulate) {
  for (long it = blockIdx.x * 256l + threadIdx.x; it < items; it += (long)gridDim.x * 256) {
    const long pix = it / cg;
    const int c = (int)(it - pix * cg) * 8;
    float va[8], vb[8], vy[8];
    if constexpr (sizeof(T) == 2) {         // the addends' last reads: non-temporal
      Raw8<T> ra, rb;
      load_raw8_nt(a + pix * a_ld + a_off + c, ra);
      unpack8(ra, va);
      if (b) { load_raw8_nt(b + pix * b_ld + b_off + c, rb); unpack8(rb, vb); }
    } else {
      Vec8<T>::load(a + pix * a_ld + a_off + c, va);
      if (b) Vec8<T>::load(b + pix * b_ld + b_off + c, vb);
    }
    if (accumulate) Vec8<T>::load(y + pix * y_ld + y_off + c, vy);
#pragma unroll
    for (int k = 0; k < 8; ++k) va[k] = (b ? va[k] + vb[k] : va[k]) + (accumulate ? vy[k] : 0.0f);
    Vec8<T>::store(y + pix * y_ld + y_off + c, va);
  }
}

// Backward of y = a + b: g -> ga (+)= g and gb (+)= g in one pass (g read once)
template <typename T>
__global__ __launch_bounds__(256) void add_grad2_kernel(long items, int cg, const T* g, int g_ld, int g_off, T* y1,
                                                        int ld1, int off1, int acc1, T* y2, int ld2, int off2,
                                                        int acc2) {
  for (long it = blockIdx.x * 256l + threadIdx.x; it < items; it += (long)gridDim.x * 256) {
    const long pix = it / cg;
    const int c = (int)(it - pix * cg) * 8;
    float vg[8], v1[8], v2[8];
    if constexpr (sizeof(T) == 2) {         // the sum gradient's last read: non-temporal
      Raw8<T> rg;
      load_raw8_nt(g + pix * g_ld + g_off + c, rg);
      unpack8(rg, vg);
    } else {
      Vec8<T>::load(g + pix * g_ld + g_off + c, vg);
    }
    if (acc1) Vec8<T>::load(y1 + pix * ld1 + off1 + c, v1);
    if (acc2) Vec8<T>::load(y2 + pix * ld2 + off2 + c, v2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v1[k] = acc1 ? v1[k] + vg[k] : vg[k];
      v2[k] = acc2 ? v2[k] + vg[k] : vg[k];
    }
    Vec8<T>::store(y1 + pix * ld1 + off1 + c, v1);
    Vec8<T>::store(y2 + pix * ld2 + off2 + c, v2);
  }
}
static unsigned add_grid(long items) { return (unsigned)std::min<long>((items + 255) / 256, 16384); }

}  // namespace yms

using namespace yms;

extern "C" {

int yms_dwconv_stats_rows(const yms_dw_shape* s) {
  if (!dw_shape_ok(s)) return 0;
  if (dw_fm(s)) return s->n * ((s->h + 15) / 16);
  int tx, ty;
  return dw_fwd_tiles(s, tx, ty);
}

yms_status yms_dwconv_fwd(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const float* w, void* y,
                          int y_ld, int y_off, const float* scale, const float* shift, int act, float* stats,
                          int stats_ld, void* stream) {
  if (!dw_shape_ok(s) || !x || !w || !y || !dw_view_ok(x_ld, x_off, s->c) || !dw_view_ok(y_ld, y_off, s->c))
    return YMS_ERR_INVALID;
  if (stats && stats_ld < s->c) return YMS_ERR_INVALID;
  if (!dw_image_fits(s, x_ld) || !dw_image_fits(s, y_ld)) return YMS_ERR_UNSUPPORTED;
  if (stats && (long)yms_dwconv_stats_rows(s) * 2 * stats_ld * 4 >= (long)NT_OOB) return YMS_ERR_UNSUPPORTED;
  DwParams p{};
  p.src = (const char*)x; p.src_ld = x_ld; p.src_off = x_off; p.w = w;
  p.dst = (char*)y; p.dst_ld = y_ld; p.dst_off = y_off;
  p.scale = scale; p.shift = shift; p.act = act; p.stats = stats; p.stats_ld = stats_ld;
  if (stats) p.stats_cnt = stats + (long)yms_dwconv_stats_rows(s) * 2 * stats_ld;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  hipStream_t st = (hipStream_t)stream;
  if (dw_fm(s)) {
    int upb;
    const dim3 grid = dw_launch(dw_fm_grid(s, upb), p);
    YMS_DW_T16(s->dtype, YMS_DW_NCB(dw_fm_ncb(s), {
      if (stats) hipLaunchKernelGGL((dwconv_mfma_kernel<TT, 7, NCBB, DW_FWD_STATS>), grid, dim3(256), 0, st, p, upb);
      else hipLaunchKernelGGL((dwconv_mfma_kernel<TT, 7, NCBB, DW_FWD_AFFINE>), grid, dim3(256), 0, st, p, upb);
    }));
    return launch_status();
  }
  const dim3 grid = dw_launch(dw_strip_grid(s, p), p);
  const int TX = dw_fwd_tx(s);
  if (dw_fwd_g(s) == 8) {
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, {
      if (stats) hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_FWD_STATS, TXX, 8>), grid, dim3(512), 0, st, p);
      else hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_FWD_AFFINE, TXX, 8>), grid, dim3(512), 0, st, p);
    }));
    return launch_status();
  }
  if (dw_fwd_g(s) == 7) {
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, {
      if (stats) hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_FWD_STATS, TXX, 7>), grid, dim3(448), 0, st, p);
      else hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_FWD_AFFINE, TXX, 7>), grid, dim3(448), 0, st, p);
    }));
    return launch_status();
  }
  YMS_DW_T(s->dtype, YMS_DW_K(s->k, YMS_DW_TXS(TX, {
    if (stats) hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_FWD_STATS, TXX>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_FWD_AFFINE, TXX>), grid, dim3(256), 0, st, p);
  })));
  return launch_status();
}

yms_status yms_dwconv_dgrad(const yms_dw_shape* s, const void* dz, int dz_ld, int dz_off, const float* w, void* dx,
                            int dx_ld, int dx_off, int accumulate, void* stream) {
  if (!dw_shape_ok(s) || !dz || !w || !dx || !dw_view_ok(dz_ld, dz_off, s->c) || !dw_view_ok(dx_ld, dx_off, s->c))
    return YMS_ERR_INVALID;
  if (!dw_image_fits(s, dz_ld) || !dw_image_fits(s, dx_ld)) return YMS_ERR_UNSUPPORTED;
  DwParams p{};
  p.src = (const char*)dz; p.src_ld = dz_ld; p.src_off = dz_off; p.w = w;
  p.dst = (char*)dx; p.dst_ld = dx_ld; p.dst_off = dx_off; p.accumulate = accumulate;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  hipStream_t st = (hipStream_t)stream;
  if (dw_fm(s)) {
    int upb;
    const dim3 grid = dw_launch(dw_fm_grid(s, upb), p);
    YMS_DW_T16(s->dtype, YMS_DW_NCB(dw_fm_ncb(s), hipLaunchKernelGGL((dwconv_mfma_kernel<TT, 7, NCBB, DW_DGRAD>), grid,
                                                                      dim3(256), 0, st, p, upb)));
    return launch_status();
  }
  const dim3 grid = dw_launch(dw_strip_grid(s, p), p);
  const int TX = dw_fwd_tx(s);
  if (dw_fwd_g(s) == 8) {
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_DGRAD, TXX, 8>), grid, dim3(512), 0,
                                                           st, p)));
    return launch_status();
  }
  if (dw_fwd_g(s) == 7) {
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, hipLaunchKernelGGL((dwconv_kernel<TT, 3, DW_DGRAD, TXX, 7>), grid, dim3(448), 0,
                                                           st, p)));
    return launch_status();
  }
  YMS_DW_T(s->dtype, YMS_DW_K(s->k, YMS_DW_TXS(TX, hipLaunchKernelGGL((dwconv_kernel<TT, KK, DW_DGRAD, TXX>), grid,
                                                                     dim3(256), 0, st, p))));
  return launch_status();
}

size_t yms_dwconv_wgrad_ws_bytes(const yms_dw_shape* s) {
  if (!dw_shape_ok(s)) return 0;
  const size_t row = (size_t)s->k * s->k * s->c * sizeof(float);
  if (dw_wg3(s)) {
    DwParams p{};
    return (size_t)dw_wg3_grid(s, p).x * row;
  }
  if (dw_wgm(s)) {
    const DwWgmCfg c = dw_wgm_cfg(s);
    return (size_t)c.groups * row;
  }
  return (size_t)(dw_wg2(s) ? dw_wg2_blocks(s) : dw_wgrad_blocks(s)) * row;
}

yms_status yms_dwconv_wgrad(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const void* dz, int dz_ld,
                            int dz_off, float* ws, size_t ws_bytes, float* dw, int accumulate, void* stream) {
  if (!dw_shape_ok(s) || !x || !dz || !ws || !dw || !dw_view_ok(x_ld, x_off, s->c) || !dw_view_ok(dz_ld, dz_off, s->c))
    return YMS_ERR_INVALID;
  if (ws_bytes < yms_dwconv_wgrad_ws_bytes(s)) return YMS_ERR_INVALID;
  DwParams p{};
  p.src = (const char*)x; p.src_ld = x_ld; p.src_off = x_off;
  p.N = s->n; p.H = s->h; p.W = s->w; p.C = s->c;
  hipStream_t st = (hipStream_t)stream;
  const int KK2 = s->k * s->k;
  int blocks;
  if (dw_wg3(s)) {
    if (!dw_image_fits(s, x_ld)) return YMS_ERR_UNSUPPORTED;
    const dim3 g2 = dw_wg3_grid(s, p), grid = dw_launch(g2, p);
    const int TX = dw_fwd_tx(s);
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, hipLaunchKernelGGL((dwconv_wgrad3_kernel<TT, TXX, 4>), grid, dim3(256), 0, st,
                                                           p, (const char*)dz, dz_ld, dz_off, ws)));
    blocks = (int)g2.x;
  } else if (dw_wgm(s)) {
    if (!dw_image_fits(s, x_ld) || !dw_image_fits(s, dz_ld)) return YMS_ERR_UNSUPPORTED;
    const DwWgmCfg c = dw_wgm_cfg(s);
    blocks = c.groups;
    const dim3 grid((unsigned)(((long)c.groups * c.ncg + 7) / 8 * 8));
#define YMS_DWM_L(KV, NV, NBV)                                                                              \
  hipLaunchKernelGGL((dwconv_wgrad_mfma_kernel<TT, KV, NV, DW_WGM_CG, NBV>), grid, dim3(32 * DW_WGM_CG), 0, st, p,     \
                     (const char*)dz, dz_ld, dz_off, ws, c.nj, c.upb, c.ncg, c.groups)
    YMS_DW_T16(s->dtype, {
      if (c.nch == 1 && c.nb == 2) {
        if (s->k == 5) YMS_DWM_L(5, 1, 2);
        else if (s->k == 7) YMS_DWM_L(7, 1, 2);
        else YMS_DWM_L(9, 1, 2);
      } else if (c.nch == 1) {
        if (s->k == 5) YMS_DWM_L(5, 1, 1);
        else if (s->k == 7) YMS_DWM_L(7, 1, 1);
        else YMS_DWM_L(9, 1, 1);
      } else if (c.nch == 2) {
        if (s->k == 5) YMS_DWM_L(5, 2, 1);
        else if (s->k == 7) YMS_DWM_L(7, 2, 1);
        else YMS_DWM_L(9, 2, 1);
      } else {
        YMS_DWM_L(5, 3, 1);
      }
    });
#undef YMS_DWM_L
  } else if (dw_wg2(s)) {
    blocks = dw_wg2_blocks(s);
    const dim3 grid((unsigned)blocks, (unsigned)((s->c + DW_CB - 1) / DW_CB));
    const int TX = dw_fwd_tx(s);
    YMS_DW_T16(s->dtype, YMS_DW_TXS(TX, {
      if (s->k == 5) hipLaunchKernelGGL((dwconv_wgrad2_kernel<TT, 5, TXX>), grid, dim3(DW_WG_NT), 0, st, p,
                                        (const char*)dz, dz_ld, dz_off, ws);
      else if (s->k == 7) hipLaunchKernelGGL((dwconv_wgrad2_kernel<TT, 7, TXX>), grid, dim3(DW_WG_NT), 0, st, p,
                                             (const char*)dz, dz_ld, dz_off, ws);
      else hipLaunchKernelGGL((dwconv_wgrad2_kernel<TT, 9, TXX>), grid, dim3(DW_WG_NT), 0, st, p, (const char*)dz,
                              dz_ld, dz_off, ws);
    }));
  } else {
    dw_tiles(s, p.tiles_x, p.tiles_y);
    blocks = dw_wgrad_blocks(s);
    const dim3 grid((unsigned)blocks, (unsigned)((s->c + DW_CB - 1) / DW_CB));
    YMS_DW_T(s->dtype, YMS_DW_K(s->k, hipLaunchKernelGGL((dwconv_wgrad_kernel<TT, KK>), grid, dim3(DW_WG_NT), 0, st, p,
                                                        (const char*)dz, dz_ld, dz_off, ws)));
  }
  yms_status e = launch_status();
  if (e != YMS_OK) return e;
  if (blocks <= DW_FEW_ROWS)
    hipLaunchKernelGGL(dwconv_wgrad_reduce_few_kernel, dim3((unsigned)((s->c * KK2 + 255) / 256)), dim3(256), 0, st, ws,
                       blocks, s->c, KK2, dw, accumulate);
  else
    hipLaunchKernelGGL(dwconv_wgrad_reduce_kernel, dim3((unsigned)((s->c * KK2 + 63) / 64)), dim3(1024), 0, st, ws,
                       blocks, s->c, KK2, dw, accumulate);
  return launch_status();
}

yms_status yms_add_views(int dtype, long npix, int c, const void* a, int a_ld, int a_off, const void* b, int b_ld,
                         int b_off, void* y, int y_ld, int y_off, int accumulate, void* stream) {
  if (npix <= 0 || c <= 0 || c % 8 || !a || !y || !dw_view_ok(a_ld, a_off, c) || !dw_view_ok(y_ld, y_off, c))
    return YMS_ERR_INVALID;
  if (b && !dw_view_ok(b_ld, b_off, c)) return YMS_ERR_INVALID;
  const long items = npix * (c / 8);
  YMS_DW_T(dtype, hipLaunchKernelGGL((add_views_kernel<TT>), dim3(add_grid(items)), dim3(256), 0, (hipStream_t)stream,
                                     items, c / 8, (const TT*)a, a_ld, a_off, (const TT*)b, b_ld, b_off, (TT*)y, y_ld,
                                     y_off, accumulate));
  return launch_status();
}

yms_status yms_add_grad2(int dtype, long npix, int c, const void* g, int g_ld, int g_off, void* y1, int ld1,
                         int off1, int acc1, void* y2, int ld2, int off2, int acc2, void* stream) {
  if (npix <= 0 || c <= 0 || c % 8 || !g || !y1 || !y2 || !dw_view_ok(g_ld, g_off, c) || !dw_view_ok(ld1, off1, c) ||
      !dw_view_ok(ld2, off2, c))
    return YMS_ERR_INVALID;
  const long items = npix * (c / 8);
  YMS_DW_T(dtype, hipLaunchKernelGGL((add_grad2_kernel<TT>), dim3(add_grid(items)), dim3(256), 0, (hipStream_t)stream,
                                     items, c / 8, (const TT*)g, g_ld, g_off, (TT*)y1, ld1, off1, acc1, (TT*)y2, ld2,
                                     off2, acc2));
  return launch_status();
}

}  // extern "C"

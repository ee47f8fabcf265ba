// Implicit-GEMM convolution for gfx950 (MI355X) on MFMA, NHWC activations.
//
// Replaces the reference's Conv = Conv2d(bias=False) -> BatchNorm2d -> SiLU
// (yolov8/model/components.py:69-77), its residual add (Bottleneck, :87-93), the channel
// concatenations feeding C2f/SPPF/neck/head (:119, :146; yolov8_neck.py:79-91;
// yolov8_head.py:122 -- producers write at a channel offset of the consumer's buffer),
// the head's biased 1x1 nn.Conv2d (yolov8_head.py:86-109) and the autograd of all of them.
//
// GEMM views (rows = pixels, 16-B "chunks" of 8 bf16/f16 or 4 f32 channels along K):
//   forward : Y[pix][co]  = sum_{tap,ci} X[src(pix,tap)][ci] * W[co][tap,ci]      (NT)
//   dgrad   : DX[pix][ci] = sum_{tap,co} DZ[src'(pix,tap)][co] * W[co][ci][tap]    (NT)
//   wgrad   : DW[co][tap,ci] = sum_pix DZ[pix][co] * X[src(pix,tap)][ci]           (TT)
// NT tiles are staged global->regs->LDS as [rows][64 B of K] (80-B padded pitch, bank-
// conflict-free for ds_read_b128) and consumed by v_mfma_f32_32x32x16_{bf16,f16}
// (or v_mfma_f32_32x32x2_f32 for the exact-fp32 path).  TT tiles are staged as
// [32 pixels][cols] and read with ds_read_b64_tr_b16 (hardware transpose) so both
// operands get 8 consecutive pixels per lane.  wgrad is split over pixels into fp32
// partial slabs that a second kernel reduces deterministically (no atomics).
#include "conv_common.hpp"
#include "conv_direct.hpp"
#include "wgrad_halo.hpp"
#include "wgrad_ring.hpp"

namespace yms {

struct NTParams {
  const char* src;
  const char* wp;
  char* dst;
  int src_ld, src_off, dst_ld, dst_off;
  const float* scale;
  const float* shift;
  int act;
  const char* res;
  int res_ld, res_off;
  float* stats;
  int stats_ld;
  float* stats_cnt; // per-row pixel counts (right after the rows, conv_common.hpp contract)
  int SH, SW;       // source spatial dims
  int OW;           // row-space width
  int stride, pad;
  int cpt;          // 16-B chunks per tap along source channels
  uint64_t cpt_magic;   // kc / cpt == (kc * cpt_magic) >> 32 for every kc < nkt * 8 (host-checked)
  uint32_t src_bytes;   // byte extent of the source view's buffer (raw-buffer num_records, < 2^31)
  int Kc;           // valid K chunks
  int nkt;          // K tiles (4 chunks each)
  int M;            // rows (pixels)
  int Ncols;        // valid output columns
  int tiles_n;
  FastDiv div_ow, div_ohw;
  // MODE_DGRAD2: one GEMM per output-parity class (ry, rx) = (blockIdx.y >> 1, blockIdx.y & 1).
  // Class rows are the dx pixels (n, 2a+ry, 2b+rx); its taps are kh = kh0 + 2*jy, kw = kw0 + 2*jx,
  // reading dz at (a + c0y - jy, b + c0x - jx); weights are packed per class.
  int OH, OWx;                      // dx spatial dims (for the output pixel index)
  int cls_M[4], cls_nkt[4], cls_Kc[4], cls_ntx[4], cls_c0y[4], cls_c0x[4];
  long cls_woff[4];                 // byte offset of the class' packed weight block
  FastDiv cls_div_w[4], cls_div_hw[4];
};

// 16-B zero chunk: out-of-image / out-of-K im2col lanes load from here, so the A loads are
// branch-free (no exec-masked regions around each global load).
__device__ __attribute__((aligned(64))) u32x4 g_zero_chunk[4];

// 16-bit types (GL): k-tiles are staged global->LDS directly with global_load_lds_dwordx4 into
// an ST-deep ring of unpadded 128-B rows; 16-B chunk c of row r lives in slot
// c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 for 16 consecutive rows), which is realised
// by swizzling each lane's global SOURCE address since the LDS image of one wave-instruction is
// lane-linear.  The wait for k-tile kt is a counted vmcnt that leaves ST-2 later tiles in
// flight across a raw s_barrier.  fp32 keeps the register-staged double buffer.
template <typename T, int KS, int MODE, int EPI, int BM, int BN, int WGM, int WGN, int ST>
__global__ __launch_bounds__(256, 2) void conv_nt_kernel(NTParams p) {
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int RSTEP = 256 / NT_KCH;                      // rows covered by one load pass
  constexpr int A_SLOTS = BM / RSTEP;
  constexpr int B_CHUNKS = BN * NT_KCH;
  constexpr int B_SLOTS = (B_CHUNKS + 255) / 256;
  constexpr bool F32 = sizeof(T) == 4;
  constexpr bool GL = !F32;
  constexpr int PITCH = GL ? 128 : NT_ROWP;
  constexpr int NSTAGE = GL ? ST : 2;
  constexpr int TILE_BYTES = (BM + BN) * PITCH;
  constexpr int EPI_P = BN + 4;                            // fp32 staging pitch (floats)
  constexpr int SMEM = (NSTAGE * TILE_BYTES > BM * EPI_P * 4) ? NSTAGE * TILE_BYTES : BM * EPI_P * 4;
  static_assert(!GL || B_CHUNKS % 256 == 0, "GL loader needs whole B passes");
  static_assert(TM >= 1 && TN >= 1 && A_SLOTS >= 1, "bad tile");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = wg % p.tiles_n, tile_m = wg / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  int M = p.M, nkt = p.nkt, Kc = p.Kc, ntx = 1, cls = 0;
  const char* wp = p.wp;
  FastDiv dv_w = p.div_ow, dv_hw = p.div_ohw;
  if (MODE == MODE_DGRAD2) {
    cls = blockIdx.y;
    M = p.cls_M[cls];
    nkt = p.cls_nkt[cls];
    Kc = p.cls_Kc[cls];
    ntx = p.cls_ntx[cls];
    wp = p.wp + p.cls_woff[cls];
    dv_w = p.cls_div_w[cls];
    dv_hw = p.cls_div_hw[cls];
    if (m0 >= M) return;   // uniform: this class has fewer row tiles
  }

  // ---- im2col loader state (A side): fixed chunk column q, rows r0 + RSTEP*i ----
  // (GL: the thread fills LDS slot tid&7 of rows r0 + 32i, i.e. chunk (tid&7) ^ ((tid>>4)&7))
  const int q = GL ? ((tid & 7) ^ ((tid >> 4) & 7)) : (tid & (NT_KCH - 1)), r0 = tid / NT_KCH;
  // Per row slot: the element offset of its tap-(0,0) source pixel (32-bit; the host checks
  // the source fits) and a bit mask of the taps that land inside the image.  Per k-tile the
  // A address is then offset + delta(tap) + channel chunk, with no per-tap bounds arithmetic.
  // Tap t displaces the source pixel by (dy, dx): forward (+t/KS, +t%KS); stride-1 dgrad
  // (-t/KS, -t%KS); stride-2 dgrad parity class (-jy, -jx).
  constexpr int NTAPS = MODE == MODE_DGRAD2 ? 4 : KS * KS;
  constexpr int SGN = MODE == MODE_FWD ? 1 : -1;
  auto tap_dyx = [&](int t, int& dy, int& dx) {
    if (MODE == MODE_DGRAD2) {
      dy = ntx == 1 ? t : (t >> 1);
      dx = ntx == 1 ? 0 : (t & 1);
    } else {
      dy = t / KS;
      dx = t - (t / KS) * KS;
    }
  };
  int a_off[A_SLOTS];
  uint32_t a_msk[A_SLOTS];
#pragma unroll
  for (int i = 0; i < A_SLOTS; ++i) {
    const int m = m0 + r0 + RSTEP * i;
    const bool row_ok = m < M;
    const uint32_t mm = row_ok ? (uint32_t)m : 0u;
    const uint32_t n = fdiv(mm, dv_hw);
    const uint32_t rem = mm - n * dv_hw.d;
    const uint32_t oy = fdiv(rem, dv_w);
    const uint32_t ox = rem - oy * dv_w.d;
    int y0, x0;
    if (MODE == MODE_FWD) {
      y0 = (int)oy * p.stride - p.pad;
      x0 = (int)ox * p.stride - p.pad;
    } else if (MODE == MODE_DGRAD) {
      y0 = (int)oy + p.pad;
      x0 = (int)ox + p.pad;
    } else {
      y0 = (int)oy + p.cls_c0y[cls];
      x0 = (int)ox + p.cls_c0x[cls];
    }
    a_off[i] = (((int)n * p.SH + y0) * p.SW + x0) * p.src_ld + p.src_off;
    uint32_t msk = 0;
#pragma unroll
    for (int t = 0; t < NTAPS; ++t) {
      int dy, dx;
      tap_dyx(t, dy, dx);
      const int iy = y0 + SGN * dy, ix = x0 + SGN * dx;
      if (row_ok && iy >= 0 && iy < p.SH && ix >= 0 && ix < p.SW) msk |= 1u << t;
    }
    a_msk[i] = msk;
  }
  int tap = q / p.cpt, cc = q - (q / p.cpt) * p.cpt;
  constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B chunk

  u32x4 a_reg[A_SLOTS], b_reg[B_SLOTS];

  // GL: buf = ring stage to fill with LDS-DMA; register path: buf unused (a_reg/b_reg)
  auto load_tile = [&](int kt, int buf) {
    char* lds_a = smem + buf * TILE_BYTES + wave * 1024;
    char* lds_b = smem + buf * TILE_BYTES + BM * PITCH + wave * 1024;
    (void)lds_a; (void)lds_b;
    const int kc = kt * NT_KCH + q;
    const bool kok = kc < Kc;
    int dy, dx;
    tap_dyx(tap, dy, dx);
    const int delta = SGN * (dy * p.SW + dx) * p.src_ld + cc * EPC;
    const uint32_t tbit = 1u << (tap & 31);
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const bool ok = kok && (a_msk[i] & tbit);
      const char* ap = ok ? p.src + (long)(a_off[i] + delta) * (long)sizeof(T)
                          : reinterpret_cast<const char*>(g_zero_chunk);
      if constexpr (GL) glds16(ap, lds_a + i * 256 * 16);
      else a_reg[i] = *reinterpret_cast<const u32x4*>(ap);
    }
#pragma unroll
    for (int j = 0; j < B_SLOTS; ++j) {
      const int c = tid + 256 * j;
      if (B_CHUNKS >= 256 * (j + 1) || c < B_CHUNKS) {
        const int row = c / NT_KCH, qq = GL ? q : c % NT_KCH;   // GL: swizzled source chunk
        const long off = ((long)(n0 + row) * (nkt * NT_KCH) + kt * NT_KCH + qq) * 16;
        if constexpr (GL) glds16(wp + off, lds_b + j * 256 * 16);
        else b_reg[j] = *reinterpret_cast<const u32x4*>(wp + off);
      }
    }
    // advance the tap cursor by one k-tile of chunks
    cc += NT_KCH;
    while (cc >= p.cpt) { cc -= p.cpt; ++tap; }
  };

  auto store_tile = [&](int buf) {
    char* A = smem + buf * TILE_BYTES;
    char* B = A + BM * NT_ROWP;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i)
      *reinterpret_cast<u32x4*>(A + (r0 + RSTEP * i) * NT_ROWP + q * 16) = a_reg[i];
#pragma unroll
    for (int j = 0; j < B_SLOTS; ++j) {
      const int c = tid + 256 * j;
      if (B_CHUNKS >= 256 * (j + 1) || c < B_CHUNKS)
        *reinterpret_cast<u32x4*>(B + (c / NT_KCH) * NT_ROWP + (c % NT_KCH) * 16) = b_reg[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  const int lr = lane & 31, lh = lane >> 5;
  // The whole 128-B k-tile is always computed: chunks beyond K are zero on both sides (A
  // loads the zero chunk, packed weights are zero-padded), so no branches split the MFMA
  // stream and the fragment reads of substep s+1 overlap the MFMAs of substep s.
  auto compute = [&](int buf) {
    const char* A = smem + buf * TILE_BYTES;
    const char* B = A + BM * PITCH;
    if constexpr (!F32) {
      u32x4 af[2][TM], bfr[2][TN];
      const int swz = (lr >> 1) & 7;   // rows of a fragment differ from lr by multiples of 16
      auto frags = [&](int s, int slot) {
        const int co = ((2 * s + lh) ^ swz) * 16;
#pragma unroll
        for (int a = 0; a < TM; ++a)
          af[slot][a] = *reinterpret_cast<const u32x4*>(A + (wm * WTM + a * 32 + lr) * PITCH + co);
#pragma unroll
        for (int b = 0; b < TN; ++b)
          bfr[slot][b] = *reinterpret_cast<const u32x4*>(B + (wn * WTN + b * 32 + lr) * PITCH + co);
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
    } else {
      // fp32: per 64-B substep lane (r,h) holds k = 8h..8h+7; MFMA j pairs element j of both halves.
#pragma unroll
      for (int s = 0; s < NT_KCH / 4; ++s) {
        {
          float af[TM][8], bfr[TN][8];
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            const float4* src = reinterpret_cast<const float4*>(A + (wm * WTM + a * 32 + lr) * NT_ROWP + 64 * s + 32 * lh);
            float4 u = src[0], v = src[1];
            af[a][0] = u.x; af[a][1] = u.y; af[a][2] = u.z; af[a][3] = u.w;
            af[a][4] = v.x; af[a][5] = v.y; af[a][6] = v.z; af[a][7] = v.w;
          }
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const float4* src = reinterpret_cast<const float4*>(B + (wn * WTN + b * 32 + lr) * NT_ROWP + 64 * s + 32 * lh);
            float4 u = src[0], v = src[1];
            bfr[b][0] = u.x; bfr[b][1] = u.y; bfr[b][2] = u.z; bfr[b][3] = u.w;
            bfr[b][4] = v.x; bfr[b][5] = v.y; bfr[b][6] = v.z; bfr[b][7] = v.w;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
              for (int b = 0; b < TN; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][j], bfr[b][j], acc[a][b], 0, 0, 0);
        }
      }
    }
  };

  if constexpr (GL) {
    // ---- main loop: ST-deep LDS-DMA ring, one raw barrier per 128-B k-tile ----
    constexpr int NG = A_SLOTS + B_SLOTS;   // LDS-DMA instructions per thread per k-tile
#pragma unroll
    for (int s0 = 0; s0 < ST - 1; ++s0)
      if (s0 < nkt) load_tile(s0, s0);
    int stage = 0;
    for (int kt = 0; kt < nkt; ++kt) {
      // k-tiles issued after kt (at most ST-2 of them) may stay in flight
      const int ahead = nkt - 1 - kt;
      if (ST >= 4 && ahead >= 2) wait_vmcnt<(ST >= 4 ? 2 * NG : 0)>();
      else if (ST >= 3 && ahead >= 1) wait_vmcnt<(ST >= 3 ? NG : 0)>();
      else wait_vmcnt<0>();
      raw_barrier();                        // k-tile kt visible to all; stage of kt-1 free
      if (kt + ST - 1 < nkt) {
        int ns = stage + ST - 1;
        if (ns >= ST) ns -= ST;
        load_tile(kt + ST - 1, ns);
      }
      compute(stage);
      if (++stage == ST) stage = 0;
    }
    __syncthreads();
  } else {
    // ---- main loop: register-staged double buffer, one barrier per 128-B k-tile ----
    load_tile(0, 0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nkt;
      if (more) load_tile(kt + 1, 0);
      compute(cur);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: stage the fp32 tile in LDS, then 16-B coalesced row segments ----
  float* st = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rl = wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        st[rl * EPI_P + wn * WTN + b * 32 + lr] = acc[a][b][i];
      }
  __syncthreads();
  constexpr int CH = BN / 8;              // 8-channel chunks per row
  constexpr int RS = 256 / CH;            // row lanes
  constexpr int NR = BM / RS;             // rows per thread
  const int ch = tid % CH, rr = tid / CH;
  const int col0 = n0 + ch * 8;
  const int nv = p.Ncols - col0;          // valid channels in this chunk (may be <= 0)
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = 1.0f;
    sh[i] = 0.0f;
    if (EPI == EPI_AFFINE && i < nv) {
      if (p.scale) sc[i] = p.scale[col0 + i];
      if (p.shift) sh[i] = p.shift[col0 + i];
    }
  }
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int rl = rr + RS * j;
    int row = m0 + rl;
    float v[8];
    const float4 u0 = *reinterpret_cast<const float4*>(st + rl * EPI_P + ch * 8);
    const float4 u1 = *reinterpret_cast<const float4*>(st + rl * EPI_P + ch * 8 + 4);
    v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w;
    v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
    if (row >= M || nv <= 0) continue;
    if (MODE == MODE_DGRAD2) {
      const uint32_t n = fdiv((uint32_t)row, dv_hw);
      const uint32_t rem = (uint32_t)row - n * dv_hw.d;
      const uint32_t ya = fdiv(rem, dv_w);
      const uint32_t xb = rem - ya * dv_w.d;
      row = ((int)n * p.OH + 2 * (int)ya + (cls >> 1)) * p.OWx + 2 * (int)xb + (cls & 1);
    }
    T* dst = reinterpret_cast<T*>(p.dst) + (long)row * p.dst_ld + p.dst_off + col0;
    if (EPI == EPI_AFFINE) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float a = v[i] * sc[i] + sh[i];
        if (p.act == YMS_ACT_SILU) a = silu_f(a);
        v[i] = a;
      }
      if (p.res) {
        float r[8];
        load8(reinterpret_cast<const T*>(p.res) + (long)row * p.res_ld + p.res_off + col0, nv, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += r[i];
      }
    } else if (EPI == EPI_ACCUM) {
      float r[8];
      load8(dst, nv, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += r[i];
    }
    store8(dst, nv, v);
  }
  if (EPI == EPI_STATS) {
    // one statistics row per 128-row tile (BM == 128): sum and centred M2 of each column over
    // the valid rows, two passes down the fp32 staging tile (read-only since the barrier above)
    static_assert(EPI != EPI_STATS || BM == 128, "statistics rows are 128 output rows");
    if (tid < BN) {
      const int nrow = min(BM, M - m0);
      float t1 = 0.f, t2 = 0.f;
      for (int r = 0; r < nrow; ++r) t1 += st[r * EPI_P + tid];
      const float mu = t1 / (float)nrow;
      for (int r = 0; r < nrow; ++r) {
        const float d = st[r * EPI_P + tid] - mu;
        t2 += d * d;
      }
      float* so = p.stats + (long)tile_m * 2 * p.stats_ld;
      so[n0 + tid] = t1;
      so[p.stats_ld + n0 + tid] = t2;
      if (tile_n == 0 && tid == 0) p.stats_cnt[tile_m] = (float)nrow;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Persistent NT kernel (16-bit types).  Each block walks output tiles lb, lb+G, lb+2G, ...
// (lb = XCD-remapped block id, G = grid size) as ONE flattened (tile, k-tile) stream: the
// ST-deep LDS-DMA ring keeps prefetching across tile boundaries, so a tile's epilogue overlaps
// the next tile's loads and no pipeline fill/drain is paid per tile.  The epilogue applies
// the affine/SiLU to the fp32 accumulators in registers (BN statistics are reduced from them
// by cross-lane adds), stages the tile as T through the ring stage just consumed, and writes
// 16-B row segments (+ residual / + accumulate in fp32).
// ------------------------------------------------------------------------------------------
constexpr int NTP_MAX_AFFINE_COLS = 512;   // wider affine outputs use conv_nt_kernel
template <typename T, int KS, int MODE, int EPI, int BM, int BN, int WGM, int WGN, int ST, bool UNI, int OCC = 2>
__global__ __launch_bounds__(WGM * WGN * 64, OCC) void conv_ntp_kernel(NTParams p) {
  constexpr int NTHR = WGM * WGN * 64;
  constexpr int RPP = NTHR / NT_KCH;                       // rows per load pass (one slot)
  constexpr int SLOT = RPP * 128;                          // LDS bytes per slot
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_SLOTS = BM / RPP;
  constexpr bool B_PART = BN < RPP;                         // only the first BN/8 waves load B
  constexpr int B_SLOTS = B_PART ? 1 : BN / RPP;
  constexpr int STAGE = (BM + BN) * 128;
  // statistics: per-wave column partials [WGM][2][BN] + the combiner threads' running moments
  // [3][SROWS*BN] (kept in LDS: three more live VGPRs would cost a block per CU)
  constexpr int RED = (EPI == EPI_STATS) ? (WGM * 2 + 3 * (BM / 128 > 0 ? BM / 128 : 1)) * BN * 4 : 0;
  constexpr int PRM = (EPI == EPI_AFFINE) ? 2 * NTP_MAX_AFFINE_COLS * 4 : 0;
  static_assert((B_PART || BN % RPP == 0) && BM % RPP == 0 && BN <= NTHR, "tile");
  // the output tile is staged through the ring stage just consumed, in NH passes of HR rows
  constexpr int NH = (BM * BN * (int)sizeof(T) > STAGE) ? 2 : 1;
  constexpr int HR = BM / NH;
  static_assert(HR * BN * (int)sizeof(T) <= STAGE && HR % (BM / WGM) == 0, "staging must fit one ring stage");
  // BN statistics: every block walks tiles of ONE column tile (the grid is a multiple of tiles_n),
  // so it keeps per-column running moments of its tiles (Chan merges, in the combiner threads'
  // registers) and writes one row per 128-row half of its tiles, slot lb / tiles_n, at the end
  // (yms_conv_stats_rows = SROWS x grid / tiles_n, counts after the rows)
  constexpr int SROWS = BM / 128 > 0 ? BM / 128 : 1;
  static_assert(BM % 128 == 0 && WGM % SROWS == 0, "statistics rows");
  __shared__ __attribute__((aligned(16))) char smem[ST * STAGE + RED + PRM + 16];
  float* red = reinterpret_cast<float*>(smem + ST * STAGE);
  float* prm = reinterpret_cast<float*>(smem + ST * STAGE + RED);   // [scale | shift] per column

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int lr = lane & 31, lh = lane >> 5;
  int M = p.M, nkt = p.nkt, Kc = p.Kc, ntx = 1, cls = 0;
  const char* wp = p.wp;
  FastDiv dv_w = p.div_ow, dv_hw = p.div_ohw;
  if (MODE == MODE_DGRAD2) {
    cls = blockIdx.y;
    M = p.cls_M[cls];
    nkt = p.cls_nkt[cls];
    Kc = p.cls_Kc[cls];
    ntx = p.cls_ntx[cls];
    wp = p.wp + p.cls_woff[cls];
    dv_w = p.cls_div_w[cls];
    dv_hw = p.cls_div_hw[cls];
  }
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int ntiles = ((M + BM - 1) / BM) * p.tiles_n;
  if (lb >= ntiles || nkt <= 0) return;
  const int my_tiles = (ntiles - lb + G - 1) / G;
  const int total = my_tiles * nkt;
  if constexpr (EPI == EPI_AFFINE) {
    // per-column BN scale/shift kept in LDS: an epilogue global load would make the compiler
    // drain (vmcnt(0)) the LDS-DMA prefetch of the next tile
    for (int c = tid; c < p.Ncols; c += NTHR) {
      prm[c] = p.scale ? p.scale[c] : 1.0f;
      prm[NTP_MAX_AFFINE_COLS + c] = p.shift ? p.shift[c] : 0.0f;
    }
    __syncthreads();
  }

  // ---- loader (runs ST-1 steps ahead of compute) ----
  // Raw-buffer LDS-DMA (buffer_load_dwordx4 ... lds): a lane whose im2col element lies outside
  // the image (or past K) gets voffset = NT_OOB, beyond the resource's num_records, and the
  // hardware writes zeros into its LDS slot -- no exec-masked branches, no 64-bit address
  // arithmetic.  UNI (cpt % 8 == 0): every lane of a k-tile sits in the same tap, so the tap
  // offset is scalar and each A slot costs one bit test, one add and one select.
  constexpr int NTAPS = MODE == MODE_DGRAD2 ? 4 : KS * KS;
  constexpr int SGN = MODE == MODE_FWD ? 1 : -1;
  constexpr int ES = (int)sizeof(T);
  const __amdgpu_buffer_rsrc_t rs_a =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, (int)p.src_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_b = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, NT_RSRC3);
  auto tap_dyx = [&](int t, int& dy, int& dx) {
    if (MODE == MODE_DGRAD2) {
      dy = ntx == 1 ? t : (t >> 1);
      dx = ntx == 1 ? 0 : (t & 1);
    } else {
      dy = t / KS;
      dx = t - (t / KS) * KS;
    }
  };
  const int q = (tid & 7) ^ ((tid >> 4) & 7), r0 = tid >> 3;   // swizzled source chunk, first row
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int tap_row = p.SW * p.src_ld * ES;                    // bytes per source image row
  int a_base[A_SLOTS];                                          // byte offset of tap 0 (+ lane chunk)
  uint32_t a_msk[A_SLOTS];
  uint32_t b_base[B_SLOTS];
  int tap = 0, cc = 0, ld_kt = 0, ld_tile = lb;
  auto setup_rows = [&](int t) {
    const int m0 = (t / p.tiles_n) * BM;
    const int n0 = (t % p.tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int m = m0 + r0 + RPP * i;
      const bool row_ok = m < M;
      const uint32_t mm = row_ok ? (uint32_t)m : 0u;
      const uint32_t n = fdiv(mm, dv_hw);
      const uint32_t rem = mm - n * dv_hw.d;
      const uint32_t oy = fdiv(rem, dv_w);
      const uint32_t ox = rem - oy * dv_w.d;
      int y0, x0;
      if (MODE == MODE_FWD) {
        y0 = (int)oy * p.stride - p.pad;
        x0 = (int)ox * p.stride - p.pad;
      } else if (MODE == MODE_DGRAD) {
        y0 = (int)oy + p.pad;
        x0 = (int)ox + p.pad;
      } else {
        y0 = (int)oy + p.cls_c0y[cls];
        x0 = (int)ox + p.cls_c0x[cls];
      }
      a_base[i] = ((((int)n * p.SH + y0) * p.SW + x0) * p.src_ld + p.src_off) * ES + (UNI ? q * 16 : 0);
      uint32_t msk = 0;
#pragma unroll
      for (int tt = 0; tt < NTAPS; ++tt) {
        int dy, dx;
        tap_dyx(tt, dy, dx);
        const int iy = y0 + SGN * dy, ix = x0 + SGN * dx;
        if (row_ok && iy >= 0 && iy < p.SH && ix >= 0 && ix < p.SW) msk |= 1u << tt;
      }
      a_msk[i] = msk;
    }
#pragma unroll
    for (int j = 0; j < B_SLOTS; ++j)
      b_base[j] = (uint32_t)(((n0 + j * RPP + r0) * (nkt * NT_KCH) + q) * 16);
    tap = 0;
    cc = 0;
  };
  setup_rows(ld_tile);
  auto issue = [&](int stage) {
    char* lds_a = smem + stage * STAGE + wv * 1024;
    char* lds_b = smem + stage * STAGE + BM * 128 + wv * 1024;
    if constexpr (UNI) {
      // scalar tap / channel position of this k-tile
      int dy, dx;
      tap_dyx(tap, dy, dx);
      const int delta = SGN * (dy * tap_row + dx * p.src_ld * ES) + cc * 16;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const uint32_t vo = ((a_msk[i] >> tap) & 1u) ? (uint32_t)(a_base[i] + delta) : NT_OOB;
        blds16(rs_a, lds_a + i * SLOT, vo);
      }
      cc += NT_KCH;
      if (cc >= p.cpt) { cc = 0; ++tap; }
    } else {
      // per-lane K position: kc = kt*8 + q, tap = kc / cpt (exact multiply-shift, host-checked)
      const int kc = ld_kt * NT_KCH + q;
      const int lt = (int)(((uint64_t)(uint32_t)kc * p.cpt_magic) >> 32);
      const int lc = kc - lt * p.cpt;
      int dy, dx;
      if (MODE == MODE_DGRAD2) {
        dy = ntx == 1 ? lt : (lt >> 1);
        dx = ntx == 1 ? 0 : (lt & 1);
      } else if (KS == 3) {
        dy = (lt * 11) >> 5;          // lt / 3 for lt < 9
        dx = lt - 3 * dy;
      } else {
        dy = 0;
        dx = 0;
      }
      const int delta = SGN * (dy * tap_row + dx * p.src_ld * ES) + lc * 16;
      const uint32_t tb = kc < Kc ? (1u << lt) : 0u;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const uint32_t vo = (a_msk[i] & tb) ? (uint32_t)(a_base[i] + delta) : NT_OOB;
        blds16(rs_a, lds_a + i * SLOT, vo);
      }
    }
    const int kb = ld_kt * (NT_KCH * 16);
    if (!B_PART || wv * 8 < BN) {
#pragma unroll
      for (int j = 0; j < B_SLOTS; ++j)
        blds16(rs_b, lds_b + j * SLOT, b_base[j] + kb);
    }
    if (++ld_kt == nkt) {           // next tile of this block
      ld_kt = 0;
      ld_tile += G;
      if (ld_tile < ntiles) setup_rows(ld_tile);
    }
  };

  // ---- compute ----
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;
  const int swz = (lr >> 1) & 7;
  auto compute = [&](int stage) {
    const char* A = smem + stage * STAGE;
    const char* B = A + BM * 128;
    u32x4 af[2][TM], bfr[2][TN];
    auto frags = [&](int s, int slot) {
      const int co = ((2 * s + lh) ^ swz) * 16;
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[slot][a] = *reinterpret_cast<const u32x4*>(A + (wm * WTM + a * 32 + lr) * 128 + co);
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

  // ---- epilogue of one tile (staging through ring stage `stage`) ----
  auto lds_barrier = [&]() {
    __builtin_amdgcn_s_waitcnt((0xF) | (3 << 14) | (0x7 << 4) | (0 << 8));   // lgkmcnt(0) only
    raw_barrier();
  };
  // combiner thread (sr, c) = tid < BN*SROWS owns running-moment slot tid (n, sum, M2)
  float* const run = red + WGM * 2 * BN;
  if constexpr (EPI == EPI_STATS) {
    if (tid < BN * SROWS) {
      run[tid] = 0.f;
      run[BN * SROWS + tid] = 0.f;
      run[2 * BN * SROWS + tid] = 0.f;
    }
  }
  auto epilogue = [&](int t, int stage) {
    const int tile_m = t / p.tiles_n, m0 = tile_m * BM, n0 = (t % p.tiles_n) * BN;
    T* stg = reinterpret_cast<T*>(smem + stage * STAGE);
    // per-column parameters / statistics from the fp32 accumulators
    if constexpr (EPI == EPI_STATS) {
      const int nw = min(WTM, max(0, M - (m0 + wm * WTM)));   // valid rows of this wave
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        float s1, s2;
        wave_col_moments<TM>(acc, b, nw, lh, s1, s2);
        if (lh == 0) {
          red[(wm * 2 + 0) * BN + wn * WTN + b * 32 + lr] = s1;
          red[(wm * 2 + 1) * BN + wn * WTN + b * 32 + lr] = s2;
        }
      }
    }
    if constexpr (EPI == EPI_AFFINE) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n0 + wn * WTN + b * 32 + lr;
        const bool cv = col < p.Ncols;
        const float sc = cv ? prm[col] : 1.0f;
        const float sh = cv ? prm[NTP_MAX_AFFINE_COLS + col] : 0.0f;
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
    constexpr int CH = BN / 8;      // 16-B chunks per staged row
    constexpr int RS = NTHR / CH;   // rows per pass
    const int ch = tid % CH, rr = tid / CH;
    const int col0 = n0 + ch * 8;
    const int nv = p.Ncols - col0;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      // h = 0: every wave has finished reading `stage` as MFMA operands; h > 0: every thread
      // has finished reading the previous pass out of the staging rows
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
      if constexpr (EPI == EPI_STATS) {
        if (h == 0 && tid < BN * SROWS) {
          const int sr = tid / BN, c = tid - sr * BN;
          constexpr int WPR = WGM / SROWS;    // wave rows per statistics row
          const int r0 = m0 + sr * 128;
          const int nt = min(128, max(0, M - r0));
          if (nt > 0) {
            float t1, t2;
            merge_moments<WPR, WTM>(red + (sr * WPR * 2 + 0) * BN + c, red + (sr * WPR * 2 + 1) * BN + c, 2 * BN,
                                    nt, t1, t2);
            const float rn = run[tid];
            if (rn == 0.f) {
              run[tid] = (float)nt;
              run[BN * SROWS + tid] = t1;
              run[2 * BN * SROWS + tid] = t2;
            } else {
              const float rs = run[BN * SROWS + tid];
              const float nn = rn + (float)nt;
              const float d = t1 / (float)nt - rs / rn;
              run[2 * BN * SROWS + tid] += t2 + d * d * (rn * (float)nt / nn);
              run[BN * SROWS + tid] = rs + t1;
              run[tid] = nn;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < HR / RS; ++j) {
        const int rl = rr + RS * j;
        int row = m0 + h * HR + rl;
        if (row >= M || nv <= 0) continue;
        float v[8];
        unpack8(*reinterpret_cast<const Raw8<T>*>(stg + rl * BN + ch * 8), v);
        if (MODE == MODE_DGRAD2) {
          const uint32_t n = fdiv((uint32_t)row, dv_hw);
          const uint32_t rem = (uint32_t)row - n * dv_hw.d;
          const uint32_t ya = fdiv(rem, dv_w);
          const uint32_t xb = rem - ya * dv_w.d;
          row = ((int)n * p.OH + 2 * (int)ya + (cls >> 1)) * p.OWx + 2 * (int)xb + (cls & 1);
        }
        T* dst = reinterpret_cast<T*>(p.dst) + (long)row * p.dst_ld + p.dst_off + col0;
        if (EPI == EPI_AFFINE && p.res) {
          float r[8];
          load8(reinterpret_cast<const T*>(p.res) + (long)row * p.res_ld + p.res_off + col0, nv, r);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += r[i];
        } else if (EPI == EPI_ACCUM) {
          float r[8];
          load8(dst, nv, r);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += r[i];
        }
        store8(dst, nv, v);
      }
    }
  };

  // ---- flattened (tile, k-tile) stream ----
  constexpr int NG = A_SLOTS + B_SLOTS;
#pragma unroll
  for (int s0 = 0; s0 < ST - 1; ++s0)
    if (s0 < total) issue(s0);
  int stage = 0, ckt = 0, ctile = lb;
  for (int g = 0; g < total; ++g) {
    const int ahead = total - 1 - g;
    // tile g landed; up to ST-2 later tiles stay in flight (counts are per wave: B_PART waves
    // past the B rows issue only the A loads)
    if (!B_PART || wv * 8 < BN) wait_tiles<NG, ST - 2>(ahead);
    else wait_tiles<A_SLOTS, ST - 2>(ahead);
    raw_barrier();
    if (g + ST - 1 < total) {
      int ns = stage + ST - 1;
      if (ns >= ST) ns -= ST;
      issue(ns);
    }
    compute(stage);
    if (++ckt == nkt) {
      epilogue(ctile, stage);
      ckt = 0;
      ctile += G;
    }
    if (++stage == ST) stage = 0;
  }
  if constexpr (EPI == EPI_STATS) {
    if (tid < BN * SROWS) {
      const int sr = tid / BN, c = tid - sr * BN;
      const int row = (lb / p.tiles_n) * SROWS + sr, n0 = (lb % p.tiles_n) * BN;
      float* so = p.stats + (long)row * 2 * p.stats_ld;
      so[n0 + c] = run[BN * SROWS + tid];
      so[p.stats_ld + n0 + c] = run[2 * BN * SROWS + tid];
      if (n0 == 0 && c == 0) p.stats_cnt[row] = run[tid];
    }
  }
}

// ------------------------------------------------------------------------------------------
// wgrad: TT GEMM over pixels with ds_read_b64_tr_b16 operands, split-K partial slabs.
// ------------------------------------------------------------------------------------------
struct TTParams {
  const char* x;
  const char* dz;
  float* slab;
  int x_ld, x_off, dz_ld, dz_off;
  int SH, SW, OW, stride, pad;
  int cpt;       // chunks per tap of x channels
  int Kc;        // valid kf chunks
  int M;         // pixels (rows of dz)
  int cout8;     // cout rounded up to 8 (valid dz channels incl. zero pad)
  int nkt;       // pixel tiles of KP
  uint32_t dz_bytes, x_bytes;   // raw-buffer extents of dz and x (< 2^31)
  int kt_per_split;
  int tiles_n;   // kf tiles
  int tiles_m_n; // row tiles x kf tiles
  int slab_rows, slab_ld;
  FastDiv div_ow, div_ohw;
};

// raw-buffer 16-B load into registers; an offset at or past num_records returns zeros
// (device-only wrapper, see blds16)
__device__ __forceinline__ u32x4 bld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
#else
  (void)r; (void)voff;
  return u32x4{0u, 0u, 0u, 0u};
#endif
}

// KP pixels per k-tile, NW waves per block, OCC blocks per CU.  Operands are register-staged
// through raw-buffer loads (out-of-image / out-of-range lanes read zeros: no branches, 32-bit
// offsets) into padded LDS images consumed by the transposing ds_read_b64_tr_b16.
template <typename T, int KS, int BM, int BN, int KP, int NW, int OCC>
__global__ __launch_bounds__(NW * 64, OCC) void conv_wgrad_kernel(TTParams p) {
  constexpr int NTHR = NW * 64;
  // 32- and 96-row tiles (cout <= 32, <= 96) lay all waves along the kf columns
  constexpr int WGN = (BM == 32 || BM == 96) ? NW : (NW == 8 && BN >= 128) ? 4 : 2, WGM = NW / WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0 && KP % 16 == 0, "wgrad tile");
  constexpr int SZ = sizeof(T);
  constexpr bool F32 = SZ == 4;
  constexpr int EPC = 16 / SZ;                 // elements per chunk
  // LDS pitches (conflict-free tr reads: a pitch that is a multiple of the 256-B bank span
  // would put the 4 rows one tr-read group touches on the same banks)
  constexpr int PA = BM * SZ + ((BM * SZ + 64) % 256 == 0 ? 128 : 64), PB = BN * SZ + 64;
  constexpr int CA = BM / EPC, CB = BN / EPC;  // chunks per LDS row
  constexpr int A_SLOTS = (KP * CA + NTHR - 1) / NTHR, B_SLOTS = (KP * CB + NTHR - 1) / NTHR;
  constexpr int TILE = KP * (PA + PB);
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  // 1-D grid, split-major logical order: the tiles sharing a pixel split (its dz rows and x
  // im2col columns) are consecutive logical ids, which xcd_remap keeps on one XCD's L2
  const int tmn = p.tiles_m_n;
  // (measured: grouping pays from 4 tiles per split up; below that plain dispatch order is faster)
  const int lid = tmn >= 4 ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int wg = lid % tmn;
  const int tile_n = wg % p.tiles_n, tile_m = wg / p.tiles_n;
  const int split = lid / tmn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(p.nkt, kt0 + p.kt_per_split);

  const __amdgpu_buffer_rsrc_t rs_a =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dz, (short)0, (int)p.dz_bytes, NT_RSRC3);
  const __amdgpu_buffer_rsrc_t rs_b =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, NT_RSRC3);
  const uint32_t dz_row = (uint32_t)(p.dz_ld * SZ);
  // A-side (dz) slots: fixed pixel row within the k-tile and fixed channel chunk
  int a_row[A_SLOTS];
  uint32_t a_col[A_SLOTS];
#pragma unroll
  for (int i = 0; i < A_SLOTS; ++i) {
    const int c = tid + NTHR * i;
    a_row[i] = c / CA;
    const int ch = m0 + (c - a_row[i] * CA) * EPC;
    a_col[i] = (c < KP * CA && ch < p.cout8) ? (uint32_t)((p.dz_off + ch) * SZ) : NT_OOB;
  }
  // B-side (x im2col) chunk columns are fixed per slot: precompute tap decomposition.
  int b_row[B_SLOTS], b_kh[B_SLOTS], b_kw[B_SLOTS], b_cc[B_SLOTS], b_col[B_SLOTS];
  bool b_kok[B_SLOTS];
#pragma unroll
  for (int j = 0; j < B_SLOTS; ++j) {
    const int c = tid + NTHR * j;
    b_row[j] = c / CB;
    b_col[j] = c - b_row[j] * CB;
    const int kc = n0 / EPC + b_col[j];
    b_kok[j] = (c < KP * CB) && kc < p.Kc;
    const int t = kc / p.cpt;
    b_cc[j] = kc - t * p.cpt;
    b_kh[j] = t / KS;
    b_kw[j] = t - b_kh[j] * KS;
  }
  u32x4 a_reg[A_SLOTS], b_reg[B_SLOTS];

  auto load_tile = [&](int kt) {
    const int q0 = kt * KP;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int qpix = q0 + a_row[i];
      const bool ok = a_col[i] != NT_OOB && qpix < p.M;
      a_reg[i] = bld16(rs_a, ok ? (uint32_t)qpix * dz_row + a_col[i] : NT_OOB);
    }
#pragma unroll
    for (int j = 0; j < B_SLOTS; ++j) {
      const int qpix = q0 + b_row[j];
      bool ok = b_kok[j] && qpix < p.M;
      const uint32_t mm = ok ? (uint32_t)qpix : 0u;
      const uint32_t n = fdiv(mm, p.div_ohw);
      const uint32_t rem = mm - n * p.div_ohw.d;
      const uint32_t oy = fdiv(rem, p.div_ow);
      const uint32_t ox = rem - oy * p.div_ow.d;
      const int iy = (int)oy * p.stride - p.pad + b_kh[j];
      const int ix = (int)ox * p.stride - p.pad + b_kw[j];
      ok = ok && iy >= 0 && iy < p.SH && ix >= 0 && ix < p.SW;
      const uint32_t e = (uint32_t)((((int)n * p.SH + iy) * p.SW + ix) * p.x_ld + p.x_off);
      b_reg[j] = bld16(rs_b, ok ? e * SZ + (uint32_t)(b_cc[j] * 16) : NT_OOB);
    }
  };
  auto store_tile = [&](int buf) {
    char* A = smem + buf * TILE;
    char* B = A + KP * PA;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int c = tid + NTHR * i;
      if (c < KP * CA) *reinterpret_cast<u32x4*>(A + (c / CA) * PA + (c % CA) * 16) = a_reg[i];
    }
#pragma unroll
    for (int j = 0; j < B_SLOTS; ++j) {
      const int c = tid + NTHR * j;
      if (c < KP * CB) *reinterpret_cast<u32x4*>(B + b_row[j] * PB + b_col[j] * 16) = b_reg[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.0f;

  const int lr = lane & 31, lh = lane >> 5;
  // tr-read lane geometry (16-lane groups): group g, block row qq, column quad pp
  const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
  const int th = g >> 1, tcb = 16 * (g & 1);

  auto compute = [&](int buf) {
    const char* A = smem + buf * TILE;
    const char* B = A + KP * PA;
    if constexpr (!F32) {
#pragma unroll
      for (int s = 0; s < KP / 16; ++s) {
        u32x4 af[TM], bfr[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int col = wm * WTM + a * 32 + tcb + 4 * pp;
          const int row = 16 * s + 8 * th + qq;
          const YMS_LDS s16x4* p0 = (const YMS_LDS s16x4*)(A + row * PA + col * 2);
          const YMS_LDS s16x4* p1 = (const YMS_LDS s16x4*)(A + (row + 4) * PA + col * 2);
          s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)p0);
          s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)p1);
          uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
          af[a] = u32x4{u0.x, u0.y, u1.x, u1.y};
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int col = wn * WTN + b * 32 + tcb + 4 * pp;
          const int row = 16 * s + 8 * th + qq;
          const YMS_LDS s16x4* p0 = (const YMS_LDS s16x4*)(B + row * PB + col * 2);
          const YMS_LDS s16x4* p1 = (const YMS_LDS s16x4*)(B + (row + 4) * PB + col * 2);
          s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)p0);
          s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YMS_LDS s16x4*)p1);
          uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
          bfr[b] = u32x4{u0.x, u0.y, u1.x, u1.y};
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b] = Mfma<T>::mma(af[a], bfr[b], acc[a][b]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KP / 2; ++j) {
        float av[TM], bv[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
          av[a] = *reinterpret_cast<const float*>(A + (2 * j + lh) * PA + (wm * WTM + a * 32 + lr) * 4);
#pragma unroll
        for (int b = 0; b < TN; ++b)
          bv[b] = *reinterpret_cast<const float*>(B + (2 * j + lh) * PB + (wn * WTN + b * 32 + lr) * 4);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
      }
    }
  };

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      compute(cur);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
    }
  }
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

// dw[co][ci][kh][kw] (+)= sum_s slab[s][co][tap*cin8 + ci].  Block = 32 float4 lanes (128
// consecutive slab columns of one row) x 8 split lanes; every lane keeps two independent
// float4 accumulators, the 8 split lanes are combined through LDS in a fixed order
// (deterministic).  Reads are 16 B/lane, fully coalesced along the slab row.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* slab, int splits, long slab_elems,
                                                           int slab_ld, int cout, int cin, int cin8, int ks,
                                                           float* dw, int accumulate) {
  __shared__ float4 red[8][33];
  const int lx = threadIdx.x & 31, ly = threadIdx.x >> 5;
  const int kf = ks * ks * cin8;                // valid slab columns
  const int cpr = (kf + 127) / 128;             // column blocks per row
  const int co = blockIdx.x / cpr;
  const int col = (blockIdx.x - co * cpr) * 128 + lx * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  if (col < kf) {
    const float* base = slab + (long)co * slab_ld + col;
    int z = ly;
    for (; z + 8 < splits; z += 16) {
      const float4 u = *reinterpret_cast<const float4*>(base + (long)z * slab_elems);
      const float4 v = *reinterpret_cast<const float4*>(base + (long)(z + 8) * slab_elems);
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
      b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
    }
    if (z < splits) {
      const float4 u = *reinterpret_cast<const float4*>(base + (long)z * slab_elems);
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
  }
  red[ly][lx] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  __syncthreads();
  if (ly == 0 && col < kf) {
    float4 t = red[0][lx];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float4 u = red[k][lx];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = col + e;
      const int tap = c / cin8, ci = c - tap * cin8;
      if (ci < cin) {
        const long o = (((long)co * cin + ci) * ks + tap / ks) * ks + tap % ks;
        dw[o] = accumulate ? dw[o] + tv[e] : tv[e];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// weight packing
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* w, T* out, int cout, int cin, int ks, int rows,
                                   int kp_elems, int c8_in, int for_dgrad) {
  // fwd  : out[co][tap*cin8 + ci]   = w[co][ci][tap]        rows = cout_pad
  // dgrad: out[ci][tap*cout8 + co]  = w[co][ci][tap]        rows = cin_pad
  const long total = (long)rows * kp_elems;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int r = (int)(t / kp_elems);
    const int k = (int)(t % kp_elems);
    const int tap = k / c8_in, c = k % c8_in;
    float v = 0.f;
    if (tap < ks * ks) {
      const int co = for_dgrad ? c : r;
      const int ci = for_dgrad ? r : c;
      if (co < cout && ci < cin) v = w[((long)co * cin + ci) * ks * ks + tap];
    }
    out[t] = (T)v;
  }
}

// All of a plan's weight packs in one launch (training repacks every step): block (x, job)
// handles rows x, x + gridDim.x, ... of job `job`; 32-bit index math only.
__global__ __launch_bounds__(256) void pack_weight_batched_kernel(const yms_pack_job* jobs, char* dst_base) {
  yms_pack_job j = jobs[blockIdx.y];
  j.packed = dst_base + (uintptr_t)j.packed;     // offsets relative to the (per-call) arena base
  const int kk = j.ks * j.ks;
  for (int r = blockIdx.x; r < j.rows; r += gridDim.x) {
    for (int k = threadIdx.x; k < j.kp_elems; k += 256) {
      const int tap = k / j.c8_in, c = k - tap * j.c8_in;
      float v = 0.f;
      if (tap < kk) {
        const int co = j.for_dgrad ? c : r;
        const int ci = j.for_dgrad ? r : c;
        if (co < j.cout && ci < j.cin) {
          const bool hi = j.w2 && co >= j.split;
          v = (hi ? j.w2 : j.w)[((long)(hi ? co - j.split : co) * j.cin + ci) * kk + tap];
        }
      }
      const long o = (long)r * j.kp_elems + k;
      if (j.dtype == YMS_BF16) reinterpret_cast<bf16*>(j.packed)[o] = (bf16)v;
      else if (j.dtype == YMS_F16) reinterpret_cast<f16*>(j.packed)[o] = (f16)v;
      else reinterpret_cast<float*>(j.packed)[o] = v;
    }
  }
}

// stride-2 dgrad: 4 parity-class blocks, block c = [cin_pad128][kp_c]; K = (jy, jx, co8)
struct Dg2Pack {
  long off[4];       // element offset of each class block
  int kp[4];         // elements per row of each class block
  int ntx[4], kh0[4], kw0[4];
};
template <typename T>
__global__ void pack_weight_dgrad2_kernel(const float* w, T* out, int cout, int cin, int ks, int rows, int c8,
                                          Dg2Pack g, long total) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    int c = 0;
    while (c < 3 && t >= g.off[c + 1]) ++c;
    const long e = t - g.off[c];
    const int r = (int)(e / g.kp[c]);       // ci
    const int k = (int)(e % g.kp[c]);
    const int tl = k / c8, co = k % c8;
    const int jy = tl / g.ntx[c], jx = tl % g.ntx[c];
    const int kh = g.kh0[c] + 2 * jy, kw = g.kw0[c] + 2 * jx;
    float v = 0.f;
    if (kh < ks && kw < ks && co < cout && r < cin) v = w[((long)co * cin + r) * ks * ks + kh * ks + kw];
    out[t] = (T)v;
  }
  (void)rows;
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int elem_size(int dt) { return dt == YMS_F32 ? 4 : 2; }

struct PackGeo {
  int rows, c8_in, cpt, kc, nkt, kp_elems;
};
static PackGeo pack_geo(const yms_conv_shape* s, int for_dgrad) {
  PackGeo g;
  const int es = elem_size(s->dtype);
  const int cin_k = for_dgrad ? s->cout : s->cin;    // channels along K
  const int cout_r = for_dgrad ? s->cin : s->cout;   // rows
  g.c8_in = (int)rup(cin_k, 8);
  g.cpt = g.c8_in * es / 16;
  g.kc = s->k * s->k * g.cpt;
  g.nkt = cdiv(g.kc, NT_KCH);
  g.kp_elems = g.nkt * NT_KCH * 16 / es;
  g.rows = (int)rup(cout_r, 128);
  return g;
}

struct Dg2Geo {
  int M[4], nkt[4], Kc[4], ntx[4], nty[4], c0y[4], c0x[4], kh0[4], kw0[4], Ha[4], Wa[4], kp[4];
  long off_elems[5];
  int rows, cpt;
};
static Dg2Geo dg2_geo(const yms_conv_shape* s) {
  Dg2Geo g;
  const int es = elem_size(s->dtype);
  const int c8 = (int)rup(s->cout, 8);
  g.cpt = c8 * es / 16;
  g.rows = (int)rup(s->cin, 128);
  g.off_elems[0] = 0;
  for (int c = 0; c < 4; ++c) {
    const int ry = c >> 1, rx = c & 1;
    const int kh0 = (ry + s->pad) & 1, kw0 = (rx + s->pad) & 1;
    g.kh0[c] = kh0;
    g.kw0[c] = kw0;
    g.nty[c] = (s->k - kh0 + 1) / 2;
    g.ntx[c] = (s->k - kw0 + 1) / 2;
    g.c0y[c] = (ry + s->pad - kh0) / 2;
    g.c0x[c] = (rx + s->pad - kw0) / 2;
    g.Ha[c] = (s->h - ry + 1) / 2;
    g.Wa[c] = (s->w - rx + 1) / 2;
    g.M[c] = s->n * g.Ha[c] * g.Wa[c];
    g.Kc[c] = g.nty[c] * g.ntx[c] * g.cpt;
    g.nkt[c] = std::max(1, cdiv(g.Kc[c], NT_KCH));
    g.kp[c] = g.nkt[c] * NT_KCH * 16 / es;
    g.off_elems[c + 1] = g.off_elems[c] + (long)g.rows * g.kp[c];
  }
  return g;
}

static bool shape_ok(const yms_conv_shape* s) {
  if (!s || s->n <= 0 || s->h <= 0 || s->w <= 0 || s->cin <= 0 || s->cout <= 0) return false;
  if (!(s->k == 1 || s->k == 3) || !(s->stride == 1 || s->stride == 2)) return false;
  if (s->dtype < 0 || s->dtype > 2) return false;
  if (s->ho != (s->h + 2 * s->pad - s->k) / s->stride + 1) return false;
  if (s->wo != (s->w + 2 * s->pad - s->k) / s->stride + 1) return false;
  if ((long)s->n * s->h * s->w >= (1l << 31) || (long)s->n * s->ho * s->wo >= (1l << 31)) return false;
  return true;
}
static bool view_ok(int ld, int off, int c) { return ld % 8 == 0 && off % 8 == 0 && off + c <= ld; }

struct TileChoice { int cfg, bn; };
static TileChoice choose_tile(int ncols) {
  // One column tile whenever N <= 128: every extra column tile re-reads the whole im2col
  // A operand, which costs more than the padded MFMA columns at these sizes.
  if (ncols <= 32) return TileChoice{2, 32};
  if (ncols <= 64) return TileChoice{1, 64};
  if (ncols <= 128) return TileChoice{0, 128};
  // wider: 128-column tiles unless that pads by more than 25%
  const long p128 = rup(ncols, 128), p64 = rup(ncols, 64);
  if (p128 * 4 > ncols * 5 && p64 < p128) return TileChoice{1, 64};
  return TileChoice{0, 128};
}

static int cu_count() { return conv_cu_count(); }

// forward: statistics (training) grids persistent at 1x (the side-stream wgrads hold CUs: 4x
// measured 19.43 -> 19.9 ms/step); eval grids 4x (finer work units balance around the
// overlapped NMS of the serving pipeline: 2.65 -> 2.58 ms/batch).  (Round 4, measured and dropped:
// 256-row tiles of 16 waves at 1 block per CU.)
static int nt_fwd_mult(bool stats) { return stats ? 1 : 4; }
// dgrad grids: one block per output tile (no persistent cap)
constexpr int NT_DGRAD_MULT = 1 << 16;

struct NtpGeo { int bm, bn, occ; };
static NtpGeo ntp_geo(int cfg) {
  if (cfg == 0) return NtpGeo{128, 128, 2};
  if (cfg == 1) return NtpGeo{128, 64, 3};
  return NtpGeo{256, 32, 2};
}

// persistent grid: OCC resident blocks per CU (x mult), at most one block per tile.  Statistics
// launches round it down to a multiple of tiles_n, so every block walks tiles of one column tile
// (conv_ntp_kernel's per-block statistics slots).
static long ntp_grid(long M, int tiles_n, int bm, long occ_blocks_per_cu, bool stats) {
  const long ntiles = (long)cdiv(M, bm) * tiles_n;
  long g = std::max<long>(1, std::min<long>(ntiles, occ_blocks_per_cu * cu_count()));
  if (stats) g = std::max<long>(tiles_n, g - g % tiles_n);
  return g;
}

// p.M is the largest parity class for DGRAD2
template <typename K>
static void launch_persistent(K kernel, const NTParams& p, int bm, unsigned gy, hipStream_t st, long occ, int nthr,
                              bool stats) {
  const unsigned gx = (unsigned)ntp_grid(p.M, p.tiles_n, bm, occ, stats);
  hipLaunchKernelGGL(kernel, dim3(gx, gy), dim3(nthr), 0, st, p);
}

template <typename T, int KS, int MODE, int EPI, bool UNI>
static void launch_ntp(const NTParams& p0, int cfg, unsigned gy, hipStream_t st) {
  NTParams p = p0;
  // dgrad grids: one block per output tile by default.  The weight gradients run beside dgrad on
  // the side stream, and persistent blocks that start late on CUs the wgrad kernels hold would
  // each still owe their fixed share of tiles (interleaved A/B: 19.91 -> 19.74 ms/step).
  const bool stats = EPI == EPI_STATS;
  const long mult = MODE == MODE_FWD ? nt_fwd_mult(stats) : NT_DGRAD_MULT;
  const NtpGeo g = ntp_geo(cfg);
  p.tiles_n = cdiv(p.Ncols, g.bn);
  // 8-wave blocks at 2-3 per CU (4-6 waves per SIMD) hide the ds_read -> MFMA and barrier
  // latencies that 4-wave blocks expose
  // (round 4, measured and dropped: 256 x 128 tiles of 8 waves with 64 x 64 wave tiles, 5-40 %
  // slower, and 128 x 128 tiles of 4 such waves, within +-5 %: profiles/r04b_conv_micro_v*.txt)
  if (cfg == 0) {
    launch_persistent(conv_ntp_kernel<T, KS, MODE, EPI, 128, 128, 2, 4, 2, UNI, 2>, p, 128, gy, st, g.occ * mult, 512, stats);
  } else if (cfg == 1) {
    launch_persistent(conv_ntp_kernel<T, KS, MODE, EPI, 128, 64, 4, 2, 2, UNI, 3>, p, 128, gy, st, g.occ * mult, 512, stats);
  } else {
    launch_persistent(conv_ntp_kernel<T, KS, MODE, EPI, 256, 32, 8, 1, 2, UNI, 2>, p, 256, gy, st, g.occ * mult, 512, stats);
  }
}

template <typename T, int KS, int MODE, int EPI>
static void launch_nt(const NTParams& p0, int cfg, hipStream_t st) {
  NTParams p = p0;
  const unsigned gy = MODE == MODE_DGRAD2 ? 4u : 1u;
  if constexpr (sizeof(T) == 2) {
    if (EPI != EPI_AFFINE || p.Ncols <= NTP_MAX_AFFINE_COLS) {
      if (p.cpt % NT_KCH == 0) launch_ntp<T, KS, MODE, EPI, true>(p, cfg, gy, st);
      else launch_ntp<T, KS, MODE, EPI, false>(p, cfg, gy, st);
      return;
    }
  }
  if (cfg == 0) {
    p.tiles_n = cdiv(p.Ncols, 128);
    dim3 grid((unsigned)(cdiv(p.M, 128) * p.tiles_n), gy);
    hipLaunchKernelGGL((conv_nt_kernel<T, KS, MODE, EPI, 128, 128, 2, 2, 2>), grid, dim3(256), 0, st, p);
  } else if (cfg == 1) {
    p.tiles_n = cdiv(p.Ncols, 64);
    dim3 grid((unsigned)(cdiv(p.M, 128) * p.tiles_n), gy);
    hipLaunchKernelGGL((conv_nt_kernel<T, KS, MODE, EPI, 128, 64, 2, 2, 3>), grid, dim3(256), 0, st, p);
  } else {
    p.tiles_n = cdiv(p.Ncols, 32);
    dim3 grid((unsigned)(cdiv(p.M, 128) * p.tiles_n), gy);
    hipLaunchKernelGGL((conv_nt_kernel<T, KS, MODE, EPI, 128, 32, 4, 1, 3>), grid, dim3(256), 0, st, p);
  }
}

// raw-buffer source extent and the exact kc / cpt multiply-shift for the 16-bit loader
static bool set_src_geometry(NTParams& p, long n, long h, long w, long ld, int es, int max_kc) {
  const long bytes = n * h * w * ld * es;
  if (es == 2 && bytes >= (1l << 31) - (1l << 20)) return false;
  p.src_bytes = (uint32_t)std::min<long>(bytes, 0x7fffffffl);
  p.cpt_magic = ((1ull << 32) + (uint64_t)p.cpt - 1) / (uint64_t)p.cpt;
  for (int kc = 0; kc < max_kc; ++kc)
    if ((int)(((uint64_t)(uint32_t)kc * p.cpt_magic) >> 32) != kc / p.cpt) return false;
  return true;
}

// the NT loader addresses its source with 32-bit element offsets
static bool offsets32(long n, long h, long w, long ld) { return n * h * w * ld < (1l << 31) - (1l << 20); }

template <int MODE, int EPI>
static yms_status dispatch_nt(const NTParams& p, int dtype, int ks, int cfg, hipStream_t st) {
#define YMS_NT_CASE(T)                                          \
  if constexpr (MODE == MODE_DGRAD2) launch_nt<T, 3, MODE, EPI>(p, cfg, st);   \
  else if (ks == 1) launch_nt<T, 1, MODE, EPI>(p, cfg, st);     \
  else launch_nt<T, 3, MODE, EPI>(p, cfg, st);
  if (dtype == YMS_BF16) { YMS_NT_CASE(bf16) }
  else if (dtype == YMS_F16) { YMS_NT_CASE(f16) }
  else { YMS_NT_CASE(float) }
#undef YMS_NT_CASE
  return launch_status();
}


struct WgradPlan {
  int bm, bn, tiles_m, tiles_n, nkt, kt_per_split, splits, slab_rows, slab_ld, cin8, cpt, kc, kp;
};
static WgradPlan wgrad_plan(const yms_conv_shape* s) {
  WgradPlan w;
  const int es = elem_size(s->dtype);
  w.cin8 = (int)rup(s->cin, 8);
  w.cpt = w.cin8 * es / 16;
  w.kc = s->k * s->k * w.cpt;
  const int kf = s->k * s->k * w.cin8;
  w.bm = s->cout <= 32 ? 32 : s->cout <= 64 ? 64 : s->cout <= 96 ? 96 : 128;
  w.bn = kf <= 64 ? 64 : 128;
  w.tiles_m = cdiv(s->cout, w.bm);
  w.tiles_n = cdiv(kf, w.bn);
  w.slab_rows = w.tiles_m * w.bm;
  w.slab_ld = w.tiles_n * w.bn;
  w.kp = 32;
  const long M = (long)s->n * s->ho * s->wo;
  w.nkt = cdiv(M, w.kp);
  const int blocks = w.tiles_m * w.tiles_n;
  // about 4 workgroups per CU (2-4 resident by LDS), at least 512 pixels per split
  int splits = std::max(1, std::min(cdiv(w.nkt, 512 / w.kp), cdiv(4 * cu_count(), blocks)));
  // deep layers: every split writes (and the reduce re-reads) a full fp32 slab of the weight
  // gradient, which can exceed the layer's own x + dz bytes several times over.  Cap the slab
  // round trip at `ratio` x the algorithmic bytes, keeping at least `min_blocks` workgroups.
  // (interleaved A/B, YOLOv8-s step: off 19.71/19.71/19.81 ms, ratio 1 19.62/19.64/19.76 ms;
  // YOLO-MS-S 40.11/40.12 -> 40.04/40.02 ms -- the wgrads run on the side stream, so the
  // step gains only the HBM contention the slabs caused).  Round 4: the step keeps improving down
  // to ~0.05, where min_blocks binds (YOLOv8-s 18.23 -> 17.93 ms, YOLO-MS-S 36.22 -> 35.66 ms;
  // profiles/r04ad_wgrad_slab_ratio_ab.txt): fewer, longer side-stream blocks and ~no slab bytes.
  // (read per call, as the ring / halo kernels do: tests switch them at run time)
  const double ratio = getenv("YMS_WG_SLAB_RATIO") ? atof(getenv("YMS_WG_SLAB_RATIO")) : 0.05;
  const int min_blocks = 256;
  if (ratio > 0.0) {
    const double data = (double)M * (double)(rup(s->cout, 8) + w.cin8) * es;
    const double slab_rt = 2.0 * 4.0 * (double)w.slab_rows * (double)w.slab_ld;
    const int cap = std::max((int)(ratio * data / slab_rt), cdiv(min_blocks, blocks));
    splits = std::max(1, std::min(splits, cap));
  }
  w.kt_per_split = cdiv(w.nkt, splits);
  w.splits = cdiv(w.nkt, w.kt_per_split);
  return w;
}

template <typename T, int KS, int KP, int NW, int OCC>
static void launch_wgrad_v(const TTParams& p, int bm, int bn, dim3 grid, hipStream_t st) {
  // 32-row tiles: 2 / 4 waves of 32 x 32 along kf; 64-row tiles keep 4 waves (2 x 2)
  if (bm == 32 && bn == 64)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 32, 64, KP, 2, OCC>), grid, dim3(128), 0, st, p);
  else if (bm == 32)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 32, 128, KP, 4, OCC>), grid, dim3(256), 0, st, p);
  else if (bm == 96 && bn == 64)   // (its registers allow 3 blocks per SIMD's worth, not 4)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 96, 64, KP, 2, (OCC > 3 ? 3 : OCC)>), grid, dim3(128), 0, st, p);
  else if (bm == 96)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 96, 128, KP, 4, OCC>), grid, dim3(256), 0, st, p);
  else if (bm == 64 && bn == 64)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 64, 64, KP, 4, OCC>), grid, dim3(256), 0, st, p);
  else if (bm == 64)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 64, 128, KP, 4, OCC>), grid, dim3(256), 0, st, p);
  else if (bn == 64)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 128, 64, KP, NW, OCC>), grid, dim3(NW * 64), 0, st, p);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, 128, 128, KP, NW, OCC>), grid, dim3(NW * 64), 0, st, p);
}

// (round 3, measured and dropped: 64-pixel k-tiles, 8-wave blocks, 3-4 blocks per CU)
template <typename T, int KS>
static void launch_wgrad(const TTParams& p, int bm, int bn, dim3 grid, hipStream_t st) {
  launch_wgrad_v<T, KS, 32, 4, 2>(p, bm, bn, grid, st);
}

}  // namespace yms

int yms::conv_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

using namespace yms;

extern "C" {

size_t yms_conv_packed_elems(const yms_conv_shape* s, int for_dgrad) {
  if (!shape_ok(s)) return 0;
  if (for_dgrad && s->stride == 2) return (size_t)dg2_geo(s).off_elems[4];
  PackGeo g = pack_geo(s, for_dgrad);
  return (size_t)g.rows * g.kp_elems;
}

yms_status yms_pack_job_init(const yms_conv_shape* s, const float* w, void* packed, int for_dgrad,
                             yms_pack_job* job) {
  if (!shape_ok(s) || !w || !job) return YMS_ERR_INVALID;   // packed may be an offset (0 allowed)
  if (for_dgrad && s->stride == 2) return YMS_ERR_UNSUPPORTED;   // parity-class packing: yms_conv_pack_weight
  PackGeo g = pack_geo(s, for_dgrad);
  job->w = w;
  job->packed = packed;
  job->cout = s->cout;
  job->cin = s->cin;
  job->ks = s->k;
  job->rows = g.rows;
  job->kp_elems = g.kp_elems;
  job->c8_in = g.c8_in;
  job->for_dgrad = for_dgrad;
  job->dtype = s->dtype;
  job->w2 = nullptr;
  job->split = 0;
  return YMS_OK;
}

yms_status yms_conv_pack_weights_batched(int njobs, const yms_pack_job* jobs_dev, void* dst_base, void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs_dev)) return YMS_ERR_INVALID;
  if (njobs == 0) return YMS_OK;
  if (njobs > 65535) return YMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(pack_weight_batched_kernel, dim3(64, (unsigned)njobs), dim3(256), 0, (hipStream_t)stream,
                     jobs_dev, (char*)dst_base);
  return launch_status();
}

yms_status yms_conv_pack_weight(const yms_conv_shape* s, const float* w, void* packed,
                                int for_dgrad, void* stream) {
  if (!shape_ok(s) || !w || !packed) return YMS_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  if (for_dgrad && s->stride == 2) {
    Dg2Geo d = dg2_geo(s);
    Dg2Pack pk;
    for (int c = 0; c < 4; ++c) {
      pk.off[c] = d.off_elems[c];
      pk.kp[c] = d.kp[c];
      pk.ntx[c] = d.ntx[c];
      pk.kh0[c] = d.kh0[c];
      pk.kw0[c] = d.kw0[c];
    }
    const long total = d.off_elems[4];
    const int c8 = (int)rup(s->cout, 8);
    dim3 grid((unsigned)std::min<long>(cdiv(total, 256), 4096));
    if (s->dtype == YMS_BF16)
      hipLaunchKernelGGL(pack_weight_dgrad2_kernel<bf16>, grid, dim3(256), 0, st, w, (bf16*)packed, s->cout, s->cin, s->k, d.rows, c8, pk, total);
    else if (s->dtype == YMS_F16)
      hipLaunchKernelGGL(pack_weight_dgrad2_kernel<f16>, grid, dim3(256), 0, st, w, (f16*)packed, s->cout, s->cin, s->k, d.rows, c8, pk, total);
    else
      hipLaunchKernelGGL(pack_weight_dgrad2_kernel<float>, grid, dim3(256), 0, st, w, (float*)packed, s->cout, s->cin, s->k, d.rows, c8, pk, total);
    return launch_status();
  }
  PackGeo g = pack_geo(s, for_dgrad);
  const long total = (long)g.rows * g.kp_elems;
  dim3 grid((unsigned)std::min<long>(cdiv(total, 256), 4096));
  if (s->dtype == YMS_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16>, grid, dim3(256), 0, st, w, (bf16*)packed, s->cout, s->cin, s->k, g.rows, g.kp_elems, g.c8_in, for_dgrad);
  else if (s->dtype == YMS_F16)
    hipLaunchKernelGGL(pack_weight_kernel<f16>, grid, dim3(256), 0, st, w, (f16*)packed, s->cout, s->cin, s->k, g.rows, g.kp_elems, g.c8_in, for_dgrad);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, grid, dim3(256), 0, st, w, (float*)packed, s->cout, s->cin, s->k, g.rows, g.kp_elems, g.c8_in, for_dgrad);
  return launch_status();
}

int yms_conv_stats_rows(const yms_conv_shape* s) {
  if (!shape_ok(s)) return 0;
  DirectGeo dg;
  if (conv_direct_geometry(s, 0, &dg)) return dg.grid;   // conv_direct_kernel: one row per block
  const long M = (long)s->n * s->ho * s->wo;
  if (s->dtype == YMS_F32) return (int)cdiv(M, 128);     // conv_nt_kernel: one row per 128-row tile
  const NtpGeo g = ntp_geo(choose_tile(s->cout).cfg);    // conv_ntp_kernel: one slot per block
  const int tiles_n = cdiv(s->cout, g.bn);
  return (int)(ntp_grid(M, tiles_n, g.bm, (long)g.occ * nt_fwd_mult(true), true) / tiles_n) * (g.bm / 128);
}
int yms_conv_stats_ld(const yms_conv_shape* s) {
  if (!shape_ok(s)) return 0;
  return (int)rup(s->cout, 128);
}

yms_status yms_conv_fwd(const yms_conv_shape* s, const void* x, int x_ld, int x_off,
                        const void* wpacked, void* y, int y_ld, int y_off,
                        const float* scale, const float* shift, int act,
                        const void* res, int res_ld, int res_off, float* stats, void* stream) {
  if (!shape_ok(s) || !x || !wpacked || !y) return YMS_ERR_INVALID;
  if (!view_ok(x_ld, x_off, s->cin) || !view_ok(y_ld, y_off, s->cout)) return YMS_ERR_INVALID;
  if (res && !view_ok(res_ld, res_off, s->cout)) return YMS_ERR_INVALID;
  const int es = elem_size(s->dtype);
  {
    // small-channel 3x3: the direct kernel (conv_direct.hip), statistics included
    DirectGeo dg;
    if (conv_direct_geometry(s, 0, &dg))
      return conv_direct_launch(s, 0, dg, x, x_ld, x_off, wpacked, y, y_ld, y_off, scale, shift, act, res, res_ld,
                                res_off, stats, 0, (hipStream_t)stream);
  }
  PackGeo g = pack_geo(s, 0);
  NTParams p{};
  p.src = (const char*)x;
  p.wp = (const char*)wpacked;
  p.dst = (char*)y;
  p.src_ld = x_ld; p.src_off = x_off; p.dst_ld = y_ld; p.dst_off = y_off;
  p.scale = scale; p.shift = shift; p.act = act;
  p.res = (const char*)res; p.res_ld = res_ld; p.res_off = res_off;
  p.stats = stats;
  p.stats_ld = (int)rup(s->cout, 128);
  if (stats) p.stats_cnt = stats + (long)yms_conv_stats_rows(s) * 2 * p.stats_ld;
  p.SH = s->h; p.SW = s->w; p.OW = s->wo;
  if (!offsets32(s->n, s->h, s->w, x_ld)) return YMS_ERR_UNSUPPORTED;
  p.stride = s->stride; p.pad = s->pad;
  p.cpt = g.cpt; p.Kc = g.kc; p.nkt = g.nkt;
  if (!set_src_geometry(p, s->n, s->h, s->w, x_ld, es, g.nkt * NT_KCH)) return YMS_ERR_UNSUPPORTED;
  p.M = s->n * s->ho * s->wo;
  p.Ncols = s->cout;
  p.div_ow = make_fastdiv(s->wo);
  p.div_ohw = make_fastdiv(s->ho * s->wo);
  (void)es;
  TileChoice tc = choose_tile(s->cout);
  hipStream_t st = (hipStream_t)stream;
  if (stats) return dispatch_nt<MODE_FWD, EPI_STATS>(p, s->dtype, s->k, tc.cfg, st);
  return dispatch_nt<MODE_FWD, EPI_AFFINE>(p, s->dtype, s->k, tc.cfg, st);
}

yms_status yms_conv_dgrad(const yms_conv_shape* s, const void* dz, int dz_ld, int dz_off,
                          const void* wpacked_t, void* dx, int dx_ld, int dx_off,
                          int accumulate, void* stream) {
  if (!shape_ok(s) || !dz || !wpacked_t || !dx) return YMS_ERR_INVALID;
  if (!view_ok(dz_ld, dz_off, s->cout) || !view_ok(dx_ld, dx_off, s->cin)) return YMS_ERR_INVALID;
  {
    DirectGeo dg;
    if (conv_direct_geometry(s, 1, &dg))
      return conv_direct_launch(s, 1, dg, dz, dz_ld, dz_off, wpacked_t, dx, dx_ld, dx_off, nullptr, nullptr, 0,
                                nullptr, 0, 0, nullptr, accumulate, (hipStream_t)stream);
  }
  NTParams p{};
  p.src = (const char*)dz;
  p.wp = (const char*)wpacked_t;
  p.dst = (char*)dx;
  p.src_ld = dz_ld; p.src_off = dz_off; p.dst_ld = dx_ld; p.dst_off = dx_off;
  p.SH = s->ho; p.SW = s->wo; p.OW = s->w;
  if (!offsets32(s->n, s->ho, s->wo, dz_ld)) return YMS_ERR_UNSUPPORTED;
  p.stride = s->stride; p.pad = s->pad;
  p.Ncols = s->cin;
  p.OH = s->h; p.OWx = s->w;
  TileChoice tc = choose_tile(s->cin);
  hipStream_t st = (hipStream_t)stream;
  if (s->stride == 2) {
    Dg2Geo d = dg2_geo(s);
    const int es = elem_size(s->dtype);
    p.cpt = d.cpt;
    if (!set_src_geometry(p, s->n, s->ho, s->wo, dz_ld, es, *std::max_element(d.nkt, d.nkt + 4) * NT_KCH))
      return YMS_ERR_UNSUPPORTED;
    p.M = 0;
    for (int c = 0; c < 4; ++c) {
      p.cls_M[c] = d.M[c];
      p.cls_nkt[c] = d.nkt[c];
      p.cls_Kc[c] = d.Kc[c];
      p.cls_ntx[c] = d.ntx[c];
      p.cls_c0y[c] = d.c0y[c];
      p.cls_c0x[c] = d.c0x[c];
      p.cls_woff[c] = d.off_elems[c] * es;
      p.cls_div_w[c] = make_fastdiv(std::max(1, d.Wa[c]));
      p.cls_div_hw[c] = make_fastdiv(std::max(1, d.Ha[c] * d.Wa[c]));
      p.M = std::max(p.M, d.M[c]);
    }
    if (p.M == 0) return YMS_OK;
    if (accumulate) return dispatch_nt<MODE_DGRAD2, EPI_ACCUM>(p, s->dtype, s->k, tc.cfg, st);
    return dispatch_nt<MODE_DGRAD2, EPI_STORE>(p, s->dtype, s->k, tc.cfg, st);
  }
  PackGeo g = pack_geo(s, 1);
  p.cpt = g.cpt; p.Kc = g.kc; p.nkt = g.nkt;
  if (!set_src_geometry(p, s->n, s->ho, s->wo, dz_ld, elem_size(s->dtype), g.nkt * NT_KCH))
    return YMS_ERR_UNSUPPORTED;
  p.M = s->n * s->h * s->w;
  p.div_ow = make_fastdiv(s->w);
  p.div_ohw = make_fastdiv(s->h * s->w);
  if (accumulate) return dispatch_nt<MODE_DGRAD, EPI_ACCUM>(p, s->dtype, s->k, tc.cfg, st);
  return dispatch_nt<MODE_DGRAD, EPI_STORE>(p, s->dtype, s->k, tc.cfg, st);
}

int yms_conv_dgrad_bnred_rows(const yms_conv_shape* s) {
  DirectGeo dg;
  if (!shape_ok(s) || s->cin % 8 != 0 || !conv_direct_geometry(s, 1, &dg, true)) return 0;
  return dg.grid;
}

yms_status yms_conv_dgrad_bnred(const yms_conv_shape* s, const void* dz, int dz_ld, int dz_off,
                                const void* wpacked_t, void* dx, int dx_ld, int dx_off, int accumulate,
                                const void* z, int z_ld, int z_off, const float* scale, const float* shift,
                                const float* mean_invstd, int act, float* ws, void* stream) {
  if (!shape_ok(s) || !dz || !wpacked_t || !dx || !z || !scale || !shift || !mean_invstd || !ws)
    return YMS_ERR_INVALID;
  if (!view_ok(dz_ld, dz_off, s->cout) || !view_ok(dx_ld, dx_off, s->cin) || !view_ok(z_ld, z_off, s->cin))
    return YMS_ERR_INVALID;
  if (act != YMS_ACT_NONE && act != YMS_ACT_SILU) return YMS_ERR_INVALID;
  DirectGeo dg;
  if (s->cin % 8 != 0 || !conv_direct_geometry(s, 1, &dg, true)) return YMS_ERR_UNSUPPORTED;
  const DirectBnRed b{z, z_ld, z_off, scale, shift, mean_invstd, act, ws};
  return conv_direct_launch(s, 1, dg, dz, dz_ld, dz_off, wpacked_t, dx, dx_ld, dx_off, nullptr, nullptr, 0, nullptr,
                            0, 0, nullptr, accumulate, (hipStream_t)stream, &b);
}

size_t yms_conv_wgrad_ws_bytes(const yms_conv_shape* s) {
  if (!shape_ok(s)) return 0;
  WHPlan wh;
  if (wgrad_halo_plan(s, &wh)) return (size_t)wh.splits * wh.wk * wh.slab_rows * wh.slab_ld * sizeof(float);
  WRPlan wr;
  if (wgrad_ring_plan(s, &wr)) return (size_t)wr.splits * wr.slab_rows * wr.slab_ld * sizeof(float);
  WgradPlan w = wgrad_plan(s);
  return (size_t)w.splits * w.slab_rows * w.slab_ld * sizeof(float);
}

// fewer split-K partial slabs when the caller's workspace holds fewer than the plan asks for (a
// workspace sized under other YMS_WG_* settings than the call's): units of work (patches / k-tiles)
// per split grow until `splits` slabs of slab_bytes fit; false when not even one fits
static bool fit_splits(size_t ws_bytes, size_t slab_bytes, int units, int& per, int& splits) {
  const size_t cap = ws_bytes / slab_bytes;
  if (cap < 1) return false;
  if ((size_t)splits > cap) {
    per = cdiv(units, (int)cap);
    splits = cdiv(units, per);
  }
  return true;
}

yms_status yms_conv_wgrad(const yms_conv_shape* s, const void* x, int x_ld, int x_off,
                          const void* dz, int dz_ld, int dz_off, float* ws, size_t ws_bytes,
                          float* dw, int accumulate, void* stream) {
  if (!shape_ok(s) || !x || !dz || !ws || !dw) return YMS_ERR_INVALID;
  if (!view_ok(x_ld, x_off, s->cin) || !view_ok(dz_ld, dz_off, s->cout)) return YMS_ERR_INVALID;
  {
    // 3x3: the halo-tiled kernel (wgrad_halo.hip) stages each input patch once for all nine taps
    WHPlan wh;
    if (wgrad_halo_plan(s, &wh)) {
      if (!fit_splits(ws_bytes, (size_t)wh.wk * wh.slab_rows * wh.slab_ld * sizeof(float), wh.npatch, wh.pps, wh.splits))
        return YMS_ERR_INVALID;
      yms_status e = wgrad_halo_launch(s, wh, x, x_ld, x_off, dz, dz_ld, dz_off, ws, (hipStream_t)stream);
      if (e != YMS_OK) return e;
      const int cin8 = (int)rup(s->cin, 8);
      const int kf = 9 * cin8;
      dim3 g2((unsigned)(s->cout * cdiv(kf, 128)));
      hipLaunchKernelGGL(wgrad_reduce_kernel, g2, dim3(256), 0, (hipStream_t)stream, ws, wh.splits * wh.wk,
                         (long)wh.slab_rows * wh.slab_ld, wh.slab_ld, s->cout, s->cin, cin8, s->k, dw, accumulate);
      return launch_status();
    }
  }
  {
    // 1x1 / 3x3 with > 32 output channels: both operands on an LDS-DMA ring (wgrad_ring.hip)
    WRPlan wr;
    if (wgrad_ring_plan(s, &wr)) {
      if (!fit_splits(ws_bytes, (size_t)wr.slab_rows * wr.slab_ld * sizeof(float), wr.nkt, wr.kt_per_split, wr.splits))
        return YMS_ERR_INVALID;
      yms_status e = wgrad_ring_launch(s, wr, x, x_ld, x_off, dz, dz_ld, dz_off, ws, (hipStream_t)stream);
      if (e != YMS_OK) return e;
      const int kf = s->k * s->k * wr.cin8;
      dim3 g2((unsigned)(s->cout * cdiv(kf, 128)));
      hipLaunchKernelGGL(wgrad_reduce_kernel, g2, dim3(256), 0, (hipStream_t)stream, ws, wr.splits,
                         (long)wr.slab_rows * wr.slab_ld, wr.slab_ld, s->cout, s->cin, wr.cin8, s->k, dw, accumulate);
      return launch_status();
    }
  }
  WgradPlan w = wgrad_plan(s);
  if (!fit_splits(ws_bytes, (size_t)w.slab_rows * w.slab_ld * sizeof(float), w.nkt, w.kt_per_split, w.splits))
    return YMS_ERR_INVALID;
  TTParams p{};
  p.x = (const char*)x; p.dz = (const char*)dz; p.slab = ws;
  p.x_ld = x_ld; p.x_off = x_off; p.dz_ld = dz_ld; p.dz_off = dz_off;
  p.SH = s->h; p.SW = s->w; p.OW = s->wo; p.stride = s->stride; p.pad = s->pad;
  p.cpt = w.cpt; p.Kc = w.kc;
  p.M = s->n * s->ho * s->wo;
  p.cout8 = (int)rup(s->cout, 8);
  p.nkt = w.nkt; p.kt_per_split = w.kt_per_split; p.tiles_n = w.tiles_n;
  p.slab_rows = w.slab_rows; p.slab_ld = w.slab_ld;
  p.div_ow = make_fastdiv(s->wo);
  p.div_ohw = make_fastdiv(s->ho * s->wo);
  {
    const long es = elem_size(s->dtype);
    const long dzb = (long)p.M * dz_ld * es, xb = (long)s->n * s->h * s->w * x_ld * es;
    if (dzb >= (1l << 31) - (1l << 20) || xb >= (1l << 31) - (1l << 20)) return YMS_ERR_UNSUPPORTED;
    p.dz_bytes = (uint32_t)dzb;
    p.x_bytes = (uint32_t)xb;
  }
  hipStream_t st = (hipStream_t)stream;
  p.tiles_m_n = w.tiles_m * w.tiles_n;
  dim3 grid((unsigned)(w.tiles_m * w.tiles_n * w.splits));
  if (s->dtype == YMS_BF16) {
    if (s->k == 1) launch_wgrad<bf16, 1>(p, w.bm, w.bn, grid, st); else launch_wgrad<bf16, 3>(p, w.bm, w.bn, grid, st);
  } else if (s->dtype == YMS_F16) {
    if (s->k == 1) launch_wgrad<f16, 1>(p, w.bm, w.bn, grid, st); else launch_wgrad<f16, 3>(p, w.bm, w.bn, grid, st);
  } else {
    if (s->k == 1) launch_wgrad<float, 1>(p, w.bm, w.bn, grid, st); else launch_wgrad<float, 3>(p, w.bm, w.bn, grid, st);
  }
  yms_status e = launch_status();
  if (e != YMS_OK) return e;
  const int kf = s->k * s->k * w.cin8;
  dim3 g2((unsigned)(s->cout * cdiv(kf, 128)));
  hipLaunchKernelGGL(wgrad_reduce_kernel, g2, dim3(256), 0, st, ws, w.splits,
                     (long)w.slab_rows * w.slab_ld, w.slab_ld, s->cout, s->cin, w.cin8, s->k, dw, accumulate);
  return launch_status();
}

}  // extern "C"

// Device helpers shared by the convolution kernels (conv_igemm.hip, conv_direct.hip, stem.hip,
// wgrad_*.hip, dwconv.hip): MFMA wrappers, counted vmcnt waits, the raw barrier,
// raw-buffer LDS-DMA and the XCD-aware block remap.
#pragma once
#include "yms_common.hpp"

namespace yms {

constexpr int NT_KCH = 8;     // 16-B chunks of K per k-tile row (128 B)
constexpr int NT_ROWP = 144;  // LDS pitch: 128 B + 16 B pad (conflict-free ds_read_b128 over 16 rows)

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_DGRAD2 = 2 };  // DGRAD2: stride-2 dgrad by output parity
enum { EPI_AFFINE = 0, EPI_STATS = 1, EPI_STORE = 2, EPI_ACCUM = 3 };

// XCD-aware block order: hardware dispatches consecutive workgroup ids round-robin over the
// 8 XCDs; remap (bijectively) so that consecutive LOGICAL ids -- the N tiles of one row
// tile, and neighbouring row tiles that share im2col halo rows -- run on the same XCD and
// share its L2 (MI355X_MICROARCH.md, Workgroup dispatch).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, k = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  static __device__ __forceinline__ f32x16 mma(const u32x4& a, const u32x4& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mfma<f16> {
  static __device__ __forceinline__ f32x16 mma(const u32x4& a, const u32x4& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// s_waitcnt vmcnt(N) alone (expcnt/lgkmcnt left at their maxima), gfx9 encoding
template <int N> __device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}
// wait until at most min(n, MAXN) k-tiles of NG loads each are still in flight
template <int NG, int MAXN> __device__ __forceinline__ void wait_tiles(int n) {
  if constexpr (MAXN > 0) {
    if (n >= MAXN) { wait_vmcnt<MAXN * NG>(); return; }
    wait_tiles<NG, MAXN - 1>(n);
  } else {
    wait_vmcnt<0>();
  }
}
// workgroup barrier that does NOT drain the vector-memory counter (so LDS-DMA loads of later
// k-tiles stay in flight across it); the clobbers keep the compiler from moving LDS accesses
// across it.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// raw-buffer LDS-DMA of 16 B per lane; an offset at or past the resource's num_records loads
// zeros.  (The builtin is wrapped so the host pass of a kernel template never sees it: clang
// silently drops the host stub of a template kernel that names it directly.)
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (YMS_LDS void*)lds_wave_base, 16, voff, 0, 0, 0);
#endif
}
__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

constexpr uint32_t NT_OOB = 0x80000000u;    // voffset past every A resource (num_records < 2^31)
constexpr int NT_RSRC3 = 0x00020000;        // buffer descriptor word 3 (gfx9 raw buffer, 32-bit data)

// ------------------------------------------------------------------------------------------
// BN training statistics contract (consumed by yms_bn_finalize, bn_pool.hip): one row per
// 128 output pixels (row r covers pixels [128r, min(128r + 128, M))), row[0][c] = sum of z,
// row[1][c] = sum of (z - mean_r)^2 about that row's OWN mean.  Centred second moments keep
// the variance exact to fp32 rounding however large |mean| / std is (sum z^2 - n mean^2 loses
// (mean/std)^2 x eps relative precision, which the deep MS-Block graphs amplify).
// ------------------------------------------------------------------------------------------
// One wave's 32-column MFMA block (TM tiles of 32 rows; accumulator i of lane half lh is row
// a*32 + (i&3) + 8*(i>>2) + 4*lh): sum and centred M2 over its first nw rows, two passes over
// the registers, combined across the two lane halves.
template <int TM, typename Acc>
__device__ __forceinline__ void wave_col_moments(const Acc& acc, int b, int nw, int lh, float& s1, float& m2) {
  float s = 0.f, q = 0.f;
  if (nw >= TM * 32) {                    // wave-uniform: every row valid, no per-element selects
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) s += acc[a][b][i];
    s += __shfl_xor(s, 32);
    const float mu = s * (1.0f / (TM * 32));
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float d = acc[a][b][i] - mu;
        q += d * d;
      }
  } else {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh < nw) s += acc[a][b][i];
    s += __shfl_xor(s, 32);
    const float mu = nw > 0 ? s / (float)nw : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh < nw) {
          const float d = acc[a][b][i] - mu;
          q += d * d;
        }
  }
  q += __shfl_xor(q, 32);
  s1 = s;
  m2 = q;
}

// Chan merge of NP consecutive row groups of R rows each (group w: sum s[w*stride], M2
// m[w*stride]); only the first nrows rows exist.  -> sum and M2 about the merged mean.
template <int NP, int R>
__device__ __forceinline__ void merge_moments(const float* s, const float* m, int stride, int nrows, float& t1,
                                              float& t2) {
  nrows = min(nrows, NP * R);
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NP; ++w) tot += s[w * stride];
  const float mu = nrows > 0 ? tot / (float)nrows : 0.f;
  float q = 0.f;
#pragma unroll
  for (int w = 0; w < NP; ++w) {
    const int nw = min(R, max(0, nrows - w * R));
    if (nw > 0) {
      const float d = s[w * stride] / (float)nw - mu;
      q += m[w * stride] + (float)nw * d * d;
    }
  }
  t1 = tot;
  t2 = q;
}


// host: CU count of the current device (persistent grids)
int conv_cu_count();

}  // namespace yms

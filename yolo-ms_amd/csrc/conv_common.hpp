// Device helpers shared by the implicit-GEMM convolution kernels (conv_igemm.hip) and the
// halo-tiled 3x3 kernel (conv_halo.hip): MFMA wrappers, counted vmcnt waits, the raw barrier,
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


// host: CU count of the current device (persistent grids)
int conv_cu_count();

}  // namespace yms

// Shared device helpers for the YOLO-MS / YOLOv8 hot path on MI355X (gfx950, CDNA4).
// Wave64 everywhere; NHWC activations with a channel stride `ld` and channel offset `off`
// (both multiples of 8 elements, so every 8-channel group is 16-byte aligned for 16-bit
// types and 32-byte aligned for fp32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/yms.h"

namespace yms {

typedef __bf16 bf16;
typedef _Float16 f16;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));   // 16-B register chunk (SROA-friendly, unlike HIP's uint4 struct)

#define YMS_LDS __attribute__((address_space(3)))

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

// SiLU / sigmoid with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE divide
// (~10 VALU ops): these run in every conv epilogue and BN kernel.
__device__ __forceinline__ float sigmoid_f(float a) { return __builtin_amdgcn_rcpf(1.0f + __expf(-a)); }
__device__ __forceinline__ float silu_f(float a) { return a * sigmoid_f(a); }
// SiLU'(a) = s (1 + a (1 - s)), s = sigmoid(a); hardware reciprocal (1 ulp) -- gradients only
__device__ __forceinline__ float dsilu_f(float a) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-a));
  return s * (1.0f + a * (1.0f - s));
}

// 8 consecutive channel values as floats (16-bit types: one 16-B load; fp32: two).
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <typename T16> struct Vec8_16 {
  typedef T16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ void load(const T16* p, float (&v)[8]) {
    v8 a = *reinterpret_cast<const v8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  static __device__ __forceinline__ void store(T16* p, const float (&v)[8]) {
    v8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (T16)v[i];
    *reinterpret_cast<v8*>(p) = a;
  }
};
template <> struct Vec8<bf16> : Vec8_16<bf16> {};
template <> struct Vec8<f16> : Vec8_16<f16> {};

// Masked 8-channel access for views whose logical channel count is not a multiple of 8.
template <typename T>
__device__ __forceinline__ void load8(const T* p, int valid, float (&v)[8]) {
  if (valid >= 8) {
    Vec8<T>::load(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (i < valid) ? (float)p[i] : 0.0f;
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, int valid, const float (&v)[8]) {
  if (valid >= 8) {
    Vec8<T>::store(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < valid) p[i] = (T)v[i];
  }
}

// 8 channel values kept in their storage format (4 VGPRs for 16-bit types, 8 for fp32) so
// that several pixels' loads can be in flight per thread without spending 8 VGPRs each.
// Barrier ordering LDS only: outstanding global loads (register prefetches of later work) and
// stores stay in flight across it, unlike __syncthreads()'s vmcnt(0).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <typename T> struct Raw8 { u32x4 v[sizeof(T) / 2]; };

template <typename T>
__device__ __forceinline__ void load_raw8(const T* p, int valid, Raw8<T>& r) {
  if (valid >= 8) {
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 2); ++k) r.v[k] = reinterpret_cast<const u32x4*>(p)[k];
  } else {
    T t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = (i < valid) ? p[i] : (T)0.0f;
    __builtin_memcpy(&r, t, sizeof(t));
  }
}
// the same 16-B chunk(s) with the non-temporal hint: the last read of a streamed tensor, so its
// lines do not displace ones the concurrent kernels still reuse from L2 / the Infinity Cache
template <typename T>
__device__ __forceinline__ void load_raw8_nt(const T* p, Raw8<T>& r) {
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 2); ++k)
    r.v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + k);
}
template <typename T>
__device__ __forceinline__ void unpack8(const Raw8<T>& r, float (&f)[8]) {
  T t[8];
  __builtin_memcpy(t, &r, sizeof(t));
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)t[i];
}
// bf16 -> fp32 is a 16-bit shift: done on the 32-bit words, so the 16-B chunk stays one value (the
// element-wise form above lets hipcc re-split rows of chunks into u16 + misaligned b128 reads)
template <>
__device__ __forceinline__ void unpack8<bf16>(const Raw8<bf16>& r, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(r.v[0][j] << 16);
    f[2 * j + 1] = __uint_as_float(r.v[0][j] & 0xffff0000u);
  }
}

// Unsigned 31-bit fast division by a runtime constant (Granlund-Montgomery).
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  if (d == 1) { f.m = 0; f.s = 0; }
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.m);
  return (uint32_t)(((uint64_t)hi + n) >> f.s);
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline long rup(long a, long b) { return (a + b - 1) / b * b; }

inline yms_status launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? YMS_OK : YMS_ERR_LAUNCH;
}

}  // namespace yms

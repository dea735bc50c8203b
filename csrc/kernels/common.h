// Shared device helpers for the pyrecover_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63; wave-level reductions use __shfl_xor over 64 lanes.
//   * bf16/fp16 are moved as 16-byte vectors (8 elements) per lane; fp32 as 2x16 B.
//   * all math is fp32 ("opmath"), outputs are rounded once with the hardware cvt
//     (v_cvt_pk_bf16_f32, RNE, NaN-preserving).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace pra {

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---- scalar conversion ---------------------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<__bf16>(__bf16 v) { return (float)v; }
template <> __device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return (__bf16)v; }
template <> __device__ __forceinline__ __half from_f<__half>(float v) { return __float2half_rn(v); }

// round-trip through the storage type (reproduces torch's per-op rounding)
template <typename T> __device__ __forceinline__ float rnd(float v) { return to_f<T>(from_f<T>(v)); }

// ---- 8-wide vector load/store (16 B for 16-bit types, 32 B for fp32) -----------------
template <typename T> struct Vec8 { float v[8]; };

template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, float (&o)[8]);
template <>
__device__ __forceinline__ void load8<__bf16>(const __bf16* __restrict__ p, float (&o)[8]) {
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void load8<__half>(const __half* __restrict__ p, float (&o)[8]) {
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  const __half* h = reinterpret_cast<const __half*>(&raw);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = __half2float(h[i]);
}
template <>
__device__ __forceinline__ void load8<_Float16>(const _Float16* __restrict__ p, float (&o)[8]) {
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  const _Float16* h = reinterpret_cast<const _Float16*>(&raw);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (float)h[i];
}
template <>
__device__ __forceinline__ void load8<float>(const float* __restrict__ p, float (&o)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <typename T>
__device__ __forceinline__ void store8(T* __restrict__ p, const float (&v)[8]);
template <>
__device__ __forceinline__ void store8<__bf16>(__bf16* __restrict__ p, const float (&v)[8]) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (__bf16)v[i];
  *reinterpret_cast<bf16x8*>(p) = b;
}
template <>
__device__ __forceinline__ void store8<__half>(__half* __restrict__ p, const float (&v)[8]) {
  uint4 raw;
  __half* h = reinterpret_cast<__half*>(&raw);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = __float2half_rn(v[i]);
  *reinterpret_cast<uint4*>(p) = raw;
}
template <>
__device__ __forceinline__ void store8<float>(float* __restrict__ p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// ---- reductions ------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NW waves; `scratch` must hold NW floats. Deterministic order.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += scratch[i];
  __syncthreads();
  return r;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

}  // namespace pra

#define PRA_DISPATCH_FLOAT(dtype, T, ...)                          \
  switch (dtype) {                                                 \
    case ::pra::kF32: { using T = float; __VA_ARGS__; break; }     \
    case ::pra::kBF16: { using T = __bf16; __VA_ARGS__; break; }   \
    case ::pra::kF16: { using T = __half; __VA_ARGS__; break; }    \
    default: return hipErrorInvalidValue;                          \
  }

// bf16 / fp16 only (kernels that pack elements into 16-bit LDS tiles)
#define PRA_DISPATCH_16BIT(dtype, T, ...)                          \
  switch (dtype) {                                                 \
    case ::pra::kBF16: { using T = __bf16; __VA_ARGS__; break; }   \
    case ::pra::kF16: { using T = __half; __VA_ARGS__; break; }    \
    default: return hipErrorInvalidValue;                          \
  }

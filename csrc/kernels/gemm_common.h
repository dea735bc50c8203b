// Shared pieces of the hand-written MFMA GEMMs (gemm_wgrad.hip, gemm_nt.hip), gfx950 only.
//
// Both kernels use the same machine: 256 x 256 workgroup tiles, 4 waves of 128 x 128, 32-deep
// k-stages staged global -> LDS by LDS-DMA (global_load_lds_dwordx4 in the SGPR-base form) into a
// 5-stage ring (all 160 KiB of LDS), counted vmcnt waits + raw s_barrier, v_mfma_f32_16x16x32
// (the shape the chip holds the higher clock on), XCD-aware tile order and a deterministic split-K
// tail. They differ in the LDS image and the fragment reads: the weight-gradient kernel reads
// K-slow operands through ds_read_b64_tr_b16, the NT kernel K-contiguous ones with ds_read_b128.
#pragma once
#include "common.h"

#include <type_traits>

namespace pra {
namespace gm {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <typename T> struct Elem;
template <> struct Elem<__bf16> { typedef bf16x8 v8; };
template <> struct Elem<_Float16> { typedef f16x8 v8; };
template <typename T>
using V8 = typename Elem<T>::v8;
template <int N>
using IC = std::integral_constant<int, N>;

// f(IC<I>{}) for I in [I0, N): a compile-time loop (a 128-step #pragma unroll body with nested loops
// can stay rolled, which turns register arrays into scratch)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

constexpr int BM = 256, BN = 256, BK = 32, NTH = 256, NS = 5;
constexpr int TILE = BK * 256;              // elements per staged operand tile (16 KiB)
constexpr int NI = TILE * 2 / (NTH * 16);   // LDS-DMA instructions per lane per operand tile (4)
constexpr int GM = 8;                       // M-tiles per group of the tile order

template <typename T>
__device__ __forceinline__ uint32_t pack_x2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (T)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (T)b) << 16);
}

// one 16-B-per-lane LDS-DMA with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit byte
// offset ("saddr" form): lane l's 16 bytes land at LDS byte lds + 16 l (M0 = wave-uniform LDS
// base; one wait state between the M0 write and the load). M0 is not declared clobbered (the
// compiler reserves it and warns): nothing in these kernels reads M0.
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

// The same DMA as two statements, for schedules that put an MFMA between the M0 write and the load
// (the MFMA is the wait state, so no s_nop): m0_set, >= 1 other instruction, dma16s_go.
__device__ __forceinline__ void m0_set(uint32_t lds) { asm volatile("s_mov_b32 m0, %0" ::"s"(lds)); }
__device__ __forceinline__ void dma16s_go(const void* sbase, uint32_t voff) {
  asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase) : "memory");
}

// s_waitcnt vmcnt(N) for a compile-time N
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N == 0 || N == 8 || N == 15 || N == 16 || N == 18 || N == 24 || N == 32 || N == 48, "add the count");
  if constexpr (N == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  if constexpr (N == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// XCD-contiguous index of workgroup `orig` among n: undoes the round-robin placement of
// consecutive workgroups over the 8 XCDs (bijective for any n)
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int xcd = orig % 8, q = n / 8, r = n % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// group-M tile order: GM M-tiles share each B column panel, so the workgroups resident on one
// XCD at a time share a few A and B panels in its L2
__device__ __forceinline__ void tile_origin(int lin, int tiles_m, int tiles_n, long& m0, long& n0) {
  const int group = lin / (GM * tiles_n), first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  m0 = (long)(first_m + (lin % (GM * tiles_n)) % gsz) * BM;
  n0 = (long)((lin % (GM * tiles_n)) / gsz) * BN;
}

}  // namespace gm

// Split of the partial last round (host side, shared by the GEMM launchers): the R = nwg % cus
// tail tiles are split S ways over K when that fills whole rounds better (S <= smax, ties -> the
// smaller S). Returns S (1 = unsplit).
inline int gemm_tail_split(int nwg, int cus, int nk, int smax) {
  if (nwg <= cus || nwg % cus == 0) return 1;
  const int R = nwg % cus;
  double best = 1.0;  // unsplit: one more round
  int S = 1;
  for (int c = 2; c <= smax && c <= 8 && c <= nk; ++c) {
    const double t = (double)((R * c + cus - 1) / cus) / c;
    if (t < best - 1e-9) best = t, S = c;
  }
  return S;
}

}  // namespace pra

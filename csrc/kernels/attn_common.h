// Device helpers shared by the attention kernels (attention.hip, attention_fwd64.hip): the LDS
// tile image, MFMA operand reads, LDS-DMA / register staging, and the row-per-lane epilogue.
// gfx950 only; every function lives in namespace pra::attn.
#pragma once
#include "common.h"

#include <type_traits>

namespace pra {
namespace attn {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// LDS image of a [rows][D] bf16 tile: 8-row x 32-column sub-tiles of 512 B, the four 16-B
// chunks of each 64-B sub-tile row XOR-swizzled by (row >> 2) & 3 (cdna guide T10, image (a)).
// Conflict-free for ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads of the
// 32x32x16 operands, and -- unlike a whole-row XOR -- every k-step / column block / row block
// (row base a multiple of 16) is a compile-time byte offset from one of two lane-constant bases,
// so fragment reads need 4 address registers instead of one per k-step.
template <int D>
__device__ __forceinline__ int lay_byte(int r, int ch) {  // byte offset of 16-B chunk ch of row r
  return (D * 16) * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}
template <int D>
__device__ __forceinline__ void lay_inverse(int o, int& r, int& ch) {  // byte offset -> (row, chunk)
  const int rg = o / (D * 16), rem = o % (D * 16);
  const int sub = rem / 512, r7 = (rem % 512) / 64, slot = (rem % 64) / 16;
  r = 8 * rg + r7;
  ch = 4 * sub + (slot ^ ((r >> 2) & 3));
}

// Element traits: the kernels are instantiated for bf16 (v_mfma_f32_32x32x16_bf16) and fp16
// (v_mfma_f32_32x32x16_f16); both move as 8 x 16-bit per lane and accumulate in fp32.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <typename T> struct Elem;
template <> struct Elem<__bf16> { typedef bf16x8 v8; };
template <> struct Elem<_Float16> { typedef f16x8 v8; };
template <typename T>
using V8 = typename Elem<T>::v8;

template <typename T>
__device__ __forceinline__ V8<T> lds_read16(const T* tile, int byte_off) {
  return *reinterpret_cast<const V8<T>*>(reinterpret_cast<const char*>(tile) + byte_off);
}
template <typename T>
__device__ __forceinline__ i16x4 tr4(const T* tile, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_i16x4*)(reinterpret_cast<const char*>(tile) + byte_off));
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ V8<T> pack8(const f32x16& x, int s) {
  V8<T> r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (T)x[8 * s + j];
  return r;
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// Row-per-lane epilogue of a 32 x (32 NDB) accumulator tile X^T (lane l32 holds row l32 of X, register r
// of block db holds column 32 db + crow(r, h2)): v_permlane32_swap hands each half-wave the other's
// 4-column group, so every lane stores 8 contiguous 16-bit values (16 B) per instruction instead of two
// separate 8-B pieces (cdna guide T21: halves the store-issue tail). p = &X[row][0], values * f.
// All 64 lanes must execute it (the swap); `ok` guards only the stores.
template <typename T>
__device__ __forceinline__ uint32_t pack_x2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (T)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (T)b) << 16);
}
// rt (optional): this lane's row of the RoPE table (float2 (cos, sin) per column pair, the layout of
// the RoPE kernels); the inverse rotation of each (2i, 2i+1) pair is applied to the fp32 values
// before they are rounded (the backward's dQ / dK leave the kernel already un-rotated, so the
// separate inverse-RoPE pass over dq|dk is gone). A pair never straddles lanes: register k (even) of
// block db holds column 32 db + crow(k, h2), and k + 1 the next column.
__device__ __forceinline__ void rot_inv(float& a, float& b, float c, float s) {  // (a + ib)(c - is)
  const float o0 = __builtin_fmaf(a, c, -(b * -s));
  const float o1 = __builtin_fmaf(a, -s, b * c);
  a = o0;
  b = o1;
}
template <typename T, int NDB>
__device__ __forceinline__ void store_rows16(const f32x16 (&acc)[NDB], float f, T* p, bool ok, int h2,
                                             const float2* rt = nullptr) {
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int a = 8 * m, c = 8 * m + 4;  // register groups rr = 2m (A) and 2m + 1 (B)
      float va[4], vc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        va[j] = acc[db][a + j] * f;
        vc[j] = acc[db][c + j] * f;
      }
      if (rt != nullptr) {  // pairs 16 db + 8 m + 2 h2 + {0, 1} (A) and + 4 (B)
        const float4 ta = *reinterpret_cast<const float4*>(rt + 16 * db + 8 * m + 2 * h2);
        const float4 tc = *reinterpret_cast<const float4*>(rt + 16 * db + 8 * m + 4 + 2 * h2);
        rot_inv(va[0], va[1], ta.x, ta.y);
        rot_inv(va[2], va[3], ta.z, ta.w);
        rot_inv(vc[0], vc[1], tc.x, tc.y);
        rot_inv(vc[2], vc[3], tc.z, tc.w);
      }
      const auto x0 = __builtin_amdgcn_permlane32_swap(pack_x2<T>(vc[0], vc[1]), pack_x2<T>(va[0], va[1]), false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(pack_x2<T>(vc[2], vc[3]), pack_x2<T>(va[2], va[3]), false, false);
      if (ok)
        *reinterpret_cast<uint4*>(p + 32 * db + 16 * m + 8 * (1 - h2)) = make_uint4(x0[0], x1[0], x0[1], x1[1]);
    }
}

// store_rows16's register layout written as fp32 (no lane exchange): the lane's 4-column groups
// sit at 32 db + 16 m + 4 h2 (registers 8m..8m+3) and 8 further on (8m+4..8m+7)
template <int NDB>
__device__ __forceinline__ void store_rows16_f32(const f32x16 (&acc)[NDB], float f, float* p, int h2,
                                                 const float2* rt = nullptr) {
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int a = 8 * m, c = 8 * m + 4;
      float va[4], vc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        va[j] = acc[db][a + j] * f;
        vc[j] = acc[db][c + j] * f;
      }
      if (rt != nullptr) {
        const float4 ta = *reinterpret_cast<const float4*>(rt + 16 * db + 8 * m + 2 * h2);
        const float4 tc = *reinterpret_cast<const float4*>(rt + 16 * db + 8 * m + 4 + 2 * h2);
        rot_inv(va[0], va[1], ta.x, ta.y);
        rot_inv(va[2], va[3], ta.z, ta.w);
        rot_inv(vc[0], vc[1], tc.x, tc.y);
        rot_inv(vc[2], vc[3], tc.z, tc.w);
      }
      *reinterpret_cast<float4*>(p + 32 * db + 16 * m + 4 * h2) = make_float4(va[0], va[1], va[2], va[3]);
      *reinterpret_cast<float4*>(p + 32 * db + 16 * m + 8 + 4 * h2) = make_float4(vc[0], vc[1], vc[2], vc[3]);
    }
}

// lanes i and i^32 exchange through v_permlane32_swap (no LDS round trip)
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Stage ROWS x D rows of a [.., ld]-strided bf16 tensor into registers (global loads only).
// Chunk assignment: a ds_write_b128 is serviced in 8-lane groups over 32 banks (128 B), so each
// group of 8 lanes takes the same 4 chunks (one 64-B sub-tile row) of two ADJACENT rows -- 64 B
// apart in the image, i.e. 128 distinct bytes mod 128 (conflict-free). Row-major (8 consecutive
// chunks of one row per group) put chunk c and c + 4 on the same banks (2-way on every store).
template <typename T, int D, int ROWS, int NT = 256>
struct Stage {
  static constexpr int CH = D / 8;
  static constexpr int R64 = 64 / CH;  // rows covered by 64 consecutive chunk indices
  static constexpr int CPT = (ROWS * CH + NT - 1) / NT;
  static constexpr bool EXACT = CPT * NT == ROWS * CH;  // else the last pass is partial
  static_assert(ROWS * CH % 64 == 0, "whole 64-chunk blocks");
  uint4 r[CPT];
  __device__ __forceinline__ static void rc(int idx, int& row, int& c) {
    const int l = idx & 63, gi = l >> 3, j = l & 7;
    row = R64 * (idx >> 6) + 2 * (gi % (R64 / 2)) + (j >> 2);
    c = 4 * (gi / (R64 / 2)) + (j & 3);
  }
  __device__ __forceinline__ void load(const T* g, long ld, int row0, int nrows_valid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = i * NT + threadIdx.x;
      if (!EXACT && idx >= ROWS * CH) continue;
      int row, c;
      rc(idx, row, c);
      if (row0 + row < nrows_valid)
        r[i] = *reinterpret_cast<const uint4*>(g + (long)(row0 + row) * ld + c * 8);
      else
        r[i] = make_uint4(0, 0, 0, 0);
    }
  }
  // every row in bounds (no per-row branch: the load count is a compile-time constant, so counted
  // vmcnt waits stay exact across it)
  __device__ __forceinline__ void load_all(const T* g, long ld, int row0) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = i * NT + threadIdx.x;
      if (!EXACT && idx >= ROWS * CH) continue;
      int row, c;
      rc(idx, row, c);
      r[i] = *reinterpret_cast<const uint4*>(g + (long)(row0 + row) * ld + c * 8);
    }
  }
  __device__ __forceinline__ void store(T* tile) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = i * NT + threadIdx.x;
      if (!EXACT && idx >= ROWS * CH) continue;
      int row, c;
      rc(idx, row, c);
      *reinterpret_cast<uint4*>(reinterpret_cast<char*>(tile) + lay_byte<D>(row, c)) = r[i];
    }
  }
};

// LDS-DMA staging (global_load_lds_dwordx4) of a ROWS x D tile into the LDS image. The DMA
// writes 1 KiB per wave-instruction linearly (base + 16 B * lane), so each lane fetches the
// (row, chunk) that the image places at its linear position.
// No VGPR staging; rows must be in bounds (callers guarantee S % tile == 0).
// Instruction i of a lane covers image bytes i * NWV KiB further on: exactly RSTEP more rows, same
// chunk and same XOR swizzle (the swizzle depends on row bits the step does not touch), so one
// lane offset plus a wave-uniform row step addresses every instruction (1 VGPR instead of NI).
template <typename T, int D, int ROWS, int NWV = 4>
struct GStage {
  static constexpr int CH = D / 8;
  static constexpr int NI = ROWS * CH / (NWV * 64);
  static constexpr int RSTEP = NWV * 1024 / (D * 16) * 8;
  static_assert(NI * NWV * 64 == ROWS * CH, "tile must split evenly over the block");
  static_assert(RSTEP % 16 == 0, "row step must keep the swizzle");
  int off0;  // element offset of this lane's first source chunk relative to the tile's first row
  long step;  // elements between consecutive instructions' source rows (RSTEP rows)
  __device__ __forceinline__ void init(long ld) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int row, ch;
    lay_inverse<D>((wid * 64 + lane) * 16, row, ch);
    off0 = row * (int)ld + ch * 8;
    step = (long)RSTEP * ld;
  }
  __device__ __forceinline__ void issue(const T* g, T* tile) const {
    const int wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g + i * step + off0),
                                       (__attribute__((address_space(3))) void*)(tile + (i * NWV + wid) * 512), 16, 0,
                                       0);
  }
};

// C-layout row of register r for lane half h (32x32 accumulator)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Lane-constant LDS byte offsets of the MFMA operand reads (image above). For a row base r0 that
// is a multiple of 16, everything else is a compile-time immediate on the ds_read.
template <typename T, int D>
struct LaneOff {
  int re, ro;  // ds_read_b128 of row l32, chunk 2*ks + h2: even / odd ks
  int tl, th;  // ds_read_b64_tr_b16 blocks (rows +0..7 / +8..15) of the transposed 32x16 operand
  __device__ __forceinline__ void init(int lane) {
    const int l32 = lane & 31, h2 = lane >> 5;
    re = lay_byte<D>(l32, h2);
    ro = lay_byte<D>(l32, 2 + h2);
    // group g = lane/16, lane 4q+p of the group supplies row 4(g>>1)+q, columns 16(g&1)+4p..+3
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int r = 4 * (g >> 1) + q, ch = 2 * (g & 1) + (p >> 1);
    tl = lay_byte<D>(r, ch) + 8 * (p & 1);
    th = lay_byte<D>(r + 8, ch) + 8 * (p & 1);
  }
  // transposed operand: rows [r0, r0+16) (r0 % 16 == 0), columns [32 db, 32 db + 32)
  __device__ __forceinline__ V8<T> tr(const T* tile, int r0, int db) const {
    const i16x4 lo = tr4(tile, r0 * 2 * D + 512 * db + tl);
    const i16x4 hi = tr4(tile, r0 * 2 * D + 512 * db + th);
    return __builtin_bit_cast(V8<T>, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
  // row operand: rows [r0, r0+32) (r0 % 16 == 0), k-step ks (columns 16 ks .. 16 ks + 15)
  __device__ __forceinline__ V8<T> rowk(const T* tile, int r0, int ks) const {
    return lds_read16(tile, r0 * 2 * D + 512 * (ks >> 1) + ((ks & 1) ? ro : re));
  }
};

template <int N>
using IC = std::integral_constant<int, N>;

}  // namespace attn
}  // namespace pra

// Memory-bound elementwise kernels: RoPE (in place on the fused QKV activation), SwiGLU
// forward/backward, embedding gather + deterministic embedding backward.
//
// All kernels move 8 elements (16 B for bf16) per lane and use grid-stride loops capped at
// 256 CUs x 8 blocks, per the CDNA4 memory-bound recipe.
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace pra {

static inline int grid_for(size_t work_items, int block = 256) {
  size_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// ----------------------------------------------------------------------------------------
// RoPE, interleaved-pair convention of the reference (model.py:101-127): the pair
// (x[2i], x[2i+1]) is multiplied by cis(pos * freq_i) in fp32 and rounded back.
// x points at the first rotated column of token 0; `ld` is the token row stride; the first
// `ncols` columns of each row (q heads followed by k heads, head_dim D each) are rotated.
// tab is float2[S][D/2] = (cos, sin). sign = -1 applies the inverse rotation (backward).
// (a + ib) * (c + is) with the FMA placement spelled out, so every RoPE kernel (row-major,
// transposing, register-tile) rounds identically whatever the compiler's contraction choices.
__device__ __forceinline__ void rot_pair(float a, float b, float c, float s, float& o0, float& o1) {
  o0 = __builtin_fmaf(a, c, -(b * s));
  o1 = __builtin_fmaf(a, s, b * c);
}

template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(T* __restrict__ x, const float2* __restrict__ tab,
                                                   long ntok, int ld, int ncols, int D, int S,
                                                   int pos_offset, float sign) {
  const int vpr = ncols / 8;  // 8-element vectors per row
  const long total = ntok * vpr;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const long t = idx / vpr;
    const int col = (int)(idx - t * vpr) * 8;
    const int pos = (int)(t % S) + pos_offset;
    const int pi = (col % D) / 2;  // first pair index
    T* p = x + t * (long)ld + col;
    float v[8];
    load8<T>(p, v);
    const float4* tp = reinterpret_cast<const float4*>(tab + (size_t)pos * (D / 2) + pi);
    float4 cs01 = tp[0], cs23 = tp[1];
    float c[4] = {cs01.x, cs01.z, cs23.x, cs23.z};
    float s[4] = {cs01.y * sign, cs01.w * sign, cs23.y * sign, cs23.w * sign};
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = v[2 * k], b = v[2 * k + 1];
      rot_pair(a, b, c[k], s[k], o[2 * k], o[2 * k + 1]);
    }
    store8<T>(p, o);
  }
}

// ----------------------------------------------------------------------------------------
// SwiGLU (reference model.py:268-269, `w2(silu(w1 x) * w3 x)`), with the reference's bf16
// rounding points: a = round(silu(g)), y = round(a * u).
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ g, const T* __restrict__ u,
                                                         T* __restrict__ y, long ntok, int F, int ldg,
                                                         int ldu, int ldy) {
  const int vpr = F / 8;
  const long total = ntok * vpr;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const long t = idx / vpr;
    const int col = (int)(idx - t * vpr) * 8;
    float gv[8], uv[8], o[8];
    load8<T>(g + t * ldg + col, gv);
    load8<T>(u + t * ldu + col, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rnd<T>(silu_f(gv[j])) * uv[j];
    store8<T>(y + t * ldy + col, o);
  }
}

// dg = silu'(g) * round(dy * u), du = round(dy * round(silu(g)))
template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* g, const T* u,
                                                         T* dg, T* du, long ntok, int F, int ldg, int ldu,
                                                         int lddy) {
  const int vpr = F / 8;
  const long total = ntok * vpr;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const long t = idx / vpr;
    const int col = (int)(idx - t * vpr) * 8;
    float gv[8], uv[8], dv[8], og[8], ou[8];
    load8<T>(g + t * ldg + col, gv);
    load8<T>(u + t * ldu + col, uv);
    load8<T>(dy + t * lddy + col, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-gv[j]));
      const float a = rnd<T>(gv[j] * sg);
      const float da = rnd<T>(dv[j] * uv[j]);
      ou[j] = dv[j] * a;
      og[j] = da * sg * (1.f + gv[j] * (1.f - sg));
    }
    store8<T>(dg + t * ldg + col, og);
    store8<T>(du + t * ldu + col, ou);
  }
}

// Same op with every load of a lane issued before its first store: dg/du alias g/u (in-place
// backward), so in the grid-stride loop above the compiler may not move a row's loads above an
// earlier row's stores and each lane has only 3 x 16 B in flight. Block = 16 R tokens x 128 columns
// (2-D grid: no 64-bit index division); lane = one 16-B column chunk of tokens r, r + 16, ...
template <typename T>
struct Raw8 {  // 8 packed elements (16 B for 16-bit types, 32 B for fp32) held while loads are in flight
  uint4 w[sizeof(T) / 2];
};
template <typename T>
__device__ __forceinline__ Raw8<T> ld_raw8(const T* p) {
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.w[i] = reinterpret_cast<const uint4*>(p)[i];
  return r;
}

template <typename T, int R>
__global__ __launch_bounds__(256) void swiglu_bwd_tile_kernel(const T* dy, const T* g, const T* u, T* dg, T* du,
                                                              long ntok, int F, int ldg, int ldu, int lddy) {
  const int col = blockIdx.x * 128 + (threadIdx.x & 15) * 8;
  if (col >= F) return;
  const long t0 = (long)blockIdx.y * (16 * R) + (threadIdx.x >> 4);
  Raw8<T> G[R], U[R], DY[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const long t = t0 + 16 * i;
    if (t < ntok) {
      G[i] = ld_raw8(g + t * ldg + col);
      U[i] = ld_raw8(u + t * ldu + col);
      DY[i] = ld_raw8(dy + t * lddy + col);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const long t = t0 + 16 * i;
    if (t >= ntok) continue;
    float gv[8], uv[8], dv[8], og[8], ou[8];
    load8<T>(reinterpret_cast<const T*>(&G[i]), gv);
    load8<T>(reinterpret_cast<const T*>(&U[i]), uv);
    load8<T>(reinterpret_cast<const T*>(&DY[i]), dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // identical math / rounding to swiglu_bwd_kernel
      const float sg = 1.f / (1.f + __expf(-gv[j]));
      const float a = rnd<T>(gv[j] * sg);
      const float da = rnd<T>(dv[j] * uv[j]);
      ou[j] = dv[j] * a;
      og[j] = da * sg * (1.f + gv[j] * (1.f - sg));
    }
    store8<T>(dg + t * ldg + col, og);
    store8<T>(du + t * ldu + col, ou);
  }
}

// ----------------------------------------------------------------------------------------
// Embedding gather: out[t] = W[ids[t]]; one wave per token.
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const T* __restrict__ W,
                                                        T* __restrict__ out, long ntok, int D, long V) {
  const int lane = threadIdx.x & 63;
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  long id = ids[t];
  if (id < 0 || id >= V) id = 0;  // out-of-range ids are a caller bug; never read out of bounds
  const T* src = W + id * (long)D;
  T* dst = out + t * (long)D;
  for (int c = lane * 8; c < D; c += 512) {
    float v[8];
    load8<T>(src + c, v);
    store8<T>(dst + c, v);
  }
}

// Deterministic embedding backward over ids sorted (stably) ascending: the wave that owns a
// segment start sums the segment's dout rows in sorted (= original token) order.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                        const int64_t* __restrict__ perm, const T* __restrict__ dout,
                                                        T* __restrict__ dW, long ntok, int D, long V,
                                                        int accumulate) {
  const int lane = threadIdx.x & 63;
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= ntok) return;
  const long v = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == v) return;
  if (v < 0 || v >= V) return;
  long end = i + 1;
  while (end < ntok && sorted_ids[end] == v) ++end;
  for (int c = lane * 8; c < D; c += 512) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (accumulate) load8<T>(dW + v * (long)D + c, acc);
    for (long j = i; j < end; ++j) {
      float r[8];
      load8<T>(dout + perm[j] * (long)D + c, r);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += r[k];
    }
    store8<T>(dW + v * (long)D + c, acc);
  }
}

// ---------------------------------------------------------------------------------------
// 2-D transpose of a 16-bit [R, C] matrix into [C, R] (R, C multiples of 64, 16-B aligned rows;
// host-checked): one wave moves a 64x64 tile with no LDS and no barrier. Lane
// (g = lane & 7, ch = lane >> 3) loads the 8x8 sub-block rows 8g..8g+7, cols 8ch..8ch+7 as
// eight 16-B loads (each instruction: 8 rows x 128 contiguous bytes), transposes it in VGPRs
// with 32 v_perm_b32, and writes eight 16-B stores (each instruction: 8 output rows x 128 B).
// 128 B in flight per lane and no LDS bank conflicts (an LDS-tiled version read its tile
// column-wise with 8-way conflicts, which capped it near HBM rate even in isolation).
__device__ __forceinline__ void transpose8x8_b16(const uint4 (&in)[8], uint4 (&out)[8]) {
  const uint32_t* a = reinterpret_cast<const uint32_t*>(in);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const uint32_t sel = (m & 1) ? 0x07060302u : 0x05040100u;  // hi halves / lo halves
#pragma unroll
    for (int e = 0; e < 4; ++e)  // out row m, dword e = (in row 2e, in row 2e+1) at column m
      o[m * 4 + e] = __builtin_amdgcn_perm(a[(2 * e + 1) * 4 + (m >> 1)], a[(2 * e) * 4 + (m >> 1)], sel);
  }
}

__global__ __launch_bounds__(256) void transpose_reg_kernel(const uint16_t* __restrict__ src,
                                                            uint16_t* __restrict__ dst, long ld_src,
                                                            long ld_dst, int tiles_c, long n_tiles) {
  const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= n_tiles) return;
  const long r0 = (tile / tiles_c) * 64, c0 = (tile % tiles_c) * 64;
  const int lane = threadIdx.x & 63, g = lane & 7, ch = lane >> 3;
  const uint16_t* s = src + (r0 + 8 * g) * ld_src + c0 + 8 * ch;
  uint4 in[8], out[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) in[k] = *reinterpret_cast<const uint4*>(s + k * ld_src);
  transpose8x8_b16(in, out);
  uint16_t* d = dst + (c0 + 8 * ch) * ld_dst + r0 + 8 * g;
#pragma unroll
  for (int m = 0; m < 8; ++m) *reinterpret_cast<uint4*>(d + m * ld_dst) = out[m];
}

// ---------------------------------------------------------------------------------------
// Transposing epilogues. The weight-gradient GEMM wants dY^T (K = tokens contiguous, see
// transpose_kernel); the two producers of the largest dY's write it directly, in the same pass
// that writes the row-major result (needed by the data-gradient GEMM):
//   swiglu_bwd_t: dgu = [dg | du] (in place over gu) and dguT = dgu^T        (W1|W3 weight grad)
//   rope_t:       x = inverse-RoPE(x) on the q|k columns (in place), xT = x^T (QKV weight grad)
// Block = 64 tokens x 64 columns; values go through an LDS tile to 16-B transposed stores. The
// tile's 16-B chunks are XOR-swizzled by (row >> 3) so the column-wise reads are conflict-free.
__device__ __forceinline__ void store_tile_t(uint16_t (*tile)[72], uint16_t* dst, long ld_dst, long c0, long t0) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + 256 * i, rg = idx & 7, c = idx >> 3;
    const int pc = (((c >> 3) ^ rg) << 3) | (c & 7);  // swizzled column (rows rg*8.. have r >> 3 == rg)
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[rg * 8 + 2 * j][pc] | ((uint32_t)tile[rg * 8 + 2 * j + 1][pc] << 16);
    *reinterpret_cast<uint4*>(dst + (c0 + c) * ld_dst + t0 + rg * 8) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__device__ __forceinline__ int swz(int r, int ch) { return ch ^ ((r >> 3) & 7); }

template <typename T>
__device__ __forceinline__ void unpack8(const uint4& w, float (&o)[8]) {
  const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = to_f<T>(e[j]);
}

template <typename T>
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  T tmp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) tmp[j] = from_f<T>(v[j]);
  return *reinterpret_cast<const uint4*>(tmp);
}

// swiglu_bwd_t: dgu = [dg | du] in place over gu and dguT = dgu^T, same math and rounding as
// swiglu_bwd_kernel. gu is updated in place, so it cannot be __restrict__ and the compiler may not
// move a later row's loads of gu above an earlier row's stores: every load of the block's NT 64x64
// tiles is issued before the first store (NT = 2: 6 x 16 B x 2 in flight per lane, each row 256
// contiguous bytes per operand; ~10% faster than the register-tile form, which loses occupancy).
template <typename T, int NT>
__global__ __launch_bounds__(256) void swiglu_bwd_t_hoist_kernel(const T* __restrict__ dy, T* gu,
                                                                 T* __restrict__ guT, int F, int ldgu, int lddy,
                                                                 long ntok) {
  __shared__ __attribute__((aligned(16))) uint16_t tg[NT][64][72], tu[NT][64][72];
  constexpr int CPR = 8 * NT;  // 16-B chunks per tile row
  constexpr int IT = 2 * NT;   // rows x chunks per lane
  const long t0 = (long)blockIdx.y * 64;
  const int c0 = blockIdx.x * 64 * NT;
  uint4 G[IT], U[IT], DY[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int idx = threadIdx.x + 256 * i, r = idx / CPR, cc = idx % CPR;
    const long t = t0 + r;
    const int col = c0 + cc * 8;
    G[i] = *reinterpret_cast<const uint4*>(gu + t * ldgu + col);
    U[i] = *reinterpret_cast<const uint4*>(gu + t * ldgu + F + col);
    DY[i] = *reinterpret_cast<const uint4*>(dy + t * lddy + col);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int idx = threadIdx.x + 256 * i, r = idx / CPR, cc = idx % CPR;
    const long t = t0 + r;
    const int col = c0 + cc * 8;
    float gv[8], uv[8], dv[8], og[8], ou[8];
    unpack8<T>(G[i], gv);
    unpack8<T>(U[i], uv);
    unpack8<T>(DY[i], dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // identical math / rounding to swiglu_bwd_kernel
      const float sg = 1.f / (1.f + __expf(-gv[j]));
      const float a = rnd<T>(gv[j] * sg);
      const float da = rnd<T>(dv[j] * uv[j]);
      ou[j] = dv[j] * a;
      og[j] = da * sg * (1.f + gv[j] * (1.f - sg));
    }
    const uint4 pg = pack8<T>(og), pu = pack8<T>(ou);
    *reinterpret_cast<uint4*>(gu + t * ldgu + col) = pg;
    *reinterpret_cast<uint4*>(gu + t * ldgu + F + col) = pu;
    const int tl = cc / 8, ch = cc % 8;
    *reinterpret_cast<uint4*>(&tg[tl][r][swz(r, ch) * 8]) = pg;
    *reinterpret_cast<uint4*>(&tu[tl][r][swz(r, ch) * 8]) = pu;
  }
  __syncthreads();
#pragma unroll
  for (int tl = 0; tl < NT; ++tl) {
    store_tile_t(tg[tl], reinterpret_cast<uint16_t*>(guT), ntok, c0 + 64 * tl, t0);
    store_tile_t(tu[tl], reinterpret_cast<uint16_t*>(guT), ntok, F + c0 + 64 * tl, t0);
  }
}

// ---------------------------------------------------------------------------------------
// Register-tile transposing epilogues (swiglu_fwd_t, rope_t): one wave per 64-token x 64-column tile, lane (g, ch) owns tokens 8g..8g+7 x columns 8ch..8ch+7, so its eight row
// vectors are the 8x8 block the transposed store needs (transpose8x8_b16). No LDS, no barrier,
// every operand's eight row loads issued before any math. Same math and rounding as above.
// tile of this wave (tiles_c column tiles per 64-token row of tiles); false past the end
__device__ __forceinline__ bool wave_tile(int tiles_c, long n_tiles, long& t0, int& c0, int& g, int& ch) {
  const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= n_tiles) return false;
  t0 = (tile / tiles_c) * 64;
  c0 = (int)(tile % tiles_c) * 64;
  g = threadIdx.x & 7;
  ch = (threadIdx.x >> 3) & 7;
  return true;
}

__device__ __forceinline__ void store_t_reg(const uint4 (&rows)[8], uint16_t* dst, long ld_dst, long c0, long t0,
                                            int g, int ch) {
  uint4 out[8];
  transpose8x8_b16(rows, out);
  uint16_t* d = dst + (c0 + 8 * ch) * ld_dst + t0 + 8 * g;
#pragma unroll
  for (int m = 0; m < 8; ++m) *reinterpret_cast<uint4*>(d + m * ld_dst) = out[m];
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_t_reg_kernel(const T* __restrict__ gu, T* __restrict__ a,
                                                               T* __restrict__ aT, int F, int ldgu, int lda,
                                                               long ntok, long n_tiles) {
  long t0;
  int c0, g, ch;
  if (!wave_tile(F / 64, n_tiles, t0, c0, g, ch)) return;
  const int col = c0 + 8 * ch;
  uint4 G[8], U[8], A[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const T* row = gu + (t0 + 8 * g + k) * ldgu + col;
    G[k] = *reinterpret_cast<const uint4*>(row);
    U[k] = *reinterpret_cast<const uint4*>(row + F);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float gv[8], uv[8], o[8];
    unpack8<T>(G[k], gv);
    unpack8<T>(U[k], uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rnd<T>(silu_f(gv[j])) * uv[j];
    A[k] = pack8<T>(o);
    *reinterpret_cast<uint4*>(a + (t0 + 8 * g + k) * lda + col) = A[k];
  }
  store_t_reg(A, reinterpret_cast<uint16_t*>(aT), ntok, c0, t0, g, ch);
}

template <typename T>
__global__ __launch_bounds__(256) void rope_t_reg_kernel(T* x, T* __restrict__ xT, const float2* __restrict__ tab,
                                                         int ld, int ncols, int nrot, int D, int S, float sign,
                                                         long ntok, long n_tiles) {
  long t0;
  int c0, g, ch;
  if (!wave_tile(ncols / 64, n_tiles, t0, c0, g, ch)) return;
  const int col = c0 + 8 * ch;
  uint4 X[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) X[k] = *reinterpret_cast<const uint4*>(x + (t0 + 8 * g + k) * ld + col);
  if (col < nrot) {  // same math as rope_kernel
    const int pi = (col % D) / 2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long t = t0 + 8 * g + k;
      const float4* tp = reinterpret_cast<const float4*>(tab + (size_t)(t % S) * (D / 2) + pi);
      const float4 cs01 = tp[0], cs23 = tp[1];
      const float c[4] = {cs01.x, cs01.z, cs23.x, cs23.z};
      const float sn[4] = {cs01.y * sign, cs01.w * sign, cs23.y * sign, cs23.w * sign};
      float v[8], o[8];
      unpack8<T>(X[k], v);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        rot_pair(v[2 * q], v[2 * q + 1], c[q], sn[q], o[2 * q], o[2 * q + 1]);
      }
      X[k] = pack8<T>(o);
      *reinterpret_cast<uint4*>(x + t * ld + col) = X[k];
    }
  }
  store_t_reg(X, reinterpret_cast<uint16_t*>(xT), ntok, c0, t0, g, ch);
}

}  // namespace pra

extern "C" {

hipError_t pra_rope(int dtype, void* x, const void* tab, long ntok, int ld, int ncols, int D, int S,
                    int pos_offset, int inverse, hipStream_t s) {
  if (ncols % 8 || D % 8 || ld % 8) return hipErrorInvalidValue;
  const int grid = pra::grid_for((size_t)ntok * (ncols / 8));
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::rope_kernel<T>), dim3(grid), dim3(256), 0, s, (T*)x,
                                        (const float2*)tab, ntok, ld, ncols, D, S, pos_offset,
                                        inverse ? -1.f : 1.f));
  return hipGetLastError();
}

hipError_t pra_swiglu_fwd(int dtype, const void* g, const void* u, void* y, long ntok, int F, int ldg,
                          int ldu, int ldy, hipStream_t s) {
  if (F % 8 || ldg % 8 || ldu % 8 || ldy % 8) return hipErrorInvalidValue;
  const int grid = pra::grid_for((size_t)ntok * (F / 8));
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::swiglu_fwd_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)g,
                                        (const T*)u, (T*)y, ntok, F, ldg, ldu, ldy));
  return hipGetLastError();
}

// variant (A/B): 0 = grid-stride kernel, 1 / -1 = hoisted tile kernel, 4 tokens per lane, 2 = 8 per lane
hipError_t pra_swiglu_bwd(int dtype, const void* dy, const void* g, const void* u, void* dg, void* du,
                          long ntok, int F, int ldg, int ldu, int lddy, int variant, hipStream_t s) {
  if (F % 8 || ldg % 8 || ldu % 8 || lddy % 8) return hipErrorInvalidValue;
  if (variant == 0) {
    const int grid = pra::grid_for((size_t)ntok * (F / 8));
    PRA_DISPATCH_FLOAT(dtype, T,
                       hipLaunchKernelGGL((pra::swiglu_bwd_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)dy,
                                          (const T*)g, (const T*)u, (T*)dg, (T*)du, ntok, F, ldg, ldu, lddy));
  } else if (variant == 2) {
    const dim3 grid((unsigned)((F + 127) / 128), (unsigned)((ntok + 127) / 128));
    PRA_DISPATCH_FLOAT(dtype, T,
                       hipLaunchKernelGGL((pra::swiglu_bwd_tile_kernel<T, 8>), grid, dim3(256), 0, s, (const T*)dy,
                                          (const T*)g, (const T*)u, (T*)dg, (T*)du, ntok, F, ldg, ldu, lddy));
  } else {
    const dim3 grid((unsigned)((F + 127) / 128), (unsigned)((ntok + 63) / 64));
    PRA_DISPATCH_FLOAT(dtype, T,
                       hipLaunchKernelGGL((pra::swiglu_bwd_tile_kernel<T, 4>), grid, dim3(256), 0, s, (const T*)dy,
                                          (const T*)g, (const T*)u, (T*)dg, (T*)du, ntok, F, ldg, ldu, lddy));
  }
  return hipGetLastError();
}

hipError_t pra_embedding_fwd(int dtype, const int64_t* ids, const void* W, void* out, long ntok, int D, long V,
                             hipStream_t s) {
  if (D % 8) return hipErrorInvalidValue;
  const int grid = (int)((ntok + 3) / 4);
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::embed_fwd_kernel<T>), dim3(grid), dim3(256), 0, s, ids, (const T*)W,
                                        (T*)out, ntok, D, V));
  return hipGetLastError();
}

hipError_t pra_embedding_bwd(int dtype, const int64_t* sorted_ids, const int64_t* perm, const void* dout,
                             void* dW, long ntok, int D, long V, int accumulate, hipStream_t s) {
  if (D % 8) return hipErrorInvalidValue;
  const int grid = (int)((ntok + 3) / 4);
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::embed_bwd_kernel<T>), dim3(grid), dim3(256), 0, s, sorted_ids, perm,
                                        (const T*)dout, (T*)dW, ntok, D, V, accumulate));
  return hipGetLastError();
}

hipError_t pra_transpose16(const void* src, void* dst, long R, long C, long ld_src, long ld_dst, hipStream_t s) {
  if (R % 64 || C % 64 || ld_src % 8 || ld_dst % 8) return hipErrorInvalidValue;
  const long n_tiles = (R / 64) * (C / 64);
  hipLaunchKernelGGL(pra::transpose_reg_kernel, dim3((unsigned)((n_tiles + 3) / 4)), dim3(256), 0, s,
                     (const uint16_t*)src, (uint16_t*)dst, ld_src, ld_dst, (int)(C / 64), n_tiles);
  return hipGetLastError();
}

// a = swiglu(gu) [ntok, F] (ld lda) and aT = a^T [F, ntok]; ntok, F multiples of 64.
hipError_t pra_swiglu_fwd_t(int dtype, const void* gu, void* a, void* aT, long ntok, int F, int ldgu, int lda,
                            hipStream_t s) {
  if (ntok % 64 || F % 64 || ldgu % 8 || lda % 8) return hipErrorInvalidValue;
  const long n_tiles = (ntok / 64) * (F / 64);
  PRA_DISPATCH_16BIT(dtype, T,
                     hipLaunchKernelGGL((pra::swiglu_fwd_t_reg_kernel<T>), dim3((unsigned)((n_tiles + 3) / 4)),
                                        dim3(256), 0, s, (const T*)gu, (T*)a, (T*)aT, F, ldgu, lda, ntok, n_tiles));
  return hipGetLastError();
}

// dgu = [dg | du] in place over gu [ntok, 2F] (ld ldgu) and guT [2F, ntok]; ntok, F multiples of 64.
hipError_t pra_swiglu_bwd_t(int dtype, const void* dy, void* gu, void* guT, long ntok, int F, int ldgu, int lddy,
                            hipStream_t s) {
  if (ntok % 64 || F % 64 || ldgu % 8 || lddy % 8) return hipErrorInvalidValue;
  if (F % 128 == 0) {
    dim3 grid((unsigned)(F / 128), (unsigned)(ntok / 64));
    PRA_DISPATCH_16BIT(dtype, T,
                       hipLaunchKernelGGL((pra::swiglu_bwd_t_hoist_kernel<T, 2>), grid, dim3(256), 0, s, (const T*)dy,
                                          (T*)gu, (T*)guT, F, ldgu, lddy, ntok));
  } else {
    dim3 grid((unsigned)(F / 64), (unsigned)(ntok / 64));
    PRA_DISPATCH_16BIT(dtype, T,
                       hipLaunchKernelGGL((pra::swiglu_bwd_t_hoist_kernel<T, 1>), grid, dim3(256), 0, s, (const T*)dy,
                                          (T*)gu, (T*)guT, F, ldgu, lddy, ntok));
  }
  return hipGetLastError();
}

// x [ntok, ncols] (ld): RoPE (inverse if `inverse`) on columns [0, nrot), in place; xT = x^T.
hipError_t pra_rope_t(int dtype, void* x, void* xT, const void* tab, long ntok, int ld, int ncols, int nrot, int D,
                      int S, int inverse, hipStream_t s) {
  if (ntok % 64 || ncols % 64 || nrot % 8 || D % 8 || ld % 8) return hipErrorInvalidValue;
  const long n_tiles = (ntok / 64) * (ncols / 64);
  PRA_DISPATCH_16BIT(dtype, T,
                     hipLaunchKernelGGL((pra::rope_t_reg_kernel<T>), dim3((unsigned)((n_tiles + 3) / 4)), dim3(256), 0,
                                        s, (T*)x, (T*)xT, (const float2*)tab, ld, ncols, nrot, D, S,
                                        inverse ? -1.f : 1.f, ntok, n_tiles));
  return hipGetLastError();
}

}  // extern "C"

// Weight-gradient GEMM for gfx950 (CDNA4) on row-major activations:
//
//     C[M][N] (+)= sum_k A[k][m] * B[k][n]        (dW = dY^T X, K = tokens)
//
// A = dY [K, M] and B = X [K, N] are the activations exactly as the forward/backward produce them
// (row-major, token rows). For this contraction both operands are "K-slow": consecutive k are a
// row stride apart. hipBLASLt runs that layout ~25-30% slower than K-contiguous operands, which is
// why the default path transposes dY and X first (transpose_reg_kernel + transposing epilogues,
// ops/fused.py _wgrad_into). Here the transpose happens inside the LDS read instead:
//
//  * tiles of BK = 32 token rows x 256 columns are staged global -> LDS by LDS-DMA
//    (global_load_lds_dwordx4, no VGPR round trip) into a sub-tiled XOR-swizzled image; a ring of
//    4 stages keeps 3 in flight across the barriers (counted vmcnt, raw s_barrier);
//  * MFMA operands (32 columns x 16 k) come from ds_read_b64_tr_b16, the gfx950 transposing LDS
//    read, so K-slow data feeds v_mfma_f32_32x32x16_bf16 directly;
//  * block tile 256 x 256, 4 waves of 128 x 128 (16 accumulators of 32 x 32 each);
//  * XCD-aware tile order: the round-robin placement of consecutive workgroups over the 8 XCDs is
//    undone, and each XCD walks its tiles in groups of 8 M-tiles, so the 32 workgroups resident on
//    one XCD share 8 A and ~4 B column panels in its L2;
//  * epilogue: v_permlane32_swap pairs lane halves so each lane writes 16 contiguous bytes; the
//    accumulate mode (gradient accumulation) adds the existing C in fp32 and rounds once, like
//    addmm's beta = 1.
//
// Deterministic (fixed summation order), so resumed runs stay bit-identical.
// Requires M % 256 == 0, N % 256 == 0, K % 32 == 0, 16-B aligned rows (host-checked).
#include "common.h"

#include <stdlib.h>

#include <type_traits>

namespace pra {
namespace wg {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <typename T> struct Elem;
template <> struct Elem<__bf16> { typedef bf16x8 v8; };
template <> struct Elem<_Float16> { typedef f16x8 v8; };
template <typename T>
using V8 = typename Elem<T>::v8;

constexpr int BM = 256, BN = 256, BK = 32, TD = 256, NTH = 256, NS = 4;

constexpr int TILE = BK * TD;                 // elements per staged operand tile (16 KiB)
constexpr int NI = TILE * 2 / (NTH * 16);     // LDS-DMA instructions per lane per operand tile (4)

// LDS image of a [BK][TD] tile: 8-row x 32-column sub-tiles of 512 B, the four 16-B chunks of each
// 64-B sub-tile row XOR-swizzled by (row >> 2) & 3. One ds_read_b64_tr_b16 reads exactly one
// 512-B sub-tile (8 k rows x 32 columns), so it is conflict-free.
__device__ __forceinline__ int lay_byte(int r, int ch) {
  return (TD * 16) * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}
__device__ __forceinline__ void lay_inverse(int o, int& r, int& ch) {
  const int rg = o / (TD * 16), rem = o % (TD * 16);
  const int sub = rem / 512, r7 = (rem % 512) / 64, slot = (rem % 64) / 16;
  r = 8 * rg + r7;
  ch = 4 * sub + (slot ^ ((r >> 2) & 3));
}

template <typename T>
__device__ __forceinline__ i16x4 tr4(const T* tile, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(reinterpret_cast<const char*>(tile) + byte_off));
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ uint32_t pack_x2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (T)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (T)b) << 16);
}

template <int N>
using IC = std::integral_constant<int, N>;

// the same with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit byte offset ("saddr"
// form): no per-instruction 64-bit VALU address add
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

// s_waitcnt vmcnt(N) for a compile-time N
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N == 0 || N == 8 || N == 16 || N == 24 || N == 32, "add the count");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
}

// one 16-B-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at LDS byte
// lds + 16 l (M0 = wave-uniform LDS base; one wait state between the M0 write and the load).
// M0 is not declared clobbered (the compiler reserves it and warns): nothing in this kernel
// reads M0 (gfx950 ds_* instructions do not use it).
__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory");
}

template <typename T, bool ACC>
__global__ __launch_bounds__(NTH) void wgrad_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                    T* __restrict__ C, int M, int N, int K, long lda, long ldb,
                                                    long ldc) {
  // NS stages x (A tile, B tile), 128 KiB. The LDS-DMA is issued from inline asm (dma16): the
  // compiler does not see it as an LDS write, so it neither drains it with vmcnt(0) before every
  // fragment read nor at barriers; ordering is the counted vmcnt + s_barrier below.
  __shared__ __attribute__((aligned(1024))) T smem[NS * 2 * TILE];

  // ---- tile of this workgroup: undo the XCD round robin, then group-M order -------------------
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  int wgid;
  {
    const int orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, r = nwg % 8;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  constexpr int GM = 8;
  const int group = wgid / (GM * tiles_n), first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (wgid % (GM * tiles_n)) % gsz;
  const int tn = (wgid % (GM * tiles_n)) / gsz;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;  // 2 x 2 waves of 128 x 128

  // ---- LDS-DMA source offsets: instruction i of wave w fills image bytes [(4i + w) KiB, +1 KiB) --
  int offa[NI], offb[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    int r, ch;
    lay_inverse(((i * 4 + wid) * 64 + lane) * 16, r, ch);
    offa[i] = r * (int)lda + ch * 8;
    offb[i] = r * (int)ldb + ch * 8;
  }
  const T* Ab = A + m0;
  const T* Bb = B + n0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)smem;
  // all 2 NI DMA instructions of stage kt into ring slot s
  auto issue = [&](int s, int kt) {
    const T* ga = Ab + (long)kt * BK * lda;
    const T* gb = Bb + (long)kt * BK * ldb;
    const uint32_t la = lds0 + (uint32_t)(s * 2 * TILE) * sizeof(T), lb = la + TILE * sizeof(T);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      dma16(ga + offa[i], __builtin_amdgcn_readfirstlane(la + (i * 4 + wid) * 1024));
      dma16(gb + offb[i], __builtin_amdgcn_readfirstlane(lb + (i * 4 + wid) * 1024));
    }
  };

  // ---- transposed operand reads: group g = lane / 16, lane 4q + p of the group supplies k row
  // 4 (g >> 1) + q, columns 16 (g & 1) + 4p .. + 3 (8 B); the hardware hands each lane 4 k values
  // of one column. Two reads (k rows +0..7 and +8..15) make the 32 x 16 operand.
  int tl, th;
  {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int r = 4 * (g >> 1) + q, ch = 2 * (g & 1) + (p >> 1);
    tl = lay_byte(r, ch) + 8 * (p & 1);
    th = lay_byte(r + 8, ch) + 8 * (p & 1);
  }
  auto frag = [&](const T* tile, int ks, int db) -> V8<T> {
    const int base = ks * 16 * 2 * TD + 512 * db;
    const i16x4 lo = tr4(tile, base + tl);
    const i16x4 hi = tr4(tile, base + th);
    return __builtin_bit_cast(V8<T>, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // D[n][m] = sum_k B[k][n] A[k][m]: the lane holds column m (= row of C), registers hold n, which
  // is the row-per-lane layout of the epilogue below.
  auto load_frags = [&](V8<T> (&fa)[4], V8<T> (&fb)[4], const T* ta, const T* tb, int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(ta, ks, wm * 4 + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag(tb, ks, wn * 4 + j);
  };

  const int nk = K / BK;
  // Every step issues exactly one stage of DMA (a stage past the end re-loads the last stage into
  // the slot nobody reads again), so the counted waits are the same on every step: at the barrier
  // of step kt the stage kt + 2 (8 instructions per lane) may stay in flight -> vmcnt(8).
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) issue(p, min(p, nk - 1));
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  V8<T> fa0[4], fb0[4], fa1[4], fb1[4];
  load_frags(fa0, fb0, smem, smem + TILE, 0);

  auto mma = [&](const V8<T> (&ca)[4], const V8<T> (&cb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(cb[j], ca[i], acc[i][j]);
  };
  auto interleave = [&](auto id_c) {  // MFMA, fragment read, MFMA, ...
    constexpr int id = decltype(id_c)::value;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, id);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, id);
    }
  };
  // step kt (ring slot s): k-step 0's MFMAs under the reads of k-step 1; then, mid-stage, the
  // counted wait + barrier that publish stage kt + 1 (and free stage kt - 1's slot for stage
  // kt + 3's DMA); k-step 1's MFMAs under the reads of stage kt + 1's first k-step. The MFMA pipe
  // still holds k-step 0's work while the wave waits at the barrier.
  auto step = [&](auto s_c, int kt) {
    constexpr int s = decltype(s_c)::value, sn = (s + 1) % NS;
    const T* ta = smem + s * 2 * TILE;
    const T* nta = smem + sn * 2 * TILE;
    load_frags(fa1, fb1, ta, ta + TILE, 1);
    mma(fa0, fb0);
    interleave(IC<0>{});
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue((s + NS - 1) % NS, min(kt + NS - 1, nk - 1));
    load_frags(fa0, fb0, nta, nta + TILE, 0);
    mma(fa1, fb1);
    interleave(IC<1>{});
  };
  for (int kt = 0; kt < nk; kt += NS) {
    step(IC<0>{}, kt);
    if (kt + 1 < nk) step(IC<1>{}, kt + 1);
    if (kt + 2 < nk) step(IC<2>{}, kt + 2);
    if (kt + 3 < nk) step(IC<3>{}, kt + 3);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends

  // ---- epilogue: row m = m0 + 128 wm + 32 i + l32; columns n0 + 128 wn + 32 j + crow(r, h2) ---
  const int l32 = lane & 31, h2 = lane >> 5;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    T* crow_p = C + (m0 + 128 * wm + 32 * i + l32) * ldc + n0 + 128 * wn;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        const int a = 8 * mm, c = 8 * mm + 4;  // registers of columns 16mm + 4h2 + 0..3 / 16mm + 8 + 4h2 + 0..3
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][c + q]),
                                                         __float_as_uint(acc[i][j][a + q]), false, false);
          v[q] = __uint_as_float(x[0]);
          v[4 + q] = __uint_as_float(x[1]);
        }
        // lane half h2 now holds the 8 contiguous columns 16mm + 8 (1 - h2) .. + 7
        T* p = crow_p + 32 * j + 16 * mm + 8 * (1 - h2);
        if constexpr (ACC) {
          const uint4 old = *reinterpret_cast<const uint4*>(p);
          const T* o = reinterpret_cast<const T*>(&old);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)o[e];
        }
        *reinterpret_cast<uint4*>(p) = make_uint4(pack_x2<T>(v[0], v[1]), pack_x2<T>(v[2], v[3]),
                                                  pack_x2<T>(v[4], v[5]), pack_x2<T>(v[6], v[7]));
      }
  }
}


// ---------------------------------------------------------------------------------------------
// The same GEMM on v_mfma_f32_16x16x32_bf16 (default): under load the chip holds a higher clock on
// the 16x16x32 shape than on 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH 'DVFS give-back'
// item 7). One 32-deep stage is one k-step; the wave's 128 x 128 tile is 8 x 8 accumulators of
// 16 x 16. Operand (16 columns x 32 k): 16-lane group g reads k rows 4g..4g+3 (lo) and
// 16+4g..16+4g+3 (hi) with ds_read_b64_tr_b16, so lane l of the group gets column l, k = {4g..4g+3,
// 16+4g..+3}; A and B use the same k permutation, so the dot products are unchanged.
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Work decomposition: tiles of 256 x 256 in group-M order (8 M-tiles per group). When the tile
// count is not a multiple of the CU count, the R tiles of the partial last round are split S ways
// over K (the launcher picks S so the split units fill whole rounds best): grid = (nwg - R) whole
// tiles + R * S split units, dispatched in that order. Each split unit writes its fp32 partial to
// ws and takes a ticket; the last arriver of a tile sums the S partials in part order (its own from
// ws too) -- deterministic, and nothing ever waits on another
// workgroup.
// NS16: ring depth (4 stages = 128 KiB, 5 = all 160 KiB of LDS)
template <typename T, bool ACC, int NS16>
__global__ __launch_bounds__(NTH) void wgrad16_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                      T* __restrict__ C, int M, int N, int K, long lda, long ldb,
                                                      long ldc, float* __restrict__ ws, int* __restrict__ tickets,
                                                      int n_split, int S) {
  __shared__ __attribute__((aligned(1024))) T smem[NS16 * 2 * TILE];
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n, nk = K / BK;
  // XCD-contiguous index of workgroup `orig` among n (undo the round-robin placement over the 8 XCDs)
  auto xcd_remap = [](int orig, int n) {
    const int xcd = orig % 8, q = n / 8, r = n % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  };
  constexpr int GM = 8;
  auto tile_origin = [&](int lin, long& m0, long& n0) __attribute__((always_inline)) {
    const int group = lin / (GM * tiles_n), first_m = group * GM;
    const int gsz = min(tiles_m - first_m, GM);
    m0 = (long)(first_m + (lin % (GM * tiles_n)) % gsz) * BM;
    n0 = (long)((lin % (GM * tiles_n)) / gsz) * BN;
  };

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  uint32_t offa[NI], offb[NI];  // per-lane byte offsets of the DMA sources within a stage
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    int r, ch;
    lay_inverse(((i * 4 + wid) * 64 + lane) * 16, r, ch);
    offa[i] = (uint32_t)((r * (int)lda + ch * 8) * (int)sizeof(T));
    offb[i] = (uint32_t)((r * (int)ldb + ch * 8) * (int)sizeof(T));
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)smem;
  const uint32_t ldsw = __builtin_amdgcn_readfirstlane(lds0 + wid * 1024);  // this wave's DMA base

  // lane offsets of the transposed reads: [column-block parity][lo/hi]
  int oa[2][2], ob[2][2];
  {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int ch = 2 * par + (p >> 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 16 * h + 4 * g + q;
        const int o = lay_byte(r, ch) + 8 * (p & 1);
        oa[par][h] = o + 512 * 4 * wm;  // wave's 128 columns = 4 sub-tiles of 32
        ob[par][h] = o + 512 * 4 * wn;
      }
    }
  }
  // 16-column block f (0..7) of the wave's 128 columns
  auto fragA = [&](const T* tile, int f) __attribute__((always_inline)) -> V8<T> {
    const i16x4 lo = tr4(tile, oa[f & 1][0] + 512 * (f >> 1));
    const i16x4 hi = tr4(tile, oa[f & 1][1] + 512 * (f >> 1));
    return __builtin_bit_cast(V8<T>, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto fragB = [&](const T* tile, int f) __attribute__((always_inline)) -> V8<T> {
    const i16x4 lo = tr4(tile, ob[f & 1][0] + 512 * (f >> 1));
    const i16x4 hi = tr4(tile, ob[f & 1][1] + 512 * (f >> 1));
    return __builtin_bit_cast(V8<T>, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x4 acc[8][8];
  V8<T> fa0[8], fb0[8], fa1[8], fb1[8];

  // acc = sum over the 32-deep stages [k0, k1) of tile (m0, n0)
  auto run = [&](long m0, long n0, int k0, int k1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* Ab = A + m0;
    const T* Bb = B + n0;
    // DMA instruction u (0..2NI-1) of stage kt into slot s: SGPR base + per-lane byte offset
    auto dma = [&](int s, int kt, int u) __attribute__((always_inline)) {
      const int i = u >> 1;
      const uint32_t lds = ldsw + (uint32_t)((s * 2 * TILE + (u & 1) * TILE) * sizeof(T) + i * 4 * 1024);
      const T* g = (u & 1) ? Bb + (long)kt * BK * ldb : Ab + (long)kt * BK * lda;
      dma16s(g, (u & 1) ? offb[i] : offa[i], lds);
    };
    // every step issues exactly one stage of DMA (a stage past k1 re-loads stage k1 - 1 into the
    // slot nobody reads again), so the counted waits are the same on every step
#pragma unroll
    for (int p = 0; p < NS16 - 1; ++p)
#pragma unroll
      for (int u = 0; u < 2 * NI; ++u) dma(p, min(k0 + p, k1 - 1), u);
    wait_vm<2 * NI * (NS16 - 2)>();  // stage k0 landed; the younger stages stay in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      fa0[f] = fragA(smem, f);
      fb0[f] = fragB(smem + TILE, f);
    }
    // step kt (slot s, fragments in ca/cb): m-blocks 0..3 (32 MFMAs); counted wait + barrier
    // publish stage kt + 1 and free the slot of stage kt - 1; m-blocks 4..7 in 8 groups of 4
    // MFMAs, each with 4 fragment reads of stage kt + 1 and one DMA instruction of stage kt + 3.
    auto step = [&](auto s_c, V8<T> (&ca)[8], V8<T> (&cb)[8], V8<T> (&na)[8], V8<T> (&nb)[8], int kt) {
      constexpr int s = decltype(s_c)::value % NS16, sn = (s + 1) % NS16, sd = (s + NS16 - 1) % NS16;
      const T* nta = smem + sn * 2 * TILE;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
      wait_vm<2 * NI * (NS16 - 3)>();  // stage kt + 1 landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int kd = min(kt + NS16 - 1, k1 - 1);
#pragma unroll
      for (int gi = 0; gi < 8; ++gi) {
        na[gi] = fragA(nta, gi);
        nb[gi] = fragB(nta + TILE, gi);
        const int i = 4 + (gi >> 1);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int j = 4 * (gi & 1) + jj;
          acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        dma(sd, kd, gi);
      }
    };
    // unrolled by lcm(NS16, 2): compile-time ring slot and fragment register set
    static_assert(NS16 == 4 || NS16 == 5, "unroll below");
    constexpr int UNR = NS16 == 4 ? 4 : 10;
    for (int kt = k0; kt < k1; kt += UNR) {
      auto st = [&](auto j_c) __attribute__((always_inline)) {
        constexpr int j = decltype(j_c)::value;
        if (kt + j < k1) {
          if constexpr (j % 2 == 0)
            step(IC<j>{}, fa0, fb0, fa1, fb1, kt + j);
          else
            step(IC<j>{}, fa1, fb1, fa0, fb0, kt + j);
        }
      };
      st(IC<0>{}); st(IC<1>{}); st(IC<2>{}); st(IC<3>{});
      if constexpr (UNR == 10) {
        st(IC<4>{}); st(IC<5>{}); st(IC<6>{}); st(IC<7>{}); st(IC<8>{}); st(IC<9>{});
      }
    }
    // no LDS-DMA may land after this point (next tile's prologue / end of the workgroup), and no
    // wave may still read a slot the next prologue overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  // epilogue: D[n][m] per 16 x 16 block: lane holds m = l & 15, n = 4 (l >> 4) + 0..3 (8 B)
  const int l16 = lane & 15, g4 = lane >> 4;
  auto store_c = [&](long m0, long n0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      T* rowp = C + (m0 + 128 * wm + 16 * i + l16) * ldc + n0 + 128 * wn + 4 * g4;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        T* p = rowp + 16 * j;
        if constexpr (ACC) {
          const uint2 old = *reinterpret_cast<const uint2*>(p);
          const T* o = reinterpret_cast<const T*>(&old);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)o[e];
        }
        *reinterpret_cast<uint2*>(p) = make_uint2(pack_x2<T>(v[0], v[1]), pack_x2<T>(v[2], v[3]));
      }
    }
  };
  const int ndp = nwg - n_split;  // whole tiles first, then n_split tiles x S split units
  const bool split = (int)blockIdx.x >= ndp;
  int lin, k0 = 0, k1 = nk, part = 0, st = 0;
  if (!split) {
    lin = xcd_remap(blockIdx.x, ndp);
  } else {
    // part-major, XCD-contiguous: the units resident together on one XCD are consecutive tiles
    // (group-M order) of the SAME K range, so they share A/B panel slices in L2 like the
    // data-parallel rounds (W13 at S = 2: 1.37 -> 1.40 PF over tile-major order)
    const int u = xcd_remap((int)blockIdx.x - ndp, n_split * S);
    part = u / n_split;
    st = u % n_split;
    lin = ndp + st;
    k0 = (int)((long)nk * part / S);
    k1 = (int)((long)nk * (part + 1) / S);
  }
  long m0, n0;
  tile_origin(lin, m0, n0);
  run(m0, n0, k0, k1);
  if (split) {
    // fp32 partial in register order (thread t's register r at r * NTH + t)
    float* w = ws + ((long)st * S + part) * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) w[((i * 8 + j) * 4 + e) * NTH + tid] = acc[i][j][e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);  // the one LDS array (free after run)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(tickets + st, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = ticket == S - 1;
      if (ticket == S - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!*last) return;
    // sum the S partials in part order (its own included, re-read from ws: same order whoever is last)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < S; ++p) {
      const float* wp = ws + ((long)st * S + p) * (BM * BN);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] += wp[((i * 8 + j) * 4 + e) * NTH + tid];
    }
  }
  store_c(m0, n0);
}

// zeroes the split tail's tickets (a kernel node, ordered before the GEMM in a captured graph)
__global__ __launch_bounds__(256) void zero_i32_kernel(int* __restrict__ p, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0;
}

}  // namespace wg
}  // namespace pra

extern "C" {

// C[M][N] (+)= A^T B with A [K][M] (row stride lda), B [K][N] (row stride ldb), C row stride ldc.
// ws: pra_wgrad_ws_floats() fp32 scratch and tickets: pra_wgrad_ticket_count() ints (the split tail;
// both may be null, then the tail runs as a partial data-parallel round).
long pra_wgrad_ws_floats() { return 256L * 256 * 256 * 4; }  // 256 MiB: 1024 partial tiles
int pra_wgrad_ticket_count() { return 256; }

hipError_t pra_wgrad_gemm(int dtype, const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                          long ldc, int accumulate, float* ws, int* tickets, hipStream_t s) {
  using namespace pra::wg;
  if (M % BM || N % BN || K % BK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8) return hipErrorInvalidValue;
  if ((long)(BK - 1) * lda + M > 0x7fffffffL || (long)(BK - 1) * ldb + N > 0x7fffffffL) return hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  const char* e = getenv("PRA_WGRAD_MFMA");  // read per call: in-process A/B
  const bool m32 = e && atoi(e) == 32;
  const char* en = getenv("PRA_WGRAD_STAGES");  // 16x16 ring depth: 4 or 5 (default)
  const bool ns5 = !(en && atoi(en) == 4);
  // 16x16 kernel: split the tiles of a partial last round S ways over K (S in 1..2 minimising the
  // rounds the split units take; ties -> smaller S). 7B shapes: W13 (96 tail tiles, S = 2) 1.31 ->
  // 1.40 PF; W2 (176 tail tiles) would need S = 4, measured slower (1.39 -> 1.24 PF), so unsplit.
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return hipErrorInvalidValue;
  int n_split = 0, S = 1;
  const char* es = getenv("PRA_WGRAD_SPLIT");  // 0 disables the split tail
  if (!m32 && ws && tickets && nwg > cus && nwg % cus != 0 && !(es && atoi(es) == 0)) {
    const int R = nwg % cus, nk = K / BK;
    double best = 1.0;  // unsplit: one more round
    const char* esm = getenv("PRA_WGRAD_SPLIT_MAX");  // largest split considered (default 2)
    const int smax = esm ? atoi(esm) : 2;
    for (int c = 2; c <= smax && c <= 8 && c <= nk; ++c) {
      const double t = (double)((R * c + cus - 1) / cus) / c;
      if (t < best - 1e-9) best = t, S = c;
    }
    if (S > 1 && (long)R * S * BM * BN <= pra_wgrad_ws_floats() && R <= pra_wgrad_ticket_count()) n_split = R;
    else S = 1;
  }
  // tickets are zeroed by a kernel, not hipMemsetAsync: replayed from a captured HIP graph
  // (train.py --compile), the memset node's zeros were not seen by the GEMM's ticket atomics and
  // most split tiles were never reduced (tests/test_kernels_gpu.py, graph-capture test)
  if (n_split) hipLaunchKernelGGL(zero_i32_kernel, dim3((n_split + 255) / 256), dim3(256), 0, s, tickets, n_split);
  const dim3 grid(m32 ? nwg : nwg - n_split + n_split * S), block(NTH);
#define PRA_WG_LAUNCH(TT)                                                                                     \
  if (m32) {                                                                                                  \
    if (accumulate)                                                                                           \
      hipLaunchKernelGGL((wgrad_kernel<TT, true>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C, M, N, \
                         K, lda, ldb, ldc);                                                                   \
    else                                                                                                      \
      hipLaunchKernelGGL((wgrad_kernel<TT, false>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C, M, \
                         N, K, lda, ldb, ldc);                                                                \
  } else if (ns5) {                                                                                           \
    if (accumulate)                                                                                           \
      hipLaunchKernelGGL((wgrad16_kernel<TT, true, 5>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C,  \
                         M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);                                    \
    else                                                                                                      \
      hipLaunchKernelGGL((wgrad16_kernel<TT, false, 5>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C, \
                         M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);                                    \
  } else {                                                                                                    \
    if (accumulate)                                                                                           \
      hipLaunchKernelGGL((wgrad16_kernel<TT, true, 4>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C,  \
                         M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);                                    \
    else                                                                                                      \
      hipLaunchKernelGGL((wgrad16_kernel<TT, false, 4>), grid, block, 0, s, (const TT*)A, (const TT*)B, (TT*)C, \
                         M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);                                    \
  }
  if (dtype == pra::kBF16) {
    PRA_WG_LAUNCH(__bf16)
  } else if (dtype == pra::kF16) {
    PRA_WG_LAUNCH(_Float16)
  } else {
    return hipErrorInvalidValue;
  }
#undef PRA_WG_LAUNCH
  return hipGetLastError();
}

}  // extern "C"

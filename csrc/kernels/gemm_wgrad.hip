// Weight-gradient GEMM for gfx950 (CDNA4) on row-major activations:
//
//     C[M][N] (+)= sum_k A[k][m] * B[k][n]        (dW = dY^T X, K = tokens)
//
// A = dY [K, M] and B = X [K, N] are the activations exactly as the forward/backward produce them
// (row-major, token rows). For this contraction both operands are "K-slow": consecutive k are a
// row stride apart. hipBLASLt runs that layout ~25-30% slower than K-contiguous operands (it needs
// transposed copies to be fast). Here the transpose happens inside the LDS read instead:
//
//  * tiles of BK = 32 token rows x 256 columns are staged global -> LDS by LDS-DMA into a
//    sub-tiled XOR-swizzled image; the ring/wait/barrier machine is gemm_common.h's (5 stages);
//  * MFMA operands (16 columns x 32 k) come from ds_read_b64_tr_b16, the gfx950 transposing LDS
//    read, so K-slow data feeds v_mfma_f32_16x16x32 directly;
//  * block tile 256 x 256, 4 waves of 128 x 128 (8 x 8 accumulators of 16 x 16);
//  * XCD-aware group-M tile order and the deterministic split-K tail (gemm_common.h);
//  * the accumulate mode (gradient accumulation) adds the existing C in fp32 and rounds once, like
//    addmm's beta = 1.
//
// Deterministic (fixed summation order), so resumed runs stay bit-identical.
// Requires M % 256 == 0, N % 256 == 0, K % 32 == 0, 16-B aligned rows (host-checked).
// Measured history (32x32x16 MFMA, 4-stage ring, ...): profiles/wgrad_mfma_r2.md. Round 4: the
// two-buffer 64-deep-chunk schedule that lifted the NT kernel +6-7% (gemm_nt.hip run2b) ran this
// kernel 3-6% SLOWER than the 5-stage ring (1.32-1.45 vs 1.40-1.49 PF; profiles/r4/
// wgrad_two_buffer_vs_ring.log; the cause was not isolated -- each fragment here is two
// ds_read_b64_tr_b16, so a chunk boundary carries 32 outstanding LDS reads per k-substep, more than
// the 4-bit lgkmcnt can count); removed.
#include "gemm_common.h"

#include <stdlib.h>

namespace pra {
namespace wg {

using namespace gm;

// LDS image of a [BK][256] tile: 8-row x 32-column sub-tiles of 512 B, the four 16-B chunks of
// each 64-B sub-tile row XOR-swizzled by (row >> 2) & 3. One ds_read_b64_tr_b16 reads exactly one
// 512-B sub-tile (8 k rows x 32 columns), so it is conflict-free.
constexpr int TD = 256;
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

// ---------------------------------------------------------------------------------------------
// v_mfma_f32_16x16x32: under load the chip holds a higher clock on the 16x16x32 shape than on
// 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH 'DVFS give-back' item 7). One 32-deep stage
// is one k-step; the wave's 128 x 128 tile is 8 x 8 accumulators of 16 x 16. Operand (16 columns x 32 k): 16-lane group g reads k rows 4g..4g+3 (lo) and
// 16+4g..16+4g+3 (hi) with ds_read_b64_tr_b16, so lane l of the group gets column l, k = {4g..4g+3,
// 16+4g..+3}; A and B use the same k permutation, so the dot products are unchanged.

// Work decomposition: tiles of 256 x 256 in group-M order (8 M-tiles per group). When the tile
// count is not a multiple of the CU count, the R tiles of the partial last round are split S ways
// over K (the launcher picks S so the split units fill whole rounds best): grid = (nwg - R) whole
// tiles + R * S split units, dispatched in that order. Each split unit writes its fp32 partial to
// ws and takes a ticket; the last arriver of a tile sums the S partials in part order (its own from
// ws too) -- deterministic, and nothing ever waits on another
// workgroup.
// EXP (timing experiments only, tools/gemm_exp.py; results are garbage): bit 0 = no main-loop
// LDS-DMA (prologue stages only), bit 1 = no main-loop fragment reads (stale registers)
// 1: each DMA group's M0 write first, its load last (no s_nop): 4096x4096x32768 1481-1509 -> 1514-1538
// TF, 11008x4096x32768 1366-1376 -> 1407-1410 TF (tools/wgrad_variants.hip,
// profiles/r4/wgrad_m0split_ab.log)
#ifndef PRA_WG_SMAX
#define PRA_WG_SMAX 2  // largest K-split of a partial last round (W2 at 4: 11% slower, profiles/r4/wgrad_w2_tail_split_ab.log)
#endif
#ifndef PRA_WG_M0SPLIT
#define PRA_WG_M0SPLIT 1
#endif

template <typename T, bool ACC, int EXP = 0>
__global__ __launch_bounds__(NTH) void wgrad16_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                      T* __restrict__ C, int M, int N, int K, long lda, long ldb,
                                                      long ldc, float* __restrict__ ws, int* __restrict__ tickets,
                                                      int n_split, int S) {
  __shared__ __attribute__((aligned(1024))) T smem[NS * 2 * TILE];
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n, nk = K / BK;

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
    auto dma_lds = [&](int s, int u) __attribute__((always_inline)) {
      return ldsw + (uint32_t)((s * 2 * TILE + (u & 1) * TILE) * sizeof(T) + (u >> 1) * 4 * 1024);
    };
    // (advancing the stage base pointers by one stage per step instead of recomputing them per DMA
    // cut the loop's SALU from ~40 to ~15 per stage and measured equal: profiles/r4/wgrad_incptr_ab.log)
    auto dma_go = [&](int kt, int u) __attribute__((always_inline)) {
      const T* g = (u & 1) ? Bb + (long)kt * BK * ldb : Ab + (long)kt * BK * lda;
      dma16s_go(g, (u & 1) ? offb[u >> 1] : offa[u >> 1]);
    };
    auto dma = [&](int s, int kt, int u) __attribute__((always_inline)) {
      const T* g = (u & 1) ? Bb + (long)kt * BK * ldb : Ab + (long)kt * BK * lda;
      dma16s(g, (u & 1) ? offb[u >> 1] : offa[u >> 1], dma_lds(s, u));
    };
    // every step issues exactly one stage of DMA (a stage past k1 re-loads stage k1 - 1 into the
    // slot nobody reads again), so the counted waits are the same on every step
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
#pragma unroll
      for (int u = 0; u < 2 * NI; ++u) dma(p, min(k0 + p, k1 - 1), u);
    wait_vm<2 * NI * (NS - 2)>();  // stage k0 landed; the younger stages stay in flight
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
      constexpr int s = decltype(s_c)::value % NS, sn = (s + 1) % NS, sd = (s + NS - 1) % NS;
      const T* nta = smem + sn * 2 * TILE;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
      if constexpr (!(EXP & 1)) wait_vm<2 * NI * (NS - 3)>();  // stage kt + 1 landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int kd = min(kt + NS - 1, k1 - 1);
#pragma unroll
      for (int gi = 0; gi < 8; ++gi) {
        // PRA_WG_M0SPLIT: the group's M0 write goes first and its DMA last, so the group's MFMAs
        // are the wait state (no s_nop)
        if constexpr (PRA_WG_M0SPLIT && !(EXP & 1)) {
          m0_set(dma_lds(sd, gi));
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!(EXP & 2)) {
          na[gi] = fragA(nta, gi);
          nb[gi] = fragB(nta + TILE, gi);
        }
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
        if constexpr (PRA_WG_M0SPLIT && !(EXP & 1))
          dma_go(kd, gi);
        else if constexpr (!(EXP & 1))
          dma(sd, kd, gi);
      }

    };
    // unrolled by lcm(NS, 2) = 10: compile-time ring slot and fragment register set
    constexpr int UNR = 10;
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
      st(IC<0>{}); st(IC<1>{}); st(IC<2>{}); st(IC<3>{}); st(IC<4>{});
      st(IC<5>{}); st(IC<6>{}); st(IC<7>{}); st(IC<8>{}); st(IC<9>{});
    }
    // no LDS-DMA may land after this point (next tile's prologue / end of the workgroup), and no
    // wave may still read a slot the next prologue overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  // epilogue: D[n][m] per 16 x 16 block: lane holds m = l & 15, n = 4 (l >> 4) + 0..3 (8 B)
  const int l16 = lane & 15, g4 = lane >> 4;
  auto store_c = [&](long m0, long n0) __attribute__((always_inline)) {
    // (16-B stores through v_permlane16_swap, as gemm_nt.hip's ST16 epilogue, measured equal here: the
    // epilogue is ~1% of a K = 32768 tile; profiles/r4/wgrad_st16_epilogue_ab.log)
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
  // fp32 partial of the current accumulators into ws slot `slot` (thread t's register r at r * NTH + t)
  auto put_partial = [&](long slot) __attribute__((always_inline)) {
    float* w = ws + slot * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) w[((i * 8 + j) * 4 + e) * NTH + tid] = acc[i][j][e];
  };
  // publish the partial, take a ticket of `tick`; true on the last of `n` arrivals (which then sees
  // every other partial: release / acquire at agent scope around the ticket)
  auto arrive = [&](int* tick, int n) __attribute__((always_inline)) -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);  // the one LDS array (free after run)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = ticket == n - 1;
      if (ticket == n - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    const bool l = *last;
    __syncthreads();  // the flag's LDS word is the next tile's DMA target
    return l;
  };
  auto add_partial = [&](long slot) __attribute__((always_inline)) {
    const float* wp = ws + slot * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] += wp[((i * 8 + j) * 4 + e) * NTH + tid];
  };
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
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
  tile_origin(lin, tiles_m, tiles_n, m0, n0);
  run(m0, n0, k0, k1);
  if (split) {
    put_partial((long)st * S + part);
    if (!arrive(tickets + st, S)) return;
    // sum the S partials in part order (its own included, re-read from ws: same order whoever is last)
    zero_acc();
    for (int p = 0; p < S; ++p) add_partial((long)st * S + p);
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

// (A deterministic stream-K schedule -- persistent data-parallel rounds plus a stream-K remainder --
// was correct but slower on every shape measured, the concurrently active tiles losing L2 reuse:
// profiles/r5/wgrad_bench_7b*.log, wgrad_bench_8b_b1.log. Removed in round 6.)
extern "C" {

// C[M][N] (+)= A^T B with A [K][M] (row stride lda), B [K][N] (row stride ldb), C row stride ldc.
// ws / tickets: sized by pra_wgrad_ws_floats / pra_wgrad_ticket_count (the split tail; both may be
// null, then the tail runs as a partial data-parallel round).
// fp32 partial-tile floats / tickets the split tail of an [M, N, K] weight gradient needs (0 = none)
long pra_wgrad_ws_floats(int M, int N, int K, int cus) {
  using namespace pra::gm;
  const int nwg = (M / BM) * (N / BN);
  const int S = pra::gemm_tail_split(nwg, cus, K / BK, PRA_WG_SMAX);
  return S > 1 ? (long)(nwg % cus) * S * BM * BN : 0;
}
int pra_wgrad_ticket_count(int M, int N, int K, int cus) {
  using namespace pra::gm;
  const int nwg = (M / BM) * (N / BN);
  return pra::gemm_tail_split(nwg, cus, K / BK, PRA_WG_SMAX) > 1 ? nwg % cus : 0;
}

hipError_t pra_wgrad_gemm(int dtype, const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                          long ldc, int accumulate, float* ws, int* tickets, int cus, hipStream_t s) {
  using namespace pra::gm;
  if (M % BM || N % BN || K % BK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8 || cus <= 0) return hipErrorInvalidValue;
  if ((long)(BK - 1) * lda + M > 0x7fffffffL || (long)(BK - 1) * ldb + N > 0x7fffffffL) return hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // split the tiles of a partial last round S ways over K (S <= 2; 7B shapes: W13's 96 tail tiles
  // S = 2, 1.31 -> 1.40 PF; W2's 176 would need S = 4, measured slower, so unsplit)
  const int Sx = pra::gemm_tail_split(nwg, cus, K / BK, PRA_WG_SMAX);
  const int n_split = Sx > 1 && ws && tickets ? nwg % cus : 0;
  const int S = n_split ? Sx : 1;
  // tickets are zeroed by a kernel, not hipMemsetAsync: replayed from a captured HIP graph
  // (train.py --compile), the memset node's zeros were not seen by the GEMM's ticket atomics and
  // most split tiles were never reduced (tests/test_kernels_gpu.py, graph-capture test)
  if (n_split) hipLaunchKernelGGL(pra::wg::zero_i32_kernel, dim3((n_split + 255) / 256), dim3(256), 0, s, tickets, n_split);
  const dim3 grid(nwg - n_split + n_split * S), block(NTH);
#define PRA_WG_LAUNCH(TT)                                                                                    \
  if (accumulate)                                                                                            \
    hipLaunchKernelGGL((pra::wg::wgrad16_kernel<TT, true>), grid, block, 0, s, (const TT*)A, (const TT*)B,     \
                       (TT*)C, M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);                             \
  else                                                                                                       \
    hipLaunchKernelGGL((pra::wg::wgrad16_kernel<TT, false>), grid, block, 0, s, (const TT*)A, (const TT*)B,    \
                       (TT*)C, M, N, K, lda, ldb, ldc, ws, tickets, n_split, S);
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

// timing experiments (see wgrad16_kernel's EXP): bf16, no accumulate, no split tail. Measured at
// 32768 x 4096 x 16384: 1.40 PF as is, 1.78 PF without the main-loop LDS-DMA, 1.53 PF without the
// fragment reads (profiles/r3/gemm_wgrad_exp.log)
hipError_t pra_wgrad_gemm_exp(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                              long ldc, int exp, hipStream_t s) {
  using namespace pra::gm;
  if (M % BM || N % BN || K % BK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8) return hipErrorInvalidValue;
  const dim3 grid((M / BM) * (N / BN)), block(NTH);
#define PRA_WG_EXP(E)                                                                                        \
  hipLaunchKernelGGL((pra::wg::wgrad16_kernel<__bf16, false, E>), grid, block, 0, s, (const __bf16*)A,         \
                     (const __bf16*)B, (__bf16*)C, M, N, K, lda, ldb, ldc, nullptr, nullptr, 0, 1)
  switch (exp) {
    case 1: PRA_WG_EXP(1); break;
    case 2: PRA_WG_EXP(2); break;
    case 3: PRA_WG_EXP(3); break;
    default: PRA_WG_EXP(0); break;
  }
#undef PRA_WG_EXP
  return hipGetLastError();
}

}  // extern "C"

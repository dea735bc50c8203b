// Forward / data-gradient GEMM for gfx950 (CDNA4) with fused epilogues:
//
//     C[M][N] = sum_k A[m][k] * B[n][k]        (Y = X W^T, dX = dY W with W^T shadows)
//
// Both operands are K-contiguous (row-major activations [tokens, in] and weights [out, in]), the
// "NT" layout of every forward projection and of the data gradients (ops/fused.py keeps
// transposed weight shadows so dX = dY W is NT too). Reference GEMM sites: model.py:171-177
// (wq/wk/wv/wo), :264-269 (w1/w3/w2), :367 (output head).
//
// Machine (gemm_common.h): 256 x 256 tile, 4 waves of 128 x 128, v_mfma_f32_16x16x32, XCD-aware
// group-M order, deterministic split-K tail, counted vmcnt + raw s_barrier. K % 64 == 0 (every
// production shape): 64-deep chunks in two LDS buffers (run2b below, 128-B rows). K % 64 == 32:
// 32-deep stages by LDS-DMA into a 5-stage ring (run). Operand tiles of the ring are [256 rows][32 k]
// (64-B rows) in LDS; MFMA operand
// fragments (16 rows x 32 k) are ONE ds_read_b128 per lane: lane l reads row l & 15, k 8(l >> 4)..+7,
// exactly the MFMA operand map. The 16-B chunks of each row are XOR-swizzled by g((row >> 2) & 3),
// g = {0, 2, 3, 1}, which makes every ds_read_b128 lane group cover the 16 slots of a bank row once
// (conflict-free); the LDS-DMA writes linearly and the swizzle is applied to its global source
// address instead.
//
// Orientation: acc = mfma(B fragment, A fragment), so a lane holds one output row m and 4
// consecutive columns n in its 4 registers: RoPE pairs (2i, 2i+1) are in one lane; with ST16 two
// 16 x 16 blocks are paired through v_permlane16_swap so each lane writes 16 contiguous bytes.
//
// Epilogues (EPI):
//   0 plain:        C = A B^T (bf16/fp16 rounding once)
//   1 SwiGLU fwd:   B = W1|W3 [2F][K]; the B tile interleaves 128 gate rows with the matching
//                   128 up rows so gate and up of a feature land in one lane; writes
//                   gu = [g | u] (C, [M][2F]) and a = round(silu(g)) * u (C2, [M][F])
//                   (the rounding points of swiglu_fwd_kernel, reference model.py:268-269)
//   2 SwiGLU bwd:   C = da = dY W2 is never stored; the epilogue reads g, u from gu (C, in place)
//                   and overwrites them with dg, du (swiglu_bwd_kernel's math)
//   3 RoPE:         C = QKV with the interleaved-pair rotation (rope_kernel's math, reference
//                   model.py:101-127) applied to the first `nrot` columns (q and k heads)
// Requires M % 256 == 0, N % 256 == 0 (EPI 1: F % 128 == 0), K % 32 == 0, 16-B aligned rows.
#include "gemm_common.h"

#include <stdlib.h>

namespace pra {
namespace nt {

using namespace gm;

template <typename T>
struct Epi {
  T* c2;             // EPI 1: a [M][F]
  long ldc2;
  int F;             // EPI 1 / 2: gu holds g at [0, F) and u at [F, 2F)
  const float2* tab; // EPI 3: (cos, sin) [S][D/2]
  int S, D, nrot;    // EPI 3
};

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ void rot_pair(float a, float b, float c, float s, float& o0, float& o1) {
  o0 = __builtin_fmaf(a, c, -(b * s));
  o1 = __builtin_fmaf(a, s, b * c);
}
template <typename T>
__device__ __forceinline__ float rnd16(float v) {
  return (float)(T)v;
}
template <typename T>
__device__ __forceinline__ void unpack4(uint2 w, float (&o)[4]) {
  const T* h = reinterpret_cast<const T*>(&w);
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (float)h[e];
}

// Diagnostic build only (tools/nt_stamps.hip defines PRA_NT_STAMPS): per-wave s_memtime sums of the
// two-buffer loop's phases, written once per wave at the end of the tile. The stamps sit where
// lgkmcnt is already 0 (after the phase-1 drain, after each barrier, before the vmcnt wait), so
// the counted LDS waits are unchanged.
#ifdef PRA_NT_STAMPS
__device__ unsigned long long* pra_nt_stamp_out;
#define PRA_NT_STAMP(v)                  \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    v = __builtin_amdgcn_s_memtime();    \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#else
#define PRA_NT_STAMP(v) \
  do {                  \
  } while (0)
#endif

// SCHED 1 (hipBLASLt's chunk order, 4 barriers) vs 0 (3 phases, 2 barriers) and VOFF (per-DMA row
// offsets in VGPRs) at 32768x4096x4096, three interleaved rounds: 3-phase 1438, 4-barrier 1445,
// 4-barrier + VOFF 1449, 3-phase + VOFF 1454 TF (the VGPR offsets take ~50 cycles per chunk off
// phase 2); hipBLASLt 1508-1580 on this shape (profiles/r4/gemm_nt_hipblaslt_order*.log)
#ifndef PRA_NT_SCHED
#define PRA_NT_SCHED 0
#endif
// ST16: epilogue stores of 16 B (v_permlane16_swap pairs two 16-column blocks) instead of 8 B: per
// 256x256 tile 11.8k instead of 16.1k cycles from loop end to stores retired; 32768x11008x4096
// 1434 -> 1466 TF (profiles/r4/gemm_nt_st16_epilogue.log)
// (Persistent workgroups walking per-XCD tile ranges through atomic counters, with the next tile's
// prologue DMAs issued before the current tile's epilogue stores, measured 0.2-1.1% slower:
// profiles/r4/gemm_nt_persistent_ab.log.)
#ifndef PRA_NT_EPI2_PIPE  // SwiGLU backward epilogue with row-block loads two blocks ahead (epi2_pipe)
#define PRA_NT_EPI2_PIPE 1
#endif
#ifndef PRA_NT_EPI2_DEPTH  // row blocks of g / u in flight in epi2_pipe (32 VGPRs each)
#define PRA_NT_EPI2_DEPTH 3
#endif
#ifndef PRA_NT_ST16
#define PRA_NT_ST16 1
#endif
#ifndef PRA_NT_VOFF
#define PRA_NT_VOFF 1
#endif
#ifndef PRA_NT_P1
#define PRA_NT_P1 32
#endif
#ifndef PRA_NT_RS1
#define PRA_NT_RS1 1
#endif
#ifndef PRA_NT_P3
#define PRA_NT_P3 16
#endif
#ifndef PRA_NT_RS3
#define PRA_NT_RS3 1
#endif
// M0SPLIT 1: 1432-1449 vs 1429-1431 TF without (32768x4096x4096; per-chunk phase 2 1467 vs 1515
// cycles); spreading the fragment reads one per two or three MFMAs (RS > 1) was 2-9% slower:
// profiles/r4/gemm_nt_schedule_variants*.log
#ifndef PRA_NT_M0SPLIT
#define PRA_NT_M0SPLIT 1
#endif

// PRA_NT_SCHED 1 event tables: the MFMA index after which DMA d (A rows 0..7, B rows 8..15) of
// chunk t + 2 issues, and after which fragment read 8 g + r issues (g: 0 fb1, 1 fa1 of chunk t;
// 2 fb0, 3 fa0 of chunk t + 1)
constexpr int kNt4Dma[16] = {61, 64, 85, 87, 89, 94, 98, 124, 22, 25, 28, 31, 34, 52, 55, 58};
constexpr int kNt4Read[32] = {1,   3,   5,   7,   9,   11,  13,  15,  24, 27, 30, 33, 36, 38, 40, 42,
                              69,  71,  73,  75,  77,  79,  81,  83,  106, 108, 110, 112, 114, 116, 118, 120};
constexpr int nt4_dma_at(int q) {
  for (int d = 0; d < 16; ++d)
    if (kNt4Dma[d] == q) return d;
  return -1;
}
constexpr int nt4_read_at(int q) {
  for (int i = 0; i < 32; ++i)
    if (kNt4Read[i] == q) return i;
  return -1;
}

// the XOR swizzle of the 16-B chunk of row r: g((r >> 2) & 3), g = {0, 2, 3, 1}
__device__ __forceinline__ int swz(int r) {
  const int q = (r >> 2) & 3;
  return (q >> 1) | (((q & 1) ^ (q >> 1)) << 1);
}

// KB: k depth of one LDS stage. 32: 5-stage ring of [256][32] images (64-B rows). 64: 2-chunk ring
// of [256][64] images (128-B rows: every LDS-DMA instruction reads whole 128-B lines, 8 rows x 128 B,
// instead of 16 rows x 64 B; MI355X guide: fragment-shaped 64-B row pieces cost +18-45%).
template <typename T, int EPI, int KB>
__global__ __launch_bounds__(NTH) void gemm_nt_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                      T* __restrict__ C, int M, int N, int K, long lda, long ldb,
                                                      long ldc, Epi<T> ep, float* __restrict__ ws,
                                                      int* __restrict__ tickets, int n_split, int S) {
  constexpr int TILE64 = 64 * 256;  // elements of a [256][64] operand chunk (32 KiB)
  __shared__ __attribute__((aligned(1024))) T smem[KB == 64 ? 4 * TILE64 : NS * 2 * TILE];
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n, nk = K / KB;

  // wid through readfirstlane: the compiler then knows it is wave-uniform, and every per-instruction
  // DMA base derived from it stays in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // DMA instruction i of wave w fills LDS bytes [(4i + w) KiB, +1 KiB) of an operand tile: rows
  // 16 (4i + w) + lane / 4, swizzled chunk lane & 3 -> global chunk (lane & 3) ^ swz(row)
  uint32_t offa[NI], offb[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = (i * 4 + wid) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    offa[i] = (uint32_t)((r * (int)lda + c * 8) * (int)sizeof(T));
    int br = r;
    if constexpr (EPI == 1) {  // rows of W1|W3: 64 gate rows then the 64 matching up rows per wave half
      const int f = (r >> 4) & 7;
      br = (f >= 4 ? ep.F : 0) + (r >> 7) * 64 + (f & 3) * 16 + (r & 15);
    }
    offb[i] = (uint32_t)(((long)br * ldb + c * 8) * (long)sizeof(T));
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)smem;
  const uint32_t ldsw = __builtin_amdgcn_readfirstlane(lds0 + wid * 1024);  // this wave's DMA base

  // fragment reads: row (l & 15) of the 16-row block, chunk (l >> 4) at its swizzled slot
  const int fo = (lane & 15) * 64 + (((lane >> 4) ^ swz(lane & 15)) * 16);
  const int foa = fo + 8192 * wm, fob = fo + 8192 * wn;  // wave's 128 rows = 8 blocks of 1 KiB
  auto frag = [&](const T* tile, int off) __attribute__((always_inline)) -> V8<T> {
    return *reinterpret_cast<const V8<T>*>(reinterpret_cast<const char*>(tile) + off);
  };

  // KB = 64 images: row r at r * 128 B, 16-B chunk c at slot c ^ ((r >> 1) & 7): every ds_read_b128
  // lane group (16 rows x one chunk) covers the 16 slots of a bank row once. DMA instruction i
  // (0..7) of wave w fills bytes [(4i + w) KiB, +1 KiB): rows r = 32 i + 8 w + lane / 8, slot
  // lane & 7. (r >> 1) & 7 = (4 (w & 1) + lane / 16) & 7 does not depend on i, so the per-lane
  // source offset is one VGPR and the per-instruction part goes into the wave-uniform base.
  uint32_t voa64 = 0, vob64 = 0;
  int f64[2] = {0, 0};
  if constexpr (KB == 64) {
    const int c = (lane & 7) ^ ((4 * (wid & 1) + (lane >> 4)) & 7);
    voa64 = (uint32_t)(((lane >> 3) * (int)lda + c * 8) * (int)sizeof(T));
    vob64 = (uint32_t)((long)((lane >> 3) * ldb + c * 8) * (long)sizeof(T));
    // fragment of k-substep `sub` (0/1): row (l & 15), chunk (l >> 4) + 4 sub at its swizzled slot
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
      f64[sub] = (lane & 15) * 128 + ((((lane >> 4) + 4 * sub) ^ ((lane >> 1) & 7)) * 16);
  }
  // first tile row (A) / weight row (B) of DMA instruction i of this wave (wave-uniform)
  auto row_a64 = [&](int i) __attribute__((always_inline)) -> int { return 32 * i + 8 * wid; };
  auto row_b64 = [&](int i) __attribute__((always_inline)) -> int {
    if constexpr (EPI == 1) {  // W1|W3 rows: 64 gate rows then the 64 matching up rows per wave half
      const int f = (2 * i + (wid >> 1)) & 7;
      return (f >= 4 ? ep.F : 0) + (i >> 2) * 64 + (f & 3) * 16 + 8 * (wid & 1);
    } else {
      return 32 * i + 8 * wid;
    }
  };

  f32x4 acc[8][8];
  V8<T> fa0[8], fb0[8], fa1[8], fb1[8];

  // epilogue: lane holds row m0 + 128 wm + 16 i + (l & 15), columns n0 + 128 wn + 16 j + 4 (l >> 4) + 0..3
  const int l16 = lane & 15, g4 = lane >> 4;

  // SwiGLU backward epilogue (EPI 2, ST16 layout) with the g / u loads of row block i + 2 in flight
  // while block i is computed and stored. The one-block-at-a-time form waited a full load (and the
  // previous block's stores, which count in vmcnt) per row block: 8 serialized HBM round trips per
  // tile, and every CU reaches its epilogue at the same time (tiles run in lockstep rounds), so the
  // fused GEMM ran 675 us slower than the plain one at 7B W2 (profiles/r4/gemm_nt_bench_swiglu_epilogues.log),
  // as slow as the separate kernel. The main loop's fragment registers are dead here, so the
  // three in-flight blocks (96 VGPRs) fit.
  auto epi2_pipe = [&](long m0, long n0) __attribute__((always_inline)) {
    const long so = (16 * (g4 & 1) + 8 * (g4 >> 1)) - 4 * g4;
    auto gptr = [&](int i) __attribute__((always_inline)) -> T* {
      return C + (m0 + 128 * wm + 16 * i + l16) * ldc + n0 + 128 * wn + 4 * g4 + so;
    };
    constexpr int DEPTH = PRA_NT_EPI2_DEPTH;  // row blocks in flight
    uint4 gb[DEPTH][4], ub[DEPTH][4];
    auto load = [&](int i, uint4 (&g8)[4], uint4 (&u8)[4]) __attribute__((always_inline)) {
      const T* gp = gptr(i);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        g8[q] = *reinterpret_cast<const uint4*>(gp + 32 * q);
        u8[q] = *reinterpret_cast<const uint4*>(gp + ep.F + 32 * q);
      }
    };
#pragma unroll
    for (int i = 0; i < DEPTH - 1; ++i) load(i, gb[i], ub[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + DEPTH - 1 < 8) load(i + DEPTH - 1, gb[(i + DEPTH - 1) % DEPTH], ub[(i + DEPTH - 1) % DEPTH]);
      const uint4 (&g8)[4] = gb[i % DEPTH];
      const uint4 (&u8)[4] = ub[i % DEPTH];
      uint2 gw[8], uw[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // back to this lane's own 4 columns of blocks 2q, 2q + 1
        const auto g0 = __builtin_amdgcn_permlane16_swap(g8[q].x, g8[q].z, false, false);
        const auto g1 = __builtin_amdgcn_permlane16_swap(g8[q].y, g8[q].w, false, false);
        const auto u0 = __builtin_amdgcn_permlane16_swap(u8[q].x, u8[q].z, false, false);
        const auto u1 = __builtin_amdgcn_permlane16_swap(u8[q].y, u8[q].w, false, false);
        gw[2 * q] = make_uint2(g0[0], g1[0]);
        gw[2 * q + 1] = make_uint2(g0[1], g1[1]);
        uw[2 * q] = make_uint2(u0[0], u1[0]);
        uw[2 * q + 1] = make_uint2(u0[1], u1[1]);
      }
      uint2 ogw[8], ouw[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g[4], u[4], og[4], ou[4];
        unpack4<T>(gw[j], g);
        unpack4<T>(uw[j], u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // the math of the one-block form below, element for element
          const float d = rnd16<T>(acc[i][j][e]);
          const float sg = 1.f / (1.f + __expf(-g[e]));
          const float a = rnd16<T>(g[e] * sg);
          const float dd = rnd16<T>(d * u[e]);
          ou[e] = d * a;
          og[e] = dd * sg * (1.f + g[e] * (1.f - sg));
        }
        ogw[j] = make_uint2(pack_x2<T>(og[0], og[1]), pack_x2<T>(og[2], og[3]));
        ouw[j] = make_uint2(pack_x2<T>(ou[0], ou[1]), pack_x2<T>(ou[2], ou[3]));
      }
      T* gp = gptr(i);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 2 * q;
        const auto g0 = __builtin_amdgcn_permlane16_swap(ogw[j].x, ogw[j + 1].x, false, false);
        const auto g1 = __builtin_amdgcn_permlane16_swap(ogw[j].y, ogw[j + 1].y, false, false);
        const auto u0 = __builtin_amdgcn_permlane16_swap(ouw[j].x, ouw[j + 1].x, false, false);
        const auto u1 = __builtin_amdgcn_permlane16_swap(ouw[j].y, ouw[j + 1].y, false, false);
        *reinterpret_cast<uint4*>(gp + 16 * j) = make_uint4(g0[0], g1[0], g0[1], g1[1]);
        *reinterpret_cast<uint4*>(gp + ep.F + 16 * j) = make_uint4(u0[0], u1[0], u0[1], u1[1]);
      }
    }
  };

  auto store_c = [&](long m0, long n0) __attribute__((always_inline)) {
    if constexpr (EPI == 2 && PRA_NT_ST16 && PRA_NT_EPI2_PIPE) {
      epi2_pipe(m0, n0);
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long row = m0 + 128 * wm + 16 * i + l16;
      if constexpr (EPI == 0 || EPI == 3) {
        T* rowp = C + row * ldc + n0 + 128 * wn + 4 * g4;
        int pos = 0;
        if constexpr (EPI == 3) pos = (int)(row % ep.S);
        auto vals = [&](int j, float (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e];
          if constexpr (EPI == 3) {
            const int col = (int)n0 + 128 * wn + 16 * j + 4 * g4;
            if (col < ep.nrot) {
              const float4 cs = *reinterpret_cast<const float4*>(ep.tab + (long)pos * (ep.D / 2) + (col % ep.D) / 2);
              float a0 = rnd16<T>(v[0]), b0 = rnd16<T>(v[1]), a1 = rnd16<T>(v[2]), b1 = rnd16<T>(v[3]);
              rot_pair(a0, b0, cs.x, cs.y, v[0], v[1]);
              rot_pair(a1, b1, cs.z, cs.w, v[2], v[3]);
            }
          }
        };
        if constexpr (PRA_NT_ST16) {
          // blocks j, j + 1 through v_permlane16_swap (lane rows g4 even <-> odd): lane row g4
          // ends up with 8 consecutive columns, 16 (j + (g4 & 1)) + 8 (g4 >> 1) + 0..7, and stores
          // them as one 16-B write (32 instead of 64 store instructions per lane)
          T* sp = C + row * ldc + n0 + 128 * wn + 16 * (g4 & 1) + 8 * (g4 >> 1);
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            float va[4], vb[4];
            vals(j, va);
            vals(j + 1, vb);
            const auto s0 = __builtin_amdgcn_permlane16_swap(pack_x2<T>(va[0], va[1]), pack_x2<T>(vb[0], vb[1]), false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(pack_x2<T>(va[2], va[3]), pack_x2<T>(vb[2], vb[3]), false, false);
            *reinterpret_cast<uint4*>(sp + 16 * j) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v[4];
            vals(j, v);
            *reinterpret_cast<uint2*>(rowp + 16 * j) = make_uint2(pack_x2<T>(v[0], v[1]), pack_x2<T>(v[2], v[3]));
          }
        }
      } else if constexpr (EPI == 1) {
        // features f0 + 16 j + 4 g4 + 0..3 (j < 4): gate in acc[i][j], up in acc[i][j + 4]
        const long f0 = n0 / 2 + 64 * wn + 4 * g4;
        T* gp = C + row * ldc + f0;
        T* up = gp + ep.F;
        T* ap = ep.c2 + row * ep.ldc2 + f0;
        auto gua = [&](int j, uint32_t (&o)[6]) __attribute__((always_inline)) {  // g, u, a packed pairs
          float g[4], u[4], a[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            g[e] = rnd16<T>(acc[i][j][e]);
            u[e] = rnd16<T>(acc[i][j + 4][e]);
            a[e] = rnd16<T>(silu_f(g[e])) * u[e];
          }
          o[0] = pack_x2<T>(g[0], g[1]); o[1] = pack_x2<T>(g[2], g[3]);
          o[2] = pack_x2<T>(u[0], u[1]); o[3] = pack_x2<T>(u[2], u[3]);
          o[4] = pack_x2<T>(a[0], a[1]); o[5] = pack_x2<T>(a[2], a[3]);
        };
        if constexpr (PRA_NT_ST16) {  // as EPI 0: features 16 (j + (g4 & 1)) + 8 (g4 >> 1) + 0..7 per lane
          const long s0 = (16 * (g4 & 1) + 8 * (g4 >> 1)) - 4 * g4;
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            uint32_t x[6], y[6];
            gua(j, x);
            gua(j + 1, y);
            T* dst[3] = {gp + s0 + 16 * j, up + s0 + 16 * j, ap + s0 + 16 * j};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const auto w0 = __builtin_amdgcn_permlane16_swap(x[2 * k], y[2 * k], false, false);
              const auto w1 = __builtin_amdgcn_permlane16_swap(x[2 * k + 1], y[2 * k + 1], false, false);
              *reinterpret_cast<uint4*>(dst[k]) = make_uint4(w0[0], w1[0], w0[1], w1[1]);
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t x[6];
            gua(j, x);
            *reinterpret_cast<uint2*>(gp + 16 * j) = make_uint2(x[0], x[1]);
            *reinterpret_cast<uint2*>(up + 16 * j) = make_uint2(x[2], x[3]);
            *reinterpret_cast<uint2*>(ap + 16 * j) = make_uint2(x[4], x[5]);
          }
        }
      } else {  // EPI == 2: dg = silu'(g) * round(da * u), du = round(da * round(silu(g))) in place over gu
        T* gp = C + row * ldc + n0 + 128 * wn + 4 * g4;
        T* up = gp + ep.F;
        uint2 gw[8], uw[8];
        if constexpr (PRA_NT_ST16) {
          // 16-B loads at the ST16 positions, swapped back to this lane's own 4 columns of blocks
          // j and j + 1 (v_permlane16_swap is its own inverse on this pairing)
          const long so = (16 * (g4 & 1) + 8 * (g4 >> 1)) - 4 * g4;
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const uint4 g8 = *reinterpret_cast<const uint4*>(gp + so + 16 * j);
            const uint4 u8 = *reinterpret_cast<const uint4*>(up + so + 16 * j);
            const auto g0 = __builtin_amdgcn_permlane16_swap(g8.x, g8.z, false, false);
            const auto g1 = __builtin_amdgcn_permlane16_swap(g8.y, g8.w, false, false);
            const auto u0 = __builtin_amdgcn_permlane16_swap(u8.x, u8.z, false, false);
            const auto u1 = __builtin_amdgcn_permlane16_swap(u8.y, u8.w, false, false);
            gw[j] = make_uint2(g0[0], g1[0]);
            gw[j + 1] = make_uint2(g0[1], g1[1]);
            uw[j] = make_uint2(u0[0], u1[0]);
            uw[j + 1] = make_uint2(u0[1], u1[1]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {  // all loads first: one wait for the whole row block
            gw[j] = *reinterpret_cast<const uint2*>(gp + 16 * j);
            uw[j] = *reinterpret_cast<const uint2*>(up + 16 * j);
          }
        }
        uint2 ogw[8], ouw[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g[4], u[4], og[4], ou[4];
          unpack4<T>(gw[j], g);
          unpack4<T>(uw[j], u);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = rnd16<T>(acc[i][j][e]);
            const float sg = 1.f / (1.f + __expf(-g[e]));
            const float a = rnd16<T>(g[e] * sg);
            const float dd = rnd16<T>(d * u[e]);
            ou[e] = d * a;
            og[e] = dd * sg * (1.f + g[e] * (1.f - sg));
          }
          ogw[j] = make_uint2(pack_x2<T>(og[0], og[1]), pack_x2<T>(og[2], og[3]));
          ouw[j] = make_uint2(pack_x2<T>(ou[0], ou[1]), pack_x2<T>(ou[2], ou[3]));
          if constexpr (!PRA_NT_ST16) {
            *reinterpret_cast<uint2*>(gp + 16 * j) = ogw[j];
            *reinterpret_cast<uint2*>(up + 16 * j) = ouw[j];
          }
        }
        if constexpr (PRA_NT_ST16) {
          const long so = (16 * (g4 & 1) + 8 * (g4 >> 1)) - 4 * g4;
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const auto g0 = __builtin_amdgcn_permlane16_swap(ogw[j].x, ogw[j + 1].x, false, false);
            const auto g1 = __builtin_amdgcn_permlane16_swap(ogw[j].y, ogw[j + 1].y, false, false);
            const auto u0 = __builtin_amdgcn_permlane16_swap(ouw[j].x, ouw[j + 1].x, false, false);
            const auto u1 = __builtin_amdgcn_permlane16_swap(ouw[j].y, ouw[j + 1].y, false, false);
            *reinterpret_cast<uint4*>(gp + so + 16 * j) = make_uint4(g0[0], g1[0], g0[1], g1[1]);
            *reinterpret_cast<uint4*>(up + so + 16 * j) = make_uint4(u0[0], u1[0], u0[1], u1[1]);
          }
        }
      }
    }
  };

  // KB = 64: two LDS buffers of one 64-deep chunk each (A and B [256][64], 64 KiB per buffer).
  // Every fragment of a chunk lives in registers (k-substep 0 in fa0/fb0, 1 in fa1/fb1), so its
  // buffer is free as soon as every wave has read it: one third into chunk t (barrier 1) the LDS-DMA
  // of chunk t + 2 starts into that buffer, spread one instruction per 5 MFMAs, and it has until
  // 7/8 into chunk t + 1 (counted vmcnt + barrier 2) to land -- about 1.5 chunks of MFMAs (the
  // round-3 5-unit ring gave its B unit one 32-deep substep: 1.33-1.41 vs 1.40-1.49 PF here,
  // profiles/r4/gemm_nt_sched_ab.log). Per chunk and wave, 128 MFMAs in 3 phases:
  //   phase 1 (MFMA 0..31):   k-substep-1 fragment reads of chunk t under the first 16 MFMAs
  //   lgkmcnt(0) + barrier 1 (buffer t free in every wave)
  //   phase 2 (MFMA 32..111): 16 LDS-DMA instructions of chunk t + 2 into buffer t
  //   vmcnt(16) + barrier 2 (chunk t + 1 landed and published; chunk t + 2 stays in flight)
  //   phase 3 (MFMA 112..127): k-substep-0 fragment reads of chunk t + 1 from the other buffer
  // The schedule of hipBLASLt's direct-to-LDS 256x256x64 kernels (PGR2/PLR1), on our LDS image.
  // Measured and not kept (profiles/r4/): the same loop as persistent workgroups walking several
  // tiles (1-6% slower: static tile assignment loses the hardware's dynamic dispatch), on a padded
  // unswizzled LDS image (5-8% slower: 2-way bank conflicts), with buffer-form LDS-DMA (equal).
#ifdef PRA_NT_STAMPS
  unsigned long long ts1, ts2, ts3, ts4, ts4p = 0, sw1 = 0, sp2 = 0, sw2 = 0, sp31 = 0, nch = 0;
  unsigned long long tk0 = 0, tk1 = 0, tk2 = 0, tk3 = 0;  // tile: start, prologue landed, loop end, stored
#endif
  auto run2b = [&](long m0, long n0, int c0, int c1) __attribute__((always_inline)) {
    const T* Ab = A + m0 * lda;
    const T* Bb = B + (EPI == 1 ? n0 / 2 : n0) * ldb;
    // DMA instruction d (0..15: A rows for d < 8, B rows after) of chunk c into buffer b; chunks
    // past the end re-load the last chunk (uniform issue counts; nobody reads those bytes)
    auto dma = [&](int b, int c, int d) __attribute__((always_inline)) {
      c = min(c, c1 - 1);
      const int i = d & 7;
      const uint32_t lds = ldsw + (uint32_t)((b * 2 + (d >> 3)) * TILE64 * sizeof(T) + i * 4 * 1024);
      if (d >= 8)
        dma16s(Bb + (long)row_b64(i) * ldb + (long)c * 64, vob64, lds);
      else
        dma16s(Ab + (long)row_a64(i) * lda + (long)c * 64, voa64, lds);
    };
    auto fragA = [&](int b, int sub, int f) __attribute__((always_inline)) {
      return frag(smem + b * 2 * TILE64, f64[sub] + 16384 * wm + 2048 * f);
    };
    auto fragB = [&](int b, int sub, int f) __attribute__((always_inline)) {
      return frag(smem + (b * 2 + 1) * TILE64, f64[sub] + 16384 * wn + 2048 * f);
    };
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B rows first (d = 8..15, then 0..7): the 4-barrier schedule waits for a chunk's B half
    // before its A half
#pragma unroll
    for (int e = 0; e < 16; ++e) dma(0, c0, (e + 8) & 15);
#pragma unroll
    for (int e = 0; e < 16; ++e) dma(1, c0 + 1, (e + 8) & 15);
    wait_vm<16>();  // chunk c0 landed; c0 + 1 stays in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    PRA_NT_STAMP(tk1);
    fa0[0] = fragA(0, 0, 0);
#pragma unroll
    for (int f = 0; f < 8; ++f) fb0[f] = fragB(0, 0, f);
#pragma unroll
    for (int f = 1; f < 8; ++f) fa0[f] = fragA(0, 0, f);
    // MFMA q (0..127) of a chunk: k-substep q / 64, A fragment (q % 64) / 8, B fragment q % 8
    auto mf = [&](int q) __attribute__((always_inline)) {
      const int i = (q & 63) >> 3, j = q & 7;
      if (q < 64)
        acc[i][j] = mfma16(fb0[j], fa0[i], acc[i][j]);
      else
        acc[i][j] = mfma16(fb1[j], fa1[i], acc[i][j]);
    };
    // schedule knobs (defaults: the production schedule; tools/nt_stamps.hip builds variants):
    // P1 / P3 MFMAs in phases 1 / 3, one fragment read per RS1 / RS3 MFMAs, phase 2 = the rest with
    // the 16 DMAs spread evenly; M0SPLIT puts one MFMA between each DMA's M0 write and its load
    constexpr int P1 = PRA_NT_P1, RS1 = PRA_NT_RS1, P3 = PRA_NT_P3, RS3 = PRA_NT_RS3;
    constexpr int MD = (128 - P1 - P3) / 16;
    static_assert(P1 >= 16 * RS1 && P3 >= 16 * RS3 && P3 <= 64 && (128 - P1 - P3) % 16 == 0 && MD >= 2,
                  "NT schedule knobs");
    auto dma_lds = [&](int b, int d) __attribute__((always_inline)) {
      return ldsw + (uint32_t)((b * 2 + (d >> 3)) * TILE64 * sizeof(T) + (d & 7) * 4 * 1024);
    };
    // PRA_NT_VOFF: each DMA's row offset lives in a VGPR (16 loop-invariant registers), so the SGPR
    // base only moves once per chunk and operand instead of once per DMA (hipBLASLt's form)
    uint32_t vo[PRA_NT_VOFF ? 16 : 1];
    if constexpr (PRA_NT_VOFF) {
#pragma unroll
      for (int d = 0; d < 16; ++d)
        vo[d] = d >= 8 ? vob64 + (uint32_t)((long)row_b64(d & 7) * ldb * (long)sizeof(T))
                       : voa64 + (uint32_t)((long)row_a64(d & 7) * lda * (long)sizeof(T));
    }
    auto dma_go = [&](int c, int d) __attribute__((always_inline)) {
      c = min(c, c1 - 1);
      const int i = d & 7;
      if constexpr (PRA_NT_VOFF)
        dma16s_go((d >= 8 ? Bb : Ab) + (long)c * 64, vo[PRA_NT_VOFF ? d : 0]);
      else if (d >= 8)
        dma16s_go(Bb + (long)row_b64(i) * ldb + (long)c * 64, vob64);
      else
        dma16s_go(Ab + (long)row_a64(i) * lda + (long)c * 64, voa64);
    };
    auto chunk = [&](auto b_c, int t) __attribute__((always_inline)) {
      constexpr int b = decltype(b_c)::value;
      // phase 1: MFMA 0..P1-1; k-substep-1 fragments of chunk t (B first: MFMA 64..71 need fb1[0..7])
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
#pragma unroll
        for (int k = 0; k < RS1; ++k) mf(r * RS1 + k);
        if (r < 8)
          fb1[r] = fragB(b, 1, r);
        else
          fa1[r - 8] = fragA(b, 1, r - 8);
        __builtin_amdgcn_sched_group_barrier(0x008, RS1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int q = 16 * RS1; q < P1; ++q) mf(q);
      if constexpr (P1 > 16 * RS1) __builtin_amdgcn_sched_group_barrier(0x008, P1 - 16 * RS1, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0), visible to the compiler's wait counting
      PRA_NT_STAMP(ts1);
      __builtin_amdgcn_s_barrier();  // every wave holds chunk t: buffer b is free
      PRA_NT_STAMP(ts2);
      __builtin_amdgcn_sched_barrier(0);
      // phase 2: MFMA P1..127-P3 with the 16 DMA instructions of chunk t + 2 into buffer b
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        if constexpr (PRA_NT_M0SPLIT) {
          m0_set(dma_lds(b, d));
          __builtin_amdgcn_sched_barrier(0);
          mf(P1 + MD * d);
          __builtin_amdgcn_sched_barrier(0);
          dma_go(t + 2, d);
#pragma unroll
          for (int k = 1; k < MD; ++k) mf(P1 + MD * d + k);
        } else {
          dma(b, t + 2, d);
#pragma unroll
          for (int k = 0; k < MD; ++k) mf(P1 + MD * d + k);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      PRA_NT_STAMP(ts3);
      wait_vm<16>();  // chunk t + 1 landed (chunk t + 2's 16 instructions stay in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      PRA_NT_STAMP(ts4);
#ifdef PRA_NT_STAMPS
      sw1 += ts2 - ts1; sp2 += ts3 - ts2; sw2 += ts4 - ts3;
      if (ts4p) sp31 += ts1 - ts4p;
      ts4p = ts4; ++nch;
#endif
      __builtin_amdgcn_sched_barrier(0);
      // phase 3: MFMA 128-P3..127 (k-substep 1: fa0 / fb0 are free); k-substep-0 fragments of
      // chunk t + 1 (buffer b ^ 1) in first-use order
#pragma unroll
      for (int r = 0; r < 16; ++r) {
#pragma unroll
        for (int k = 0; k < RS3; ++k) mf(128 - P3 + r * RS3 + k);
        if (r == 0)
          fa0[0] = fragA(b ^ 1, 0, 0);
        else if (r < 9)
          fb0[r - 1] = fragB(b ^ 1, 0, r - 1);
        else
          fa0[r - 8] = fragA(b ^ 1, 0, r - 8);
        __builtin_amdgcn_sched_group_barrier(0x008, RS3, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int q = 128 - P3 + 16 * RS3; q < 128; ++q) mf(q);
      if constexpr (P3 > 16 * RS3) __builtin_amdgcn_sched_group_barrier(0x008, P3 - 16 * RS3, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    // PRA_NT_SCHED 1: hipBLASLt's 256x256x64 DTL/PGR2 chunk order (read off its gfx950 ISA), four
    // barriers per chunk so every phase frees or publishes one operand half:
    //   MFMA 0-19    B k-substep-1 reads of chunk t (1 per 2 MFMA); lgkmcnt(0) + barrier 1: B half free
    //   MFMA 20-50   5 B DMAs of chunk t + 2, A k-substep-1 reads; lgkmcnt(0) + barrier 2: A half free
    //   MFMA 51-67   3 B + 2 A DMAs; vmcnt(18) + barrier 3: chunk t + 1's B half landed
    //   MFMA 68-104  B k-substep-0 reads of chunk t + 1 (fb0 is free after MFMA 63), 5 A DMAs;
    //                vmcnt(15) + barrier 4: chunk t + 1 landed
    //   MFMA 105-127 A k-substep-0 reads of chunk t + 1, the last A DMA
    // Every DMA's M0 write sits one MFMA ahead of its load.
    auto chunk4 = [&](auto b_c, int t) __attribute__((always_inline)) {
      constexpr int b = decltype(b_c)::value;
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, 128>([&](auto q_c) __attribute__((always_inline)) {
        constexpr int q = decltype(q_c)::value;
        mf(q);
        constexpr int rd = nt4_read_at(q), dd = nt4_dma_at(q), md = nt4_dma_at(q + 1);
        if constexpr (rd >= 0) {
          constexpr int g = rd >> 3, r = rd & 7;
          if constexpr (g == 0) fb1[r] = fragB(b, 1, r);
          if constexpr (g == 1) fa1[r] = fragA(b, 1, r);
          if constexpr (g == 2) fb0[r] = fragB(b ^ 1, 0, r);
          if constexpr (g == 3) fa0[r] = fragA(b ^ 1, 0, r);
        }
        if constexpr (dd >= 0) dma_go(t + 2, dd);
        if constexpr (md >= 0) m0_set(dma_lds(b, md));  // one MFMA ahead of its load
        if constexpr (q == 19 || q == 50) {
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
          if constexpr (q == 19) PRA_NT_STAMP(ts1);
          __builtin_amdgcn_s_barrier();
          if constexpr (q == 19) PRA_NT_STAMP(ts2);
        }
        if constexpr (q == 67) {
          PRA_NT_STAMP(ts3);
          wait_vm<18>();
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          PRA_NT_STAMP(ts4);
        }
        if constexpr (q == 104) {
          wait_vm<15>();
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
      });
#ifdef PRA_NT_STAMPS
      sw1 += ts2 - ts1; sp2 += ts3 - ts2; sw2 += ts4 - ts3;
      if (ts4p) sp31 += ts1 - ts4p;
      ts4p = ts4; ++nch;
#endif
    };
    // four chunks per iteration with compile-time buffers (a 2-chunk body with a conditional
    // second chunk broke the accumulator register coalescing: 100+ spills)
    for (int t = c0; t < c1; t += 4) {
      if constexpr (PRA_NT_SCHED == 1) {
        if (t < c1) chunk4(IC<0>{}, t);
        if (t + 1 < c1) chunk4(IC<1>{}, t + 1);
        if (t + 2 < c1) chunk4(IC<0>{}, t + 2);
        if (t + 3 < c1) chunk4(IC<1>{}, t + 3);
      } else {
        if (t < c1) chunk(IC<0>{}, t);
        if (t + 1 < c1) chunk(IC<1>{}, t + 1);
        if (t + 2 < c1) chunk(IC<0>{}, t + 2);
        if (t + 3 < c1) chunk(IC<1>{}, t + 3);
      }
    }
    // no LDS-DMA may land after this point, and no wave may still read a buffer the split
    // tail's flag overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PRA_NT_STAMP(tk2);
  };

  auto run = [&](long m0, long n0, int k0, int k1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* Ab = A + m0 * lda;
    const T* Bb = B + (EPI == 1 ? n0 / 2 : n0) * ldb;  // EPI 1: 128 features per 256-row tile
    auto dma = [&](int s, int kt, int u) __attribute__((always_inline)) {
      const int i = u >> 1;
      const uint32_t lds = ldsw + (uint32_t)((s * 2 * TILE + (u & 1) * TILE) * sizeof(T) + i * 4 * 1024);
      const T* g = (u & 1) ? Bb + (long)kt * BK : Ab + (long)kt * BK;
      dma16s(g, (u & 1) ? offb[i] : offa[i], lds);
    };
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
#pragma unroll
      for (int u = 0; u < 2 * NI; ++u) dma(p, min(k0 + p, k1 - 1), u);
    wait_vm<2 * NI * (NS - 2)>();  // stage k0 landed; the younger stages stay in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      fa0[f] = frag(smem, foa + 1024 * f);
      fb0[f] = frag(smem + TILE, fob + 1024 * f);
    }
    // step kt (slot s, fragments in ca/cb): m-blocks 0..3 (32 MFMAs); counted wait + barrier
    // publish stage kt + 1 and free the slot of stage kt - 1; m-blocks 4..7 in 8 groups of 4
    // MFMAs, each with 2 fragment reads of stage kt + 1 and one DMA instruction of stage kt + 4.
    auto step = [&](auto s_c, V8<T>(&ca)[8], V8<T>(&cb)[8], V8<T>(&na)[8], V8<T>(&nb)[8], int kt) {
      constexpr int s = decltype(s_c)::value % NS, sn = (s + 1) % NS, sd = (s + NS - 1) % NS;
      const T* nta = smem + sn * 2 * TILE;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
      wait_vm<2 * NI * (NS - 3)>();  // stage kt + 1 landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int kd = min(kt + NS - 1, k1 - 1);
#pragma unroll
      for (int gi = 0; gi < 8; ++gi) {
        na[gi] = frag(nta, foa + 1024 * gi);
        nb[gi] = frag(nta + TILE, fob + 1024 * gi);
        const int i = 4 + (gi >> 1);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int j = 4 * (gi & 1) + jj;
          acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        dma(sd, kd, gi);
      }
    };
    constexpr int UNR = 10;  // lcm(NS, 2): compile-time ring slot and fragment register set
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
    // no LDS-DMA may land after this point, and no wave may still read a slot the next
    // prologue overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  const int ndp = nwg - n_split;  // whole tiles first, then n_split tiles x S split units
  const bool split = (int)blockIdx.x >= ndp;
  int lin, k0 = 0, k1 = nk, part = 0, st = 0;
  if (!split) {
    lin = xcd_remap(blockIdx.x, ndp);
  } else {
    const int u = xcd_remap((int)blockIdx.x - ndp, n_split * S);
    part = u / n_split;
    st = u % n_split;
    lin = ndp + st;
    k0 = (int)((long)nk * part / S);
    k1 = (int)((long)nk * (part + 1) / S);
  }
  long m0, n0;
  tile_origin(lin, tiles_m, tiles_n, m0, n0);
  PRA_NT_STAMP(tk0);
  if constexpr (KB == 64)
    run2b(m0, n0, k0, k1);
  else
    run(m0, n0, k0, k1);
  if (split) {
    // fp32 partial in register order (thread t's register r at r * NTH + t); the last arriver of
    // the tile sums the S partials in part order and runs the epilogue (deterministic)
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
#ifdef PRA_NT_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores have left the wave
  PRA_NT_STAMP(tk3);
  if (lane == 0 && pra_nt_stamp_out) {
    unsigned long long* o = pra_nt_stamp_out + ((long)blockIdx.x * 4 + wid) * 8;
    o[0] = sw1; o[1] = sp2; o[2] = sw2; o[3] = sp31; o[4] = nch; o[5] = tk2 - tk1; o[6] = tk1 - tk0;
    o[7] = tk3 - tk2;
  }
#endif
}

__global__ __launch_bounds__(256) void zero_i32_kernel(int* __restrict__ p, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0;
}

}  // namespace nt
}  // namespace pra

extern "C" {

// fp32 partial-tile floats and tickets the split tail of an [M, N, K] NT GEMM needs (0 = none)
long pra_gemm_nt_ws_floats(int M, int N, int K, int cus) {
  using namespace pra::gm;
  const int nwg = (M / BM) * (N / BN);
  const int S = pra::gemm_tail_split(nwg, cus, K / BK, 2);
  return S > 1 ? (long)(nwg % cus) * S * BM * BN : 0;
}
int pra_gemm_nt_ticket_count(int M, int N, int K, int cus) {
  using namespace pra::gm;
  const int nwg = (M / BM) * (N / BN);
  return pra::gemm_tail_split(nwg, cus, K / BK, 2) > 1 ? nwg % cus : 0;
}

// C = A B^T with the epilogue `epi` (see the file comment). A [M][K] (row stride lda), B [N][K]
// (ldb), C [M][N] (ldc; EPI 1: gu [M][2F] with N = 2F, EPI 2: gu [M][2F] with N = F).
// ws/tickets: sized by pra_gemm_nt_ws_floats / pra_gemm_nt_ticket_count (null when those are 0).
hipError_t pra_gemm_nt(int dtype, int epi, const void* A, const void* B, void* C, int M, int N, int K, long lda,
                       long ldb, long ldc, void* c2, long ldc2, int F, const void* tab, int S, int D, int nrot,
                       float* ws, int* tickets, int cus, hipStream_t s) {
  using namespace pra::gm;
  if (M % BM || N % BN || K % BK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8 || cus <= 0) return hipErrorInvalidValue;
  if (epi < 0 || epi > 3) return hipErrorInvalidValue;
  if (epi == 1 && (N != 2 * F || F % 128 || c2 == nullptr || ldc2 % 8)) return hipErrorInvalidValue;
  if (epi == 2 && (F != N || ldc < 2L * F)) return hipErrorInvalidValue;
  if (epi == 3 && (tab == nullptr || S <= 0 || D % 8 || D <= 0 || nrot % D || nrot > N)) return hipErrorInvalidValue;
  // per-lane DMA offsets are 32-bit byte offsets from the tile's row base
  const long brows = epi == 1 ? (long)F + 128 : 256;
  if (255L * lda * 2 + 2L * K > 0xffffffffL || brows * ldb * 2 + 2L * K > 0xffffffffL) return hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // 128-B-row chunks whenever K allows; the 64-B-row stage ring serves K % 64 == 32
  const int KBx = K % 64 == 0 ? 64 : 32;
  const int Ssplit = pra::gemm_tail_split(nwg, cus, K / KBx, 2);
  const int n_split = Ssplit > 1 && ws && tickets ? nwg % cus : 0;
  const int Sx = n_split ? Ssplit : 1;
  if (n_split)
    hipLaunchKernelGGL(pra::nt::zero_i32_kernel, dim3((n_split + 255) / 256), dim3(256), 0, s, tickets, n_split);
  const dim3 grid(nwg - n_split + n_split * Sx), block(NTH);
#define PRA_NT_LAUNCH(TT, E)                                                                                  \
  {                                                                                                           \
    pra::nt::Epi<TT> ep{(TT*)c2, ldc2, F, (const float2*)tab, S, D, nrot};                                    \
    if (KBx == 64)                                                                                            \
      hipLaunchKernelGGL((pra::nt::gemm_nt_kernel<TT, E, 64>), grid, block, 0, s, (const TT*)A, (const TT*)B,  \
                         (TT*)C, M, N, K, lda, ldb, ldc, ep, ws, tickets, n_split, Sx);                       \
    else                                                                                                      \
      hipLaunchKernelGGL((pra::nt::gemm_nt_kernel<TT, E, 32>), grid, block, 0, s, (const TT*)A, (const TT*)B,  \
                         (TT*)C, M, N, K, lda, ldb, ldc, ep, ws, tickets, n_split, Sx);                       \
  }
#define PRA_NT_EPI(TT)                   \
  switch (epi) {                         \
    case 0: PRA_NT_LAUNCH(TT, 0) break;  \
    case 1: PRA_NT_LAUNCH(TT, 1) break;  \
    case 2: PRA_NT_LAUNCH(TT, 2) break;  \
    default: PRA_NT_LAUNCH(TT, 3) break; \
  }
  if (dtype == pra::kBF16) {
    PRA_NT_EPI(__bf16)
  } else if (dtype == pra::kF16) {
    PRA_NT_EPI(_Float16)
  } else {
    return hipErrorInvalidValue;
  }
#undef PRA_NT_EPI
#undef PRA_NT_LAUNCH
  return hipGetLastError();
}

}  // extern "C"

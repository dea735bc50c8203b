// Flash attention forward + deterministic backward for fp32 models (--model-dtype fp32) on gfx950,
// head_dim 64/128, causal or full, native GQA. Same algorithm and kernel split as attention.hip
// (replaces the reference's SDPA call for fp32 tensors, reference model.py:179-230),
// but every product runs on the f32-input MFMA v_mfma_f32_32x32x2_f32: exact fp32 products at the
// f32 vector rate (157 TF/s, 1/16 of bf16), so an fp32 model keeps fp32 attention math instead of
// rounding q/k/v to 16 bits, and never materialises the S x S score matrix.
//
// Operand layouts of v_mfma_f32_32x32x2_f32 (one block): A[i][k] from lane i + 32k, B[k][j] from
// lane j + 32k, C[i][j] in lane j + 32 h, register r for row i = crow(r, h). An MFMA sums over its
// two k, so a product over a long dimension may visit that dimension in any order as long as A and
// B agree. The kernels use two orders:
//  * over head_dim d: k-step s of the half-wave h2 takes d = (D/2) h2 + s, so a lane's operand is a
//    contiguous run of one row (Q and dO rows live in registers, K / V rows are float4 LDS reads);
//  * over keys / queries of a 32-row accumulator: k-step s of half-wave h2 takes row crow(s, h2),
//    exactly the row that lane's register s of the previous product's accumulator holds, so P and
//    dS feed the next MFMA straight from their accumulator registers.
//
// Kernels (one wave = 32 rows on the MFMA lanes):
//  * fwd:  4 waves x 32 queries; S^T = K Q^T (query on the lane: lane-local softmax, one
//          permlane32 swap per row reduction), online softmax, O^T += V^T P^T; 64-key K/V tiles in
//          LDS with 4-float row padding (conflict-free float4 row reads and float column reads).
//  * dQ:   same shape; also writes delta = rowsum(dO * O) for the dK/dV kernel.
//  * dK/dV: 4 waves x 32 keys, each wave's K/V rows in registers (one wave per SIMD, 512-register
//          file); loops over the query heads of its kv head and 32-query Q/dO tiles in LDS.
// Determinism: no atomics; every output element has one writer and a fixed summation order.
#include "common.h"

namespace pra {
namespace attnf {

__device__ __forceinline__ f32x16 mfma2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ROWS x D fp32 rows of a [.., ld]-strided tensor into an LDS tile with row stride D + 4 floats
// (block-wide, float4 per thread per pass; rows >= nvalid are zero-filled)
template <int D, int ROWS>
__device__ __forceinline__ void stage(float* tile, const float* g, long ld, int row0, int nvalid) {
  constexpr int CH = D / 4, LD = D + 4;
#pragma unroll
  for (int i = 0; i < ROWS * CH / 256; ++i) {
    const int idx = i * 256 + threadIdx.x, r = idx / CH, c = idx % CH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row0 + r < nvalid) v = *reinterpret_cast<const float4*>(g + (long)(row0 + r) * ld + 4 * c);
    *reinterpret_cast<float4*>(tile + r * LD + 4 * c) = v;
  }
}

// half-row of a global row into registers: x[s] = row[(D/2) h2 + s]
template <int D>
__device__ __forceinline__ void load_half(float (&x)[D / 2], const float* row, int h2, bool ok) {
#pragma unroll
  for (int j = 0; j < D / 8; ++j) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) v = *reinterpret_cast<const float4*>(row + (D / 2) * h2 + 4 * j);
    x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
  }
}

// acc (+)= Rows x^T over d: A = the LDS tile's rows r0 .. r0+31 (lane row l32), B = x, the lane's
// half-row of the other operand (the accumulator's column index is x's row)
template <int D>
__device__ __forceinline__ f32x16 dot_rows(f32x16 acc, const float* tile, int r0, int l32, int h2,
                                           const float (&x)[D / 2]) {
  const float* p = tile + (r0 + l32) * (D + 4) + (D / 2) * h2;
#pragma unroll
  for (int j = 0; j < D / 8; ++j) {
    const float4 t = *reinterpret_cast<const float4*>(p + 4 * j);
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma2(tv[e], x[4 * j + e], acc);
  }
  return acc;
}

// Row-per-lane epilogue of a 32 x D accumulator X^T (lane l32 = row, block db register r = column
// 32 db + crow(r, h2)): 4 contiguous floats per register quad -> float4 stores.
template <int NDB>
__device__ __forceinline__ void store_rows(const f32x16 (&acc)[NDB], float f, float* p, bool ok, int h2) {
  if (!ok) return;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(p + 32 * db + 8 * q + 4 * h2) =
          make_float4(acc[db][4 * q] * f, acc[db][4 * q + 1] * f, acc[db][4 * q + 2] * f, acc[db][4 * q + 3] * f);
}

// ======================================================================================
// Forward: block = 4 waves x 32 queries, 64-key tiles.
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fwd_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                     const float* __restrict__ V, float* __restrict__ O,
                                                     float* __restrict__ LSE, int S, int Hq, int Hkv, long ldq,
                                                     long ldk, long ldv, long ldo, float scale_log2, int skv) {
  constexpr int KT = 64, QT = 128, NDB = D / 32, LD = D + 4;
  __shared__ __attribute__((aligned(16))) float Ks[KT * LD];
  __shared__ __attribute__((aligned(16))) float Vs[KT * LD];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = S / QT, BH = gridDim.x / nqt;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heavy (late) query tiles first
  const int bh = blockIdx.x % BH, hq = bh % Hq, b = bh / Hq, hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + 32 * wid, qrow = qw + l32;
  const float* Kb = K + (long)b * S * ldk + hk * D;
  const float* Vb = V + (long)b * S * ldv + hk * D;

  float qr[D / 2];
  load_half<D>(qr, Q + ((long)b * S + qrow) * ldq + hq * D, h2, true);
  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m_i = -INFINITY, l_i = 0.f;
  const int kend = CAUSAL ? q0 + QT : S;
  for (int k0 = 0; k0 < kend; k0 += KT) {
    __syncthreads();
    stage<D, KT>(Ks, Kb, ldk, k0, S);
    stage<D, KT>(Vs, Vb, ldv, k0, S);
    __syncthreads();
    if (CAUSAL && k0 > qw + 31) continue;  // wave-uniform: every key of the tile is masked
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = dot_rows<D>(f32x16{}, Ks, 32 * kb, l32, h2, qr);  // S^T = K Q^T
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + 32 * kb + crow(r, h2);
        if ((CAUSAL && key > qrow) || (!CAUSAL && key >= skv)) s[kb][r] = -INFINITY;
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    mx = half_max(mx) * scale_log2;
    if (mx > m_i) {  // exact online rescale (per lane: each lane owns its query row)
      const float alpha = fexp2(m_i - mx);
      l_i *= alpha;
#pragma unroll
      for (int i = 0; i < NDB; ++i) o[i] *= alpha;
      m_i = mx;
    }
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[kb][r] = fexp2(fmaf(s[kb][r], scale_log2, -m_i));
        rs += s[kb][r];
      }
    l_i += half_sum(rs);
    // O^T[d][q] += V^T[d][key] P^T[key][q]: k-step r of half-wave h2 = key crow(r, h2)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db] = mfma2(Vs[(32 * kb + crow(r, h2)) * LD + 32 * db + l32], s[kb][r], o[db]);
  }
  store_rows<NDB>(o, 1.f / l_i, O + ((long)b * S + qrow) * ldo + hq * D, true, h2);
  if (h2 == 0) LSE[((long)b * Hq + hq) * S + qrow] = (m_i + __log2f(l_i)) * 0.69314718055994531f;
}

// ======================================================================================
// Backward dQ: block = 4 waves x 32 queries, 64-key tiles; writes delta = rowsum(dO * O).
//   S^T = K Q^T, dP^T = V dO^T (query on the lane), dQ^T += K^T dS^T
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void bwd_dq_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                        const float* __restrict__ V, const float* __restrict__ dO,
                                                        const float* __restrict__ O, const float* __restrict__ LSE,
                                                        float* __restrict__ Delta, float* __restrict__ dQ, int S, int Hq,
                                                        int Hkv, long ldq, long ldk, long ldv, long lddo, long ldo,
                                                        long lddq, float scale, float scale_log2, int skv) {
  constexpr int KT = 64, QT = 128, NDB = D / 32, LD = D + 4;
  __shared__ __attribute__((aligned(16))) float Ks[KT * LD];
  __shared__ __attribute__((aligned(16))) float Vs[KT * LD];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = S / QT, BH = gridDim.x / nqt;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH, hq = bh % Hq, b = bh / Hq, hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + 32 * wid, qrow = qw + l32;
  const float* Kb = K + (long)b * S * ldk + hk * D;
  const float* Vb = V + (long)b * S * ldv + hk * D;

  float qr[D / 2], dr[D / 2];
  load_half<D>(qr, Q + ((long)b * S + qrow) * ldq + hq * D, h2, true);
  load_half<D>(dr, dO + ((long)b * S + qrow) * lddo + hq * D, h2, true);
  float dl;
  {
    float orow[D / 2];
    load_half<D>(orow, O + ((long)b * S + qrow) * ldo + hq * D, h2, true);
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < D / 2; ++s) part = fmaf(orow[s], dr[s], part);
    dl = half_sum(part);
    if (h2 == 0) Delta[((long)b * Hq + hq) * S + qrow] = dl;
  }
  const float lse2 = LSE[((long)b * Hq + hq) * S + qrow] * 1.4426950408889634f;
  f32x16 dq[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dq[i] = f32x16{};
  const int kend = CAUSAL ? q0 + QT : S;
  for (int k0 = 0; k0 < kend; k0 += KT) {
    __syncthreads();
    stage<D, KT>(Ks, Kb, ldk, k0, S);
    stage<D, KT>(Vs, Vb, ldv, k0, S);
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (CAUSAL && k0 + 32 * kb > qw + 31) continue;
      f32x16 s = dot_rows<D>(f32x16{}, Ks, 32 * kb, l32, h2, qr);
      f32x16 dp = dot_rows<D>(f32x16{}, Vs, 32 * kb, l32, h2, dr);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + 32 * kb + crow(r, h2);
        float p = fexp2(fmaf(s[r], scale_log2, -lse2));
        if ((CAUSAL && key > qrow) || (!CAUSAL && key >= skv)) p = 0.f;
        dp[r] = p * (dp[r] - dl);
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[db] = mfma2(Ks[(32 * kb + crow(r, h2)) * LD + 32 * db + l32], dp[r], dq[db]);
    }
  }
  store_rows<NDB>(dq, scale, dQ + ((long)b * S + qrow) * lddq + hq * D, true, h2);
}

// ======================================================================================
// Backward dK/dV: block = (b, kv head, 128 keys), 4 waves x 32 keys with the wave's K and V rows in
// registers; loops over the kv head's query heads and 32-query Q/dO tiles staged in LDS.
//   S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void bwd_dkdv_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    float* __restrict__ dK, float* __restrict__ dV, int S, int Hq, int Hkv, long ldq, long ldk, long ldv,
    long lddo, long lddk, long lddv, float scale, float scale_log2, int skv) {
  constexpr int KB = 128, QT = 32, NDB = D / 32, LD = D + 4;
  __shared__ __attribute__((aligned(16))) float Qs[QT * LD];
  __shared__ __attribute__((aligned(16))) float Ds[QT * LD];
  __shared__ float rowc[2][QT];  // lse * log2(e) | delta of the tile's queries
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nkb = S / KB, BH = gridDim.x / nkb;
  const int kbk = (int)(blockIdx.x / BH);  // causal: early key blocks have the most work
  const int bh = blockIdx.x % BH, hk = bh % Hkv, b = bh / Hkv, nrep = Hq / Hkv;
  const int k0 = kbk * KB, kw = k0 + 32 * wid, krow = kw + l32;

  float kr[D / 2], vr[D / 2];
  load_half<D>(kr, K + ((long)b * S + krow) * ldk + hk * D, h2, true);
  load_half<D>(vr, V + ((long)b * S + krow) * ldv + hk * D, h2, true);
  f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) { dkt[i] = f32x16{}; dvt[i] = f32x16{}; }
  const bool kvalid = CAUSAL || krow < skv;
  const int qstart = CAUSAL ? k0 : 0;
  for (int hq = hk * nrep; hq < (hk + 1) * nrep; ++hq) {
    const float* Qh = Q + (long)b * S * ldq + hq * D;
    const float* Dh = dO + (long)b * S * lddo + hq * D;
    for (int q0 = qstart; q0 < S; q0 += QT) {
      __syncthreads();
      stage<D, QT>(Qs, Qh, ldq, q0, S);
      stage<D, QT>(Ds, Dh, lddo, q0, S);
      if (threadIdx.x < 2 * QT) {
        const int w = threadIdx.x / QT, i = threadIdx.x % QT;
        const long o = ((long)b * Hq + hq) * S + q0 + i;
        rowc[w][i] = w ? Delta[o] : LSE[o] * 1.4426950408889634f;
      }
      __syncthreads();
      if (CAUSAL && q0 + QT - 1 < kw) continue;  // wave-uniform: every query precedes the wave's keys
      f32x16 s = dot_rows<D>(f32x16{}, Qs, 0, l32, h2, kr);   // A = Q rows, B = K^T
      f32x16 dp = dot_rows<D>(f32x16{}, Ds, 0, l32, h2, vr);  // A = dO rows, B = V^T
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = crow(r, h2);
        float p = fexp2(fmaf(s[r], scale_log2, -rowc[0][qi]));
        if ((CAUSAL && q0 + qi < krow) || !kvalid) p = 0.f;
        s[r] = p;
        dp[r] = p * (dp[r] - rowc[1][qi]);
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = crow(r, h2);
          dvt[db] = mfma2(Ds[qi * LD + 32 * db + l32], s[r], dvt[db]);
          dkt[db] = mfma2(Qs[qi * LD + 32 * db + l32], dp[r], dkt[db]);
        }
    }
  }
  store_rows<NDB>(dkt, scale, dK + ((long)b * S + krow) * lddk + hk * D, true, h2);
  store_rows<NDB>(dvt, 1.f, dV + ((long)b * S + krow) * lddv + hk * D, true, h2);
}

}  // namespace attnf
}  // namespace pra

extern "C" {

// fp32 tensors [B, S, H, D] (token stride ld*); S % 128 == 0 (the binding zero-pads), D 64 or 128.
hipError_t pra_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, float* lse, int B, int S, int Hq,
                            int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal, int skv,
                            hipStream_t st) {
  using namespace pra::attnf;
  if (S % 128 || (D != 64 && D != 128) || Hq % Hkv || skv <= 0 || skv > S) return hipErrorInvalidValue;
  if (ldq % 4 || ldk % 4 || ldv % 4 || ldo % 4) return hipErrorInvalidValue;
  const dim3 grid((S / 128) * Hq * B), block(256);
  const float sl2 = scale * 1.4426950408889634f;
#define LAUNCH(DD, CC) \
  hipLaunchKernelGGL((fwd_kernel<DD, CC>), grid, block, 0, st, q, k, v, o, lse, S, Hq, Hkv, ldq, ldk, ldv, ldo, sl2, skv)
  if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
  else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  return hipGetLastError();
}

hipError_t pra_attn_bwd_f32(const float* q, const float* k, const float* v, const float* o, const float* dout,
                            const float* lse, float* delta, float* dq, float* dk, float* dv, int B, int S, int Hq,
                            int Hkv, int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk,
                            long lddv, float scale, int causal, int skv, hipStream_t st) {
  using namespace pra::attnf;
  if (S % 128 || (D != 64 && D != 128) || Hq % Hkv || skv <= 0 || skv > S) return hipErrorInvalidValue;
  if (ldq % 4 || ldk % 4 || ldv % 4 || ldo % 4 || lddo % 4 || lddq % 4 || lddk % 4 || lddv % 4)
    return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  {  // dQ first: it writes delta
    const dim3 grid((S / 128) * Hq * B);
#define LAUNCH(DD, CC)                                                                                      \
  hipLaunchKernelGGL((bwd_dq_kernel<DD, CC>), grid, dim3(256), 0, st, q, k, v, dout, o, lse, delta, dq, S, Hq, \
                     Hkv, ldq, ldk, ldv, lddo, ldo, lddq, scale, sl2, skv)
    if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
    else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  }
  {
    const dim3 grid((S / 128) * Hkv * B);
#define LAUNCH(DD, CC)                                                                                         \
  hipLaunchKernelGGL((bwd_dkdv_kernel<DD, CC>), grid, dim3(256), 0, st, q, k, v, dout, lse, delta, dk, dv, S, Hq, \
                     Hkv, ldq, ldk, ldv, lddo, lddk, lddv, scale, sl2, skv)
    if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
    else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  }
  return hipGetLastError();
}

}  // extern "C"

// Flash attention forward + deterministic backward for gfx950 (CDNA4), bf16, head_dim 64/128,
// causal or full, native GQA (kv head = q head / (Hq/Hkv); no repeat_kv copies).
//
// Replaces the reference's SDPA / flash-attn call (reference model.py:179-230; N1/N2 in
// SURVEY §2.2). Tensors are read straight out of the fused QKV activation: q/k/v are
// [B, S, H, D] views with an arbitrary token stride, so no transpose/contiguous copies.
//
// Design (all MFMA work on v_mfma_f32_32x32x16_bf16, wave64):
//  * forward: 256-thread block = 4 waves = 128 query rows (32 per wave); K/V tiles of 64 keys
//    staged global->regs->LDS, double-buffered, one barrier per tile. "Swapped" products:
//    S^T = K Q^T puts one query per lane, so softmax row statistics are lane-local (plus one
//    xor-32 exchange), and O^T = V^T P^T reuses the S^T accumulator registers directly as the
//    B operand (bf16-packed). V^T fragments come from ds_read_b64_tr_b16 (hardware transpose).
//  * every LDS tile uses one XOR-swizzled image that is conflict-free for both ds_read_b128
//    row reads and ds_read_b64_tr_b16 transposed reads (row r, 16-B chunk c -> c ^ x(r)).
//  * backward is split into two deterministic kernels (no float atomics, so a resumed run is
//    bit-identical to an uninterrupted one): dK/dV (keys resident per wave, loop over query
//    tiles and over the Hq/Hkv query heads of the kv head) and dQ (queries resident, loop
//    over key tiles). P is recomputed from the saved log-sum-exp.
#include "common.h"

namespace pra {
namespace attn {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// XOR swizzle of 16-B chunk c in row r (see header). D=128: 16 chunks/256-B rows;
// D=64: 8 chunks/128-B rows.
template <int D>
__device__ __forceinline__ int swz(int r, int c) {
  if constexpr (D == 128) return c ^ (((r & 3) << 2) | ((r >> 2) & 3));
  else return c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
}
template <int D>
__device__ __forceinline__ int lds_off(int r, int c) {  // element offset of chunk c of row r
  return r * D + swz<D>(r, c) * 8;
}

__device__ __forceinline__ bf16x8 lds_row8(const __bf16* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
__device__ __forceinline__ i16x4 tr4(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
}

// Transposed operand fragment for the "accumulator as next operand" pattern: for a tile
// stored [rows=k][cols=n] in LDS, lane l receives column n = c0 + (l&31) and the 8 rows
// k = r0 + 8*(j>>2) + 4*(l>>5) + (j&3), j=0..7 (matching the permuted k order of a 32x32
// accumulator reused as an operand, cdna guide §3).
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* tile, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int row = r0 + 4 * (g >> 1) + q;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const int c = col >> 3, w = col & 7;
  i16x4 lo = tr4(tile + lds_off<D>(row, c) + w);
  i16x4 hi = tr4(tile + lds_off<D>(row + 8, c) + w);
  i16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Stage ROWS x D rows of a [.., ld]-strided bf16 tensor into registers (global loads only).
template <int D, int ROWS>
struct Stage {
  static constexpr int CH = D / 8;
  static constexpr int CPT = ROWS * CH / 256;
  uint4 r[CPT];
  __device__ __forceinline__ void load(const __bf16* g, long ld, int row0, int nrows_valid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = i * 256 + threadIdx.x;
      const int row = idx / CH, c = idx % CH;
      if (row0 + row < nrows_valid)
        r[i] = *reinterpret_cast<const uint4*>(g + (long)(row0 + row) * ld + c * 8);
      else
        r[i] = make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(__bf16* tile) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = i * 256 + threadIdx.x;
      const int row = idx / CH, c = idx % CH;
      *reinterpret_cast<uint4*>(tile + lds_off<D>(row, c)) = r[i];
    }
  }
};

// C-layout row of register r for lane half h (32x32 accumulator)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ======================================================================================
// Forward
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K,
                                                     const __bf16* __restrict__ V, __bf16* __restrict__ O,
                                                     float* __restrict__ LSE, int S, int Hq, int Hkv, long ldq,
                                                     long ldk, long ldv, long ldo, float scale_log2) {
  constexpr int KT = 64, QT = 128;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][2][KT * D];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = (S + QT - 1) / QT;
  const int BH = gridDim.x / nqt;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heavy (late) query tiles first
  const int bh = blockIdx.x % BH;
  const int hq = bh % Hq, b = bh / Hq;
  const int hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + wid * 32;

  const __bf16* Qb = Q + (long)b * S * ldq + hq * D;
  const __bf16* Kb = K + (long)b * S * ldk + hk * D;
  const __bf16* Vb = V + (long)b * S * ldv + hk * D;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[qw + l32][16 ks + 8 h2 .. +7]
  bf16x8 qf[NKS];
  const int qrow = qw + l32;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (qrow < S)
      qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (long)qrow * ldq + 16 * ks + 8 * h2);
    else
      qf[ks] = bf16x8{};
  }

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m_i = -INFINITY, l_i = 0.f;

  const int kend = CAUSAL ? min(S, q0 + QT) : S;
  const int nkt = (kend + KT - 1) / KT;

  Stage<D, KT> sk, sv;
  sk.load(Kb, ldk, 0, S);
  sv.load(Vb, ldv, 0, S);
  sk.store(smem[0][0]);
  sv.store(smem[0][1]);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const int k0 = kt * KT;
    if (kt + 1 < nkt) {
      sk.load(Kb, ldk, k0 + KT, S);
      sv.load(Vb, ldv, k0 + KT, S);
    }
    if (!(CAUSAL && k0 > qw + 31)) {
      const __bf16* kt_lds = smem[cur][0];
      const __bf16* vt_lds = smem[cur][1];
      f32x16 s[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        s[kb] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 kf = lds_row8(kt_lds, lds_off<D>(kb * 32 + l32, 2 * ks + h2));
          s[kb] = mfma(kf, qf[ks], s[kb]);
        }
      }
      // online softmax in the log2 domain; query = qw + l32 is lane-local
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = s[kb][r] * scale_log2;
          if constexpr (CAUSAL) {
            const int key = k0 + kb * 32 + crow(r, h2);
            if (key > qrow) v = -INFINITY;
          }
          s[kb][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_i, mx);
      const float alpha = fexp2(m_i - m_new);
      float rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(s[kb][r] - m_new);
          s[kb][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
      m_i = m_new;
#pragma unroll
      for (int i = 0; i < NDB; ++i) o[i] *= alpha;
      // O^T[d][q] += V^T[d][key] * P^T[key][q]
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pf = pack8(s[kb], s2);
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const bf16x8 vf = tr_frag<D>(vt_lds, kb * 32 + 16 * s2, db * 32, lane);
            o[db] = mfma(vf, pf, o[db]);
          }
        }
    }
    if (kt + 1 < nkt) {
      sk.store(smem[cur ^ 1][0]);
      sv.store(smem[cur ^ 1][1]);
    }
    __syncthreads();
  }

  if (qrow < S) {
    const float inv = 1.f / l_i;
    __bf16* op = O + ((long)b * S + qrow) * ldo + hq * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        bf16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (__bf16)(o[db][4 * rr + j] * inv);
        *reinterpret_cast<bf16x4*>(op + db * 32 + 8 * rr + 4 * h2) = w;
      }
    if (h2 == 0) LSE[((long)b * Hq + hq) * S + qrow] = (m_i + __log2f(l_i)) * 0.69314718055994531f;
  }
}

// ======================================================================================
// Backward preprocess: delta[b,h,q] = sum_d dO[q,h,d] * O[q,h,d]  (fp32)
// ======================================================================================
template <int D>
__global__ __launch_bounds__(256) void bwd_pre_kernel(const __bf16* __restrict__ O, const __bf16* __restrict__ dO,
                                                      float* __restrict__ delta, int B, int S, int Hq, long ldo,
                                                      long lddo) {
  constexpr int LPR = D / 8;            // lanes per row
  constexpr int RPB = 256 / LPR;        // rows per block
  const long row = (long)blockIdx.x * RPB + threadIdx.x / LPR;  // row = (b*S + q)*Hq + h
  const int sub = threadIdx.x % LPR;
  const long total = (long)B * S * Hq;
  float acc = 0.f;
  if (row < total) {
    const long bq = row / Hq;
    const int h = (int)(row % Hq);
    float a[8], c[8];
    load8<__bf16>(O + bq * ldo + h * D + sub * 8, a);
    load8<__bf16>(dO + bq * lddo + h * D + sub * 8, c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * c[j];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < total && sub == 0) {
    const long bq = row / Hq;
    const int h = (int)(row % Hq);
    const long b = bq / S, q = bq % S;
    delta[(b * Hq + h) * S + q] = acc;
  }
}

// ======================================================================================
// Backward dK/dV: block = (b, kv head, 128-key tile); wave owns 32 keys in registers.
// Loops over the query heads of the kv head and over 32-row query tiles.
//   S  = Q K^T   (key on lane)      P  = exp2(S*c - lse2)
//   dP = dO V^T  (key on lane)      dS = P * (dP - delta)
//   dV^T += dO^T P                  dK^T += Q^T dS      (accumulators reused as B operands)
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void bwd_dkdv_kernel(
    const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ V,
    const __bf16* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    __bf16* __restrict__ dK, __bf16* __restrict__ dV, int S, int Hq, int Hkv, long ldq, long ldk, long ldv,
    long lddo, long lddk, long lddv, float scale, float scale_log2) {
  constexpr int KB = 128, QT = 32;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][2][QT * D];  // [buf][Q/dO]
  __shared__ __attribute__((aligned(16))) float rowc[2][2][QT];        // [buf][lse*/delta]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nkb = S / KB;
  const int BH = gridDim.x / nkb;
  const int kbk = (int)(blockIdx.x / BH);  // causal: early key tiles have the most work
  const int bh = blockIdx.x % BH;
  const int hk = bh % Hkv, b = bh / Hkv;
  const int nrep = Hq / Hkv;
  const int k0 = kbk * KB, kw = k0 + wid * 32;
  const int krow = kw + l32;

  // K/V fragments as B operands: lane holds K[krow][16 ks + 8 h2 .. +7]
  bf16x8 kf[NKS], vf[NKS];
  {
    const __bf16* Kr = K + ((long)b * S + krow) * ldk + hk * D + 8 * h2;
    const __bf16* Vr = V + ((long)b * S + krow) * ldv + hk * D + 8 * h2;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(Kr + 16 * ks);
      vf[ks] = *reinterpret_cast<const bf16x8*>(Vr + 16 * ks);
    }
  }
  f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) { dkt[i] = f32x16{}; dvt[i] = f32x16{}; }

  const int qstart = CAUSAL ? k0 : 0;
  const int nqt = (S - qstart) / QT;
  const int total = nqt * nrep;
  const float inv_c = 1.f / scale_log2;

  Stage<D, QT> sq, sd;
  auto stage_load = [&](int it) {
    const int hq = hk * nrep + it / nqt;
    const int q0 = qstart + (it % nqt) * QT;
    sq.load(Q + (long)b * S * ldq + hq * D, ldq, q0, S);
    sd.load(dO + (long)b * S * lddo + hq * D, lddo, q0, S);
  };
  auto stage_rows = [&](int it, int buf) {
    const int hq = hk * nrep + it / nqt;
    const int q0 = qstart + (it % nqt) * QT;
    if (threadIdx.x < QT)
      rowc[buf][0][threadIdx.x] = -LSE[((long)b * Hq + hq) * S + q0 + threadIdx.x] * 1.4426950408889634f * inv_c;
    else if (threadIdx.x < 2 * QT)
      rowc[buf][1][threadIdx.x - QT] = -Delta[((long)b * Hq + hq) * S + q0 + threadIdx.x - QT];
  };

  if (total > 0) {
    stage_load(0);
    sq.store(smem[0][0]);
    sd.store(smem[0][1]);
    stage_rows(0, 0);
  }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int q0 = qstart + (it % nqt) * QT;
    if (it + 1 < total) stage_load(it + 1);
    if (!(CAUSAL && q0 + QT - 1 < kw)) {
      const __bf16* qt_lds = smem[cur][0];
      const __bf16* dt_lds = smem[cur][1];
      f32x16 s, dp;
      // row constants as the initial accumulators (rows = queries crow(r,h2))
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 a = *reinterpret_cast<const float4*>(&rowc[cur][0][8 * rr + 4 * h2]);
        const float4 c = *reinterpret_cast<const float4*>(&rowc[cur][1][8 * rr + 4 * h2]);
        s[4 * rr + 0] = a.x; s[4 * rr + 1] = a.y; s[4 * rr + 2] = a.z; s[4 * rr + 3] = a.w;
        dp[4 * rr + 0] = c.x; dp[4 * rr + 1] = c.y; dp[4 * rr + 2] = c.z; dp[4 * rr + 3] = c.w;
      }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 qa = lds_row8(qt_lds, lds_off<D>(l32, 2 * ks + h2));
        s = mfma(qa, kf[ks], s);
        const bf16x8 da = lds_row8(dt_lds, lds_off<D>(l32, 2 * ks + h2));
        dp = mfma(da, vf[ks], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fexp2(s[r] * scale_log2);
        if constexpr (CAUSAL) {
          if (krow > q0 + crow(r, h2)) p = 0.f;
        }
        s[r] = p;
        dp[r] = p * dp[r];
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(s, s2);
        const bf16x8 df = pack8(dp, s2);
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const bf16x8 doT = tr_frag<D>(dt_lds, 16 * s2, db * 32, lane);
          dvt[db] = mfma(doT, pf, dvt[db]);
          const bf16x8 qT = tr_frag<D>(qt_lds, 16 * s2, db * 32, lane);
          dkt[db] = mfma(qT, df, dkt[db]);
        }
      }
    }
    if (it + 1 < total) {
      sq.store(smem[cur ^ 1][0]);
      sd.store(smem[cur ^ 1][1]);
      stage_rows(it + 1, cur ^ 1);
    }
    __syncthreads();
  }

  __bf16* dkp = dK + ((long)b * S + krow) * lddk + hk * D;
  __bf16* dvp = dV + ((long)b * S + krow) * lddv + hk * D;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      bf16x4 wk, wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wk[j] = (__bf16)(dkt[db][4 * rr + j] * scale);
        wv[j] = (__bf16)(dvt[db][4 * rr + j]);
      }
      *reinterpret_cast<bf16x4*>(dkp + db * 32 + 8 * rr + 4 * h2) = wk;
      *reinterpret_cast<bf16x4*>(dvp + db * 32 + 8 * rr + 4 * h2) = wv;
    }
}

// ======================================================================================
// Backward dQ: block = (b, q head, 128 query rows), wave owns 32 queries; loop over key tiles.
//   S^T = K Q^T, dP^T = V dO^T (query on lane; lse/delta are lane constants)
//   dQ^T += K^T dS^T
// ======================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void bwd_dq_kernel(
    const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ V,
    const __bf16* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    __bf16* __restrict__ dQ, int S, int Hq, int Hkv, long ldq, long ldk, long ldv, long lddo, long lddq,
    float scale, float scale_log2) {
  constexpr int KT = 64, QT = 128;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][2][KT * D];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = (S + QT - 1) / QT;
  const int BH = gridDim.x / nqt;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH;
  const int hq = bh % Hq, b = bh / Hq;
  const int hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + wid * 32;
  const int qrow = qw + l32;

  const __bf16* Kb = K + (long)b * S * ldk + hk * D;
  const __bf16* Vb = V + (long)b * S * ldv + hk * D;

  bf16x8 qf[NKS], df[NKS];
  {
    const __bf16* Qr = Q + ((long)b * S + qrow) * ldq + hq * D + 8 * h2;
    const __bf16* Dr = dO + ((long)b * S + qrow) * lddo + hq * D + 8 * h2;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (qrow < S) {
        qf[ks] = *reinterpret_cast<const bf16x8*>(Qr + 16 * ks);
        df[ks] = *reinterpret_cast<const bf16x8*>(Dr + 16 * ks);
      } else {
        qf[ks] = bf16x8{};
        df[ks] = bf16x8{};
      }
    }
  }
  float lse_c = 0.f, dl = 0.f;
  if (qrow < S) {
    lse_c = -LSE[((long)b * Hq + hq) * S + qrow] * 1.4426950408889634f / scale_log2;
    dl = -Delta[((long)b * Hq + hq) * S + qrow];
  }

  f32x16 dqt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dqt[i] = f32x16{};

  const int kend = CAUSAL ? min(S, q0 + QT) : S;
  const int nkt = (kend + KT - 1) / KT;

  Stage<D, KT> sk, sv;
  sk.load(Kb, ldk, 0, S);
  sv.load(Vb, ldv, 0, S);
  sk.store(smem[0][0]);
  sv.store(smem[0][1]);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const int k0 = kt * KT;
    if (kt + 1 < nkt) {
      sk.load(Kb, ldk, k0 + KT, S);
      sv.load(Vb, ldv, k0 + KT, S);
    }
    if (!(CAUSAL && k0 > qw + 31)) {
      const __bf16* kt_lds = smem[cur][0];
      const __bf16* vt_lds = smem[cur][1];
      // one 32-key half at a time keeps the live accumulator set at 2 x 16 registers
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = lse_c; dp[r] = dl; }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 ka = lds_row8(kt_lds, lds_off<D>(kb * 32 + l32, 2 * ks + h2));
          s = mfma(ka, qf[ks], s);
          const bf16x8 va = lds_row8(vt_lds, lds_off<D>(kb * 32 + l32, 2 * ks + h2));
          dp = mfma(va, df[ks], dp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fexp2(s[r] * scale_log2);
          if constexpr (CAUSAL) {
            if (k0 + kb * 32 + crow(r, h2) > qrow) p = 0.f;
          }
          dp[r] = p * dp[r];
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 dsf = pack8(dp, s2);
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const bf16x8 kT = tr_frag<D>(kt_lds, kb * 32 + 16 * s2, db * 32, lane);
            dqt[db] = mfma(kT, dsf, dqt[db]);
          }
        }
      }
    }
    if (kt + 1 < nkt) {
      sk.store(smem[cur ^ 1][0]);
      sv.store(smem[cur ^ 1][1]);
    }
    __syncthreads();
  }

  if (qrow < S) {
    __bf16* dqp = dQ + ((long)b * S + qrow) * lddq + hq * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        bf16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (__bf16)(dqt[db][4 * rr + j] * scale);
        *reinterpret_cast<bf16x4*>(dqp + db * 32 + 8 * rr + 4 * h2) = w;
      }
  }
}

}  // namespace attn
}  // namespace pra

using namespace pra::attn;

extern "C" {

// All tensors bf16, layout [B, S, H, D] with token stride ld* (elements); LSE/Delta fp32 [B, Hq, S].
hipError_t pra_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq,
                        int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal,
                        hipStream_t st) {
  if (S % 64 || (D != 64 && D != 128) || Hq % Hkv) return hipErrorInvalidValue;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return hipErrorInvalidValue;
  const int nqt = (S + 127) / 128;
  dim3 grid(nqt * Hq * B), block(256);
  const float sl2 = scale * 1.4426950408889634f;
#define LAUNCH(DD, CC)                                                                                        \
  hipLaunchKernelGGL((fwd_kernel<DD, CC>), grid, block, 0, st, (const __bf16*)q, (const __bf16*)k,             \
                     (const __bf16*)v, (__bf16*)o, lse, S, Hq, Hkv, ldq, ldk, ldv, ldo, sl2)
  if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
  else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  return hipGetLastError();
}

hipError_t pra_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv,
                        int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk, long lddv,
                        float scale, int causal, hipStream_t st) {
  if (S % 128 || (D != 64 && D != 128) || Hq % Hkv) return hipErrorInvalidValue;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 8 || lddo % 8 || lddq % 4 || lddk % 4 || lddv % 4)
    return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  {
    const int rpb = 256 / (D / 8);
    const long rows = (long)B * S * Hq;
    const int grid = (int)((rows + rpb - 1) / rpb);
    if (D == 128)
      hipLaunchKernelGGL((bwd_pre_kernel<128>), dim3(grid), dim3(256), 0, st, (const __bf16*)o,
                         (const __bf16*)dout, delta, B, S, Hq, ldo, lddo);
    else
      hipLaunchKernelGGL((bwd_pre_kernel<64>), dim3(grid), dim3(256), 0, st, (const __bf16*)o,
                         (const __bf16*)dout, delta, B, S, Hq, ldo, lddo);
  }
  {
    dim3 grid((S / 128) * Hkv * B);
#define LAUNCH(DD, CC)                                                                                         \
  hipLaunchKernelGGL((bwd_dkdv_kernel<DD, CC>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,     \
                     (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dk, (__bf16*)dv, S, Hq, Hkv, ldq, \
                     ldk, ldv, lddo, lddk, lddv, scale, sl2)
    if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
    else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  }
  {
    dim3 grid(((S + 127) / 128) * Hq * B);
#define LAUNCH(DD, CC)                                                                                         \
  hipLaunchKernelGGL((bwd_dq_kernel<DD, CC>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,       \
                     (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dq, S, Hq, Hkv, ldq, ldk, ldv,   \
                     lddo, lddq, scale, sl2)
    if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
    else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  }
  return hipGetLastError();
}

}  // extern "C"

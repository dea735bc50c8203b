// Fused flash-attention backward for gfx950: dQ, dK and dV of one (batch, kv head) in ONE workgroup,
// deterministic (no float atomics), head_dim 128, bf16 / fp16, causal or full (no key padding).
//
// The split backward (attention.hip: a dQ kernel, then a dK/dV kernel) computes S = Q K^T and
// dP = dO V^T twice: 7 MFMA products per (query, key) tile instead of the 5 the math needs
// (S, dP, dV^T += dO^T P, dK^T += Q^T dS, dQ += dS K). The usual fusion sums dQ across the key-block
// workgroups with float atomics, which makes every run's gradients differ in the last bits. Here a
// workgroup owns a whole (batch, kv head) -- all its key blocks and every query head of its GQA group
// -- and walks the key blocks in order, so the dQ sum has ONE writer and a fixed order:
//
//   for each 256-key block kb (K, V resident in LDS, K pre-multiplied by c = scale log2 e):
//     for each query head hq of the group, each 32-query tile q0 the block can see:
//       8 waves x 32 keys: S' = Q (cK)^T - lse log2 e, dP' = dO V^T - delta   (row constants = the
//         accumulators' initial values), P = exp2(S'), dS = P dP'; dV^T += dO^T P, dK^T += Q^T dS
//         (accumulators in registers for the whole block); dS -> LDS (key-major image)
//       barrier
//       waves 0-3, 32 head dims each: dQ^T = (cK)^T dS^T over the block's 256 keys (16 MFMAs), added
//         to the tile's fp32 partial of the previous blocks (kept in a workspace, read back by the
//         same lane that wrote it); the last block that sees the tile writes dQ = ln2 * sum (with
//         the inverse RoPE) instead.
//     dK, dV of the block -> global (with dK's inverse RoPE)
//
// LDS: K 64 KB + V 64 KB + Q / dO tile 16 KB + dS 16 KB = 160 KB (one workgroup per CU). Q / dO are
// register-staged one tile ahead. The row constants come from bwd_rowc_kernel (one streaming pass
// over O and dO) and are read as float4 straight into the accumulators.
//
// Used when (B Hkv) workgroups fill whole rounds of the chip (7B-class MHA at batch >= 8); GQA at
// small batch keeps the split kernels, whose grids have S / 256 times more workgroups.
// Replaces the reference's SDPA backward (reference model.py:179-230).
#include "attn_common.h"
#include "common.h"
#include "launchers.h"

namespace pra {
namespace attn {

// RC[i] = -lse[i] log2(e), RC[nrc + i] = -delta[i], delta = rowsum(dO * O); i = (b Hq + hq) S + q.
// 16 lanes per row (8 elements each at D = 128), rows in TOKEN order (t Hq + hq), so a wave reads
// 4 consecutive 256-B head rows of one token: in (b, hq, q) order consecutive rows were a token
// stride (8 KiB at 7B) apart and the pass took 0.47 ms instead of ~0.1 at B16 S2048 H32.
template <typename T>
__global__ __launch_bounds__(256) void bwd_rowc_kernel(const T* __restrict__ O, const T* __restrict__ dO,
                                                       const float* __restrict__ LSE, float* __restrict__ RC,
                                                       long nrc, int S, int Hq, long ldo, long lddo) {
  constexpr int D = 128;
  const long row = ((long)blockIdx.x * 256 + threadIdx.x) >> 4;  // token-major: tok Hq + hq
  const int sub = threadIdx.x & 15;
  const long r = row < nrc ? row : nrc - 1;  // (nrc % 16 == 0: whole groups; clamp keeps the shuffles uniform)
  const long tok = r / Hq;
  const int hq = (int)(r % Hq);
  const V8<T> o8 = *reinterpret_cast<const V8<T>*>(O + tok * ldo + hq * D + 8 * sub);
  const V8<T> d8 = *reinterpret_cast<const V8<T>*>(dO + tok * lddo + hq * D + 8 * sub);
  float part = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) part = fmaf((float)o8[j], (float)d8[j], part);
  part += __shfl_xor(part, 8, 16);
  part += __shfl_xor(part, 4, 16);
  part += __shfl_xor(part, 2, 16);
  part += __shfl_xor(part, 1, 16);
  if (sub == 0 && row < nrc) {
    const long b = tok / S, q = tok % S;
    const long i = (b * Hq + hq) * S + q;
    RC[i] = -LSE[i] * 1.4426950408889634f;
    RC[nrc + i] = -part;
  }
}

// Variant switches (tools/attn_variants.sh). PRA_FUSED_MAXV=112 caps the kernel at 224 VGPRs
// (amdgpu_num_vgpr counts VGPR + AGPR pairs on gfx90a+), so one 64-VGPR wave of the overlapped AdamW
// update fits on each SIMD beside it; with PRA_FUSED_LATE_ACC=1 the dQ partial is read after the dS
// barrier instead of held in 16 registers across the tile. Measured (profiles/r5/attn_fused/): alone
// 2.28 vs 2.21 ms, and the overlapped 7B step did not improve (1063.3 vs 1058.7 ms split), so both off.
#ifndef PRA_FUSED_LATE_ACC
#define PRA_FUSED_LATE_ACC 0
#endif
#ifndef PRA_FUSED_MAXV
#define PRA_FUSED_MAXV 0
#endif
#if PRA_FUSED_MAXV
#define PRA_FUSED_VGPR_ATTR __attribute__((amdgpu_num_vgpr(PRA_FUSED_MAXV)))
#else
#define PRA_FUSED_VGPR_ATTR
#endif

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(512, 1) PRA_FUSED_VGPR_ATTR void bwd_fused_kernel(
    const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V, const T* __restrict__ dO,
    const float* __restrict__ RC, long nrc, T* __restrict__ dQ, T* __restrict__ dK, T* __restrict__ dV,
    float* __restrict__ dQacc, int S, int Hq, int Hkv, long ldq, long ldk, long ldv, long lddo, long lddq,
    long lddk, long lddv, float scale, float scale_log2, const float2* __restrict__ rtab) {
  constexpr int D = 128, NW = 8, KB = 32 * NW, QT = 32, NKS = D / 16, NDB = D / 32;
  constexpr int KVT = KB * D, QDT = QT * D;
  // one __shared__ object per operand (separate alias scopes: a read of one never waits for a DMA
  // still filling another)
  __shared__ __attribute__((aligned(16))) T Ks[KVT];
  __shared__ __attribute__((aligned(16))) T Vs[KVT];
  __shared__ __attribute__((aligned(16))) T Qs[QDT];
  __shared__ __attribute__((aligned(16))) T Ds[QDT];
  __shared__ __attribute__((aligned(16))) T Ss[KB * QT];  // dS, key-major: row = key, 32 queries (64 B)

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int hk = (int)(blockIdx.x % Hkv), b = (int)(blockIdx.x / Hkv);
  const int nrep = Hq / Hkv, nkb = S / KB, nqs = S / QT;
  LaneOff<T, D> lo;  // K / V / Q / dO images ([rows][128])
  lo.init(lane);
  LaneOff<T, QT> ls;  // dS image ([256][32])
  ls.init(lane);
  const T* Kw = Ks + wid * 32 * D;
  const T* Vw = Vs + wid * 32 * D;
  GStage<T, D, KB, NW> gk, gv;
  gk.init(ldk);
  gv.init(ldv);
  Stage<T, D, QT, NW * 64> sq, sd;
  // this lane's dS row (its key) in the image: queries 8 g + 4 h2 .. + 3 sit in chunk g at byte 8 h2,
  // chunk XOR-swizzled by row bits 2-3 (lay_byte<32>)
  const int srw = wid * 32 + l32;
  char* const srow = reinterpret_cast<char*>(Ss) + 512 * (srw >> 3) + 64 * (srw & 7) + 8 * h2;
  const int ssw = (l32 >> 2) & 3;
  auto sput = [&](int g, uint2 v) { *reinterpret_cast<uint2*>(srow + 16 * (g ^ ssw)) = v; };
  const float ln2 = 0.69314718055994531f;
  // this workgroup's scratch line (4 KiB after the dQ partials): the stand-in address of the
  // loads / stores a wave issues only to keep the memory-operation count uniform
  float* const scratch = dQacc + nrc * D + (long)blockIdx.x * 1024 + 4 * lane;

  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * KB, kw = k0 + wid * 32, krow = kw + l32;
    const int qstart = CAUSAL ? k0 : 0;
    const int nqt = (S - qstart) / QT;
    const int total = nqt * nrep;
    gk.issue(K + ((long)b * S + k0) * ldk + hk * D, Ks);
    gv.issue(V + ((long)b * S + k0) * ldv + hk * D, Vs);
    auto stage = [&](int it) {
      const int hq = hk * nrep + it / nqt, q0 = qstart + (it % nqt) * QT;
      sq.load_all(Q + (long)b * S * ldq + hq * D, ldq, q0);
      sd.load_all(dO + (long)b * S * lddo + hq * D, lddo, q0);
    };
    stage(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {  // K *= c in place: each wave rescales its own 32 rows (8 KiB of the image); the others read
       // them only after the first tile's barrier
      char* kp = reinterpret_cast<char*>(Ks) + wid * 32 * D * (int)sizeof(T);
#pragma unroll
      for (int i = 0; i < 32 * D * (int)sizeof(T) / 1024; ++i) {
        V8<T>& c8 = *reinterpret_cast<V8<T>*>(kp + i * 1024 + lane * 16);
        V8<T> v8 = c8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v8[j] = (T)((float)v8[j] * scale_log2);
        c8 = v8;
      }
    }
    f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i) {
      dkt[i] = f32x16{};
      dvt[i] = f32x16{};
    }

    // four scratch stores: the loop is entered with the same memory-operation history as its back edge
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(scratch + 256 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int it = 0; it < total; ++it) {
      const int hq = hk * nrep + it / nqt, q0 = qstart + (it % nqt) * QT;
      const long rci = ((long)b * Hq + hq) * S + q0;
      // row constants of query rows crow(r, h2) = 8 rr + 4 h2 + 0..3 as the S / dP initial values
      f32x16 sa, dp;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 a = *reinterpret_cast<const float4*>(RC + rci + 8 * rr + 4 * h2);
        const float4 c = *reinterpret_cast<const float4*>(RC + nrc + rci + 8 * rr + 4 * h2);
        sa[4 * rr] = a.x; sa[4 * rr + 1] = a.y; sa[4 * rr + 2] = a.z; sa[4 * rr + 3] = a.w;
        dp[4 * rr] = c.x; dp[4 * rr + 1] = c.y; dp[4 * rr + 2] = c.z; dp[4 * rr + 3] = c.w;
      }
      // dQ^T partial of this tile from the earlier key blocks (waves 0-3; the same lane wrote it).
      // Every global load / store of the tile loop is issued by EVERY wave on EVERY path, in the same
      // number (waves 4-7 and the first visit read / write a per-workgroup scratch line instead): CDNA4's
      // vmcnt counts loads and stores in order, and the compiler's wait at a join is the strictest of
      // its paths -- one path without the stores made it wait for the NEXT tile's Q / dO loads
      // (vmcnt(0)) in the middle of this tile's MFMA chain.
      const bool first = kb == 0;
      const bool last = CAUSAL ? (q0 / KB == kb) : (kb == nkb - 1);
      float* const slot = dQacc + ((((long)b * Hq + hq) * nqs + q0 / QT) * 4 + (wid & 3)) * 1024 + 4 * lane;
      const bool real = wid < 4 && !first;
      const float* src = real ? slot : scratch;
      f32x16 acc = f32x16{};
#if !PRA_FUSED_LATE_ACC
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(src + 256 * i);
        acc[4 * i] = real ? v.x : 0.f;
        acc[4 * i + 1] = real ? v.y : 0.f;
        acc[4 * i + 2] = real ? v.z : 0.f;
        acc[4 * i + 3] = real ? v.w : 0.f;
      }
#endif
      sq.store(Qs);
      sd.store(Ds);
      __syncthreads();  // Q / dO of this tile (and, at it = 0, the block's scaled K) visible
      stage(it + 1 < total ? it + 1 : it);  // (the last tile re-loads itself: same load count every tile)
      if (!(CAUSAL && q0 + QT - 1 < kw)) {
        if (CAUSAL && q0 == kw) {  // diagonal tile: keys after the query are masked on S's initial values
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (l32 > crow(r, h2)) sa[r] = -INFINITY;
        }
        V8<T> xa = lo.rowk(Qs, 0, 0), xb = lo.rowk(Kw, 0, 0);
#pragma unroll
        for (int st = 0; st < 2 * NKS; ++st) {
          const int ks = st % NKS;
          V8<T> na = xa, nb = xb;
          if (st + 1 < 2 * NKS) {
            const int nks = (st + 1) % NKS;
            na = lo.rowk(st + 1 < NKS ? Qs : Ds, 0, nks);
            nb = lo.rowk(st + 1 < NKS ? Kw : Vw, 0, nks);
          }
          if (st < NKS) sa = mfma(xa, xb, sa);
          else dp = mfma(xa, xb, dp);
          (void)ks;
          xa = na;
          xb = nb;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(sa[r]);
          sa[r] = p;
          dp[r] = p * dp[r];
        }
        const V8<T> p0 = pack8<T>(sa, 0), p1 = pack8<T>(sa, 1), d0 = pack8<T>(dp, 0), d1 = pack8<T>(dp, 1);
        V8<T> ot = lo.tr(Ds, 0, 0), qt = lo.tr(Qs, 0, 0);
#pragma unroll
        for (int st = 0; st < 2 * NDB; ++st) {
          const int s2 = st / NDB, db = st % NDB;
          V8<T> no = ot, nq = qt;
          if (st + 1 < 2 * NDB) {
            no = lo.tr(Ds, 16 * ((st + 1) / NDB), (st + 1) % NDB);
            nq = lo.tr(Qs, 16 * ((st + 1) / NDB), (st + 1) % NDB);
          }
          dvt[db] = mfma(ot, s2 ? p1 : p0, dvt[db]);
          dkt[db] = mfma(qt, s2 ? d1 : d0, dkt[db]);
          ot = no;
          qt = nq;
        }
        // dS of query rows 8 g + 4 h2 .. + 3 (d0 elements 0-3 | 4-7, d1 elements 0-3 | 4-7)
        const uint4 u0 = __builtin_bit_cast(uint4, d0), u1 = __builtin_bit_cast(uint4, d1);
        sput(0, make_uint2(u0.x, u0.y));
        sput(1, make_uint2(u0.z, u0.w));
        sput(2, make_uint2(u1.x, u1.y));
        sput(3, make_uint2(u1.z, u1.w));
      } else {  // every key of this wave is after every query of the tile: dS = 0
#pragma unroll
        for (int g = 0; g < 4; ++g) sput(g, make_uint2(0u, 0u));
      }
      __syncthreads();  // dS of all 256 keys in LDS
#if PRA_FUSED_LATE_ACC
      // the partial is read here (under the 16 MFMAs below) instead of held in 16 registers across
      // the tile: fewer VGPRs, so a wave of the overlapped AdamW update fits beside the block
      float4 pv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = *reinterpret_cast<const float4*>(src + 256 * i);
#endif
      if (wid < 4) {
        V8<T> ka = lo.tr(Ks, 0, wid), sb = ls.tr(Ss, 0, 0);
#pragma unroll
        for (int ks = 0; ks < KB / 16; ++ks) {
          V8<T> nk = ka, ns = sb;
          if (ks + 1 < KB / 16) {
            nk = lo.tr(Ks, 16 * (ks + 1), wid);
            ns = ls.tr(Ss, 16 * (ks + 1), 0);
          }
          acc = mfma(ka, sb, acc);
          ka = nk;
          sb = ns;
        }
      }
#if PRA_FUSED_LATE_ACC
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[4 * i] += real ? pv[i].x : 0.f;
        acc[4 * i + 1] += real ? pv[i].y : 0.f;
        acc[4 * i + 2] += real ? pv[i].z : 0.f;
        acc[4 * i + 3] += real ? pv[i].w : 0.f;
      }
#endif
      if (wid < 4 && last) {
        const f32x16 fin[1] = {acc};
        store_rows16<T, 1>(fin, ln2, dQ + ((long)b * S + q0 + l32) * lddq + hq * D + 32 * wid, true, h2,
                           rtab ? rtab + (long)(q0 + l32) * (D / 2) + 16 * wid : nullptr);
        if (!rtab) {  // two more (scratch) stores: at least four memory operations on every path
          *reinterpret_cast<float4*>(scratch) = make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(scratch + 256) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      } else {
        float* const dst = wid < 4 ? slot : scratch;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<float4*>(dst + 256 * i) = make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]);
      }
    }
    store_rows16<T, NDB>(dkt, scale, dK + ((long)b * S + krow) * lddk + hk * D, true, h2,
                         rtab ? rtab + (long)krow * (D / 2) : nullptr);
    store_rows16<T, NDB>(dvt, 1.f, dV + ((long)b * S + krow) * lddv + hk * D, true, h2);
    __syncthreads();  // every wave is done with K / V / dS before the next block's DMA overwrites them
  }
}

}  // namespace attn
}  // namespace pra

extern "C" {

// Host-checked preconditions (pra_attn_bwd_fused_ok): D = 128, S % 256 == 0, Hq % Hkv == 0, strides % 8.
// ws: 2 B Hq S floats of row constants, then B Hq S D floats of dQ partials, then B Hkv 1024 floats of
// per-workgroup scratch.
hipError_t pra_attn_bwd_fused(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout,
                              const float* lse, float* ws, void* dq, void* dk, void* dv, int B, int S, int Hq,
                              int Hkv, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk,
                              long lddv, float scale, int causal, const float* rope_tab, hipEvent_t mid_event,
                              hipStream_t st) {
  using namespace pra::attn;
  if (S % 256 || S <= 0 || Hq % Hkv || B <= 0) return hipErrorInvalidValue;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 8 || lddo % 8 || lddq % 8 || lddk % 8 || lddv % 8)
    return hipErrorInvalidValue;
  const long nrc = (long)B * Hq * S;
  float* rc = ws;
  float* acc = ws + 2 * nrc;
  const float sl2 = scale * 1.4426950408889634f;
  const float2* rt = reinterpret_cast<const float2*>(rope_tab);
  const dim3 g0((unsigned)((nrc * 16 + 255) / 256)), g1((unsigned)(B * Hkv));
#define PRA_FUSED(TT)                                                                                          \
  hipLaunchKernelGGL((bwd_rowc_kernel<TT>), g0, dim3(256), 0, st, (const TT*)o, (const TT*)dout, lse, rc, nrc, S, \
                     Hq, ldo, lddo);                                                                           \
  if (mid_event != nullptr && hipEventRecord(mid_event, st) != hipSuccess) return hipErrorInvalidResourceHandle; \
  if (causal)                                                                                                  \
    hipLaunchKernelGGL((bwd_fused_kernel<TT, true>), g1, dim3(512), 0, st, (const TT*)q, (const TT*)k,         \
                       (const TT*)v, (const TT*)dout, rc, nrc, (TT*)dq, (TT*)dk, (TT*)dv, acc, S, Hq, Hkv, ldq,  \
                       ldk, ldv, lddo, lddq, lddk, lddv, scale, sl2, rt);                                      \
  else                                                                                                         \
    hipLaunchKernelGGL((bwd_fused_kernel<TT, false>), g1, dim3(512), 0, st, (const TT*)q, (const TT*)k,        \
                       (const TT*)v, (const TT*)dout, rc, nrc, (TT*)dq, (TT*)dk, (TT*)dv, acc, S, Hq, Hkv, ldq,  \
                       ldk, ldv, lddo, lddq, lddk, lddv, scale, sl2, rt)
  if (dtype == pra::kBF16) {
    PRA_FUSED(__bf16);
#if !PRA_ATTN_HARNESS
  } else if (dtype == pra::kF16) {
    PRA_FUSED(_Float16);
#endif
  } else {
    return hipErrorInvalidValue;
  }
#undef PRA_FUSED
  return hipGetLastError();
}

}  // extern "C"

// Flash attention forward + deterministic backward for gfx950 (CDNA4), bf16 or fp16, head_dim 64/128,
// causal or full, native GQA (kv head = q head / (Hq/Hkv); no repeat_kv copies).
//
// Replaces the reference's SDPA / flash-attn call (reference model.py:179-230; N1/N2 in
// SURVEY §2.2). Tensors are read straight out of the fused QKV activation: q/k/v are
// [B, S, H, D] views with an arbitrary token stride, so no transpose/contiguous copies.
//
// Design (all MFMA work on v_mfma_f32_32x32x16_bf16, wave64):
//  * forward: 512-thread block = 8 waves = 256 query rows (32 per wave, 2 waves per SIMD); K/V
//    tiles of 64 keys staged global->regs->LDS (issue-early / write-late), double-buffered, one
//    barrier per tile; online softmax with an exact deferred rescale (skipped when no row max
//    grows). "Swapped" products:
//    S^T = K Q^T puts one query per lane, so softmax row statistics are lane-local (plus one
//    xor-32 exchange), and O^T = V^T P^T reuses the S^T accumulator registers directly as the
//    B operand (bf16-packed). V^T fragments come from ds_read_b64_tr_b16 (hardware transpose).
//  * every LDS tile uses one sub-tiled, XOR-swizzled image that is conflict-free for both
//    ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads (lay_byte below).
//  * backward is split into two deterministic kernels (no float atomics, so a resumed run is
//    bit-identical to an uninterrupted one): dK/dV (K/V of 128 keys resident in LDS, dK/dV
//    accumulators in registers, loop over query tiles and over the Hq/Hkv query heads of the kv
//    head) and dQ (queries resident, K/V tiles by LDS-DMA, loop over key tiles). P is
//    recomputed from the saved log-sum-exp. Both run at 2 waves per SIMD with no spills.
//
//  * long query loops (S * Hq/Hkv >= 8192) use a dK/dV kernel with one wave per SIMD and two query
//    sub-tiles in flight (bwd_dkdv_p2_kernel); the dQ kernel interleaves the softmax of one 32-key
//    half between the MFMAs of the other (PIPE). Both schedules are explicit sched_barrier regions.
//
// Measured on MI355X (tools/attn_bench.py, B4 S2048 H32 D128 causal): fwd 0.214 ms (640 TF),
// bwd 0.645 ms (530 TF at the 2.5x-forward convention); B16 H64/8 non-causal fwd 835 TF.
// B1 S8192 H32/8 causal: bwd 2.68 -> 1.91 ms with the pipelined kernels (719 TF model, 1.0 PF executed).
#include "attn_common.h"
#include "common.h"
#include "launchers.h"

#include <type_traits>

// Variant switches (tools/attn_variants.sh builds the standalone harness per setting)
#ifndef PRA_FWD_MINBLK
#define PRA_FWD_MINBLK 2
#endif
#ifndef PRA_FWD_PRESCALE
#define PRA_FWD_PRESCALE 0
#endif
#ifndef PRA_DQ_PRESCALE
#define PRA_DQ_PRESCALE 0
#endif

namespace pra {
namespace attn {

// Block -> (query tile, batch * head) of the forward / dQ grids (nqt * BH blocks).
// grp = 0: heavy (late) query tiles first across the whole grid, consecutive blocks on different
// heads. grp = G > 0 (host: BH % 8 == 0 and (BH / 8) % G == 0): XCD-grouped. Workgroups are
// dispatched to the 8 XCDs round-robin (block i on XCD i % 8), so XCD x walks its own contiguous
// range of BH / 8 heads, G heads at a time with all their query tiles (heaviest first): the query
// tiles of a head run together on one XCD and read its K/V tiles from HBM once, the other tiles
// hitting that XCD's L2 (grp 0 re-reads every head's K/V from HBM once per query tile at MHA).
// Adjacent heads (one GQA group) share an XCD.
// `sched` is the group size. (Pairing long and short 32-row groups on each SIMD measured neutral:
// profiles/r5/attn_order/; removed in round 6.)
__device__ __forceinline__ void block_tile(int nqt, int BH, int sched, int& qt, int& bh) {
  const int i = blockIdx.x, grp = sched & 0xffff;
  if (grp <= 0) {
    qt = nqt - 1 - i / BH;
    bh = i % BH;
    return;
  }
  const int x = i & 7, j = i >> 3, per = BH >> 3, span = grp * nqt;
  const int g = j / span, r = j - g * span;
  qt = nqt - 1 - r / grp;
  bh = x * per + g * grp + r % grp;
}



// ======================================================================================
// Forward
// ======================================================================================
// Block = NW waves x 32 query rows (NW = 8: one 512-thread block per CU, 2 waves per SIMD), so
// each staged K/V tile feeds 8 waves' MFMAs.
template <typename T, int D, bool CAUSAL, int NW>
__global__ __launch_bounds__(NW * 64, 2) void fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                         const T* __restrict__ V, T* __restrict__ O,
                                                         float* __restrict__ LSE, int S, int Hq, int Hkv, long ldq,
                                                         long ldk, long ldv, long ldo, float scale_log2, int skv) {
  constexpr int KT = 64, QT = 32 * NW;
  constexpr int NKS = D / 16, NDB = D / 32, TILE = KT * D;
  __shared__ __attribute__((aligned(16))) T smem[4 * TILE];  // K0 V0 K1 V1

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = (S + QT - 1) / QT;
  const int BH = gridDim.x / nqt;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heavy (late) query tiles first
  const int bh = blockIdx.x % BH;
  const int hq = bh % Hq, b = bh / Hq;
  const int hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + wid * 32;

  const T* Qb = Q + (long)b * S * ldq + hq * D;
  const T* Kb = K + (long)b * S * ldk + hk * D;
  const T* Vb = V + (long)b * S * ldv + hk * D;

  LaneOff<T, D> lo;
  lo.init(lane);
  V8<T> qf[NKS];  // B operand of S^T = K Q^T: lane holds Q[qw + l32][16 ks + 8 h2 .. +7]
  const int qrow = qw + l32;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
    qf[ks] = qrow < S ? *reinterpret_cast<const V8<T>*>(Qb + (long)qrow * ldq + 16 * ks + 8 * h2) : V8<T>{};

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m_i = -INFINITY, l_i = 0.f;  // running max (log2 units of scaled scores) and sum

  const int kend = CAUSAL ? min(S, q0 + QT) : S;
  const int nkt = (kend + KT - 1) / KT;

  Stage<T, D, KT, NW * 64> sk, sv;
  sk.load(Kb, ldk, 0, S);
  sv.load(Vb, ldv, 0, S);
  sk.store(smem);
  sv.store(smem + TILE);
  __syncthreads();
  // the younger half of an 8-wave block loses VALU arbitration; one static priority bump evens it
  if (NW == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);

  auto body = [&](auto cc, int kt) {
    constexpr int CUR = decltype(cc)::value;
    const T* Kt = smem + 2 * CUR * TILE;
    const T* Vt = Kt + TILE;
    const int k0 = kt * KT;
    const bool more = kt + 1 < nkt;
    if (more) {  // issue-early / write-late staging of the next K/V tile (T14)
      sk.load(Kb, ldk, k0 + KT, S);
      sv.load(Vb, ldv, k0 + KT, S);
    }
    if (!(CAUSAL && k0 > qw + 31)) {
      // S^T = K Q^T, two 32-key halves, next fragments issued before the current MFMAs
      f32x16 s0 = f32x16{}, s1 = f32x16{};
      V8<T> a0 = lo.rowk(Kt, 0, 0), a1 = lo.rowk(Kt, 32, 0);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        V8<T> n0 = a0, n1 = a1;
        if (ks + 1 < NKS) {
          n0 = lo.rowk(Kt, 0, ks + 1);
          n1 = lo.rowk(Kt, 32, ks + 1);
        }
        s0 = mfma(a0, qf[ks], s0);
        s1 = mfma(a1, qf[ks], s1);
        a0 = n0;
        a1 = n1;
      }
      if (CAUSAL && k0 + KT - 1 > qw) {  // diagonal tile: mask keys beyond the query
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (k0 + crow(r, h2) > qrow) s0[r] = -INFINITY;
          if (k0 + 32 + crow(r, h2) > qrow) s1[r] = -INFINITY;
        }
      }
      if (!CAUSAL && k0 + KT > skv) {  // zero-padded sequence: keys >= skv do not exist
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (k0 + crow(r, h2) >= skv) s0[r] = -INFINITY;
          if (k0 + 32 + crow(r, h2) >= skv) s1[r] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
      mx = half_max(mx) * scale_log2;
      // exact deferred rescale: only when some row's running max grows in this wave
      if (!__all(mx <= m_i)) {
        const float m_new = fmaxf(m_i, mx);
        const float alpha = fexp2(m_i - m_new);
        l_i *= alpha;
#pragma unroll
        for (int i = 0; i < NDB; ++i) o[i] *= alpha;
        m_i = m_new;
      }
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = fexp2(fmaf(s0[r], scale_log2, -m_i));
        s1[r] = fexp2(fmaf(s1[r], scale_log2, -m_i));
        rs += s0[r] + s1[r];
      }
      l_i += half_sum(rs);
      const V8<T> p00 = pack8<T>(s0, 0), p01 = pack8<T>(s0, 1), p10 = pack8<T>(s1, 0), p11 = pack8<T>(s1, 1);
      // O^T[d][q] += V^T[d][key] P^T[key][q]; V^T fragments prefetched one MFMA ahead
      V8<T> vc = lo.tr(Vt, 0, 0);
#pragma unroll
      for (int st = 0; st < 4 * NDB; ++st) {
        const int k4 = st / NDB, db = st % NDB;
        V8<T> vn = vc;
        if (st + 1 < 4 * NDB) vn = lo.tr(Vt, ((st + 1) / NDB) * 16, (st + 1) % NDB);
        const V8<T> pf = k4 == 0 ? p00 : k4 == 1 ? p01 : k4 == 2 ? p10 : p11;
        o[db] = mfma(vc, pf, o[db]);
        vc = vn;
      }
    }
    if (more) {
      sk.store(smem + 2 * (1 - CUR) * TILE);
      sv.store(smem + 2 * (1 - CUR) * TILE + TILE);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    body(IC<0>{}, kt);
    if (kt + 1 < nkt) body(IC<1>{}, kt + 1);
  }

  {
    const float inv = 1.f / l_i;
    store_rows16<T, NDB>(o, inv, O + ((long)b * S + qrow) * ldo + hq * D, qrow < S, h2);
    if (qrow < S && h2 == 0) LSE[((long)b * Hq + hq) * S + qrow] = (m_i + __log2f(l_i)) * 0.69314718055994531f;
  }
}

// ======================================================================================
// Forward, cross-tile software pipeline (default): same block shape and math as fwd_kernel, but each
// wave keeps the scores of two key tiles live, so the MFMAs of one tile overlap the softmax VALU
// of the other (explicit sched_barrier regions, as in the backward kernels):
//   iteration t:  [S(t+1) = K_{t+1} Q^T | exp / row-sum / pack of tile t]
//                 [O^T += V_t^T P_t      | causal mask + row max of tile t+1]
//                 (exact deferred rescale of O and l when a row max grows, before tile t+1's P.V)
// K/V tiles rotate through a 3-deep LDS ring (96 KB at D = 128): tile t+2 is register-staged during
// iteration t and written into the slot tile t-1 vacated, one barrier per tile. In causal mode a
// wave's only diagonal tile is its last one.
// ======================================================================================
template <typename T, int D, bool CAUSAL, int NW>
__global__ __launch_bounds__(NW * 64, PRA_FWD_MINBLK) void fwd_p_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                           const T* __restrict__ V, T* __restrict__ O,
                                                           float* __restrict__ LSE, int S, int Hq, int Hkv, long ldq,
                                                           long ldk, long ldv, long ldo, float scale_log2, float thr,
                                                           int grp) {
  constexpr int KT = 64, QT = 32 * NW;
  constexpr int NKS = D / 16, NDB = D / 32, TILE = KT * D;
  // (K V) x 3, one __shared__ object per ring slot: the LDS lowering gives each object its own alias
  // scope, so the reads of slot t (ds_read_b64_tr_b16 in particular) are not made to wait
  // (vmcnt(0)) for the LDS-DMA still filling slot t + 2 -- with one array the compiler drained the
  // in-flight DMA before the first transposed read of every tile (9 mid-loop vmcnt(0); now 0)
  __shared__ __attribute__((aligned(16))) T kv0[2 * TILE];
  __shared__ __attribute__((aligned(16))) T kv1[2 * TILE];
  __shared__ __attribute__((aligned(16))) T kv2[2 * TILE];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = (S + QT - 1) / QT;
  const int BH = gridDim.x / nqt;
  int qt, bh;
  block_tile(nqt, BH, grp, qt, bh);
  const int hq = bh % Hq, b = bh / Hq;
  const int hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + wid * 32;

  const T* Qb = Q + (long)b * S * ldq + hq * D;
  const T* Kb = K + (long)b * S * ldk + hk * D;
  const T* Vb = V + (long)b * S * ldv + hk * D;

  LaneOff<T, D> lo;
  lo.init(lane);
  V8<T> qf[NKS];
  const int qrow = qw + l32;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    qf[ks] = qrow < S ? *reinterpret_cast<const V8<T>*>(Qb + (long)qrow * ldq + 16 * ks + 8 * h2) : V8<T>{};
#if PRA_FWD_PRESCALE
    // Q pre-multiplied by scale * log2(e) (rounded to T: ~2^-9 relative per element, ~0.1% on P at
    // D = 128), so the scores come out of the MFMA in log2 units, already minus the running max
    // (the accumulator starts at -m: negm below): the softmax needs one v_exp per score, no FMA
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[ks][j] = (T)((float)qf[ks][j] * scale_log2);
#endif
  }

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m_i = -INFINITY, l_i = 0.f;

  const int kend = CAUSAL ? min(S, q0 + QT) : S;
  const int nkt = (kend + KT - 1) / KT;
  const int lastw = CAUSAL ? min(nkt - 1, (qw + 31) / KT) : nkt - 1;  // this wave's last tile

  GStage<T, D, KT, NW> gk, gv;  // LDS-DMA (S % 64 == 0: tiles are always full)
  gk.init(ldk);
  gv.init(ldv);
  auto slot = [&](int t) { return t == 0 ? kv0 : kv1; };  // prologue tiles 0 and 1 only
#pragma unroll
  for (int t = 0; t < 2; ++t)
    if (t < nkt) {
      gk.issue(Kb + (long)t * KT * ldk, slot(t));
      gv.issue(Vb + (long)t * KT * ldv, slot(t) + TILE);
    }
  __syncthreads();
  if (NW == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);

  // masks keys beyond the query (only ever needed on a wave's last tile in causal mode)
  auto mask = [&](f32x16& s0, f32x16& s1, int k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (k0 + crow(r, h2) > qrow) s0[r] = -INFINITY;
      if (k0 + 32 + crow(r, h2) > qrow) s1[r] = -INFINITY;
    }
  };
  auto rowmax = [&](const f32x16& s0, const f32x16& s1) {
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
    return PRA_FWD_PRESCALE ? half_max(mx) : half_max(mx) * scale_log2;
  };
  f32x16 negm;  // -m_i in every register: the initial accumulator of a score tile (PRA_FWD_PRESCALE)

  f32x16 c0 = f32x16{}, c1 = f32x16{};  // scores of the tile being finished (two 32-key halves)
  if (lastw >= 0) {
    const T* Kt = slot(0);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      c0 = mfma(lo.rowk(Kt, 0, ks), qf[ks], c0);
      c1 = mfma(lo.rowk(Kt, 32, ks), qf[ks], c1);
    }
    if (CAUSAL && lastw == 0) mask(c0, c1, 0);
    m_i = rowmax(c0, c1);
#if PRA_FWD_PRESCALE
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      c0[r] -= m_i;
      c1[r] -= m_i;
    }
#endif
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) negm[r] = -m_i;

  // the ring slot of tile t is a compile-time constant (loop unrolled by 3), so every LDS operand
  // address is a lane-constant base plus an immediate offset
  auto body = [&](auto cur_c, int t) {
    constexpr int CUR = decltype(cur_c)::value;
    T* const s_cur = CUR == 0 ? kv0 : CUR == 1 ? kv1 : kv2;
    T* const s_nxt = CUR == 0 ? kv1 : CUR == 1 ? kv2 : kv0;
    T* const s_nn = CUR == 0 ? kv2 : CUR == 1 ? kv0 : kv1;
    if (t + 2 < nkt) {  // LDS-DMA of tile t + 2 into the slot tile t - 1 vacated
      gk.issue(Kb + (long)(t + 2) * KT * ldk, s_nn);
      gv.issue(Vb + (long)(t + 2) * KT * ldv, s_nn + TILE);
    }
    if (t <= lastw) {
      const T* Kn = s_nxt;
      const T* Vt = s_cur + TILE;
      auto iter = [&](auto next_c, auto diag_c) {
        constexpr bool NEXT = decltype(next_c)::value, DIAG = decltype(diag_c)::value;
        // Phase A exponentiates 24 of tile t's 32 scores per lane (all of c0, the first half of c1)
        // and phase B the last 8 (c1[8..15], only read by the P.V k-step of its second half) in its
        // first half, so both phases carry about the same VALU per MFMA (B16 S2048 H32 fwd 0.747 ->
        // 0.734 ms, B1 S8192 H32/8 0.520 -> 0.508 ms against all 32 in phase A).
        constexpr int NEA = 24;
        constexpr int RA = NKS, EA = NEA / RA;  // phase A: regions / softmax elements per region
        constexpr int RB = 2 * NDB, EB = 32 / RB;
        constexpr int EBX = (32 - NEA) / (RB / 2);  // phase B exponentials per region
#if PRA_FWD_PRESCALE
        f32x16 n0 = negm, n1 = negm;
#else
        f32x16 n0 = f32x16{}, n1 = f32x16{};
#endif
        float rs = 0.f, mx = -INFINITY;
        auto expo = [&](int e) {  // element e of the 32 scores of tile t
#if PRA_FWD_PRESCALE
          if (e < 16) {
            c0[e] = fexp2(c0[e]);
            rs += c0[e];
          } else {
            c1[e - 16] = fexp2(c1[e - 16]);
            rs += c1[e - 16];
          }
#else
          if (e < 16) {
            c0[e] = fexp2(fmaf(c0[e], scale_log2, -m_i));
            rs += c0[e];
          } else {
            c1[e - 16] = fexp2(fmaf(c1[e - 16], scale_log2, -m_i));
            rs += c1[e - 16];
          }
#endif
        };
        // phase A: S(t+1) | exp, row sum of tile t
        V8<T> a0 = lo.rowk(Kn, 0, 0), a1 = lo.rowk(Kn, 32, 0);
#pragma unroll
        for (int k = 0; k < RA; ++k) {
          V8<T> b0 = a0, b1 = a1;
          if (NEXT && k + 1 < RA) {
            b0 = lo.rowk(Kn, 0, k + 1);
            b1 = lo.rowk(Kn, 32, k + 1);
          }
          if (NEXT) {
            n0 = mfma(a0, qf[k], n0);
            n1 = mfma(a1, qf[k], n1);
          }
#pragma unroll
          for (int e = 0; e < EA; ++e) expo(k * EA + e);
          a0 = b0;
          a1 = b1;
          __builtin_amdgcn_sched_barrier(0);
        }
        V8<T> p[4] = {pack8<T>(c0, 0), pack8<T>(c0, 1), pack8<T>(c1, 0), pack8<T>(c1, 1)};
        if (NEXT && DIAG) mask(n0, n1, (t + 1) * KT);
        // phase B: O^T += V_t^T P_t | row max of tile t+1
        V8<T> vc[2] = {lo.tr(Vt, 0, 0), lo.tr(Vt, (1 / NDB) * 16, 1 % NDB)};
#pragma unroll
        for (int k = 0; k < RB; ++k) {
          V8<T> vn[2] = {vc[0], vc[1]};
          if (k + 1 < RB) {
            const int s0 = 2 * (k + 1), s1 = s0 + 1;
            vn[0] = lo.tr(Vt, (s0 / NDB) * 16, s0 % NDB);
            vn[1] = lo.tr(Vt, (s1 / NDB) * 16, s1 % NDB);
          }
          const int s0 = 2 * k, s1 = s0 + 1;
          o[s0 % NDB] = mfma(vc[0], p[s0 / NDB], o[s0 % NDB]);
          o[s1 % NDB] = mfma(vc[1], p[s1 / NDB], o[s1 % NDB]);
          if (k < RB / 2) {
#pragma unroll
            for (int e = 0; e < EBX; ++e) expo(NEA + k * EBX + e);
            if (k == RB / 2 - 1) {  // P of keys 48..63 complete (first read in region 3 RB / 4)
              p[3] = pack8<T>(c1, 1);
              l_i += half_sum(rs);
            }
          }
          if (NEXT) {
#pragma unroll
            for (int e = 0; e < EB; ++e) {
              const int i = k * EB + e;
              mx = fmaxf(mx, i < 16 ? n0[i] : n1[i - 16]);
            }
          }
          vc[0] = vn[0];
          vc[1] = vn[1];
          __builtin_amdgcn_sched_barrier(0);
        }
        if (NEXT) {
#if PRA_FWD_PRESCALE
          mx = half_max(mx);  // max growth over m_i (the scores are relative to it)
          if (!__all(mx <= thr)) {  // deferred rescale (tile t's P.V is already in O)
            const float dlt = fmaxf(mx, 0.f);
            const float alpha = fexp2(-dlt);
            l_i *= alpha;
#pragma unroll
            for (int i = 0; i < NDB; ++i) o[i] *= alpha;
            m_i += dlt;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              n0[r] -= dlt;
              n1[r] -= dlt;
              negm[r] = -m_i;
            }
          }
#else
          mx = half_max(mx) * scale_log2;
          if (!__all(mx <= m_i + thr)) {  // deferred rescale (tile t's P.V is already in O)
            const float m_new = fmaxf(m_i, mx);
            const float alpha = fexp2(m_i - m_new);
            l_i *= alpha;
#pragma unroll
            for (int i = 0; i < NDB; ++i) o[i] *= alpha;
            m_i = m_new;
          }
#endif
          c0 = n0;
          c1 = n1;
        }
      };
      if (t + 1 > lastw) iter(std::false_type{}, std::false_type{});
      else if (CAUSAL && t + 1 == lastw) iter(std::true_type{}, std::true_type{});
      else iter(std::true_type{}, std::false_type{});
    }
    __syncthreads();  // tile t + 2 landed (vmcnt(0) before the barrier); tile t's slot is free
  };
  for (int t = 0; t < nkt; t += 3) {
    body(IC<0>{}, t);
    if (t + 1 < nkt) body(IC<1>{}, t + 1);
    if (t + 2 < nkt) body(IC<2>{}, t + 2);
  }

  {
    const float inv = 1.f / l_i;
    store_rows16<T, NDB>(o, inv, O + ((long)b * S + qrow) * ldo + hq * D, qrow < S, h2);
    if (qrow < S && h2 == 0) LSE[((long)b * Hq + hq) * S + qrow] = (m_i + __log2f(l_i)) * 0.69314718055994531f;
  }
}

// ======================================================================================
// Backward dK/dV: block = (b, kv head, 32*NW-key tile); wave owns 32 keys. K and V of the block
// stay resident in LDS (read as MFMA operands, so only the dK/dV accumulators live in registers
// and the kernel fits 2 waves/SIMD); 32-row Q/dO tiles stream through a single LDS buffer,
// register-staged one tile ahead. Loops over the query heads of the kv head (GQA) and query tiles.
//   S  = Q K^T   (key on lane)      P  = exp2(S*c - lse*log2e)
//   dP = dO V^T  (key on lane)      dS = P * (dP - delta)
//   dV^T += dO^T P                  dK^T += Q^T dS      (accumulators reused as B operands)
// NW = 8 (256 keys, 144 KB LDS, one 512-thread block per CU): each staged Q/dO tile feeds twice
// the keys per barrier, and the per-query constants are staged in LDS and read as float4.
// NW = 4 (128 keys, 80 KB, two blocks per CU): the constants arrive as one float per lane and are
// broadcast with ds_bpermute (no LDS left for them).
// ======================================================================================
// KREG (NW = 8 only): the wave's K row fragments (32 VGPRs at D = 128) are read from LDS once and
// kept in registers, cutting the per-tile LDS reads from 48 to 40 KB per wave.
template <typename T, int D, bool CAUSAL, int NW, bool KREG = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void bwd_dkdv_kernel(
    const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
    const T* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    T* __restrict__ dK, T* __restrict__ dV, int S, int Hq, int Hkv, long ldq, long ldk, long ldv,
    long lddo, long lddk, long lddv, float scale, float scale_log2, int skv, const float2* __restrict__ rtab,
    int grp) {
  constexpr int KB = 32 * NW, QT = 32, NT = NW * 64;
  constexpr int NKS = D / 16, NDB = D / 32;
  constexpr int KVT = KB * D, QDT = QT * D;
  constexpr bool ROWC_LDS = NW == 8;
  // Q and dO first: their (transposed) reads then use 16-bit immediate offsets off one base
  __shared__ __attribute__((aligned(16))) T smem[2 * KVT + 2 * QDT];  // Q dO K V
  __shared__ __attribute__((aligned(16))) float rowc[ROWC_LDS ? 2 : 1][32];  // lse*log2e | delta
  T* const Qs = smem;
  T* const Ds = smem + QDT;
  T* const Ks = smem + 2 * QDT;
  T* const Vs = smem + 2 * QDT + KVT;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nkb = S / KB;
  const int BH = gridDim.x / nkb;
  int kbk, bh;
  block_tile(nkb, BH, grp, kbk, bh);
  kbk = nkb - 1 - kbk;  // causal: early key tiles have the most work
  const int hk = bh % Hkv, b = bh / Hkv;
  const int nrep = Hq / Hkv;
  const int kg = wid;  // this wave's 32-key group
  const int k0 = kbk * KB, kw = k0 + kg * 32;
  const int krow = kw + l32;

  {
    GStage<T, D, KB, NW> gk, gv;
    gk.init(ldk);
    gv.init(ldv);
    gk.issue(K + ((long)b * S + k0) * ldk + hk * D, Ks);
    gv.issue(V + ((long)b * S + k0) * ldv + hk * D, Vs);
  }
  const T* Kw = Ks + kg * 32 * D;
  const T* Vw = Vs + kg * 32 * D;
  LaneOff<T, D> lo;
  lo.init(lane);

  f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) { dkt[i] = f32x16{}; dvt[i] = f32x16{}; }

  const int qstart = CAUSAL ? k0 : 0;
  const int nqt = (S - qstart) / QT;
  const int total = nqt * nrep;
  // lane reads the row constant of query row l32 of the tile: lse*log2e (h2 = 0) or delta (h2 = 1);
  // NW = 8 stages them negated: they are the S / dP accumulators' initial values (below)
  const float rc_mul = ROWC_LDS ? (h2 ? -1.f : -1.4426950408889634f) : (h2 ? 1.f : 1.4426950408889634f);
  const float* rc_base = (h2 ? Delta : LSE) + (long)b * Hq * S + l32;
  int bp_base = 4 * (4 * h2);  // ds_bpermute byte address of lane crow(0, h2)
  asm volatile("" : "+v"(bp_base));  // opaque: per-row offsets then fold into the ds offset field

  Stage<T, D, QT, NT> sq, sd;
  float rc_next = 0.f;
  auto stage_load = [&](int it) {
    const int hq = hk * nrep + it / nqt;
    const int q0 = qstart + (it % nqt) * QT;
    sq.load(Q + (long)b * S * ldq + hq * D, ldq, q0, S);
    sd.load(dO + (long)b * S * lddo + hq * D, lddo, q0, S);
    if (ROWC_LDS && wid == 0) rc_next = rc_base[(long)hq * S + q0] * rc_mul;
  };
  if (total > 0) stage_load(0);
  if constexpr (ROWC_LDS) {
    // K pre-multiplied by c = scale * log2(e) in LDS, once per block (one extra rounding of K to T):
    // each wave rescales its own 32 contiguous rows (8 KiB of the image), which only it reads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    char* kb = reinterpret_cast<char*>(Ks) + kg * 32 * D * (int)sizeof(T);
#pragma unroll
    for (int i = 0; i < 32 * D * (int)sizeof(T) / 1024; ++i) {
      V8<T>& c8 = *reinterpret_cast<V8<T>*>(kb + i * 1024 + lane * 16);
      V8<T> v8 = c8;
#pragma unroll
      for (int j = 0; j < 8; ++j) v8[j] = (T)((float)v8[j] * scale_log2);
      c8 = v8;
    }
  }
  static_assert(!KREG || ROWC_LDS, "KREG reads the prescaled K image of the NW = 8 kernel");
  V8<T> kf[KREG ? NKS : 1];
  if constexpr (KREG) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) kf[ks] = lo.rowk(Kw, 0, ks);  // the wave's own rows (rescaled above)
  }

  for (int it = 0; it < total; ++it) {
    const int hq = hk * nrep + it / nqt;
    const int q0 = qstart + (it % nqt) * QT;
    sq.store(Qs);
    sd.store(Ds);
    float rcv = 0.f;
    if constexpr (ROWC_LDS) {
      if (wid == 0) rowc[h2][l32] = rc_next;
    } else {
      rcv = rc_base[(long)hq * S + q0] * rc_mul;
    }
    __syncthreads();
    if (it + 1 < total) stage_load(it + 1);
    if (!(CAUSAL && q0 + QT - 1 < kw)) {
      const bool diag = CAUSAL && q0 == kw;
      f32x16 s = f32x16{}, dp = f32x16{};
      if constexpr (ROWC_LDS) {
        // S' = (c K) Q^T - lse log2(e), dP' = dO V^T - delta: the accumulators start at the
        // (negated) row constants of their query rows crow(r, h2); on the diagonal tile the causal
        // mask rides on the S initial values (-inf)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const float4 a = *reinterpret_cast<const float4*>(&rowc[0][8 * rr + 4 * h2]);
          const float4 c = *reinterpret_cast<const float4*>(&rowc[1][8 * rr + 4 * h2]);
          s[4 * rr] = a.x; s[4 * rr + 1] = a.y; s[4 * rr + 2] = a.z; s[4 * rr + 3] = a.w;
          dp[4 * rr] = c.x; dp[4 * rr + 1] = c.y; dp[4 * rr + 2] = c.z; dp[4 * rr + 3] = c.w;
        }
        if (diag) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (l32 > crow(r, h2)) s[r] = -INFINITY;
        }
      }
      // S chain then dP chain: one operand pair in flight ahead of each MFMA
      V8<T> xa = lo.rowk(Qs, 0, 0), xb = KREG ? kf[0] : lo.rowk(Kw, 0, 0);
#pragma unroll
      for (int st = 0; st < 2 * NKS; ++st) {
        const int ks = st % NKS;
        V8<T> na = xa, nb = xb;
        if (st + 1 < 2 * NKS) {
          const int nks = (st + 1) % NKS;
          na = lo.rowk(st + 1 < NKS ? Qs : Ds, 0, nks);
          if (KREG && st + 1 < NKS)
            nb = kf[KREG ? nks : 0];
          else
            nb = lo.rowk(st + 1 < NKS ? Kw : Vw, 0, nks);
        }
        if (st < NKS) s = mfma(xa, xb, s);
        else dp = mfma(xa, xb, dp);
        xa = na; xb = nb;
      }
      if constexpr (ROWC_LDS) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fexp2(s[r]);
          if (!CAUSAL && krow >= skv) p = 0.f;  // padded key
          s[r] = p;
          dp[r] = p * dp[r];
        }
      } else {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float lse4[4], dl4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int src = bp_base + 4 * (j + 8 * rr);
            lse4[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(rcv)));
            dl4[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(src + 128, __float_as_int(rcv)));
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * rr + j;
            float p = fexp2(fmaf(s[r], scale_log2, -lse4[j]));
            if (diag && l32 > crow(r, h2)) p = 0.f;
            if (!CAUSAL && krow >= skv) p = 0.f;  // padded key
            s[r] = p;
            dp[r] = p * (dp[r] - dl4[j]);
          }
        }
      }
      const V8<T> p0 = pack8<T>(s, 0), p1 = pack8<T>(s, 1), d0 = pack8<T>(dp, 0), d1 = pack8<T>(dp, 1);
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
        ot = no; qt = nq;
      }
    }
    __syncthreads();
  }

  // rtab: inverse RoPE on dK (table rows = positions; padded rows >= skv are discarded, clamp them)
  store_rows16<T, NDB>(dkt, scale, dK + ((long)b * S + krow) * lddk + hk * D, true, h2,
                       rtab ? rtab + (long)min(krow, skv - 1) * (D / 2) : nullptr);
  store_rows16<T, NDB>(dvt, 1.f, dV + ((long)b * S + krow) * lddv + hk * D, true, h2);
}

// ======================================================================================
// Backward dK/dV, ring-staged (NW = 8, S % 256 == 0): the bwd_dkdv_kernel<.., 8, .., KREG> math with
//  * K of the wave's 32 keys loaded straight from global memory into registers (pre-multiplied by
//    scale log2(e) there), so K takes no LDS and its 8 row reads per query tile are gone;
//  * V of the block resident in LDS (LDS-DMA), read as the dP chain's row operand;
//  * Q / dO tiles and their row constants (-lse log2(e), -delta: the dQ kernel's RC2 output) moved by
//    LDS-DMA into a double buffer one tile ahead: no VGPR staging, no ds_write, and ONE barrier per
//    32-query tile instead of two.
// LDS: 64 KB (V) + 2 x 16.25 KB at D = 128.
// ======================================================================================
template <typename T, int D, bool CAUSAL>
__global__ __launch_bounds__(512, 1) void bwd_dkdv_r_kernel(
    const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V, const T* __restrict__ dO,
    const float* __restrict__ RC, long nrc, T* __restrict__ dK, T* __restrict__ dV, int S, int Hq, int Hkv,
    long ldq, long ldk, long ldv, long lddo, long lddk, long lddv, float scale, float scale_log2, int skv,
    const float2* __restrict__ rtab, int grp) {
  constexpr int NW = 8, KB = 32 * NW, QT = 32;
  constexpr int NKS = D / 16, NDB = D / 32;
  constexpr int KVT = KB * D, QDT = QT * D;
  __shared__ __attribute__((aligned(16))) T Vs[KVT];
  // per buffer: Q | dO tiles, then 64 floats: -lse log2(e) [32] | -delta [32] (one object per buffer:
  // separate alias scopes, so reads of one buffer do not wait for the DMA filling the other)
  __shared__ __attribute__((aligned(16))) T qd0[2 * QDT];
  __shared__ __attribute__((aligned(16))) T qd1[2 * QDT];
  __shared__ __attribute__((aligned(16))) float rc0[64];
  __shared__ __attribute__((aligned(16))) float rc1[64];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nkb = S / KB;
  const int BH = gridDim.x / nkb;
  int kbk, bh;
  block_tile(nkb, BH, grp, kbk, bh);
  kbk = nkb - 1 - kbk;  // causal: early key tiles have the most work
  const int hk = bh % Hkv, b = bh / Hkv;
  const int nrep = Hq / Hkv;
  const int kg = wid;  // this wave's 32-key group
  const int k0 = kbk * KB, kw = k0 + kg * 32;
  const int krow = kw + l32;

  GStage<T, D, KB, NW> gv;
  gv.init(ldv);
  gv.issue(V + ((long)b * S + k0) * ldv + hk * D, Vs);
  GStage<T, D, QT, NW> gq, gd;
  gq.init(ldq);
  gd.init(lddo);
  const T* Kw = nullptr;
  (void)Kw;
  const T* Vw = Vs + kg * 32 * D;
  LaneOff<T, D> lo;
  lo.init(lane);

  // the wave's K rows as the S chain's B operand: lane holds K[krow][16 ks + 8 h2 .. + 7] * c
  V8<T> kf[NKS];
  {
    const T* kr = K + ((long)b * S + krow) * ldk + hk * D + 8 * h2;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = *reinterpret_cast<const V8<T>*>(kr + 16 * ks);
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[ks][j] = (T)((float)kf[ks][j] * scale_log2);
    }
  }

  f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) { dkt[i] = f32x16{}; dvt[i] = f32x16{}; }

  const int qstart = CAUSAL ? k0 : 0;
  const int nqt = (S - qstart) / QT;
  const int total = nqt * nrep;
  const long rc_b = (long)b * Hq * S;
  auto issue = [&](int it, T* qd, float* rc) {
    const int hq = hk * nrep + it / nqt;
    const int q0 = qstart + (it % nqt) * QT;
    gq.issue(Q + ((long)b * S + q0) * ldq + hq * D, qd);
    gd.issue(dO + ((long)b * S + q0) * lddo + hq * D, qd + QDT);
    if (wid == 0 && lane < 16) {  // 2 x 128 B of row constants: lanes 0-7 -lse log2(e), 8-15 -delta
      const float* src = RC + (lane < 8 ? 0 : nrc) + rc_b + (long)hq * S + q0 + 4 * (lane & 7);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)rc, 16, 0, 0);
    }
  };
  if (total > 0) issue(0, qd0, rc0);
  __syncthreads();  // V and tile 0 landed (vmcnt(0) before the barrier)

  auto body = [&](auto cc, int it) {
    constexpr int CUR = decltype(cc)::value;
    T* const qd = CUR ? qd1 : qd0;
    const float* rc = CUR ? rc1 : rc0;
    if (it + 1 < total) issue(it + 1, CUR ? qd0 : qd1, CUR ? rc0 : rc1);
    const T* Qs = qd;
    const T* Ds = qd + QDT;
    const int q0 = qstart + (it % nqt) * QT;
    if (!(CAUSAL && q0 + QT - 1 < kw)) {
      const bool diag = CAUSAL && q0 == kw;
      // S' = (c K) Q^T - lse log2(e), dP' = dO V^T - delta: the accumulators start at the row
      // constants of their query rows crow(r, h2); the causal mask rides on S's initial values
      f32x16 sa, dp;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 a = *reinterpret_cast<const float4*>(rc + 8 * rr + 4 * h2);
        const float4 c = *reinterpret_cast<const float4*>(rc + 32 + 8 * rr + 4 * h2);
        sa[4 * rr] = a.x; sa[4 * rr + 1] = a.y; sa[4 * rr + 2] = a.z; sa[4 * rr + 3] = a.w;
        dp[4 * rr] = c.x; dp[4 * rr + 1] = c.y; dp[4 * rr + 2] = c.z; dp[4 * rr + 3] = c.w;
      }
      if (diag) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (l32 > crow(r, h2)) sa[r] = -INFINITY;
      }
      V8<T> xa = lo.rowk(Qs, 0, 0), xb = kf[0];
#pragma unroll
      for (int st = 0; st < 2 * NKS; ++st) {
        const int ks = st % NKS;
        V8<T> na = xa, nb = xb;
        if (st + 1 < 2 * NKS) {
          const int nks = (st + 1) % NKS;
          na = lo.rowk(st + 1 < NKS ? Qs : Ds, 0, nks);
          nb = st + 1 < NKS ? kf[nks] : lo.rowk(Vw, 0, nks);
        }
        if (st < NKS) sa = mfma(xa, xb, sa);
        else dp = mfma(xa, xb, dp);
        xa = na; xb = nb;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fexp2(sa[r]);
        if (!CAUSAL && krow >= skv) p = 0.f;  // padded key
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
        ot = no; qt = nq;
      }
    }
    __syncthreads();  // tile it + 1 landed; this buffer is free for tile it + 2
  };
  for (int it = 0; it < total; it += 2) {
    body(IC<0>{}, it);
    if (it + 1 < total) body(IC<1>{}, it + 1);
  }

  store_rows16<T, NDB>(dkt, scale, dK + ((long)b * S + krow) * lddk + hk * D, true, h2,
                       rtab ? rtab + (long)min(krow, skv - 1) * (D / 2) : nullptr);
  store_rows16<T, NDB>(dvt, 1.f, dV + ((long)b * S + krow) * lddv + hk * D, true, h2);
}

// ======================================================================================
// Backward dK/dV, one wave per SIMD, two query sub-tiles in flight: block = (b, kv head, 128
// keys), 4 waves x 32 keys; each step stages 64 queries (sub-tiles A and B of 32). With the whole
// 512-entry register file per wave, a wave keeps S/dP of both sub-tiles live and runs them as a
// two-stage pipeline, the softmax VALU of one sub-tile interleaved (sched_group_barrier) between
// the MFMAs of the other -- instead of two waves per SIMD alternating MFMA and VALU phases in
// lockstep between barriers (bwd_dkdv_kernel):
//   [S,dP of A] -> [S,dP of B | softmax A] -> [dV,dK += A | softmax B] -> [dV,dK += B]
// K/V of the block land in LDS (64 KB at D = 128) and each wave keeps its own rows' fragments in
// registers from then on. Q/dO steps (32 KB) and their per-query constants arrive by LDS-DMA into a
// double buffer, issued one step ahead. The constants are -lse log2(e) and -delta, written by the dQ
// kernel (RC2), and they are the INITIAL values of the S and dP accumulators; with K pre-multiplied
// by c = scale log2(e) and the causal mask folded into the S initial values on diagonal steps,
// S' = (c K) Q^T - lse log2(e) and dP' = dO V^T - delta leave the MFMA chains ready: each score
// costs exp2(S') and dS = P dP' (4 VALU fewer per element than exp2(fma(S, c, -lse log2e)), a mask
// select and P (dP - delta), in this VALU-bound one-wave kernel).
// ======================================================================================
template <typename T, int D, bool CAUSAL>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void bwd_dkdv_p2_kernel(
    const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
    const T* __restrict__ dO, const float* __restrict__ NLS, const float* __restrict__ NDelta,
    T* __restrict__ dK, T* __restrict__ dV, int S, int Hq, int Hkv, long ldq, long ldk, long ldv,
    long lddo, long lddk, long lddv, float scale, float scale_log2, int skv, const float2* __restrict__ rtab,
    int nsplit, float* __restrict__ part) {
  constexpr int NW = 4, KB = 32 * NW, QS = 64;
  constexpr int NKS = D / 16, NDB = D / 32;
  constexpr int KVT = KB * D, QDT = QS * D;
  // Q0 dO0 Q1 dO1 (steps, double-buffered) | K V | row constants [buf][-lse log2(e), -delta][64]
  __shared__ __attribute__((aligned(16))) T smem[4 * QDT + 2 * KVT];
  __shared__ __attribute__((aligned(16))) float rowc[2][2][QS];
  T* const Ks = smem + 4 * QDT;
  T* const Vs = Ks + KVT;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nkb = S / KB;
  const int BH = gridDim.x / nkb;
  const int kbk = (int)(blockIdx.x / BH);  // causal: early key blocks have the most work
  const int bh = blockIdx.x % BH;  // (b, kv head, split)
  const int sp = bh % nsplit, hk = (bh / nsplit) % Hkv, b = bh / (nsplit * Hkv);
  // split > 1: the block covers nrep of the kv head's Hq / Hkv query heads and leaves fp32 partial
  // dK/dV in `part` for dkdv_reduce_kernel (small grids: see dkdv_split)
  const int nrep = (Hq / Hkv) / nsplit;
  const int hq0 = hk * (Hq / Hkv) + sp * nrep;
  const int k0 = kbk * KB, kw = k0 + wid * 32;

  GStage<T, D, QS, NW> gq, gd;
  gq.init(ldq);
  gd.init(lddo);
  const int qstart = CAUSAL ? k0 : 0;
  const int nqs = (S - qstart) / QS;
  const int total = nqs * nrep;
  auto issue_step = [&](int t, int buf) {
    const int hq = hq0 + t / nqs;
    const int q0 = qstart + (t % nqs) * QS;
    gq.issue(Q + ((long)b * S + q0) * ldq + hq * D, smem + buf * 2 * QDT);
    gd.issue(dO + ((long)b * S + q0) * lddo + hq * D, smem + buf * 2 * QDT + QDT);
    if (wid < 2) {  // wave 0: -lse log2(e), wave 1: -delta (one dword per lane)
      const float* src = (wid ? NDelta : NLS) + ((long)b * Hq + hq) * S + q0 + lane;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)&rowc[buf][wid][0], 4, 0, 0);
    }
  };
  {
    GStage<T, D, KB, NW> gk, gv;
    gk.init(ldk);
    gv.init(ldv);
    gk.issue(K + ((long)b * S + k0) * ldk + hk * D, Ks);
    gv.issue(V + ((long)b * S + k0) * ldv + hk * D, Vs);
  }
  if (total > 0) issue_step(0, 0);
  const T* Kw = Ks + wid * 32 * D;
  const T* Vw = Vs + wid * 32 * D;
  LaneOff<T, D> lo;
  lo.init(lane);

  f32x16 dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) { dkt[i] = f32x16{}; dvt[i] = f32x16{}; }
  __syncthreads();  // K/V and step 0 have landed
  // the wave's K and V row fragments (B operands of S and dP, the same for every step) are read
  // from LDS once and kept in registers (B1 S8192 H32/8 dK/dV+dQ 1.871 -> 1.851 ms,
  // profiles/r3/attn_ab_kvreg.log)
  // K is pre-multiplied by c = scale * log2(e) once (one extra rounding of K to T), so S = (c K) Q^T
  // needs no per-score multiply before its exp2
  V8<T> kf[NKS], vf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    kf[ks] = lo.rowk(Kw, 0, ks);
#pragma unroll
    for (int j = 0; j < 8; ++j) kf[ks][j] = (T)((float)kf[ks][j] * scale_log2);
    vf[ks] = lo.rowk(Vw, 0, ks);
  }

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int q0 = qstart + (it % nqs) * QS;
    if (it + 1 < total) issue_step(it + 1, 1 - cur);  // lands under this step's MFMAs
    const T* Qs = smem + cur * 2 * QDT;
    const T* Ds = Qs + QDT;
    const float* lrow = &rowc[cur][0][0];
    const float* drow = &rowc[cur][1][0];

    // a score (query q0 + 32 u + crow(r, h2), key kw + l32) is masked iff crow(r, 0) < lim - 32 u
    //
    // The step is written as 2 * (NKS + 2 NDB) explicit regions separated by sched_barrier(0), each
    // issuing the LDS reads of the NEXT region's MFMA operands, its own two MFMAs, and a slice of the
    // pending softmax (VALU), so every MFMA gap carries VALU work:
    //   regions [0, NKS)            S, dP of sub-tile A
    //   [NKS, 2 NKS)                S, dP of B        | softmax of A (16 / NKS rows per region)
    //   [2 NKS, 2 NKS + 2 NDB)      dV, dK += A       | softmax of B
    //   [2 NKS + 2 NDB, end)        dV, dK += B
    auto step = [&](auto mask_c) {
      constexpr bool MASK = decltype(mask_c)::value;
      constexpr int R1 = NKS, R3 = 2 * NDB, NR = 2 * R1 + 2 * R3;
      constexpr int EA = 16 / R1, EB = 16 / R3;  // softmax rows per region
      const int lim = kw + l32 - q0 - 4 * h2;
      // accumulators start at the row constants of their query rows (register r: row crow(r, h2))
      auto rc16 = [&](const float* row) {
        f32x16 a;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const f32x4 c = *reinterpret_cast<const f32x4*>(row + 8 * rr + 4 * h2);
          a[4 * rr] = c[0]; a[4 * rr + 1] = c[1]; a[4 * rr + 2] = c[2]; a[4 * rr + 3] = c[3];
        }
        return a;
      };
      f32x16 sa = rc16(lrow), sb = rc16(lrow + 32), pa = rc16(drow), pb = rc16(drow + 32);
      // the causal mask rides on the S initial values (-inf: exp2 gives exactly 0), and only on the
      // steps that cross the diagonal (wave-uniform), so the softmax itself carries no mask select
      if (MASK && q0 < kw + 32) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (crow(r, 0) < lim) sa[r] = -INFINITY;
          if (crow(r, 0) < lim - 32) sb[r] = -INFINITY;
        }
      }
      V8<T> pA[2], gA[2], pB[2], gB[2];
      auto fetch = [&](int k, V8<T> (&o)[4]) {
        if (k < 2 * R1) {
          const int ks = k % R1, r0 = 32 * (k / R1);
          o[0] = lo.rowk(Qs, r0, ks);
          o[2] = lo.rowk(Ds, r0, ks);
          o[1] = kf[ks];
          o[3] = vf[ks];
        } else if (k < NR) {
          const int st = (k - 2 * R1) % R3, s2 = st / NDB, db = st % NDB, r0 = 32 * ((k - 2 * R1) / R3);
          o[0] = lo.tr(Ds, r0 + 16 * s2, db);
          o[1] = lo.tr(Qs, r0 + 16 * s2, db);
        }
      };
      auto soft = [&](f32x16& sv, f32x16& dp, int u, int r) {
        float p = fexp2(sv[r]);  // sv = (c K) Q^T - lse log2(e), -inf where masked
        if (!CAUSAL && kw + l32 >= skv) p = 0.f;  // padded key
        sv[r] = p;
        dp[r] = p * dp[r];  // dp = dP - delta
      };
      V8<T> cur[4], nxt[4];
      fetch(0, cur);
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        fetch(k + 1, nxt);
        if (k < R1) {
          sa = mfma(cur[0], cur[1], sa);
          pa = mfma(cur[2], cur[3], pa);
        } else if (k < 2 * R1) {
          sb = mfma(cur[0], cur[1], sb);
          pb = mfma(cur[2], cur[3], pb);
#pragma unroll
          for (int e = 0; e < EA; ++e) soft(sa, pa, 0, (k - R1) * EA + e);
          if (k == 2 * R1 - 1) {
            pA[0] = pack8<T>(sa, 0); pA[1] = pack8<T>(sa, 1); gA[0] = pack8<T>(pa, 0); gA[1] = pack8<T>(pa, 1);
          }
        } else {
          const int j = k - 2 * R1, st = j % R3, s2 = st / NDB, db = st % NDB;
          const bool second = j >= R3;
          dvt[db] = mfma(cur[0], second ? pB[s2] : pA[s2], dvt[db]);
          dkt[db] = mfma(cur[1], second ? gB[s2] : gA[s2], dkt[db]);
          if (!second) {
#pragma unroll
            for (int e = 0; e < EB; ++e) soft(sb, pb, 1, j * EB + e);
            if (j == R3 - 1) {
              pB[0] = pack8<T>(sb, 0); pB[1] = pack8<T>(sb, 1); gB[0] = pack8<T>(pb, 0); gB[1] = pack8<T>(pb, 1);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // one code path (the causal mask is a per-element select that is a no-op off the diagonal
    // band): a second instantiation makes the compiler shuffle the AGPR accumulators between them
    if (!CAUSAL || q0 + QS - 1 >= kw) step(std::integral_constant<bool, CAUSAL>{});  // else fully masked
    __syncthreads();  // next step landed (vmcnt(0) before the barrier); this step's buffer is free
  }

  const int krow = kw + l32;
  // rtab: inverse RoPE on dK (table rows = positions; padded rows >= skv are discarded, clamp them)
  const float2* rt = rtab ? rtab + (long)min(krow, skv - 1) * (D / 2) : nullptr;
  if (part == nullptr) {
    store_rows16<T, NDB>(dkt, scale, dK + ((long)b * S + krow) * lddk + hk * D, true, h2, rt);
    store_rows16<T, NDB>(dvt, 1.f, dV + ((long)b * S + krow) * lddv + hk * D, true, h2);
  } else {  // [split][dK, dV][B][S][Hkv][D] fp32 (scale and inverse RoPE are linear: applied per part)
    const long n = (long)(BH / nsplit) * S * D;
    float* pk = part + (long)sp * 2 * n + ((long)b * S + krow) * Hkv * D + hk * D;
    store_rows16_f32<NDB>(dkt, scale, pk, h2, rt);
    store_rows16_f32<NDB>(dvt, 1.f, pk + n, h2);
  }
}

// dK, dV = sum of the split dK/dV kernel's fp32 parts (fixed order: deterministic), cast to T
template <typename T>
__global__ __launch_bounds__(256) void dkdv_reduce_kernel(const float* __restrict__ part, int nsplit, long n, int hd,
                                                          T* __restrict__ dK, long lddk, T* __restrict__ dV,
                                                          long lddv) {
  const long e = ((long)blockIdx.x * 256 + threadIdx.x) * 4;  // n % 4 == 0, hd % 4 == 0
  if (e >= 2 * n) return;
  float4 a = *reinterpret_cast<const float4*>(part + e);
  for (int j = 1; j < nsplit; ++j) {
    const float4 c = *reinterpret_cast<const float4*>(part + (long)j * 2 * n + e);
    a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
  }
  const bool isv = e >= n;
  const long r = isv ? e - n : e, tok = r / hd;
  T* dst = (isv ? dV + tok * lddv : dK + tok * lddk) + (r - tok * hd);
  *reinterpret_cast<uint2*>(dst) = make_uint2(pack_x2<T>(a.x, a.y), pack_x2<T>(a.z, a.w));
}

// ======================================================================================
// Backward dQ: block = (b, q head, 128 query rows), wave owns 32 queries; loop over 64-key tiles
// (double-buffered in LDS, staged issue-early / write-late).
//   S^T = K Q^T, dP^T = V dO^T (query on lane; lse/delta are lane constants)
//   dQ^T += K^T dS^T
// ======================================================================================
// PIPE: the same tile work as explicit sched_barrier regions -- S/dP of the second 32-key half
// interleaved with the softmax of the first, dQ of the first with the softmax of the second (see
// bwd_dkdv_p2_kernel) -- instead of two back-to-back MFMA -> VALU -> MFMA halves.
template <typename T, int D, bool CAUSAL, int NW, bool PIPE = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void bwd_dq_kernel(
    const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
    const T* __restrict__ dO, const T* __restrict__ O, const float* __restrict__ LSE, float* __restrict__ Delta,
    T* __restrict__ dQ, int S, int Hq, int Hkv, long ldq, long ldk, long ldv, long lddo, long ldo, long lddq,
    float scale, float scale_log2, int skv, const float2* __restrict__ rtab, float* __restrict__ RC2, long nrc,
    int grp) {
  constexpr int KT = 64, QT = 32 * NW;
  constexpr int NKS = D / 16, NDB = D / 32, TILE = KT * D;
  // K0 V0 | K1 V1: one __shared__ object per buffer, so the reads of one buffer do not wait
  // (vmcnt(0)) for the LDS-DMA filling the other (per-object alias scopes; see fwd_p_kernel)
  __shared__ __attribute__((aligned(16))) T kvb0[2 * TILE];
  __shared__ __attribute__((aligned(16))) T kvb1[2 * TILE];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h2 = lane >> 5, l32 = lane & 31;
  const int nqt = (S + QT - 1) / QT;
  const int BH = gridDim.x / nqt;
  int qt, bh;
  block_tile(nqt, BH, grp, qt, bh);
  const int hq = bh % Hq, b = bh / Hq;
  const int hk = hq / (Hq / Hkv);
  const int q0 = qt * QT, qw = q0 + wid * 32;
  const int qrow = qw + l32;

  const T* Kb = K + (long)b * S * ldk + hk * D;
  const T* Vb = V + (long)b * S * ldv + hk * D;

  LaneOff<T, D> lo;
  lo.init(lane);
  V8<T> qf[NKS], df[NKS];
  {
    const T* Qr = Q + ((long)b * S + qrow) * ldq + hq * D + 8 * h2;
    const T* Dr = dO + ((long)b * S + qrow) * lddo + hq * D + 8 * h2;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (qrow < S) {
        qf[ks] = *reinterpret_cast<const V8<T>*>(Qr + 16 * ks);
        df[ks] = *reinterpret_cast<const V8<T>*>(Dr + 16 * ks);
      } else {
        qf[ks] = V8<T>{};
        df[ks] = V8<T>{};
      }
    }
  }
  // delta = rowsum(dO * O) of this lane's query row, computed here (this kernel runs before the
  // dK/dV kernel and publishes it; no separate preprocess pass): the lane holds half of the dO row
  // (columns 16 ks + 8 h2 ..), its partner lane l ^ 32 the other half.
  float lse2 = 0.f, dl = 0.f;
  {
    float part = 0.f;
    if (qrow < S) lse2 = LSE[((long)b * Hq + hq) * S + qrow] * 1.4426950408889634f;
    if (qrow < S) {
      const T* Orow = O + ((long)b * S + qrow) * ldo + hq * D + 8 * h2;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const V8<T> o8 = *reinterpret_cast<const V8<T>*>(Orow + 16 * ks);
#pragma unroll
        for (int j = 0; j < 8; ++j) part = fmaf((float)o8[j], (float)df[ks][j], part);
      }
    }
    dl = half_sum(part);  // all 64 lanes (permlane32 swap)
#if PRA_DQ_PRESCALE
    // PIPE path: Q pre-multiplied by scale log2(e) (as the forward's PRA_FWD_PRESCALE), and the S / dP
    // accumulators start at -lse log2(e) / -delta, so p = exp2(S') and dS = p dP' need no FMA / sub
    if (PIPE) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[ks][j] = (T)((float)qf[ks][j] * scale_log2);
    }
#endif
    if (qrow < S && h2 == 0) {
      const long i = ((long)b * Hq + hq) * S + qrow;
      Delta[i] = dl;
      if (RC2 != nullptr) {  // row constants of the pipelined dK/dV kernel: -lse log2(e), -delta
        RC2[i] = -lse2;
        RC2[nrc + i] = -dl;
      }
    }
  }

  f32x16 dqt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dqt[i] = f32x16{};

  const int kend = CAUSAL ? min(S, q0 + QT) : S;
  const int nkt = (kend + KT - 1) / KT;

  GStage<T, D, KT, NW> gk, gv;
  gk.init(ldk);
  gv.init(ldv);
  gk.issue(Kb, kvb0);
  gv.issue(Vb, kvb0 + TILE);
  __syncthreads();
  auto body = [&](auto cc, int kt) {
    constexpr int CUR = decltype(cc)::value;
    T* const cur_b = CUR ? kvb1 : kvb0;
    T* const oth_b = CUR ? kvb0 : kvb1;
    const T* Kt = cur_b;
    const T* Vt = Kt + TILE;
    const int k0 = kt * KT;
    if (kt + 1 < nkt) {  // LDS-DMA of the next tile runs under this tile's MFMAs
      gk.issue(Kb + (long)(k0 + KT) * ldk, oth_b);
      gv.issue(Vb + (long)(k0 + KT) * ldv, oth_b + TILE);
    }
    if constexpr (PIPE) {
      // a score (key k0 + 32 kb + crow(r, h2), query qrow) is masked iff crow(r, 0) > lim - 32 kb
      auto tile = [&](auto mask_c) {
        constexpr bool MASK = decltype(mask_c)::value;
        constexpr int R1 = NKS, R3 = NDB, NR = 2 * R1 + 2 * R3;
        constexpr int EA = 16 / R1, EB = 16 / R3;
        const int lim = qrow - k0 - 4 * h2;
#if PRA_DQ_PRESCALE == 1
        f32x16 s0, s1, p0, p1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s0[r] = -lse2;
          p0[r] = -dl;
        }
        s1 = s0;
        p1 = p0;
#elif PRA_DQ_PRESCALE == 2  // S chains only (16 registers of constants instead of 32)
        f32x16 s0, s1, p0 = f32x16{}, p1 = f32x16{};
#pragma unroll
        for (int r = 0; r < 16; ++r) s0[r] = -lse2;
        s1 = s0;
#else
        f32x16 s0 = f32x16{}, s1 = f32x16{}, p0 = f32x16{}, p1 = f32x16{};
#endif
        V8<T> g0[2], g1[2];
        auto fetch = [&](int k, V8<T> (&o)[4]) {
          if (k < 2 * R1) {
            const int ks = k % R1, r0 = 32 * (k / R1);
            o[0] = lo.rowk(Kt, r0, ks);
            o[1] = lo.rowk(Vt, r0, ks);
          } else if (k < NR) {
            const int j = (k - 2 * R1) % R3, r0 = 32 * ((k - 2 * R1) / R3);
            // two dQ MFMAs per region: steps st = 2 j, 2 j + 1 (s2 = st / NDB, db = st % NDB)
            o[0] = lo.tr(Kt, r0 + 16 * ((2 * j) / NDB), (2 * j) % NDB);
            o[2] = lo.tr(Kt, r0 + 16 * ((2 * j + 1) / NDB), (2 * j + 1) % NDB);
          }
        };
        auto soft = [&](f32x16& sv, f32x16& dp, int kb, int r) {
#if PRA_DQ_PRESCALE == 1
          float p = fexp2(sv[r]);
          if (MASK && crow(r, 0) > lim - 32 * kb) p = 0.f;
          dp[r] = p * dp[r];
#elif PRA_DQ_PRESCALE == 2
          float p = fexp2(sv[r]);
          if (MASK && crow(r, 0) > lim - 32 * kb) p = 0.f;
          dp[r] = p * (dp[r] - dl);
#else
          float p = fexp2(fmaf(sv[r], scale_log2, -lse2));
          if (MASK && crow(r, 0) > lim - 32 * kb) p = 0.f;
          dp[r] = p * (dp[r] - dl);
#endif
        };
        V8<T> cur[4], nxt[4];
        fetch(0, cur);
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          fetch(k + 1, nxt);
          if (k < 2 * R1) {
            const int ks = k % R1;
            if (k < R1) {
              s0 = mfma(cur[0], qf[ks], s0);
              p0 = mfma(cur[1], df[ks], p0);
            } else {
              s1 = mfma(cur[0], qf[ks], s1);
              p1 = mfma(cur[1], df[ks], p1);
#pragma unroll
              for (int e = 0; e < EA; ++e) soft(s0, p0, 0, (k - R1) * EA + e);
              if (k == 2 * R1 - 1) { g0[0] = pack8<T>(p0, 0); g0[1] = pack8<T>(p0, 1); }
            }
          } else {
            const int jj = k - 2 * R1, j = jj % R3;
            const bool second = jj >= R3;
            const int st0 = 2 * j, st1 = 2 * j + 1;
            dqt[st0 % NDB] = mfma(cur[0], second ? g1[st0 / NDB] : g0[st0 / NDB], dqt[st0 % NDB]);
            dqt[st1 % NDB] = mfma(cur[2], second ? g1[st1 / NDB] : g0[st1 / NDB], dqt[st1 % NDB]);
            if (!second) {
#pragma unroll
              for (int e = 0; e < EB; ++e) soft(s1, p1, 1, j * EB + e);
              if (j == R3 - 1) { g1[0] = pack8<T>(p1, 0); g1[1] = pack8<T>(p1, 1); }
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (!CAUSAL || k0 + KT - 1 <= qw) tile(std::false_type{});  // (non-causal + padded keys: PIPE off)
      else if (k0 <= qw + 31) tile(std::true_type{});  // diagonal tile (else fully masked)
    } else {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int kh = k0 + 32 * kb;
      if (CAUSAL && kh > qw + 31) continue;  // wave-uniform: this key half is fully masked
      f32x16 s = f32x16{}, dp = f32x16{};
      V8<T> ka = lo.rowk(Kt, 32 * kb, 0), va = lo.rowk(Vt, 32 * kb, 0);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        V8<T> nk = ka, nv = va;
        if (ks + 1 < NKS) {
          nk = lo.rowk(Kt, 32 * kb, ks + 1);
          nv = lo.rowk(Vt, 32 * kb, ks + 1);
        }
        s = mfma(ka, qf[ks], s);
        dp = mfma(va, df[ks], dp);
        ka = nk; va = nv;
      }
      const bool diag = CAUSAL && kh + 31 > qw;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fexp2(fmaf(s[r], scale_log2, -lse2));
        if (diag && kh + crow(r, h2) > qrow) p = 0.f;
        if (!CAUSAL && kh + crow(r, h2) >= skv) p = 0.f;  // padded key
        dp[r] = p * (dp[r] - dl);
      }
      const V8<T> d0 = pack8<T>(dp, 0), d1 = pack8<T>(dp, 1);
      V8<T> kc = lo.tr(Kt, 32 * kb, 0);
#pragma unroll
      for (int st = 0; st < 2 * NDB; ++st) {
        const int s2 = st / NDB, db = st % NDB;
        V8<T> kn = kc;
        if (st + 1 < 2 * NDB) kn = lo.tr(Kt, 32 * kb + 16 * ((st + 1) / NDB), (st + 1) % NDB);
        dqt[db] = mfma(kc, s2 ? d1 : d0, dqt[db]);
        kc = kn;
      }
    }
    }
    __syncthreads();  // the DMA'd tile has landed (vmcnt(0)) and this tile is free
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    body(IC<0>{}, kt);
    if (kt + 1 < nkt) body(IC<1>{}, kt + 1);
  }

  store_rows16<T, NDB>(dqt, scale, dQ + ((long)b * S + qrow) * lddq + hq * D, qrow < S, h2,
                       rtab ? rtab + (long)min(qrow, skv - 1) * (D / 2) : nullptr);
}

}  // namespace attn
}  // namespace pra

using namespace pra::attn;

namespace {

// Kernel selection knobs. Set through pra_attn_set_options (pyrecover_amd.ops.fused reads the
// PYRECOVER_ATTN_* environment once; tests switch them per case); the launchers read no environment.
struct AttnOptions {
  // forward: -1 = by shape (pipelined fwd_p_kernel for causal, fwd_kernel for full attention),
  // 0 = fwd_kernel, 1 = fwd_p_kernel (a 16x16x32 forward of fwd_kernel's structure measured 0.766 vs
  // 0.727 ms for fwd_p_kernel, profiles/r5/attn/fwd16_vs_fwd.log, and was removed). The pipelined kernel's non-causal instantiation spills at
  // D = 128, and padded non-causal keys (skv < S) need fwd_kernel's key bound.
  // (B8 S2048 H32: 0.460 -> 0.422 ms; S8192 H32/8: 0.654 -> 0.615 ms with the pipelined kernel.)
  int fwd_pipe = -1;
  // Rescale threshold of the pipelined forward (cdna guide T13), log2 units: O and l are rescaled
  // only when some row's max grows by more than thr, so P stays below 2^thr (fp32 accumulators;
  // bf16 P keeps its relative precision). 0 = exact rescale at every growth.
  float fwd_thr = 8.f;
  // dK/dV: -1 = by shape (dkdv_use_p2), 0 = two-wave bwd_dkdv_kernel, 1 = pipelined bwd_dkdv_p2_kernel
  int dkdv_impl = -1;
  // dQ: -1/1 = region-pipelined bwd_dq_kernel<PIPE>, 0 = plain (padded non-causal keys: always plain)
  int dq_pipe = -1;
  // pipelined dK/dV kernel, query heads per block: 1 = all of the kv head's Hq / Hkv heads in one
  // block (default), n = Hq / Hkv / n heads per block plus an fp32 reduction, -1 = by grid size
  // (dkdv_split) when no side-stream job waits for the window. Not by default: it pays only without
  // the overlapped optimizer, and its fp32 partial sums would make the gradients depend on whether
  // the optimizer overlaps (tests/test_xgmi_gpu.py compares the two bitwise)
  int dkdv_split = 1;
  // two-wave dK/dV kernel (NW = 8, D = 128): 2 = ring-staged bwd_dkdv_r_kernel (K in registers,
  // Q/dO by LDS-DMA, one barrier per query tile; B16 S2048 H32 bwd 2.39 -> 2.27 ms,
  // profiles/r5/attn/harness_dkdv_ring.log), 1 = bwd_dkdv_kernel with K fragments held in registers
  // (KREG), 0 = bwd_dkdv_kernel reading K from LDS, -1 = KREG unless a side-stream job waits for the
  // dK/dV window (below) (r4: KREG 2.387 -> 2.358 ms alone, but 1058.0 vs 1055.5 ms in the 7B step:
  // profiles/r4/attn_ab_dkdv_kreg_b16.log, step_ab_7b_b16_kreg.log), -2 (default) = the ring kernel
  // unless a side-stream job waits for the window, else 0: the ring kernel's 242 VGPRs leave no
  // room on the SIMDs for the overlapped AdamW waves (the LDS kernel's 215 do), so in the overlapped
  // 7B B16 step it is not faster (1054.7 vs 1053.3 ms, profiles/r5/step_ab_ring.log)
  int dkdv_kreg = -2;
  // fused backward (attention_bwd_fused.hip: dQ, dK, dV in one workgroup per (batch, kv head)):
  // -1 = by shape (attn_bwd_use_fused), 0 = never (split dQ + dK/dV kernels; the default), 1 = whenever
  // it applies. Not the default: alone it is faster (7B B16 step without the AdamW update 1032.7 ->
  // 1025.7 ms), but its 256-VGPR waves leave no room for the overlapped update's waves, which the split
  // dK/dV kernel hosts (with the update 1045.4 vs 1048.3 ms; profiles/r5/attn_fused/). The choice must
  // not depend on the window (dQ differs in the last bits), so it is a run-wide setting.
  int bwd_fused = 0;
  // where the side-stream window (mid_event) opens in the split backward: 0 = between the dQ and
  // the dK/dV kernels, 1 = before the dQ kernel (the update then runs beside both), -1 (default) = by
  // shape (window_before_dq): before dQ at <= 4096 tokens per call, where the dK/dV kernel alone is
  // too short a window (same-process A/B: Llama-3-8B B1 S2048 110.06 -> 109.61 ms, 7B B1 98.62 ->
  // 97.96 ms; at 8192 tokens slower: 8B S8192 B1 +2.35%, 8B S2048 B4 +0.33%, 7B B16 +0.5%;
  // profiles/r5/window/). Bitwise neutral: only the event moves.
  int bwd_window = -1;
  // block order of the pipelined forward (block_tile): 0 = heavy query tiles first across the grid,
  // G > 0 = XCD-grouped, G heads per group; -1 = by shape (attn_grp)
  int fwd_order = 0;
  int dq_order = 0;    // the same for the dQ kernel
  int dkdv_order = 0;  // and the two-wave / ring dK/dV kernels (key tiles, lightest last)
  // (A higher s_setprio for the backward kernels' waves than the overlapped AdamW update's, 1 or 3,
  // dK/dV and dQ: neutral in the 7B B16 step, 1058.0 / 1058.2 vs 1058.0 ms; profiles/r6/
  // step_ab_7b_b16_bwd_prio.log. Removed.)
};
AttnOptions g_attn_opts;

static bool window_before_dq(int B, int S) {
  const int w = g_attn_opts.bwd_window;
  return w == 1 || (w < 0 && (long)B * S <= 4096);
}

// Heads per XCD group for an nqt x BH grid under option `order`, 0 when the grid does not split.
// By shape (order < 0): at least the rep = Hq / Hkv query heads that share a kv head (forward and dQ
// grids; 1 for the dK/dV grids, whose heads are kv heads), and at least 32 blocks (one per CU of
// an XCD) per group. B16 S2048 H32 D128 causal (harness, profiles/r5/attn_order/): forward
// 0.740 -> 0.650 ms, dQ + dK/dV 2.31 -> 2.11 ms; B1 S8192 H32/8 forward 0.508 -> 0.499 ms.
static int attn_grp(int order, int nqt, int BH, int rep) {
  if (order == 0 || BH % 8) return 0;
  int g = order > 0 ? order : 1;
  if (order < 0)
    while ((g * 2 <= rep || g * 2 * nqt <= 32) && (BH / 8) % (g * 2) == 0) g *= 2;
  return (BH / 8) % g == 0 ? g : 0;
}

// All tensors bf16 or fp16 (T), layout [B, S, H, D] with token stride ld* (elements); LSE/Delta fp32 [B, Hq, S].
template <typename T>
hipError_t attn_fwd_t(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq,
                        int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal, int skv,
                        hipStream_t st) {
  if (S % 64 || (D != 64 && D != 128) || Hq % Hkv) return hipErrorInvalidValue;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 8) return hipErrorInvalidValue;
  constexpr int NW = 8;
  const int nqt = (S + 32 * NW - 1) / (32 * NW);
  dim3 grid(nqt * Hq * B), block(NW * 64);
  const float sl2 = scale * 1.4426950408889634f;
  const AttnOptions& op = g_attn_opts;
  const bool pipe = (causal || skv >= S) && (op.fwd_pipe >= 0 ? op.fwd_pipe != 0 : (causal != 0));
  const float thr = op.fwd_thr;
  const int grp = attn_grp(op.fwd_order, nqt, Hq * B, Hq / Hkv);
#define LAUNCH(DD, CC)                                                                                        \
  if (pipe)                                                                                                   \
    hipLaunchKernelGGL((fwd_p_kernel<T, DD, CC, NW>), grid, block, 0, st, (const T*)q, (const T*)k,         \
                       (const T*)v, (T*)o, lse, S, Hq, Hkv, ldq, ldk, ldv, ldo, sl2, thr, grp);             \
  else                                                                                                        \
    hipLaunchKernelGGL((fwd_kernel<T, DD, CC, NW>), grid, block, 0, st, (const T*)q, (const T*)k,           \
                       (const T*)v, (T*)o, lse, S, Hq, Hkv, ldq, ldk, ldv, ldo, sl2, skv)
  if (D == 128) { if (causal) LAUNCH(128, true); else LAUNCH(128, false); }
  else { if (causal) LAUNCH(64, true); else LAUNCH(64, false); }
#undef LAUNCH
  return hipGetLastError();
}

// dK/dV kernel choice. D = 64: 64 KB of LDS and <= 256 VGPRs, so two pipelined one-wave blocks share
// a CU and hide each other's prologue (B16 S2048 H16: 0.74 -> 0.68 ms bwd). At D = 128 the pipelined
// kernel wins only while the two-wave kernel's grid ((S/256) Hkv B blocks, one per CU) is at most one
// round of the chip's 256 CUs, where its causal work imbalance is exposed: S 8192 GQA 32/8 bwd B1
// 2.56 -> 1.98 ms with p2, but B4 7.30 (two-wave) vs 7.89 ms (p2) (profiles/attn_dkdv_select_r2.log).
static bool dkdv_use_p2(int B, int S, int Hq, int Hkv, int D) {
  const int impl = g_attn_opts.dkdv_impl;
  const long grid2 = (long)(S / 256) * Hkv * B;
  return impl == 1 || (impl < 0 && (D == 64 || ((long)(Hq / Hkv) * S >= 8192 && grid2 <= 256)));
}

// Window rule (dkdv_split / dkdv_kreg = -1): when the caller hands a mid_event, a side-stream job
// (the overlapped AdamW update, ops/sched.py) runs beside the dK/dV kernel, and a shorter kernel only
// pushes the rest of that job onto the GEMMs after it. In the step, the faster variants then lose:
// Llama-3-8B B1 S2048 109.1 ms split vs 108.3 unsplit (eager update: 109.7 vs 113.6), 7B B16
// 1058.0 KREG vs 1055.5 (profiles/r4/step_ab_*_split_sched.log, *_kreg.log). So both apply only
// when no job waits for the window (e.g. gradient-accumulation micro-steps, no overlapped update).
//
// GQA at small batch: the pipelined dK/dV grid is (S / 128) Hkv B blocks, one per CU at D = 128
// (Llama-3-8B B1 S2048 bwd 0.297 -> 0.206 (2 splits) -> 0.172 ms (4); S8192: 1.717 ms unsplit, the
// best: profiles/r4/attn_ab_dkdv_split_*.log)
// -- 128 blocks (half the chip) for Llama-3-8B B1 S2048 H32/8, and the causal work per block falls
// 16:1 from the first key block to the last. Splitting the kv head's query heads over n blocks gives
// n times the grid; with the heavy key blocks dispatched first, a CU that drew a light block picks
// up the next one, so two rounds of blocks even out to ~ (S/128 + 1) / 2 steps of work per CU. The
// price is an fp32 partial per split and one reduction pass (2 n B S Hkv D floats).
static int dkdv_split(int B, int S, int Hq, int Hkv, int D) {
  const int nrep = Hq / Hkv;
  int n = g_attn_opts.dkdv_split;
  if (n < 0) {
    const long grid = (long)(S / 128) * Hkv * B, want = D == 64 ? 1024 : 512;
    n = 1;
    while (grid * n < want && nrep % (2 * n) == 0) n *= 2;
  }
  return (n >= 1 && nrep % n == 0) ? n : 1;
}

// Fused backward (attention_bwd_fused.hip) applies at D = 128, S % 256 == 0 without key padding. By
// shape it runs when its grid -- one workgroup per (batch, kv head), each walking all S / 256 key
// blocks -- fills whole rounds of the chip (>= 90% of the slots of its last round busy): 7B-class MHA
// at batch >= 8. Its choice never depends on the AdamW window (mid_event), so overlapped and plain
// optimizer steps see the same gradients.
static int device_cus() {
  static int cus[64] = {0};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
  if (cus[d] == 0 && (hipDeviceGetAttribute(&cus[d], hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cus[d] <= 0))
    cus[d] = 256;
  return cus[d];
}
static bool fused_shape_ok(int S, int D) { return D == 128 && S % 256 == 0; }
static bool attn_bwd_use_fused(int B, int S, int Hq, int Hkv, int D, int skv) {
  const int mode = g_attn_opts.bwd_fused;
  if (mode == 0 || !fused_shape_ok(S, D) || skv != S) return false;
  if (mode == 1) return true;
  const long grid = (long)B * Hkv, cus = device_cus();
  const long rounds = (grid + cus - 1) / cus;
  return grid >= cus && grid * 10 >= rounds * cus * 9;
}

// fp32 workspace of pra_attn_bwd, in floats: delta, the row constants (-lse log2(e), -delta) of the
// pipelined dK/dV kernel and the fused kernel, the dK/dV split partials, or the fused kernel's dQ partials
long attn_bwd_ws_floats(int B, int S, int Hq, int Hkv, int D) {
  const long nrc = (long)B * Hq * S;
  const bool p2 = dkdv_use_p2(B, S, Hq, Hkv, D);
  const int n = p2 ? dkdv_split(B, S, Hq, Hkv, D) : 1;
  const long split = 3 * nrc + (n > 1 ? 2L * n * B * S * Hkv * D : 0);
  const long fused = g_attn_opts.bwd_fused != 0 && fused_shape_ok(S, D) ? 3 * nrc + nrc * D + 1024L * B * Hkv : 0;
  return split > fused ? split : fused;
}

template <typename T>
hipError_t attn_bwd_t(const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv,
                        int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk, long lddv,
                        float scale, int causal, int skv, const float* rope_tab, hipEvent_t mid_event,
                        hipStream_t st) {
  if (S % 128 || (D != 64 && D != 128) || Hq % Hkv) return hipErrorInvalidValue;
  const float2* rt = reinterpret_cast<const float2*>(rope_tab);
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 8 || lddo % 8 || lddq % 8 || lddk % 8 || lddv % 8)
    return hipErrorInvalidValue;
  if (attn_bwd_use_fused(B, S, Hq, Hkv, D, skv)) {
    // the window (mid_event) opens after the memory-bound row-constant pass, beside the fused kernel
    const long nrc = (long)B * Hq * S;
    return pra_attn_bwd_fused(std::is_same<T, __bf16>::value ? pra::kBF16 : pra::kF16, q, k, v, o, dout, lse,
                              delta + nrc, dq, dk, dv, B, S, Hq, Hkv, ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv,
                              scale, causal, rope_tab, mid_event, st);
  }
  const float sl2 = scale * 1.4426950408889634f;
  // 8-wave (256-row) blocks; S % 256 != 0 (S % 128 == 0) takes the 4-wave instantiations
  const int nw = S % 256 ? 4 : 8;
  // delta: fp32 workspace [3][B * Hq * S]: delta, then the pipelined dK/dV kernel's row constants
  // (-lse log2(e), -delta), written by the dQ kernel only when that kernel runs
  const long nrc = (long)B * Hq * S;
  const bool p2 = dkdv_use_p2(B, S, Hq, Hkv, D);
  const bool ring = (g_attn_opts.dkdv_kreg == 2 || (g_attn_opts.dkdv_kreg == -2 && mid_event == nullptr)) && !p2 &&
                    nw == 8 && D == 128;  // bwd_dkdv_r_kernel
  float* rc2 = (p2 || ring) ? delta + nrc : nullptr;
  // dQ first: it also computes delta = rowsum(dO * O), which the dK/dV kernel reads
  const bool win_early = window_before_dq(B, S);
  if (mid_event != nullptr && win_early) {
    const hipError_t e = hipEventRecord(mid_event, st);
    if (e != hipSuccess) return e;
  }
  {
    dim3 grid((S / (32 * nw)) * Hq * B);
    // the pipelined kernel has no key bound: padded non-causal sequences take the plain one
    const bool pipe = (causal || skv >= S) && g_attn_opts.dq_pipe != 0;
    const int gq = attn_grp(g_attn_opts.dq_order, S / (32 * nw), Hq * B, Hq / Hkv);
#define LAUNCH(DD, CC, NWW)                                                                                     \
  if (pipe)                                                                                                     \
    hipLaunchKernelGGL((bwd_dq_kernel<T, DD, CC, NWW, true>), grid, dim3(NWW * 64), 0, st, (const T*)q,       \
                       (const T*)k, (const T*)v, (const T*)dout, (const T*)o, lse, delta, (T*)dq, S, Hq, Hkv,  \
                       ldq, ldk, ldv, lddo, ldo, lddq, scale, sl2, skv, rt, rc2, nrc, gq);                          \
  else                                                                                                          \
    hipLaunchKernelGGL((bwd_dq_kernel<T, DD, CC, NWW>), grid, dim3(NWW * 64), 0, st, (const T*)q,             \
                       (const T*)k, (const T*)v, (const T*)dout, (const T*)o, lse, delta, (T*)dq, S, Hq, Hkv,  \
                       ldq, ldk, ldv, lddo, ldo, lddq, scale, sl2, skv, rt, rc2, nrc, gq)
    if (nw == 8) {
      if (D == 128) { if (causal) LAUNCH(128, true, 8); else LAUNCH(128, false, 8); }
      else { if (causal) LAUNCH(64, true, 8); else LAUNCH(64, false, 8); }
    } else {
      if (D == 128) { if (causal) LAUNCH(128, true, 4); else LAUNCH(128, false, 4); }
      else { if (causal) LAUNCH(64, true, 4); else LAUNCH(64, false, 4); }
    }
#undef LAUNCH
  }
  if (mid_event != nullptr && !win_early) {  // between dQ and dK/dV
    const hipError_t e = hipEventRecord(mid_event, st);
    if (e != hipSuccess) return e;
  }
  const bool window = mid_event != nullptr;
  if (p2) {
    const int ns = window && g_attn_opts.dkdv_split < 0 ? 1 : dkdv_split(B, S, Hq, Hkv, D);
    float* part = ns > 1 ? delta + 3 * nrc : nullptr;  // attn_bwd_ws_floats
    dim3 g1((S / 128) * Hkv * B * ns);
#define LAUNCH1(DD, CC)                                                                                       \
  hipLaunchKernelGGL((bwd_dkdv_p2_kernel<T, DD, CC>), g1, dim3(256), 0, st, (const T*)q, (const T*)k,        \
                     (const T*)v, (const T*)dout, rc2, rc2 + nrc, (T*)dk, (T*)dv, S, Hq, Hkv, ldq, ldk, ldv,   \
                     lddo, lddk, lddv, scale, sl2, skv, rt, ns, part)
    if (D == 128) { if (causal) LAUNCH1(128, true); else LAUNCH1(128, false); }
    else { if (causal) LAUNCH1(64, true); else LAUNCH1(64, false); }
#undef LAUNCH1
    if (ns > 1) {
      const long n = (long)B * S * Hkv * D;
      hipLaunchKernelGGL((dkdv_reduce_kernel<T>), dim3((unsigned)((2 * n / 4 + 255) / 256)), dim3(256), 0, st,
                         (const float*)part, ns, n, Hkv * D, (T*)dk, lddk, (T*)dv, lddv);
    }
  } else if (ring) {
    dim3 grid((S / 256) * Hkv * B);
#define LAUNCHR(DD, CC)                                                                                       \
  hipLaunchKernelGGL((bwd_dkdv_r_kernel<T, DD, CC>), grid, dim3(512), 0, st, (const T*)q, (const T*)k,        \
                     (const T*)v, (const T*)dout, rc2, nrc, (T*)dk, (T*)dv, S, Hq, Hkv, ldq, ldk, ldv, lddo,   \
                     lddk, lddv, scale, sl2, skv, rt, gk)
    const int gk = attn_grp(g_attn_opts.dkdv_order, S / 256, Hkv * B, 1);
    if (causal) LAUNCHR(128, true); else LAUNCHR(128, false);
#undef LAUNCHR
  } else {
    dim3 grid((S / (32 * nw)) * Hkv * B);
#define LAUNCH(DD, CC, NWW, ...)                                                                                \
  hipLaunchKernelGGL((bwd_dkdv_kernel<T, DD, CC, NWW, ##__VA_ARGS__>), grid, dim3(NWW * 64), 0, st, (const T*)q,   \
                     (const T*)k,                                                                               \
                     (const T*)v, (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Hq, Hkv, ldq, ldk, ldv, lddo,  \
                     lddk, lddv, scale, sl2, skv, rt, gk)
    const int gk = attn_grp(g_attn_opts.dkdv_order, S / (32 * nw), Hkv * B, 1);
    const bool kreg = g_attn_opts.dkdv_kreg == 1 || (g_attn_opts.dkdv_kreg < 0 && !window);
    if (nw == 8 && D == 128 && kreg) {
      if (causal) LAUNCH(128, true, 8, true); else LAUNCH(128, false, 8, true);
    } else if (nw == 8) {
      if (D == 128) { if (causal) LAUNCH(128, true, 8); else LAUNCH(128, false, 8); }
      else { if (causal) LAUNCH(64, true, 8); else LAUNCH(64, false, 8); }
    } else {
      if (D == 128) { if (causal) LAUNCH(128, true, 4); else LAUNCH(128, false, 4); }
      else { if (causal) LAUNCH(64, true, 4); else LAUNCH(64, false, 4); }
    }
#undef LAUNCH
  }
  return hipGetLastError();
}

}  // namespace

extern "C" {

hipError_t pra_attn_fwd(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int B, int S,
                        int Hq, int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal,
                        int skv, hipStream_t st) {
  if (skv <= 0 || skv > S) return hipErrorInvalidValue;
  if (dtype == pra::kF32)
    return pra_attn_fwd_f32((const float*)q, (const float*)k, (const float*)v, (float*)o, lse, B, S, Hq, Hkv, D, ldq,
                            ldk, ldv, ldo, scale, causal, skv, st);
  if (dtype == pra::kBF16)
    return attn_fwd_t<__bf16>(q, k, v, o, lse, B, S, Hq, Hkv, D, ldq, ldk, ldv, ldo, scale, causal, skv, st);
#if !PRA_ATTN_HARNESS
  if (dtype == pra::kF16)
    return attn_fwd_t<_Float16>(q, k, v, o, lse, B, S, Hq, Hkv, D, ldq, ldk, ldv, ldo, scale, causal, skv, st);
#endif
  return hipErrorInvalidValue;
}

hipError_t pra_attn_bwd(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv,
                        int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk, long lddv,
                        float scale, int causal, int skv, const float* rope_tab, hipEvent_t mid_event,
                        hipStream_t st) {
  if (skv <= 0 || skv > S) return hipErrorInvalidValue;
  if (dtype == pra::kF32) {
    if (rope_tab != nullptr) return hipErrorInvalidValue;  // the fp32 kernels have no fused inverse RoPE
    return pra_attn_bwd_f32((const float*)q, (const float*)k, (const float*)v, (const float*)o, (const float*)dout,
                            lse, delta, (float*)dq, (float*)dk, (float*)dv, B, S, Hq, Hkv, D, ldq, ldk, ldv, ldo, lddo,
                            lddq, lddk, lddv, scale, causal, skv, st);
  }
  if (dtype == pra::kBF16)
    return attn_bwd_t<__bf16>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, D, ldq, ldk, ldv, ldo, lddo,
                              lddq, lddk, lddv, scale, causal, skv, rope_tab, mid_event, st);
#if !PRA_ATTN_HARNESS
  if (dtype == pra::kF16)
    return attn_bwd_t<_Float16>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, D, ldq, ldk, ldv, ldo, lddo,
                                lddq, lddk, lddv, scale, causal, skv, rope_tab, mid_event, st);
#endif
  return hipErrorInvalidValue;
}

// Kernel selection (see AttnOptions); not thread-safe against concurrent launches (set between steps).
void pra_attn_set_options(int fwd_pipe, float fwd_thr, int dkdv_impl, int dq_pipe, int dkdv_split, int dkdv_kreg,
                          int bwd_fused, int bwd_window) {
  g_attn_opts.bwd_fused = bwd_fused;
  g_attn_opts.bwd_window = bwd_window;
  g_attn_opts.fwd_pipe = fwd_pipe;
  g_attn_opts.fwd_thr = fwd_thr;
  g_attn_opts.dkdv_impl = dkdv_impl;
  g_attn_opts.dq_pipe = dq_pipe;
  g_attn_opts.dkdv_split = dkdv_split;
  g_attn_opts.dkdv_kreg = dkdv_kreg;
}

void pra_attn_set_order(int fwd, int dq, int dkdv) {
  g_attn_opts.fwd_order = fwd;
  g_attn_opts.dq_order = dq;
  g_attn_opts.dkdv_order = dkdv;
}

long pra_attn_bwd_workspace(int dtype, int B, int S, int Hq, int Hkv, int D) {
  if (dtype == pra::kF32) return 3L * B * Hq * S;
  return attn_bwd_ws_floats(B, S, Hq, Hkv, D);
}

}  // extern "C"

// Standalone attention benchmark + checker (no torch): links one build of csrc/kernels/attention.hip
// (tools/attn_variants.sh builds one executable per -D variant) and times pra_attn_fwd / pra_attn_bwd
// on random bf16 data with hipEvents, then checks one (batch, kv-head) group against an fp64 CPU
// reference (O, LSE, dQ, dK, dV). Used to iterate on kernel schedules without rebuilding the torch
// extension; the same kernels are what pyrecover_amd._C runs.
//
//   attn_harness B S Hq Hkv D causal iters [check=1] [mode=both|fwd|bwd]
//
// Output: one line per measured pass, `fwd_ms=.. fwd_tf=.. bwd_ms=.. bwd_tf=.. max_err_*=..`.
// TFLOP/s: forward 4 B Hq S^2 D (x 1/2 causal); backward 2.5 x forward (the convention of README.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "kernels/common.h"
#include "kernels/launchers.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char** argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: %s B S Hq Hkv D causal iters [check] [mode]\n", argv[0]);
    return 1;
  }
  const int B = atoi(argv[1]), S = atoi(argv[2]), Hq = atoi(argv[3]), Hkv = atoi(argv[4]), D = atoi(argv[5]);
  const int causal = atoi(argv[6]), iters = atoi(argv[7]);
  const int check = argc > 8 ? atoi(argv[8]) : 1;
  const std::string mode = argc > 9 ? argv[9] : "both";
  const bool do_fwd = mode != "bwd", do_bwd = mode != "fwd";
  // fused QKV activation layout, as the model passes it: token stride (Hq + 2 Hkv) D
  const long ldqkv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const size_t nqkv = (size_t)B * S * ldqkv, no = (size_t)B * S * ldo;
  std::vector<uint16_t> h_qkv(nqkv), h_do(no);
  std::mt19937 rng(1234);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : h_qkv) x = f2bf(nd(rng));
  for (auto& x : h_do) x = f2bf(nd(rng));
  uint16_t *qkv, *o, *dout, *dq, *dk, *dv;
  float *lse, *ws;
  CK(hipMalloc(&qkv, nqkv * 2));
  CK(hipMalloc(&o, no * 2));
  CK(hipMalloc(&dout, no * 2));
  CK(hipMalloc(&dq, no * 2));
  CK(hipMalloc(&dk, (size_t)B * S * Hkv * D * 2));
  CK(hipMalloc(&dv, (size_t)B * S * Hkv * D * 2));
  CK(hipMalloc(&lse, (size_t)B * Hq * S * 4));
  // PRA_BWD_FUSED=0/1: split dQ + dK/dV kernels or the fused backward; PRA_FWD_PIPE=0/1: forward
  // kernel (fwd_kernel / pipelined fwd_p_kernel); unset = the defaults
  {
    const char* f = getenv("PRA_FWD_PIPE");
    const char* e = getenv("PRA_BWD_FUSED");
    if (f || e) pra_attn_set_options(f ? atoi(f) : -1, 8.f, -1, -1, 1, -2, e ? atoi(e) : 0, 0);
    // PRA_ATTN_ORDER="f,q,k": block order of the forward / dQ / dK/dV grids (pra_attn_set_order)
    int of = 0, oq = 0, ok = 0;
    if (const char* o = getenv("PRA_ATTN_ORDER")) sscanf(o, "%d,%d,%d", &of, &oq, &ok);
    pra_attn_set_order(of, oq, ok);
  }
  const long nws = pra_attn_bwd_workspace(pra::kBF16, B, S, Hq, Hkv, D);
  CK(hipMalloc(&ws, (size_t)nws * 4));
  CK(hipMemcpy(qkv, h_qkv.data(), nqkv * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, h_do.data(), no * 2, hipMemcpyHostToDevice));
  const uint16_t* q = qkv;
  const uint16_t* k = qkv + (long)Hq * D;
  const uint16_t* v = qkv + (long)(Hq + Hkv) * D;
  const float scale = 1.f / std::sqrt((float)D);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto fwd = [&] {
    CK(pra_attn_fwd(pra::kBF16, q, k, v, o, lse, B, S, Hq, Hkv, D, ldqkv, ldqkv, ldqkv, ldo, scale, causal, S, st));
  };
  auto bwd = [&] {
    CK(pra_attn_bwd(pra::kBF16, q, k, v, o, dout, lse, ws, dq, dk, dv, B, S, Hq, Hkv, D, ldqkv, ldqkv, ldqkv, ldo, ldo,
                    ldo, (long)Hkv * D, (long)Hkv * D, scale, causal, S, nullptr, nullptr, st));
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double ffl = 4.0 * B * Hq * (double)S * S * D * (causal ? 0.5 : 1.0);
  fwd();
  CK(hipStreamSynchronize(st));
  for (int pass = 0; pass < 3; ++pass) {
    double fms = 0, bms = 0;
    if (do_fwd) {
      for (int i = 0; i < 2; ++i) fwd();
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) fwd();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      fms = ms / iters;
    }
    if (do_bwd) {
      for (int i = 0; i < 2; ++i) bwd();
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) bwd();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      bms = ms / iters;
    }
    printf("pass=%d B=%d S=%d Hq=%d Hkv=%d D=%d causal=%d fwd_ms=%.4f fwd_tf=%.1f bwd_ms=%.4f bwd_tf=%.1f\n", pass, B,
           S, Hq, Hkv, D, causal, fms, fms > 0 ? ffl / fms / 1e9 : 0.0, bms, bms > 0 ? 2.5 * ffl / bms / 1e9 : 0.0);
    fflush(stdout);
  }
  if (!check) return 0;
  // reference for batch 0, kv head 0 and its query heads (fp64 on the CPU, bf16 inputs)
  fwd();
  bwd();
  CK(hipStreamSynchronize(st));
  std::vector<uint16_t> h_o(no), h_dq(no), h_dk((size_t)B * S * Hkv * D), h_dv((size_t)B * S * Hkv * D);
  std::vector<float> h_lse((size_t)B * Hq * S);
  CK(hipMemcpy(h_o.data(), o, no * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_dq.data(), dq, no * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_dk.data(), dk, h_dk.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_dv.data(), dv, h_dv.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_lse.data(), lse, h_lse.size() * 4, hipMemcpyDeviceToHost));
  const int rep = Hq / Hkv;
  auto at = [&](long tok, long col) { return (double)bf2f(h_qkv[tok * ldqkv + col]); };
  double eo = 0, el = 0, edq = 0, edk = 0, edv = 0, so = 0, sdq = 0, sdk = 0, sdv = 0;
  std::vector<double> dK((size_t)S * D, 0.0), dV((size_t)S * D, 0.0);
  std::vector<double> p(S), dp(S), oref(D), dqr(D);
  for (int hh = 0; hh < rep; ++hh) {
    const int hq = hh;  // kv head 0
    for (int i = 0; i < S; ++i) {
      const int kend = causal ? i + 1 : S;
      double m = -1e300;
      for (int j = 0; j < kend; ++j) {
        double s = 0;
        for (int d = 0; d < D; ++d) s += at(i, (long)hq * D + d) * at(j, (long)Hq * D + d);
        p[j] = s * scale;
        m = std::max(m, p[j]);
      }
      double l = 0;
      for (int j = 0; j < kend; ++j) l += (p[j] = std::exp(p[j] - m));
      for (int j = 0; j < kend; ++j) p[j] /= l;
      const double lse_ref = m + std::log(l);
      el = std::max(el, std::fabs(lse_ref - h_lse[(size_t)hq * S + i]));
      std::fill(oref.begin(), oref.end(), 0.0);
      for (int j = 0; j < kend; ++j)
        for (int d = 0; d < D; ++d) oref[d] += p[j] * at(j, (long)(Hq + Hkv) * D + d);
      // the backward consumes the kernel's bf16 O (delta = rowsum(dO * O)), as in training
      double delta = 0;
      for (int d = 0; d < D; ++d) {
        const double og = bf2f(h_o[(size_t)i * ldo + (long)hq * D + d]);
        eo = std::max(eo, std::fabs(oref[d] - og));
        so = std::max(so, std::fabs(oref[d]));
        delta += bf2f(h_do[(size_t)i * ldo + (long)hq * D + d]) * og;
      }
      std::fill(dqr.begin(), dqr.end(), 0.0);
      for (int j = 0; j < kend; ++j) {
        double s = 0;
        for (int d = 0; d < D; ++d) s += bf2f(h_do[(size_t)i * ldo + (long)hq * D + d]) * at(j, (long)(Hq + Hkv) * D + d);
        dp[j] = s;
        const double ds = p[j] * (dp[j] - delta);
        for (int d = 0; d < D; ++d) {
          dqr[d] += ds * at(j, (long)Hq * D + d) * scale;
          dK[(size_t)j * D + d] += ds * at(i, (long)hq * D + d) * scale;
          dV[(size_t)j * D + d] += p[j] * bf2f(h_do[(size_t)i * ldo + (long)hq * D + d]);
        }
      }
      for (int d = 0; d < D; ++d) {
        edq = std::max(edq, std::fabs(dqr[d] - bf2f(h_dq[(size_t)i * ldo + (long)hq * D + d])));
        sdq = std::max(sdq, std::fabs(dqr[d]));
      }
    }
  }
  for (int j = 0; j < S; ++j)
    for (int d = 0; d < D; ++d) {
      edk = std::max(edk, std::fabs(dK[(size_t)j * D + d] - bf2f(h_dk[(size_t)j * Hkv * D + d])));
      edv = std::max(edv, std::fabs(dV[(size_t)j * D + d] - bf2f(h_dv[(size_t)j * Hkv * D + d])));
      sdk = std::max(sdk, std::fabs(dK[(size_t)j * D + d]));
      sdv = std::max(sdv, std::fabs(dV[(size_t)j * D + d]));
    }
  const bool ok = eo <= 2e-2 * so && el <= 1e-2 && edq <= 3e-2 * sdq && edk <= 3e-2 * sdk && edv <= 3e-2 * sdv;
  printf("check %s: o %.3e/%.3e lse %.3e dq %.3e/%.3e dk %.3e/%.3e dv %.3e/%.3e\n", ok ? "OK" : "FAIL", eo, so, el,
         edq, sdq, edk, sdk, edv, sdv);
  return ok ? 0 : 3;
}

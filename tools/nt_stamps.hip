// Where does the NT GEMM's two-buffer main loop spend its cycles? Standalone diagnostic: builds
// csrc/kernels/gemm_nt.hip with PRA_NT_STAMPS (per-wave s_memtime sums per loop phase) or without
// (same driver, the production kernel), warms the chip for ~2 s of back-to-back launches (the GEMMs
// run at the power-limited clock), times 50 launches, and with stamps prints the per-chunk cycle
// split:
//   w1   lgkmcnt drain + barrier 1         p2  phase 2 (80 MFMA + 16 LDS-DMA of chunk t + 2)
//   w2   vmcnt(16) + barrier 2            p31 phase 3 + next chunk's phase 1 (48 MFMA + 32 LDS reads)
// Ideal at 16 cycles per 16x16x32 MFMA: p2 1280, p31 768, w1 = w2 = 0 -> 2048 cycles per chunk.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels [-DPRA_NT_STAMPS] tools/nt_stamps.hip -o nt
//   ./nt [M N K [warm_seconds]]
#include "../csrc/kernels/gemm_nt.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void fill_bf16(__bf16* p, long n, unsigned seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (__bf16)(((float)(h & 0xffff) / 32768.f - 1.f));
  }
}

// C[m][n] of sampled (m, n) pairs by a plain dot product (fp32), for a correctness check of the variant
__global__ void sample_ref(const __bf16* A, const __bf16* B, const __bf16* C, int M, int N, int K, float* err) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  const unsigned h = (unsigned)s * 2654435761u;
  const int m = (int)(h % (unsigned)M), n = (int)((h >> 7) % (unsigned)N);
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc += (float)A[(long)m * K + k] * (float)B[(long)n * K + k];
  err[s] = fabsf((float)C[(long)m * N + n] - acc) / fmaxf(1.f, fabsf(acc));
}

// cycles between two back-to-back stamps (the cost of one stamp)
__global__ void stamp_cost(unsigned long long* o) {
  unsigned long long a = __builtin_amdgcn_s_memtime();
  unsigned long long b = __builtin_amdgcn_s_memtime();
  unsigned long long c = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { o[0] = b - a; o[1] = c - b; }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 32768, N = argc > 2 ? atoi(argv[2]) : 4096;
  const int K = argc > 3 ? atoi(argv[3]) : 4096;
  const double warm = argc > 4 ? atof(argv[4]) : 2.0;
  const int epi = argc > 5 ? atoi(argv[5]) : 0;  // 0 plain, 1 SwiGLU (C = gu [M][N], a [M][N/2]),
                                                   // 2 SwiGLU backward (C = gu [M][2N] read and overwritten)
  const int cus = 256;
  __bf16 *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2 * (epi == 2 ? 2 : 1)));
  if (epi == 2) hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, C, 2L * M * N, 3u);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, A, (long)M * K, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, B, (long)N * K, 2u);
  const long wsf = pra_gemm_nt_ws_floats(M, N, K, cus);
  const int nt = pra_gemm_nt_ticket_count(M, N, K, cus);
  float* ws = nullptr;
  int* tk = nullptr;
  if (wsf) CK(hipMalloc(&ws, wsf * 4));
  if (nt) CK(hipMalloc(&tk, nt * 4));
  const int nwg = (M / 256) * (N / 256);
  const long nst = 2L * nwg * 4 * 8;
  unsigned long long* st = nullptr;
  CK(hipMalloc(&st, nst * 8));
  CK(hipMemset(st, 0, nst * 8));
#ifdef PRA_NT_STAMPS
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pra::nt::pra_nt_stamp_out), &st, sizeof(st)));
  {
    hipLaunchKernelGGL(stamp_cost, dim3(1), dim3(64), 0, 0, st);
    unsigned long long h[2];
    CK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
    printf("stamp cost: %llu %llu cycles\n", h[0], h[1]);
    CK(hipMemset(st, 0, nst * 8));
  }
#endif
  __bf16* C2 = nullptr;
  if (epi == 1) CK(hipMalloc(&C2, (size_t)M * (N / 2) * 2));
  auto launch = [&]() {
    if (epi == 2)  // C is gu [M][2N], dg / du written over g / u launch after launch: timing only (the math is
                   // checked by tests/test_gemm_nt_gpu.py)
      return pra_gemm_nt(pra::kBF16, 2, A, B, C, M, N, K, K, K, 2L * N, nullptr, 0, N, nullptr, 0, 0, 0, ws, tk, cus, 0);
    return pra_gemm_nt(pra::kBF16, epi, A, B, C, M, N, K, K, K, N, C2, N / 2, N / 2, nullptr, 0, 0, 0, ws, tk, cus, 0);
  };
  CK(launch());
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  int nwarm = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < warm) {
    for (int i = 0; i < 20; ++i) CK(launch());
    CK(hipDeviceSynchronize());
    nwarm += 20;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 50;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12;
#ifdef PRA_NT_STAMPS
  const char* kind = "stamps";
#else
  const char* kind = "plain";
#endif
  float* err;
  CK(hipMalloc(&err, 4096 * 4));
  if (epi == 0) hipLaunchKernelGGL(sample_ref, dim3(64), dim3(64), 0, 0, A, B, C, M, N, K, err);
  else CK(hipMemset(err, 0, 4096 * 4));  // (the SwiGLU epilogue is checked by tests/test_gemm_nt_gpu.py)
  std::vector<float> he(4096);
  CK(hipMemcpy(he.data(), err, 4096 * 4, hipMemcpyDeviceToHost));
  const float maxerr = *std::max_element(he.begin(), he.end());
  printf("{\"kind\": \"%s\", \"epi\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"warm_launches\": %d, \"ms\": %.4f, "
         "\"tflops\": %.1f, \"max_rel_err_4096_samples\": %.5f}\n", kind, epi, M, N, K, nwarm, ms, tf, maxerr);
  if (!(maxerr < 0.02f)) {
    fprintf(stderr, "WRONG RESULT\n");
    return 2;
  }
#ifdef PRA_NT_STAMPS
  std::vector<unsigned long long> h(nst);
  CK(hipMemcpy(h.data(), st, nst * 8, hipMemcpyDeviceToHost));
  double s[4] = {0, 0, 0, 0}, n = 0;
  std::vector<double> wait_per_chunk, p2_per_chunk;
  for (long w = 0; w < nst / 8; ++w) {
    const unsigned long long* o = &h[w * 8];
    if (o[4] < 2) continue;
    for (int j = 0; j < 4; ++j) s[j] += (double)o[j];
    n += (double)o[4];
    wait_per_chunk.push_back((double)(o[0] + o[2]) / o[4]);
    p2_per_chunk.push_back((double)o[1] / o[4]);
  }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)(q * (v.size() - 1))];
  };
  // p31 has one sample fewer per wave than the others (no predecessor for the first chunk)
  printf("waves %zu chunks %.0f | per chunk: w1 %.0f p2 %.0f w2 %.0f p31 %.0f cycles\n", wait_per_chunk.size(), n,
         s[0] / n, s[1] / n, s[2] / n, s[3] / (n - wait_per_chunk.size()));
  {  // per tile: prologue (DMA issue to chunk 0 landed), main loop, epilogue (stores issued and left)
    double pro = 0, loop = 0, epi = 0, nt = 0;
    for (long w = 0; w < nst / 8; ++w) {
      const unsigned long long* o = &h[w * 8];
      if (o[4] < 2) continue;
      pro += (double)o[6]; loop += (double)o[5]; epi += (double)o[7]; nt += 1;
    }
    printf("per tile: prologue %.0f main loop %.0f epilogue %.0f cycles\n", pro / nt, loop / nt, epi / nt);
  }
  printf("w1+w2 per chunk p10/p50/p90: %.0f %.0f %.0f | p2 p10/p50/p90: %.0f %.0f %.0f\n", pct(wait_per_chunk, 0.1),
         pct(wait_per_chunk, 0.5), pct(wait_per_chunk, 0.9), pct(p2_per_chunk, 0.1), pct(p2_per_chunk, 0.5),
         pct(p2_per_chunk, 0.9));
#endif
  return 0;
}

// Standalone timing of the MFMA weight-gradient GEMM (csrc/kernels/gemm_wgrad.hip), for A/B of
// compile-time schedule variants (-DPRA_WG_M0SPLIT=0/1): ~2 s of back-to-back launches on random
// data (the GEMMs run at the power-limited clock), then 20 timed launches and a sampled fp32 check.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels [-DPRA_WG_M0SPLIT=1] tools/wgrad_variants.hip -o wg
//   ./wg [M N K [warm_seconds]]      C[M][N] = A^T B, A [K][M], B [K][N]
#include "../csrc/kernels/gemm_wgrad.hip"

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

__global__ void sample_ref(const __bf16* A, const __bf16* B, const __bf16* C, int M, int N, int K, float* err) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  const unsigned h = (unsigned)s * 2654435761u;
  const int m = (int)(h % (unsigned)M), n = (int)((h >> 7) % (unsigned)N);
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc += (float)A[(long)k * M + m] * (float)B[(long)k * N + n];
  err[s] = fabsf((float)C[(long)m * N + n] - acc) / fmaxf(1.f, fabsf(acc));
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096;
  const int K = argc > 3 ? atoi(argv[3]) : 32768;
  const double warm = argc > 4 ? atof(argv[4]) : 2.0;
  const int cus = 256;
  __bf16 *A, *B, *C;
  CK(hipMalloc(&A, (size_t)K * M * 2));
  CK(hipMalloc(&B, (size_t)K * N * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, A, (long)K * M, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, B, (long)K * N, 2u);
  const long wsf = pra_wgrad_ws_floats(M, N, K, cus);
  const int nt = pra_wgrad_ticket_count(M, N, K, cus);
  float* ws = nullptr;
  int* tk = nullptr;
  if (wsf) CK(hipMalloc(&ws, wsf * 4));
  if (nt) CK(hipMalloc(&tk, nt * 4));
  auto launch = [&]() { return pra_wgrad_gemm(pra::kBF16, A, B, C, M, N, K, M, N, N, 0, ws, tk, cus, 0); };
  CK(launch());
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  int nwarm = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < warm) {
    for (int i = 0; i < 10; ++i) CK(launch());
    CK(hipDeviceSynchronize());
    nwarm += 10;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  float* err;
  CK(hipMalloc(&err, 4096 * 4));
  hipLaunchKernelGGL(sample_ref, dim3(64), dim3(64), 0, 0, A, B, C, M, N, K, err);
  std::vector<float> he(4096);
  CK(hipMemcpy(he.data(), err, 4096 * 4, hipMemcpyDeviceToHost));
  const float maxerr = *std::max_element(he.begin(), he.end());
  printf("{\"m0split\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"warm_launches\": %d, \"ms\": %.4f, \"tflops\": %.1f, "
         "\"max_rel_err_4096_samples\": %.5f}\n", PRA_WG_M0SPLIT, M, N, K, nwarm, ms, 2.0 * M * N * K / (ms * 1e-3) / 1e12,
         maxerr);
  return maxerr < 0.02f ? 0 : 2;
}

// Reduction kernel of the intra-node xGMI all-reduce (csrc/dist/xgmi.cpp, pyrecover_amd/parallel/
// xgmi.py): dst = src_0 + src_1 + ... + src_{W-1}, summed in fp32 in rank order and rounded
// once, so every rank reduces its slice identically (bit-reproducible, unlike a ring that rounds
// at every hop). The sources are this rank's own slice and the peers' slices already copied into
// local staging by the copy engines.
#include "common.h"

namespace pra {

struct SrcList {
  const void* p[16];
};

template <typename T>
__global__ __launch_bounds__(256) void sum_slices_kernel(SrcList src, int nsrc, T* __restrict__ dst, long n) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float acc[8], v[8];
    load8<T>(reinterpret_cast<const T*>(src.p[0]) + i * 8, acc);
    for (int r = 1; r < nsrc; ++r) {
      load8<T>(reinterpret_cast<const T*>(src.p[r]) + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    store8<T>(dst + i * 8, acc);
  }
  for (long i = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float acc = to_f<T>(reinterpret_cast<const T*>(src.p[0])[i]);
    for (int r = 1; r < nsrc; ++r) acc += to_f<T>(reinterpret_cast<const T*>(src.p[r])[i]);
    dst[i] = from_f<T>(acc);
  }
}

}  // namespace pra

extern "C" hipError_t pra_sum_slices(int dtype, const void* const* srcs, int nsrc, void* dst, long n, hipStream_t s) {
  if (nsrc < 1 || nsrc > 16) return hipErrorInvalidValue;
  for (int r = 0; r < nsrc; ++r)
    if (reinterpret_cast<uintptr_t>(srcs[r]) % 16) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(dst) % 16) return hipErrorInvalidValue;
  pra::SrcList l{};
  for (int r = 0; r < nsrc; ++r) l.p[r] = srcs[r];
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::sum_slices_kernel<T>), dim3(blocks), dim3(256), 0, s, l, nsrc, (T*)dst,
                                        n));
  return hipGetLastError();
}

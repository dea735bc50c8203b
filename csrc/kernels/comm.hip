// Reduction kernel of the intra-node xGMI all-reduce (csrc/dist/xgmi.cpp, pyrecover_amd/parallel/
// xgmi.py): dst = src_0 + src_1 + ... + src_{W-1}, summed in fp32 in rank order and rounded
// once, so every rank reduces its slice identically (bit-reproducible, unlike a ring that rounds
// at every hop). The sources are this rank's own slice and the peers' slices, read straight from
// their IPC-mapped gradient buffers over xGMI (the pull reduce-scatter of XgmiEngine), or copies of
// them in local staging (the copy-engine path).
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

// Device-to-device copy for the checkpoint snapshot's HBM hop (csrc/runtime/ckpt_engine.h): 16 B
// per lane, 4 in flight per thread, grid-stride. hipMemcpyAsync D2D on this stack ran the 38-GiB
// snapshot of the 7B state far below HBM bandwidth (the step after an async save took 0.71 s
// instead of 0.17 s); this copy is bandwidth-bound and, launched on the engine's low-priority
// stream, shares the CUs with the training step instead of blocking its next update.
namespace pra {
__global__ __launch_bounds__(256) void copy16_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, long n16) {
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void copy1_kernel(unsigned char* __restrict__ dst, const unsigned char* __restrict__ src,
                                                    long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
}  // namespace pra

extern "C" hipError_t pra_copy_d2d(void* dst, const void* src, long nbytes, hipStream_t s) {
  if (nbytes <= 0) return hipSuccess;
  const bool al = reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0;
  // a misaligned region would otherwise go through the 1-byte kernel whole: the runtime's copy
  // engine path is faster there (checkpoint regions are 64-B aligned, so this is a fallback)
  if (!al && nbytes > 4096) return hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, s);
  const long n16 = al ? nbytes / 16 : 0;
  if (n16 > 0) {
    long blocks = (n16 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(pra::copy16_kernel, dim3(blocks), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n16);
  }
  const long tail = nbytes - n16 * 16;
  if (tail > 0)
    hipLaunchKernelGGL(pra::copy1_kernel, dim3((tail + 255) / 256), dim3(256), 0, s,
                       (unsigned char*)dst + n16 * 16, (const unsigned char*)src + n16 * 16, tail);
  return hipGetLastError();
}

// All-gather phase of the pull all-reduce (csrc/dist/xgmi.cpp XgmiEngine): every peer's reduced
// slice is pulled from its IPC-mapped buffer into this rank's buffer in ONE kernel, the W - 1 source
// GPUs spread over blockIdx.y, so the pulls from all peers (all xGMI links) run at once. Slices are
// 16-B aligned (8-element cuts); a tail of n % 16 bytes is copied bytewise by the last block row.
namespace pra {
struct CopyList {
  const void* src[16];
  void* dst[16];
  long nbytes[16];
};
__global__ __launch_bounds__(256) void pull_gather_kernel(CopyList l) {
  const int k = blockIdx.y;
  const long n16 = l.nbytes[k] / 16;
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(l.src[k]);
  uint4* __restrict__ dst = reinterpret_cast<uint4*>(l.dst[k]);
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
  const long tail = l.nbytes[k] - n16 * 16;
  if (blockIdx.x == 0 && threadIdx.x < tail)
    reinterpret_cast<unsigned char*>(l.dst[k])[n16 * 16 + threadIdx.x] =
        reinterpret_cast<const unsigned char*>(l.src[k])[n16 * 16 + threadIdx.x];
}
}  // namespace pra

extern "C" hipError_t pra_pull_gather(const void* const* srcs, void* const* dsts, const long* nbytes, int n,
                                      hipStream_t s) {
  if (n < 0 || n > 16) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  pra::CopyList l{};
  long mx = 0;
  for (int k = 0; k < n; ++k) {
    if (reinterpret_cast<uintptr_t>(srcs[k]) % 16 || reinterpret_cast<uintptr_t>(dsts[k]) % 16) return hipErrorInvalidValue;
    l.src[k] = srcs[k];
    l.dst[k] = dsts[k];
    l.nbytes[k] = nbytes[k];
    mx = nbytes[k] > mx ? nbytes[k] : mx;
  }
  long bx = (mx / 16 + 1023) / 1024;  // ~4 x 16 B per thread per pass
  if (bx > 512) bx = 512;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(pra::pull_gather_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, s, l);
  return hipGetLastError();
}

// Replica checksum (pyrecover_amd/parallel/consistency.py): a 64-bit position-weighted hash of a
// buffer's 32-bit words, h = sum_i w_i (2 i + 1) mod 2^64, and the fp64 sum of its elements. Two
// replicas of a parameter / moment buffer agree on both only if they are (almost surely) bitwise
// equal; the hash changes when any word changes or two words swap. Two passes (per-block partials,
// then one ordered sum): integer results are exact in any order and the fp64 sum is reproducible
// on identical data, with no atomics.
namespace pra {
template <typename T>
__global__ __launch_bounds__(256) void checksum_kernel(const uint4* __restrict__ x, long n16, double* __restrict__ psum,
                                                       unsigned long long* __restrict__ phash) {
  constexpr int E = 16 / sizeof(T);  // elements per 16-B vector
  double s = 0.0;
  unsigned long long h = 0ull;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
    const uint4 v = x[i];
    const unsigned long long w0 = 4ull * (unsigned long long)i;
    h += (unsigned long long)v.x * (2ull * w0 + 1ull) + (unsigned long long)v.y * (2ull * w0 + 3ull) +
         (unsigned long long)v.z * (2ull * w0 + 5ull) + (unsigned long long)v.w * (2ull * w0 + 7ull);
    const T* e = reinterpret_cast<const T*>(&v);
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < E; ++j) part += to_f<T>(e[j]);
    s += (double)part;
  }
  __shared__ double ss[256];
  __shared__ unsigned long long hh[256];
  ss[threadIdx.x] = s;
  hh[threadIdx.x] = h;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      ss[threadIdx.x] += ss[threadIdx.x + o];
      hh[threadIdx.x] += hh[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    psum[blockIdx.x] = ss[0];
    phash[blockIdx.x] = hh[0];
  }
}
__global__ __launch_bounds__(64) void checksum_final_kernel(const double* __restrict__ psum,
                                                            const unsigned long long* __restrict__ phash, int nb,
                                                            double* __restrict__ out_sum,
                                                            unsigned long long* __restrict__ out_hash) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  unsigned long long h = 0ull;
  for (int i = 0; i < nb; ++i) {
    s += psum[i];
    h += phash[i];
  }
  out_sum[0] = s;
  out_hash[0] = h;
}
}  // namespace pra

extern "C" int pra_checksum_blocks() { return 1024; }

// ws: pra_checksum_blocks() doubles + as many u64; nbytes % 16 == 0, 16-B aligned
extern "C" hipError_t pra_checksum(int dtype, const void* x, long nbytes, double* ws_sum, unsigned long long* ws_hash,
                                   double* out_sum, unsigned long long* out_hash, hipStream_t s) {
  if (nbytes % 16 || reinterpret_cast<uintptr_t>(x) % 16) return hipErrorInvalidValue;
  const int nb = pra_checksum_blocks();
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::checksum_kernel<T>), dim3(nb), dim3(256), 0, s, (const uint4*)x,
                                        nbytes / 16, ws_sum, ws_hash));
  hipLaunchKernelGGL(pra::checksum_final_kernel, dim3(1), dim3(64), 0, s, ws_sum, ws_hash, nb, out_sum, out_hash);
  return hipGetLastError();
}

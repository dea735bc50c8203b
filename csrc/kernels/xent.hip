// Fused causal-LM cross-entropy over bf16/fp16/fp32 logits (reference train.py:263-266:
// `cross_entropy(logits.float(), labels, reduction="sum") / labels.ne(-100).sum()`).
//
// Forward: one 256-thread block per row, a single streaming pass with an online
// (max, sum-exp) pair per lane -> per-row log-sum-exp and loss, no fp32 copy of the logits.
// A single-block kernel then sums the row losses in a fixed order and divides by the
// number of non-ignored labels, all on device (no host sync for `n_items`).
// Backward: d logits = (softmax - onehot) * grad_out / n_items, written IN PLACE over the
// logits (they are dead after the backward), so the [T, V] activation is never duplicated.
#include "common.h"

namespace pra {

template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ lse_out, float* __restrict__ loss_row,
                                                       long V, long ld, long ignore_index) {
  __shared__ float sm[4], ss[4];
  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  const int tid = threadIdx.x;
  float m = -INFINITY, s = 0.f;
  const long V8 = (V / 8) * 8;
  for (long c = (long)tid * 8; c < V8; c += 2048) {
    float v[8];
    load8<T>(x + c, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    const float nm = fmaxf(m, lm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(v[j] - nm);
    s = s * __expf(m - nm) + acc;
    m = nm;
  }
  for (long c = V8 + tid; c < V; c += 256) {  // tail (V not a multiple of 8)
    const float v = to_f<T>(x[c]);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  // combine (m, s) across the wave then the block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if ((tid & 63) == 0) { sm[tid >> 6] = m; ss[tid >> 6] = s; }
  __syncthreads();
  if (tid == 0) {
    float M = sm[0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < 4; ++i) S += (sm[i] == -INFINITY ? 0.f : ss[i] * __expf(sm[i] - M));
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const long lab = labels[row];
    loss_row[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - to_f<T>(x[lab]);
  }
}

// out[0] = sum(loss_row) / n_valid ; out[1] = n_valid (as float). One block, fixed order.
__global__ __launch_bounds__(256) void xent_reduce_kernel(const float* __restrict__ loss_row,
                                                          const int64_t* __restrict__ labels, float* __restrict__ out,
                                                          long T, long ignore_index) {
  __shared__ float red[4];
  float s = 0.f, n = 0.f;
  for (long i = threadIdx.x; i < T; i += 256) {
    s += loss_row[i];
    n += (labels[i] != ignore_index) ? 1.f : 0.f;
  }
  s = block_sum<4>(s, red);
  n = block_sum<4>(n, red);
  if (threadIdx.x == 0) {
    out[0] = s / n;
    out[1] = n;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ stats,
                                                       const float* __restrict__ grad_out, long V, long ld,
                                                       long ignore_index) {
  const long row = blockIdx.x;
  T* x = logits + row * ld;
  const long lab = labels[row];
  const bool ign = (lab == ignore_index);
  const float scale = ign ? 0.f : grad_out[0] / stats[1];
  const float l = lse[row];
  const long V8 = (V / 8) * 8;
  for (long c = (long)threadIdx.x * 8; c < V8; c += 2048) {
    float v[8];
    load8<T>(x + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__expf(v[j] - l) - ((c + j) == lab ? 1.f : 0.f)) * scale;
    store8<T>(x + c, v);
  }
  for (long c = V8 + threadIdx.x; c < V; c += 256) {
    const float v = to_f<T>(x[c]);
    x[c] = from_f<T>((__expf(v - l) - (c == lab ? 1.f : 0.f)) * scale);
  }
}

}  // namespace pra

extern "C" {

// stats: float[2] device buffer -> {mean loss, n_valid}
hipError_t pra_xent_fwd(int dtype, const void* logits, const int64_t* labels, float* lse, float* loss_row,
                        float* stats, long T, long V, long ld, long ignore_index, hipStream_t s) {
  if (ld % 8) return hipErrorInvalidValue;
  PRA_DISPATCH_FLOAT(dtype, LT,
                     hipLaunchKernelGGL((pra::xent_fwd_kernel<LT>), dim3(T), dim3(256), 0, s, (const LT*)logits,
                                        labels, lse, loss_row, V, ld, ignore_index));
  hipLaunchKernelGGL(pra::xent_reduce_kernel, dim3(1), dim3(256), 0, s, loss_row, labels, stats, T, ignore_index);
  return hipGetLastError();
}

hipError_t pra_xent_bwd(int dtype, void* logits, const int64_t* labels, const float* lse, const float* stats,
                        const float* grad_out, long T, long V, long ld, long ignore_index, hipStream_t s) {
  if (ld % 8) return hipErrorInvalidValue;
  PRA_DISPATCH_FLOAT(dtype, LT,
                     hipLaunchKernelGGL((pra::xent_bwd_kernel<LT>), dim3(T), dim3(256), 0, s, (LT*)logits, labels,
                                        lse, stats, grad_out, V, ld, ignore_index));
  return hipGetLastError();
}

}  // extern "C"

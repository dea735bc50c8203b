// Flat-buffer AdamW and gradient-norm kernels.
//
// The engine keeps every trainable parameter, its gradient and both Adam moments in four
// flat, identically-ordered device buffers, so the optimizer step is ONE streaming kernel
// over N elements (14 B/elem for bf16 p/g/m/v: read 8, write 6) instead of a multi-tensor
// launch list. Math follows torch's fused AdamW (`_fused_adamw_`, used by the reference's
// `--fused-optimizer`, train.py:120-122): fp32 opmath, one rounding per stored value.
//
//   p  = p * (1 - lr*wd)
//   m  = lerp(m, g, 1-b1)            v = b2*v + (1-b2)*g*g
//   p  = p - (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
//
// `gscale` pre-multiplies the gradient (1/world_size after a SUM all-reduce, and/or a
// clip coefficient read from device memory when `gscale_dev` is non-null). `hyper_dev`, when
// non-null, supplies {lr, bc1, bc2_sqrt} from device memory so a captured HIP graph of the
// training step replays with the current learning rate and bias corrections.
#include "common.h"

namespace pra {

template <typename P, typename S>
__global__ __launch_bounds__(256) void adamw_kernel(P* __restrict__ p, const P* __restrict__ g, S* __restrict__ m,
                                                    S* __restrict__ v, long n, float lr, float b1, float b2,
                                                    float eps, float wd, float bc1, float bc2_sqrt, float gscale,
                                                    const float* __restrict__ gscale_dev,
                                                    const float* __restrict__ hyper_dev) {
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  if (hyper_dev) {  // step-dependent scalars from device memory (graph-captured step)
    lr = hyper_dev[0];
    bc1 = hyper_dev[1];
    bc2_sqrt = hyper_dev[2];
  }
  const float decay = 1.f - lr * wd;
  const float step_size = lr / bc1;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long o = i * 8;
    float pv[8], gv[8], mv[8], vv[8];
    load8<P>(p + o, pv);
    load8<P>(g + o, gv);
    load8<S>(m + o, mv);
    load8<S>(v + o, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gr = gv[j] * gs;
      pv[j] *= decay;
      mv[j] = mv[j] + (1.f - b1) * (gr - mv[j]);
      vv[j] = b2 * vv[j] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(vv[j]) / bc2_sqrt + eps;
      pv[j] = pv[j] - step_size * mv[j] / denom;
    }
    store8<P>(p + o, pv);
    store8<S>(m + o, mv);
    store8<S>(v + o, vv);
  }
  // tail
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    float pv = to_f<P>(p[o]), gr = to_f<P>(g[o]) * gs, mv = to_f<S>(m[o]), vv = to_f<S>(v[o]);
    pv *= decay;
    mv = mv + (1.f - b1) * (gr - mv);
    vv = b2 * vv + (1.f - b2) * gr * gr;
    pv = pv - step_size * mv / (sqrtf(vv) / bc2_sqrt + eps);
    p[o] = from_f<P>(pv);
    m[o] = from_f<S>(mv);
    v[o] = from_f<S>(vv);
  }
}

// Sum of squares of a flat buffer -> fp32 partials[gridDim.x]; then a 1-block fixed-order
// finish computes total norm and clip coefficient min(1, max_norm/(norm+1e-6)).
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, long n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    load8<T>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    const float v = to_f<T>(x[o]);
    s += v * v;
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void norm_finish_kernel(const float* __restrict__ partial, int np, float* __restrict__ out,
                                                          float max_norm, float pre_scale) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) s += partial[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * pre_scale;
    out[0] = norm;
    out[1] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
  }
}

}  // namespace pra

extern "C" {

// pdtype: param/grad dtype; sdtype: moment dtype
hipError_t pra_adamw_flat(int pdtype, int sdtype, void* p, const void* g, void* m, void* v, long n, float lr,
                          float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float gscale,
                          const float* gscale_dev, const float* hyper_dev, hipStream_t s) {
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (pdtype != sdtype) return hipErrorInvalidValue;
  PRA_DISPATCH_FLOAT(pdtype, T,
                     hipLaunchKernelGGL((pra::adamw_kernel<T, T>), dim3(blocks), dim3(256), 0, s, (T*)p, (const T*)g,
                                        (T*)m, (T*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale, gscale_dev,
                                        hyper_dev));
  return hipGetLastError();
}

int pra_sumsq_partials() { return 1024; }

// out: float[2] = {norm, clip_coef}; ws: float[pra_sumsq_partials()]
hipError_t pra_grad_norm(int dtype, const void* x, long n, float* ws, float* out, float max_norm, float pre_scale,
                         hipStream_t s) {
  const int np = 1024;
  PRA_DISPATCH_FLOAT(dtype, T,
                     hipLaunchKernelGGL((pra::sumsq_kernel<T>), dim3(np), dim3(256), 0, s, (const T*)x, n, ws));
  hipLaunchKernelGGL(pra::norm_finish_kernel, dim3(1), dim3(256), 0, s, ws, np, out, max_norm, pre_scale);
  return hipGetLastError();
}

}  // extern "C"

// Flat-buffer AdamW and gradient-norm kernels.
//
// The engine keeps every trainable parameter, its gradient and both Adam moments in four
// flat, identically-ordered device buffers, so the optimizer step is ONE streaming kernel
// over N elements (14 B/elem for bf16 p/g/m/v: read 8, write 6) instead of a multi-tensor
// launch list. Math follows torch's fused AdamW (`_fused_adamw_`, used by the reference's
// `--fused-optimizer`, train.py:120-122): fp32 opmath, one rounding per stored value; the default
// FAST instantiation takes the two divisions and the square root from the hardware (1 ulp) instead
// of torch's correctly rounded sequences (see adamw_elem).
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

// One AdamW element update with every fused multiply-add written out, so all kernels that use it
// (flat, tiled + transposed) round identically whatever the compiler's contraction choices.
// FAST: the two divisions and the square root on the hardware v_rcp_f32 / v_sqrt_f32 (1 ulp each)
// instead of the correctly rounded IEEE sequences (~10 VALU per division): ~17 instead of ~60 VALU
// per element, which matters because the update runs beside the attention backward on a side
// stream. m and v are computed exactly as before; p's update term differs by at most a few fp32
// ulps before its bf16 rounding. !FAST keeps torch _fused_adamw_'s correctly rounded divisions.
template <bool FAST>
__device__ __forceinline__ void adamw_elem(float& p, float& m, float& v, float g, float gs, float decay, float b1,
                                           float b2, float eps, float bc2_sqrt, float step_size) {
  const float gr = g * gs;
  p *= decay;
  m = fmaf(1.f - b1, gr - m, m);
  v = fmaf(b2, v, (1.f - b2) * (gr * gr));
  if constexpr (FAST) {
    const float denom = fmaf(__builtin_amdgcn_sqrtf(v), __builtin_amdgcn_rcpf(bc2_sqrt), eps);
    p = fmaf(-step_size, m * __builtin_amdgcn_rcpf(denom), p);
  } else {
    const float denom = __fdiv_rn(sqrtf(v), bc2_sqrt) + eps;
    p = fmaf(-step_size, __fdiv_rn(m, denom), p);
  }
}

template <typename P, typename S, bool FAST>
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
    for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[j], mv[j], vv[j], gv[j], gs, decay, b1, b2, eps, bc2_sqrt, step_size);
    store8<P>(p + o, pv);
    store8<S>(m + o, mv);
    store8<S>(v + o, vv);
  }
  // tail
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    float pv = to_f<P>(p[o]), mv = to_f<S>(m[o]), vv = to_f<S>(v[o]);
    adamw_elem<FAST>(pv, mv, vv, to_f<P>(g[o]), gs, decay, b1, b2, eps, bc2_sqrt, step_size);
    p[o] = from_f<P>(pv);
    m[o] = from_f<S>(mv);
    v[o] = from_f<S>(vv);
  }
}

// AdamW over one row-major [rows, cols] weight matrix that ALSO writes its transposed copy
// pt [cols, rows] (the data-gradient GEMM's operand, parallel/flat.py "weight shadows") from the
// updated values it already holds: the separate transpose pass re-read the whole model after
// every update (13.5 GB/step at 7B). Block = one 64 x 64 tile; the updated p tile goes through
// LDS (padded rows) to 16-B transposed stores. Same math and rounding as adamw_kernel.
template <typename P, bool FAST>
__global__ __launch_bounds__(256) void adamw_t_kernel(P* __restrict__ p, const P* __restrict__ g, P* __restrict__ m,
                                                      P* __restrict__ v, P* __restrict__ pt, int rows, int cols,
                                                      float lr, float b1, float b2, float eps, float wd, float bc1,
                                                      float bc2_sqrt, float gscale, const float* __restrict__ gscale_dev,
                                                      const float* __restrict__ hyper_dev) {
  __shared__ uint16_t tile[64][72];
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  if (hyper_dev) {
    lr = hyper_dev[0];
    bc1 = hyper_dev[1];
    bc2_sqrt = hyper_dev[2];
  }
  const float decay = 1.f - lr * wd;
  const float step_size = lr / bc1;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + 256 * k, r = idx >> 3, ch = idx & 7;
    const long o = (r0 + r) * cols + c0 + 8 * ch;
    float pv[8], gv[8], mv[8], vv[8];
    load8<P>(p + o, pv);
    load8<P>(g + o, gv);
    load8<P>(m + o, mv);
    load8<P>(v + o, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[j], mv[j], vv[j], gv[j], gs, decay, b1, b2, eps, bc2_sqrt, step_size);
    store8<P>(p + o, pv);
    store8<P>(m + o, mv);
    store8<P>(v + o, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][8 * ch + j] = __builtin_bit_cast(uint16_t, from_f<P>(pv[j]));
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + 256 * k, c = idx >> 3, rg = idx & 7;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[8 * rg + 2 * j][c] | ((uint32_t)tile[8 * rg + 2 * j + 1][c] << 16);
    *reinterpret_cast<uint4*>(pt + (c0 + c) * rows + r0 + 8 * rg) = make_uint4(w[0], w[1], w[2], w[3]);
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
                          const float* gscale_dev, const float* hyper_dev, int fast, hipStream_t s) {
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (pdtype != sdtype) return hipErrorInvalidValue;
  if (fast) {
    PRA_DISPATCH_FLOAT(pdtype, T,
                       hipLaunchKernelGGL((pra::adamw_kernel<T, T, true>), dim3(blocks), dim3(256), 0, s, (T*)p,
                                          (const T*)g, (T*)m, (T*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                          gscale_dev, hyper_dev));
  } else {
    PRA_DISPATCH_FLOAT(pdtype, T,
                       hipLaunchKernelGGL((pra::adamw_kernel<T, T, false>), dim3(blocks), dim3(256), 0, s, (T*)p,
                                          (const T*)g, (T*)m, (T*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                          gscale_dev, hyper_dev));
  }
  return hipGetLastError();
}

// AdamW of one [rows, cols] matrix + its transposed copy pt [cols, rows] (rows, cols % 64 == 0;
// 16-bit params, moments of the same dtype).
hipError_t pra_adamw_t(int dtype, void* p, const void* g, void* m, void* v, void* pt, int rows, int cols, float lr,
                       float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float gscale,
                       const float* gscale_dev, const float* hyper_dev, int fast, hipStream_t s) {
  if (rows % 64 || cols % 64 || rows <= 0 || cols <= 0) return hipErrorInvalidValue;
  // (A strip kernel walking 4 tiles per block was faster in isolation, 22.7 -> 21.3 ms per 7B step,
  // but slower overlapped with the backward GEMMs on the side stream: 1074.5 vs 1069.6 ms/step,
  // profiles/adamw_t_strip_ab_r2.log. Removed.)
  const dim3 grid(cols / 64, rows / 64);
  if (fast) {
    PRA_DISPATCH_16BIT(dtype, T,
                       hipLaunchKernelGGL((pra::adamw_t_kernel<T, true>), grid, dim3(256), 0, s, (T*)p, (const T*)g,
                                          (T*)m, (T*)v, (T*)pt, rows, cols, lr, b1, b2, eps, wd, bc1, bc2_sqrt,
                                          gscale, gscale_dev, hyper_dev));
  } else {
    PRA_DISPATCH_16BIT(dtype, T,
                       hipLaunchKernelGGL((pra::adamw_t_kernel<T, false>), grid, dim3(256), 0, s, (T*)p, (const T*)g,
                                          (T*)m, (T*)v, (T*)pt, rows, cols, lr, b1, b2, eps, wd, bc1, bc2_sqrt,
                                          gscale, gscale_dev, hyper_dev));
  }
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

// Flat-buffer AdamW and gradient-norm kernels.
//
// The engine keeps every trainable parameter, its gradient and both Adam moments in four
// flat, identically-ordered device buffers, so the optimizer step is ONE streaming kernel
// over N elements (14 B/elem for bf16 p/g/m/v: read 8, write 6) instead of a multi-tensor
// launch list. Math follows torch's fused AdamW (`_fused_adamw_`, used by the reference's
// `--fused-optimizer`, train.py:120-122) bit for bit in the default (!FAST) instantiation: the same
// mixed fp64/fp32 expression tree as ATen's adam_math (ATen/native/hip/fused_adam_utils.cuh: double
// lr/betas/eps/weight decay against fp32 values, fp32 bias corrections, correctly rounded fp32
// division and square root). The FAST instantiation (opt-in) takes the two divisions and the square
// root from the hardware (1 ulp) in pure fp32 (see adamw_elem).
//
//   p  = p - lr*wd*p
//   m  = b1*m + (1-b1)*g             v = b2*v + (1-b2)*g*g
//   p  = p - (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
//
// `gscale` pre-multiplies the gradient (1/world_size after a SUM all-reduce, and/or a
// clip coefficient read from device memory when `gscale_dev` is non-null). `hyper_dev`, when
// non-null, supplies {lr, bc1, bc2_sqrt} from device memory so a captured HIP graph of the
// training step replays with the current learning rate and bias corrections.
#include "common.h"

namespace pra {

// Scalars of one update, prepared once per thread from the host (or device, graph mode) values.
struct AdamCoef {
  double lr_wd, b1, b2, eps;  // torch's double hyper-parameters
  float bc2f, step_size;      // torch's fp32 bias correction and (float)(lr / bc1_f)
  float decay, b1f, b2f, epsf, rbc2;  // FAST: pure fp32 forms
};

__device__ __forceinline__ AdamCoef adam_coef(double lr, double b1, double b2, double eps, double wd, double bc1,
                                              double bc2_sqrt, const double* __restrict__ hyper_dev) {
  if (hyper_dev) {  // step-dependent scalars from device memory (graph-captured step)
    lr = hyper_dev[0];
    bc1 = hyper_dev[1];
    bc2_sqrt = hyper_dev[2];
  }
  AdamCoef c;
  c.lr_wd = lr * wd;
  c.b1 = b1;
  c.b2 = b2;
  c.eps = eps;
  const float bc1f = (float)bc1;  // ATen passes the double bias corrections as opmath_t (fp32)
  c.bc2f = (float)bc2_sqrt;
  c.step_size = (float)(lr / (double)bc1f);
  c.decay = (float)(1.0 - c.lr_wd);
  c.b1f = (float)b1;
  c.b2f = (float)b2;
  c.epsf = (float)eps;
  c.rbc2 = __builtin_amdgcn_rcpf(c.bc2f);
  return c;
}

// One AdamW element update with every fused multiply-add written out, so all kernels that use it
// (flat, tiled + transposed) round identically whatever the compiler's contraction choices.
// !FAST: ATen adam_math's expression tree. Its double sub-expressions are contracted the way hipcc
// contracts ATen's source (fadd(fmul a b, fmul c d) -> fma(a, b, c*d); p - x*p -> fma(-x, p, p));
// each is rounded once to fp32, then the fp32 tail (step_size*m)/denom is correctly rounded.
// FAST: the two divisions and the square root on the hardware v_rcp_f32 / v_sqrt_f32 (1 ulp each),
// all in fp32: ~17 instead of ~60 VALU per element. p differs from torch by a few fp32 ulps before
// its bf16 rounding (opt-in: PYRECOVER_ADAMW_FAST=1).
template <bool FAST>
__device__ __forceinline__ void adamw_elem(float& p, float& m, float& v, float g, float gs, const AdamCoef& c) {
  const float gr = g * gs;
  if constexpr (FAST) {
    p *= c.decay;
    m = fmaf(1.f - c.b1f, gr - m, m);
    v = fmaf(c.b2f, v, (1.f - c.b2f) * (gr * gr));
    const float denom = fmaf(__builtin_amdgcn_sqrtf(v), c.rbc2, c.epsf);
    p = fmaf(-c.step_size, m * __builtin_amdgcn_rcpf(denom), p);
  } else {
    const double pd = (double)p, gd = (double)gr;
    p = (float)fma(-c.lr_wd, pd, pd);
    m = (float)fma(c.b1, (double)m, (1.0 - c.b1) * gd);
    v = (float)fma(c.b2, (double)v, ((1.0 - c.b2) * gd) * gd);
    // m and v are rounded to fp32 here and again to 16 bits when stored, as in ATen's kernel. The
    // empty asm pins the fp32 values: without it the compiler may fuse the two roundings into one
    // (double -> bf16 through round-to-odd) in some instantiations and not in others, which moved
    // 13-77 of 4M values by one ulp between otherwise identical kernels.
    __asm__ volatile("" : "+v"(m), "+v"(v));
    // sqrtf / '/' as ATen writes them (std::sqrt, operator/): correctly rounded under hipcc's default
    // -fhip-fp32-correctly-rounded-divide-sqrt; __fsqrt_rn measured 1 ulp low on 0.08% of elements
    const float denom = (float)((double)(sqrtf(v) / c.bc2f) + c.eps);
    p = p - (c.step_size * m) / denom;
  }
}

// 16-B non-temporal loads and stores: the update streams every byte once, so its traffic is kept out
// of the caches the backward kernels beside it use.
typedef unsigned int pra_u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ pra_u32x4 ld16(const void* ptr) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const pra_u32x4*>(ptr));
  return *reinterpret_cast<const pra_u32x4*>(ptr);
}
template <bool NT>
__device__ __forceinline__ void st16(void* ptr, pra_u32x4 w) {
  if constexpr (NT) {
    __builtin_nontemporal_store(w, reinterpret_cast<pra_u32x4*>(ptr));
  } else {
    *reinterpret_cast<pra_u32x4*>(ptr) = w;
  }
}
// 16-B register <-> 8 floats, written exactly as load8 / store8 (common.h) write them: the exact
// AdamW's bitwise agreement with torch depends on how the compiler folds its double -> float ->
// 16-bit roundings, and a different packing sequence measured 13-77 of 4M p values one ulp apart.
template <typename P>
__device__ __forceinline__ void unpack8(pra_u32x4 w, float (&o)[8]) {
  if constexpr (sizeof(P) == 2 && __is_same(P, __bf16)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    uint4 raw = make_uint4(w[0], w[1], w[2], w[3]);
    const __half* h = reinterpret_cast<const __half*>(&raw);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = __half2float(h[i]);
  }
}
template <typename P>
__device__ __forceinline__ pra_u32x4 pack8(const float (&v)[8]) {
  if constexpr (__is_same(P, __bf16)) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)v[i];
    return __builtin_bit_cast(pra_u32x4, b);
  } else {
    uint4 raw;
    __half* h = reinterpret_cast<__half*>(&raw);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = __float2half_rn(v[i]);
    pra_u32x4 w;
    w[0] = raw.x;
    w[1] = raw.y;
    w[2] = raw.z;
    w[3] = raw.w;
    return w;
  }
}

template <typename P, typename S, bool FAST>
__global__ __launch_bounds__(256) void adamw_kernel(P* __restrict__ p, const P* __restrict__ g, S* __restrict__ m,
                                                    S* __restrict__ v, long n, double lr, double b1, double b2,
                                                    double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                                                    const float* __restrict__ gscale_dev,
                                                    const double* __restrict__ hyper_dev) {
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  const AdamCoef c = adam_coef(lr, b1, b2, eps, wd, bc1, bc2_sqrt, hyper_dev);
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long o = i * 8;
    float pv[8], gv[8], mv[8], vv[8];
    load8<P>(p + o, pv);
    load8<P>(g + o, gv);
    load8<S>(m + o, mv);
    load8<S>(v + o, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[j], mv[j], vv[j], gv[j], gs, c);
    store8<P>(p + o, pv);
    store8<S>(m + o, mv);
    store8<S>(v + o, vv);
  }
  // tail
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    float pv = to_f<P>(p[o]), mv = to_f<S>(m[o]), vv = to_f<S>(v[o]);
    adamw_elem<FAST>(pv, mv, vv, to_f<P>(g[o]), gs, c);
    p[o] = from_f<P>(pv);
    m[o] = from_f<S>(mv);
    v[o] = from_f<S>(vv);
  }
}

// Flat 16-bit AdamW (p, g, m, v of one dtype): U chunks of 8 per thread, all their loads issued
// before the math (more bytes in flight per wave), non-temporal. Same math as adamw_kernel.
template <typename P, bool FAST, int U>
__global__ __launch_bounds__(256) void adamw16_kernel(P* __restrict__ p, const P* __restrict__ g, P* __restrict__ m,
                                                      P* __restrict__ v, long n, double lr, double b1, double b2,
                                                      double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                                                      const float* __restrict__ gscale_dev,
                                                      const double* __restrict__ hyper_dev) {
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  const AdamCoef c = adam_coef(lr, b1, b2, eps, wd, bc1, bc2_sqrt, hyper_dev);
  const long n8 = n / 8, stride = (long)gridDim.x * 256 * U;
  for (long i0 = (long)blockIdx.x * 256 * U + threadIdx.x; i0 < n8; i0 += stride) {
    float pv[U][8], gv[U][8], mv[U][8], vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long o = (i0 + 256 * u) * 8;
      if (i0 + 256 * u < n8) {
        unpack8<P>(ld16<true>(p + o), pv[u]);
        unpack8<P>(ld16<true>(g + o), gv[u]);
        unpack8<P>(ld16<true>(m + o), mv[u]);
        unpack8<P>(ld16<true>(v + o), vv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long o = (i0 + 256 * u) * 8;
      if (i0 + 256 * u < n8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[u][j], mv[u][j], vv[u][j], gv[u][j], gs, c);
        st16<true>(p + o, pack8<P>(pv[u]));
        st16<true>(m + o, pack8<P>(mv[u]));
        st16<true>(v + o, pack8<P>(vv[u]));
      }
    }
  }
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    float pv = to_f<P>(p[o]), mv = to_f<P>(m[o]), vv = to_f<P>(v[o]);
    adamw_elem<FAST>(pv, mv, vv, to_f<P>(g[o]), gs, c);
    p[o] = from_f<P>(pv);
    m[o] = from_f<P>(mv);
    v[o] = from_f<P>(vv);
  }
}

// AdamW with fp32 master weights (--master-weights fp32): the update runs on the fp32
// master pm and fp32 moments (same adamw_elem math), and the 16-bit model parameter p the forward
// reads is pm rounded once. g is the 16-bit gradient.
template <typename P, bool FAST>
__global__ __launch_bounds__(256) void adamw_master_kernel(P* __restrict__ p, float* __restrict__ pm,
                                                           const P* __restrict__ g, float* __restrict__ m,
                                                           float* __restrict__ v, long n, double lr, double b1,
                                                           double b2, double eps, double wd, double bc1,
                                                           double bc2_sqrt, float gscale,
                                                           const float* __restrict__ gscale_dev,
                                                           const double* __restrict__ hyper_dev) {
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  const AdamCoef c = adam_coef(lr, b1, b2, eps, wd, bc1, bc2_sqrt, hyper_dev);
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long o = i * 8;
    float pv[8], gv[8], mv[8], vv[8];
    load8<float>(pm + o, pv);
    load8<P>(g + o, gv);
    load8<float>(m + o, mv);
    load8<float>(v + o, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[j], mv[j], vv[j], gv[j], gs, c);
    store8<float>(pm + o, pv);
    store8<float>(m + o, mv);
    store8<float>(v + o, vv);
    store8<P>(p + o, pv);
  }
  for (long o = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    float pv = pm[o], mv = m[o], vv = v[o];
    adamw_elem<FAST>(pv, mv, vv, to_f<P>(g[o]), gs, c);
    pm[o] = pv;
    m[o] = mv;
    v[o] = vv;
    p[o] = from_f<P>(pv);
  }
}

// AdamW over one row-major [rows, cols] weight matrix that ALSO writes its transposed copy
// pt [cols, rows] (the data-gradient GEMM's operand, parallel/flat.py "weight shadows") from the
// updated values it already holds: the separate transpose pass re-read the whole model after
// every update (13.5 GB/step at 7B). Block = one 64 x 64 tile; the updated p tile goes through
// LDS (padded rows) to 16-B transposed stores. Same math and rounding as adamw_kernel.
template <typename P, bool FAST, int TILE, bool NT>
__global__ __launch_bounds__(256) void adamw_t_kernel(P* __restrict__ p, const P* __restrict__ g, P* __restrict__ m,
                                                      P* __restrict__ v, P* __restrict__ pt, int rows, int cols,
                                                      double lr, double b1, double b2, double eps, double wd,
                                                      double bc1, double bc2_sqrt, float gscale,
                                                      const float* __restrict__ gscale_dev,
                                                      const double* __restrict__ hyper_dev) {
  constexpr int CH = TILE / 8;            // 8-element chunks per tile row
  constexpr int PASSES = TILE * CH / 256;  // chunks per thread
  __shared__ uint16_t tile[TILE][TILE + 8];
  const float gs = gscale_dev ? gscale * gscale_dev[0] : gscale;
  const AdamCoef c = adam_coef(lr, b1, b2, eps, wd, bc1, bc2_sqrt, hyper_dev);
  const long r0 = (long)blockIdx.y * TILE, c0 = (long)blockIdx.x * TILE;
#pragma unroll
  for (int k = 0; k < PASSES; ++k) {
    const int idx = threadIdx.x + 256 * k, r = idx / CH, ch = idx % CH;
    const long o = (r0 + r) * cols + c0 + 8 * ch;
    float pv[8], gv[8], mv[8], vv[8];
    unpack8<P>(ld16<NT>(p + o), pv);
    unpack8<P>(ld16<NT>(g + o), gv);
    unpack8<P>(ld16<NT>(m + o), mv);
    unpack8<P>(ld16<NT>(v + o), vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) adamw_elem<FAST>(pv[j], mv[j], vv[j], gv[j], gs, c);
    st16<NT>(p + o, pack8<P>(pv));
    st16<NT>(m + o, pack8<P>(mv));
    st16<NT>(v + o, pack8<P>(vv));
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][8 * ch + j] = __builtin_bit_cast(uint16_t, from_f<P>(pv[j]));
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PASSES; ++k) {
    const int idx = threadIdx.x + 256 * k, cc = idx / CH, rg = idx % CH;
    pra_u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[8 * rg + 2 * j][cc] | ((uint32_t)tile[8 * rg + 2 * j + 1][cc] << 16);
    st16<NT>(pt + (c0 + cc) * rows + r0 + 8 * rg, w);
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
hipError_t pra_adamw_flat(int pdtype, int sdtype, void* p, const void* g, void* m, void* v, long n, double lr,
                          double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                          const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s) {
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (pdtype != sdtype) return hipErrorInvalidValue;
  if (pdtype != ::pra::kF32) {
    // 16-bit: two iterations per thread, non-temporal (Llama-3-8B-shape matrices in isolation 4.82 ->
    // 5.28-5.46 TB/s; 8B B1 step -0.76%: profiles/r6/adamw/)
    long nb = (n / 8 + 511) / 512;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    if (fast) {
      PRA_DISPATCH_16BIT(pdtype, T,
                         hipLaunchKernelGGL((pra::adamw16_kernel<T, true, 2>), dim3(nb), dim3(256), 0, s, (T*)p,
                                            (const T*)g, (T*)m, (T*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                            gscale_dev, hyper_dev));
    } else {
      PRA_DISPATCH_16BIT(pdtype, T,
                         hipLaunchKernelGGL((pra::adamw16_kernel<T, false, 2>), dim3(nb), dim3(256), 0, s,
                                            (T*)p, (const T*)g, (T*)m, (T*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt,
                                            gscale, gscale_dev, hyper_dev));
    }
    return hipGetLastError();
  }
  // fp32 parameters and moments
  if (fast) {
    hipLaunchKernelGGL((pra::adamw_kernel<float, float, true>), dim3(blocks), dim3(256), 0, s, (float*)p,
                       (const float*)g, (float*)m, (float*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale, gscale_dev,
                       hyper_dev);
  } else {
    hipLaunchKernelGGL((pra::adamw_kernel<float, float, false>), dim3(blocks), dim3(256), 0, s, (float*)p,
                       (const float*)g, (float*)m, (float*)v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale, gscale_dev,
                       hyper_dev);
  }
  return hipGetLastError();
}

// AdamW of one [rows, cols] matrix + its transposed copy pt [cols, rows] (rows, cols % 64 == 0;
// 16-bit params, moments of the same dtype): 128 x 128 tiles where both dims allow, else 64 x 64;
// non-temporal (Llama-3-8B B1 with shadows -1.03%, 7B B16 within noise: profiles/r6/adamw/).
hipError_t pra_adamw_t(int dtype, void* p, const void* g, void* m, void* v, void* pt, int rows, int cols, double lr,
                       double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                       const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s) {
  if (rows % 64 || cols % 64 || rows <= 0 || cols <= 0) return hipErrorInvalidValue;
  // (A strip kernel walking 4 tiles per block was faster in isolation, 22.7 -> 21.3 ms per 7B step,
  // but slower overlapped with the backward GEMMs on the side stream: 1074.5 vs 1069.6 ms/step,
  // profiles/adamw_t_strip_ab_r2.log. Removed.)
  const int tile = (rows % 128 == 0 && cols % 128 == 0) ? 128 : 64;
  const dim3 grid(cols / tile, rows / tile);
#define PRA_ADAMW_T(FASTV, TILEV)                                                                              \
  PRA_DISPATCH_16BIT(dtype, T,                                                                                  \
                     hipLaunchKernelGGL((pra::adamw_t_kernel<T, FASTV, TILEV, true>), grid, dim3(256), 0, s,    \
                                        (T*)p, (const T*)g, (T*)m, (T*)v, (T*)pt, rows, cols, lr, b1, b2, eps,   \
                                        wd, bc1, bc2_sqrt, gscale, gscale_dev, hyper_dev))
  if (tile == 128 && fast) {
    PRA_ADAMW_T(true, 128);
  } else if (tile == 128) {
    PRA_ADAMW_T(false, 128);
  } else if (fast) {
    PRA_ADAMW_T(true, 64);
  } else {
    PRA_ADAMW_T(false, 64);
  }
#undef PRA_ADAMW_T
  return hipGetLastError();
}

hipError_t pra_adamw_master(int pdtype, void* p, float* pm, const void* g, float* m, float* v, long n, double lr,
                            double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                            const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s) {
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (fast) {
    PRA_DISPATCH_16BIT(pdtype, T,
                       hipLaunchKernelGGL((pra::adamw_master_kernel<T, true>), dim3(blocks), dim3(256), 0, s, (T*)p,
                                          pm, (const T*)g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                          gscale_dev, hyper_dev));
  } else {
    PRA_DISPATCH_16BIT(pdtype, T,
                       hipLaunchKernelGGL((pra::adamw_master_kernel<T, false>), dim3(blocks), dim3(256), 0, s, (T*)p,
                                          pm, (const T*)g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                          gscale_dev, hyper_dev));
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

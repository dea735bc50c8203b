// RMSNorm forward/backward with an optional fused residual add (gfx950).
//
// Semantics follow the reference RMSNorm (reference model.py:25-49):
//     y = type_as(x_f32 * rsqrt(mean(x_f32^2) + eps)) * weight
// i.e. the normalized value is rounded to the storage dtype before the weight multiply,
// and the weight multiply is itself rounded. The fused variant first forms
//     h = x + delta   (rounded to the storage dtype, exactly like the reference's
//                      `h = x + self.attention(...)` in model.py:325-327)
// and normalizes h.
//
// Layout: one wave64 per row, 4 rows per 256-thread block, 8 elements (16 B) per lane per
// chunk, the whole row held in registers (NV chunks of 512 elements), so every element
// is read from HBM exactly once.
#include "common.h"

namespace pra {

template <typename T, int NV, bool HAS_DELTA>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ delta, const T* __restrict__ w,
    T* __restrict__ h_out, T* __restrict__ y, float* __restrict__ rstd_out, int rows, int D,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * D;
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < D) {
      load8<T>(x + base + c, v[i]);
      if constexpr (HAS_DELTA) {
        float d[8];
        load8<T>(delta + base + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = rnd<T>(v[i][j] + d[j]);
        store8<T>(h_out + base + c, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < D) {
      float wv[8], o[8];
      load8<T>(w + c, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rnd<T>(v[i][j] * r) * wv[j];
      store8<T>(y + base + c, o);
    }
  }
  if (lane == 0) rstd_out[row] = r;
}

// Backward. For each row:
//   nb  = round(h * rstd)                    (the forward's rounded normalized value)
//   dnb = round(dy * w)                      (grad of the weight multiply)
//   dx  = rstd * (dnb - h * rstd^2 * sum(dnb*h)/D)
//   out = round(round(dx) + dres)            (fused residual-path grad, if given)
// A 256-thread block owns rows b, b+G, ...; each thread owns NVB 8-wide column chunks, so
// h/dy/w/dw live in registers (64 floats at NVB=2). dw partial sums (fp32) per block go to
// `dw_partial[block][D]`; a second deterministic kernel reduces them in fixed order.
template <typename T, int NVB, bool HAS_DRES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ h, const T* __restrict__ w,
    const float* __restrict__ rstd, const T* dres, T* dx, float* __restrict__ dw_partial,
    int rows, int D) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  float wv[NVB][8];
  float dw[NVB][8];
#pragma unroll
  for (int i = 0; i < NVB; ++i) {
    const int c = (i * 256 + tid) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[i][j] = 0.f;
    if (c < D) load8<T>(w + c, wv[i]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * D;
    const float r = rstd[row];
    float hv[NVB][8], g[NVB][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int c = (i * 256 + tid) * 8;
      if (c < D) {
        float d[8];
        load8<T>(h + base + c, hv[i]);
        load8<T>(dy + base + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float nb = rnd<T>(hv[i][j] * r);
          dw[i][j] += d[j] * nb;
          g[i][j] = rnd<T>(d[j] * wv[i][j]);
          dot += g[i][j] * hv[i][j];
        }
      }
    }
    dot = block_sum<4>(dot, red);
    const float k = r * r * dot / (float)D;
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int c = (i * 256 + tid) * 8;
      if (c < D) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rnd<T>(r * (g[i][j] - hv[i][j] * k));
        if constexpr (HAS_DRES) {
          float d[8];
          load8<T>(dres + base + c, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = o[j] + d[j];
        }
        store8<T>(dx + base + c, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NVB; ++i) {
    const int c = (i * 256 + tid) * 8;
    if (c < D) store8<float>(dw_partial + (size_t)blockIdx.x * D + c, dw[i]);
  }
}

// Deterministic two-stage column reduction of the P partial rows:
//   stage 1: grid (ceil(D/256), kColsumSplit): block (x, y) sums rows [y*ceil(P/S), ...) of 256
//            columns (4 per lane, 16-B loads, 4 waves interleaving rows, 4 loads in flight per lane),
//            reduced through LDS in fixed order -> part2[y][D]
//   stage 2: out[c] = (accumulate ? out[c] : 0) + part2[0][c] + ... + part2[S-1][c]
// (Was 64 columns x 4 row groups with 4-B loads: 20 us for the 16.8 MB of partials of a Llama-3-8B
// batch-1 backward, 0.8 TB/s; 65 calls = 1.3 ms of that step.)
constexpr int kColsumSplit = 16;

__global__ __launch_bounds__(256) void colsum_stage1(const float* __restrict__ part, float* __restrict__ part2,
                                                     int P, int D) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;  // D % 8 == 0: c < D implies c + 3 < D
  const int per = (P + kColsumSplit - 1) / kColsumSplit;
  const int r0 = blockIdx.y * per, r1 = min(P, r0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < D) {
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += 4) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)r * D + c);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  red[rg][lane] = s;
  __syncthreads();
  if (rg == 0 && c < D) {
    float4 o = red[0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      o.x += red[k][lane].x;
      o.y += red[k][lane].y;
      o.z += red[k][lane].z;
      o.w += red[k][lane].w;
    }
    *reinterpret_cast<float4*>(part2 + (size_t)blockIdx.y * D + c) = o;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_stage2(const float* __restrict__ part2, T* __restrict__ out, int D,
                                                     int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  float s = part2[c];
#pragma unroll
  for (int k = 1; k < kColsumSplit; ++k) s += part2[(size_t)k * D + c];
  if (accumulate) s += to_f<T>(out[c]);
  out[c] = from_f<T>(s);
}

// ======================================================================================
// LayerNorm (norm_type="layernorm", GPT-2-shape presets) with the same fused residual add.
//   y = round((h - mean) * rstd * w + b)  (fp32 math, one rounding, like torch's layer_norm)
// Backward: dxhat = dy*w; dx = rstd*(dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)) (+ dres);
// dw = sum(dy*xhat), db = sum(dy) -> partial rows [P][2D] reduced by the same colsum.
template <typename T, int NV, bool HAS_DELTA>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ delta, const T* __restrict__ w, const T* __restrict__ bias,
    T* __restrict__ h_out, T* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows,
    int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * D;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < D) {
      load8<T>(x + base + c, v[i]);
      if constexpr (HAS_DELTA) {
        float d[8];
        load8<T>(delta + base + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = rnd<T>(v[i][j] + d[j]);
        store8<T>(h_out + base + c, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[i][j] - mean;
        ss += t * t;
      }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < D) {
      float wv[8], bv[8], o[8];
      load8<T>(w + c, wv);
      load8<T>(bias + c, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * r * wv[j] + bv[j];
      store8<T>(y + base + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = r;
  }
}

template <typename T, int NVB, bool HAS_DRES>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ h, const T* __restrict__ w, const float* __restrict__ mean_in,
    const float* __restrict__ rstd, const T* dres, T* dx, float* __restrict__ part, int rows, int D) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  float wv[NVB][8], dw[NVB][8], db[NVB][8];
#pragma unroll
  for (int i = 0; i < NVB; ++i) {
    const int c = (i * 256 + tid) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { dw[i][j] = 0.f; db[i][j] = 0.f; }
    if (c < D) load8<T>(w + c, wv[i]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * D;
    const float mu = mean_in[row], r = rstd[row];
    float xh[NVB][8], g[NVB][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int c = (i * 256 + tid) * 8;
      if (c < D) {
        float d[8];
        load8<T>(h + base + c, xh[i]);
        load8<T>(dy + base + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (xh[i][j] - mu) * r;
          dw[i][j] += d[j] * xh[i][j];
          db[i][j] += d[j];
          g[i][j] = d[j] * wv[i][j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
        }
      }
    }
    s1 = block_sum<4>(s1, red) / (float)D;
    s2 = block_sum<4>(s2, red) / (float)D;
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int c = (i * 256 + tid) * 8;
      if (c < D) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rnd<T>(r * (g[i][j] - s1 - xh[i][j] * s2));
        if constexpr (HAS_DRES) {
          float d[8];
          load8<T>(dres + base + c, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = o[j] + d[j];
        }
        store8<T>(dx + base + c, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NVB; ++i) {
    const int c = (i * 256 + tid) * 8;
    if (c < D) {
      store8<float>(part + (size_t)blockIdx.x * 2 * D + c, dw[i]);
      store8<float>(part + (size_t)blockIdx.x * 2 * D + D + c, db[i]);
    }
  }
}

template <typename T, int NV>
static hipError_t ln_fwd_impl(const void* x, const void* delta, const void* w, const void* b, void* h_out, void* y,
                              float* mean, float* rstd, int rows, int D, float eps, hipStream_t s) {
  dim3 grid((rows + 3) / 4), block(256);
  if (delta)
    hipLaunchKernelGGL((layernorm_fwd_kernel<T, NV, true>), grid, block, 0, s, (const T*)x, (const T*)delta,
                       (const T*)w, (const T*)b, (T*)h_out, (T*)y, mean, rstd, rows, D, eps);
  else
    hipLaunchKernelGGL((layernorm_fwd_kernel<T, NV, false>), grid, block, 0, s, (const T*)x, (const T*)nullptr,
                       (const T*)w, (const T*)b, (T*)nullptr, (T*)y, mean, rstd, rows, D, eps);
  return hipGetLastError();
}

template <typename T, int NVB>
static hipError_t ln_bwd_impl(const void* dy, const void* h, const void* w, const float* mean, const float* rstd,
                              const void* dres, void* dx, void* dwb, float* ws, int ws_rows, int rows, int D,
                              int accumulate, hipStream_t s) {
  if (dres)
    hipLaunchKernelGGL((layernorm_bwd_kernel<T, NVB, true>), dim3(ws_rows), dim3(256), 0, s, (const T*)dy,
                       (const T*)h, (const T*)w, mean, rstd, (const T*)dres, (T*)dx, ws, rows, D);
  else
    hipLaunchKernelGGL((layernorm_bwd_kernel<T, NVB, false>), dim3(ws_rows), dim3(256), 0, s, (const T*)dy,
                       (const T*)h, (const T*)w, mean, rstd, (const T*)nullptr, (T*)dx, ws, rows, D);
  const int D2 = 2 * D;
  float* part2 = ws + (size_t)ws_rows * D2;
  hipLaunchKernelGGL(colsum_stage1, dim3((D2 + 255) / 256, kColsumSplit), dim3(256), 0, s, ws, part2, ws_rows, D2);
  hipLaunchKernelGGL((colsum_stage2<T>), dim3((D2 + 255) / 256), dim3(256), 0, s, part2, (T*)dwb, D2, accumulate);
  return hipGetLastError();
}

template <typename T, int NV>
static hipError_t fwd_impl(const void* x, const void* delta, const void* w, void* h_out, void* y,
                           float* rstd, int rows, int D, float eps, hipStream_t s) {
  dim3 grid((rows + 3) / 4), block(256);
  if (delta)
    hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, NV, true>), grid, block, 0, s, (const T*)x,
                       (const T*)delta, (const T*)w, (T*)h_out, (T*)y, rstd, rows, D, eps);
  else
    hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, NV, false>), grid, block, 0, s, (const T*)x,
                       (const T*)nullptr, (const T*)w, (T*)nullptr, (T*)y, rstd, rows, D, eps);
  return hipGetLastError();
}

template <typename T, int NVB>
static hipError_t bwd_impl(const void* dy, const void* h, const void* w, const float* rstd,
                           const void* dres, void* dx, void* dw, float* ws, int ws_rows, int rows,
                           int D, int accumulate, hipStream_t s) {
  const int blocks = ws_rows;
  if (dres)
    hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, NVB, true>), dim3(blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)h, (const T*)w, rstd, (const T*)dres, (T*)dx, ws, rows, D);
  else
    hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, NVB, false>), dim3(blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)h, (const T*)w, rstd, (const T*)nullptr, (T*)dx, ws, rows, D);
  float* part2 = ws + (size_t)ws_rows * D;
  hipLaunchKernelGGL(colsum_stage1, dim3((D + 255) / 256, kColsumSplit), dim3(256), 0, s, ws, part2, ws_rows, D);
  hipLaunchKernelGGL((colsum_stage2<T>), dim3((D + 255) / 256), dim3(256), 0, s, part2, (T*)dw, D, accumulate);
  return hipGetLastError();
}

#define PRA_NV_DISPATCH(D, NV, ...)                 \
  if ((D) <= 512) { constexpr int NV = 1; __VA_ARGS__; } \
  else if ((D) <= 1024) { constexpr int NV = 2; __VA_ARGS__; } \
  else if ((D) <= 2048) { constexpr int NV = 4; __VA_ARGS__; } \
  else if ((D) <= 4096) { constexpr int NV = 8; __VA_ARGS__; } \
  else if ((D) <= 8192) { constexpr int NV = 16; __VA_ARGS__; } \
  else return hipErrorInvalidValue;

#define PRA_NVB_DISPATCH(D, NVB, ...)                 \
  if ((D) <= 2048) { constexpr int NVB = 1; __VA_ARGS__; } \
  else if ((D) <= 4096) { constexpr int NVB = 2; __VA_ARGS__; } \
  else if ((D) <= 8192) { constexpr int NVB = 4; __VA_ARGS__; } \
  else if ((D) <= 16384) { constexpr int NVB = 8; __VA_ARGS__; } \
  else return hipErrorInvalidValue;

}  // namespace pra

extern "C" {

// Number of fp32 workspace rows (each D floats) the backward needs for `rows` rows.
// Blocks of the backward kernel (= fp32 partial rows of dw); the workspace must hold
// pra_rmsnorm_bwd_ws_rows(rows) + pra_rmsnorm_bwd_ws_extra() rows of D floats.
// 1024 blocks = 4 per CU: each block walks its rows one at a time (load -> block reduce -> store),
// so several blocks per CU are what keeps enough HBM requests in flight.
int pra_rmsnorm_bwd_ws_rows(int rows) { return rows < 1024 ? rows : 1024; }
int pra_rmsnorm_bwd_ws_extra() { return pra::kColsumSplit; }

hipError_t pra_rmsnorm_fwd(int dtype, const void* x, const void* delta, const void* w, void* h_out,
                           void* y, float* rstd, int rows, int D, float eps, hipStream_t s) {
  if (D % 8 != 0) return hipErrorInvalidValue;
  PRA_DISPATCH_FLOAT(dtype, T, PRA_NV_DISPATCH(D, NV, return pra::fwd_impl<T, NV>(x, delta, w, h_out, y, rstd, rows, D, eps, s)));
  return hipSuccess;
}

// LayerNorm: dwb = [dw | db] (2*D contiguous, e.g. the flat gradient slot of weight|bias);
// workspace = (pra_rmsnorm_bwd_ws_rows(rows) + pra_rmsnorm_bwd_ws_extra()) * 2 * D floats.
hipError_t pra_layernorm_fwd(int dtype, const void* x, const void* delta, const void* w, const void* b, void* h_out,
                             void* y, float* mean, float* rstd, int rows, int D, float eps, hipStream_t s) {
  if (D % 8 != 0) return hipErrorInvalidValue;
  PRA_DISPATCH_FLOAT(dtype, T, PRA_NV_DISPATCH(D, NV, return pra::ln_fwd_impl<T, NV>(x, delta, w, b, h_out, y, mean, rstd, rows, D, eps, s)));
  return hipSuccess;
}

hipError_t pra_layernorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* mean,
                             const float* rstd, const void* dres, void* dx, void* dwb, float* ws, int rows, int D,
                             int accumulate, hipStream_t s) {
  if (D % 8 != 0) return hipErrorInvalidValue;
  const int ws_rows = pra_rmsnorm_bwd_ws_rows(rows);
  PRA_DISPATCH_FLOAT(dtype, T, PRA_NVB_DISPATCH(D, NVB, return pra::ln_bwd_impl<T, NVB>(dy, h, w, mean, rstd, dres, dx, dwb, ws, ws_rows, rows, D, accumulate, s)));
  return hipSuccess;
}

hipError_t pra_rmsnorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* rstd,
                           const void* dres, void* dx, void* dw, float* ws, int rows, int D,
                           int accumulate, hipStream_t s) {
  if (D % 8 != 0) return hipErrorInvalidValue;
  const int ws_rows = pra_rmsnorm_bwd_ws_rows(rows);
  PRA_DISPATCH_FLOAT(dtype, T, PRA_NVB_DISPATCH(D, NVB, return pra::bwd_impl<T, NVB>(dy, h, w, rstd, dres, dx, dw, ws, ws_rows, rows, D, accumulate, s)));
  return hipSuccess;
}

}  // extern "C"

// C ABI of the HIP kernels in csrc/kernels/*.hip. The kernel translation units do not include
// any torch header; csrc/bindings.cpp adapts torch tensors to these raw-pointer launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {
int pra_rmsnorm_bwd_ws_extra();
int pra_rmsnorm_bwd_ws_rows(int rows);
hipError_t pra_rmsnorm_fwd(int dtype, const void* x, const void* delta, const void* w, void* h_out, void* y,
                           float* rstd, int rows, int D, float eps, hipStream_t s);
hipError_t pra_rmsnorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* rstd,
                           const void* dres, void* dx, void* dw, float* ws, int rows, int D, int accumulate,
                           hipStream_t s);

hipError_t pra_layernorm_fwd(int dtype, const void* x, const void* delta, const void* w, const void* b, void* h_out,
                             void* y, float* mean, float* rstd, int rows, int D, float eps, hipStream_t s);
hipError_t pra_layernorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* mean,
                             const float* rstd, const void* dres, void* dx, void* dwb, float* ws, int rows, int D,
                             int accumulate, hipStream_t s);

hipError_t pra_rope(int dtype, void* x, const void* tab, long ntok, int ld, int ncols, int D, int S,
                    int pos_offset, int inverse, hipStream_t s);
hipError_t pra_swiglu_fwd(int dtype, const void* g, const void* u, void* y, long ntok, int F, int ldg, int ldu,
                          int ldy, hipStream_t s);
hipError_t pra_swiglu_bwd(int dtype, const void* dy, const void* g, const void* u, void* dg, void* du, long ntok,
                          int F, int ldg, int ldu, int lddy, int variant, hipStream_t s);
hipError_t pra_embedding_fwd(int dtype, const int64_t* ids, const void* W, void* out, long ntok, int D, long V,
                             hipStream_t s);
hipError_t pra_embedding_bwd(int dtype, const int64_t* sorted_ids, const int64_t* perm, const void* dout, void* dW,
                             long ntok, int D, long V, int accumulate, hipStream_t s);

hipError_t pra_swiglu_fwd_t(int dtype, const void* gu, void* a, void* aT, long ntok, int F, int ldgu, int lda,
                            hipStream_t s);
hipError_t pra_swiglu_bwd_t(int dtype, const void* dy, void* gu, void* guT, long ntok, int F, int ldgu, int lddy,
                            hipStream_t s);
hipError_t pra_rope_t(int dtype, void* x, void* xT, const void* tab, long ntok, int ld, int ncols, int nrot, int D,
                      int S, int inverse, hipStream_t s);
hipError_t pra_transpose16(const void* src, void* dst, long R, long C, long ld_src, long ld_dst, hipStream_t s);
// C[M][N] (+)= A^T B, A [K][M], B [K][N] row-major (weight gradient on row-major activations);
// M, N multiples of 256, K of 32 (gemm_wgrad.hip)
hipError_t pra_wgrad_gemm(int dtype, const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                          long ldc, int accumulate, float* ws, int* tickets, int cus, hipStream_t s);
hipError_t pra_wgrad_gemm_exp(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                              long ldc, int exp, hipStream_t s);
long pra_wgrad_ws_floats(int M, int N, int K, int cus);
int pra_wgrad_ticket_count(int M, int N, int K, int cus);
// C = A B^T, A [M][K], B [N][K] (both K-contiguous) with a fused epilogue (gemm_nt.hip):
// epi 0 plain, 1 SwiGLU forward (C = gu [M][2F], c2 = a [M][F]), 2 SwiGLU backward in place over
// gu (C), 3 RoPE on the first nrot columns (tab float2 [S][D/2])
hipError_t pra_gemm_nt(int dtype, int epi, const void* A, const void* B, void* C, int M, int N, int K, long lda,
                       long ldb, long ldc, void* c2, long ldc2, int F, const void* tab, int S, int D, int nrot,
                       float* ws, int* tickets, int cus, hipStream_t s);
long pra_gemm_nt_ws_floats(int M, int N, int K, int cus);
int pra_gemm_nt_ticket_count(int M, int N, int K, int cus);

hipError_t pra_xent_fwd(int dtype, const void* logits, const int64_t* labels, float* lse, float* loss_row,
                        float* stats, long T, long V, long ld, long ignore_index, hipStream_t s);
hipError_t pra_xent_bwd(int dtype, void* logits, const int64_t* labels, const float* lse, const float* stats,
                        const float* grad_out, long T, long V, long ld, long ignore_index, hipStream_t s);

hipError_t pra_adamw_flat(int pdtype, int sdtype, void* p, const void* g, void* m, void* v, long n, double lr,
                          double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                          const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s);
// fp32-master AdamW: updates pm / m / v (fp32) and writes p = round(pm) (16-bit params)
hipError_t pra_adamw_master(int pdtype, void* p, float* pm, const void* g, float* m, float* v, long n, double lr,
                            double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                            const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s);
int pra_sumsq_partials();
hipError_t pra_grad_norm(int dtype, const void* x, long n, float* ws, float* out, float max_norm, float pre_scale,
                         hipStream_t s);

// dst <- src, nbytes, device memory (16-B vector path when both are 16-B aligned)
hipError_t pra_copy_d2d(void* dst, const void* src, long nbytes, hipStream_t s);
int pra_checksum_blocks();
hipError_t pra_checksum(int dtype, const void* x, long nbytes, double* ws_sum, unsigned long long* ws_hash,
                        double* out_sum, unsigned long long* out_hash, hipStream_t s);
hipError_t pra_sum_slices(int dtype, const void* const* srcs, int nsrc, void* dst, long n, hipStream_t s);
// n (<= 16) copies src[k] -> dst[k] of nbytes[k] in one kernel (16-B aligned pointers)
hipError_t pra_pull_gather(const void* const* srcs, void* const* dsts, const long* nbytes, int n, hipStream_t s);

hipError_t pra_adamw_t(int dtype, void* p, const void* g, void* m, void* v, void* pt, int rows, int cols, double lr,
                       double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt, float gscale,
                       const float* gscale_dev, const double* hyper_dev, int fast, hipStream_t s);

hipError_t pra_attn_fwd(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq,
                        int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal,
                        int skv, hipStream_t st);
// delta: fp32 workspace of 3 * B * Hq * S floats (delta and the pipelined dK/dV kernel's row constants)
hipError_t pra_attn_bwd(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv,
                        int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk, long lddv,
                        float scale, int causal, int skv, const float* rope_tab, hipEvent_t mid_event,
                        hipStream_t st);
void pra_attn_set_options(int fwd_pipe, float fwd_thr, int dkdv_impl, int dq_pipe, int dkdv_split, int dkdv_kreg,
                          int bwd_fused, int bwd_window);
// block order of the forward / dQ / dK/dV grids: 0 = heavy tiles first, G > 0 = XCD-grouped with G heads
// per group, -1 = by shape (attention.hip block_tile)
void pra_attn_set_order(int fwd, int dq, int dkdv);
// fused dQ/dK/dV backward (attention_bwd_fused.hip); ws: 2 B Hq S row constants + B Hq S 128 dQ partials
hipError_t pra_attn_bwd_fused(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout,
                              const float* lse, float* ws, void* dq, void* dk, void* dv, int B, int S, int Hq,
                              int Hkv, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk,
                              long lddv, float scale, int causal, const float* rope_tab, hipEvent_t mid_event,
                              hipStream_t st);
// floats of fp32 workspace pra_attn_bwd needs at `delta` (delta, row constants, split dK/dV parts)
long pra_attn_bwd_workspace(int dtype, int B, int S, int Hq, int Hkv, int D);
// fp32 flash attention (attention_f32.hip, f32-input MFMA); pra_attn_fwd / pra_attn_bwd route kF32 here
hipError_t pra_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, float* lse, int B, int S, int Hq,
                            int Hkv, int D, long ldq, long ldk, long ldv, long ldo, float scale, int causal, int skv,
                            hipStream_t st);
hipError_t pra_attn_bwd_f32(const float* q, const float* k, const float* v, const float* o, const float* dout,
                            const float* lse, float* delta, float* dq, float* dk, float* dv, int B, int S, int Hq,
                            int Hkv, int D, long ldq, long ldk, long ldv, long ldo, long lddo, long lddq, long lddk,
                            long lddv, float scale, int causal, int skv, hipStream_t st);
}

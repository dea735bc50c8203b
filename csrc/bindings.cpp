// Torch <-> HIP kernel adapter for pyrecover_amd._C.
//
// Every op validates shapes/strides/dtypes on the host BEFORE launching (a mis-shaped launch
// of a hand-written kernel could fault the GPU), then calls the raw launcher on the current
// HIP stream of the tensor's device.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <roctracer/roctx.h>

#include <atomic>
#include <cstdlib>

#include "kernels/launchers.h"

namespace {

// roctx range per op ("pyrecover::attn_fwd", ...) so rocprofv3 --marker-trace / --selected-regions
// timelines show which framework op launched each kernel. Off by default (one branch per op);
// enabled by set_roctx(True) (train.py --profile) or PYRECOVER_ROCTX=1.
std::atomic<bool> g_roctx{[] {
  const char* e = std::getenv("PYRECOVER_ROCTX");
  return e != nullptr && e[0] == '1';
}()};
struct Range {
  bool on;
  explicit Range(const char* name) : on(g_roctx.load(std::memory_order_relaxed)) {
    if (on) roctxRangePushA(name);
  }
  ~Range() {
    if (on) roctxRangePop();
  }
};

int dt(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "pyrecover_amd: unsupported dtype ", t.scalar_type());
  }
}

hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pyrecover_amd: ", what, " failed: ", hipGetErrorString(e));
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "pyrecover_amd: ", name, " must be a GPU tensor");
}

// Every pointer handed to a kernel must live on the launch device (a host or foreign-device
// pointer in a kernel argument is a GPU memory fault, not an exception).
void same_dev(const at::Tensor& ref, const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.defined() && t.is_cuda() && t.device() == ref.device(), "pyrecover_amd: ", name,
              " must be on ", ref.device(), " (got ", t.defined() ? t.device().str() : std::string("undefined"), ")");
}

void check_row_major(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "pyrecover_amd: ", name, " must be 2-D with unit inner stride");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "pyrecover_amd: ", name, " must be 16-B aligned");
}

// ---------------------------------------------------------------------------------------
std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& delta, const at::Tensor& w,
                                    double eps) {
  const Range range_("pyrecover::rmsnorm_fwd");
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "rmsnorm_fwd: x and w must be contiguous");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(w.numel() == D && w.scalar_type() == x.scalar_type(), "rmsnorm_fwd: weight mismatch");
  same_dev(x, w, "rmsnorm weight");
  if (delta.has_value()) same_dev(x, *delta, "rmsnorm delta");
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "rmsnorm_fwd: D must be a multiple of 8 and <= 8192");
  const c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty_like(x);
  at::Tensor rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor h;
  const void* dptr = nullptr;
  if (delta.has_value()) {
    TORCH_CHECK(delta->sizes() == x.sizes() && delta->is_contiguous() && delta->scalar_type() == x.scalar_type(),
                "rmsnorm_fwd: delta mismatch");
    h = at::empty_like(x);
    dptr = delta->data_ptr();
  }
  check(pra_rmsnorm_fwd(dt(x), x.data_ptr(), dptr, w.data_ptr(), h.defined() ? h.data_ptr() : nullptr,
                        y.data_ptr(), rstd.data_ptr<float>(), (int)rows, (int)D, (float)eps, stream_of(x)),
        "rmsnorm_fwd");
  return {h.defined() ? h : x, y, rstd};
}

at::Tensor rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w, const at::Tensor& rstd,
                       const c10::optional<at::Tensor>& dres, at::Tensor dw, bool accumulate) {
  const Range range_("pyrecover::rmsnorm_bwd");
  check_dev(dy, "dy");
  TORCH_CHECK(dy.is_contiguous() && h.is_contiguous() && dy.sizes() == h.sizes(), "rmsnorm_bwd: dy/h mismatch");
  const int64_t D = h.size(-1);
  const int64_t rows = h.numel() / D;
  TORCH_CHECK(w.numel() == D && dw.numel() == D && dw.is_contiguous() && rstd.numel() == rows,
              "rmsnorm_bwd: shape mismatch");
  TORCH_CHECK(dw.scalar_type() == h.scalar_type() && dy.scalar_type() == h.scalar_type(), "rmsnorm_bwd: dtype");
  TORCH_CHECK(rstd.scalar_type() == at::kFloat && rstd.is_contiguous(), "rmsnorm_bwd: rstd must be contiguous fp32");
  same_dev(dy, h, "h");
  same_dev(dy, w, "w");
  same_dev(dy, rstd, "rstd");
  same_dev(dy, dw, "dw");
  if (dres.has_value()) same_dev(dy, *dres, "dres");
  const c10::DeviceGuard guard(h.device());
  at::Tensor dx = at::empty_like(h);
  const void* dr = nullptr;
  if (dres.has_value()) {
    TORCH_CHECK(dres->sizes() == h.sizes() && dres->is_contiguous() && dres->scalar_type() == h.scalar_type(),
                "rmsnorm_bwd: dres mismatch");
    dr = dres->data_ptr();
  }
  const int wsr = pra_rmsnorm_bwd_ws_rows((int)rows);
  at::Tensor ws = at::empty({wsr + pra_rmsnorm_bwd_ws_extra(), D}, h.options().dtype(at::kFloat));
  check(pra_rmsnorm_bwd(dt(h), dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), dr, dx.data_ptr(),
                        dw.data_ptr(), ws.data_ptr<float>(), (int)rows, (int)D, accumulate ? 1 : 0, stream_of(h)),
        "rmsnorm_bwd");
  return dx;
}

// LayerNorm: returns (h, y, mean, rstd)
std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& delta, const at::Tensor& w,
                                      const at::Tensor& b, double eps) {
  const Range range_("pyrecover::layernorm_fwd");
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && b.is_contiguous(), "layernorm_fwd: contiguous");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(w.numel() == D && b.numel() == D && w.scalar_type() == x.scalar_type() &&
              b.scalar_type() == x.scalar_type(), "layernorm_fwd: weight/bias mismatch");
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "layernorm_fwd: D must be a multiple of 8 and <= 8192");
  same_dev(x, w, "weight");
  same_dev(x, b, "bias");
  if (delta.has_value()) {
    TORCH_CHECK(delta->sizes() == x.sizes() && delta->is_contiguous() && delta->scalar_type() == x.scalar_type(),
                "layernorm_fwd: delta mismatch");
    same_dev(x, *delta, "delta");
  }
  const c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  at::Tensor h = delta.has_value() ? at::empty_like(x) : x;
  check(pra_layernorm_fwd(dt(x), x.data_ptr(), delta.has_value() ? delta->data_ptr() : nullptr, w.data_ptr(),
                          b.data_ptr(), delta.has_value() ? h.data_ptr() : nullptr, y.data_ptr(), mean.data_ptr<float>(),
                          rstd.data_ptr<float>(), (int)rows, (int)D, (float)eps, stream_of(x)),
        "layernorm_fwd");
  return {h, y, mean, rstd};
}

// dwb: 2*D contiguous output [dw | db]
at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w, const at::Tensor& mean,
                         const at::Tensor& rstd, const c10::optional<at::Tensor>& dres, at::Tensor dwb, bool accumulate) {
  const Range range_("pyrecover::layernorm_bwd");
  check_dev(dy, "dy");
  TORCH_CHECK(dy.is_contiguous() && h.is_contiguous() && dy.sizes() == h.sizes(), "layernorm_bwd: dy/h mismatch");
  const int64_t D = h.size(-1);
  const int64_t rows = h.numel() / D;
  TORCH_CHECK(w.numel() == D && dwb.numel() == 2 * D && dwb.is_contiguous() && rstd.numel() == rows &&
              mean.numel() == rows, "layernorm_bwd: shapes");
  TORCH_CHECK(dwb.scalar_type() == h.scalar_type() && dy.scalar_type() == h.scalar_type() &&
              rstd.scalar_type() == at::kFloat && mean.scalar_type() == at::kFloat, "layernorm_bwd: dtypes");
  for (const at::Tensor& t : {h, w, mean, rstd, dwb}) same_dev(dy, t, "layernorm operand");
  if (dres.has_value()) {
    TORCH_CHECK(dres->sizes() == h.sizes() && dres->is_contiguous() && dres->scalar_type() == h.scalar_type(),
                "layernorm_bwd: dres");
    same_dev(dy, *dres, "dres");
  }
  const c10::DeviceGuard guard(h.device());
  at::Tensor dx = at::empty_like(h);
  const int wsr = pra_rmsnorm_bwd_ws_rows((int)rows);
  at::Tensor ws = at::empty({wsr + pra_rmsnorm_bwd_ws_extra(), 2 * D}, h.options().dtype(at::kFloat));
  check(pra_layernorm_bwd(dt(h), dy.data_ptr(), h.data_ptr(), w.data_ptr(), mean.data_ptr<float>(),
                          rstd.data_ptr<float>(), dres.has_value() ? dres->data_ptr() : nullptr, dx.data_ptr(),
                          dwb.data_ptr(), ws.data_ptr<float>(), (int)rows, (int)D, accumulate ? 1 : 0, stream_of(h)),
        "layernorm_bwd");
  return dx;
}

// In-place RoPE on the first `ncols` columns of each row of a 2-D [tokens, ld] buffer.
void rope_(at::Tensor x2d, int64_t ncols, const at::Tensor& tab, int64_t head_dim, int64_t seq_len,
           int64_t pos_offset, bool inverse) {
  const Range range_("pyrecover::rope");
  check_dev(x2d, "x");
  check_row_major(x2d, "rope x");
  TORCH_CHECK(tab.scalar_type() == at::kFloat && tab.is_contiguous(), "rope: table must be contiguous fp32");
  same_dev(x2d, tab, "rope table");
  TORCH_CHECK(tab.numel() >= (seq_len + pos_offset) * head_dim, "rope: table too small");
  TORCH_CHECK(ncols <= x2d.size(1) && ncols % head_dim == 0 && head_dim % 8 == 0, "rope: bad ncols/head_dim");
  TORCH_CHECK(x2d.size(0) % seq_len == 0, "rope: tokens must be a multiple of seq_len");
  const c10::DeviceGuard guard(x2d.device());
  check(pra_rope(dt(x2d), x2d.data_ptr(), tab.data_ptr(), x2d.size(0), (int)x2d.stride(0), (int)ncols, (int)head_dim,
                 (int)seq_len, (int)pos_offset, inverse ? 1 : 0, stream_of(x2d)),
        "rope");
}

// gu: [T, 2F] (gate | up) -> y [T, F]
at::Tensor swiglu_fwd(const at::Tensor& gu) {
  const Range range_("pyrecover::swiglu_fwd");
  check_dev(gu, "gu");
  check_row_major(gu, "gu");
  TORCH_CHECK(gu.size(1) % 16 == 0, "swiglu: 2F must be a multiple of 16");
  const int64_t F = gu.size(1) / 2;
  const c10::DeviceGuard guard(gu.device());
  at::Tensor y = at::empty({gu.size(0), F}, gu.options());
  const char* base = (const char*)gu.data_ptr();
  check(pra_swiglu_fwd(dt(gu), base, base + F * gu.element_size(), y.data_ptr(), gu.size(0), (int)F,
                       (int)gu.stride(0), (int)gu.stride(0), (int)F, stream_of(gu)),
        "swiglu_fwd");
  return y;
}

// dgu may alias gu (in-place backward).
at::Tensor swiglu_bwd(const at::Tensor& dy, const at::Tensor& gu, c10::optional<at::Tensor> out, int64_t variant) {
  const Range range_("pyrecover::swiglu_bwd");
  check_dev(gu, "gu");
  check_row_major(gu, "gu");
  check_row_major(dy, "dy");
  const int64_t F = gu.size(1) / 2;
  TORCH_CHECK(dy.size(0) == gu.size(0) && dy.size(1) == F && dy.scalar_type() == gu.scalar_type(), "swiglu_bwd: dy");
  same_dev(gu, dy, "dy");
  if (out.has_value()) same_dev(gu, *out, "out");
  const c10::DeviceGuard guard(gu.device());
  at::Tensor dgu = out.has_value() ? *out : at::empty_like(gu);
  TORCH_CHECK(dgu.sizes() == gu.sizes() && dgu.strides() == gu.strides(), "swiglu_bwd: out layout");
  const char* g = (const char*)gu.data_ptr();
  char* o = (char*)dgu.data_ptr();
  const int64_t es = gu.element_size();
  check(pra_swiglu_bwd(dt(gu), dy.data_ptr(), g, g + F * es, o, o + F * es, gu.size(0), (int)F, (int)gu.stride(0),
                       (int)gu.stride(0), (int)dy.stride(0), (int)variant, stream_of(gu)),
        "swiglu_bwd");
  return dgu;
}

// gu: [T, 2F] -> (a [T, F], a^T [F, T]) in one pass (same math as swiglu_fwd).
std::vector<at::Tensor> swiglu_fwd_t(const at::Tensor& gu) {
  const Range range_("pyrecover::swiglu_fwd_t");
  check_dev(gu, "gu");
  check_row_major(gu, "gu");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.element_size() == 2, "swiglu_fwd_t: 16-bit dtype required");
  TORCH_CHECK(T % 64 == 0 && F % 64 == 0 && gu.size(1) == 2 * F, "swiglu_fwd_t: tokens and F must be multiples of 64");
  const c10::DeviceGuard guard(gu.device());
  at::Tensor a = at::empty({T, F}, gu.options());
  at::Tensor aT = at::empty({F, T}, gu.options());
  check(pra_swiglu_fwd_t(dt(gu), gu.data_ptr(), a.data_ptr(), aT.data_ptr(), T, (int)F, (int)gu.stride(0), (int)F,
                         stream_of(gu)),
        "swiglu_fwd_t");
  return {a, aT};
}

// In place: gu <- [dg | du] (the SwiGLU backward, same math as swiglu_bwd); returns dgu^T [2F, T].
at::Tensor swiglu_bwd_t_(const at::Tensor& dy, at::Tensor gu) {
  const Range range_("pyrecover::swiglu_bwd_t");
  check_dev(gu, "gu");
  check_row_major(gu, "gu");
  check_row_major(dy, "dy");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.element_size() == 2, "swiglu_bwd_t: 16-bit dtype required");
  TORCH_CHECK(dy.size(0) == T && dy.size(1) == F && dy.scalar_type() == gu.scalar_type(), "swiglu_bwd_t: dy");
  TORCH_CHECK(T % 64 == 0 && F % 64 == 0, "swiglu_bwd_t: tokens and F must be multiples of 64");
  same_dev(gu, dy, "dy");
  const c10::DeviceGuard guard(gu.device());
  at::Tensor guT = at::empty({2 * F, T}, gu.options());
  check(pra_swiglu_bwd_t(dt(gu), dy.data_ptr(), gu.data_ptr(), guT.data_ptr(), T, (int)F, (int)gu.stride(0),
                         (int)dy.stride(0), stream_of(gu)),
        "swiglu_bwd_t");
  return guT;
}

// In place RoPE (inverse if requested) on the first `nrot` columns of x2d [T, C]; returns x2d^T.
at::Tensor rope_t_(at::Tensor x2d, int64_t nrot, const at::Tensor& tab, int64_t head_dim, int64_t seq_len,
                   bool inverse) {
  const Range range_("pyrecover::rope_t");
  check_dev(x2d, "x");
  check_row_major(x2d, "rope_t x");
  TORCH_CHECK(x2d.element_size() == 2, "rope_t: 16-bit dtype required");
  TORCH_CHECK(tab.scalar_type() == at::kFloat && tab.is_contiguous(), "rope_t: table must be contiguous fp32");
  same_dev(x2d, tab, "rope table");
  TORCH_CHECK(tab.numel() >= seq_len * head_dim, "rope_t: table too small");
  const int64_t T = x2d.size(0), C = x2d.size(1);
  TORCH_CHECK(nrot <= C && nrot % head_dim == 0 && head_dim % 8 == 0, "rope_t: bad nrot/head_dim");
  TORCH_CHECK(T % seq_len == 0 && T % 64 == 0 && C % 64 == 0, "rope_t: shape must tile by 64");
  const c10::DeviceGuard guard(x2d.device());
  at::Tensor xT = at::empty({C, T}, x2d.options());
  check(pra_rope_t(dt(x2d), x2d.data_ptr(), xT.data_ptr(), tab.data_ptr(), T, (int)x2d.stride(0), (int)C, (int)nrot,
                   (int)head_dim, (int)seq_len, inverse ? 1 : 0, stream_of(x2d)),
        "rope_t");
  return xT;
}

at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& W) {
  const Range range_("pyrecover::embedding_fwd");
  check_dev(W, "W");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.device() == W.device(),
              "embedding: ids must be contiguous int64 on the weight's device");
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && W.size(1) % 8 == 0, "embedding: bad weight");
  const c10::DeviceGuard guard(W.device());
  auto sizes = ids.sizes().vec();
  sizes.push_back(W.size(1));
  at::Tensor out = at::empty(sizes, W.options());
  check(pra_embedding_fwd(dt(W), ids.data_ptr<int64_t>(), W.data_ptr(), out.data_ptr(), ids.numel(), (int)W.size(1),
                          W.size(0), stream_of(W)),
        "embedding_fwd");
  return out;
}

// Deterministic dense embedding gradient into dW (overwrites unless accumulate).
void embedding_bwd(const at::Tensor& ids, const at::Tensor& dout, at::Tensor dW, bool accumulate) {
  const Range range_("pyrecover::embedding_bwd");
  check_dev(dW, "dW");
  TORCH_CHECK(dW.is_contiguous() && dout.is_contiguous() && dout.size(-1) == dW.size(1), "embedding_bwd: shapes");
  TORCH_CHECK(dout.numel() / dW.size(1) == ids.numel(), "embedding_bwd: ids/dout mismatch");
  TORCH_CHECK(ids.scalar_type() == at::kLong && dout.scalar_type() == dW.scalar_type(), "embedding_bwd: dtypes");
  same_dev(dW, ids, "ids");
  same_dev(dW, dout, "dout");
  const c10::DeviceGuard guard(dW.device());
  auto flat = ids.reshape({-1});
  auto sorted = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
  at::Tensor sids = std::get<0>(sorted).contiguous();
  at::Tensor perm = std::get<1>(sorted).contiguous();
  if (!accumulate) dW.zero_();
  check(pra_embedding_bwd(dt(dW), sids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dout.data_ptr(), dW.data_ptr(),
                          flat.numel(), (int)dW.size(1), dW.size(0), accumulate ? 1 : 0, stream_of(dW)),
        "embedding_bwd");
}

// logits [T, V] (row stride ld), labels [T] -> (lse [T], loss_row [T], stats [2] = {mean loss, n_valid})
std::vector<at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& labels, int64_t ignore_index) {
  const Range range_("pyrecover::xent_fwd");
  check_dev(logits, "logits");
  check_row_major(logits, "logits");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == logits.size(0),
              "xent: labels must be contiguous int64 [T]");
  same_dev(logits, labels, "labels");
  const c10::DeviceGuard guard(logits.device());
  const int64_t T = logits.size(0);
  auto fo = logits.options().dtype(at::kFloat);
  at::Tensor lse = at::empty({T}, fo), loss_row = at::empty({T}, fo), stats = at::empty({2}, fo);
  check(pra_xent_fwd(dt(logits), logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                     loss_row.data_ptr<float>(), stats.data_ptr<float>(), T, logits.size(1), logits.stride(0),
                     ignore_index, stream_of(logits)),
        "xent_fwd");
  return {lse, loss_row, stats};
}

void xent_bwd_(at::Tensor logits, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& stats,
               const at::Tensor& grad_out, int64_t ignore_index) {
  const Range range_("pyrecover::xent_bwd");
  check_dev(logits, "logits");
  check_row_major(logits, "logits");
  TORCH_CHECK(grad_out.scalar_type() == at::kFloat && grad_out.numel() == 1 && grad_out.is_cuda(),
              "xent_bwd: grad_out must be a 1-element fp32 GPU tensor");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == logits.size(0),
              "xent_bwd: labels");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == logits.size(0) && stats.numel() == 2 &&
              stats.scalar_type() == at::kFloat, "xent_bwd: lse/stats");
  same_dev(logits, labels, "labels");
  same_dev(logits, lse, "lse");
  same_dev(logits, stats, "stats");
  same_dev(logits, grad_out, "grad_out");
  const c10::DeviceGuard guard(logits.device());
  check(pra_xent_bwd(dt(logits), logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                     stats.data_ptr<float>(), grad_out.data_ptr<float>(), logits.size(0), logits.size(1),
                     logits.stride(0), ignore_index, stream_of(logits)),
        "xent_bwd");
}

void adamw_flat_(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, double lr, double b1, double b2,
                 double eps, double wd, double bc1, double bc2_sqrt, double gscale,
                 const c10::optional<at::Tensor>& gscale_dev, const c10::optional<at::Tensor>& hyper_dev, bool fast) {
  const Range range_("pyrecover::adamw_flat");
  check_dev(p, "p");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adamw: contiguous");
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adamw: sizes");
  TORCH_CHECK(g.scalar_type() == p.scalar_type() && m.scalar_type() == v.scalar_type(), "adamw: dtypes");
  same_dev(p, g, "grad");
  same_dev(p, m, "exp_avg");
  same_dev(p, v, "exp_avg_sq");
  const c10::DeviceGuard guard(p.device());
  const float* gsd = nullptr;
  if (gscale_dev.has_value()) {
    TORCH_CHECK(gscale_dev->scalar_type() == at::kFloat && gscale_dev->numel() >= 1, "adamw: gscale_dev fp32");
    same_dev(p, *gscale_dev, "gscale_dev");
    gsd = gscale_dev->data_ptr<float>();
  }
  const double* hyd = nullptr;
  if (hyper_dev.has_value()) {
    TORCH_CHECK(hyper_dev->scalar_type() == at::kDouble && hyper_dev->numel() >= 3, "adamw: hyper_dev fp64[3]");
    same_dev(p, *hyper_dev, "hyper_dev");
    hyd = hyper_dev->data_ptr<double>();
  }
  check(pra_adamw_flat(dt(p), dt(m), p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), lr, b1,
                       b2, eps, wd, bc1, bc2_sqrt, (float)gscale, gsd,
                       hyd, fast ? 1 : 0, stream_of(p)),
        "adamw_flat");
}

// fp32-master AdamW: pm, m, v fp32; p (16-bit) <- round(pm); g has p's dtype.
void adamw_master_(at::Tensor p, at::Tensor pm, const at::Tensor& g, at::Tensor m, at::Tensor v, double lr, double b1,
                   double b2, double eps, double wd, double bc1, double bc2_sqrt, double gscale,
                   const c10::optional<at::Tensor>& gscale_dev, const c10::optional<at::Tensor>& hyper_dev, bool fast) {
  const Range range_("pyrecover::adamw_master");
  check_dev(p, "p");
  TORCH_CHECK(p.is_contiguous() && pm.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(),
              "adamw_master: contiguous");
  TORCH_CHECK(p.numel() == pm.numel() && p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(),
              "adamw_master: sizes");
  TORCH_CHECK(p.element_size() == 2 && g.scalar_type() == p.scalar_type(), "adamw_master: 16-bit p and g");
  TORCH_CHECK(pm.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw_master: fp32 master and moments");
  for (const at::Tensor& t : {pm, g, m, v}) same_dev(p, t, "adamw_master operand");
  const c10::DeviceGuard guard(p.device());
  const float* gsd = nullptr;
  if (gscale_dev.has_value()) {
    TORCH_CHECK(gscale_dev->scalar_type() == at::kFloat && gscale_dev->numel() >= 1, "adamw_master: gscale_dev fp32");
    same_dev(p, *gscale_dev, "gscale_dev");
    gsd = gscale_dev->data_ptr<float>();
  }
  const double* hyd = nullptr;
  if (hyper_dev.has_value()) {
    TORCH_CHECK(hyper_dev->scalar_type() == at::kDouble && hyper_dev->numel() >= 3, "adamw_master: hyper_dev fp64[3]");
    same_dev(p, *hyper_dev, "hyper_dev");
    hyd = hyper_dev->data_ptr<double>();
  }
  check(pra_adamw_master(dt(p), p.data_ptr(), pm.data_ptr<float>(), g.data_ptr(), m.data_ptr<float>(),
                         v.data_ptr<float>(), p.numel(), lr, b1, b2, eps, wd, bc1, bc2_sqrt, (float)gscale, gsd, hyd,
                         fast ? 1 : 0, stream_of(p)),
        "adamw_master");
}

// AdamW of one row-major weight matrix p [rows, cols] that also writes pt = p^T [cols, rows].
void adamw_t_(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, at::Tensor pt, double lr, double b1,
              double b2, double eps, double wd, double bc1, double bc2_sqrt, double gscale,
              const c10::optional<at::Tensor>& gscale_dev, const c10::optional<at::Tensor>& hyper_dev, bool fast) {
  const Range range_("pyrecover::adamw_t");
  check_dev(p, "p");
  TORCH_CHECK(p.dim() == 2 && p.is_contiguous() && g.sizes() == p.sizes() && m.sizes() == p.sizes() &&
                  v.sizes() == p.sizes() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(),
              "adamw_t: p/g/m/v must be contiguous [rows, cols]");
  const int64_t rows = p.size(0), cols = p.size(1);
  TORCH_CHECK(pt.dim() == 2 && pt.size(0) == cols && pt.size(1) == rows && pt.is_contiguous(), "adamw_t: pt [cols, rows]");
  TORCH_CHECK(rows % 64 == 0 && cols % 64 == 0, "adamw_t: rows and cols must be multiples of 64");
  TORCH_CHECK(p.element_size() == 2, "adamw_t: 16-bit parameters required");
  for (const at::Tensor& t : {g, m, v, pt}) {
    same_dev(p, t, "adamw_t operand");
    TORCH_CHECK(t.scalar_type() == p.scalar_type(), "adamw_t: dtypes must match");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "adamw_t: operands must be 16-B aligned");
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0, "adamw_t: p must be 16-B aligned");
  const c10::DeviceGuard guard(p.device());
  const float* gsd = nullptr;
  if (gscale_dev.has_value()) {
    TORCH_CHECK(gscale_dev->scalar_type() == at::kFloat && gscale_dev->numel() >= 1, "adamw_t: gscale_dev fp32");
    same_dev(p, *gscale_dev, "gscale_dev");
    gsd = gscale_dev->data_ptr<float>();
  }
  const double* hyd = nullptr;
  if (hyper_dev.has_value()) {
    TORCH_CHECK(hyper_dev->scalar_type() == at::kDouble && hyper_dev->numel() >= 3, "adamw_t: hyper_dev fp64[3]");
    same_dev(p, *hyper_dev, "hyper_dev");
    hyd = hyper_dev->data_ptr<double>();
  }
  check(pra_adamw_t(dt(p), p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pt.data_ptr(), (int)rows,
                    (int)cols, lr, b1, b2, eps, wd, bc1, bc2_sqrt, (float)gscale, gsd, hyd, fast ? 1 : 0, stream_of(p)),
        "adamw_t");
}

// dst = src^T for a 2-D 16-bit tensor (bf16/fp16) with R, C multiples of 64 (dst: optional
// preallocated [C, R] row-major output).
at::Tensor transpose2d(const at::Tensor& src, c10::optional<at::Tensor> out) {
  const Range range_("pyrecover::transpose2d");
  check_dev(src, "src");
  check_row_major(src, "src");
  TORCH_CHECK(src.element_size() == 2, "transpose2d: 16-bit dtype required");
  const int64_t R = src.size(0), C = src.size(1);
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0 && src.stride(0) % 8 == 0, "transpose2d: R, C must be multiples of 64");
  const c10::DeviceGuard guard(src.device());
  at::Tensor dst;
  if (out.has_value()) {
    dst = *out;
    same_dev(src, dst, "out");
    check_row_major(dst, "out");
    TORCH_CHECK(dst.size(0) == C && dst.size(1) == R && dst.scalar_type() == src.scalar_type() &&
                    dst.stride(0) % 8 == 0,
                "transpose2d: out must be [C, R] of the same dtype");
  } else {
    dst = at::empty({C, R}, src.options());
  }
  check(pra_transpose16(src.data_ptr(), dst.data_ptr(), R, C, src.stride(0), dst.stride(0), stream_of(src)),
        "transpose2d");
  return dst;
}

// CU count of a tensor's device (cached per device)
int device_cus(const at::Tensor& t) {
  static int cached[64] = {0};
  const int d = t.device().index();
  if (d >= 0 && d < 64 && cached[d] > 0) return cached[d];
  int cus = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && cus > 0,
              "pyrecover_amd: device attribute");
  if (d >= 0 && d < 64) cached[d] = cus;
  return cus;
}

// out [M, N] (+)= a^T b with a [K, M], b [K, N] (both row-major, K = tokens): the weight gradient
// dW = dY^T X straight from the activations (no transposed copies), hand-written MFMA kernel.
void wgrad_mm_(const at::Tensor& a, const at::Tensor& b, at::Tensor out, bool accumulate) {
  const Range range_("pyrecover::wgrad_mm");
  check_dev(a, "a");
  check_row_major(a, "a");
  check_row_major(b, "b");
  check_row_major(out, "out");
  same_dev(a, b, "b");
  same_dev(a, out, "out");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && out.size(1) == N, "wgrad_mm: shapes [K,M] x [K,N] -> [M,N]");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.scalar_type() == out.scalar_type() && a.element_size() == 2,
              "wgrad_mm: bf16/fp16 operands of one dtype");
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 32 == 0 && K > 0, "wgrad_mm: M, N % 256 and K % 32");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "wgrad_mm: 16-B rows");
  const c10::DeviceGuard guard(a.device());
  // scratch of the split tail (fp32 partial tiles + tickets), sized exactly for the launcher's
  // split choice, from the caching allocator (graph-capture safe); none when tiles fill whole rounds
  const int cus = device_cus(a);
  const long nws = pra_wgrad_ws_floats((int)M, (int)N, (int)K, cus);
  at::Tensor ws, tickets;
  if (nws > 0) {
    ws = at::empty({(int64_t)nws}, a.options().dtype(at::kFloat));
    tickets = at::empty({(int64_t)pra_wgrad_ticket_count((int)M, (int)N, (int)K, cus)}, a.options().dtype(at::kInt));
  }
  check(pra_wgrad_gemm(dt(a), a.data_ptr(), b.data_ptr(), out.data_ptr(), (int)M, (int)N, (int)K, a.stride(0),
                       b.stride(0), out.stride(0), accumulate ? 1 : 0, ws.defined() ? ws.data_ptr<float>() : nullptr,
                       tickets.defined() ? tickets.data_ptr<int>() : nullptr, cus, stream_of(a)),
        "wgrad_mm");
}

// timing experiments of the weight-gradient kernel (results are garbage; tools/gemm_exp.py)
void wgrad_mm_exp_(const at::Tensor& a, const at::Tensor& b, at::Tensor out, int64_t exp) {
  check_dev(a, "a");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "wgrad_mm_exp: bf16");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && out.size(1) == N, "wgrad_mm_exp: shapes");
  const c10::DeviceGuard guard(a.device());
  check(pra_wgrad_gemm_exp(a.data_ptr(), b.data_ptr(), out.data_ptr(), (int)M, (int)N, (int)K, a.stride(0), b.stride(0),
                           out.stride(0), (int)exp, stream_of(a)),
        "wgrad_mm_exp");
}

// NT GEMM with a fused epilogue (gemm_nt.hip): a [M, K], b [N, K] row-major (K-contiguous).
//   epi 0: out [M, N] = a b^T
//   epi 1: SwiGLU forward, b = W1|W3 [2F, K]: out = gu [M, 2F], out2 = a [M, F]
//   epi 2: SwiGLU backward, b [F, K] (W2^T): da = a b^T is consumed in the epilogue, which
//          overwrites g, u in out = gu [M, 2F] with dg, du
//   epi 3: RoPE on the first nrot columns of out [M, N] (tab float32 [S, D/2, 2])
void gemm_nt_(const at::Tensor& a, const at::Tensor& b, at::Tensor out, int64_t epi,
              const c10::optional<at::Tensor>& out2, const c10::optional<at::Tensor>& tab, int64_t S, int64_t D,
              int64_t nrot) {
  const Range range_("pyrecover::gemm_nt");
  check_dev(a, "a");
  check_row_major(a, "a");
  check_row_major(b, "b");
  check_row_major(out, "out");
  same_dev(a, b, "b");
  same_dev(a, out, "out");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: a [M, K] and b [N, K]");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.scalar_type() == out.scalar_type() && a.element_size() == 2,
              "gemm_nt: bf16/fp16 operands of one dtype");
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 32 == 0 && K > 0, "gemm_nt: M, N % 256 and K % 32");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm_nt: 16-B rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "gemm_nt: 16-B aligned operands (the epilogue stores 16 B per lane)");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm_nt: epi in 0..3");
  int64_t F = 0;
  void* c2 = nullptr;
  int64_t ldc2 = 0;
  const void* tabp = nullptr;
  if (epi == 0 || epi == 3) {
    TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm_nt: out [M, N]");
  }
  if (epi == 1) {
    F = N / 2;
    TORCH_CHECK(N % 2 == 0 && F % 128 == 0, "gemm_nt swiglu: b = W1|W3 [2F, K], F % 128");
    TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm_nt swiglu: gu [M, 2F]");
    TORCH_CHECK(out2.has_value(), "gemm_nt swiglu: needs out2 = a [M, F]");
    check_row_major(*out2, "out2");
    same_dev(a, *out2, "out2");
    TORCH_CHECK(out2->scalar_type() == a.scalar_type() && out2->size(0) == M && out2->size(1) == F &&
                    out2->stride(0) % 8 == 0,
                "gemm_nt swiglu: a [M, F]");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(out2->data_ptr()) % 16 == 0, "gemm_nt swiglu: 16-B aligned out2");
    c2 = out2->data_ptr();
    ldc2 = out2->stride(0);
  }
  if (epi == 2) {
    F = N;
    TORCH_CHECK(out.size(0) == M && out.size(1) == 2 * F, "gemm_nt swiglu bwd: gu [M, 2F] with b [F, K]");
  }
  if (epi == 3) {
    TORCH_CHECK(tab.has_value(), "gemm_nt rope: needs tab");
    same_dev(a, *tab, "tab");
    TORCH_CHECK(tab->scalar_type() == at::kFloat && tab->is_contiguous() && tab->numel() >= S * (D / 2) * 2,
                "gemm_nt rope: tab float32 [>= S, D/2, 2]");
    TORCH_CHECK(S > 0 && D > 0 && D % 8 == 0 && nrot % D == 0 && nrot <= N && M % S == 0,
                "gemm_nt rope: S, D % 8, nrot % D, tokens % S");
    tabp = tab->data_ptr();
  }
  const c10::DeviceGuard guard(a.device());
  const int cus = device_cus(a);
  const long nws = pra_gemm_nt_ws_floats((int)M, (int)N, (int)K, cus);
  at::Tensor ws, tickets;
  // split tail scratch (exactly R * S partial tiles) and the tickets / tile counters, from the
  // caching allocator (graph-safe)
  if (nws > 0) ws = at::empty({(int64_t)nws}, a.options().dtype(at::kFloat));
  const int ntk = pra_gemm_nt_ticket_count((int)M, (int)N, (int)K, cus);
  if (ntk > 0) tickets = at::empty({(int64_t)ntk}, a.options().dtype(at::kInt));
  check(pra_gemm_nt(dt(a), (int)epi, a.data_ptr(), b.data_ptr(), out.data_ptr(), (int)M, (int)N, (int)K, a.stride(0),
                    b.stride(0), out.stride(0), c2, ldc2, (int)F, tabp, (int)S, (int)D, (int)nrot,
                    ws.defined() ? ws.data_ptr<float>() : nullptr, tickets.defined() ? tickets.data_ptr<int>() : nullptr,
                    cus, stream_of(a)),
        "gemm_nt");
}

// returns fp32 [2] = {norm, clip_coef}
at::Tensor grad_norm(const at::Tensor& x, double max_norm, double pre_scale) {
  const Range range_("pyrecover::grad_norm");
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous(), "grad_norm: contiguous");
  const c10::DeviceGuard guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor ws = at::empty({pra_sumsq_partials()}, fo), out = at::empty({2}, fo);
  check(pra_grad_norm(dt(x), x.data_ptr(), x.numel(), ws.data_ptr<float>(), out.data_ptr<float>(), (float)max_norm,
                      (float)pre_scale, stream_of(x)),
        "grad_norm");
  return out;
}

// replica checksum of a contiguous buffer: {fp64 sum of its elements, 64-bit word hash (int64 bits)}
std::vector<at::Tensor> checksum(const at::Tensor& x) {
  const Range range_("pyrecover::checksum");
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous(), "checksum: contiguous");
  const c10::DeviceGuard guard(x.device());
  const int nb = pra_checksum_blocks();
  auto sum = at::empty({1}, x.options().dtype(at::kDouble)), hash = at::empty({1}, x.options().dtype(at::kLong));
  auto ws_s = at::empty({nb}, x.options().dtype(at::kDouble)), ws_h = at::empty({nb}, x.options().dtype(at::kLong));
  check(pra_checksum(dt(x), x.data_ptr(), x.numel() * x.element_size(), ws_s.data_ptr<double>(),
                     reinterpret_cast<unsigned long long*>(ws_h.data_ptr<int64_t>()), sum.data_ptr<double>(),
                     reinterpret_cast<unsigned long long*>(hash.data_ptr<int64_t>()), stream_of(x)),
        "checksum");
  return {sum, hash};
}

// q/k/v/o views [B, S, H, D] with stride(3)==1, stride(2)==D, stride(0)==S*stride(1).
void check_bshd(const at::Tensor& t, const char* name, int64_t B, int64_t S, int64_t H, int64_t D,
                at::ScalarType dtype) {
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == S && t.size(2) == H && t.size(3) == D,
              "attention: ", name, " must be [B, S, H, D] = [", B, ", ", S, ", ", H, ", ", D, "], got ", t.sizes());
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) == D && (B == 1 || S == 1 || t.stride(0) == S * t.stride(1)),
              "attention: ", name, " must have token-major layout with contiguous heads, strides ", t.strides());
  TORCH_CHECK(t.scalar_type() == dtype, "attention: ", name, " must be ", dtype, " like q");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "attention: ", name, " must be 16-B aligned");
}

void check_attn_dtype(const at::Tensor& q) {
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 || q.scalar_type() == at::kHalf || q.scalar_type() == at::kFloat,
              "attention: the HIP kernels take bf16, fp16 or fp32 (got ", q.scalar_type(),
              "); fp64 models run the attention in torch (pyrecover_amd.ops.fused)");
}

// Sequences that do not tile (S % 64 forward, S % 128 backward) run on zero-padded copies of
// length round_up(S, 128). Causal attention is exact on the padding as is: a real query never
// sees a later (padded) key, and padded query rows carry dO = 0, so they add nothing to dK/dV.
// Non-causal attention passes the real length as the key bound `skv` (keys >= skv are masked).
constexpr int64_t kSeqPad = 128;
int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
at::Tensor pad_seq(const at::Tensor& t, int64_t Sp) {
  at::Tensor out = at::zeros({t.size(0), Sp, t.size(2), t.size(3)}, t.options());
  out.narrow(1, 0, t.size(1)).copy_(t);
  return out;
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                 bool causal) {
  const Range range_("pyrecover::attn_fwd");
  check_dev(q, "q");
  check_attn_dtype(q);
  const int64_t B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  check_bshd(q, "q", B, S, Hq, D, q.scalar_type());
  check_bshd(k, "k", B, S, Hkv, D, q.scalar_type());
  check_bshd(v, "v", B, S, Hkv, D, q.scalar_type());
  same_dev(q, k, "k");
  same_dev(q, v, "v");
  TORCH_CHECK(D == 64 || D == 128, "attention: head_dim must be 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "attention: n_heads must be a multiple of n_kv_heads");
  TORCH_CHECK(S > 0 && (S % 64 == 0 || S <= (int64_t)INT32_MAX - kSeqPad), "attention: bad seq_len");
  const c10::DeviceGuard guard(q.device());
  const int64_t fwd_tile = q.scalar_type() == at::kFloat ? 128 : 64;  // fp32 kernel: 128-query blocks
  if (S % fwd_tile) {
    const int64_t Sp = round_up(S, kSeqPad);
    at::Tensor qp = pad_seq(q, Sp), kp = pad_seq(k, Sp), vp = pad_seq(v, Sp);
    at::Tensor o = at::empty({B, Sp, Hq, D}, q.options());
    at::Tensor lse = at::empty({B, Hq, Sp}, q.options().dtype(at::kFloat));
    check(pra_attn_fwd(dt(q), qp.data_ptr(), kp.data_ptr(), vp.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                       (int)B, (int)Sp, (int)Hq, (int)Hkv, (int)D, qp.stride(1), kp.stride(1), vp.stride(1),
                       o.stride(1), (float)scale, causal ? 1 : 0, (int)S, stream_of(q)),
          "attn_fwd");
    return {o.narrow(1, 0, S).contiguous(), lse.narrow(2, 0, S).contiguous()};
  }
  at::Tensor o = at::empty({B, S, Hq, D}, q.options());
  at::Tensor lse = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  check(pra_attn_fwd(dt(q), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), (int)B,
                     (int)S, (int)Hq, (int)Hkv, (int)D, q.stride(1), k.stride(1), v.stride(1), o.stride(1),
                     (float)scale, causal ? 1 : 0, (int)S, stream_of(q)),
        "attn_fwd");
  return {o, lse};
}

// Writes dq/dk/dv into caller-provided [B,S,H,D] views (e.g. slices of a fused dQKV buffer).
void attn_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
              const at::Tensor& dout, const at::Tensor& lse, at::Tensor dq, at::Tensor dk, at::Tensor dv, double scale,
              bool causal, c10::optional<at::Tensor> rope_tab, int64_t mid_event) {
  const Range range_("pyrecover::attn_bwd");
  // mid_event (optional, a torch.cuda.Event's cuda_event handle): recorded on the stream between the
  // dQ and dK/dV kernels, so another stream can start work under the dK/dV kernel
  hipEvent_t mev = reinterpret_cast<hipEvent_t>(mid_event);
  check_dev(q, "q");
  check_attn_dtype(q);
  const int64_t B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  const at::ScalarType ty = q.scalar_type();
  check_bshd(q, "q", B, S, Hq, D, ty);
  check_bshd(k, "k", B, S, Hkv, D, ty);
  check_bshd(v, "v", B, S, Hkv, D, ty);
  check_bshd(o, "o", B, S, Hq, D, ty);
  check_bshd(dout, "dout", B, S, Hq, D, ty);
  check_bshd(dq, "dq", B, S, Hq, D, ty);
  check_bshd(dk, "dk", B, S, Hkv, D, ty);
  check_bshd(dv, "dv", B, S, Hkv, D, ty);
  TORCH_CHECK(D == 64 || D == 128, "attention: head_dim must be 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "attention: n_heads must be a multiple of n_kv_heads");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == B * Hq * S && lse.is_contiguous(), "attention: lse");
  for (const at::Tensor& t : {k, v, o, dout, lse, dq, dk, dv}) same_dev(q, t, "attention operand");
  // optional RoPE table [>= S, D/2, 2] fp32 (cos, sin): dq / dk are stored with the inverse rotation
  const float* rtab = nullptr;
  if (rope_tab.has_value()) {
    TORCH_CHECK(ty != at::kFloat, "attention: the fp32 backward has no fused inverse RoPE (pass rope_tab=None)");
    const at::Tensor& tb = *rope_tab;
    TORCH_CHECK(tb.scalar_type() == at::kFloat && tb.is_contiguous() && tb.numel() >= S * D &&
                    tb.numel() % D == 0, "attention: rope table must be contiguous fp32 [>= S, D/2, 2]");
    same_dev(q, tb, "rope table");
    rtab = tb.data_ptr<float>();
  }
  const c10::DeviceGuard guard(q.device());
  if (S % kSeqPad) {
    const int64_t Sp = round_up(S, kSeqPad);
    at::Tensor qp = pad_seq(q, Sp), kp = pad_seq(k, Sp), vp = pad_seq(v, Sp), op = pad_seq(o, Sp),
               dop = pad_seq(dout, Sp);
    // padded rows: any finite lse (their dO is zero)
    at::Tensor lp = at::zeros({B, Hq, Sp}, lse.options());
    lp.narrow(2, 0, S).copy_(lse.view({B, Hq, S}));
    at::Tensor dqp = at::empty_like(qp), dkp = at::empty_like(kp), dvp = at::empty_like(vp);
    at::Tensor delta = at::empty({pra_attn_bwd_workspace(dt(q), (int)B, (int)Sp, (int)Hq, (int)Hkv, (int)D)},
                                 q.options().dtype(at::kFloat));
    check(pra_attn_bwd(dt(q), qp.data_ptr(), kp.data_ptr(), vp.data_ptr(), op.data_ptr(), dop.data_ptr(),
                       lp.data_ptr<float>(), delta.data_ptr<float>(), dqp.data_ptr(), dkp.data_ptr(), dvp.data_ptr(),
                       (int)B, (int)Sp, (int)Hq, (int)Hkv, (int)D, qp.stride(1), kp.stride(1), vp.stride(1),
                       op.stride(1), dop.stride(1), dqp.stride(1), dkp.stride(1), dvp.stride(1), (float)scale,
                       causal ? 1 : 0, (int)S, rtab, mev, stream_of(q)),
          "attn_bwd");
    dq.copy_(dqp.narrow(1, 0, S));
    dk.copy_(dkp.narrow(1, 0, S));
    dv.copy_(dvp.narrow(1, 0, S));
    return;
  }
  at::Tensor delta = at::empty({pra_attn_bwd_workspace(dt(q), (int)B, (int)S, (int)Hq, (int)Hkv, (int)D)},
                               q.options().dtype(at::kFloat));
  check(pra_attn_bwd(dt(q), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                     lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                     (int)B, (int)S, (int)Hq, (int)Hkv, (int)D, q.stride(1), k.stride(1), v.stride(1), o.stride(1),
                     dout.stride(1), dq.stride(1), dk.stride(1), dv.stride(1), (float)scale, causal ? 1 : 0, (int)S,
                     rtab, mev, stream_of(q)),
        "attn_bwd");
}

}  // namespace

void register_ckpt_engine(pybind11::module& m);  // csrc/runtime/ckpt_engine.cpp
void register_xgmi(pybind11::module& m);         // csrc/dist/xgmi.cpp

PYBIND11_MODULE(_C, m) {
  m.doc() = "pyrecover_amd native ops (HIP/gfx950 kernels + checkpoint engine)";
  m.def("set_roctx", [](bool on) { g_roctx.store(on); });
  m.def("roctx_enabled", []() { return g_roctx.load(); });
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("rope_", &rope_);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd, pybind11::arg("dy"), pybind11::arg("gu"), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("variant") = -1);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd_", &xent_bwd_);
  namespace py = pybind11;
  m.def("adamw_flat_", &adamw_flat_, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lr"),
        py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("bc1"), py::arg("bc2_sqrt"),
        py::arg("gscale"), py::arg("gscale_dev") = py::none(), py::arg("hyper_dev") = py::none(),
        py::arg("fast") = false);
  m.def("adamw_t_", &adamw_t_, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pt"), py::arg("lr"),
        py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("bc1"), py::arg("bc2_sqrt"),
        py::arg("gscale"), py::arg("gscale_dev") = py::none(), py::arg("hyper_dev") = py::none(),
        py::arg("fast") = false);
  m.def("adamw_master_", &adamw_master_, py::arg("p"), py::arg("pm"), py::arg("g"), py::arg("m"), py::arg("v"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("bc1"), py::arg("bc2_sqrt"),
        py::arg("gscale"), py::arg("gscale_dev") = py::none(), py::arg("hyper_dev") = py::none(),
        py::arg("fast") = false);
  m.def("grad_norm", &grad_norm);
  m.def("checksum", &checksum);
  m.def("wgrad_mm_", &wgrad_mm_);
  m.def("wgrad_mm_exp_", &wgrad_mm_exp_);
  m.def("gemm_nt_", &gemm_nt_, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("epi") = 0,
        py::arg("out2") = py::none(), py::arg("tab") = py::none(), py::arg("S") = 0, py::arg("D") = 0,
        py::arg("nrot") = 0);
  m.def("transpose2d", &transpose2d, py::arg("src"), py::arg("out") = py::none());
  m.def("swiglu_bwd_t_", &swiglu_bwd_t_);
  m.def("swiglu_fwd_t", &swiglu_fwd_t);
  m.def("rope_t_", &rope_t_);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd, pybind11::arg("q"), pybind11::arg("k"), pybind11::arg("v"), pybind11::arg("o"),
        pybind11::arg("dout"), pybind11::arg("lse"), pybind11::arg("dq"), pybind11::arg("dk"), pybind11::arg("dv"),
        pybind11::arg("scale"), pybind11::arg("causal"), pybind11::arg("rope_tab") = pybind11::none(),
        pybind11::arg("mid_event") = 0);
  m.def("attn_set_order", [](int fwd, int dq, int dkdv) { pra_attn_set_order(fwd, dq, dkdv); },
        "block order of the attention grids: 0 = heavy tiles first, G > 0 = XCD-grouped with G heads per group, "
        "-1 = by shape", pybind11::arg("fwd"), pybind11::arg("dq"), pybind11::arg("dkdv"));
  m.def("attn_set_options", [](int fwd_pipe, double fwd_thr, int dkdv_impl, int dq_pipe, int dkdv_split, int dkdv_kreg,
                               int bwd_fused, int bwd_window) {
    pra_attn_set_options(fwd_pipe, (float)fwd_thr, dkdv_impl, dq_pipe, dkdv_split, dkdv_kreg, bwd_fused, bwd_window);
  }, "attention kernel selection: fwd_pipe / dkdv_impl / dq_pipe = -1 (by shape), 0 or 1; fwd_thr = rescale "
     "threshold (log2); dkdv_split = -1 (by grid) or query-head splits of the pipelined dK/dV kernel; "
     "dkdv_kreg = 2: ring-staged dK/dV kernel, -2 (default): ring unless a side-stream job waits for the dK/dV window, 1: two-wave dK/dV kernel keeps K in registers, 0: K in LDS; "
     "bwd_fused = -1 (by shape), 0 (split kernels) or 1: fused dQ/dK/dV kernel; bwd_window = 0: side-stream window between dQ and dK/dV, 1: before dQ");
  register_ckpt_engine(m);
  register_xgmi(m);
}

"""The hand-written NT GEMM (csrc/kernels/gemm_nt.hip) and its fused epilogues, on the GPU:

* plain C = A B^T against an fp32 oracle (bf16 and fp16; shapes with a split-K tail; strided
  operands and output), and at the 7B step's production shapes (T = 32768);
* each fused epilogue against the same GEMM followed by the separate kernel it replaces,
  BITWISE: SwiGLU forward (gu and a), SwiGLU backward (dg, du in place over gu), RoPE on q/k;
* deterministic (two launches bitwise equal) and correct under HIP-graph replay.
"""
import pytest
import torch

from pyrecover_amd import _ext

pytestmark = pytest.mark.gpu


def _C():
    return _ext.native()


def _rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).to(dtype)


def _rel_err(out, ref):
    return ((out.float() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(256, 256, 32), (512, 768, 256), (1024, 512, 1056), (512, 512, 4160),
                                   (4096, 4352, 128),  # 272 tiles: split-K tail (S = 2)
                                   (2048, 256 * 33, 96)])
def test_gemm_nt_plain_matches_oracle(cuda, dtype, M, N, K):
    C = _C()
    a, b = _rnd(M, K, dtype=dtype), _rnd(N, K, dtype=dtype)
    out = torch.empty(M, N, device="cuda", dtype=dtype)
    C.gemm_nt_(a, b, out)
    ref = a.double() @ b.double().t()
    assert _rel_err(out, ref.float()) < 8e-3
    out2 = torch.empty_like(out)
    C.gemm_nt_(a, b, out2)
    assert torch.equal(out, out2)  # deterministic (fixed summation order, split tail included)


def test_gemm_nt_strided_operands_and_output(cuda):
    C = _C()
    M, N, K = 512, 512, 256
    abig, bbig = _rnd(M, K + 64), _rnd(N, K + 32)
    a, b = abig[:, 16:16 + K], bbig[:, 8:8 + K]
    obig = torch.zeros(M, N + 256, device="cuda", dtype=torch.bfloat16)
    out = obig[:, 128:128 + N]
    C.gemm_nt_(a, b, out)
    ref = a.float() @ b.float().t()
    assert _rel_err(out, ref) < 8e-3
    assert obig[:, :128].abs().sum().item() == 0 and obig[:, 128 + N:].abs().sum().item() == 0


def test_gemm_nt_rejects_bad_shapes(cuda):
    C = _C()
    a, b = _rnd(300, 64), _rnd(256, 64)
    with pytest.raises(RuntimeError):
        C.gemm_nt_(a, b, torch.empty(300, 256, device="cuda", dtype=torch.bfloat16))
    a, b = _rnd(256, 48), _rnd(256, 48)
    with pytest.raises(RuntimeError):
        C.gemm_nt_(a, b, torch.empty(256, 256, device="cuda", dtype=torch.bfloat16))


@pytest.mark.parametrize("T,F,D", [(512, 384, 256), (4096, 1280, 512), (2048, 128 * 43, 128)])
def test_swiglu_fwd_epilogue_bitwise_vs_unfused(cuda, T, F, D):
    C = _C()
    x, w13 = _rnd(T, D), _rnd(2 * F, D, scale=0.2)
    gu = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    C.gemm_nt_(x, w13, gu, 1, a)
    gu0 = torch.empty_like(gu)
    C.gemm_nt_(x, w13, gu0)
    # the epilogue's a is exactly swiglu_fwd of the gu it stored
    assert torch.equal(a, C.swiglu_fwd(gu))
    if (T // 256) * (2 * F // 256) <= 256:
        assert torch.equal(gu, gu0)  # same tiles' sums, bit for bit
    else:
        # with a split-K tail, gate/up interleaving puts some elements in split tiles in one
        # launch and in whole tiles in the other (fp32 sums in another order): <= 1 bf16 ulp
        assert torch.allclose(gu.float(), gu0.float(), rtol=2 ** -7, atol=1e-6)
    # and the math itself against fp32
    ref = x.float() @ w13.float().t()
    g, u = ref[:, :F].bfloat16().float(), ref[:, F:].bfloat16().float()
    aref = torch.nn.functional.silu(g).bfloat16().float() * u
    assert _rel_err(a, aref) < 2e-2


@pytest.mark.parametrize("T,F,D", [(512, 256, 256), (4096, 768, 512), (2048, 256 * 43, 128)])
def test_swiglu_bwd_epilogue_bitwise_vs_unfused(cuda, T, F, D):
    C = _C()
    dy, w2t = _rnd(T, D), _rnd(F, D, scale=0.2)
    gu = _rnd(T, 2 * F, scale=3.0)
    g1 = gu.clone()
    C.gemm_nt_(dy, w2t, g1, 2)
    da = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    C.gemm_nt_(dy, w2t, da)
    g2 = gu.clone()
    C.swiglu_bwd(da, g2, g2)
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("T,S,nq,nk,D", [(512, 256, 512, 256, 128), (4096, 2048, 1024, 256, 128),
                                         (1024, 512, 512, 512, 64)])
def test_rope_epilogue_bitwise_vs_unfused(cuda, T, S, nq, nk, D):
    from pyrecover_amd.ops.reference import precompute_freqs_cis, rope_table

    C = _C()
    N = nq + 2 * nk
    x, w = _rnd(T, 512), _rnd(N, 512, scale=0.2)
    tab = rope_table(precompute_freqs_cis(D, S, 10000.0)).cuda()
    q1 = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_nt_(x, w, q1, 3, None, tab, S, D, nq + nk)
    q2 = torch.empty_like(q1)
    C.gemm_nt_(x, w, q2)
    C.rope_(q2, nq + nk, tab, D, S, 0, False)
    assert torch.equal(q1, q2)


@pytest.mark.parametrize("K,N", [(4096, 12288), (4096, 22016), (11008, 4096)])
def test_gemm_nt_production_shapes_vs_fp32(cuda, K, N):
    """The 7B step's QKV / W1|W3 forward and W2 forward shapes at T = 32768 tokens."""
    C = _C()
    T = 32768
    x, w = _rnd(T, K), _rnd(N, K, scale=0.05)
    out = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_nt_(x, w, out)
    ref = torch.mm(x.float(), w.float().t())
    err = (out.float() - ref).abs()
    # bf16 output rounding dominates: |err| <= 2^-8 |ref| + a K-dependent fp32 accumulation term
    assert (err <= ref.abs() * 2 ** -8 + 1e-3 * (K / 4096) ** 0.5).all().item()


def test_gemm_nt_split_tail_under_hip_graph(cuda):
    """The split tail's tickets are zeroed by a kernel node: a replayed graph after the inputs
    changed must reduce every split tile again."""
    C = _C()
    M, N, K = 4096, 4352, 256
    a, b = _rnd(M, K), _rnd(N, K)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        C.gemm_nt_(a, b, out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        C.gemm_nt_(a, b, out)
    for _ in range(3):
        a.copy_(_rnd(M, K))
        g.replay()
        torch.cuda.synchronize()
        ref = torch.empty_like(out)
        C.gemm_nt_(a, b, ref)
        assert torch.equal(out, ref)


def test_auto_site_rule_runs_fused_swiglu_from_8192_tokens(cuda, monkeypatch):
    """Default site list: the W1|W3 projection takes the NT kernel with the SwiGLU epilogue from
    NT_AUTO_MIN_TOKENS tokens and NT_AUTO_MIN_K model width (and at least two rounds of 256x256
    tiles), hipBLASLt otherwise; the fused output matches the fp32 oracle."""
    from pyrecover_amd.ops import fused

    monkeypatch.setattr(fused, "GEMM_AUTO", True)
    monkeypatch.setattr(fused, "GEMM_SITES", fused._NT_AUTO)
    D, F, T = fused.NT_AUTO_MIN_K, 128 * 22, fused.NT_AUTO_MIN_TOKENS
    w13 = _rnd(2 * F, D, scale=0.02)
    x = _rnd(T, D)
    assert fused._nt_ok(x, w13, "w13")
    assert not fused._nt_ok(x, w13, "o")  # plain sites stay on the library
    assert not fused._nt_ok(x[: T // 2], w13, "w13")  # too few tokens
    assert not fused._nt_ok(x[:, : D // 4].contiguous(), w13[:, : D // 4].contiguous(), "w13")  # too shallow
    gu = torch.empty(T, 2 * F, dtype=x.dtype, device=x.device)
    a = torch.empty(T, F, dtype=x.dtype, device=x.device)
    _C().gemm_nt_(x, w13, gu, 1, a)
    g, u = (x.float() @ w13.float().t()).split(F, dim=1)
    ref = torch.nn.functional.silu(g) * u
    assert _rel_err(a, ref) < 2e-2

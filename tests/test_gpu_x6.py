"""Split-fp32 ("x6") GEMMs (csrc/abcd_x6.h) are fp32-accurate.

Each fp32 operand is split exactly into three bf16 planes and the six cross
terms with i + j <= 2 run on the bf16 matrix cores with fp32 accumulation;
the dropped terms are below 2^-24 |a||b|.  Here the library's GEMM entry
points, at shapes that dispatch to each x6 kernel (gemm_x6r: frame-streaming,
K <= 160 and K <= 256; gemm_x6f: K > 256; gemm_x6t / gemm_x6s: the K-major
weight-gradient reductions over packed frames, N = 1024 / N = 129), are
bounded against a float64 product: their error may not exceed a small
multiple of the error of torch's own fp32 GEMM on the same operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _err(c, ref):
    return float((c.double() - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("M,N,K", [(32768, 1024, 144), (32768, 512, 256), (16384, 1024, 400)])
def test_x6_frame_gemm_fp32_accurate(M, N, K):
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g) * 0.1
    C = torch.empty(M, N, device="cuda")
    ws = Nn.workspace(64 << 20, "cuda")
    Nn.check(Nn.lib().abcd_gemm_nt(M, N, K, Nn.ptr(A), K, Nn.ptr(B), K, Nn.ptr(C), N, None, Nn.ptr(ws), ws.numel(),
                                   Nn.stream()), "gemm_nt")
    ref = A.double() @ B.double().t()
    e32 = _err(A @ B.t(), ref)
    e6 = _err(C, ref)
    assert e6 <= 4 * e32 + 1e-7, (e6, e32)


@pytest.mark.parametrize("M,N,K,ldb", [(1024, 1024, 20000, 1024), (1024, 129, 20000, 144)])
def test_x6_weight_gradient_gemm_fp32_accurate(M, N, K, ldb):
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(12)
    A = torch.randn(K, M, device="cuda", generator=g)
    Bf = torch.randn(K, ldb, device="cuda", generator=g)
    Bf[:, N:] = 0
    C = torch.empty(M, N, device="cuda")
    ws = Nn.workspace(256 << 20, "cuda")
    Nn.check(Nn.lib().abcd_gemm_tn(M, N, K, Nn.ptr(A), M, Nn.ptr(Bf), ldb, Nn.ptr(C), N, Nn.ptr(ws), ws.numel(),
                                   Nn.stream()), "gemm_tn")
    B = Bf[:, :N]
    ref = A.double().t() @ B.double()
    e32 = _err(A.t() @ B, ref)
    e6 = _err(C, ref)
    assert e6 <= 4 * e32 + 1e-7, (e6, e32)

"""The 320-channel token linear (sdk_token_linear, csrc/token.hip) on the MI355X (run with -m gpu):
out = [res +] x W^T + b — SpatialTransformer.proj_in (reference openai_model/attention.py:293-300) and the
self-attention's to_out + residual (:203-206, :251) — against fp32 torch on the same fp16 inputs and
against the tiled GEMM it replaces (same fp16 rounding points: acc + b, then + res)."""
import math

import pytest
import torch

from gpu_util import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops(sdk):
    from sd_amd import ops as o
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return o


def _case(M, seed, bias=True):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(320, 320, generator=g) / math.sqrt(320)).half()
    b = torch.randn(320, generator=g) * 0.2 if bias else None
    x = torch.randn(M, 320, generator=g).half()
    res = torch.randn(M, 320, generator=g).half()
    return w, b, x, res


@pytest.mark.parametrize("M", [65536, 4096, 32, 1000, 7])
def test_token_linear_vs_fp32(ops, M):
    """The bench row count, full and ragged last blocks (32-token blocks), fewer rows than one block."""
    w, b, x, res = _case(M, M)
    pk = ops.PackedTokenLinear(w, b, torch.device(DEV))
    out = ops.token_linear(pk, x.to(DEV), residual=res.to(DEV))
    ref = x.float() @ w.float().T + b + res.float()
    upd = out.float().cpu() - res.float()
    e = ((upd - (ref - res.float())).norm() / (ref - res.float()).norm()).item()
    print(f"[token_linear] M={M}: update rel-L2 {e:.2e}", flush=True)
    assert out.shape == (M, 320) and out.dtype == torch.float16
    assert e < 2e-3 and rel_l2(out, ref) < 2e-3
    plain = ops.token_linear(pk, x.to(DEV))
    assert rel_l2(plain, x.float() @ w.float().T + b) < 2e-3


def test_token_linear_matches_tiled_gemm(ops):
    """Same fp16 rounding points as ops.linear (the tiled LDS-DMA GEMM): only fp32 summation order differs."""
    M = 65536
    w, b, x, res = _case(M, 3)
    dev = torch.device(DEV)
    pc = ops.PackedConv([(w.float(), 320)], b, device=dev)
    xd, rd = x.to(DEV), res.to(DEV)
    tiled = ops.linear(pc, xd, residual=rd)
    mine = ops.token_linear(ops.PackedTokenLinear(w, b, dev), xd, residual=rd)
    d = (mine.float() - tiled.float()).abs()
    print(f"[token_linear] vs tiled GEMM: max |diff| {d.max().item():.3e}, equal {torch.equal(mine, tiled)}", flush=True)
    assert rel_l2(mine, tiled) < 1e-3


def test_token_linear_in_place_strided_no_bias_deterministic(ops):
    M = 4100
    w, _, x, res = _case(M, 5, bias=False)
    dev = torch.device(DEV)
    pk = ops.PackedTokenLinear(w.reshape(320, 320, 1, 1), None, dev)     # a 1x1 conv weight
    xs = torch.zeros(M, 328, dtype=torch.float16, device=DEV)
    xs[:, :320] = x.to(DEV)
    xv = xs[:, :320]                                                      # row stride 328
    expect = ops.token_linear(pk, xv, residual=res.to(DEV))
    assert rel_l2(expect, x.float() @ w.float().T + res.float()) < 2e-3
    r = res.to(DEV)
    ops.token_linear(pk, xv, residual=r, out=r)                           # x = proj(x') + x in place
    assert torch.equal(r, expect)
    assert torch.equal(ops.token_linear(pk, xv, residual=res.to(DEV)), expect)


def test_token_linear_rejects(ops, sdk):
    from sd_amd import _lib
    assert ops.token_linear_supported(320, 320) and not ops.token_linear_supported(640, 640)
    with pytest.raises(ValueError):
        ops.PackedTokenLinear(torch.zeros(640, 640).half(), None, torch.device(DEV))
    x = torch.zeros(64, 320, dtype=torch.float16, device=DEV)
    a = _lib.TokenLinearArgs()
    a.x, a.w, a.out = x.data_ptr(), x.data_ptr(), x.data_ptr()
    a.x_ld = a.out_ld = 320
    a.rows, a.in_features, a.out_features = 64, 320, 320
    assert _lib.lib().sdk_token_linear(a, None) != 0          # x overlaps out
    a.in_features = a.out_features = 640
    assert _lib.lib().sdk_token_linear(a, None) != 0


@pytest.mark.parametrize("M,with_res", [(65536, False), (1000, True), (7, False)])
def test_token_linear_ln_matches_layer_norm(ops, M, with_res):
    """sdk_token_linear_ln: proj_in + norm1 in one launch.  out is bitwise the plain token linear's, out_ln
    bitwise sdk_layer_norm of that out (the shared quad row math), and both within fp tolerance of fp32."""
    w, b, x, res = _case(M, 11 + M)
    dev = torch.device(DEV)
    g = torch.Generator().manual_seed(M)
    gamma = (1 + 0.1 * torch.randn(320, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(320, generator=g)).to(DEV)
    pk = ops.PackedTokenLinear(w, b, dev)
    xd, rd = x.to(DEV), (res.to(DEV) if with_res else None)
    plain = ops.token_linear(pk, xd, residual=rd)
    out, out_ln = ops.token_linear(pk, xd, residual=rd, norm=(gamma, beta, 1e-5))
    assert torch.equal(out, plain)
    sep = ops.layer_norm(plain, gamma, beta, 1e-5)
    d = (out_ln.float() - sep.float()).abs().max().item()
    print(f"[token_linear_ln] M={M}: max |diff| vs layer_norm {d:.3e}", flush=True)
    assert torch.equal(out_ln, sep)
    ref = torch.nn.functional.layer_norm(plain.float(), (320,), gamma.float(), beta.float(), 1e-5)
    assert rel_l2(out_ln, ref.cpu()) < 2e-3
    # repeated launches are bitwise stable
    for _ in range(3):
        o2, l2 = ops.token_linear(pk, xd, residual=rd, norm=(gamma, beta, 1e-5))
        assert torch.equal(o2, out) and torch.equal(l2, out_ln)


def test_token_linear_ln_rejects_overlap(ops, sdk):
    from sd_amd import _lib
    x = torch.zeros(64, 320, dtype=torch.float16, device=DEV)
    o = torch.zeros(64, 320, dtype=torch.float16, device=DEV)
    gb = torch.ones(320, dtype=torch.float32, device=DEV)
    w = torch.zeros(320, 320, dtype=torch.float16, device=DEV)
    a = _lib.TokenLinearArgs()
    a.x, a.w, a.out = x.data_ptr(), w.data_ptr(), o.data_ptr()
    a.x_ld = a.out_ld = 320
    a.rows, a.in_features, a.out_features = 64, 320, 320
    L = _lib.lib()
    assert L.sdk_token_linear_ln(a, gb.data_ptr(), gb.data_ptr(), 1e-5, o.data_ptr(), 320, None) != 0   # out_ln == out
    assert L.sdk_token_linear_ln(a, gb.data_ptr(), gb.data_ptr(), 1e-5, x.data_ptr(), 320, None) != 0   # out_ln == x
    assert L.sdk_token_linear_ln(a, None, gb.data_ptr(), 1e-5, w.data_ptr(), 320, None) != 0

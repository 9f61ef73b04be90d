"""The fused GEGLU feed-forward (sdk_feed_forward, csrc/ff.hip) on the MI355X (run with -m gpu):
out = res + W2 (a * gelu(g)) + b2, [a | g] = t W1^T + b1 (reference openai_model/attention.py:129-172,
called at :253), against fp32 torch on the same fp16 inputs and against the two-GEMM path it replaces."""
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


def _weights(C, F, seed):
    g = torch.Generator().manual_seed(seed)
    w1 = (torch.randn(2 * F, C, generator=g) / math.sqrt(C)).half()
    b1 = torch.randn(2 * F, generator=g) * 0.2
    w2 = (torch.randn(C, F, generator=g) / math.sqrt(F)).half()
    b2 = torch.randn(C, generator=g) * 0.2
    return w1, b1, w2, b2, g


def _ref(t, w1, b1, w2, b2, res):
    F = w1.shape[0] // 2
    y = t.float() @ w1.float().T + b1
    h = (y[:, :F] * torch.nn.functional.gelu(y[:, F:])).half().float()   # the kernel feeds fp16 h to W2
    out = h @ w2.float().T + b2
    return out + res.float() if res is not None else out


@pytest.mark.parametrize("M,F", [(512, 1280), (300, 1280), (128, 32), (1000, 64)])
def test_feed_forward_vs_fp32(ops, M, F):
    """Full and ragged row counts (the last 128-token block partly outside), one pair of feature blocks."""
    C = 320
    w1, b1, w2, b2, g = _weights(C, F, M + F)
    t = torch.randn(M, C, generator=g).half()
    res = torch.randn(M, C, generator=g).half()
    pf = ops.PackedFF(w1, b1, w2, b2, torch.device(DEV))
    out = ops.feed_forward(pf, t.to(DEV), residual=res.to(DEV))
    ref = _ref(t, w1, b1, w2, b2, res)
    upd = (out.float().cpu() - res.float())
    e = ((upd - (ref - res.float())).norm() / (ref - res.float()).norm()).item()
    print(f"[ff] M={M} F={F}: update rel-L2 {e:.2e}", flush=True)
    assert out.shape == (M, C) and out.dtype == torch.float16
    assert e < 2e-3
    assert rel_l2(out, ref) < 2e-3


def test_feed_forward_matches_two_gemm_path(ops):
    """The SD-1 64x64 block (C = 320, F = 1280): the fused kernel and the GEGLU GEMM + output GEMM
    compute the same fp16 roundings (h, acc + b2, + res) and differ only in fp32 summation order."""
    C, F, M = 320, 1280, 4096
    w1, b1, w2, b2, g = _weights(C, F, 7)
    t = torch.randn(M, C, generator=g).half().to(DEV)
    res = torch.randn(M, C, generator=g).half().to(DEV)
    dev = torch.device(DEV)
    pc1 = ops.PackedConv([(w1.float(), C)], b1, geglu=True, device=dev)
    pc2 = ops.PackedConv([(w2.float(), F)], b2, device=dev)
    two = ops.linear(pc2, ops.linear(pc1, t, out_mode=ops.OUT_GEGLU_F16), residual=res)
    one = ops.feed_forward(ops.PackedFF(w1, b1, w2, b2, dev), t, residual=res)
    d = (one.float() - two.float()).abs()
    print(f"[ff] fused vs two GEMMs: max |diff| {d.max().item():.3e}, rel-L2 {rel_l2(one, two):.2e}", flush=True)
    assert rel_l2(one, two) < 1e-3


def test_feed_forward_no_residual_no_bias_and_in_place(ops):
    C, F, M = 320, 128, 384
    w1, _, w2, _, g = _weights(C, F, 3)
    t = torch.randn(M, C, generator=g).half()
    pf = ops.PackedFF(w1, None, w2, None, torch.device(DEV))
    out = ops.feed_forward(pf, t.to(DEV))
    ref = _ref(t, w1, torch.zeros(2 * F), w2, torch.zeros(C), None)
    assert rel_l2(out, ref) < 2e-3
    # residual and output in one buffer (x = ff(norm3(x)) + x written in place)
    res = torch.randn(M, C, generator=g).half().to(DEV)
    expect = ops.feed_forward(pf, t.to(DEV), residual=res.clone())
    ops.feed_forward(pf, t.to(DEV), residual=res, out=res)
    assert torch.equal(res, expect)


def test_feed_forward_deterministic(ops):
    C, F, M = 320, 1280, 2048
    w1, b1, w2, b2, g = _weights(C, F, 11)
    t = torch.randn(M, C, generator=g).half().to(DEV)
    res = torch.randn(M, C, generator=g).half().to(DEV)
    pf = ops.PackedFF(w1, b1, w2, b2, torch.device(DEV))
    a = ops.feed_forward(pf, t, residual=res)
    b = ops.feed_forward(pf, t, residual=res)
    assert torch.equal(a, b)


def test_feed_forward_rejects(ops, sdk):
    from sd_amd import _lib
    assert not ops.ff_supported(640, 2560) and not ops.ff_supported(320, 1288) and ops.ff_supported(320, 1280)
    with pytest.raises(ValueError):
        ops.PackedFF(torch.zeros(5120, 640).half(), None, torch.zeros(640, 2560).half(), None, torch.device(DEV))
    a = _lib.FfArgs()
    a.rows, a.channels, a.features = 128, 640, 2560
    assert _lib.lib().sdk_feed_forward(a, None) != 0

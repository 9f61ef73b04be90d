"""The reassociated cross-attention (openai_model/attention.py ReassocContext) is the reference's
CrossAttention math (openai_model/attention.py:96-117: q = t Wq^T, softmax(scale q_h K_h^T) V_h, o Wo^T + b)
regrouped: fp32 identity on the CPU, plus the GPU kernels it runs on (segment softmax, per-image
weights) — the latter in tests/test_gpu_reassoc.py."""
import torch

import sd_amd_loader

sd_amd_loader.load()
from sd_amd.openai_model.attention import _reassoc_applies, reassoc_weights  # noqa: E402


def _reference_block(t, k, v, wq, wo, bo, scale):
    B, L, H, d = k.shape
    N = t.shape[1]
    q = (t @ wq.T).view(B, N, H, d)
    s = torch.einsum("bnhe,bjhe->bhnj", q, k) * scale
    o = torch.einsum("bhnj,bjhe->bnhe", s.softmax(-1), v).reshape(B, N, H * d)
    return o @ wo.T + bo


def _reassociated_block(t, k, v, wq, wo, bo, scale):
    B, L, H, d = k.shape
    w1, w2 = reassoc_weights(k, v, wq, wo)
    s = torch.einsum("bnc,bkc->bnk", t, w1) * scale                       # [B, N, H*L]
    p = s.view(B, -1, H, L).softmax(-1).reshape(B, -1, H * L)           # per-head segments
    return torch.einsum("bnk,bck->bnc", p, w2) + bo


def test_reassociation_is_the_reference_math_fp32():
    g = torch.Generator().manual_seed(3)
    B, N, C, H, d, L = 2, 24, 64, 4, 16, 7
    t = torch.randn(B, N, C, generator=g, dtype=torch.float64)
    k = torch.randn(B, L, H, d, generator=g, dtype=torch.float64)
    v = torch.randn(B, L, H, d, generator=g, dtype=torch.float64)
    wq = torch.randn(H * d, C, generator=g, dtype=torch.float64) / C ** 0.5
    wo = torch.randn(C, H * d, generator=g, dtype=torch.float64) / (H * d) ** 0.5
    bo = torch.randn(C, generator=g, dtype=torch.float64)
    ref = _reference_block(t, k, v, wq, wo, bo, d ** -0.5)
    got = _reassociated_block(t, k, v, wq, wo, bo, d ** -0.5)
    assert torch.allclose(got, ref, rtol=1e-10, atol=1e-10)


def test_reassociation_applies_where_it_saves_flops():
    # SD-1: 8 heads x 77 keys -> 640 columns vs 1280 channels (2.1x fewer FLOPs); not at 640 / 320, not
    # SD-2's 20 heads x 64 at 1280 (1540 columns)
    assert _reassoc_applies(1280, 8, 77)
    assert not _reassoc_applies(640, 8, 77)
    assert not _reassoc_applies(320, 8, 77)
    assert not _reassoc_applies(1280, 20, 77)

"""Tile visiting order of unsplit conv plans (sdk_conv_args.tile_group_m, conv.hip item_coords): the order
only changes which workgroup computes which tile, so every grouping — M-panel major, groups of 8 / 16
panels, and a group size that leaves a short last group — gives bitwise the same output, GroupNorm
statistics included.  Shapes: the 32² GEGLU FF1 GEMM (reference openai_model/attention.py:129-141) and a 64²
ResBlock 3x3 conv on the zero-bordered GroupNorm output (openai_model/model.py:181-207).  Run with -m gpu."""
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
    yield o
    o.TILE_GROUP_M = None


def _rand(*shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).half()


@pytest.mark.parametrize("variant", (20, 8, 2, 22))
def test_geglu_gemm_order_invariant(ops, variant):
    M, K, N = 16384, 640, 5120
    x = _rand(M, K, seed=1).to(DEV)
    w = torch.randn(N, K, generator=torch.Generator().manual_seed(2)) / math.sqrt(K)
    b = torch.randn(N, generator=torch.Generator().manual_seed(3)) * 0.1
    pc = ops.PackedConv([(w, K)], b, geglu=True, device=DEV)
    outs = {}
    for gm in (1, 8, 16, 3):
        ops.TILE_GROUP_M = gm
        try:
            outs[gm] = ops.conv2d(pc, x.view(1, M, 1, K), ksize=1, pad=0, out_mode=ops.OUT_GEGLU_F16,
                                  variant=variant, split_k=1).view(M, N // 2)
        except RuntimeError:
            pytest.skip(f"variant {variant} has no GEGLU plan here")
    ops.TILE_GROUP_M = None
    for gm in (8, 16, 3):
        assert torch.equal(outs[gm], outs[1]), f"gm {gm}"
    xf = x[:2048].float().cpu()
    h = xf @ w.half().float().T + b
    a, g = h[:, :N // 2], h[:, N // 2:]
    ref = a * torch.nn.functional.gelu(g)
    assert rel_l2(outs[1][:2048], ref) < 3e-3


@pytest.mark.parametrize("variant", (22, 24))
def test_conv3x3_order_invariant_with_gn_stats(ops, variant):
    B, H, W, Ci, Co = 16, 64, 64, 320, 320
    x = _rand(B, H + 2, W + 2, Ci, seed=4).to(DEV)
    g = torch.Generator().manual_seed(5)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)
    pc = ops.PackedConv([(w, Ci)], torch.randn(Co, generator=g), device=DEV)
    res = _rand(B, H, W, Co, seed=6).to(DEV)
    outs = {}
    for gm in (1, 8, 5):
        ops.TILE_GROUP_M = gm
        outs[gm] = ops.conv2d(pc, x, pad=0, residual=res, variant=variant, split_k=1, gn_stats=True)
    ops.TILE_GROUP_M = None
    for gm in (8, 5):
        assert torch.equal(outs[gm], outs[1]), f"gm {gm}"
        p1, pg = getattr(outs[1], ops.GN_ATTR, None), getattr(outs[gm], ops.GN_ATTR, None)
        assert p1 is not None and pg is not None
        assert torch.equal(p1[0], pg[0])

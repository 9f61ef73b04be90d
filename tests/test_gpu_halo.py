"""Halo-tile 3x3 conv (conv.hip conv_halo_kernel, variants 36 / 37) on the MI355X (run with -m gpu).

The halo kernel stages the padded input rows of a tile once per 64-channel block and forms the nine
taps from LDS; its K order, wave tiling and MFMA shape equal the LDS-DMA configs 22 (256x320) and
23 (128x320), so its outputs must be BITWISE equal to theirs, and within the fp16 tolerance of an
fp32 conv of the same fp16 inputs (rel-L2 <= 2e-3).  Shapes cover the SD levels (64x64, 32x32,
16x16 single-image tiles; 8x8 multi-image tiles), split-K on channel-block boundaries, a ragged last
tile (batch not a multiple of the images per tile), a 2-source concat, the embedding row, the
residual and the GroupNorm statistics emitted by the epilogue."""
import math

import pytest
import torch
import torch.nn.functional as F

from gpu_util import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TWIN = {36: 22, 37: 23}


@pytest.fixture(scope="module")
def ops(sdk):
    from sd_amd import ops as o
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return o


def _rand(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).half()


def _ran(ops, fn):
    """(result, variant the plan ran) of one conv call."""
    ops.PROFILER.start()
    try:
        y = fn()
    finally:
        ops.PROFILER.stop()
    return y, ops.PROFILER.records[-1][1]


def _padded(x):
    return F.pad(x.float().permute(0, 3, 1, 2), (1, 1, 1, 1)).permute(0, 2, 3, 1).half().contiguous()


@pytest.mark.parametrize("variant", [36, 37])
@pytest.mark.parametrize("B,H,W,Ci,Co,split", [
    (2, 64, 64, 320, 320, 1),       # SD 64x64 level
    (2, 32, 32, 640, 640, 1),       # 32x32
    (2, 16, 16, 1280, 1280, 4),     # 16x16, split-K over channel blocks
    (3, 8, 8, 128, 320, 1),         # multi-image tiles, ragged last tile
    (1, 16, 16, 128, 320, 2),       # one channel block per split
    (2, 48, 48, 192, 320, 1),       # C5-shaped level (tiles not row-aligned)
])
def test_halo_conv_matches_twin_and_fp32(ops, variant, B, H, W, Ci, Co, split):
    x = _rand(B, H, W, Ci, seed=H + Ci)
    w = torch.randn(Co, Ci, 3, 3, generator=torch.Generator().manual_seed(Co)) / math.sqrt(Ci * 9)
    b = torch.randn(Co, generator=torch.Generator().manual_seed(Co + 1)) * 0.1
    pc = ops.PackedConv([(w, Ci)], b, device=DEV)
    xp = _padded(x).to(DEV)
    y, ran = _ran(ops, lambda: ops.conv2d(pc, xp, pad=0, variant=variant, split_k=split))
    if ran != variant:
        assert (variant, H) == (36, 8), "the halo plan should exist for this shape"
        pytest.skip("4 images per 256-pixel tile overflow the ring: the planner runs")
    yt = ops.conv2d(pc, xp, pad=0, variant=TWIN[variant], split_k=split)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float(), b, padding=1).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert rel_l2(y, ref) < 2e-3
    assert torch.equal(y, yt), f"variant {variant} differs from its LDS-DMA twin {TWIN[variant]}"


@pytest.mark.parametrize("variant", [36, 37])
def test_halo_plan_is_taken(ops, variant):
    """The plan really runs the halo kernel (not a fallback) on an applicable shape, and falls back
    to the planner on one it cannot take (a masked pad-1 conv)."""
    x = _rand(2, 16, 16, 64, seed=5)
    w = torch.randn(320, 64, 3, 3) / 24
    pc = ops.PackedConv([(w, 64)], None, device=DEV)
    _, r0 = _ran(ops, lambda: ops.conv2d(pc, _padded(x).to(DEV), pad=0, variant=variant))
    _, r1 = _ran(ops, lambda: ops.conv2d(pc, x.to(DEV), pad=1, variant=variant))
    assert r0 == variant and r1 != variant


@pytest.mark.parametrize("variant", [36, 37])
def test_halo_concat_rowbias_residual_gn_stats(ops, variant):
    """Two-source concat input (c_split a multiple of 64), the per-image embedding row, the residual
    add and the emitted GroupNorm statistics — the ResBlock conv's full epilogue."""
    B, H, W, C1, C2, Co = 2, 32, 32, 128, 192, 320
    a, c = _rand(B, H, W, C1, seed=7), _rand(B, H, W, C2, seed=8)
    ap, cp = _padded(a).to(DEV), _padded(c).to(DEV)
    g = torch.Generator().manual_seed(11)
    w = torch.randn(Co, C1 + C2, 3, 3, generator=g) / math.sqrt((C1 + C2) * 9)
    b = torch.randn(Co, generator=g) * 2 + 3
    emb = torch.randn(B, Co + 8, generator=g)
    res = _rand(B, H, W, Co, seed=9)
    pc = ops.PackedConv([(w, C1 + C2)], b, device=DEV)
    kw = dict(pad=0, row_bias=(emb.to(DEV), 8), residual=res.to(DEV), gn_stats=True, split_k=1)
    y, ran = _ran(ops, lambda: ops.conv2d(pc, (ap, cp), variant=variant, **kw))
    assert ran == variant
    yt = ops.conv2d(pc, (ap, cp), variant=TWIN[variant], **kw)
    xcat = torch.cat([a, c], -1).float().permute(0, 3, 1, 2)
    ref = F.conv2d(xcat, w.half().float(), b, padding=1).permute(0, 2, 3, 1) + emb[:, None, None, 8:] + res.float()
    assert rel_l2(y, ref) < 3e-3
    assert torch.equal(y, yt)
    pp, nch, _ = getattr(y, ops.GN_ATTR)
    pt, ncht, _ = getattr(yt, ops.GN_ATTR)
    assert nch == ncht and torch.equal(pp, pt)


@pytest.mark.parametrize("variant", [36, 37])
@pytest.mark.parametrize("B,H,W,C0,C1,C2,Co,split", [
    (2, 32, 32, 320, 320, 320, 320, 1),      # decoder ResBlock conv2 + 1x1 over the concat input
    (2, 16, 16, 640, 640, 320, 640, 1),
    (1, 16, 16, 640, 1280, 0, 640, 3),       # split-K: splits start in the 3x3 and in the 1x1 segment
    (3, 8, 8, 128, 192, 64, 320, 2),         # multi-image tiles
])
def test_halo_fused_shortcut_segment(ops, variant, B, H, W, C0, C1, C2, Co, split):
    """ResBlock conv2 with the nin_shortcut folded in as a second K segment (a plain 1x1 over the raw,
    possibly concatenated block input): its A tiles are staged in the idle halo ring after the 3x3 K-steps."""
    h = _rand(B, H, W, C0, seed=21)
    a = _rand(B, H, W, C1, seed=22)
    c = _rand(B, H, W, C2, seed=23) if C2 else None
    g = torch.Generator().manual_seed(24)
    w2 = torch.randn(Co, C0, 3, 3, generator=g) / math.sqrt(C0 * 9)
    ws = torch.randn(Co, C1 + C2, 1, 1, generator=g) / math.sqrt(C1 + C2)
    b = torch.randn(Co, generator=g) * 0.1
    res_src = (a.to(DEV), c.to(DEV)) if C2 else a.to(DEV)
    pc = ops.PackedConv([(w2, C0), (ws, C1 + C2)], b, device=DEV)
    hp = _padded(h).to(DEV)
    y, ran = _ran(ops, lambda: ops.conv2d(pc, hp, pad=0, seg2=(res_src, None, False), variant=variant, split_k=split))
    if ran != variant:
        assert (variant, H) == (36, 8), "the halo plan should exist for this shape"
        pytest.skip("4 images per 256-pixel tile overflow the ring: the planner runs")
    xin = torch.cat([a, c], -1) if C2 else a
    ref = (F.conv2d(h.float().permute(0, 3, 1, 2), w2.half().float(), b, padding=1) +
           F.conv2d(xin.float().permute(0, 3, 1, 2), ws.half().float())).permute(0, 2, 3, 1)
    assert rel_l2(y, ref) < 2e-3
    if split == 1:
        yt = ops.conv2d(pc, hp, pad=0, seg2=(res_src, None, False), variant=TWIN[variant], split_k=1)
        assert torch.equal(y, yt)


@pytest.mark.parametrize("variant", [36, 37])
@pytest.mark.parametrize("B,H,W,C0,C1,Co,split,skip", [
    (2, 64, 64, 320, 0, 320, 1, None),          # ResBlock conv1 at the 64x64 level
    (2, 32, 32, 320, 320, 640, 1, None),        # decoder conv1 over a 2-source concat
    (2, 32, 32, 640, 0, 640, 1, "residual"),    # conv2 + identity skip
    (2, 32, 32, 640, 0, 640, 1, "fused"),       # conv2 + nin_shortcut as a second K segment
    (1, 16, 16, 1280, 0, 1280, 4, None),        # 16x16 level, split-K on channel blocks
    (1, 48, 48, 320, 0, 320, 1, None),          # tiles not row-aligned (C5-shaped level)
])
def test_halo_groupnorm_fused_equals_materialised(ops, variant, B, H, W, C0, C1, Co, split, skip):
    """GroupNorm + SiLU applied by the halo kernel to its own staged input (raw input, pad 1, virtual zero
    border) equals the conv over the materialised zero-bordered GN output (sdk_group_norm_apply_padded,
    pad 0) BIT FOR BIT — the same transform arithmetic, the same K order — with the embedding row, the
    residual / fused shortcut and the emitted statistics; and matches an fp32 reference."""
    g = torch.Generator().manual_seed(B * 131 + H + C0 + C1)
    a = (torch.randn(B, H, W, C0, generator=g) * 2 + 0.5).half()
    c = (torch.randn(B, H, W, C1, generator=g) - 1).half() if C1 else None
    src = (a.to(DEV), c.to(DEV)) if C1 else a.to(DEV)
    Ci = C0 + C1
    gamma = (torch.rand(Ci, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(Ci, generator=g) * 0.2).to(DEV)
    sc, sh = ops.group_norm_affine(src, gamma, beta, 1e-5, 32)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)
    b = torch.randn(Co, generator=g) * 0.1
    emb = torch.randn(B, Co, generator=g)
    segs, kw = [(w, Ci)], dict(row_bias=(emb.to(DEV), 0), gn_stats=True, split_k=split)
    xin = torch.cat([a, c], -1) if C1 else a
    if skip == "residual":
        res = _rand(B, H, W, Co, seed=3)
        kw["residual"] = res.to(DEV)
    elif skip == "fused":
        s_in = _rand(B, H, W, 192, seed=4)
        ws = torch.randn(Co, 192, 1, 1, generator=g) / math.sqrt(192)
        segs.append((ws, 192))
        kw["seg2"] = (s_in.to(DEV), None, False)
    pc = ops.PackedConv(segs, b, device=DEV)
    y, ran = _ran(ops, lambda: ops.conv2d(pc, src, pad=1, gn=(sc, sh), silu=True, variant=variant, **kw))
    assert ran == variant, "the GroupNorm-fused halo plan should exist for this shape"
    xa = ops.group_norm_apply(src, (sc, sh), silu=True, pad=1)
    ym, ranm = _ran(ops, lambda: ops.conv2d(pc, xa, pad=0, variant=variant, **kw))
    assert ranm == variant
    assert torch.equal(y, ym), "fused GroupNorm differs from the materialised one"
    pp, nch, _ = getattr(y, ops.GN_ATTR)
    pm, nchm, _ = getattr(ym, ops.GN_ATTR)
    assert nch == nchm and torch.equal(pp, pm)
    # fp32 reference of the whole block
    xr = xin.float().permute(0, 3, 1, 2)
    xn = F.silu(F.group_norm(xr, 32, gamma.cpu(), beta.cpu(), 1e-5)).half().float()
    ref = F.conv2d(xn, w.half().float(), b, padding=1).permute(0, 2, 3, 1) + emb[:, None, None, :]
    if skip == "residual":
        ref = ref + res.float()
    elif skip == "fused":
        ref = ref + F.conv2d(s_in.float().permute(0, 3, 1, 2), ws.half().float()).permute(0, 2, 3, 1)
    assert rel_l2(y, ref) < 3e-3


def test_groupnorm_finalize_from_producer_statistics(ops):
    """sdk_group_norm_finalize from the statistics a producing conv emitted equals the statistics pass."""
    g = torch.Generator().manual_seed(77)
    x = _rand(2, 32, 32, 128, seed=8)
    w = torch.randn(320, 128, 3, 3, generator=g) / math.sqrt(128 * 9)
    pc = ops.PackedConv([(w, 128)], torch.randn(320, generator=g) + 1, device=DEV)
    y = ops.conv2d(pc, _padded(x).to(DEV), pad=0, gn_stats=True, variant=36)
    assert getattr(y, ops.GN_ATTR, None) is not None
    gamma = (torch.rand(320, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(320, generator=g) * 0.1).to(DEV)
    s1, t1 = ops.group_norm_scale_shift(y, gamma, beta, 1e-5, 32)
    s0, t0 = ops.group_norm_affine(y.clone(), gamma, beta, 1e-5, 32)
    assert rel_l2(s1, s0) < 1e-5 and rel_l2(t1, t0) < 1e-5


@pytest.mark.parametrize("variant", [22, 23, 5, 7])
@pytest.mark.parametrize("B,H,W,C0,C1,C2,Co,split", [
    (2, 32, 32, 320, 320, 320, 320, 1),      # decoder ResBlock conv2 + 1x1 over a two-source concat
    (1, 16, 16, 640, 1280, 0, 640, 3),       # split-K: splits start in the 3x3 and in the 1x1 segment
    (2, 16, 16, 640, 640, 640, 1280, 2),
])
def test_lds_dma_fused_shortcut_segment_linear_issue(ops, variant, B, H, W, C0, C1, C2, Co, split):
    """The LDS-DMA tile kernels on the same two-segment convs (their linear A issue, conv.hip SIMPLE = 2: three
    per-lane row offsets, the K step's segment / source / tap offset in the scalar soffset) vs fp32, at split 1
    and with splits that start in either segment (bitwise equality with the halo kernel at split 1:
    test_halo_fused_shortcut_segment)."""
    h = _rand(B, H, W, C0, seed=31)
    a = _rand(B, H, W, C1, seed=32)
    c = _rand(B, H, W, C2, seed=33) if C2 else None
    g = torch.Generator().manual_seed(34)
    w2 = torch.randn(Co, C0, 3, 3, generator=g) / math.sqrt(C0 * 9)
    ws = torch.randn(Co, C1 + C2, 1, 1, generator=g) / math.sqrt(C1 + C2)
    b = torch.randn(Co, generator=g) * 0.1
    res_src = (a.to(DEV), c.to(DEV)) if C2 else a.to(DEV)
    pc = ops.PackedConv([(w2, C0), (ws, C1 + C2)], b, device=DEV)
    hp = _padded(h).to(DEV)
    y, ran = _ran(ops, lambda: ops.conv2d(pc, hp, pad=0, seg2=(res_src, None, False), variant=variant, split_k=split))
    assert ran == variant
    xin = torch.cat([a, c], -1) if C2 else a
    ref = (F.conv2d(h.float().permute(0, 3, 1, 2), w2.half().float(), b, padding=1) +
           F.conv2d(xin.float().permute(0, 3, 1, 2), ws.half().float())).permute(0, 2, 3, 1)
    assert rel_l2(y, ref) < 2e-3

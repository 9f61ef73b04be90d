"""In-launch split-K of the LDS-DMA conv / GEMM kernels (sdk_conv_args.split_inlaunch, conv.hip
conv_glds_kernel): the two K halves of a tile combine inside the launch — the second workgroup to arrive adds
the first's fp32 accumulator blob and runs the whole epilogue — instead of fp32 slabs + splitk_reduce.  The
combine adds the same two partial sums in the same order as the slab reduce, so the outputs are bitwise the
split-2 slab path's; against fp32 they are within the usual GEMM tolerance.  Shapes: the 16x16-level
projections (reference openai_model/attention.py:293-300 proj_in, :203-206 to_out) and a 3x3 ResBlock conv
(openai_model/model.py:181-207) that emits GroupNorm statistics.  Run with -m gpu."""
import math

import pytest
import torch

from gpu_util import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TILE_VARIANTS = (2, 3, 4, 6, 7, 16, 17, 18, 19, 22, 23, 24, 25, 26, 31, 32, 33)


@pytest.fixture(scope="module")
def ops(sdk):
    from sd_amd import ops as o
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return o


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).half()


@pytest.mark.parametrize("variant", TILE_VARIANTS)
def test_inlaunch_token_gemm_equals_slab_split(ops, variant):
    """4096 x 1280 x 1280 with bias + residual (the 16x16-level projection): in-launch == split-2 slabs
    bitwise, within 3e-3 of fp32, deterministic, and the arrival counters are left zero."""
    M, K, N = 4096, 1280, 1280
    x = _rand(M, K, seed=1)
    w = torch.randn(N, K, generator=torch.Generator().manual_seed(2)) / math.sqrt(K)
    b = torch.randn(N, generator=torch.Generator().manual_seed(3)) * 0.1
    r = _rand(M, N, seed=4)
    pc = ops.PackedConv([(w, K)], b, device=DEV)
    x4, r4 = x.to(DEV).view(1, M, 1, K), r.to(DEV).view(1, M, 1, N)
    run = lambda sp: ops.conv2d(pc, x4, ksize=1, pad=0, residual=r4, variant=variant, split_k=sp).view(M, N)
    y_in = run(-2)
    y_slab = run(2)
    ref = x.float() @ w.half().float().T + b
    assert rel_l2(y_in, ref + r.float()) < 3e-3
    d = (y_in.float() - y_slab.float()).abs().max().item()
    print(f"[inlaunch] variant {variant}: max |in-launch - slab| {d:.3e}", flush=True)
    assert torch.equal(y_in, y_slab)
    for _ in range(3):
        assert torch.equal(run(-2), y_in)
    torch.cuda.synchronize()
    assert int(ops.WORKSPACE.counters(DEV).abs().sum().item()) == 0


@pytest.mark.parametrize("variant", (2, 7, 22, 23, 19, 25))
def test_inlaunch_conv3x3_group_norm_statistics(ops, variant):
    """A 16x16 ResBlock 3x3 conv (640 -> 1280, bias + embedding row + residual) combined in-launch emits its
    GroupNorm statistics per M-tile like an unsplit tile; group_norm from them equals a statistics pass."""
    B, H, W, Ci, Co = 16, 16, 16, 640, 1280
    x = _rand(B, H, W, Ci, seed=5)
    g = torch.Generator().manual_seed(6)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)
    bias = torch.randn(Co, generator=g) * 2 + 3
    emb = torch.randn(B, Co + 16, generator=g)
    res = _rand(B, H, W, Co, seed=7)
    pc = ops.PackedConv([(w, Ci)], bias, device=DEV)
    kw = dict(residual=res.to(DEV), row_bias=(emb.to(DEV), 16), gn_stats=True, variant=variant)
    y = ops.conv2d(pc, x.to(DEV), split_k=-2, **kw)
    y2 = ops.conv2d(pc, x.to(DEV), split_k=2, **kw)
    assert torch.equal(y, y2)
    xr = x.float().permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xr, w.half().float(), bias, padding=1).permute(0, 2, 3, 1)
    ref = ref + emb[:, None, None, 16:] + res.float()
    assert rel_l2(y, ref) < 3e-3
    part = getattr(y, ops.GN_ATTR, None)
    assert part is not None, "the in-launch combine emits GroupNorm statistics"
    pp, nch, _ = part
    t = y.double().reshape(B, nch, H * W // nch, Co)
    mean = t.mean(2)
    m2 = ((t - mean[:, :, None]) ** 2).sum(2)
    assert torch.allclose(pp[..., 0].double(), mean, rtol=1e-5, atol=1e-4)
    assert rel_l2(pp[..., 1].double(), m2) < 1e-4
    gamma = torch.rand(Co, generator=g).to(DEV) + 0.5
    beta = (torch.randn(Co, generator=g) * 0.1).to(DEV)
    g1 = ops.group_norm(y, gamma, beta, 1e-5, 32, silu=True, pad=1)
    g0 = ops.group_norm(y.clone(), gamma, beta, 1e-5, 32, silu=True, pad=1)
    assert rel_l2(g1, g0) < 1e-3


def test_inlaunch_rows_f32_and_graph_replay(ops):
    """fp32 row output (the reassociated cross-attention's score GEMM mode) and HIP-graph capture / replay of
    an in-launch conv: the counters return to zero every replay, so replays equal the eager result."""
    M, K, N = 4096, 1280, 640
    x = _rand(M, K, seed=8).to(DEV)
    w = torch.randn(N, K, generator=torch.Generator().manual_seed(9)) / math.sqrt(K)
    pc = ops.PackedConv([(w, K)], None, device=DEV)
    run = lambda: ops.conv2d(pc, x.view(1, M, 1, K), ksize=1, pad=0, out_mode=ops.OUT_ROWS_F32, variant=23,
                             split_k=-2).view(M, N)
    y = run()
    assert rel_l2(y, x.float().cpu() @ w.half().float().T) < 2e-3
    assert torch.equal(ops.conv2d(pc, x.view(1, M, 1, K), ksize=1, pad=0, out_mode=ops.OUT_ROWS_F32, variant=23,
                                  split_k=2).view(M, N), y)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        yg = run()
    for _ in range(3):
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(yg, y)
    assert int(ops.WORKSPACE.counters(DEV).abs().sum().item()) == 0


def test_inlaunch_rejects_non_tile_plans(ops, sdk):
    from sd_amd import _lib
    M, K, N = 1024, 640, 640
    x = _rand(M, K, seed=10).to(DEV)
    pc = ops.PackedConv([(torch.randn(N, K) / math.sqrt(K), K)], None, device=DEV)
    with pytest.raises(RuntimeError):   # the phased kernel (variant 8) has no in-launch combine
        ops.conv2d(pc, x.view(1, M, 1, K), ksize=1, pad=0, variant=8, split_k=-2)
    a = _lib.ConvArgs()
    assert _lib.lib().sdk_conv2d_plan(a, None) != 0        # empty args still rejected

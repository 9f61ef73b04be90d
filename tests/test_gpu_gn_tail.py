"""GroupNorm group statistics merged inside the producing conv's launch (run with -m gpu).

sdk_conv_args.gn_group_stats: every work item that stores GroupNorm partials of an image takes a ticket on
the image's arrival counter; the last one merges the image's partials into per-group (mean, variance), and
the consumer (sdk_group_norm_groups) runs one apply launch without a finalize.  Checked per producer plan
(LDS-DMA 16x16 and 32x32 epilogues, the phased kernel, the split-K reduce, the in-launch split) against fp32
torch GroupNorm of the same fp16 tensor and against the partials path it replaces (reference
openai_model/utils.py:15-22 GroupNorm32 + nn.SiLU at model.py:178-181); the counters are left zero and
graph replay reproduces the eager bits."""
import pytest
import torch
import torch.nn.functional as F

from gpu_util import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops(sdk):
    from sd_amd import ops as o
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return o


def _producer(ops, B, H, Cin, Cout, k, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(B, H + (k - 1), H + (k - 1), Cin, generator=g) * 0.5).half().to(DEV)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.3 + 0.2        # a per-channel offset: nonzero group means
    pc = ops.PackedConv([(w.to(DEV), Cin)], b.to(DEV), device=DEV)
    res = (torch.randn(B, H, H, Cout, generator=g) * 0.5).half().to(DEV)
    return x, pc, res


def _ref_gn(y, gamma, beta, eps, silu, pad):
    t = F.group_norm(y.float().permute(0, 3, 1, 2).cpu(), 32, gamma.cpu(), beta.cpu(), eps)
    if silu:
        t = F.silu(t)
    t = t.permute(0, 2, 3, 1)
    if pad:
        t = F.pad(t, (0, 0, pad, pad, pad, pad))
    return t


# (B, H, Cin, Cout, k, variant, split): LDS-DMA 16x16 epilogue (22, 24), 32x32 (2, 7), phased 32x32 (8), split-K
# reduce (20 / 25 split 3 / 6), in-launch split (22, -2); 64x64 / 32x32 / 16x16 / 8x8 levels
CASES = [
    (2, 64, 320, 320, 3, 22, 1), (2, 32, 640, 640, 3, 24, 1), (2, 64, 320, 320, 1, 2, 1), (1, 32, 640, 640, 1, 7, 1),
    (2, 32, 320, 640, 3, 8, 1), (2, 16, 640, 1280, 3, 20, 3), (4, 8, 1280, 1280, 3, 25, 6), (2, 32, 640, 640, 3, 22, -2),
    (3, 16, 1280, 1280, 1, 19, 1),
]


@pytest.mark.parametrize("B,H,Cin,Cout,k,variant,split", CASES)
@pytest.mark.parametrize("silu,pad", [(True, 1), (False, 0)])
def test_group_tail_vs_fp32_and_partials(ops, B, H, Cin, Cout, k, variant, split, silu, pad):
    x, pc, res = _producer(ops, B, H, Cin, Cout, k, seed=B * 7 + H + Cout)
    y = ops.conv2d(pc, x, pad=0, residual=res, variant=variant, split_k=split, gn_stats=True)
    gg = getattr(y, ops.GN_GROUPS_ATTR, None)
    assert gg is not None, "the plan emits GroupNorm statistics: the group tail must run"
    assert gg[0].shape == (B, 32, 2)
    gamma = (1 + 0.1 * torch.randn(Cout)).to(DEV)
    beta = (0.1 * torch.randn(Cout)).to(DEV)
    # group statistics themselves vs fp64 of the stored fp16 tensor
    yd = y.double().cpu().view(B, H * H, 32, Cout // 32)
    mean = yd.mean(dim=(1, 3))
    var = yd.var(dim=(1, 3), unbiased=False)
    st = gg[0].cpu()
    scale = max(1.0, mean.abs().max().item(), var.max().item() ** 0.5)
    assert (st[..., 0] - mean).abs().max().item() < 1e-5 * scale     # fp32 tile partials, fp64 merges
    assert ((st[..., 1] - var).abs() / var).max().item() < 1e-4
    out = ops.group_norm(y, gamma, beta, 1e-5, 32, silu=silu, pad=pad)
    ref = _ref_gn(y, gamma, beta, 1e-5, silu, pad)
    e = rel_l2(out, ref)
    # the partials path on the same tensor (drop the group statistics: sdk_group_norm merges the partials)
    delattr(y, ops.GN_GROUPS_ATTR)
    out_p = ops.group_norm(y, gamma, beta, 1e-5, 32, silu=silu, pad=pad)
    d = (out.float() - out_p.float()).abs().max().item()
    print(f"[gn_tail] v{variant} s{split} {B}x{H}x{H}x{Cout}: rel-L2 vs fp32 {e:.2e}, max |groups - partials| {d:.2e}",
          flush=True)
    assert e < 1e-3
    assert rel_l2(out, out_p) < 5e-4
    assert torch.count_nonzero(ops.WORKSPACE.gn_counters(y.device)).item() == 0


def test_group_tail_graph_replay_and_repeat(ops):
    """Captured producer + GroupNorm: replays equal the eager result bitwise, and the counters stay zero."""
    x, pc, res = _producer(ops, 4, 16, 640, 1280, 3, seed=3)
    gamma = torch.ones(1280, device=DEV)
    beta = torch.zeros(1280, device=DEV)

    def step():
        y = ops.conv2d(pc, x, pad=0, residual=res, variant=20, split_k=3, gn_stats=True)
        return ops.group_norm(y, gamma, beta, 1e-5, 32, silu=True, pad=1)

    eager = step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(cap, eager)
    assert torch.count_nonzero(ops.WORKSPACE.gn_counters(eager.device)).item() == 0


def test_group_tail_rejects(ops, sdk):
    from sd_amd import _lib
    a = _lib.GroupNormArgs()
    y = torch.zeros(1, 8, 8, 64, dtype=torch.float16, device=DEV)
    a.src0, a.ld0, a.c_split, a.batch, a.hw, a.channels, a.groups = y.data_ptr(), 64, 64, 1, 64, 64, 32
    L = _lib.lib()
    assert L.sdk_group_norm_groups(a, 1, y.data_ptr(), 64, 8, 8, 0, None, None) != 0       # no statistics
    st = torch.zeros(1, 32, 2, dtype=torch.float64, device=DEV)
    a.c_split = 32                                                                          # a concat
    assert L.sdk_group_norm_groups(a, 1, y.data_ptr(), 64, 8, 8, 0, st.data_ptr(), None) != 0

"""The reassociated 1280-channel cross-attention on the MI355X (run with -m gpu): its two kernels
through the C ABI — the segment softmax and the GEMM with per-image weights — against fp32
torch, and the model's CrossAttention._run on that path against the three-launch path and the
fp32 reference math (openai_model/attention.py:96-117)."""
import math

import pytest
import torch

from gpu_util import rel_l2, max_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops(sdk):
    from sd_amd import ops as o
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return o


@pytest.mark.parametrize("rows,nseg,seglen,ld_p", [(300, 8, 77, 640), (64, 3, 50, 192), (5, 1, 128, 128)])
def test_segment_softmax(ops, rows, nseg, seglen, ld_p):
    g = torch.Generator().manual_seed(rows + nseg)
    s = torch.randn(rows, nseg * seglen, generator=g) * 20.0
    p = ops.segment_softmax(s.to(DEV), nseg, seglen, 0.079, ld_p=ld_p)
    assert p.shape == (rows, ld_p) and p.dtype == torch.float16
    ref = (s.view(rows, nseg, seglen) * 0.079).softmax(-1).reshape(rows, -1)
    assert max_rel(p[:, :nseg * seglen], ref) < 2e-3
    assert torch.all(p[:, nseg * seglen:].float().cpu() == 0)       # the consumer GEMM's K padding


@pytest.mark.parametrize("n_img,k,n,out_mode", [(256, 192, 200, 0), (256, 1280, 616, 3), (128, 640, 1280, 0)])
def test_linear_per_image_weights(ops, n_img, k, n, out_mode):
    """Output rows of image b use image b's weights (sdk_conv_args.weight_batch_stride); bias and
    residual in the epilogue as for the shared-weight GEMM."""
    B = 3
    g = torch.Generator().manual_seed(n + k)
    x = (torch.randn(B * n_img, k, generator=g)).half()
    npad = (n + 127) // 128 * 128
    w = torch.zeros(B, npad, k, dtype=torch.float16)
    w[:, :n] = (torch.randn(B, n, k, generator=g) / math.sqrt(k)).half()
    bias = torch.randn(n, generator=g)
    res = torch.randn(B * n_img, n, generator=g).half() if out_mode == 0 else None
    pc = ops.PerImageWeights(w.to(DEV), n, bias.to(DEV))
    y = ops.linear(pc, x.to(DEV), out_mode=out_mode, n_img=n_img, residual=None if res is None else res.to(DEV))
    ref = torch.einsum("bmk,bnk->bmn", x.float().view(B, n_img, k), w[:, :n].float()).reshape(B * n_img, n) + bias
    if res is not None:
        ref = ref + res.float()
    assert y.shape == (B * n_img, n)
    assert rel_l2(y, ref) < 2e-3


def test_linear_per_image_weights_needs_a_tile_inside_an_image(ops):
    """64 rows per image: no LDS-DMA tile fits inside one image -> an error, never a wrong answer."""
    w = torch.zeros(2, 128, 64, dtype=torch.float16, device=DEV)
    pc = ops.PerImageWeights(w, 128)
    with pytest.raises(RuntimeError, match="per-image weights"):
        ops.linear(pc, torch.zeros(128, 64, dtype=torch.float16, device=DEV), n_img=64)


@pytest.mark.parametrize("B", [2, 3])
def test_reassociated_cross_attention_block(sdk, ops, B):
    """CrossAttention._run at the SD-1 16x16 level (1280 channels, 8 heads x 160, 77 context tokens)
    on the reassociated path vs the three launches and vs the fp32 reference math."""
    from sd_amd.openai_model.attention import CrossAttention, ReassocContext
    torch.manual_seed(B)
    C, D, H, L, N = 1280, 160, 8, 77, 256
    att = CrossAttention(query_dim=C, context_dim=768, heads=H, dim_head=D)
    with torch.no_grad():
        for m in (att.to_q, att.to_k, att.to_v, att.to_out[0]):
            m.weight.normal_(0, m.in_features ** -0.5)
        att.to_out[0].bias.normal_(0, 0.1)
    att = att.to(DEV)
    att._prepare(torch.device(DEV))
    ctx = torch.randn(B * L, 768).half()
    t = torch.randn(B * N, C).half()
    res = torch.randn(B * N, C).half()
    kvr = att.context_kv(ctx.to(DEV), L)
    assert isinstance(kvr, ReassocContext)
    # a block at the 8x8 level (64 tokens: not the reassociated path) builds no per-prompt matrices
    t64 = torch.randn(B * 64, C).half().to(DEV)
    att._run(t64, t64, B, 64, kvr, L)
    assert kvr.w1 is None and kvr.w2 is None
    y_re = att._run(t.to(DEV), res.to(DEV), B, N, kvr, L).float().cpu()
    assert kvr.w1 is not None
    y_3 = att._run(t.to(DEV), res.to(DEV), B, N, kvr.kv, L).float().cpu()
    # fp32 reference on the same fp16 inputs and weights
    wq, wk, wv = (m.weight.detach().float().cpu() for m in (att.to_q, att.to_k, att.to_v))
    wo, bo = att.to_out[0].weight.detach().float().cpu(), att.to_out[0].bias.detach().float().cpu()
    q = (t.float() @ wq.T).view(B, N, H, D)
    k = (ctx.float() @ wk.T).view(B, L, H, D)
    v = (ctx.float() @ wv.T).view(B, L, H, D)
    pr = (torch.einsum("bnhe,bjhe->bhnj", q, k) * D ** -0.5).softmax(-1)
    o = torch.einsum("bhnj,bjhe->bnhe", pr, v).reshape(B * N, C)
    ref = o @ wo.T + bo + res.float()
    upd = ref - res.float()
    e_re = ((y_re - ref).norm() / upd.norm()).item()
    e_3 = ((y_3 - ref).norm() / upd.norm()).item()
    print(f"[reassoc] B={B}: update rel-L2 reassociated {e_re:.2e}, three launches {e_3:.2e}", flush=True)
    assert e_re < 5e-3 and e_3 < 5e-3

"""API soundness of the host layer on the MI355X (run with -m gpu): caller-supplied output buffers,
HIP-graph results and timestep types behave as the reference's eager modules do."""
import math
import os

import pytest
import torch

from golden_util import cfg_of, load, weights_of
from gpu_util import rel_l2

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rand(*shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).half()


def test_conv_into_reused_out_drops_stale_group_norm_statistics(sdk):
    """conv2d(gn_stats=True) into a buffer attaches its statistics; a second conv2d into the SAME buffer
    by a plan that emits none must not leave the first ones attached (C-ABI writes do not move torch's
    version counter): group_norm then equals its own statistics pass."""
    from sd_amd import ops
    B, H, W, Ci, Co = 2, 16, 16, 128, 320
    g = torch.Generator().manual_seed(1)
    w1 = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)
    w2 = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)
    pc1 = ops.PackedConv([(w1, Ci)], torch.randn(Co, generator=g) + 2, device=DEV)
    pc2 = ops.PackedConv([(w2, Ci)], torch.randn(Co, generator=g) - 1, device=DEV)
    x = _rand(B, H, W, Ci, seed=2).to(DEV)
    buf = torch.empty(B, H, W, Co, dtype=torch.float16, device=DEV)
    ops.conv2d(pc1, x, out=buf, gn_stats=True, variant=22)
    assert getattr(buf, ops.GN_ATTR, None) is not None, "the first plan emits statistics"
    ops.conv2d(pc2, x, out=buf, variant=0)                   # register-staged: emits none
    assert getattr(buf, ops.GN_ATTR, None) is None
    gamma = torch.rand(Co, generator=g).to(DEV) + 0.5
    beta = (torch.randn(Co, generator=g) * 0.1).to(DEV)
    got = ops.group_norm(buf, gamma, beta, 1e-5, 32, silu=True)
    ref = ops.group_norm(buf.clone(), gamma, beta, 1e-5, 32, silu=True)   # fresh tensor: statistics pass
    assert torch.equal(got, ref)
    # the other writers into a caller-supplied buffer drop them too
    a = torch.empty(B * H * W, Co, dtype=torch.float16, device=DEV)
    setattr(a, ops.GN_ATTR, ("stale", 1, a._version))
    ops.layer_norm(buf.view(-1, Co).contiguous(), torch.ones(Co, device=DEV), torch.zeros(Co, device=DEV), out=a)
    assert not hasattr(a, ops.GN_ATTR)


def _tiny_unet():
    from sd_amd.openai_model.model import UNetModel
    u = load("unet_tiny")
    m = UNetModel(**cfg_of(u))
    m.load_state_dict(weights_of(u))
    return m.to(DEV), u


def test_graph_replay_returns_a_fresh_tensor(sdk):
    """With graphs on, DiffusionWrapper returns a new tensor per call, as the eager path does: an eps
    kept from call 1 survives call 2 (the reference's apply_model contract)."""
    from sd_amd.Diffusion.ddpm import DiffusionWrapper
    m, u = _tiny_unet()
    dw = DiffusionWrapper.__new__(DiffusionWrapper)
    torch.nn.Module.__init__(dw)
    dw.diffusion_model, dw.conditioning_key, dw._graphed, dw._graphs_on = m, "crossattn", None, False
    x = torch.from_numpy(u["x"]).to(DEV)
    c = torch.from_numpy(u["ctx"]).to(DEV)
    t1 = torch.tensor([10, 3], device=DEV)
    t2 = torch.tensor([500, 700], device=DEV)
    e1_eager = dw(x, t1, c_crossattn=[c]).clone()
    e2_eager = dw(x, t2, c_crossattn=[c]).clone()
    dw.use_graphs(True)
    dw(x, t1, c_crossattn=[c])                               # warm-up + capture
    e1 = dw(x, t1, c_crossattn=[c])
    e2 = dw(x, t2, c_crossattn=[c])
    assert e1.data_ptr() != e2.data_ptr()
    assert torch.equal(e1, e1_eager), "call 2 overwrote call 1's result"
    assert torch.equal(e2, e2_eager)


def test_graph_and_eager_paths_treat_timesteps_alike(sdk):
    """Fractional timesteps raise on both paths (the graph path used to truncate them); integral
    float timesteps give the int64 result bit for bit on both."""
    from sd_amd.Diffusion.ddpm import DiffusionWrapper
    m, u = _tiny_unet()
    dw = DiffusionWrapper.__new__(DiffusionWrapper)
    torch.nn.Module.__init__(dw)
    dw.diffusion_model, dw.conditioning_key, dw._graphed, dw._graphs_on = m, "crossattn", None, False
    x = torch.from_numpy(u["x"]).to(DEV)
    c = torch.from_numpy(u["ctx"]).to(DEV)
    for graphs in (False, True):
        dw.use_graphs(graphs)
        with pytest.raises(ValueError):
            dw(x, torch.tensor([10.5, 3.0], device=DEV), c_crossattn=[c])
        a = dw(x, torch.tensor([10, 3], device=DEV), c_crossattn=[c]).clone()
        b = dw(x, torch.tensor([10.0, 3.0], device=DEV), c_crossattn=[c]).clone()
        assert torch.equal(a, b)

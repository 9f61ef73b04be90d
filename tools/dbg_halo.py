import math, os, sys
import torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops
from gpu_util import rel_l2
DEV = "cuda"
def _rand(*shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).half()
def _padded(x):
    return F.pad(x.float().permute(0, 3, 1, 2), (1, 1, 1, 1)).permute(0, 2, 3, 1).half().contiguous()
B, H, W, C1, C2, Co = 2, 32, 32, 128, 192, 320
a, c = _rand(B, H, W, C1, seed=7), _rand(B, H, W, C2, seed=8)
ap, cp = _padded(a).to(DEV), _padded(c).to(DEV)
g = torch.Generator().manual_seed(11)
w = torch.randn(Co, C1 + C2, 3, 3, generator=g) / math.sqrt((C1 + C2) * 9)
b = torch.randn(Co, generator=g) * 2 + 3
emb = torch.randn(B, Co + 8, generator=g)
res = _rand(B, H, W, Co, seed=9)
pc = ops.PackedConv([(w, C1 + C2)], b, device=DEV)
xcat = torch.cat([ap, cp], -1).contiguous()
for name, src, kw in [("cat", (ap, cp), {}), ("single", xcat, {}), ("rb", xcat, dict(row_bias=(emb.to(DEV), 8))),
                      ("res", xcat, dict(residual=res.to(DEV))), ("gn", xcat, dict(gn_stats=True)),
                      ("all", (ap, cp), dict(row_bias=(emb.to(DEV), 8), residual=res.to(DEV), gn_stats=True))]:
    for v, t in ((36, 22), (37, 23)):
        y = ops.conv2d(pc, src, pad=0, variant=v, **kw)
        yt = ops.conv2d(pc, src, pad=0, variant=t, **kw)
        d = (y.float() - yt.float()).abs()
        nz = (d > 0).nonzero()
        print(name, v, "equal" if torch.equal(y, yt) else f"ndiff={nz.shape[0]} max={d.max().item():.3g} first={nz[:3].tolist()}", flush=True)

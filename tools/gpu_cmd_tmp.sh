cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 120 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids
import sys, torch
sys.path.insert(0, ".")
import sd_amd_loader; sd_amd_loader.load()
from sd_amd import ops
from tools.bench_norm import timeit
for (B, H, Ci, Co) in [(16, 66, 320, 4), (16, 514, 128, 3), (8, 98, 320, 4)]:
    x = torch.randn(B, H, H, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, 3, 3, device="cuda") / (Ci * 9) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), device="cuda")
    fl = 2.0 * B * (H - 2) ** 2 * Co * Ci * 9
    for v in (4, 22, 34):
        t = timeit(lambda: ops.conv2d(pc, x, pad=0, out_mode=ops.OUT_NCHW_F32, variant=v, split_k=1), reps=5)
        print(f"B={B} {H-2}x{H-2} {Ci}->{Co} v{v}: {t:8.1f} us ({fl / t / 1e6:6.1f} TF/s)")
PY

import torch


def rel_l2(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def max_rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def check_parity(tag, got, ref, rl2_max, mabs_max):
    """Print and assert rel-L2 AND max |got - ref| / max |ref| (full-size fp16 models vs the fp32 oracle).
    Every call site states its own limits, at most ~3.5x the errors measured on MI355X
    (profiles/r5_parity_errors.txt)."""
    rl2 = rel_l2(got, ref)
    a, b = got.detach().float().cpu(), ref.detach().float().cpu()
    mab = ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
    print(f"[parity] {tag}: rel-L2 {rl2:.3e} (<= {rl2_max:.1e})  max-abs/max {mab:.3e} (<= {mabs_max:.1e})",
          flush=True)
    assert rl2 <= rl2_max, f"{tag}: rel-L2 {rl2:.3e}"
    assert mab <= mabs_max, f"{tag}: max-abs {mab:.3e}"
    return rl2, mab

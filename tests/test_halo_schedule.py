"""CPU check of the halo-tile conv's LDS ring plan (csrc/halo_sched.h): tests/halo_sim.cpp replays the
kernel's per-wave issue state machine and verifies every A-fragment read of every K-step of every tile
(right piece in the slot, issued at least one K-step before the read, the addressed padded pixel) for
the SD / SD-2 levels, multi-image tiles, ragged last tiles and split-K starts."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("halo") / "halo_sim")
    subprocess.run([gxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "stable-diffusion-from-scratch_amd", "csrc"),
                    os.path.join(ROOT, "tests", "halo_sim.cpp"), "-o", exe], check=True)
    return exe


# (batch, ho, wo, tbm, waves, max_rp, channel blocks, split, plan expected)
CASES = [
    (16, 64, 64, 256, 16, 77, 5, 1, True),     # SD 64x64 level, variant 36
    (16, 64, 64, 128, 8, 77, 15, 1, True),
    (16, 32, 32, 256, 16, 77, 10, 1, True),
    (16, 32, 32, 128, 8, 77, 30, 2, True),
    (16, 16, 16, 256, 16, 77, 20, 4, True),    # split-K over channel blocks
    (16, 16, 16, 128, 8, 77, 40, 8, True),
    (8, 96, 96, 128, 8, 77, 5, 1, True),       # SD-2 768 levels (tiles not row-aligned)
    (8, 48, 48, 256, 16, 77, 10, 3, True),
    (8, 24, 24, 128, 8, 77, 20, 2, False),     # 576-pixel images: 128-pixel tiles straddle images
    (3, 8, 8, 128, 8, 77, 4, 3, True),         # multi-image tiles, ragged last tile
    (3, 8, 8, 256, 16, 77, 4, 1, False),       # 4 images per tile overflow the ring
    (16, 128, 128, 256, 16, 77, 8, 1, True),   # VAE 128x128 (one row-half per tile)
    (2, 16, 16, 128, 8, 20, 3, 1, False),      # ring smaller than the live pieces
    # GroupNorm-fused form (lead 2: transformed in LDS the K-step after landing), 76-slot ring
    (16, 64, 64, 256, 16, 76, 5, 1, True, 2),
    (16, 32, 32, 256, 16, 76, 10, 2, True, 2),
    (16, 16, 16, 256, 16, 76, 20, 4, True, 2),
    (16, 16, 16, 128, 8, 76, 40, 8, True, 2),
    (8, 96, 96, 128, 8, 76, 5, 1, True, 2),
    (8, 48, 48, 256, 16, 76, 10, 3, True, 2),
]


@pytest.mark.parametrize("case", CASES, ids=[",".join(map(str, c[:8])) for c in CASES])
def test_halo_ring_replay(sim, case):
    args, expect, lead = list(case[:8]), case[8], case[9:]
    args += list(lead)
    out = subprocess.run([sim, *map(str, args)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    line = out.stdout.strip()
    if expect:
        assert line.startswith("OK"), line
    else:
        assert line.startswith("NOPLAN"), line

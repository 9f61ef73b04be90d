"""Build the library variants tools/gpu_det_libs.sh compares (CPU, in-tree; they travel with the snapshot):
libsdk_amd_dpp.so (DPP cross-lane moves, SDK_XLANE_DPP=1) and libsdk_amd_r3slp.so (round-3 common.h from
git HEAD~ history at commit 03be2a6, i.e. DPP reductions with free FP contraction, SLP on)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stable-diffusion-from-scratch_amd"))
import build  # noqa: E402


def main():
    print(build.build(tag="dpp", defines=["-DSDK_XLANE_DPP=1"]))
    tree = os.path.join(ROOT, "abtree", "r3csrc")
    shutil.rmtree(tree, ignore_errors=True)
    shutil.copytree(build.CSRC, tree)
    old = subprocess.run(["git", "-C", ROOT, "show", "03be2a6:stable-diffusion-from-scratch_amd/csrc/common.h"],
                         capture_output=True, text=True, check=True).stdout
    with open(os.path.join(tree, "common.h"), "w") as f:
        f.write(old)
    print(build.build(tag="r3slp", csrc=tree))


if __name__ == "__main__":
    main()

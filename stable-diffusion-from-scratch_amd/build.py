"""Build libsdk_amd.so (gfx950) in-tree with hipcc — no JIT cache, the .so ships with the repo snapshot."""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libsdk_amd.so")
SOURCES = ["conv.hip", "norm.hip", "attention.hip", "sampler.hip", "xattn.hip", "ff.hip", "token.hip", "probe.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]
# attention: IEEE mode off + no NaN semantics, so fmaxf on MFMA results is one v_max3 instead of
# canonicalising v_max x,x copies first (the inputs are finite fp16 products)
# xattn.hip: no SLP vectorisation (no packed-fp32 v_pk_* math).  With it, the fused norm3 of the
# <320, 40> block wrote garbage into 4 rows (16 lanes = one VALU pass group) of one 64-row tile in
# ~0.3 % of launches inside the UNet (never in isolation): a timing-dependent hazard around the
# packed sums feeding the quad DPP reductions; scalar fp32 code measured 0 / 2,500 differing launches
# (tools/det_probe4.py, profiles/r3_xattn_determinism.txt).  norm.hip the same, so the LayerNorm row math
# the two share (common.h) compiles to the same scalar code: the fused norms stay bit-identical to
# sdk_layer_norm.
EXTRA = {"attention.hip": ["-mno-amdgpu-ieee", "-fno-honor-nans"], "xattn.hip": ["-fno-slp-vectorize"],
         "norm.hip": ["-fno-slp-vectorize"]}


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """``diag=True`` builds libsdk_amd_diag.so: the same ABI plus the conv kernel's diagnostic
    ablations (variants 10-15, 27-30 — wrong outputs by design), for tools/ only (load it with
    SD_AMD_LIB); the product library rejects those variant ids."""
    bdir = BUILD + ("_diag" if diag else "")
    lib = LIB.replace(".so", "_diag.so") if diag else LIB
    os.makedirs(bdir, exist_ok=True)
    headers = [os.path.join(CSRC, "common.h"), os.path.join(CSRC, "halo_sched.h"), os.path.join(HERE, "..", "include", "sdk_amd.h")]
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src.replace(".hip", ".o"))
        flags_file = o + ".flags"
        fl = " ".join(FLAGS + EXTRA.get(src, []) + (["-DSDK_CONV_DIAGNOSTICS"] if diag else []))
        stale_flags = not os.path.exists(flags_file) or open(flags_file).read() != fl
        if stale_flags:
            with open(flags_file, "w") as f:
                f.write(fl)
        if force or stale_flags or _needs(o, [s] + headers):
            dflags = ["-DSDK_CONV_DIAGNOSTICS"] if diag else []
            jobs.append([HIPCC, *FLAGS, *dflags, *EXTRA.get(src, []), "-c", s, "-o", o])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(" ".join(cmd))
        return r

    with cf.ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(bdir, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _needs(lib, objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", lib])
    return lib


if __name__ == "__main__":
    import sys
    print(build(verbose=True, diag="--diag" in sys.argv))

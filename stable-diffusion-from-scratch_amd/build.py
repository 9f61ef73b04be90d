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
EXTRA = {"attention.hip": ["-mno-amdgpu-ieee", "-fno-honor-nans"]}


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, diag: bool = False, tag: str = "", defines=(),
          extra=None, csrc: str = CSRC) -> str:
    """``diag=True`` builds libsdk_amd_diag.so: the same ABI plus the conv kernel's diagnostic
    ablations (variants 10-15, 27-30 — wrong outputs by design), for tools/ only (load it with
    SD_AMD_LIB); the product library rejects those variant ids.  ``tag`` builds an A/B variant
    libsdk_amd_<tag>.so in build_<tag>/ with extra ``defines`` for every source and per-source
    ``extra`` flags, optionally from another source directory ``csrc`` (tools/ only, e.g.
    tools/gpu_det_libs.sh)."""
    suffix = "_diag" if diag else (f"_{tag}" if tag else "")
    bdir = BUILD + suffix
    lib = LIB.replace(".so", f"{suffix}.so")
    extra_flags = dict(EXTRA)
    for k, v in (extra or {}).items():
        extra_flags[k] = extra_flags.get(k, []) + list(v)
    os.makedirs(bdir, exist_ok=True)
    headers = [os.path.join(csrc, "common.h"), os.path.join(csrc, "halo_sched.h"), os.path.join(HERE, "..", "include", "sdk_amd.h")]
    jobs = []
    for src in SOURCES:
        s = os.path.join(csrc, src)
        o = os.path.join(bdir, src.replace(".hip", ".o"))
        flags_file = o + ".flags"
        dflags = (["-DSDK_CONV_DIAGNOSTICS"] if diag else []) + list(defines)
        fl = " ".join(FLAGS + extra_flags.get(src, []) + dflags)
        stale_flags = not os.path.exists(flags_file) or open(flags_file).read() != fl
        if force or stale_flags or _needs(o, [s] + headers):
            # the sidecar is rewritten only after this object compiled (run() below): an interrupted
            # or failed compile leaves no object that claims the new flags
            for stale in (o, flags_file):
                if os.path.exists(stale):
                    os.remove(stale)
            jobs.append(([HIPCC, *FLAGS, *dflags, *extra_flags.get(src, []), "-c", s, "-o", o], (flags_file, fl)))

    def run(cmd, sidecar=None):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if sidecar:
            with open(sidecar[0], "w") as f:
                f.write(sidecar[1])
        if verbose:
            print(" ".join(cmd))
        return r

    with cf.ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(lambda j: run(*j), jobs))
    objs = [os.path.join(bdir, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _needs(lib, objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", lib])
    return lib


if __name__ == "__main__":
    import sys
    print(build(verbose=True, diag="--diag" in sys.argv))

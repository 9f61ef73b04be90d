"""Build libsdk_amd.so (gfx950) in-tree with hipcc — no JIT cache, the .so ships with the repo snapshot."""
from __future__ import annotations

import concurrent.futures as cf
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libsdk_amd.so")
SOURCES = ["conv.hip", "norm.hip", "attention.hip", "sampler.hip", "xattn.hip", "ff.hip", "token.hip", "probe.hip"]
# conv.hip is compiled once per part (its SDK_CONV_PART partition: host planner + small kernels, then the tile
# kernel instantiations in four groups) so the objects build in parallel
CONV_PARTS = 6


def _units():
    """(source, object stem, extra defines) per compiled object."""
    for src in SOURCES:
        if src == "conv.hip":
            for k in range(CONV_PARTS):
                yield src, f"conv_p{k}", [f"-DSDK_CONV_PART={k}"]
        else:
            yield src, src.replace(".hip", ""), []
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]
# attention: IEEE mode off + no NaN semantics, so fmaxf on MFMA results is one v_max3 instead of
# canonicalising v_max x,x copies first (the inputs are finite fp16 products)
EXTRA = {"attention.hip": ["-mno-amdgpu-ieee", "-fno-honor-nans"]}
# every kernel's register / scratch use is recorded from the compiler's resource remarks
# (build*/resource_usage.txt).  The token linear's ring immediates count its own global stores
# (token.hip: D + 2 * (TL_CPT + 10)), so a scratch spill or a split store there could retire a ring slot
# early: that kernel must not touch scratch and the build fails otherwise.  For the other counted-vmcnt
# kernels a spill only over-waits (an extra VMEM op never lowers the count of the DMAs a wait covers), so
# it is reported as a warning (it costs time: scratch round trips in the K loop)
REMARK = "-Rpass-analysis=kernel-resource-usage"
NO_SCRATCH = re.compile(r"token_linear320_kernel")
WARN_SCRATCH = re.compile(r"conv_glds_kernel|conv_ph_kernel|ff_geglu_kernel|xattn_block_kernel|attn_fwd_kernel")
_RES = re.compile(r"remark: (?:Function Name: (\S+)|\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+))")


def resource_usage(stderr: str):
    """[(kernel, {VGPRs, AGPRs, ScratchSize, Occupancy})] from -Rpass-analysis=kernel-resource-usage output."""
    out = []
    for m in _RES.finditer(stderr):
        if m.group(1):
            out.append((m.group(1), {}))
        elif out:
            out[-1][1][m.group(2).split(" ")[0]] = int(m.group(3))
    return out


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
    headers = [os.path.join(csrc, "common.h"), os.path.join(HERE, "..", "include", "sdk_amd.h")]
    jobs = []
    objs = []
    for src, stem, udefs in _units():
        s = os.path.join(csrc, src)
        o = os.path.join(bdir, stem + ".o")
        objs.append(o)
        flags_file = o + ".flags"
        dflags = (["-DSDK_CONV_DIAGNOSTICS"] if diag else []) + list(defines) + udefs
        fl = " ".join(FLAGS + extra_flags.get(src, []) + dflags)
        stale_flags = not os.path.exists(flags_file) or open(flags_file).read() != fl
        if force or stale_flags or _needs(o, [s] + headers) or not os.path.exists(o + ".res"):
            # the sidecar is rewritten only after this object compiled (run() below): an interrupted
            # or failed compile leaves no object that claims the new flags
            for stale in (o, flags_file):
                if os.path.exists(stale):
                    os.remove(stale)
            jobs.append(([HIPCC, *FLAGS, *dflags, *extra_flags.get(src, []), REMARK, "-c", s, "-o", o],
                         (flags_file, fl)))

    def run(cmd, sidecar=None):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if REMARK in cmd:
            usage = resource_usage(r.stderr)
            obj = cmd[cmd.index("-o") + 1]
            with open(obj + ".res", "w") as f:
                for name, u in usage:
                    f.write(f"{name} vgpr={u.get('VGPRs')} agpr={u.get('AGPRs')} scratch={u.get('ScratchSize')} "
                            f"occ={u.get('Occupancy')}\n")
            if os.path.basename(obj).startswith("token") and not any(
                    NO_SCRATCH.search(n) and "ScratchSize" in u for n, u in usage):
                # the check below must see the kernel: missing or reformatted remarks fail the build
                # rather than pass it silently (profiles/r6_resource_usage.txt is a parsed sample)
                os.remove(obj)
                raise RuntimeError("no kernel-resource-usage remark for token_linear320_kernel: cannot verify "
                                   "that it uses no scratch")
            bad = [n for n, u in usage if NO_SCRATCH.search(n) and u.get("ScratchSize", 0) > 0]
            for n, u in usage:
                if WARN_SCRATCH.search(n) and u.get("ScratchSize", 0) > 0:
                    print(f"warning: {n} uses {u['ScratchSize']} B/lane of scratch", flush=True)
            if bad:
                os.remove(obj)
                raise RuntimeError("counted-vmcnt kernels use scratch (spills break the hand-counted waits): " +
                                   ", ".join(bad))
        if sidecar:
            with open(sidecar[0], "w") as f:
                f.write(sidecar[1])
        if verbose:
            print(" ".join(cmd))
        return r

    workers = int(os.environ.get("SD_AMD_BUILD_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=min(workers, max(1, len(jobs)))) as ex:
        list(ex.map(lambda j: run(*j), jobs))
    if force or jobs or _needs(lib, objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", lib])
        with open(os.path.join(bdir, "resource_usage.txt"), "w") as f:
            for o in objs:
                if os.path.exists(o + ".res"):
                    f.write(open(o + ".res").read())
    return lib


if __name__ == "__main__":
    import sys
    print(build(verbose=True, diag="--diag" in sys.argv))

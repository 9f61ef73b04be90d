"""One UNet sampling step from a rocprofv3 kernel trace: per-kernel device time, the idle gaps
between consecutive kernels, and the step's wall span.

usage: python tools/trace_step.py <run_kernel_trace.csv> [step_index] [--list] [--seq seq.json]
(step_index default: len(steps) // 4, a graph-replayed step of the bench's warm-up sample)
--seq: the launch sequence of one UNet forward written by bench.py (BENCH_SEQ_OUT); each
record is paired in order with its dispatches (conv [+ splitk_reduce], GN partial+finalize, ...)
and a per-shape table of device times is printed.
A step = the dispatches after one ddim_step_kernel up to and including the next one.
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("sdk::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    m = re.match(r"_ZN3sdk12_GLOBAL__N_1\d+(\w+?)E", n)
    if m:
        n = m.group(1)
    n = re.sub(r"\(.*$", "", n)
    return n.replace("void ", "")[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "ddim_step_kernel" in r["Kernel_Name"]]
    # default: a step inside the warm-up sample's graph replays (a quarter into the run — not the last steps,
    # which belong to bench.py's eager, event-instrumented profiling pass)
    idx = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else max(1, len(marks) // 4)
    a, b = marks[idx - 1] + 1, marks[idx] + 1
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy, gaps = 0, []
    agg = defaultdict(lambda: [0, 0])
    prev_end = None
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        if prev_end is not None:
            gaps.append(s - prev_end)
        prev_end = e
        k = (short(r["Kernel_Name"]), f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}')
        agg[k][0] += 1
        agg[k][1] += e - s
    print(f"step {idx}: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"gaps {sum(gaps) / 1e3:.1f} us (mean {sum(gaps) / max(len(gaps), 1) / 1e3:.2f} us)")
    fam = defaultdict(float)
    for (n, g), (c, t) in agg.items():
        fam[n] += t
    for n, t in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"  {n:60s} {t / 1e3:9.1f} us")
    if "--seq" in sys.argv:
        import json
        seq = json.load(open(sys.argv[sys.argv.index("--seq") + 1]))
        fams = {"conv": ("conv_glds", "conv_ph", "conv_igemm"), "group_norm": ("gn_partial",),
                "gn_apply": ("gn_apply",), "layer_norm": ("layer_norm",), "attention": ("attn_fwd",)}
        ks = [r for r in step if "at::native" not in r["Kernel_Name"] and "rocclr" not in r["Kernel_Name"]]
        i, per = 0, defaultdict(lambda: [0, 0, 0.0])
        for kind, var, fl, sh in seq:
            while i < len(ks) and not any(f in ks[i]["Kernel_Name"] for f in fams.get(kind, (kind,))):
                i += 1
            if i >= len(ks):
                print("sequence does not match the trace step")
                break
            t = int(ks[i]["End_Timestamp"]) - int(ks[i]["Start_Timestamp"])
            i += 1
            while i < len(ks) and any(f in ks[i]["Kernel_Name"] for f in ("splitk_reduce", "gn_finalize")):
                t += int(ks[i]["End_Timestamp"]) - int(ks[i]["Start_Timestamp"])
                i += 1
            key = (kind, str(sh))
            per[key][0] += 1
            per[key][1] += t
            per[key][2] += fl or 0.0
        tot = sum(v[1] for v in per.values())
        print(f"  paired {sum(v[0] for v in per.values())} launches, {tot / 1e3:.1f} us")
        for (kind, sh), (c, t, fl) in sorted(per.items(), key=lambda x: -x[1][1]):
            tf = fl / (t * 1e-9) / 1e12 if t and fl else 0.0
            print(f"    {kind:10s} {sh:40s} x{c:3d} {t / c / 1e3:8.1f} us each {t / 1e3:8.1f} us  {tf:7.1f} TF/s")
    if "--list" in sys.argv:
        for (n, g), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
            print(f"    {n:50s} grid {g:18s} x{c:3d} {t / c / 1e3:8.1f} us each")


if __name__ == "__main__":
    main()

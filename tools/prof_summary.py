"""Summarise one tools/prof_round.sh session into profiles/.

Reads gpurun_out/prof_round/{trace/run_kernel_stats.csv, pmc_fetch/..., pmc_write/...}
and writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats table, names
shortened), profiles/<tag>_conv_traffic.json (PMC HBM bytes per conv launch) and
copies the per-shape table and the bench log.

Traffic correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming reads (global_load
dwordx4 and buffer_load ... lds alike) -> bytes = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE.
"""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONV = ("conv_glds_kernel", "conv_ph_kernel", "conv_igemm_kernel", "conv_direct_kernel",
        "conv_skinny_kernel", "splitk_reduce_kernel", "splitk_reduce_gn_kernel")


def short(name):
    n = name.replace("sdk::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(sdk::Params\)|\(Params\)", "", n)
    m = re.match(r"_ZN3sdk12_GLOBAL__N_1\d+(\w+?)E", n)
    if m:
        n = m.group(1)
    return n[:120]


def family(name):
    for c in CONV:
        if c in name:
            return "conv"
    return None


def pmc(path):
    out = {}
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def main(tag, src=os.path.join(ROOT, "gpurun_out", "prof_round")):
    prof = os.path.join(ROOT, "profiles")
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["Percentage"],
                        r["MinNs"], r["MaxNs"]])
    conv_calls = sum(int(r["Calls"]) for r in rows if family(r["Name"]) and "splitk" not in r["Name"])
    conv_ns = sum(float(r["TotalDurationNs"]) for r in rows if family(r["Name"]))
    fetch, write = pmc(os.path.join(src, "pmc_fetch", "run_counter_collection.csv")), \
        pmc(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    sys.path.insert(0, ROOT)
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    summ = {"conv_source": ops._conv_source_hash(), "tag": tag, "trace_conv_launches": conv_calls, "trace_conv_avg_us": conv_ns / max(conv_calls, 1) / 1e3}
    if fetch and write:
        fb = sum(v for n, v in fetch.values() if family(n)) * 1024 * 2
        wb = sum(v for n, v in write.values() if family(n)) * 1024
        nl = sum(1 for n, _ in fetch.values() if family(n) and "splitk" not in n)
        summ.update({"pmc_conv_launches": nl, "fetch_bytes_per_launch": fb / nl, "write_bytes_per_launch": wb / nl,
                     "traffic_bytes_per_launch": (fb + wb) / nl,
                     "note": "FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024 (gfx950 correction, MI355X_MICROARCH.md "
                             "HBM section); splitk_reduce traffic folded into its conv launch; "
                             "L2->fabric bytes (Infinity-Cache hits included)"})
        per = {}
        for did, (n, v) in fetch.items():
            k = short(n)
            e = per.setdefault(k, [0, 0.0, 0.0])
            e[0] += 1
            e[1] += v * 2048
            e[2] += write.get(did, (n, 0.0))[1] * 1024
        summ["per_kernel_MB_per_launch"] = {k: {"launches": c, "fetch_MB": round(f / c / 1e6, 3),
                                                "write_MB": round(w / c / 1e6, 3)}
                                            for k, (c, f, w) in sorted(per.items(), key=lambda x: -x[1][1])[:25]}
    for fn in (f"{tag}_conv_traffic.json", "conv_traffic.json"):     # the latter is what bench.py reads
        with open(os.path.join(prof, fn), "w") as f:
            json.dump(summ, f, indent=1)
    for fn in ("shapes.txt", "bench.log", "bench_c3.log", "bench_c5.log", "bench_c2.log", "bench_c1.log"):
        p = os.path.join(src, fn)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{fn.replace('.txt', '').replace('.log', '')}" +
                                        (".txt" if fn.endswith(".txt") else ".log")))
    print(json.dumps({k: v for k, v in summ.items() if k != "per_kernel_MB_per_launch"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))

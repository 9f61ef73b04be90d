"""Effective shader clock per kernel family from a rocprofv3 GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md 'DVFS
give-back': clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; reads high on dispatches shorter than ~0.3 ms).
usage: python tools/clock_pmc.py <run_counter_collection.csv> [min_us]
Prints, per kernel name (shortened), the dispatch count, total time and the time-weighted effective clock."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short   # noqa: E402


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        if dt * 1e6 < min_us:
            continue
        e = agg[short(r["Kernel_Name"])]
        e[0] += 1
        e[1] += dt
        e[2] += float(r["Counter_Value"]) / 8.0
    tot_t = sum(v[1] for v in agg.values())
    tot_c = sum(v[2] for v in agg.values())
    print(f"# dispatches >= {min_us:.0f} us; all: {tot_t * 1e3:.1f} ms at {tot_c / tot_t / 1e9:.3f} GHz")
    for k, (n, t, c) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{k:70s} n={n:5d} {t * 1e3:9.2f} ms  {c / t / 1e9:6.3f} GHz")


if __name__ == "__main__":
    main()

"""Summarise tools/gpu_ab_cases.sh output: per (case, library) the median / min / max us over the rounds and
the median's ratio to the first library's.  usage: python tools/ab_summary.py <log>"""
import collections
import re
import statistics
import sys


def main():
    rows = collections.defaultdict(list)
    order, tags = [], []
    for line in open(sys.argv[1]):
        m = re.match(r"r(\d+) (\S+) (\S+) v(\d+) s(-?\d+)\s+([\d.]+) us\s+([\d.]+) TF/s", line.strip())
        if not m:
            continue
        tag, case = m.group(2), f"{m.group(3)} v{m.group(4)} s{m.group(5)}"
        if case not in order:
            order.append(case)
        if tag not in tags:
            tags.append(tag)
        rows[(case, tag)].append(float(m.group(6)))
    for case in order:
        base = None
        out = []
        for t in tags:
            v = rows.get((case, t))
            if not v:
                continue
            med = statistics.median(v)
            base = base or med
            out.append(f"{t}: {med:7.1f} us [{min(v):.1f}-{max(v):.1f}, n={len(v)}] x{base / med:.3f}")
        print(f"{case:34s} " + " | ".join(out))


if __name__ == "__main__":
    main()

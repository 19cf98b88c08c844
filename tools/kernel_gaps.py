"""Idle gaps between consecutive kernels in a rocprofv3 kernel_trace.csv: how much of a wall-clock
window the GPU spends between launches. usage: kernel_gaps.py TRACE.csv [--last N]"""
import csv
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    if last:
        rows = rows[-last:]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = [rows[i + 1][0] - rows[i][1] for i in range(len(rows) - 1)]
    by_name = {}
    for i in range(len(rows) - 1):
        by_name.setdefault(rows[i + 1][2], []).append(gaps[i])
    print(f"{len(rows)} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({busy / span:.1%}), "
          f"gaps {sum(gaps) / 1e3:.1f} us")
    for name, g in sorted(by_name.items(), key=lambda kv: -sum(kv[1]))[:10]:
        print(f"  before {name:60s} n={len(g):5d} mean gap {sum(g) / len(g) / 1e3:7.2f} us  max {max(g) / 1e3:8.1f} us")


if __name__ == "__main__":
    main()

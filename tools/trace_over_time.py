"""Step-kernel duration over the launches of one run (rocprofv3 kernel_trace.csv): mean / min / max
per block of launches, and the mean of the last `--tail` launches (the timed ones).
usage: trace_over_time.py TRACE.csv [--block 100] [--tail 1000] [--kernel step_kernel]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--block", type=int, default=100)
    ap.add_argument("--tail", type=int, default=1000)
    ap.add_argument("--kernel", default="step_kernel")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    print(f"{len(d)} launches of {a.kernel}; us per launch by block of {a.block}:")
    for s in range(0, len(d), a.block):
        seg = d[s:s + a.block]
        print(f"  launches {s:5d}-{s + len(seg) - 1:5d}: mean {sum(seg) / len(seg):6.2f}  min {min(seg):6.2f}  max {max(seg):6.2f}")
    t = d[-a.tail:]
    print(f"last {len(t)} launches: mean {sum(t) / len(t):.2f} us; all launches: mean {sum(d) / len(d):.2f} us")


if __name__ == "__main__":
    main()

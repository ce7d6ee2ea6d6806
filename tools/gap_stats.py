"""Kernel time vs launch-to-launch time of back-to-back launches of one kernel, from a
rocprofv3 kernel trace (csv): for runs of consecutive launches of KERNEL (no other
kernel in between), the average duration, the gap between one launch's end and the
next one's start, and the start-to-start period (what a per-launch event figure over
back-to-back launches measures).  Usage: python tools/gap_stats.py trace.csv KERNEL"""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = sys.argv[2]
    durs, gaps, periods = [], [], []
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if name in r["Kernel_Name"]:
            durs.append((e - s) / 1e3)
            if prev is not None:
                gaps.append((s - prev[1]) / 1e3)
                periods.append((s - prev[0]) / 1e3)
            prev = (s, e)
        else:
            prev = None
    q = lambda v, p: sorted(v)[int(p * (len(v) - 1))] if v else float("nan")
    print(f"{name}: {len(durs)} launches, {len(gaps)} back-to-back pairs")
    print(f"  duration us: mean {statistics.mean(durs):.2f} median {q(durs, .5):.2f}")
    if gaps:
        print(f"  gap end->next start us: mean {statistics.mean(gaps):.2f} "
              f"median {q(gaps, .5):.2f} p10 {q(gaps, .1):.2f} p90 {q(gaps, .9):.2f}")
        print(f"  period start->start us: mean {statistics.mean(periods):.2f} "
              f"median {q(periods, .5):.2f}")


if __name__ == "__main__":
    main()

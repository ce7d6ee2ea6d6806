"""Per-dispatch durations and gaps of one kernel in a rocprofv3 kernel trace.

For the dispatches whose name contains KERNEL (in start order): mean / median duration, the
mean gap from one dispatch's end to the next one's start, and the mean period (start to
start) — how much of a back-to-back launch sequence is kernel time and how much is the gap
between kernels.  Usage: python tools/kgaps.py run_kernel_trace.csv KERNEL [skip]"""
import csv
import json
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if kern in r.get("Kernel_Name", ""):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    rows = rows[skip:]
    if len(rows) < 2:
        raise SystemExit(f"kgaps: {len(rows)} dispatches of {kern}")
    dur = sorted((e - s) / 1e3 for s, e in rows)
    gaps = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    per = [(rows[i + 1][0] - rows[i][0]) / 1e3 for i in range(len(rows) - 1)]
    print(json.dumps({"kernel": kern, "dispatches": len(rows),
                      "dur_us_mean": sum(dur) / len(dur), "dur_us_median": dur[len(dur) // 2],
                      "dur_us_min": dur[0], "dur_us_max": dur[-1],
                      "gap_us_mean": sum(gaps) / len(gaps),
                      "gap_us_median": sorted(gaps)[len(gaps) // 2],
                      "period_us_mean": sum(per) / len(per)}))


if __name__ == "__main__":
    main()

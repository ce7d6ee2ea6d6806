"""Per-kernel queue / stream map and durations of the update's dispatches in a rocprofv3
kernel trace (tools/capture_effect.py): for every kernel name, the (queue, stream) pairs
its dispatches ran on, with their count and mean duration.
Usage: python tools/queue_map.py run_kernel_trace.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    qcol = next((c for c in ("Queue_Id", "Queue_ID", "queue_id") if c in rows[0]), None)
    scol = next((c for c in ("Stream_Id", "Stream_ID", "stream_id") if c in rows[0]), None)
    print("columns:", ",".join(rows[0].keys()))
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].split("<")[0][-40:]
        key = (name, r.get(qcol, "?"), r.get(scol, "?"))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, q, s), d in sorted(agg.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        print(f"{name:40s} queue={q:>4s} stream={s:>4s} n={len(d):4d} mean={sum(d) / len(d):9.1f} us")


if __name__ == "__main__":
    main()

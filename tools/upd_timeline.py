"""Timeline of one update pipeline (k_build_keys .. k_sgd_combine) from a rocprofv3
kernel trace: start offset, gap and duration of every launch.
Usage: python tools/upd_timeline.py run_kernel_trace.csv [which-call]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_sgd_combine" in r["Kernel_Name"] or "k_sgd_tail" in r["Kernel_Name"]]
j = ends[int(sys.argv[2]) if len(sys.argv) > 2 else len(ends) // 2]
i = j
while "k_build_keys" not in rows[i]["Kernel_Name"]:
    i -= 1
t0 = prev = int(rows[i]["Start_Timestamp"])
for r in rows[i:j + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} gap={(s - prev) / 1e3:6.1f} dur={(e - s) / 1e3:8.1f} "
          f"{r['Kernel_Name'][:48]}")
    prev = e
print(f"total {(prev - t0) / 1e3:.1f} us")

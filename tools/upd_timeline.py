"""Timeline of one update pipeline (k_build_keys .. the last kernel before the next
k_build_keys) from a rocprofv3 kernel trace: start offset, gap and duration of every
launch.  Works for the split (.. k_sgd_tail) and exact (.. k_sgd_exact) modes.
Usage: python tools/upd_timeline.py run_kernel_trace.csv [which-call]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_build_keys" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
i = starts[k]
j = starts[k + 1] if k + 1 < len(starts) else len(rows)
# stop at the first kernel that is not part of the update (a lookup, a fill, a copy)
end = i
for q in range(i, j):
    n = rows[q]["Kernel_Name"]
    if "k_pooled" in n or "k_fill" in n or "elementwise" in n.lower() or "copy" in n.lower():
        break
    end = q
# the early-chain plans (side streams) may start just before k_build_keys
while i > 0 and ("k_ec_" in rows[i - 1]["Kernel_Name"] or "k_eh_" in rows[i - 1]["Kernel_Name"]):
    i -= 1
t0 = prev = last = int(rows[i]["Start_Timestamp"])
for r in rows[i:end + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} gap={(s - prev) / 1e3:6.1f} dur={(e - s) / 1e3:8.1f} "
          f"{r['Kernel_Name'][:60]}")
    prev = e
    last = max(last, e)
print(f"total {(last - t0) / 1e3:.1f} us")

"""Timeline of one update call across the caller's stream and the library's side stream
(exact mode's early chains) from a rocprofv3 kernel trace: start and end offsets from the
call's first kernel, duration and queue of every kernel.
Usage: python tools/upd_streams.py run_kernel_trace.csv [which-call]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a call starts at its first k_build_keys (main) or k_ec_count (side), whichever is first
firsts = [i for i, r in enumerate(rows)
          if "k_build_keys" in r["Kernel_Name"] or "k_ec_count" in r["Kernel_Name"]]
calls = [firsts[0]]
for i in firsts[1:]:
    if int(rows[i]["Start_Timestamp"]) - int(rows[calls[-1]]["Start_Timestamp"]) > 100_000:
        calls.append(i)
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(calls) // 2
i, j = calls[k], calls[k + 1] if k + 1 < len(calls) else len(rows)
t0 = int(rows[i]["Start_Timestamp"])
end = t0
for r in rows[i:j]:
    n = r["Kernel_Name"]
    if "k_pooled" in n or "k_fill" in n or "elementwise" in n.lower():
        break
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} dur={(e - s) / 1e3:8.1f} "
          f"q={r['Queue_Id']} {n[:56]}")
print(f"total {(end - t0) / 1e3:.1f} us")

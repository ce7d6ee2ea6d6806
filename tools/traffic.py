#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from tools/pmc_traffic.sh output.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reads exactly half of
the bytes of wide coalesced 16-B/lane reads (128-B requests tallied at 64 B), so it is
doubled; WRITE_SIZE (KiB) is exact for 16-B/lane stores.  Infinity-Cache hits are
counted by these fabric-side counters, so `hbm_bytes` is an upper bound on DRAM bytes.
Usage: tools/traffic.py PMC_DIR KERNEL_SUBSTRING WORKLOAD_TAG OUT_JSON
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(pmc_dir, tag, kernel):
    vals = {}
    for f in glob.glob(os.path.join(pmc_dir, tag, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (row["Counter_Name"], row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    by_counter = {}
    for (name, _), v in vals.items():
        by_counter.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in by_counter.items()}, {k: len(v) for k, v in by_counter.items()}


def main():
    pmc_dir, kernel, workload, out = sys.argv[1:5]
    res, n = {}, {}
    for tag in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum_TCC_MISS_sum",
                "TCC_EA0_RDREQ_sum_TCC_EA0_RDREQ_32B_sum"):
        r, c = per_dispatch(pmc_dir, tag, kernel)
        res.update(r)
        n.update(c)
    fetch = res.get("FETCH_SIZE")
    write = res.get("WRITE_SIZE")
    doc = {
        "workload": workload,
        "kernel": kernel,
        "dispatches": n,
        "raw_per_launch": res,
        "read_bytes_per_launch": 2 * 1024 * fetch if fetch is not None else None,
        "write_bytes_per_launch": 1024 * write if write is not None else None,
        "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of 128-B requests), "
                      "write = WRITE_SIZE KiB",
    }
    if fetch is not None and write is not None:
        doc["hbm_bytes_per_launch"] = doc["read_bytes_per_launch"] + doc["write_bytes_per_launch"]
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        doc["l2_hit_rate"] = res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()

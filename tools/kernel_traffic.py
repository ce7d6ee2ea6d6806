"""Fabric traffic per kernel name from separate rocprofv3 --pmc passes (one counter group per
pass, as tools/pmc_traffic.sh runs them), for a program that runs several kinds of kernel
(e.g. the exact update: sort, plans, chunk pass, chains).

For every kernel name (template arguments cut): dispatches, mean duration (from the
FETCH_SIZE pass's timestamps), fabric read bytes (2 x FETCH_SIZE KiB, the gfx950 correction,
MI355X_MICROARCH.md), write bytes (WRITE_SIZE KiB), both per dispatch, and the implied rate.
Under PMC collection kernels run one at a time, so the durations are serialised times.
Usage: python tools/kernel_traffic.py PMC_DIR [skip_dispatches] > out.txt"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)


def load(pmc_dir, tag, counter):
    vals, durs = defaultdict(dict), defaultdict(dict)
    for f in glob.glob(os.path.join(pmc_dir, tag, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                k, d = short(r["Kernel_Name"]), int(r["Dispatch_Id"])
                vals[k][d] = vals[k].get(d, 0.0) + float(r["Counter_Value"])
                durs[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return vals, durs


def main():
    pmc_dir = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    fetch, durs = load(pmc_dir, "FETCH_SIZE", "FETCH_SIZE")
    write, _ = load(pmc_dir, "WRITE_SIZE", "WRITE_SIZE")
    rows = []
    for k in fetch:
        ds = sorted(fetch[k])[skip:] or sorted(fetch[k])
        n = len(ds)
        rd = 2 * 1024 * sum(fetch[k][d] for d in ds) / n
        ws = sorted(write.get(k, {}))
        wd = 1024 * sum(write[k][d] for d in ws) / len(ws) if ws else 0.0
        us = sum(durs[k][d] for d in ds) / n
        rows.append((rd + wd, k, n, us, rd, wd))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'n':>4s} {'us':>9s} {'read MB':>9s} {'write MB':>9s} {'TB/s':>6s}")
    for tot, k, n, us, rd, wd in rows:
        print(f"{k[:60]:60s} {n:4d} {us:9.1f} {rd / 1e6:9.1f} {wd / 1e6:9.1f} "
              f"{tot / (us * 1e-6) / 1e12 if us else 0:6.2f}")


if __name__ == "__main__":
    main()

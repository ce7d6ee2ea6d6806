"""Per-kernel means of arbitrary PMC counters from one rocprofv3 --pmc pass (any counter set,
e.g. SQ_WAVE_CYCLES SQ_WAIT_ANY ... for the exact update's plan kernels).

For every kernel name (template arguments cut) matching the optional filter: dispatches, mean
duration (serialised: PMC collection runs kernels one at a time) and the per-dispatch mean of
each counter.  Usage: python tools/kernel_counters.py PMC_DIR [name_regex] > out.txt"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"^void ", "", re.sub(r"\(.*", "", name))


def main():
    pmc_dir = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    vals = defaultdict(lambda: defaultdict(dict))
    durs = defaultdict(dict)
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, d = short(r["Kernel_Name"]), int(r["Dispatch_Id"])
                if pat and not pat.search(k):
                    continue
                c = r["Counter_Name"]
                vals[k][c][d] = vals[k][c].get(d, 0.0) + float(r["Counter_Value"])
                durs[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k in sorted(durs, key=lambda k: -sum(durs[k].values()) / len(durs[k])):
        n = len(durs[k])
        line = f"{k[:48]:48s} n={n:3d} us={sum(durs[k].values()) / n:9.1f}"
        for c in sorted(vals[k]):
            v = vals[k][c]
            line += f"  {c}={sum(v.values()) / len(v):.4g}"
        print(line)


if __name__ == "__main__":
    main()

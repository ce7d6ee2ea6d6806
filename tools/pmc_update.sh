#!/bin/bash
# L2 hit / fabric reads of the update's chunk passes (tools/upd_only.py), one counter
# group per rocprofv3 pass.  Usage: tools/pmc_update.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc_upd}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $OUT
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo "$grp" | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/$tag" -o run --output-format csv -- python3 tools/upd_only.py > "$OUT/$tag.log" 2>&1 || { echo PMC_FAIL $tag; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'sgd' in n or 'combine' in n:
            agg[n[:36]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    hit = m.get('TCC_HIT_sum'); miss = m.get('TCC_MISS_sum')
    print(k, {c: f"{x:.3g}" for c, x in m.items()}, 'hit', f"{hit / (hit + miss):.2f}" if hit else '')
PY

#!/bin/bash
# Run the bench under rocprofv3 once per PMC counter group (no trace domains).
# Usage: tools/pmc_groups.sh OUTDIR "GROUP1" "GROUP2" ...   (env passes through to bench)
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for grp in "$@"; do
  tag=$(echo "$grp" | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/$tag" -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --cpu-seconds 0} > "$OUT/$tag.log" 2>&1
done

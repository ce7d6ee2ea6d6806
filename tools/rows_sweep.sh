#!/bin/bash
# Pooled-lookup rate vs table footprint (26 equal dim-128 fp32 tables, pool 20, B 65536):
# where the random-row gather rate falls from the Infinity-Cache rate to the HBM rate.
set -o pipefail
OUT=${1:-gpurun_out/rows_sweep}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for rows in 20000 40000 90000 180000 360000 1000000 3000000 10000000; do
  timeout -k 10 200 python3 bench.py --rows $rows --no-extra --cpu-seconds 0 --no-check --steps 30 --warmup 3 > "$OUT/r$rows.json" 2> "$OUT/r$rows.err" || { echo FAIL $rows; tail -5 "$OUT/r$rows.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/r$rows.json')); r=d['roofline']; print($rows, 26*$rows*512/1e9, 'GB', round(r['kernel_ms'],4), 'ms', round(r['algorithmic_GBs']), 'GB/s')"
done

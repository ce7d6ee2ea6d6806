#!/bin/bash
# HBM traffic of the bench's dominant kernel from rocprofv3 PMC counters.
# One counter group per rocprofv3 run (FETCH_SIZE and WRITE_SIZE cannot share a pass
# on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC slots"); no trace domains beside --pmc.
# Usage: tools/pmc_traffic.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:-"--steps 5 --warmup 1 --cpu-seconds 0"}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo "$grp" | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/$tag" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/$tag.log" 2>&1
done

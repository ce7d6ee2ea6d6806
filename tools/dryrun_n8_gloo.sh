#!/bin/bash
# 8 gloo ranks sharing the box's one GPU run bench.py --gpus 8 (host-staged exchange):
# checks the N = 8 plan (4,4,3,3,3,3,3,3 table-wise; equal feature ranges feature-wise)
# and that every rank holds only its own tables / slices (per_rank.table_bytes).
set -o pipefail
OUT=${1:-gpurun_out/dryrun8}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for plan in tablewise featurewise; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --backend gloo --plan $plan \
    --batch 4096 --steps 2 --warmup 1 --no-alltoall > "$OUT/$plan.json" 2> "$OUT/$plan.err" \
    || { echo DRYRUN_FAIL $plan; tail -20 "$OUT/$plan.err"; exit 1; }
  echo "$plan ok"
done

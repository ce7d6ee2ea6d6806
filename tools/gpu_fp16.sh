#!/bin/bash
# Round 4: the config-3 Float16 leg under lookup schedule knobs (no rebuild).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fp16; mkdir -p $OUT
for r in 1 2; do for v in "ET_X=0" "ET_LIGHT_BYTES=2097152" "ET_LIGHT_BYTES=1048576" "ET_NTLOAD_BYTES=134217728" "ET_SCHED=stripe" "ET_NTLOAD=0"; do
  env $v timeout -k 10 200 python3 tools/fp16_leg.py > $OUT/f.txt 2>&1 || { echo FP16_FAIL $v; tail -5 $OUT/f.txt; exit 1; }
  echo "$v $(tail -1 $OUT/f.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["julia_f16_arith"]["kernel_ms"], d["fp32_accumulate"]["kernel_ms"])')"
done; done

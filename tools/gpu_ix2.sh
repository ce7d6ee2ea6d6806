#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ix2; mkdir -p $OUT
for v in "UPD_IX_CHURN=" "UPD_IX_CHURN=alloc" "UPD_IX_CHURN=alloc,free"; do
  env $v timeout -k 10 200 python3 tools/upd_ix.py 10 2 > $OUT/ix.txt 2>&1 || { echo IX_FAIL $v; tail -5 $OUT/ix.txt; exit 1; }
  echo "$v $(tail -1 $OUT/ix.txt)"
done
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().split(chr(10))[-1]); c=d['config4_zipf_update']; print('bench', c['update_exact_ms'], c['update_split_ms'], c['forward_ms'])"

#!/bin/bash
# Round 4: feature-split tables in the headline lookup (ET_FSPLIT_BYTES / ET_FSPLIT_G).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fsplit; mkdir -p $OUT
for g in 4 8; do
ET_FSPLIT_BYTES=16777216 ET_FSPLIT_G=$g timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k config3 --timeout 300 --timeout-method thread > $OUT/pytest_g$g.log 2>&1 || { echo FS_TEST_FAIL $g; tail -30 $OUT/pytest_g$g.log; exit 1; }
echo "g$g $(tail -1 $OUT/pytest_g$g.log)"
done
for r in 1 2; do for v in "ET_X=0" "ET_FSPLIT_BYTES=16777216 ET_FSPLIT_G=4" "ET_FSPLIT_BYTES=16777216 ET_FSPLIT_G=8" "ET_FSPLIT_BYTES=16777216 ET_FSPLIT_G=2" "ET_FSPLIT_BYTES=67108864 ET_FSPLIT_G=8"; do
  env $v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extra --cpu-seconds 0 > $OUT/bench_q.txt 2>&1 || { echo BENCH_FAIL $v; tail -5 $OUT/bench_q.txt; exit 1; }
  echo "$v $(tail -1 $OUT/bench_q.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"])')"
done; done
for r in 1 2; do for v in "ET_PLAN_GATE=0" "ET_PLAN_GATE=1" "ET_PLAN_GATE=2" "ET_PLAN_GATE=3"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
for r in 1 2; do for v in "ET_CHAIN_LDS=40" "ET_CHAIN_LDS=40 ET_CHAIN_WG=256" "ET_CHAIN_LDS=20 ET_CHAIN_WG=384"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done

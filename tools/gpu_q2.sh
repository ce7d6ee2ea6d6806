#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/q2; mkdir -p $OUT
for q in 1 2; do
ET_QORDER=$q timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k config3 --timeout 300 --timeout-method thread > $OUT/pytest_q$q.log 2>&1 || { echo QTEST_FAIL $q; tail -30 $OUT/pytest_q$q.log; exit 1; }
echo "q$q $(tail -1 $OUT/pytest_q$q.log)"
done
for r in 1 2; do for v in "ET_QORDER=0" "ET_QORDER=1" "ET_QORDER=2" "ET_HEAVY_PRIO=1"; do
  env $v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extra --cpu-seconds 0 > $OUT/bench_q.txt 2>&1 || { echo BENCH_FAIL $v; tail -5 $OUT/bench_q.txt; exit 1; }
  echo "$v $(tail -1 $OUT/bench_q.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"])')"
done; done

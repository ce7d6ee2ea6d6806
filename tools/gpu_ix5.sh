#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ix5; mkdir -p $OUT
for v in "ET_SIDE_CUMASK=1" "ET_X=0"; do
env $v timeout -k 10 300 python3 tools/cfg4_only.py config2 > $OUT/c4.txt 2>&1 || { echo C4_FAIL; tail -5 $OUT/c4.txt; exit 1; }
echo "$v $(tail -1 $OUT/c4.txt)"
done
ET_SIDE_CUMASK=1 timeout -k 10 300 python3 tools/cfg4_only.py > $OUT/c4.txt 2>&1 || { echo C4_FAIL; tail -5 $OUT/c4.txt; exit 1; }
echo "cumask, no config2 $(tail -1 $OUT/c4.txt)"
for r in 1 2; do for v in "ET_X=0" "ET_LIGHT_BYTES=8388608" "ET_LIGHT_BYTES=16777216"; do
  env $v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extra --cpu-seconds 0 > $OUT/bench_q.txt 2>&1 || { echo BENCH_FAIL $v; tail -5 $OUT/bench_q.txt; exit 1; }
  echo "$v $(tail -1 $OUT/bench_q.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"])')"
done; done

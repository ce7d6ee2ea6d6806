#!/bin/bash
# Round 4: headline A/B, the final lookup vs the build before the feature-split change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/headab; mkdir -p $OUT
ALT=$PWD/tools/alt/libembtab_hip_alt.so
for r in 1 2; do for v in "ET_X=0" "ET_LIBRARY=$ALT"; do
  env $v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extra --cpu-seconds 0 > $OUT/b.txt 2>&1 || { echo BENCH_FAIL $v; tail -5 $OUT/b.txt; exit 1; }
  echo "${v##*/} $(tail -1 $OUT/b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"])')"
done; done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_fullsize.py -x -q -m gpu -k "not config4" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
echo "tests $(tail -1 $OUT/pytest.log)"
timeout -k 10 200 python3 tools/fp16_leg.py > $OUT/f.txt 2>&1 || { echo FP16_FAIL; tail -5 $OUT/f.txt; exit 1; }
echo "fp16 $(tail -1 $OUT/f.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["julia_f16_arith"]["kernel_ms"], d["fp32_accumulate"]["kernel_ms"])')"

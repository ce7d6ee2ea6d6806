#!/bin/bash
# Round 4: ds_bpermute broadcasts for 4-group waves (256-byte rows): parity, fp16-leg A/B
# against the round-3 readlane broadcast (tools/alt/libembtab_hip_alt.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/bcast; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_generic_tables.py tests/test_gpu_split.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
echo "lookup tests $(tail -1 $OUT/pytest.log)"
ALT=$PWD/tools/alt/libembtab_hip_alt.so
for r in 1 2; do for v in "ET_X=0" "ET_LIBRARY=$ALT"; do
  env $v timeout -k 10 200 python3 tools/fp16_leg.py > $OUT/f.txt 2>&1 || { echo FP16_FAIL $v; tail -5 $OUT/f.txt; exit 1; }
  echo "${v##*/} $(tail -1 $OUT/f.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["julia_f16_arith"]["kernel_ms"], d["fp32_accumulate"]["kernel_ms"])')"
  env $v timeout -k 10 200 python3 tools/fp16_classes.py > $OUT/c.txt 2>&1 || { echo FP16C_FAIL $v; tail -5 $OUT/c.txt; exit 1; }
  echo "  classes $(tail -1 $OUT/c.txt)"
done; done

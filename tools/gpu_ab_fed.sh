#!/bin/bash
# Round 4: fed chains (ET_CHAIN_FED=1: S = 1 plans walked by a summing wave + 3 gatherer
# waves through an LDS ring) and the 64-deep ring loop (ET_CHAIN_RING=1): parity on the
# exact GPU tests, then timings of one exact config-4 update per variant, and kernel traces.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fed; mkdir -p $OUT
ET_CHAIN_FED=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_fed.log 2>&1 || { echo FED_TEST_FAIL; tail -30 $OUT/pytest_fed.log; exit 1; }
tail -1 $OUT/pytest_fed.log
for v in base fed ring; do
  case $v in base) E="";; fed) E="ET_CHAIN_FED=1";; ring) E="ET_CHAIN_RING=1";; esac
  env $E timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4_$v.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4_$v.txt)"
done
ET_CHAIN_FED=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k exact --timeout 300 --timeout-method thread > $OUT/pytest_fed_full.log 2>&1 || { echo FED_FULL_FAIL; tail -30 $OUT/pytest_fed_full.log; exit 1; }
tail -1 $OUT/pytest_fed_full.log
ET_CHAIN_FED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && grep -E "chains|sgd_exact|total" $OUT/exact_timeline.txt
# 256-byte rows on the scalar-addressed loop (ET_SG256=1): lookup parity, fp16 leg A/B
ET_SG256=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_sg256.log 2>&1 || { echo SG256_TEST_FAIL; tail -30 $OUT/pytest_sg256.log; exit 1; }
tail -1 $OUT/pytest_sg256.log
for i in 1 2; do for v in 0 1; do
  ET_SG256=$v timeout -k 10 200 python3 tools/fp16_leg.py > $OUT/fp16_${v}_$i.txt 2>&1 || { echo FP16_FAIL; tail -5 $OUT/fp16_${v}_$i.txt; exit 1; }
  echo "SG256=$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/fp16_${v}_$i.txt').read().strip().splitlines()[-1]); print(round(d['julia_f16_arith']['kernel_ms'],4), round(d['fp32_accumulate']['kernel_ms'],4))")"
done; done

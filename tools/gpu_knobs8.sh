#!/bin/bash
# Round 4: EH chain placement (exclusive or not, LDS reservation, workgroups) at the new
# defaults (EH on, exact grid cap 512), then the exact GPU tests at the defaults.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/knobs8; mkdir -p $OUT
for r in 1 2; do for v in "ET_X=0" "ET_CHAIN_EXCL=1" "ET_CHAIN_EXCL=1 ET_EH_LDS=40 ET_EH_WG=64" "ET_CHAIN_EXCL=1 ET_EH_LDS=20 ET_EH_WG=128" "ET_CHAIN_EXCL=1 ET_EH_LDS=40 ET_EH_WG=48" "ET_CHAIN_EXCL=5 ET_EH_WG=40"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_upd.log 2>&1 || { echo UPD_TEST_FAIL; tail -30 $OUT/pytest_upd.log; exit 1; }
echo "upd $(tail -1 $OUT/pytest_upd.log)"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_full.log 2>&1 || { echo FULL_TEST_FAIL; tail -30 $OUT/pytest_full.log; exit 1; }
echo "full $(tail -1 $OUT/pytest_full.log)"

#!/bin/bash
# Update pipeline metadata passes: GPU parity tests of the update, then the config-4
# update alone (update_ms) and its rocprofv3 kernel stats.  Usage: tools/exp_meta.sh TAG
set -o pipefail
TAG=${1:-a}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/meta_$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullsize.py tests/test_gpu_split.py tests/test_gpu_generic_tables.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 tools/upd_only.py > $OUT/upd.txt 2>&1 || { echo UPD_FAIL; tail -20 $OUT/upd.txt; exit 1; }
cat $OUT/upd.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/upd_only.py > $OUT/upd_traced.txt 2> $OUT/prof_stderr.log || { echo TRACE_FAIL; tail -5 $OUT/prof_stderr.log; exit 1; }
echo trace ok

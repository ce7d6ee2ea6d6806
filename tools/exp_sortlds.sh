#!/bin/bash
# Radix-scatter experiment: update parity tests, config-4 update time, kernel stats.
set -o pipefail
OUT=${1:-gpurun_out/sortlds}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullsize.py tests/test_gpu_generic_tables.py tests/test_gpu_lookup.py tests/test_gpu_split.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 tools/upd_only.py > $OUT/upd.txt 2>&1 && tail -1 $OUT/upd.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/upd_only.py > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
python3 - $OUT <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1] + '/trace/run_kernel_stats.csv')))
for x in r:
    if any(k in x['Name'] for k in ('k_rs', 'k_build', 'k_sgd_chunks', 'index')):
        print(f"{x['Name'][:60]:60s} {x['Calls']:>5} {float(x['AverageNs'])/1e3:9.1f} us")
PY

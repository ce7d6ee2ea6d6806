#!/bin/bash
# Round-2 evidence for the final tree: GPU tests, default bench line, rocprofv3 kernel
# trace of the same bench command, PMC traffic passes of the headline kernel (one
# counter group per run), traffic summary.  Usage: tools/profile_r02.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r02_final}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $OUT/bench_traced.json 2> $OUT/prof_stderr.log || { echo TRACE_FAIL; tail -5 $OUT/prof_stderr.log; exit 1; }
echo trace ok
bash tools/pmc_traffic.sh $OUT/pmc --steps 5 --warmup 1 --cpu-seconds 0 --no-extra || { echo PMC_FAIL; exit 1; }
python3 tools/traffic.py $OUT/pmc k_pooled_vec criteo26_b65536 $OUT/traffic.json | tail -1

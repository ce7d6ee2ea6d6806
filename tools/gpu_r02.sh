#!/bin/bash
# Round-2 GPU session: host probe, GPU parity tests, default bench line, kernel-trace
# profile of the bench (rocprofv3 --kernel-trace --stats).  Usage: tools/gpu_r02.sh TAG
set -o pipefail
TAG=${1:-a}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_$TAG
mkdir -p $OUT
python3 -c "
import os
print('os.cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))
for f in ('/sys/fs/cgroup/cpu.max', '/proc/loadavg'):
    try: print(f, open(f).read().strip())
    except OSError as e: print(f, e)
" > $OUT/host.txt 2>&1; nproc >> $OUT/host.txt; grep -m1 'model name' /proc/cpuinfo >> $OUT/host.txt
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_traced.json 2> $OUT/prof_stderr.log || { echo TRACE_FAIL; tail -5 $OUT/prof_stderr.log; exit 1; }
echo trace ok

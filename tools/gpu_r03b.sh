#!/bin/bash
# Round 3: headline workgroup timeline, config-2 launch gaps (kernel trace), exact-update knobs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 150 python3 tools/wg_timeline.py $OUT/wg_timeline.json > $OUT/wg_timeline.txt 2>&1 || { echo TL_FAIL; tail -5 $OUT/wg_timeline.txt; exit 1; }
echo timeline ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { echo TRACE_FAIL; tail -5 $OUT/bench_traced.err; exit 1; }
f=$(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/gap_stats.py "$f" k_gather_vec > $OUT/config2_gaps.txt && cat $OUT/config2_gaps.txt
python3 tools/gap_stats.py "$f" k_pooled_vec_striped > $OUT/headline_gaps.txt && cat $OUT/headline_gaps.txt
bash tools/ab_exact.sh knobs "-" "ET_EC_WG=32 ET_CHAIN_WG=128" "ET_EC_WG=64 ET_CHAIN_WG=192" "ET_EC_WG=16 ET_CHAIN_WG=96"

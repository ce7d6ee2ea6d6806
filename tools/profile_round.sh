set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_v6 gpurun_out/pmc_v6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v6 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_v6/bench_traced.json 2> gpurun_out/prof_v6/stderr.log || { echo TRACE_FAIL; tail -5 gpurun_out/prof_v6/stderr.log; exit 1; }
echo trace ok
bash tools/pmc_traffic.sh gpurun_out/pmc_v6 --steps 5 --warmup 1 --cpu-seconds 0 --no-extra || { echo PMC_FAIL; exit 1; }
echo pmc ok
python3 tools/traffic.py gpurun_out/pmc_v6 k_pooled_vec criteo26_b65536 gpurun_out/pmc_v6/traffic.json | tail -1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_v6f.json 2> gpurun_out/bench_v6f.err || { echo BENCH_FAIL; exit 1; }
echo bench ok

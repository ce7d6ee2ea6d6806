#!/bin/bash
# Chunk-pass order experiment: config-4 update time and the chunk
# pass's kernel time / fabric traffic for the spaced (ET_SGD_ORDER=0) and windowed
# (16 / 64 chunks per grab) orders.  Usage: tools/sgd_order_exp.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/sgd_order}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in "0 2048" "16 2048" "64 2048" "16 4096" "16 1024"; do
  set -- $cfg
  ET_SGD_ORDER=$1 ET_SGD_WGRID=$2 timeout -k 10 200 python3 tools/upd_only.py > "$OUT/upd_$1_$2.txt" 2>&1 || { echo UPD_FAIL $cfg; tail -5 "$OUT/upd_$1_$2.txt"; exit 1; }
  echo "order $1 grid $2: $(tail -1 $OUT/upd_$1_$2.txt)"
done
for o in 0 16; do
  ET_SGD_ORDER=$o timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$o" -o run --output-format csv -- python3 tools/upd_only.py > "$OUT/trace_$o.log" 2>&1 || { echo TRACE_FAIL; exit 1; }
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo "$grp" | tr ' ' '_')
    ET_SGD_ORDER=$o timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc_${o}_$tag" -o run --output-format csv -- python3 tools/upd_only.py > "$OUT/pmc_${o}_$tag.log" 2>&1 || { echo PMC_FAIL; exit 1; }
  done
done
echo done

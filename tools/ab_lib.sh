#!/bin/bash
# A/B two builds of the library on one box (config-4 update), then parity tests on B.
# Put the two builds at abtmp/libA.so and abtmp/libB.so (git-ignored) before the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
LIB=embeddingtables.jl_amd/embtab/libembtab_hip.so
OUT=gpurun_out/ab_lib; mkdir -p $OUT
for i in 1 2; do for v in A B; do
  cp abtmp/lib$v.so $LIB
  timeout -k 10 200 python3 tools/upd_only.py > $OUT/r_${v}_$i.txt 2>&1 || { echo FAIL; tail -5 $OUT/r_${v}_$i.txt; exit 1; }
  echo "lib=$v $(tail -1 $OUT/r_${v}_$i.txt)"
done; done
cp abtmp/libB.so $LIB
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_B.log 2>&1; tail -1 $OUT/pytest_B.log

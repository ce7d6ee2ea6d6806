#!/bin/bash
# A/B of an environment switch on the config-4 update, alternating on one box.
# Usage: tools/ab_env.sh TAG VAR ROUNDS   (runs VAR=0 and VAR=1 ROUNDS times each)
set -o pipefail
TAG=$1; VAR=$2; N=${3:-3}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python3 tools/upd_only.py > $OUT/run_${v}_$i.txt 2>&1 || { echo FAIL; tail -5 $OUT/run_${v}_$i.txt; exit 1; }
    echo "$VAR=$v $(tail -1 $OUT/run_${v}_$i.txt)"
  done
done

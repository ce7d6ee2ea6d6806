#!/bin/bash
# One parametrised GPU-box runner (replaces the round 1-4 one-off gpu_*.sh scripts).
# Every step runs under its own time limit; the first failing step ends the call.
#
# Usage: tools/gpu_run.sh TAG STEP [STEP ...]      (outputs under gpurun_out/TAG/)
#   tests            pytest -m gpu (all GPU tests)
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (the driver's default run) -> bench.json
#   trace            rocprofv3 --kernel-trace --stats of bench.py --steps 20 --warmup 3
#   tracehead        the same with --no-extra (only the headline launches)
#   pmc              PMC traffic of the headline kernel (tools/pmc_traffic.sh, tools/traffic.py)
#   exact            kernel trace of one exact config-4 update + its timeline
#   cfg2             config 2: kernel trace (graph and eager: duration vs gap) + PMC traffic
#   classpmc         PMC traffic + time of each headline table class alone (tools/class_pmc.py)
#   lookab:LIB:S1/S2:N  the headline launch (kernel ms) with library LIB and env sets S1, S2
#                    (VAR=V,VAR=V; NONE=0 for none), alternating N times
#   expexact:VAR=V,..  the exact step with the experiment build and env VAR=V
#   upd:N            the config-4 update alone, N processes (tools/upd_only.py)
#   ab:A:B:N         the config-4 update with library builds A and B (paths), alternating N times
#   env:VAR=V,..:N   the config-4 update with the experiment build and env VAR=V (N times)
#   capture:M1,M2..  the update after each tools/capture_effect.py mode (none, capture, dummyN ...)
#   expcapture:VAR=V,..:M1,M2..  the same with the experiment build and env VAR=V
#   py:SCRIPT[:ARGS] python3 tools/SCRIPT ARGS (ARGS: '+'-separated)
#   exppy:SCRIPT[:ARGS]  the same with the experiment build (tools/exp_build.sh)
set -o pipefail
# the package loads an experiment build (ET_LIBRARY=tools/exp/...) only with this opt-in
export ET_TOOLS_EXPERIMENT=1
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
LIB=embeddingtables.jl_amd/embtab/libembtab_hip.so
EXP=tools/exp/libembtab_hip_exp.so

die() { echo "FAIL $1"; tail -25 "$2"; exit 1; }

for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || die tests "$OUT/pytest_gpu.log"
      tail -1 "$OUT/pytest_gpu.log" ;;
    tests:*)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -k "${step#tests:}" > "$OUT/pytest_k.log" 2>&1 || die tests "$OUT/pytest_k.log"
      tail -1 "$OUT/pytest_k.log" ;;
    exptests:*)
      # pytest -m gpu -k EXPR with the experiment build and env VAR=V,..: exptests:VAR=V,..:EXPR
      IFS=: read -r _ SETS EXPR <<< "$step"
      env ET_LIBRARY=$EXP $(echo "$SETS" | tr ',' ' ') timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v \
        --timeout 300 --timeout-method thread -k "$EXPR" > "$OUT/pytest_exp.log" 2>&1 || die exptests "$OUT/pytest_exp.log"
      echo "$SETS $(tail -1 "$OUT/pytest_exp.log")" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || die smoke "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 500 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || die bench "$OUT/bench.err"
      python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); c=d.get('config4_zipf_update',{}); \
print('bench', round(d['ms_per_step'],4), 'ms frac', round(d['roofline']['frac'],4), 'upd', round(c.get('update_exact_ms',0),3), \
'split', round(c.get('update_split_ms',0),3), 'fp16', round(d.get('config3_fp16',{}).get('julia_f16_arith',{}).get('kernel_ms',0),4), \
'cfg2_us', round(1e3*d.get('config2_gather',{}).get('kernel_ms',0),2))" ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
        -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > "$OUT/bench_traced.json" \
        2> "$OUT/bench_traced.err" || die trace "$OUT/bench_traced.err"
      echo "trace ok" ;;
    tracehead)
      # the headline launch alone (no extra configs), so the kernel's rocprof average is its time
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_head" -o run --output-format csv \
        -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extra > "$OUT/bench_head.json" \
        2> "$OUT/bench_head.err" || die tracehead "$OUT/bench_head.err"
      echo "tracehead ok" ;;
    pmc)
      bash tools/pmc_traffic.sh "$OUT/pmc" --steps 5 --warmup 1 --cpu-seconds 0 --no-extra || die pmc /dev/null
      python3 tools/traffic.py "$OUT/pmc" k_pooled_vec criteo26_b65536 "$OUT/pmc/traffic.json" | tail -1 ;;
    exact)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_exact" -o run --output-format csv \
        -- python3 tools/exact_cfg4.py exact > "$OUT/exact_traced.txt" 2>&1 || die exact "$OUT/exact_traced.txt"
      f=$(ls "$OUT"/prof_exact/*/run_kernel_trace.csv "$OUT"/prof_exact/run_kernel_trace.csv 2>/dev/null | head -1)
      python3 tools/upd_timeline.py "$f" > "$OUT/exact_timeline.txt" && grep -E "chains|sgd_exact|total" "$OUT/exact_timeline.txt" ;;
    updpmc)
      # fabric traffic per kernel of the exact config-4 update (tools/exact_cfg4.py, one call)
      D=$OUT/updpmc; mkdir -p "$D"
      for grp in "FETCH_SIZE" "WRITE_SIZE"; do
        timeout -s KILL 120 rocprofv3 --pmc $grp -d "$D/$grp" -o run --output-format csv \
          -- python3 tools/exact_cfg4.py exact > "$D/$grp.log" 2>&1 || die "updpmc $grp" "$D/$grp.log"
      done
      python3 tools/kernel_traffic.py "$D" > "$D/per_kernel.txt" && head -25 "$D/per_kernel.txt" ;;
    classpmc|expclasspmc:*)
      # expclasspmc:VAR=V,..: the same passes with the experiment build and env VAR=V
      SETS=""; LIBV=""; CD=classpmc
      if [ "$step" != classpmc ]; then SETS=${step#expclasspmc:}; LIBV=$EXP; CD=classpmc_exp; fi
      for c in heavy mid light all; do
        D=$OUT/$CD/$c; mkdir -p "$D"
        env ET_LIBRARY=$LIBV $(echo "$SETS" | tr ',' ' ') timeout -k 10 120 python3 tools/class_pmc.py $c 10 \
          > "$D/time.json" 2> "$D/time.err" || die classpmc "$D/time.err"
        for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
          tag=$(echo "$grp" | tr ' ' '_')
          env ET_LIBRARY=$LIBV $(echo "$SETS" | tr ',' ' ') timeout -s KILL 100 rocprofv3 --pmc $grp -d "$D/$tag" -o run --output-format csv \
            -- python3 tools/class_pmc.py $c 5 > "$D/$tag.log" 2>&1 || die "classpmc $c $tag" "$D/$tag.log"
        done
        python3 tools/traffic.py "$D" k_pooled_vec "class_$c" "$D/traffic.json" > /dev/null
        python3 -c "import json; t=json.load(open('$D/time.json')); d=json.load(open('$D/traffic.json')); \
print('$SETS $c', t['tables'], 'tables', round(t['ms_median'],4), 'ms', 'fabric', round(d.get('hbm_bytes_per_launch',0)/1e9,3), 'GB', \
'compulsory', round(t['hbm_compulsory_bytes']/1e9,3), 'GB', 'alg', round(t['algorithmic_bytes']/1e9,3), 'GB', 'L2hit', round(d.get('l2_hit_rate',0),3))"
      done ;;
    cfg2)
      D=$OUT/cfg2; mkdir -p "$D"
      for m in graph eager; do
        arg=$([ $m = eager ] && echo "--eager" || echo "")
        timeout -k 10 200 rocprofv3 --kernel-trace -d "$D/trace_$m" -o run --output-format csv \
          -- python3 tools/cfg2_trace.py 20 $arg > "$D/time_$m.json" 2> "$D/trace_$m.err" || die cfg2 "$D/trace_$m.err"
        f=$(ls "$D"/trace_$m/*/run_kernel_trace.csv "$D"/trace_$m/run_kernel_trace.csv 2>/dev/null | head -1)
        python3 tools/kgaps.py "$f" k_gather 64 > "$D/gaps_$m.json"
        echo "$m $(cat "$D/time_$m.json") $(cat "$D/gaps_$m.json")"
      done
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
        tag=$(echo "$grp" | tr ' ' '_')
        timeout -s KILL 100 rocprofv3 --pmc $grp -d "$D/$tag" -o run --output-format csv \
          -- python3 tools/cfg2_trace.py 5 --eager > "$D/$tag.log" 2>&1 || die "cfg2 $tag" "$D/$tag.log"
      done
      python3 tools/traffic.py "$D" k_gather cfg2 "$D/traffic.json" | cut -c1-400 ;;
    cfg2ab:*)
      # config 2 (graph-replayed, tools/cfg2_trace.py) with the experiment build and env sets
      IFS=: read -r _ SETSALL N <<< "$step"
      for i in $(seq 1 "${N:-2}"); do
        for SETS in $(echo "$SETSALL" | tr "/" " "); do
          env ET_LIBRARY=$EXP $(echo "$SETS" | tr ',' ' ') timeout -k 10 200 python3 tools/cfg2_trace.py 40 \
            > "$OUT/cfg2ab.json" 2> "$OUT/cfg2ab.err" || die cfg2ab "$OUT/cfg2ab.err"
          echo "$SETS $(cat "$OUT/cfg2ab.json")"
        done
      done ;;
    lookab:*)
      # the headline launch with experiment library A and env sets (VAR=V,...;VAR=V,...), N rounds
      IFS=: read -r _ LIBV SETSALL N <<< "$step"
      for i in $(seq 1 "${N:-2}"); do
        for SETS in $(echo "$SETSALL" | tr "/" " "); do
          env ET_LIBRARY=$LIBV $(echo "$SETS" | tr ',' ' ') timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 \
            --cpu-seconds 0 --no-extra --no-check > "$OUT/lookab.json" 2> "$OUT/lookab.err" || die lookab "$OUT/lookab.err"
          python3 -c "import json; d=json.load(open('$OUT/lookab.json')); print('$SETS', round(d['roofline']['kernel_ms'],4), round(d['roofline']['kernel_ms_median'],4))"
        done
      done ;;
    expexact:*)
      SETS=${step#expexact:}; T=$OUT/exp_$(echo "$SETS" | tr ',=' '__')
      env ET_LIBRARY=$EXP $(echo "$SETS" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d "$T" -o run --output-format csv -- python3 tools/exact_cfg4.py exact > "$T.txt" 2>&1 || die expexact "$T.txt"
      f=$(ls "$T"/*/run_kernel_trace.csv "$T"/run_kernel_trace.csv 2>/dev/null | head -1)
      python3 tools/upd_timeline.py "$f" > "$T.timeline" && echo "$SETS" && grep -E "chains|sgd_exact|total" "$T.timeline" ;;
    upd:*)
      for i in $(seq 1 "${step#upd:}"); do
        timeout -k 10 200 python3 tools/upd_only.py > "$OUT/upd_$i.txt" 2>&1 || die upd "$OUT/upd_$i.txt"
        echo "upd $(tail -1 "$OUT/upd_$i.txt")"
      done ;;
    ab:*)
      IFS=: read -r _ A B N <<< "$step"
      for i in $(seq 1 "${N:-2}"); do for v in A B; do
        lib=$([ $v = A ] && echo "$A" || echo "$B")
        ET_LIBRARY=$lib timeout -k 10 200 python3 tools/upd_only.py > "$OUT/ab_${v}_$i.txt" 2>&1 || die ab "$OUT/ab_${v}_$i.txt"
        echo "$v=$lib $(tail -1 "$OUT/ab_${v}_$i.txt")"
      done; done ;;
    env:*)
      IFS=: read -r _ SETS N <<< "$step"
      for i in $(seq 1 "${N:-1}"); do
        env ET_LIBRARY=$EXP $(echo "$SETS" | tr ',' ' ') timeout -k 10 200 python3 tools/upd_only.py \
          > "$OUT/env_$i.txt" 2>&1 || die env "$OUT/env_$i.txt"
        echo "$SETS $(tail -1 "$OUT/env_$i.txt")"
      done ;;
    capture:*)
      for m in $(echo "${step#capture:}" | tr ',' ' '); do
        timeout -k 10 240 python3 tools/capture_effect.py "$m" 10 >> "$OUT/capture_modes.jsonl" 2> "$OUT/capture_$m.err" \
          || die "capture $m" "$OUT/capture_$m.err"
        tail -1 "$OUT/capture_modes.jsonl"
      done ;;
    qmap:*)
      # kernel trace of the update after each capture_effect mode: queue / stream / duration
      for m in $(echo "${step#qmap:}" | tr ',' ' '); do
        timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/qmap_$m" -o run --output-format csv \
          -- python3 tools/capture_effect.py "$m" 5 > "$OUT/qmap_$m.json" 2> "$OUT/qmap_$m.err" \
          || die "qmap $m" "$OUT/qmap_$m.err"
        f=$(ls "$OUT"/qmap_$m/*/run_kernel_trace.csv "$OUT"/qmap_$m/run_kernel_trace.csv 2>/dev/null | head -1)
        python3 tools/queue_map.py "$f" > "$OUT/qmap_$m.txt" && rm -rf "$OUT/qmap_$m"
        echo "$m $(tail -1 "$OUT/qmap_$m.json")"
      done ;;
    benchargs:*)
      # the headline launch (kernel ms) with extra bench.py arguments ('+'-separated), e.g.
      # benchargs:--min-rows+313 (the tables above 312 rows only)
      A=$(echo "${step#benchargs:}" | tr '+' ' ')
      timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-extra --no-check $A \
        > "$OUT/benchargs.json" 2> "$OUT/benchargs.err" || die benchargs "$OUT/benchargs.err"
      python3 -c "import json; d=json.load(open('$OUT/benchargs.json')); print('$A', d['config']['tables'], 'tables', round(d['roofline']['kernel_ms'],4), round(d['roofline']['kernel_ms_median'],4))" ;;
    shardq)
      # queue / stream map of the world-1 sharded step (lookups + exchange stream), ADVICE r05
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/shardq" -o run --output-format csv \
        -- python3 bench.py --force-shard --steps 10 --warmup 2 --no-extra --cpu-seconds 0 \
        > "$OUT/shardq.json" 2> "$OUT/shardq.err" || die shardq "$OUT/shardq.err"
      f=$(ls "$OUT"/shardq/*/run_kernel_trace.csv "$OUT"/shardq/run_kernel_trace.csv 2>/dev/null | head -1)
      python3 tools/queue_map.py "$f" > "$OUT/shardq.txt" && rm -rf "$OUT/shardq"
      grep -E "queue" "$OUT/shardq.txt" | cut -c1-100 ;;
    expcapture:*)
      IFS=: read -r _ SETS MODES <<< "$step"
      for m in $(echo "$MODES" | tr ',' ' '); do
        env ET_LIBRARY=$EXP $(echo "$SETS" | tr ',' ' ') timeout -k 10 240 python3 tools/capture_effect.py "$m" 10 \
          > "$OUT/expcap.tmp" 2> "$OUT/expcap_$m.err" || die "expcapture $m" "$OUT/expcap_$m.err"
        echo "$SETS $(tail -1 "$OUT/expcap.tmp")" | tee -a "$OUT/expcapture.txt"
      done ;;
    py:*|exppy:*)
      IFS=: read -r KIND SCRIPT ARGS <<< "$step"
      LIBV=$([ "$KIND" = exppy ] && echo "$EXP" || echo "")
      ET_LIBRARY=$LIBV timeout -k 10 400 python3 "tools/$SCRIPT" $(echo "$ARGS" | tr '+' ' ') \
        > "$OUT/${SCRIPT%.py}.txt" 2>&1 || die "$SCRIPT" "$OUT/${SCRIPT%.py}.txt"
      tail -3 "$OUT/${SCRIPT%.py}.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

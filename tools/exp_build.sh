#!/bin/bash
# The EXPERIMENT build of the library: -DET_EXPERIMENTS compiles the tuning knobs' environment
# reads back in (ET_KNOB, csrc/et_common.h), the non-default kernel variants (the ET_W8 /
# ET_U lookup kernels, the queue orders) and the chain-item timeline
# (et_debug_chain_timeline).  Output: tools/exp/libembtab_hip_exp.so, loaded with
#   ET_LIBRARY=tools/exp/libembtab_hip_exp.so ET_<KNOB>=<value> python ...
# The package's own library (embtab/libembtab_hip.so) never reads the environment.
# EXTRA_DEFINES="A B" adds -DA -DB; EXP_NAME=x writes tools/exp/libembtab_hip_x.so instead
# (objects under tools/exp/obj_x), so a variant build leaves the default experiment build alone.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/exp
NAME=${EXP_NAME:-exp}
SUF=$([ "$NAME" = exp ] && echo "" || echo "_$NAME")
python3 - <<PY
import __graft_entry__ as g
g.build_hip(defines=["ET_EXPERIMENTS"] + "${EXTRA_DEFINES:-}".split(),
            lib="tools/exp/libembtab_hip_$NAME.so", obj_dir="tools/exp/obj$SUF")
PY
echo tools/exp/libembtab_hip_$NAME.so

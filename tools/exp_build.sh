#!/bin/bash
# The EXPERIMENT build of the library: -DET_EXPERIMENTS compiles the tuning knobs' environment
# reads back in (ET_KNOB, csrc/et_common.h) and the non-default kernel variants (the ET_W8 /
# ET_U lookup kernels, the queue orders).  Output: tools/alt/libembtab_hip_exp.so, loaded with
#   ET_LIBRARY=tools/alt/libembtab_hip_exp.so ET_<KNOB>=<value> python ...
# The package's own library (embtab/libembtab_hip.so) never reads the environment.
set -e
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.build_hip(defines=['ET_EXPERIMENTS'] + '${EXTRA_DEFINES:-}'.split(), lib='tools/alt/libembtab_hip_exp.so', obj_dir='tools/alt/obj_exp')"
echo tools/alt/libembtab_hip_exp.so

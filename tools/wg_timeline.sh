#!/bin/bash
# Profiling build of the library with per-workgroup timestamps in the striped lookup
# (-DET_WG_TIMELINE): tools/tl/libembtab_hip.so.  The package's own library is untouched.
# Build here (CPU), run tools/wg_timeline.py on the GPU box (tools/tl is listed in
# .gpurunignore so the 12 MB build does not travel with every call: drop that line first).
set -e
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.build_hip()"
mkdir -p tools/tl
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-unused-variable"
O=embeddingtables.jl_amd/csrc/obj
/opt/rocm/bin/hipcc $F -DET_WG_TIMELINE -Iinclude -c embeddingtables.jl_amd/csrc/et_lookup.hip -o tools/tl/et_lookup_tl.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/tl/libembtab_hip.so tools/tl/et_lookup_tl.o \
  $O/et_update.o $O/et_misc.o $O/et_shard.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f tools/tl/et_lookup_tl.o
echo built tools/tl/libembtab_hip.so

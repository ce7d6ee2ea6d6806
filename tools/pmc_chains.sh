#!/bin/bash
# Issue vs wait of the exact update's kernels (k_sgd_chains: early and regular chain
# launches; k_sgd_exact): one rocprofv3 --pmc pass of 8 SQ counters over
# tools/exact_cfg4.py exact, summed per dispatch.  Usage: tools/pmc_chains.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc_chains}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM \
  -d $OUT/sq -o run --output-format csv -- python3 tools/exact_cfg4.py exact > $OUT/sq.log 2>&1 || { echo PMC_FAIL; tail -5 $OUT/sq.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
disp = collections.defaultdict(dict)
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'k_sgd_chains' in n or 'k_sgd_exact' in n:
            key = (r.get('Dispatch_Id') or r.get('Correlation_Id'), n.split('(')[0][-30:])
            disp[key][r['Counter_Name']] = disp[key].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
rows = sorted(disp.items(), key=lambda kv: int(kv[0][0]))
for (d, name), m in rows[-6:]:
    wc = m.get('SQ_WAVE_CYCLES', 0) or 1
    print(f"dispatch {d} {name}: waves {m.get('SQ_WAVES', 0):.0f} wave_cycles {wc:.3g} "
          f"active_any {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} active_valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} "
          f"wait_any {m.get('SQ_WAIT_ANY', 0) / wc:.3f} wait_inst_any {m.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} "
          f"valu_insts {m.get('SQ_INSTS_VALU', 0):.3g} vmem_insts {m.get('SQ_INSTS_VMEM', 0):.3g}")
PY

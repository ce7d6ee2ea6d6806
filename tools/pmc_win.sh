set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_win
mkdir -p $OUT
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_SMEM"; do
  tag=$(echo "$grp" | cut -c1-20 | tr ' ' '_')
  ET_SGD_ORDER=0 timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/$tag" -o run --output-format csv -- python3 tools/upd_only.py > "$OUT/$tag.log" 2>&1 || { echo PMC_FAIL $tag; tail -3 $OUT/$tag.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'k_sgd' in n:
            agg[n[:24]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(k, {c: f"{sum(x)/len(x):.3g}" for c, x in v.items()})
PY

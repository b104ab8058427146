# Gram kernel counters on c3 (A A^t, K = 2M) and c3_ata: L2 hits / misses,
# fetched bytes, wait breakdown.  One rocprofv3 --pmc pass per group.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-grampmc}; mkdir -p $OUT; export TMPDIR=/tmp
for wl in ${WLS:-c3 c3_ata}; do
  B="python bench.py --no-cpu-baseline --workload $wl --steps 2 --warmup 0"
  p=0
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
    p=$((p+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/${wl}_p$p -o run --output-format csv -- $B > $OUT/${wl}_p$p.log 2>&1 || exit $?
  done
done
python - $OUT <<'PY'
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
res = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    wl = os.path.relpath(f, out).split("_p")[0]
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "k_gram" not in k or "sum" in k: continue
        res[wl][r["Counter_Name"]].append(float(r["Counter_Value"]))
for wl, d in res.items():
    print(wl, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(d.items())})
PY

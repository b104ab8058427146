#!/bin/bash
# rocprofv3 MFMA utilisation of the Gram kernel (k_gram_v) on the C3
# workload (bench.py --workload c3 computes L = ||A||^2 through A A^t):
# one --pmc pass (MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x
# SIMDs), MfmaFlopsF32 = SQ_INSTS_VALU_MFMA_MOPS_F32 x 512), kernel trace
# only; plus a --stats pass for the kernel's duration.  Summary -> $OUT.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-mfma}; mkdir -p $OUT; export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --workload ${WL:-c3} --steps 3 --warmup 1"
KSEL="${KSEL:-k_gram_v}"  # substring of the kernel name (e.g. "k_gram_v<float, 0>" = A^tA)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/stats.log 2>&1 || exit $?
echo "stats ok"
timeout -s KILL 300 rocprofv3 --pmc MfmaUtil MfmaFlopsF32 -d $OUT/mfma -o run --output-format csv -- $B > $OUT/mfma.log 2>&1 || exit $?
echo "pmc ok"
if [ "${LDS:-0}" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/lds -o run --output-format csv -- $B > $OUT/lds.log 2>&1 || exit $?
  echo "lds ok"
fi
python - "$OUT" "$KSEL" <<'PY'
import csv, glob, json, os, sys
out, ksel = sys.argv[1], sys.argv[2]
res = {}
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if ksel not in r.get("Kernel_Name", ""):
            continue
        res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
dur = None
for f in glob.glob(os.path.join(out, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if ksel in r["Name"]:
            dur = float(r["AverageNs"]) * 1e-9
s = {k: sum(v) / len(v) for k, v in res.items()}
if dur and "MfmaFlopsF32" in s:
    s["gram_kernel_s"] = dur
    s["MfmaTFLOPs_from_counter"] = s["MfmaFlopsF32"] / dur / 1e12
    s["frac_of_157.3TF"] = s["MfmaTFLOPs_from_counter"] / 157.3
print(json.dumps(s, indent=1))
json.dump(s, open(os.path.join(out, "mfma_summary.json"), "w"), indent=1)
PY

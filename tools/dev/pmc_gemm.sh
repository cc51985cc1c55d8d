#!/bin/bash
# SQ counter passes over the M = 2048 GEMM bench (dev): one rocprofv3 --pmc run per pass.
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_gemm
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
W=${W:-gemm_int4_g128_m2048}
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/bench.py" --workload $W --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    v.sort()
    print(f"{k:28s} median per dispatch {v[len(v)//2]:.4g}  (n={len(v)})")
PY

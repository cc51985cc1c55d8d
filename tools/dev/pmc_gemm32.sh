#!/bin/bash
# SQ counter passes (dev): product GEMM vs the 32x32x16 lab kernel, one rocprofv3 --pmc run per pass.
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc32
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PASSES=${PASSES:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"}
for KERN in ${KERNS:-prod lab}; do
i=0
for P in "$PASSES"; do
  i=$((i+1))
  KERNEL=$KERN timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/${KERN}$i" -o run -- python "$ROOT/tools/dev/gemm32_run.py" > "$OUT/${KERN}$i.log" 2>&1 || exit $?
done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for kern in ("prod", "lab"):
    agg = collections.defaultdict(list)
    for f in glob.glob(out + f"/{kern}*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = []
    for f in glob.glob(out + f"/{kern}*/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm" in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    durs.sort()
    d = durs[len(durs) // 2] if durs else float("nan")
    g = sorted(agg["GRBM_GUI_ACTIVE"])
    clk = g[len(g) // 2] / 8 / d / 1e9 if g and durs else float("nan")
    print(f"{kern}: median duration {d*1e6:.1f} us, effective clock {clk:.3f} GHz")
    for k, v in sorted(agg.items()):
        v.sort()
        print(f"  {k:28s} median per dispatch {v[len(v)//2]:.4g}  (n={len(v)})")
PY

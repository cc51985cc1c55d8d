#!/bin/bash
# SQ counter passes (dev) over any python command: pmc_any.sh <name> <kernel-name-substring> <script> [args]
# one rocprofv3 --pmc run per pass, medians per dispatch of the matching kernel, effective clock.
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; FILT=$2; shift 2
OUT=$ROOT/gpurun_out/pmc_$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/$@" > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" "$FILT" <<'PY'
import csv, glob, sys, collections
out, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
durs = []
for f in glob.glob(out + "/p*/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
durs.sort()
d = durs[len(durs) // 2] if durs else float("nan")
g = sorted(agg["GRBM_GUI_ACTIVE"])
clk = g[len(g) // 2] / 8 / d / 1e9 if g and durs else float("nan")
print(f"{filt}: median duration {d*1e6:.1f} us, effective clock {clk:.3f} GHz")
for k, v in sorted(agg.items()):
    v.sort()
    print(f"  {k:28s} median per dispatch {v[len(v)//2]:.4g}  (n={len(v)})")
PY

#!/bin/bash
# Round-6 GPU session (dev): the fused q/k/v + attention launch — its tests, the decode / attention
# / pipeline parity tests, the bench line (fused vs two-launch decode layer), the decode PMC pass
# and the in-graph kernel trace of the decode layers.  Stops at the first crash or timeout.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
R=${R:-r6}
stop() { echo "STOP: $1 exited $2"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_qkv_attn.py -x -v -p no:cacheprovider --timeout 150 \
  --timeout-method thread > "$OUT/${R}_qkv_attn_tests.log" 2>&1
rc=$?; echo "qkv_attn tests rc=$rc"; tail -3 "$OUT/${R}_qkv_attn_tests.log"; [ $rc -eq 0 ] || stop qkv_attn_tests $rc
if [ -n "${PARITY:-}" ]; then
  export QLIN_PARITY_OUT=$OUT/${R}_decode_parity.json QLIN_PARITY_OUT_PREFILL=$OUT/${R}_prefill_parity.json \
         QLIN_PARITY_OUT_PREFILL32=$OUT/${R}_prefill32_parity.json
  timeout -k 10 900 python -u -m pytest $PARITY -m gpu -v -p no:cacheprovider --timeout 600 \
    --timeout-method thread > "$OUT/${R}_parity_tests.log" 2>&1
  rc=$?; echo "parity tests rc=$rc"; tail -3 "$OUT/${R}_parity_tests.log"; [ $rc -le 1 ] || stop parity $rc
fi
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/${R}_bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 "$OUT/${R}_bench.log"; echo; [ $rc -eq 0 ] || stop bench $rc
STEPS=pmcd R=$R bash tools/gpu_round.sh || exit $?
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/dkt" -o run \
   -- python "$ROOT/tools/bench_decode.py" --reps 10 > "$OUT/dkt.log" 2>&1) || stop decode_kt $?
python tools/dev/kstats.py "$(find "$OUT/dkt" -name '*.db' | head -1)" 400 > "$OUT/${R}_decode_kernel_stats.txt"
cat "$OUT/${R}_decode_kernel_stats.txt"
rm -rf "$OUT/dkt"

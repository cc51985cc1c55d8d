#!/bin/bash
# Dev GPU session for decode-path changes: the attention / decode / pipeline tests (or $TESTS), the
# bench line without the CPU baseline, and the in-graph kernel durations of the decode layers.
# Stops at the first failure, crash or timeout (a failing kernel may have faulted the GPU).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
T=${TAG:-dev}
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_attn.py tests/test_gpu_decode.py tests/test_pipeline.py} \
  -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${T}_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" "$OUT/${T}_tests.log" | tail -2; grep FAILED "$OUT/${T}_tests.log" | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/${T}_bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT/${T}_bench.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print("headline", d["value"], d["roofline"]["frac"], "decode us/layer", d["decode_layer"]["us_per_layer"])
PY
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/dkt_$T" -o run \
   -- python "$ROOT/tools/bench_decode.py" --reps 10 > "$OUT/dkt_$T.log" 2>&1) || exit $?
python tools/dev/kstats.py "$(find "$OUT/dkt_$T" -name '*.db' | head -1)" 400 > "$OUT/${T}_decode_kernel_stats.txt"
head -8 "$OUT/${T}_decode_kernel_stats.txt"
rm -rf "$OUT/dkt_$T"

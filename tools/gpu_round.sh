#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace summary.
# Stops at the first crash / fault / timeout (exit codes other than 0 and pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
ok_or_stop() {  # $1 = rc, $2 = step
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi
}
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --maxfail=20 -p no:cacheprovider \
        --timeout ${TEST_CASE_TIMEOUT:-300} --timeout-method thread > "$OUT/pytest_gpu${TAG:-}.log" 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu${TAG:-}.log"; ok_or_stop $rc pytest ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; ok_or_stop $rc smoke ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; ok_or_stop $rc bench ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
         -- python "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1)
      rc=$?; echo "prof rc=$rc"; tail -3 "$OUT/prof.log"; ok_or_stop $rc prof
      find "$OUT/prof" -name "*kernel_stats.csv" -exec head -20 {} \; ;;
    pmc)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o run \
         -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/pmc.log" 2>&1)
      rc=$?; echo "pmc rc=$rc"; tail -2 "$OUT/pmc.log"; ok_or_stop $rc pmc
      python tools/pmc_traffic.py "$OUT/pmc" gemv_ "${PMC_WORKLOAD:-gemv_int4_g128}" "$OUT/pmc_traffic.json" ;;
    pmcd)  # the decode layer's traffic: every dispatch of each layer window (tools/decode_traffic.py)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcd" -o run \
         -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode --ramp-s 0 > "$OUT/pmcd.log" 2>&1)
      rc=$?; echo "pmcd rc=$rc"; tail -2 "$OUT/pmcd.log"; ok_or_stop $rc pmcd
      python tools/decode_traffic.py "$OUT/pmcd" "$OUT/${R:-r6}_decode_layer_int4_g128_pmc.json"; rm -rf "$OUT/pmcd" ;;
    pmchqq)  # FETCH_SIZE of the HQQ fp16-zero rings (configs[3]); ring per bench.py WORKLOADS
      for w in gemv_int3_g64_hqq gemv_int2_g64_hqq; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$w" -o run \
           -- python "$ROOT/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode > "$OUT/pmc_$w.log" 2>&1)
        rc=$?; echo "pmc $w rc=$rc"; ok_or_stop $rc "pmc $w"
        python tools/pmc_traffic.py "$OUT/pmc_$w" gemv_stream ${w}_batched "$OUT/${R:-r6}_${w}_batched_pmc.json" "$(case $w in *int2*) echo 96 ;; *) echo 64 ;; esac)"; rm -rf "$OUT/pmc_$w"
      done ;;
  esac
done

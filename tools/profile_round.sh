#!/bin/bash
# One GPU-box profiling session for the round's committed evidence (copy gpurun_out/prof_rN/* to
# profiles/ afterwards): bench lines per workload, rocprofv3 kernel-trace stats of the default
# bench, the FETCH_SIZE PMC pass (its own run), the decode-layer and full-size PPL parity tools.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
R=${ROUND:-r1}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP: $name exited $rc"; tail -5 "$OUT/$name.err"; exit $rc; fi
  tail -1 "$OUT/$name.out"
}
PHASE=${PHASE:-all}
ring_of() { case $1 in *int2*) echo 96 ;; *) echo 64 ;; esac; }  # bench.py WORKLOADS ring
if [ "$PHASE" != 2 ]; then
step bench_gemv_int4_g128 300 python bench.py
for w in ${WORKLOADS:-gemv_int3_g64 gemv_int2_g64 gemv_int3_g64_hqq gemv_int2_g64_hqq gemm_int4_g128_m32 gemm_int4_g128_m2048 gemm_int4_g128_m65536 gemm_int4_g64_hqq_m2048}; do
  step bench_$w 300 python bench.py --workload $w --no-cpu-baseline
done
export TMPDIR=/tmp
(cd /tmp && step kernel_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run \
   -- python "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline) || exit $?
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/${R}_gemv_int4_g128_kernel_stats.csv" \;
# FETCH_SIZE per dispatch, one pass per mode: the batched streaming launch (headline) and the
# dependent single launches (other_mode)
(cd /tmp && step pmc 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o run \
   -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode --no-decode-layer) || exit $?
python tools/pmc_traffic.py "$OUT/pmc" gemv_stream gemv_int4_g128_batched \
  "$OUT/${R}_gemv_int4_g128_batched_pmc.json" 64
(cd /tmp && step pmc_launches 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcl" \
   -o run -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode \
   --no-decode-layer --mode launches) || exit $?
python tools/pmc_traffic.py "$OUT/pmcl" "gemv_fast_kernel<4, 1, 1, 0, 0, 2, 0>" gemv_int4_g128 \
  "$OUT/${R}_gemv_int4_g128_pmc.json"
# the sub-byte rings (configs[3]): FETCH_SIZE of the batched streaming launch
for w in gemv_int3_g64 gemv_int2_g64; do
  (cd /tmp && step pmc_$w 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$w" -o run \
     -- python "$ROOT/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode \
     --no-decode-layer) || exit $?
  python tools/pmc_traffic.py "$OUT/pmc_$w" gemv_stream ${w}_batched "$OUT/${R}_${w}_batched_pmc.json" "$(ring_of $w)"
done
# the HQQ fp16-zero rings (configs[3]): FETCH_SIZE of the batched streaming launch
for w in gemv_int3_g64_hqq gemv_int2_g64_hqq; do
  (cd /tmp && step pmc_$w 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$w" -o run \
     -- python "$ROOT/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode \
     --no-decode-layer) || exit $?
  python tools/pmc_traffic.py "$OUT/pmc_$w" gemv_stream ${w}_batched "$OUT/${R}_${w}_batched_pmc.json" "$(ring_of $w)"
done
# the GEMM at configs[2] (M = 65,536): FETCH_SIZE, then the SQ passes (tools/dev/pmc_any.sh)
(cd /tmp && step pmc_gemm65536 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_gemm" -o run \
   -- python "$ROOT/bench.py" --workload gemm_int4_g128_m65536 --steps 2 --warmup 1 --no-cpu-baseline) \
   || exit $?
python tools/pmc_traffic.py "$OUT/pmc_gemm" gemm_kernel gemm_int4_g128_m65536 \
  "$OUT/${R}_gemm_int4_g128_m65536_pmc.json"
step sq_gemm65536 400 bash tools/dev/pmc_any.sh gemm65536 gemm_kernel bench.py \
  --workload gemm_int4_g128_m65536 --steps 2 --warmup 1 --no-cpu-baseline
cp "$OUT/sq_gemm65536.out" "$OUT/${R}_gemm_m65536_sq_counters.txt"
# effective clock (GRBM_GUI_ACTIVE / 8 / duration) of the product GEMM and of the same block with its
# dequant VALU skipped (power bound or issue bound?)
(cd tools/dev && make libgemmlab.so > /dev/null) || exit $?
step gclk_product 300 bash tools/dev/pmc_any.sh gclk_product gemm_kernel tools/dev/gemm_clock.py product
step gclk_nodq 300 bash tools/dev/pmc_any.sh gclk_nodq gemm_kernel tools/dev/gemm_clock.py nodq
cat "$OUT/gclk_product.out" "$OUT/gclk_nodq.out" > "$OUT/${R}_gemm_m65536_clock.txt"
fi
if [ "$PHASE" != 1 ]; then
export TMPDIR=/tmp
# the decode layer's traffic: every GEMV / attention dispatch of a --no-other-mode run
(cd /tmp && step pmc_decode 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcd" -o run \
   -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode --ramp-s 0) \
   || exit $?
python tools/decode_traffic.py "$OUT/pmcd" "$OUT/${R}_decode_layer_int4_g128_pmc.json"
step decode_layer 300 python tools/bench_decode.py
# per-launch durations of the graph-replayed decode layers (rocpd database, last 400 dispatches)
(cd /tmp && step decode_kt 300 rocprofv3 --kernel-trace -d "$OUT/dkt" -o run \
   -- python "$ROOT/tools/bench_decode.py" --reps 10) || exit $?
python tools/dev/kstats.py "$(find "$OUT/dkt" -name '*.db' | head -1)" 400 \
  > "$OUT/${R}_decode_kernel_stats.txt"
step attn_prefill 300 python tools/dev/attn_prefill_bench.py
cp "$OUT/attn_prefill.out" "$OUT/${R}_attn_prefill.txt"
# configs[4]: the 32-layer pipeline leg, one rank (the driver's multi-GPU runs: RCCL, one rank per
# GPU), and its two-rank rehearsal on one GPU (gloo)
step pipeline_n1 600 python bench.py --workload pipeline_llama3_8b_int4_g128
tail -1 "$OUT/pipeline_n1.out" > "$OUT/${R}_pipeline_n1.bench.json"
export BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1
step pipeline_n2_gloo 900 python bench.py --gpus 2 --steps 4 --warmup 1 --ring 8 --no-cpu-baseline \
  --no-decode-layer --no-other-mode --pipe-windows 4
unset BENCH_DIST_BACKEND BENCH_SHARE_GPU
tail -1 "$OUT/pipeline_n2_gloo.out" > "$OUT/${R}_pipeline_n2_gloo_rehearsal.bench.json"
step ppl_llama3_8b 500 python tools/ppl_llama3_8b.py
fi
# raw profiler outputs stay on the box (gpurun copies back at most 64 MiB): the summaries above
# are what profiles/ keeps
rm -rf "$OUT/kt" "$OUT/pmc" "$OUT/pmcl" "$OUT"/pmc_gemv_* "$OUT/pmc_gemm" "$OUT/pmcd" "$OUT/dkt" \
  "$ROOT/gpurun_out/pmc_gemm65536" "$ROOT/gpurun_out/pmc_gclk_product" "$ROOT/gpurun_out/pmc_gclk_nodq"
echo "done: $OUT"

# A/B of the default bench between the in-tree library and tools/dev/alt (same box, interleaved)
for i in 1 2 3; do
  for lib in in-tree alt; do
    if [ $lib = alt ]; then export QLIN_LIBRARY=tools/dev/alt/libqlin_gfx950.so; else unset QLIN_LIBRARY; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} | python -c "import json,sys; d=json.load(sys.stdin); print('$lib', d['roofline']['us_per_launch'])" || exit 3
  done
done

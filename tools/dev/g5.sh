set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dev/attn_prefill_bench.py > gpurun_out/apb.txt 2>&1 || exit $?
S=512 timeout -k 10 300 python -u tools/dev/attn_prefill_bench.py >> gpurun_out/apb.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pplprof -o run -- python $GRAFT_REPO_ROOT/tools/ppl_llama3_8b.py --layers 8 --windows 2 > $GRAFT_REPO_ROOT/gpurun_out/pplprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/pplprof.err || exit $?

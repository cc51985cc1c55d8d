set -u -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 $O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/pipeline_run.py --layers 8 --windows 2 --decode 16 --fused --prompt 128 > $O/pipe1.log 2>&1 || { echo pipe failed; tail -5 $O/pipe1.log; exit 1; }
grep '^{' $O/pipe1.log

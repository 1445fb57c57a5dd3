set -o pipefail
O=gpurun_out/${OUT:-r6c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -m gpu -x -v -s --timeout 150 --timeout-method thread tests/test_gpu_engine.py -k "cifar${KSEL:-}" > $O/cifar.log 2>&1 || { echo "cifar tests rc=$?"; grep -E "PASSED|FAILED|Error|assert" $O/cifar.log | head -30; exit 1; }
grep -E "PASSED|FAILED" $O/cifar.log
timeout -k 10 200 python -u -m pytest -m gpu -x -s --timeout 150 --timeout-method thread "tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle[vgg11]" > $O/vgg.log 2>&1; rc=$?
echo "vgg rc=$rc"; [ $rc -le 1 ] || exit 1
OUT=${OUT:-r6c} BENCH="--model cifar3 --steps 10 --warmup 3" PROF="--model cifar3 --steps 5 --warmup 2" bash tools/gpu_job.sh

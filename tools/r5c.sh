set -o pipefail
OUT=r5b TESTS="tests/test_gpu_programs.py tests/test_gpu_lenet_fc.py" BENCH="--steps 20 --warmup 5" bash tools/gpu_job.sh || exit 1
cat gpurun_out/r5b/bench_1.json
timeout -k 10 400 python tools/probes/lenet_phase_probe.py build/var_a1 build/var_a2 build/var_a4 build/var_a7 build/var_a3 build/var_a6 build/var_a456 build/var_a16 build/var_a32 build/var_a48 2>&1 | grep -v amdgpu.ids

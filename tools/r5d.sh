set -o pipefail
OUT=r5d TESTS="tests/test_gpu_lenet.py tests/test_gpu_engine.py::test_bench_batch_step_matches_small_batches tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle tests/test_gpu_engine.py::test_rows_dw_matches_pipe_dw" bash tools/gpu_job.sh || exit 1
timeout -k 10 200 python tools/probes/lenet_phase_probe.py 2>&1 | grep -v amdgpu.ids
MCC_AB=lenet_bwd2,lenet_fwd1 timeout -k 10 200 python tools/probes/lenet_phase_probe.py 2>&1 | grep -v amdgpu.ids
OUT=r5d2 BENCH="--steps 20 --warmup 5 --fp32-extra off;MCC_AB=lenet_bwd2,lenet_fwd1 --steps 20 --warmup 5 --fp32-extra off" bash tools/gpu_job.sh

set -o pipefail
OUT=r5j TESTS="tests/test_gpu_engine.py::test_fp32_lenet_sparse_dw_matches_dense tests/test_gpu_engine.py::test_step_matches_torch tests/test_gpu_engine.py::test_fc_igemm_bench_batch_matches_small_batches" bash tools/gpu_job.sh || exit 1
OUT=r5j BENCH="--steps 20 --warmup 5 --dtype fp32 --fp32-extra off;MCC_AB=f32_dense_dw --steps 20 --warmup 5 --dtype fp32 --fp32-extra off" PROF="--steps 3 --warmup 2 --dtype fp32 --fp32-extra off" bash tools/gpu_job.sh

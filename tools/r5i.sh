set -o pipefail
OUT=r5i TESTS="tests/test_gpu_engine.py::test_fused_block_buckets_split_at_block tests/test_gpu_rccl.py tests/test_gpu_ddp.py tests/test_gpu_hostcomm.py" bash tools/gpu_job.sh || exit 1
timeout -k 10 300 python tools/probes/cu_contention.py --reserve-sweep 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5i/cu_contention.txt
OUT=r5i BENCH="--steps 20 --warmup 5 --fp32-extra off;--steps 20 --warmup 5 --fp32-extra off --force-reduce;MCC_AB=bwd_reserve_cus=4 --steps 20 --warmup 5 --fp32-extra off --force-reduce" bash tools/gpu_job.sh

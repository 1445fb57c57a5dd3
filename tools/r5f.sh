set -o pipefail
OUT=r5f TESTS="tests/test_gpu_lenet.py" bash tools/gpu_job.sh || exit 1
timeout -k 10 200 python tools/probes/lenet_phase_probe.py 2>&1 | grep -v amdgpu.ids
MCC_AB=lenet_fwd1 timeout -k 10 200 python tools/probes/lenet_phase_probe.py 2>&1 | grep -v amdgpu.ids
MCC_AB=lenet_bwd2 timeout -k 10 200 python tools/probes/lenet_phase_probe.py 2>&1 | grep -v amdgpu.ids
PYTHONPATH=build/var_stamp timeout -k 10 200 python tools/probes/lenet_stamp_probe.py 2>&1 | grep -v amdgpu.ids

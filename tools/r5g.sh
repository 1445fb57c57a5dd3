set -o pipefail
for v in s18 t1 t2 t3; do PYTHONPATH=build/var_$v timeout -k 10 100 python tools/probes/lenet_stamp_probe.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 300 python tools/probes/lenet_phase_probe.py build/var_p18 build/var_q1 build/var_q2 build/var_q3 2>&1 | grep -v amdgpu.ids

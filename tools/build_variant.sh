#!/bin/bash
# Build the Python module with lenet.hip compiled under extra defines (phase
# ablations for timing studies), into build/var_<name>/mpi_cuda_cnn_amd/:
#   tools/build_variant.sh abl2 -DMCC_LENET_ABL=2
# then run with PYTHONPATH=build/var_abl2 (the module + a copy of the package).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
out=build/var_$name
base=$(basename ${SRC:-csrc/kernels/lenet.hip} .hip)  # SRC: the kernel file rebuilt with the defines
mkdir -p $out/obj $out/mpi_cuda_cnn_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Icsrc/include -Icsrc/kernels -Wall -Wno-unused-result \
  -mllvm -amdgpu-mfma-vgpr-form=1 "$@" -c ${SRC:-csrc/kernels/lenet.hip} -o $out/obj/$base.o
objs=$(ls build/obj/bindings/module.o build/obj/core/*.o build/obj/kernels/*.o build/obj/engine/*.o | grep -v "kernels/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/mpi_cuda_cnn_amd/_C$EXT $objs $out/obj/$base.o \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
(cd mpi_cuda_cnn_amd && find . -name '*.py' -exec install -D -m 644 {} ../$out/mpi_cuda_cnn_amd/{} \;)
echo "built $out"

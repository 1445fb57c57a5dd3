# Build for gfx950 (MI355X / CDNA4) only.  `make -j16` builds:
#   mpi_cuda_cnn_amd/_C*.so   python module (kernels + engine + CPU oracle)
#   build/bin/cnn             serial CPU trainer (reference cnn.c CLI)
#   build/bin/cnn_hip         single-GPU trainer (same CLI)
#   build/bin/cnn_dist        multi-GPU data-parallel trainer (RCCL, one process per GPU)
#   build/bin/cnnmpi          CPU data-parallel trainer over MPI (if mpicxx exists)
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PYTHON    ?= python3
MPICXX    ?= $(shell command -v mpicxx 2>/dev/null || ls /opt/conda/bin/mpicxx 2>/dev/null)

PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
EXT       := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

OPT       ?= -O3
INC       := -Icsrc/include -Icsrc/kernels
HIPFLAGS  := --offload-arch=$(ARCH) $(OPT) -std=c++20 -fPIC $(INC) -Wall -Wno-unused-result
CXXFLAGS  := $(OPT) -std=c++17 -fPIC $(INC) -Wall -Wno-unused-result
HOSTHIP   := -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
LDHIP     := -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

OBJ       := build/obj
CORE_SRC  := csrc/core/model.cpp csrc/core/cpu_net.cpp csrc/core/io.cpp csrc/core/cpu_kernels_base.cpp \
             csrc/core/cpu_kernels_v3.cpp
CORE_OBJ  := $(patsubst csrc/core/%.cpp,$(OBJ)/core/%.o,$(CORE_SRC))
KERN_SRC  := $(wildcard csrc/kernels/*.hip)
KERN_OBJ  := $(patsubst csrc/kernels/%.hip,$(OBJ)/kernels/%.o,$(KERN_SRC))
ENG_SRC   := $(wildcard csrc/engine/*.cpp)
ENG_OBJ   := $(patsubst csrc/engine/%.cpp,$(OBJ)/engine/%.o,$(ENG_SRC))
HDRS      := $(wildcard csrc/include/mcc/*.h csrc/kernels/*.h csrc/apps/*.h) csrc/core/cpu_kernels.inc

MODULE    := mpi_cuda_cnn_amd/_C$(EXT)
BINS      := build/bin/cnn build/bin/cnn_hip build/bin/cnn_dist build/bin/test_watchdog build/bin/test_comm
ifneq ($(MPICXX),)
BINS      += build/bin/cnnmpi
endif

.PHONY: all module bins clean asan checked
all: module bins
module: $(MODULE)
bins: $(BINS)

$(OBJ)/core/%.o: csrc/core/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# the AVX2/FMA build of the CPU kernels (dispatched at run time)
$(OBJ)/core/cpu_kernels_v3.o: csrc/core/cpu_kernels_v3.cpp csrc/core/cpu_kernels.inc $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -mavx2 -mfma -c $< -o $@
$(OBJ)/core/cpu_kernels_base.o: csrc/core/cpu_kernels_base.cpp csrc/core/cpu_kernels.inc $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/kernels/%.o: csrc/kernels/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# lenet.hip: MFMA results in VGPRs (no v_accvgpr_read per accumulator in the
# VALU-bound epilogues; the register file is unified on gfx950)
$(OBJ)/kernels/lenet.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form=1
# conv_direct.hip: the packed-FMA kernels use explicit float2 vectors; the SLP
# vectorizer would pair the scatter dX kernel's 98 scalar accumulators into
# v_pk_fma_f32 register pairs (866 moves and 165 spilled registers; 151
# VGPRs and no spills without it)
$(OBJ)/kernels/conv_direct.o: HIPFLAGS += -fno-slp-vectorize

$(OBJ)/engine/%.o: csrc/engine/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/bindings/module.o: csrc/bindings/module.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(HOSTHIP) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(MODULE): $(OBJ)/bindings/module.o $(CORE_OBJ) $(KERN_OBJ) $(ENG_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ $(LDHIP)

build/bin/cnn: csrc/apps/cnn.cpp $(CORE_OBJ) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -o $@ csrc/apps/cnn.cpp $(CORE_OBJ) -lm

build/bin/test_watchdog: csrc/tests/test_watchdog.cpp csrc/apps/watchdog.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -Icsrc/apps -o $@ csrc/tests/test_watchdog.cpp

# host-only rendezvous + shared-memory collectives (cnn_dist --comm host)
COMM_SRC := csrc/apps/bootstrap.cpp csrc/apps/shm_group.cpp
build/bin/test_comm: csrc/tests/test_comm.cpp $(COMM_SRC) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -Icsrc/apps -o $@ csrc/tests/test_comm.cpp $(COMM_SRC) -lrt

# MPICH's wrapper would put its own (older) libstdc++ first; link with the
# system compiler against the MPI library instead, libstdc++ static.
MPI_PREFIX := $(patsubst %/bin/mpicxx,%,$(MPICXX))
build/bin/cnnmpi: csrc/apps/cnnmpi.cpp $(CORE_OBJ) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(MPI_PREFIX)/include -o $@ csrc/apps/cnnmpi.cpp $(CORE_OBJ) \
	  $(MPI_PREFIX)/lib/libmpi.so -Wl,-rpath,$(MPI_PREFIX)/lib -static-libstdc++ -static-libgcc -lm

$(OBJ)/apps/%.o: csrc/apps/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -I$(ROCM)/include/rccl -c $< -o $@

build/bin/cnn_hip: $(OBJ)/apps/cnn_hip.o $(OBJ)/apps/trainer.o $(CORE_OBJ) $(KERN_OBJ) $(ENG_OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ $(LDHIP) -lrocprofiler-sdk-roctx

build/bin/cnn_dist: $(OBJ)/apps/cnn_dist.o $(OBJ)/apps/trainer.o $(OBJ)/apps/bootstrap.o $(OBJ)/apps/shm_group.o \
                   $(OBJ)/apps/host_comm.o $(CORE_OBJ) $(KERN_OBJ) $(ENG_OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ $(LDHIP) -lrccl -lrocprofiler-sdk-roctx

# Host sanitizers: the CPU trainer and the core library
# under AddressSanitizer + UBSan.  GPU-side sanitizers are not available on
# the MI355X pool; device code is covered by bounds reasoning + tests.
# (only cpu_kernels_v3.cpp is compiled with -mavx2 -mfma, as in the main
# build, so the sanitized binary's baseline kernel table is baseline code)
ASAN_FLAGS := -O1 -g -std=c++17 $(INC) -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined
ASAN_OBJ   := build/obj_asan
ASAN_SRC   := csrc/apps/cnn.cpp $(filter-out %_v3.cpp,$(CORE_SRC))
asan: build/bin/cnn_asan
$(ASAN_OBJ)/cpu_kernels_v3.o: csrc/core/cpu_kernels_v3.cpp csrc/core/cpu_kernels.inc $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(ASAN_FLAGS) -mavx2 -mfma -c $< -o $@
build/bin/cnn_asan: $(ASAN_SRC) $(ASAN_OBJ)/cpu_kernels_v3.o $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(ASAN_FLAGS) -o $@ $(ASAN_SRC) $(ASAN_OBJ)/cpu_kernels_v3.o -lm

# Device bounds checks (MCC_DCHECK in the pipelined conv kernels): a separate
# module under build/checked/ (same Python package, checked _C); run e.g.
#   MCC_PKG_ROOT=build/checked python -m pytest tests/test_gpu_engine.py -m gpu
checked:
	mkdir -p build/checked/mpi_cuda_cnn_amd
	$(MAKE) OBJ=build/obj_checked OPT="-O3 -DMCC_DEVICE_CHECKS" MODULE=build/checked/mpi_cuda_cnn_amd/_C$(EXT) \
	  build/checked/mpi_cuda_cnn_amd/_C$(EXT)
	cd mpi_cuda_cnn_amd && find . -name '*.py' -exec install -D -m 644 {} ../build/checked/mpi_cuda_cnn_amd/{} \;

# Run targets (the reference Makefile's test_serial / test_mpi / test_cuda,
# Makefile:38-51), on generated data unless DATA names the four IDX files:
#   make run_serial                 CPU trainer (cnn)
#   make run_mpi NP=8               CPU data-parallel over MPI (cnnmpi, if built)
#   make run_hip                    one GPU (cnn_hip, hipGraph step)
#   make run_dist NP=8              one process per GPU over RCCL (cnn_dist)
#   make run_bench NP=8             bench.py under torch.distributed.run
NP    ?= 2
SYN   ?= 20000
DATA  ?= --synthetic $(SYN)
RUNFLAGS ?=
.PHONY: run_serial run_mpi run_hip run_dist run_bench data
# the four IDX files under data/ (the reference's get_mnist, Makefile:12-35,
# without network): MNIST_SRC=DIR takes local MNIST files (raw or .gz), else
# the synthetic MNIST-shaped set; then e.g. make run_serial DATA="$$(cat data/files)"
data:
	@mkdir -p data
	$(PYTHON) tools/get_mnist.py --out data $(if $(MNIST_SRC),--src $(MNIST_SRC),--synthetic $(SYN)) > data/files.tmp
	mv data/files.tmp data/files
	@cat data/files
run_serial: build/bin/cnn
	build/bin/cnn $(DATA) $(RUNFLAGS)
run_mpi: build/bin/cnnmpi
	$(dir $(MPICXX))mpiexec -n $(NP) build/bin/cnnmpi $(DATA) $(RUNFLAGS)
run_hip: build/bin/cnn_hip
	build/bin/cnn_hip $(DATA) $(RUNFLAGS)
run_dist: build/bin/cnn_dist
	$(PYTHON) -m mpi_cuda_cnn_amd.launch -n $(NP) build/bin/cnn_dist $(DATA) $(RUNFLAGS)
run_bench: module
	$(PYTHON) -m torch.distributed.run --nnodes=1 --nproc-per-node $(NP) --master-addr 127.0.0.1 \
	  --master-port 29531 bench.py --gpus $(NP) $(RUNFLAGS)

clean:
	rm -rf build $(MODULE)

# p2p_matrix for MI355X (gfx950): RCCL over xGMI, MPI or TCP control plane.
#
#   make              build/p2p_matrix (HIP + RCCL + MPI) and the Python extension
#   make host         build/p2p_matrix_host + build/p2p_host_tests (g++ only, no GPU code)
#   make test         host unit tests + CPU pytest tier
#   make test-gpu     pytest -m gpu (run on an MI355X, e.g. via gpurun)
#   make asan         host unit tests under AddressSanitizer/UBSan (host code only)
#   make tsan         host unit tests under ThreadSanitizer (host code only)
#   make clean        removes build/ and the extension (the reference's clean
#                     target removes the misspelled "p2pmatrix", Makefile:5)
#
# Reference build (Makefile:1-2): `nvcc -lmpi -lnccl p2p_matrix.cc`.

ROCM      ?= /opt/rocm
ARCH      ?= gfx950
MPI_HOME  ?= /opt/conda
PYTHON    ?= python3
HIPCC     := $(ROCM)/bin/hipcc
CXX_HOST  ?= g++
BUILD     := build

CXXSTD    := -std=c++17
WARN      := -Wall -Wextra -Wno-unused-parameter
OPT       ?= -O3
HIPFLAGS  := $(CXXSTD) $(OPT) $(WARN) -fPIC --offload-arch=$(ARCH) -Icsrc
HOSTFLAGS := $(CXXSTD) $(OPT) $(WARN) -fPIC -Icsrc -pthread

CORE      := common units stats schedule routing bootstrap transport_host transport_shm runner step_driver report provenance app rccl_log
GPU_OBJS  := $(addprefix $(BUILD)/gpu/,$(addsuffix .o,$(CORE) transport_rccl transport_ipc topology stream_gate) kernels.o pingpong.o)
HOST_OBJS := $(addprefix $(BUILD)/host/,$(addsuffix .o,$(CORE) transport_rccl_stub))

# MPICH lives in /opt/conda; putting /opt/conda/lib on the rpath would pull in
# conda's old libstdc++ (GLIBCXX_3.4.29 missing for libamdhip64), so only the
# three MPI libraries are symlinked into build/mpilib.
MPILIB    := $(BUILD)/mpilib
MPI_LINK  := -L$(MPILIB) -lmpi -Wl,-rpath,'$$ORIGIN/mpilib'
MPI_INC   := -I$(MPI_HOME)/include

# One HIP / RCCL runtime for every entry point (RUNTIME=torch, the default):
# bench.py and the tests run inside torch processes, which load torch's
# bundled libamdhip64 / librccl; build/p2p_matrix and the extension are linked
# against the same files through build/rt (symlinks with the sonames the
# loader looks for), so a cell measured through either entry point runs on
# one RCCL.  RUNTIME=rocm links /opt/rocm's instead.  Both JSON outputs
# record the library path and version (csrc/provenance.cpp).
RUNTIME   ?= torch
TORCH_LIB := $(shell $(PYTHON) -c "import os,importlib.util as u;s=u.find_spec('torch');print(os.path.join(os.path.dirname(s.origin),'lib') if s else '')")
RTDIR     := $(BUILD)/rt
RT_LIBS   := amdhip64 hsa-runtime64 amd_comgr rocprofiler-register rccl rocm_smi64 rocm-core roctx64 drm drm_amdgpu numa
ifeq ($(RUNTIME)$(if $(TORCH_LIB),,none),torch)
RT_STAMP  := $(RTDIR)/.stamp
BIN_RPATH := -Wl,--disable-new-dtags -Wl,-rpath,'$$ORIGIN/rt'
EXT_RPATH := -Wl,--disable-new-dtags -Wl,-rpath,'$$ORIGIN/../$(RTDIR)'
else
RT_STAMP  :=
BIN_RPATH := -Wl,-rpath,$(ROCM)/lib
EXT_RPATH := -Wl,-rpath,$(ROCM)/lib
endif

PY_EXT    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND    := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
EXT       := test_nccl_p2p_amd/_p2pcore$(PY_EXT)

.PHONY: all gpu host ext tools test test-host test-gpu asan tsan clean

all: gpu host ext tools

# ./p2p_matrix: where the reference's `make` leaves its binary (Makefile:1-2
# there), so `mpirun -n N ./p2p_matrix > result.txt` works unchanged.
gpu: $(BUILD)/p2p_matrix
	ln -sf $(BUILD)/p2p_matrix p2p_matrix
host: $(BUILD)/p2p_matrix_host $(BUILD)/p2p_host_tests
ext: $(EXT)
tools: $(BUILD)/fill_probe $(BUILD)/copy_probe $(BUILD)/ipc_export_probe $(BUILD)/rccl_half_repro $(BUILD)/rccl_half_repro_rocm \
       $(BUILD)/rccl_net_repro

$(BUILD)/gpu $(BUILD)/host $(BUILD)/asan $(BUILD)/tsan:
	mkdir -p $@

$(RTDIR)/.stamp:
	mkdir -p $(RTDIR)
	for l in $(RT_LIBS); do [ ! -e $(TORCH_LIB)/lib$$l.so ] || ln -sf $(TORCH_LIB)/lib$$l.so $(RTDIR)/lib$$l.so; done
	ln -sf $(TORCH_LIB)/librccl.so $(RTDIR)/librccl.so.1
	ln -sf $(TORCH_LIB)/libamdhip64.so $(RTDIR)/libamdhip64.so.7
	touch $@

$(MPILIB)/.stamp:
	mkdir -p $(MPILIB)
	for l in libmpi.so.12 libgfortran.so.4 libquadmath.so.0; do ln -sf $(MPI_HOME)/lib/$$l $(MPILIB)/$$l; done
	ln -sf libmpi.so.12 $(MPILIB)/libmpi.so
	touch $@

HEADERS := $(wildcard csrc/*.hpp)

$(BUILD)/gpu/%.o: csrc/%.cpp $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/gpu/kernels.o: csrc/kernels.hip $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/gpu/pingpong.o: csrc/pingpong.hip $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/gpu/bootstrap_mpi.o: csrc/bootstrap_mpi.cpp $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) $(MPI_INC) -c $< -o $@

$(BUILD)/gpu/main.o: csrc/main.cpp $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/host/%.o: csrc/%.cpp $(HEADERS) | $(BUILD)/host
	$(CXX_HOST) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/host/bootstrap_mpi.o: csrc/bootstrap_mpi.cpp $(HEADERS) | $(BUILD)/host
	$(CXX_HOST) $(HOSTFLAGS) $(MPI_INC) -c $< -o $@

$(BUILD)/p2p_matrix: $(GPU_OBJS) $(BUILD)/gpu/bootstrap_mpi.o $(BUILD)/gpu/main.o $(MPILIB)/.stamp $(RT_STAMP)
	$(HIPCC) --offload-arch=$(ARCH) $(GPU_OBJS) $(BUILD)/gpu/bootstrap_mpi.o $(BUILD)/gpu/main.o -o $@ \
	    $(BIN_RPATH) -L$(ROCM)/lib -lrccl $(MPI_LINK) -pthread

$(BUILD)/p2p_matrix_host: $(HOST_OBJS) $(BUILD)/host/bootstrap_mpi.o $(BUILD)/host/main.o $(MPILIB)/.stamp
	$(CXX_HOST) $(HOST_OBJS) $(BUILD)/host/bootstrap_mpi.o $(BUILD)/host/main.o -o $@ $(MPI_LINK) -pthread

TEST_DATA := -DP2P_TEST_DATA='"$(abspath tests/data)"'

$(BUILD)/p2p_host_tests: $(HOST_OBJS) tests/host/test_main.cpp $(HEADERS)
	$(CXX_HOST) $(HOSTFLAGS) $(TEST_DATA) $(HOST_OBJS) tests/host/test_main.cpp -o $@

$(BUILD)/gpu/pymodule.o: csrc/pymodule.cpp $(HEADERS) | $(BUILD)/gpu
	$(HIPCC) $(HIPFLAGS) -fvisibility=hidden -I$(PY_INC) -I$(PYBIND) -c $< -o $@

$(EXT): $(GPU_OBJS) $(BUILD)/gpu/pymodule.o $(RT_STAMP)
	$(HIPCC) --offload-arch=$(ARCH) -shared $(GPU_OBJS) $(BUILD)/gpu/pymodule.o -o $@ \
	    $(EXT_RPATH) -L$(ROCM)/lib -lrccl -pthread

# Grid-shape probe (scripts/fill_probe.hip): standalone, no framework code.
$(BUILD)/fill_probe: scripts/fill_probe.hip | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

# Copy cache-policy / shape probe (scripts/copy_probe.hip): standalone.
$(BUILD)/copy_probe: scripts/copy_probe.hip | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

$(BUILD)/ipc_export_probe: scripts/ipc_export_probe.hip | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O2 $< -o $@

# Framework-free RCCL half-delivery reproducer (scripts/rccl_half_repro.cpp):
# raw HIP + RCCL only, linked once against the RCCL every entry point uses
# (build/rt) and once against /opt/rocm's.
$(BUILD)/rccl_half_repro: scripts/rccl_half_repro.cpp $(RT_STAMP) | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O2 $(WARN) $< -o $@ $(BIN_RPATH) -L$(ROCM)/lib -lrccl

$(BUILD)/rccl_half_repro_rocm: scripts/rccl_half_repro.cpp | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O2 $(WARN) $< -o $@ -Wl,-rpath,$(ROCM)/lib -L$(ROCM)/lib -lrccl

# Framework-free two-rank reproducer (scripts/rccl_net_repro.cpp): raw HIP +
# RCCL + MPI, one send and one receive per message between two ranks.
$(BUILD)/rccl_net_repro: scripts/rccl_net_repro.cpp $(RT_STAMP) $(MPILIB)/.stamp | $(BUILD)/gpu
	$(HIPCC) --offload-arch=$(ARCH) -O2 $(WARN) $(MPI_INC) $< -o $@ $(BIN_RPATH) -L$(ROCM)/lib -lrccl \
	    -L$(MPILIB) -lmpi -Wl,-rpath,'$$ORIGIN/mpilib'

# AddressSanitizer / UBSan on host code only (GPU sanitizers are not available):
# the unit tests, and the MPI host binary that tests/test_host_unit.py runs as
# a 3-rank job over the TCP transport.
ASAN      := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
ASAN_SRCS := $(addprefix csrc/,$(addsuffix .cpp,$(CORE) transport_rccl_stub))
asan: $(BUILD)/asan/p2p_host_tests $(BUILD)/asan/p2p_matrix_host
	ASAN_OPTIONS=detect_leaks=1 $(BUILD)/asan/p2p_host_tests

$(BUILD)/asan/p2p_host_tests: $(ASAN_SRCS) tests/host/test_main.cpp $(HEADERS) | $(BUILD)/asan
	$(CXX_HOST) $(CXXSTD) $(WARN) $(ASAN) $(TEST_DATA) -Icsrc -pthread $(ASAN_SRCS) tests/host/test_main.cpp -o $@

$(BUILD)/asan/p2p_matrix_host: $(ASAN_SRCS) csrc/bootstrap_mpi.cpp csrc/main.cpp $(HEADERS) $(MPILIB)/.stamp | $(BUILD)/asan
	$(CXX_HOST) $(CXXSTD) $(WARN) $(ASAN) -Icsrc $(MPI_INC) -pthread $(ASAN_SRCS) csrc/bootstrap_mpi.cpp csrc/main.cpp \
	    -o $@ -L$(MPILIB) -lmpi -Wl,-rpath,'$$ORIGIN/../mpilib'

# ThreadSanitizer on the same host code: the unit tests run every rank of a
# multi-rank case as a thread (TCP / shm transports, bootstrap collectives,
# the abort path against in-flight native calls), so a data race between
# ranks, the watchdog's abort and the logging is reported; any report fails.
TSAN      := -fsanitize=thread -fno-omit-frame-pointer -g -O1
tsan: $(BUILD)/tsan/p2p_host_tests $(BUILD)/tsan/p2p_matrix_host
	TSAN_OPTIONS=halt_on_error=1 $(BUILD)/tsan/p2p_host_tests

$(BUILD)/tsan/p2p_matrix_host: $(ASAN_SRCS) csrc/bootstrap_mpi.cpp csrc/main.cpp $(HEADERS) $(MPILIB)/.stamp | $(BUILD)/tsan
	$(CXX_HOST) $(CXXSTD) $(WARN) $(TSAN) -Icsrc $(MPI_INC) -pthread $(ASAN_SRCS) csrc/bootstrap_mpi.cpp csrc/main.cpp \
	    -o $@ -L$(MPILIB) -lmpi -Wl,-rpath,'$$ORIGIN/../mpilib'

$(BUILD)/tsan/p2p_host_tests: $(ASAN_SRCS) tests/host/test_main.cpp $(HEADERS) | $(BUILD)/tsan
	$(CXX_HOST) $(CXXSTD) $(WARN) $(TSAN) $(TEST_DATA) -Icsrc -pthread $(ASAN_SRCS) tests/host/test_main.cpp -o $@

test-host: $(BUILD)/p2p_host_tests
	$(BUILD)/p2p_host_tests

test: test-host
	$(PYTHON) -m pytest tests -x -q -m "not gpu"

test-gpu: all
	$(PYTHON) -m pytest tests -x -q -m gpu

clean:
	rm -rf $(BUILD) test_nccl_p2p_amd/_p2pcore*.so p2p_matrix

# QuEST for MI355X - build of the native libraries.
#
#   make            -> CPU (host) libraries, fp64 + fp32   (no GPU needed)
#   make hip        -> HIP libraries for gfx950, fp64 + fp32 (hipcc cross-compiles)
#   make all        -> both
#   make examples   -> C examples linked against the fp64 CPU library
#   make examples-hip -> the same linked against the fp64 HIP library
#
# Outputs go to quest_amd/lib/ so they travel with the repository snapshot:
#   libQuEST_cpu_f64.so  libQuEST_cpu_f32.so  libQuEST_hip_f64.so  libQuEST_hip_f32.so
# plus libQuEST.so -> libQuEST_hip_f64.so for C programs (-lQuEST).

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
BUILD     := build
LIBDIR    := quest_amd/lib
JOBS      ?= 8
WAVE_SLOTS ?= 5   # fp64 amplitudes per lane = 2^WAVE_SLOTS in the wave-tile kernel
WAVE_SLOTS32 ?= 5 # fp32: 2^WAVE_SLOTS32 per lane
WAVE_WBITS ?= 2   # fp64: 2^WAVE_WBITS waves share one wave tile (exchanging through LDS)
WAVE_WBITS32 ?= 3 # fp32: the same
# fp64 tile = 5 slots x 6 lanes x 2 wave bits (4 waves of 32 amplitudes per lane, 144 VGPRs):
# 0.7 % faster over five circuit seeds than 4 slots x 3 wave bits, 1.6 % on the bench's
# (profiles/r3/wave_shape_variants.txt)
WAVE_DBUF ?= -1   # 1/0: second register set prefetching the next tile (-1: generator default)
WAVE_LEAN ?= 1    # 1: lean register layout (4 aliased temporaries, half LDS outboxes), 0: more temporaries
WAVE_GENFLAGS ?=  # extra tools/gen_wave_asm.py flags for experiments (e.g. --nomem)
WAVE_PFA ?= 0     # fp64 next-tile prefetch of looping grids: 16-byte loads per lane into AGPRs
WAVE_PFL ?= 0     # ... and into LDS (tools/gen_wave_asm.py pf_paths)

# objects and the generated kernel are rebuilt when the wave configuration changes
WAVE_CFG   := $(BUILD)/.wave_cfg_s$(strip $(WAVE_SLOTS))_$(strip $(WAVE_SLOTS32))_w$(strip $(WAVE_WBITS))_$(strip $(WAVE_WBITS32))_d$(strip $(WAVE_DBUF))_l$(strip $(WAVE_LEAN))_p$(strip $(WAVE_PFA))_$(strip $(WAVE_PFL))

COMMON_SRC := src/api/api.cpp src/api/validation.cpp src/api/qasm.cpp src/api/common.cpp src/api/checkpoint.cpp \
              src/api/mt19937.cpp src/core/router.cpp src/core/tiles.cpp src/core/wave.cpp src/core/wave_emu.cpp src/core/trace.cpp src/comm/bootstrap.cpp
CPU_SRC    := $(COMMON_SRC) src/comm/comm_socket.cpp src/comm/comm_host.cpp src/cpu/backend_cpu.cpp
HIP_HOST   := $(COMMON_SRC) src/comm/comm_socket.cpp src/comm/comm_rccl.cpp src/comm/comm_ipc.cpp
HIP_DEV    := src/hip/backend_hip.hip src/hip/kernels_gates.hip src/hip/kernels_direct.hip src/hip/kernels_reduce.hip src/hip/kernels_misc.hip

INCLUDES   := -Iinclude -DQA_WAVE_SLOTS_F64=$(strip $(WAVE_SLOTS)) -DQA_WAVE_SLOTS_F32=$(strip $(WAVE_SLOTS32)) \
              -DQA_WAVE_WBITS_F64=$(strip $(WAVE_WBITS)) -DQA_WAVE_WBITS_F32=$(strip $(WAVE_WBITS32))
CXXFLAGS   := -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $(INCLUDES)
HIPFLAGS   := -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-function \
              -Wno-unused-result -munsafe-fp-atomics $(INCLUDES)
# the Python binding's per-gate fast path (CPython C API, src/py/gatecall.c)
PYTHON     ?= python3
PY_INC     := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PY_EXT     := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
GATECALL   := quest_amd/ops/_gatecall$(PY_EXT)
HIPHOST    := -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $(INCLUDES) -I$(ROCM)/include -D__HIP_PLATFORM_AMD__

.PHONY: cpu hip all clean examples examples-hip asan-check

cpu: $(LIBDIR)/libQuEST_cpu_f64.so $(LIBDIR)/libQuEST_cpu_f32.so $(LIBDIR)/libQuEST_cpu_f128.so $(GATECALL)
hip: $(LIBDIR)/libQuEST_hip_f64.so $(LIBDIR)/libQuEST_hip_f32.so $(LIBDIR)/libQuEST.so $(GATECALL)
all: cpu hip

# ---------------------------------------------------------------- CPU build
define cpu_rules
$(BUILD)/cpu_f$(2)/%.o: %.cpp $(wildcard include/*.h src/*/*.hpp) $(WAVE_CFG)
	@mkdir -p $$(dir $$@)
	$(CXX) $(CXXFLAGS) -fopenmp -DQuEST_PREC=$(1) -c $$< -o $$@

$(LIBDIR)/libQuEST_cpu_f$(2).so: $(patsubst %.cpp,$(BUILD)/cpu_f$(2)/%.o,$(CPU_SRC))
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -fopenmp -Wl,-Bsymbolic -o $$@ $$^ -ldl -lpthread
endef
$(eval $(call cpu_rules,2,64))
$(eval $(call cpu_rules,1,32))
# QuEST_PREC=4 (long double), host build only as in the reference
# (QuEST/CMakeLists.txt:66-70 forbids it on the GPU)
$(eval $(call cpu_rules,4,128))

$(GATECALL): src/py/gatecall.c $(wildcard include/*.h)
	gcc -O2 -fPIC -shared -std=c11 -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
	    -Iinclude -I$(PY_INC) $< -o $@

# ---------------------------------------------------------------- HIP build
define hip_rules
$(BUILD)/hip_f$(2)/%.o: %.cpp $(wildcard include/*.h src/*/*.hpp) $(WAVE_CFG)
	@mkdir -p $$(dir $$@)
	$(CXX) $(HIPHOST) -DQuEST_PREC=$(1) -c $$< -o $$@

$(BUILD)/hip_f$(2)/%.o: %.hip $(wildcard include/*.h src/*/*.hpp src/hip/*.h) $(WAVE_CFG)
	@mkdir -p $$(dir $$@)
	$(HIPCC) $$(HIPFLAGS) -I$(BUILD)/wave_f$(2) -DQuEST_PREC=$(1) -c $$< -o $$@

$(LIBDIR)/libQuEST_hip_f$(2).so: $(patsubst %.cpp,$(BUILD)/hip_f$(2)/%.o,$(HIP_HOST)) $(patsubst %.hip,$(BUILD)/hip_f$(2)/%.o,$(HIP_DEV))
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -Wl,-Bsymbolic --offload-arch=$(ARCH) -o $$@ $$^ -L$(ROCM)/lib -lamdhip64 -ldl -lpthread
endef
$(eval $(call hip_rules,2,64))
$(eval $(call hip_rules,1,32))
# ---------------------------------------------------------------- wave-tile kernel (gfx950 assembly)
# generated by tools/gen_wave_asm.py for each precision, assembled and linked
# into a code object that is embedded into that HIP library
# (src/hip/backend_hip.hip includes build/wave_f64 or build/wave_f32)
LLVM_BIN  := $(ROCM)/llvm/bin
$(WAVE_CFG):
	@mkdir -p $(BUILD)
	@rm -f $(BUILD)/.wave_cfg_*
	@touch $@
define wave_rules
$(BUILD)/wave_f$(2)/wave_kernel.s: tools/gen_wave_asm.py $(WAVE_CFG)
	@mkdir -p $$(dir $$@)
	python3 tools/gen_wave_asm.py asm --prec $(1) --slots $(3) --wbits $(4) --dbuf $(WAVE_DBUF) --lean $(strip $(WAVE_LEAN)) $(5) $(WAVE_GENFLAGS) --out $$@
$(BUILD)/wave_f$(2)/wave_kernel.o: $(BUILD)/wave_f$(2)/wave_kernel.s
	$(LLVM_BIN)/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=$(ARCH) -c $$< -o $$@
$(BUILD)/wave_f$(2)/wave_kernel.hsaco: $(BUILD)/wave_f$(2)/wave_kernel.o
	$(LLVM_BIN)/ld.lld -shared $$< -o $$@
$(BUILD)/wave_f$(2)/wave_image.inc: $(BUILD)/wave_f$(2)/wave_kernel.hsaco tools/gen_wave_asm.py
	python3 tools/gen_wave_asm.py embed --prec $(1) --slots $(3) --wbits $(4) --obj $(BUILD)/wave_f$(2)/wave_kernel.o --hsaco $$< --out $$@
$(BUILD)/hip_f$(2)/src/hip/backend_hip.o: $(BUILD)/wave_f$(2)/wave_image.inc
endef
$(eval $(call wave_rules,2,64,$(strip $(WAVE_SLOTS)),$(strip $(WAVE_WBITS)),--pfa $(strip $(WAVE_PFA)) --pfl $(strip $(WAVE_PFL))))
$(eval $(call wave_rules,1,32,$(strip $(WAVE_SLOTS32)),$(strip $(WAVE_WBITS32)),))

$(LIBDIR)/libQuEST.so: $(LIBDIR)/libQuEST_hip_f64.so
	ln -sf libQuEST_hip_f64.so $@

# ---------------------------------------------------------------- examples
EXAMPLES := tutorial_example damping_example bernstein_vazirani_circuit random_circuit_benchmark
examples: $(addprefix $(BUILD)/examples/,$(addsuffix _cpu,$(EXAMPLES)))
examples-hip: $(addprefix $(BUILD)/examples/,$(addsuffix _hip,$(EXAMPLES)))

$(BUILD)/examples/%_cpu: examples/%.c $(LIBDIR)/libQuEST_cpu_f64.so
	@mkdir -p $(dir $@)
	gcc -O2 -std=c99 -Iinclude $< -o $@ -L$(LIBDIR) -lQuEST_cpu_f64 -Wl,-rpath,$(abspath $(LIBDIR)) -lm

$(BUILD)/examples/%_hip: examples/%.c $(LIBDIR)/libQuEST_hip_f64.so
	@mkdir -p $(dir $@)
	gcc -O2 -std=c99 -Iinclude $< -o $@ -L$(LIBDIR) -lQuEST_hip_f64 -Wl,-rpath,$(abspath $(LIBDIR)) -lm

# ---------------------------------------------------------------- sanitizers
# Host build + the C API stress driver under AddressSanitizer and
# UndefinedBehaviorSanitizer (GPU sanitizers are not available here).
ASAN_FLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g -O1
$(BUILD)/asan/api_stress: $(CPU_SRC) tests/c/api_stress.c $(wildcard include/*.h src/*/*.hpp)
	@mkdir -p $(dir $@)
	gcc $(ASAN_FLAGS) -std=c99 -Iinclude -DQuEST_PREC=2 -c tests/c/api_stress.c -o $(BUILD)/asan/api_stress.o
	$(CXX) $(ASAN_FLAGS) -std=c++17 -fopenmp -Iinclude -DQuEST_PREC=2 $(CPU_SRC) $(BUILD)/asan/api_stress.o \
	    -o $@ -ldl -lpthread -lm

asan-check: $(BUILD)/asan/api_stress
	cd $(BUILD)/asan && ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 ./api_stress

clean:
	rm -rf $(BUILD) $(LIBDIR)/*.so $(GATECALL)

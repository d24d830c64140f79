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

COMMON_SRC := src/api/api.cpp src/api/validation.cpp src/api/qasm.cpp src/api/common.cpp src/api/checkpoint.cpp \
              src/api/mt19937.cpp src/core/router.cpp src/core/tiles.cpp src/core/trace.cpp src/comm/bootstrap.cpp
CPU_SRC    := $(COMMON_SRC) src/comm/comm_socket.cpp src/comm/comm_host.cpp src/cpu/backend_cpu.cpp
HIP_HOST   := $(COMMON_SRC) src/comm/comm_socket.cpp src/comm/comm_rccl.cpp
HIP_DEV    := src/hip/backend_hip.hip src/hip/kernels_gates.hip src/hip/kernels_direct.hip src/hip/kernels_reduce.hip src/hip/kernels_misc.hip

INCLUDES   := -Iinclude
CXXFLAGS   := -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $(INCLUDES)
HIPFLAGS   := -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-function \
              -Wno-unused-result -munsafe-fp-atomics $(INCLUDES)
HIPHOST    := -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $(INCLUDES) -I$(ROCM)/include -D__HIP_PLATFORM_AMD__

.PHONY: cpu hip all clean examples examples-hip asan-check

cpu: $(LIBDIR)/libQuEST_cpu_f64.so $(LIBDIR)/libQuEST_cpu_f32.so
hip: $(LIBDIR)/libQuEST_hip_f64.so $(LIBDIR)/libQuEST_hip_f32.so $(LIBDIR)/libQuEST.so
all: cpu hip

# ---------------------------------------------------------------- CPU build
define cpu_rules
$(BUILD)/cpu_f$(2)/%.o: %.cpp $(wildcard include/*.h src/*/*.hpp)
	@mkdir -p $$(dir $$@)
	$(CXX) $(CXXFLAGS) -fopenmp -DQuEST_PREC=$(1) -c $$< -o $$@

$(LIBDIR)/libQuEST_cpu_f$(2).so: $(patsubst %.cpp,$(BUILD)/cpu_f$(2)/%.o,$(CPU_SRC))
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -fopenmp -Wl,-Bsymbolic -o $$@ $$^ -ldl -lpthread
endef
$(eval $(call cpu_rules,2,64))
$(eval $(call cpu_rules,1,32))

# ---------------------------------------------------------------- HIP build
define hip_rules
$(BUILD)/hip_f$(2)/%.o: %.cpp $(wildcard include/*.h src/*/*.hpp)
	@mkdir -p $$(dir $$@)
	$(CXX) $(HIPHOST) -DQuEST_PREC=$(1) -c $$< -o $$@

$(BUILD)/hip_f$(2)/%.o: %.hip $(wildcard include/*.h src/*/*.hpp src/hip/*.h)
	@mkdir -p $$(dir $$@)
	$(HIPCC) $(HIPFLAGS) -DQuEST_PREC=$(1) -c $$< -o $$@

$(LIBDIR)/libQuEST_hip_f$(2).so: $(patsubst %.cpp,$(BUILD)/hip_f$(2)/%.o,$(HIP_HOST)) $(patsubst %.hip,$(BUILD)/hip_f$(2)/%.o,$(HIP_DEV))
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -Wl,-Bsymbolic --offload-arch=$(ARCH) -o $$@ $$^ -L$(ROCM)/lib -lamdhip64 -ldl -lpthread
endef
$(eval $(call hip_rules,2,64))
$(eval $(call hip_rules,1,32))

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
	rm -rf $(BUILD) $(LIBDIR)/*.so

# Locust-MI355X build (replaces the reference's CMake + vendored FindCUDA,
# /root/reference/MapReduce/CMakeLists.txt:1-35 and GNUmakefile:1-31).
#
#   make            -> locust_amd/_lib/liblocust.so, locust_amd/_locust*.so, build/MapReduce
#   make debug      -> same with -O0 -g
#   make asan       -> host-only ASan/UBSan build of the CPU engine + CLI (build/asan/)
#   make tsan       -> host-only ThreadSanitizer build of the same (build/tsan/)
#   make clean
#
# Device code targets gfx950 (MI355X) only.  Device helpers are header-only, so no
# relocatable device code (-fgpu-rdc) is needed, unlike the reference.
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
PYTHON    ?= python3
ARCH      ?= gfx950
OPT       ?= -O3
BUILD     := build
OBJ       := $(BUILD)/obj
LIBDIR    := locust_amd/_lib

PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
PY_EXT    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

COMMON    := -std=c++17 -fPIC -Icsrc/include -Wall -Wextra -Wno-unused-parameter
HIPFLAGS  := $(COMMON) $(OPT) --offload-arch=$(ARCH) -munsafe-fp-atomics
CXXFLAGS  := $(COMMON) $(OPT) -I$(ROCM)/include
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -ldl -lpthread

HIP_SRCS  := $(wildcard csrc/kernels/*.hip csrc/engine/*.hip csrc/comm/*.hip)
CPP_SRCS  := $(wildcard csrc/engine/*.cpp csrc/io/*.cpp csrc/comm/*.cpp)
HDRS      := $(wildcard csrc/include/locust/*.hpp csrc/include/locust/device/*.hpp csrc/engine/*.hpp csrc/kernels/*.hpp)

HIP_OBJS  := $(patsubst csrc/%.hip,$(OBJ)/%.o,$(HIP_SRCS))
CPP_OBJS  := $(patsubst csrc/%.cpp,$(OBJ)/%.o,$(CPP_SRCS))

LIB       := $(LIBDIR)/liblocust.so
PYMOD     := locust_amd/_locust$(PY_EXT)
CLI       := $(BUILD)/MapReduce

.PHONY: all clean debug asan
all: $(LIB) $(PYMOD) $(CLI)

$(OBJ)/%.o: csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ $(LDLIBS) -Wl,-soname,liblocust.so

$(OBJ)/python/bindings.o: csrc/python/bindings.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(PYMOD): $(OBJ)/python/bindings.o $(LIB)
	$(CXX) -shared -o $@ $< -L$(LIBDIR) -llocust -Wl,-rpath,'$$ORIGIN/_lib'

$(OBJ)/cli/main.o: csrc/cli/main.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(CLI): $(OBJ)/cli/main.o $(LIB)
	$(CXX) -o $@ $< -L$(LIBDIR) -llocust -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

debug:
	$(MAKE) OPT="-O0 -g" all

# Host-only sanitizer build: the CPU engine, I/O, TCP comm and the CLI with
# --backend cpu.  (GPU ASan / xnack+ is not available on the GPU pool.)
ASAN_SRCS := csrc/engine/common.cpp csrc/engine/cpu_wordcount.cpp csrc/engine/dist.cpp \
             csrc/io/io.cpp csrc/io/gen.cpp csrc/comm/tcp_comm.cpp csrc/cli/main.cpp \
             csrc/engine/trace.cpp csrc/engine/shm.cpp csrc/engine/numa.cpp csrc/engine/stage.cpp \
             csrc/cli/asan_stubs.cpp
asan: $(BUILD)/asan/MapReduce
$(BUILD)/asan/MapReduce: $(ASAN_SRCS) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) -std=c++17 -Icsrc/include -I$(ROCM)/include -O1 -g -fsanitize=address,undefined \
	  -fno-omit-frame-pointer -o $@ $(ASAN_SRCS) -L$(ROCM)/lib -lrocprofiler-sdk-roctx \
	  -Wl,-rpath,$(ROCM)/lib -lpthread

# Host-only ThreadSanitizer build of the same sources: the host threads (parallel preads,
# the streamed source's read pool, stage 2's per-spill readers, the CPU engine's ranks and
# TCP communicator threads) checked for data races.
TSAN_PROBE_SRCS := tools/read_probe.cpp csrc/io/io.cpp csrc/engine/common.cpp csrc/engine/trace.cpp \
                   csrc/engine/numa.cpp
tsan: $(BUILD)/tsan/MapReduce $(BUILD)/tsan/read_probe
# the streamed file source (FileTextSource: read pool threads, whole-line carry) alone
$(BUILD)/tsan/read_probe: $(TSAN_PROBE_SRCS) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) -std=c++17 -Icsrc/include -I$(ROCM)/include -O1 -g -fsanitize=thread \
	  -fno-omit-frame-pointer -o $@ $(TSAN_PROBE_SRCS) -L$(ROCM)/lib -lrocprofiler-sdk-roctx \
	  -Wl,-rpath,$(ROCM)/lib -lpthread
$(BUILD)/tsan/MapReduce: $(ASAN_SRCS) $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) -std=c++17 -Icsrc/include -I$(ROCM)/include -O1 -g -fsanitize=thread \
	  -fno-omit-frame-pointer -o $@ $(ASAN_SRCS) -L$(ROCM)/lib -lrocprofiler-sdk-roctx \
	  -Wl,-rpath,$(ROCM)/lib -lpthread

clean:
	rm -rf $(BUILD) $(LIBDIR) locust_amd/_locust*.so

# diagnostics: kernel micro-benchmarks
kbench: $(BUILD)/kbench
$(BUILD)/kbench: tools/kbench/kbench.hip $(LIB) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -Wno-unused-value -Wno-unused-result -o $@ $< -L$(LIBDIR) -llocust -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# diagnostics: what a GPU process's exit costs by how much of the GPU it touched
exit_probe: $(BUILD)/exit_probe
$(BUILD)/exit_probe: tools/exit_probe.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

# diagnostics: the streaming source's host read throughput (page cache -> ring pieces)
read_probe: $(BUILD)/read_probe
$(BUILD)/read_probe: tools/read_probe.cpp $(LIB)
	$(CXX) -O2 -std=c++17 -Icsrc/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< -L$(LIBDIR) -llocust -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

# diagnostics: each kernel file's code-object load time in a fresh process
module_probe: $(BUILD)/module_probe
$(BUILD)/module_probe: tools/micro/module_probe.cpp $(LIB)
	$(CXX) -O2 -std=c++17 -Icsrc/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< -L$(LIBDIR) -llocust -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

# diagnostics: instruction-fetch cost of straight-line code vs loops, cold and warm
icache_probe: $(BUILD)/icache_probe
$(BUILD)/icache_probe: tools/micro/icache_probe.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

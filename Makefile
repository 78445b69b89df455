# Build of the MI355X-native word-count engine (gfx950 / CDNA4 only).
#   make            -> cuda_mapreduce_amd/lib/libwc.so (Python binding) + ./wordcount (CLI)
#   make asan       -> build/wordcount_asan: host code under ASan/UBSan (GPU code unsanitised)
#   make -j8        parallel compile (hipcc ~10-30 s per kernel file)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
BUILD    ?= build
CXX      := g++
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
INCS     := -Iinclude -Isrc -I/opt/rocm/include
LIBS     := -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib

HIP_SRCS := $(wildcard src/kernels/*.hip)
CPP_SRCS := $(wildcard src/common/*.cpp src/engine/*.cpp src/dist/*.cpp src/cpu/*.cpp src/io/*.cpp src/output/*.cpp) src/capi.cpp
HIP_OBJS := $(patsubst src/%.hip,$(BUILD)/%.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst src/%.cpp,$(BUILD)/%.o,$(CPP_SRCS))
HEADERS  := $(wildcard include/wc/*.h include/wc/*.hpp src/*/*.hpp)

PYLIB    := cuda_mapreduce_amd/lib/libwc.so

all: $(PYLIB) wordcount

$(BUILD)/%.o: src/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(INCS) -c $< -o $@

$(BUILD)/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ $(INCS) -c $< -o $@

$(PYLIB): $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ $(LIBS)

$(BUILD)/tools/wordcount.o: tools/wordcount.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ $(INCS) -c $< -o $@

wordcount: $(BUILD)/tools/wordcount.o $(HIP_OBJS) $(CPP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ $(LIBS)

# Host-side sanitizers only: GPU ASan is not available on this pool.  Host
# sources are built by g++ with ASan/UBSan; the HIP objects (host stubs +
# gfx950 code objects) link in unsanitised.
ASAN     := -O1 -g -std=c++17 -fPIC -fsanitize=address,undefined -fno-omit-frame-pointer
ASAN_OBJS := $(patsubst src/%.cpp,$(BUILD)/asan/%.o,$(CPP_SRCS)) $(BUILD)/asan/tools/wordcount.o

$(BUILD)/asan/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(ASAN) -D__HIP_PLATFORM_AMD__ $(INCS) -c $< -o $@

$(BUILD)/asan/tools/wordcount.o: tools/wordcount.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(ASAN) -D__HIP_PLATFORM_AMD__ $(INCS) -c $< -o $@

asan: $(BUILD)/wordcount_asan
$(BUILD)/wordcount_asan: $(ASAN_OBJS) $(HIP_OBJS)
	$(CXX) -fsanitize=address,undefined -o $@ $^ $(LIBS)

clean:
	rm -rf $(BUILD) $(PYLIB) wordcount

.PHONY: all clean asan

# Build: the HIP engine (gfx950) and the CPU oracle (test infrastructure only).
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
ARCH    ?= gfx950
JOBS    ?= 8

LIB     := wiser_amd/_lib/libwiser_hip.so
ORACLE  := oracle/_build/liboracle.so
SRCS    := wiser_amd/csrc/writer.cc wiser_amd/csrc/index.cc wiser_amd/csrc/engine.cc \
           wiser_amd/csrc/server.cc wiser_amd/csrc/docstore.cc wiser_amd/csrc/snippet.cc \
           wiser_amd/csrc/kernels.hip
HDRS    := $(wildcard wiser_amd/csrc/*.h) include/wiser_hip.h
OBJDIR  := wiser_amd/_lib/obj
OBJS    := $(patsubst wiser_amd/csrc/%,$(OBJDIR)/%.o,$(SRCS))

# -ffp-contract=off everywhere: the reference build has no FMA (CMakeLists.txt:6,12)
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall \
            -Wno-unused-function
ORAFLAGS := -O3 -DNDEBUG -std=c++17 -fPIC -ffp-contract=off -Wall -shared

CLI     := wiser_amd/_lib/engine_cli
CALIB   := wiser_amd/_lib/calib_ea
DICT    := wiser_amd/_lib/dict_check

all: $(LIB) $(ORACLE) $(CLI) $(CALIB) $(DICT)

# CPU check of the term dictionary (tests/test_dictionary.py)
$(DICT): tests/cpp/dict_check.cc wiser_amd/csrc/index.h $(LIB)
	$(CXX) -O2 -std=c++17 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ tests/cpp/dict_check.cc -Lwiser_amd/_lib -lwiser_hip -Wl,-rpath,'$$ORIGIN'

# counter calibration (profiles only): known-byte reads for rocprofv3 --pmc
$(CALIB): scripts/calib_ea.hip
	@mkdir -p wiser_amd/_lib
	$(HIPCC) --offload-arch=$(ARCH) -O3 -o $@ $<

$(CLI): tests/cpp/engine_cli.cc include/wiser_hip_engine.hpp include/wiser_hip.h $(LIB)
	$(CXX) -O2 -std=c++17 -Iinclude -o $@ tests/cpp/engine_cli.cc -Lwiser_amd/_lib -lwiser_hip -Wl,-rpath,'$$ORIGIN'

$(OBJDIR)/%.o: wiser_amd/csrc/% $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lpthread -l:liblz4.so.1 -lrccl

$(ORACLE): oracle/oracle.cc oracle/oracle.h
	@mkdir -p oracle/_build
	$(CXX) $(ORAFLAGS) -o $@ oracle/oracle.cc -lpthread -l:liblz4.so.1

clean:
	rm -rf wiser_amd/_lib oracle/_build

.PHONY: all clean

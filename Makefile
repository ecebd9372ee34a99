# Build recipes (no cmake): the HIP product library, the synthetic-input
# library, and the CPU oracle (test infrastructure).  `python -c "import
# __graft_entry__ as g; g.build()"` runs `make all`.
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
PKG      := gf-pl-slam_amd
LIBDIR   := $(PKG)/lib

# -ffp-contract=off everywhere: bit-identical fp64 between kernels and oracle (pin N1)
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fPIC -shared \
            -Wall -Wno-unused-result -Iinclude
CXXFLAGS := -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall -Iinclude
# the oracle doubles as the timed CPU baseline: reference flags are -O3 -march=native
# (CMakeLists.txt:68); x86-64-v3 keeps the .so runnable on the GPU host.
ORACLEFLAGS := $(CXXFLAGS) -march=x86-64-v3

HIP_SRC  := $(wildcard $(PKG)/csrc/*.hip) $(wildcard $(PKG)/csrc/*.cpp)
HIP_HDR  := $(wildcard $(PKG)/csrc/*.hpp) include/gfpl.h

BINDIR   := $(PKG)/bin

all: $(LIBDIR)/libgfpl_hip.so $(LIBDIR)/libgfpl_synth.so oracle/liboracle.so $(LIBDIR)/libgfpl_stvo.so $(BINDIR)/plslam_gpu \
     $(BINDIR)/mirror_maphandler

$(LIBDIR)/libgfpl_hip.so: $(HIP_SRC) $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(HIP_SRC) -o $@

$(LIBDIR)/libgfpl_synth.so: $(PKG)/synth/gfpl_synth.cpp $(PKG)/synth/gfpl_synth.h include/gfpl.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(CXXFLAGS) -march=x86-64-v3 $< -o $@ -lpthread

# C++ host mirror of the reference's StVO classes over the C ABI, and the
# app/plslam_mod.cpp-style driver (both plain g++; no HIP headers needed)
$(LIBDIR)/libgfpl_stvo.so: $(PKG)/host/stvo.cpp $(PKG)/host/stvo.h include/gfpl.h $(LIBDIR)/libgfpl_hip.so
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -lgfpl_hip -Wl,-rpath,'$$ORIGIN'

$(BINDIR)/plslam_gpu: $(PKG)/host/plslam_gpu.cpp $(LIBDIR)/libgfpl_stvo.so $(LIBDIR)/libgfpl_synth.so
	@mkdir -p $(BINDIR)
	$(CXX) -O2 -std=c++17 -ffp-contract=off -Wall -Iinclude $< -o $@ -L$(LIBDIR) -lgfpl_stvo -lgfpl_hip -l:libgfpl_synth.so -lpthread \
	    -Wl,-rpath,'$$ORIGIN/../lib'

# a MapHandler-shaped caller of the mirror's StereoFrame members (tests/test_mirror_members.py)
$(BINDIR)/mirror_maphandler: tests/mirror_maphandler.cpp $(LIBDIR)/libgfpl_stvo.so $(LIBDIR)/libgfpl_synth.so
	@mkdir -p $(BINDIR)
	$(CXX) -O2 -std=c++17 -ffp-contract=off -Wall -Iinclude $< -o $@ -L$(LIBDIR) -lgfpl_stvo -lgfpl_hip -l:libgfpl_synth.so -lpthread \
	    -Wl,-rpath,'$$ORIGIN/../lib'

ORACLE_SRC := oracle/gfpl_oracle.cpp oracle/gfpl_orb_oracle.cpp oracle/gfpl_lbd_oracle.cpp oracle/gfpl_lsd_oracle.cpp
oracle/liboracle.so: $(ORACLE_SRC) oracle/gfpl_oracle.h include/gfpl.h $(PKG)/csrc/gfpl_orb_pattern.h
	$(CXX) $(ORACLEFLAGS) $(ORACLE_SRC) -o $@

# the CPU oracle (+ the synthetic generator and the host setup code it
# uses) under ASan + UBSan, driven over every test camera; aborts on the first report
ASANFLAGS := -O1 -g -std=c++17 -ffp-contract=off -Wall -Iinclude -fno-omit-frame-pointer \
             -fsanitize=address,undefined -fno-sanitize-recover=all
oracle/build/asan_driver: oracle/asan_driver.cpp $(ORACLE_SRC) oracle/gfpl_oracle.h \
                          $(PKG)/synth/gfpl_synth.cpp $(PKG)/csrc/gfpl_setup.cpp include/gfpl.h
	@mkdir -p oracle/build
	$(CXX) $(ASANFLAGS) oracle/asan_driver.cpp $(ORACLE_SRC) $(PKG)/synth/gfpl_synth.cpp \
	    $(PKG)/csrc/gfpl_setup.cpp -o $@ -lpthread
oracle-asan: oracle/build/asan_driver
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 ./oracle/build/asan_driver

oracle: oracle/liboracle.so
synth: $(LIBDIR)/libgfpl_synth.so
hip: $(LIBDIR)/libgfpl_hip.so
host: $(LIBDIR)/libgfpl_stvo.so $(BINDIR)/plslam_gpu $(BINDIR)/mirror_maphandler

clean:
	rm -f $(LIBDIR)/*.so oracle/liboracle.so $(BINDIR)/plslam_gpu $(BINDIR)/mirror_maphandler oracle/build/asan_driver

.PHONY: all clean oracle oracle-asan synth hip host

# Single hipcc build of the MI355X (gfx950) library, the C++ drop-in shim and
# the oracle (test infrastructure).  `make` is what __graft_entry__.build() runs.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG       = sparsematrix_amd
CSRC      = $(PKG)/csrc
LIB       = $(PKG)/libsparsematrix_amd.so
SHIM      = $(PKG)/libsblas.so
HIPFLAGS  = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fvisibility=hidden -Wall -Iinclude -I$(CSRC) $(EXTRA_HIPFLAGS)
SRCS_HIP  = $(wildcard $(CSRC)/*.hip)
SRCS_CPP  = $(filter-out $(CSRC)/sblas_shim.cpp,$(wildcard $(CSRC)/*.cpp))
OBJDIR    = build/obj
OBJS      = $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS_HIP)) \
            $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(SRCS_CPP))
HDRS      = include/sparsematrix.h $(wildcard $(CSRC)/*.h)

all: $(LIB) $(SHIM) oracle compat build/blas_test build/sblas_addmatmat

# C++ drop-in shim (reference class/kernel signatures) over the C ABI
$(SHIM): $(CSRC)/sblas_shim.cpp include/sblas/sparse-matrix.h include/sblas/kernel.h $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -fPIC -shared -Iinclude/sblas -Iinclude \
	    -o $@ $(CSRC)/sblas_shim.cpp -L$(PKG) -lsparsematrix_amd -Wl,-rpath,'$$ORIGIN'

# The reference's own unit tests (src/sparse/kernel_test.cc, sparse-matrix_test.cc),
# compiled UNCHANGED from /root/reference against include/sblas + libsblas.so.
# Only where /root/reference exists (the binaries travel to the GPU box).
REFSRC ?= /root/reference/src/sparse
COMPAT  = build/compat/kernel_test build/compat/sparse-matrix_test
ifneq ($(wildcard $(REFSRC)/kernel_test.cc),)
compat: $(COMPAT)
build/compat/%: $(REFSRC)/%.cc $(SHIM)
	@mkdir -p build/compat
	g++ -std=c++11 -O2 -w -Iinclude/sblas -o $@ $< -L$(PKG) -lsblas -lsparsematrix_amd \
	    -Wl,-rpath,'$$ORIGIN/../../$(PKG)'
else
compat:
endif

# The reference harness's command line over the GPU backend (tools/blas_test.cc).
build/blas_test: tools/blas_test.cc include/sblas/sparse-matrix.h $(SHIM)
	@mkdir -p build
	$(HIPCC) -O2 -std=c++17 -Iinclude/sblas -Iinclude -o $@ $< -L$(PKG) -lsblas -lsparsematrix_amd \
	    -Wl,-rpath,'$$ORIGIN/../$(PKG)'

# One AddMatMat through the C++ surface (tests/test_gpu_shim.py).
build/sblas_addmatmat: tools/sblas_addmatmat.cc include/sblas/sparse-matrix.h include/sparsematrix.h $(SHIM)
	@mkdir -p build
	$(HIPCC) -O2 -std=c++17 -Iinclude/sblas -Iinclude -o $@ $< -L$(PKG) -lsblas -lsparsematrix_amd \
	    -Wl,-rpath,'$$ORIGIN/../$(PKG)'

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) $(SHIM)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean compat

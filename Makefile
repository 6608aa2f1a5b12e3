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

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) $(SHIM)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean

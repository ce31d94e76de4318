# Build recipe for the product library (HIP, gfx950) and the CPU oracle.
#   make            -> both
#   make lib        -> unpaper-gpu_amd/lib/libunpaper_hip.so   (product)
#   make oracle     -> oracle/_build/liboracle.so              (test infrastructure)
#   make lib DIAG=1 -> the same library with the timing diagnostics of
#                      csrc/common.h (UPHIP_DIAG_*) compiled in; tuning only,
#                      built into its own object dir.  The default build has none.
# FP contraction is OFF everywhere: interpolation must round exactly like the
# reference's x86-64 scalar float code (reference meson uses nvcc --fmad=false).

HIPCC      ?= /opt/rocm/bin/hipcc
CC         ?= gcc
ARCH       ?= gfx950
JOBS       ?= 8

PKG        := unpaper-gpu_amd
CSRC       := $(PKG)/csrc
ORACLE_LIB := oracle/_build/liboracle.so

HIP_SRCS   := $(wildcard $(CSRC)/*.hip)
CPP_SRCS   := $(wildcard $(CSRC)/*.cpp)
C_SRCS     := $(wildcard $(CSRC)/*.c)
HDRS       := $(wildcard $(CSRC)/*.h) $(wildcard $(CSRC)/*.cuh) include/unpaper_hip.h

ifeq ($(DIAG),1)
OBJDIR     := $(PKG)/build_diag
LIBDIR     := $(PKG)/lib_diag
DIAGFLAGS  := -DUPHIP_DIAG
else
OBJDIR     := $(PKG)/build
LIBDIR     := $(PKG)/lib
DIAGFLAGS  :=
endif
LIB        := $(LIBDIR)/libunpaper_hip.so
HIP_OBJS   := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.hip.o,$(HIP_SRCS))
CPP_OBJS   := $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.cpp.o,$(CPP_SRCS))
C_OBJS     := $(patsubst $(CSRC)/%.c,$(OBJDIR)/%.c.o,$(C_SRCS))

HIPFLAGS   := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
              -fno-gpu-rdc $(DIAGFLAGS) -Iinclude -I$(CSRC) -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result \
              -Wno-pass-failed  # occupancy hints tuned for GRAY8 miss on RGB instantiations
CFLAGS_O   := -O2 -std=gnu11 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result

.PHONY: all lib oracle clean
all: lib oracle

lib: $(LIB)
oracle: $(ORACLE_LIB)

$(OBJDIR)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.c.o: $(CSRC)/%.c $(HDRS)
	@mkdir -p $(OBJDIR)
	$(CC) $(CFLAGS_O) -Iinclude -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS) $(C_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

$(ORACLE_LIB): oracle/oracle.c oracle/oracle.h include/unpaper_hip.h
	@mkdir -p oracle/_build
	$(CC) $(CFLAGS_O) -shared -o $@ oracle/oracle.c -lm

clean:
	rm -rf $(PKG)/build $(PKG)/build_diag $(PKG)/lib $(PKG)/lib_diag oracle/_build

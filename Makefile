# Build recipe for the product library (HIP, gfx950) and the CPU oracle.
#   make            -> both
#   make lib        -> unpaper-gpu_amd/lib/libunpaper_hip.so   (product)
#   make oracle     -> oracle/_build/liboracle.so              (test infrastructure)
#   make ctest      -> tests/c/_build/backend_ops              (C caller of the vtable; test)
#   make libm_check -> tests/c/_build/libm_check: the device's glibc sinf/cosf/powf
#                      restatement against the host libm (test)
#   make sanitize   -> tests/c/_build/sanitize: the oracle + the host codec
#                      under ASan/UBSan (host code only, no GPU)
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
else ifneq ($(VARIANT),)
# A/B builds: make lib VARIANT=name VFLAGS="-D..." -> lib_name/ (tuning only)
OBJDIR     := $(PKG)/build_$(VARIANT)
LIBDIR     := $(PKG)/lib_$(VARIANT)
DIAGFLAGS  := $(VFLAGS)
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

CTEST      := tests/c/_build/backend_ops
# the reference-side adapter (integration/) compiled against the reference's
# own headers, where they lie; skipped when the tree is absent (GPU box)
REFERENCE  ?= /root/reference
ADAPTER    := tests/c/_build/adapter_ops
# the reference's own PDF unit tests (tests/pdf_{reader,writer}_test.c, compiled
# where they lie) linked against integration/pdf_hip.c instead of MuPDF
REF_PDF_TESTS := tests/c/_build/ref_pdf_reader_test tests/c/_build/ref_pdf_writer_test \
                 tests/c/_build/ref_jbig2_decode_test

LIBM_CHECK := tests/c/_build/libm_check
SANITIZE   := tests/c/_build/sanitize
LLVMCC     := /opt/rocm/lib/llvm/bin/clang
SANFLAGS   := -fsanitize=address,undefined -fno-sanitize-recover=undefined \
              -fno-omit-frame-pointer -g -O1

.PHONY: all lib oracle ctest adapter sanitize libm_check jdec_emul j2k_emul clean
all: lib oracle ctest libm_check jdec_emul j2k_emul

lib: $(LIB)
oracle: $(ORACLE_LIB)
ctest: $(CTEST)
adapter: $(ADAPTER) $(REF_PDF_TESTS)

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
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread -lz

$(ORACLE_LIB): oracle/oracle.c oracle/jpeg_enc.c oracle/oracle.h include/unpaper_hip.h
	@mkdir -p oracle/_build
	$(CC) $(CFLAGS_O) -shared -o $@ oracle/oracle.c oracle/jpeg_enc.c -lm

# A plain C program: the reference's own callers are C (sheet_stages.c).
$(CTEST): tests/c/backend_ops.c tests/c/pages.h include/unpaper_hip.h oracle/oracle.h $(LIB) $(ORACLE_LIB)
	@mkdir -p tests/c/_build
	$(CC) -O2 -std=gnu11 -Wall -Iinclude $< -o $@ \
	  -L$(PKG)/lib -L oracle/_build -lunpaper_hip -loracle -lm \
	  -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib' -Wl,-rpath,'$$ORIGIN/../../../oracle/_build'

$(ADAPTER): tests/c/adapter_main.c tests/c/pages.h integration/backend_hip.c integration/backend_hip.h \
            integration/hip_frame.h include/unpaper_hip.h oracle/oracle.h $(LIB) $(ORACLE_LIB)
	@test -f $(REFERENCE)/imageprocess/image.h || { echo "adapter: no reference headers under $(REFERENCE)"; exit 1; }
	@mkdir -p tests/c/_build
	$(CC) -O2 -std=gnu11 -Wall -Wno-unused-variable -I$(REFERENCE) -Iinclude -Iintegration \
	  tests/c/adapter_main.c integration/backend_hip.c -o $@ \
	  -L$(PKG)/lib -L oracle/_build -lunpaper_hip -loracle -lm \
	  -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib' -Wl,-rpath,'$$ORIGIN/../../../oracle/_build'

tests/c/_build/ref_pdf_%_test: integration/pdf_hip.c include/unpaper_hip.h $(LIB)
	@test -f $(REFERENCE)/tests/pdf_$*_test.c || { echo "ref pdf tests: no reference tree under $(REFERENCE)"; exit 1; }
	@mkdir -p tests/c/_build
	$(CC) -O2 -std=gnu11 -Wall -Wno-unused-variable -Wno-unused-function -I$(REFERENCE) -Iinclude \
	  $(REFERENCE)/tests/pdf_$*_test.c integration/pdf_hip.c -o $@ \
	  -L$(PKG)/lib -lunpaper_hip -lm -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib'

tests/c/_build/ref_jbig2_decode_test: integration/jbig2_hip.c integration/pdf_hip.c include/unpaper_hip.h $(LIB)
	@test -f $(REFERENCE)/tests/jbig2_decode_test.c || { echo "ref jbig2 test: no reference tree under $(REFERENCE)"; exit 1; }
	@mkdir -p tests/c/_build
	$(CC) -O2 -std=gnu11 -Wall -Wno-unused-variable -Wno-unused-function -DUNPAPER_WITH_JBIG2 -DUNPAPER_WITH_PDF \
	  -I$(REFERENCE) -Iinclude $(REFERENCE)/tests/jbig2_decode_test.c integration/jbig2_hip.c integration/pdf_hip.c \
	  -o $@ -L$(PKG)/lib -lunpaper_hip -lm -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib'

# glibc sinf/cosf/powf(x, 2) restatement (csrc/libm_glibc.h) against this
# host's libm; plain g++, contraction off like the device build.
libm_check: $(LIBM_CHECK)
$(LIBM_CHECK): tests/c/libm_check.cpp $(CSRC)/libm_glibc.h
	@mkdir -p tests/c/_build
	g++ -O2 -std=c++17 -ffp-contract=off -Wall -I$(CSRC) $< -o $@ -lm -lpthread

# One compiler (ROCm clang) for every object so that one sanitizer runtime
# serves the program; the HIP sources are compiled for the host only.
$(SANITIZE): tests/c/sanitize_main.c oracle/oracle.c oracle/oracle.h $(CSRC)/pnm.cpp $(CSRC)/png.cpp \
             $(CSRC)/jpeg.cpp $(CSRC)/j2k.cpp $(CSRC)/pdf.cpp $(CSRC)/jbig2.cpp $(CSRC)/ccitt.cpp tests/c/san_stubs.cpp $(CSRC)/runtime.hip $(HDRS)
	@mkdir -p tests/c/_build/san
	$(LLVMCC) $(SANFLAGS) -std=gnu11 -ffp-contract=off -c oracle/oracle.c -o tests/c/_build/san/oracle.o
	$(LLVMCC) $(SANFLAGS) -std=gnu11 -Iinclude -c tests/c/sanitize_main.c -o tests/c/_build/san/main.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/pnm.cpp -o tests/c/_build/san/pnm.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/png.cpp -o tests/c/_build/san/png.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/jpeg.cpp -o tests/c/_build/san/jpeg.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/j2k.cpp -o tests/c/_build/san/j2k.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/pdf.cpp -o tests/c/_build/san/pdf.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/jbig2.cpp -o tests/c/_build/san/jbig2.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/ccitt.cpp -o tests/c/_build/san/ccitt.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c tests/c/san_stubs.cpp -o tests/c/_build/san/san_stubs.o
	$(HIPCC) --cuda-host-only -x hip $(SANFLAGS) -std=c++17 -Wno-unused-result -Wno-unused-value \
	  -Iinclude -I$(CSRC) -c $(CSRC)/runtime.hip -o tests/c/_build/san/runtime.o
	$(HIPCC) $(SANFLAGS) tests/c/_build/san/*.o -o $@ -lm -lz

# the device Huffman decoder's phases replayed on the CPU (test infrastructure)
JDEC_EMUL  := tests/c/_build/libjdec_emul.so
jdec_emul: $(JDEC_EMUL)
$(JDEC_EMUL): tests/c/jdec_emul.cpp $(CSRC)/jpeg_huff_core.h $(CSRC)/jpeg.h $(LIB)
	@mkdir -p tests/c/_build
	$(HIPCC) --cuda-host-only -x hip -O2 -std=c++17 -fPIC -shared -Wall -Iinclude -I$(CSRC) $< -o $@ \
	  -L$(PKG)/lib -lunpaper_hip -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib'

# the JPEG 2000 decode's device half replayed on the CPU (test infrastructure)
J2K_EMUL   := tests/c/_build/libj2k_emul.so
j2k_emul: $(J2K_EMUL)
$(J2K_EMUL): tests/c/j2k_emul.cpp $(CSRC)/j2k_dwt.h $(CSRC)/j2k.h $(CSRC)/j2k_t1.h $(CSRC)/j2k_t1_lane.h $(LIB)
	@mkdir -p tests/c/_build
	$(HIPCC) --cuda-host-only -x hip -O2 -std=c++17 -fPIC -shared -ffp-contract=off -Wall -Iinclude -I$(CSRC) $< -o $@ \
	  -L$(PKG)/lib -lunpaper_hip -Wl,-rpath,'$$ORIGIN/../../../$(PKG)/lib'

sanitize: $(SANITIZE)
	ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 $(SANITIZE) $(CURDIR)/tests/c/_build/san $(CURDIR)/tests/golden/reference

clean:
	rm -rf $(PKG)/build $(PKG)/build_diag $(PKG)/lib $(PKG)/lib_diag oracle/_build tests/c/_build

# Host-side AddressSanitizer build of the C-ABI (tests/test_gpu_asan.py), kept
# out of the product Makefile: the host code of dsce_api.hip instrumented
# (-fsanitize right after -Xarch_host: host only, no GPU sanitizer) and linked
# with the regular kernel objects (build them first with `make`) into the
# driver tools/asan/asan_driver.cpp.   make -f asan.mk
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
ROOT := $(abspath $(dir $(lastword $(MAKEFILE_LIST))))
INC := -I$(ROOT)/../include -I$(ROOT)/csrc
FLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off -Wall -Wno-unused-result
ASAN_FLAGS := -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer
LIBS := -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
HDR := $(ROOT)/csrc/dsce_common.h $(ROOT)/csrc/dsce_kernels.h $(ROOT)/../include/dsce.h
ASAN_DIR := $(ROOT)/build/asan
ASAN_BIN := $(ROOT)/../tools/asan/dsce_asan_driver

asan: $(ASAN_BIN)

$(ASAN_DIR)/dsce_api.o: $(ROOT)/csrc/dsce_api.hip $(HDR)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(FLAGS) $(ASAN_FLAGS) $(INC) -c $< -o $@

$(ASAN_DIR)/asan_driver.o: $(ROOT)/../tools/asan/asan_driver.cpp $(ROOT)/../include/dsce.h
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(FLAGS) $(ASAN_FLAGS) $(INC) -c $< -o $@

$(ASAN_BIN): $(ASAN_DIR)/asan_driver.o $(ASAN_DIR)/dsce_api.o $(ROOT)/build/kernels_mc.o $(ROOT)/build/kernels_setup.o
	$(HIPCC) $(FLAGS) $(ASAN_FLAGS) $^ -o $@ $(LIBS)

clean:
	rm -rf $(ASAN_DIR) $(ASAN_BIN)

.PHONY: asan clean

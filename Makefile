# Build of libcbft_hipcrypto (gfx950) and of the CPU oracle used by the tests.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CSRC    := concord-bft_amd/csrc
LIB     := concord-bft_amd/libcbft_hipcrypto.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall -Wno-unused-function
ORACLE_LIB := oracle/libcbft_oracle.so
# The row-parallel field code (bn254_row.h, fe25519_row.h: row_shr / row_shl moves with zero fill) is built
# without LLVM's DPP combiner: on this toolchain (ROCm 7.2 LLVM, gfx950) folding those moves into
# their consumers left non-zero values in lanes that must read 0 (a G2 addition came out wrong in
# one inlined copy and right in another; tools/microbench/g2r_dbg2.hip reproduces it, and the
# host SIMD emulation of the same source is exact).  Costs one v_mov_dpp per move.
ROWFLAGS := -mllvm -amdgpu-dpp-combine=false

.PHONY: all lib oracle clean shim fe_row_shim sanitize selftest
all: lib oracle cpu host shim fe_row_shim selftest

lib: $(LIB)

$(CSRC)/ed25519_verify.o: $(CSRC)/ed25519_verify.hip $(CSRC)/*.h
	$(HIPCC) $(HIPFLAGS) $(ROWFLAGS) -c $< -o $@

$(CSRC)/cbft_hipcrypto.o: $(CSRC)/cbft_hipcrypto.cpp include/cbft_hipcrypto.h $(CSRC)/ed25519_verify.h $(CSRC)/cbft_internal.h $(CSRC)/rsa_verify.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

BLS_DEPS := $(CSRC)/bls_kernels.h $(CSRC)/bls_common.h $(CSRC)/bn254_*.h $(CSRC)/row_lanes.h $(CSRC)/bls_ops.h $(CSRC)/sha256.h $(CSRC)/bls_glv.h
$(CSRC)/bls_kernels.o: $(CSRC)/bls_kernels.hip $(BLS_DEPS)
	$(HIPCC) $(HIPFLAGS) $(ROWFLAGS) -c $< -o $@

$(CSRC)/bls_pairing.o: $(CSRC)/bls_pairing.hip $(BLS_DEPS)
	$(HIPCC) $(HIPFLAGS) $(ROWFLAGS) -c $< -o $@

$(CSRC)/bls_msm_row.o: $(CSRC)/bls_msm_row.hip $(BLS_DEPS) $(CSRC)/bls_glv.h
	$(HIPCC) $(HIPFLAGS) $(ROWFLAGS) -c $< -o $@

$(CSRC)/bls_keys.o: $(CSRC)/bls_keys.hip $(BLS_DEPS)
	$(HIPCC) $(HIPFLAGS) $(ROWFLAGS) -c $< -o $@

$(CSRC)/rsa_verify.o: $(CSRC)/rsa_verify.hip $(CSRC)/rsa_verify.h $(CSRC)/sha256.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/cbft_rsa.o: $(CSRC)/cbft_rsa.cpp $(CSRC)/cbft_internal.h include/cbft_hipcrypto.h $(CSRC)/rsa_verify.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/cbft_bls.o: $(CSRC)/cbft_bls.cpp $(CSRC)/cbft_internal.h $(CSRC)/rsa_verify.h include/cbft_hipcrypto.h $(CSRC)/bls_kernels.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CSRC)/ed25519_verify.o $(CSRC)/cbft_hipcrypto.o $(CSRC)/bls_kernels.o $(CSRC)/bls_msm_row.o $(CSRC)/bls_pairing.o $(CSRC)/bls_keys.o $(CSRC)/cbft_bls.o $(CSRC)/rsa_verify.o $(CSRC)/cbft_rsa.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle: $(ORACLE_LIB)

$(ORACLE_LIB): oracle/ed25519_oracle.c oracle/sha512_oracle.h
	gcc -O2 -std=c11 -fPIC -shared -Wall -o $@ oracle/ed25519_oracle.c

clean:
	rm -f $(CSRC)/*.o $(LIB) $(ORACLE_LIB)

CPU_LIB := tools/cpu_baseline/libcbft_cpu_openssl.so
cpu: $(CPU_LIB)
$(CPU_LIB): tools/cpu_baseline/openssl_ed25519.c
	gcc -O2 -std=gnu11 -fPIC -shared -Wall -Wno-deprecated-declarations -o $@ $< -lcrypto -lpthread

# C++ plugin layer.  Product sources (concord::hip, BLS::Hip) compile against the reference's own
# headers in an integration build (tests/test_reference_boundary.py) and here against the
# restatements in ref_mirror/ (the reference's util / bftengine / threshsign libraries need
# Crypto++, RELIC and CMF-generated code that the image does not have).
HOST_LIB := concord-bft_amd/libcbft_host.so
HOST_DIR := concord-bft_amd/host
HOST_SRC := $(HOST_DIR)/src/hip_ed25519.cpp $(HOST_DIR)/src/hip_rsa.cpp $(HOST_DIR)/src/bls_hip.cpp $(HOST_DIR)/src/request_batch.cpp
MIRROR_SRC := $(wildcard $(HOST_DIR)/ref_mirror/src/*.cpp)
HOST_INC := -Iinclude -I$(HOST_DIR)/include -I$(HOST_DIR)/ref_mirror/include -DCBFT_WITH_CLIENT_KEYS_MAP
HOST_HDRS := $(wildcard $(HOST_DIR)/include/*.hpp $(HOST_DIR)/include/threshsign/*.hpp $(HOST_DIR)/ref_mirror/include/*.hpp $(HOST_DIR)/ref_mirror/include/threshsign/*.h)
host: $(HOST_LIB) tests/cpp/test_host tests/cpp/test_bls_host tools/host_bench
$(HOST_LIB): $(HOST_SRC) $(MIRROR_SRC) $(HOST_HDRS) $(LIB)
	g++ -O2 -std=c++17 -fPIC -shared -Wall $(HOST_INC) -o $@ $(HOST_SRC) $(MIRROR_SRC) -Lconcord-bft_amd -lcbft_hipcrypto -lcrypto -Wl,-rpath,'$$ORIGIN'
tests/cpp/test_host: tests/cpp/test_host.cpp $(HOST_LIB)
	g++ -O2 -std=c++17 -Wall -DCONCORD_BFT_TESTING $(HOST_INC) -o $@ $< -Lconcord-bft_amd -lcbft_host -lcbft_hipcrypto -lcrypto -lpthread -Wl,-rpath,'$$ORIGIN/../../concord-bft_amd'

tests/cpp/test_bls_host: tests/cpp/test_bls_host.cpp $(HOST_LIB)
	g++ -O2 -std=c++17 -Wall $(HOST_INC) -o $@ $< -Lconcord-bft_amd -lcbft_host -lcbft_hipcrypto -lcrypto -Wl,-rpath,'$$ORIGIN/../../concord-bft_amd'

# per-request path benchmark (bench.py runs it): threads calling verify() / verifySig()
tools/host_bench: tools/host_bench.cpp $(HOST_LIB)
	g++ -O2 -std=c++17 -Wall -DCONCORD_BFT_TESTING $(HOST_INC) -o $@ $< -Lconcord-bft_amd -lcbft_host -lcbft_hipcrypto -lcrypto -lpthread -Wl,-rpath,'$$ORIGIN/../concord-bft_amd'

# host build of the BN-P254 device code, for the CPU tests (and the "not RELIC" CPU baseline)
SHIM := tests/cpp/libbn254_shim.so
shim: $(SHIM)
$(SHIM): tests/cpp/bn254_shim.cpp $(CSRC)/bn254_*.h $(CSRC)/bls_ops.h $(CSRC)/sha256.h
	g++ -O3 -funroll-loops -std=c++17 -fPIC -shared -Wall -Wno-unknown-pragmas -I$(CSRC) -o $@ $< -lpthread

# host build of the row-parallel GF(2^255 - 19) code (fe25519_row.h) for tests/test_fe_row.py
FE_ROW_SHIM := tests/cpp/libfe_row_shim.so
fe_row_shim: $(FE_ROW_SHIM)
$(FE_ROW_SHIM): tests/cpp/fe_row_shim.cpp tests/cpp/row_emu.h $(CSRC)/fe25519_row.h $(CSRC)/row_lanes.h
	g++ -O2 -std=c++17 -fPIC -shared -Wall -Wno-unknown-pragmas -I$(CSRC) -Itests/cpp -o $@ $<

# Host-layer sanitizer builds (host code only: the HIP library itself is not instrumented).
# ASan+UBSan and TSan variants of the C++ host library and its tests; run on a GPU box with
# tools/sanitize.sh.
SAN_DIR := tests/cpp/san
sanitize: $(LIB) $(MIRROR_SRC) $(HOST_SRC)
	mkdir -p $(SAN_DIR)
	for s in address,undefined thread; do \
	  t=$$(echo $$s | cut -d, -f1); \
	  g++ -O1 -g -fno-omit-frame-pointer -fsanitize=$$s -std=c++17 -fPIC -shared $(HOST_INC) -o $(SAN_DIR)/libcbft_host_$$t.so $(HOST_SRC) $(MIRROR_SRC) -Lconcord-bft_amd -lcbft_hipcrypto -lcrypto -lpthread -Wl,-rpath,'$$ORIGIN/../../../concord-bft_amd' && \
	  g++ -O1 -g -fno-omit-frame-pointer -fsanitize=$$s -std=c++17 -DCONCORD_BFT_TESTING $(HOST_INC) -o $(SAN_DIR)/test_host_$$t tests/cpp/test_host.cpp -L$(SAN_DIR) -lcbft_host_$$t -Lconcord-bft_amd -lcbft_hipcrypto -lcrypto -lpthread -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../concord-bft_amd' && \
	  g++ -O1 -g -fno-omit-frame-pointer -fsanitize=$$s -std=c++17 $(HOST_INC) -o $(SAN_DIR)/test_bls_host_$$t tests/cpp/test_bls_host.cpp -L$(SAN_DIR) -lcbft_host_$$t -Lconcord-bft_amd -lcbft_hipcrypto -lcrypto -lpthread -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../concord-bft_amd' || exit 1; \
	done

# Microbenchmarks and probes under tools/microbench (not part of `all`; `make microbench`).
MB := tools/microbench
MICROBENCH := $(MB)/intrate $(MB)/intrate2 $(MB)/concurrency $(MB)/rowfp $(MB)/permlane_check $(MB)/pack_probe
microbench: $(MICROBENCH)
$(MB)/%: $(MB)/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -I$(CSRC) -Iinclude -o $@ $<
$(MB)/pack_probe: $(MB)/pack_probe.cpp
	$(HIPCC) -O2 -std=c++17 -o $@ $< -lpthread
.PHONY: microbench

# test-only device harness of the wave inversion (tests/test_inv_gpu.py; not the product library)
SELFTEST := tests/hip/libinv_selftest.so
selftest: $(SELFTEST)
$(SELFTEST): tests/hip/inv_selftest.hip $(CSRC)/safegcd30.h
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

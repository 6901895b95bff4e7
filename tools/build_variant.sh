#!/bin/bash
# Build an A/B variant of libcbft_hipcrypto.so: ed25519_verify.hip recompiled with extra -D flags,
# linked with the default objects of every other TU (run `make lib` first).
#   tools/build_variant.sh NAME "-DCBFT_DECODE_ROW=0 ..."   -> build/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
defs="$*"
C=concord-bft_amd/csrc
mkdir -p build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C -Wall -Wno-unused-function \
  -mllvm -amdgpu-dpp-combine=false $defs -c $C/ed25519_verify.hip -o build/ed_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/lib_$name.so build/ed_$name.o \
  $C/cbft_hipcrypto.o $C/bls_kernels.o $C/bls_msm_row.o $C/bls_pairing.o $C/bls_keys.o $C/cbft_bls.o $C/rsa_verify.o $C/cbft_rsa.o
rm -f build/ed_$name.o
echo "build/lib_$name.so ($defs)"

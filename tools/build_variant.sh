#!/bin/bash
# Build an A/B variant of libcbft_hipcrypto.so: one TU (default ed25519_verify; TU=bls_pairing etc.)
# recompiled with extra -D flags, linked with the default objects of every other TU (`make lib` first).
#   [TU=name] tools/build_variant.sh NAME "-DCBFT_INV_WAVE=0 ..."   -> build/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
defs="$*"
tu=${TU:-ed25519_verify}
C=concord-bft_amd/csrc
mkdir -p build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C -Wall -Wno-unused-function \
  -mllvm -amdgpu-dpp-combine=false $defs -c $C/$tu.hip -o build/${tu}_$name.o
objs=""
for o in ed25519_verify cbft_hipcrypto bls_kernels bls_msm_row bls_pairing bls_keys cbft_bls rsa_verify cbft_rsa; do
  if [ $o = $tu ]; then objs="$objs build/${tu}_$name.o"; else objs="$objs $C/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/lib_$name.so $objs
rm -f build/${tu}_$name.o
echo "build/lib_$name.so ($tu: $defs)"

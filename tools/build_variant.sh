#!/bin/bash
# Build a variant of libcbft_hipcrypto with extra compile flags, for A/B runs on the GPU box
# (select it there with CBFT_LIB=<path>).  Usage: tools/build_variant.sh <out.so> <flags...>
set -e
cd "$(dirname "$0")/.."
out=$1; shift
tmp=$(mktemp -d)
pids=()
for src in ed25519_verify.hip cbft_hipcrypto.cpp bls_kernels.hip bls_msm_row.hip bls_pairing.hip bls_keys.hip cbft_bls.cpp rsa_verify.hip cbft_rsa.cpp; do
  extra=()
  case $src in bls_keys.hip|bls_msm_row.hip|bls_pairing.hip) extra=(-mllvm -amdgpu-dpp-combine=false);; esac  # see Makefile ROWFLAGS
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Iconcord-bft_amd/csrc -Wno-unused-function "${extra[@]}" "$@" \
    -c concord-bft_amd/csrc/$src -o "$tmp/${src%.*}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed"; rm -rf "$tmp"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" "$tmp"/*.o
rm -rf "$tmp"
echo "built $out ($*)"

#!/bin/bash
# Build libkodr_rlnc.so in-tree for gfx950 (hipcc cross-compiles without a GPU).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
cd "$HERE"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
ARCH="${KODR_ARCH:-gfx950}"
mkdir -p build
FLAGS=(-O3 -std=c++17 -fPIC -Wall -Wno-unused-function ${KODR_EXTRA_FLAGS:-})
# the 256 coefficient bodies and row loop of the bit-sliced kernel
python3 csrc/gen_bs_bodies.py > csrc/gf_bs_bodies.inc
pids=()
"$HIPCC" --offload-arch="$ARCH" "${FLAGS[@]}" -c csrc/gf_kernels.hip -o build/gf_kernels.o & pids+=($!)
"$HIPCC" --offload-arch="$ARCH" "${FLAGS[@]}" -c csrc/gf_bs.hip -o build/gf_bs.o & pids+=($!)
"$HIPCC" "${FLAGS[@]}" -c csrc/capi.cpp -o build/capi.o & pids+=($!)
"$HIPCC" "${FLAGS[@]}" -c csrc/decoder_core.cpp -o build/decoder_core.o & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch="$ARCH" -shared -fPIC -o libkodr_rlnc.so build/gf_kernels.o build/gf_bs.o build/capi.o build/decoder_core.o \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
echo "built $HERE/libkodr_rlnc.so"

#!/bin/bash
# Build libkodr_rlnc.so in-tree for gfx950 (hipcc cross-compiles without a GPU).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
cd "$HERE"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
ARCH="${KODR_ARCH:-gfx950}"
OUT="${KODR_OUT:-libkodr_rlnc.so}"   # e.g. tune/libkodr_rlnc.so for a -DKODR_TUNE_MODES build
OBJ="${KODR_OBJ:-build}"
mkdir -p "$OBJ" "$(dirname "$OUT")"
FLAGS=(-O3 -std=c++17 -fPIC -Wall -Wno-unused-function ${KODR_EXTRA_FLAGS:-})
# the 256 coefficient bodies and row loop of the bit-sliced kernel
python3 csrc/gen_bs_bodies.py > csrc/gf_bs_bodies.inc
pids=()
"$HIPCC" --offload-arch="$ARCH" "${FLAGS[@]}" -c csrc/gf_kernels.hip -o "$OBJ"/gf_kernels.o & pids+=($!)
"$HIPCC" --offload-arch="$ARCH" "${FLAGS[@]}" -c csrc/gf_bs.hip -o "$OBJ"/gf_bs.o & pids+=($!)
"$HIPCC" --offload-arch="$ARCH" "${FLAGS[@]}" -c csrc/gf_elim.hip -o "$OBJ"/gf_elim.o & pids+=($!)
"$HIPCC" "${FLAGS[@]}" -c csrc/capi.cpp -o "$OBJ"/capi.o & pids+=($!)
"$HIPCC" "${FLAGS[@]}" -c csrc/capi_decoder.cpp -o "$OBJ"/capi_decoder.o & pids+=($!)
"$HIPCC" "${FLAGS[@]}" -c csrc/decoder_core.cpp -o "$OBJ"/decoder_core.o & pids+=($!)
for p in "${pids[@]}"; do wait "$p" || { echo "build failed" >&2; exit 1; }; done
"$HIPCC" --offload-arch="$ARCH" -shared -fPIC -o "$OUT" "$OBJ"/gf_kernels.o "$OBJ"/gf_bs.o "$OBJ"/gf_elim.o "$OBJ"/capi.o "$OBJ"/capi_decoder.o "$OBJ"/decoder_core.o \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
echo "built $HERE/$OUT"

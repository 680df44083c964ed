#!/bin/bash
# B = 1 at 32 MiB/256 on tile {1,16,2}: full kernel, no GF arithmetic (MODE 1,
# loads + tables + reduction) and no loads (MODE 2, arithmetic only), from a
# KODR_TUNE_MODES build in kodr_amd/tune_m1/; then the streaming-read probe.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export KODR_RLNC_LIB="$R/kodr_amd/tune_m1/libkodr_rlnc.so"
for rep in 1 2; do
  for mode in 0 1 2; do
    KODR_GEMM_MODE=$mode timeout -k 10 120 python tools/tune_gemm.py --M 1 --tiles "1,16,2" --iters 200 \
      | sed "s/^/mode=$mode /" || exit 1
  done
done
unset KODR_RLNC_LIB
timeout -k 10 180 python tools/probe/probe.py > gpurun_out/m1_probe.log 2>&1 || { tail -5 gpurun_out/m1_probe.log; exit 1; }
grep read_tiles gpurun_out/m1_probe.log

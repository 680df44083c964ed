#!/bin/bash
# SQ counters of gf_bs_kernel at batch B (two --pmc passes, no tracing domains).
# usage: tools/pmc_sq.sh B [lib] [mode]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
B=${1:-32}
export TMPDIR=/tmp KODR_RLNC_LIB=${2:-$R/kodr_amd/libkodr_rlnc.so}
MODE=${3:-0}
OUT="$R/gpurun_out/pmc_sq_B${B}_m$MODE"; mkdir -p "$OUT"
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/bs_modes.py" "$B" "$MODE" \
    > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_sq.py" "$OUT"

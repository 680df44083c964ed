#!/bin/bash
# Instruction-cache counters of gf_bs_kernel at batch B (two --pmc passes of
# two SQC counters each, no tracing domains).  usage: tools/pmc_icache.sh B [lib] [mode] [tag]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
B=${1:-32}
export TMPDIR=/tmp KODR_RLNC_LIB=${2:-$R/kodr_amd/libkodr_rlnc.so}
MODE=${3:-0}
OUT="$R/gpurun_out/pmc_icache_B${B}_m$MODE${4:+_$4}"; mkdir -p "$OUT"
cd /tmp
i=0
for P in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" "SQ_IFETCH SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/bs_modes.py" "$B" "$MODE" \
    > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_sq.py" "$OUT"

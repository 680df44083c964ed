#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains) for a
# gf_gemm tile.  usage: tools/pmc.sh TAG M CFG
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; M=$2; CFG=$3
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp KODR_GEMM_CFG=$CFG
cd /tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/prof_gemm.py" "$M" 40 > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "pmc $TAG ok"

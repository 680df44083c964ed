#!/bin/bash
# SQ counters of the final tree's grouped bit-sliced launches (the B = 32
# encode leg and the round trip's encode and GetPieces) from two --pmc passes
# of bench.py --no-extras (no tracing domains), per (kernel, grid)
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT="$R/gpurun_out/${1:-sq_r5}"; mkdir -p "$OUT"
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" \
    --steps 10 --warmup 3 --no-extras --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_sq_grid.py" "$OUT" | tee "$OUT/summary.txt"

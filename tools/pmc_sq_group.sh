#!/bin/bash
# SQ counters of the grouped headline launch (bench.py --no-extras --no-encode-decode: every
# gf_bs_kernel<.., true> launch in the run is a headline launch), two --pmc
# passes without tracing domains, averaged per launch by tools/pmc_sq.py.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_sq_group${1:+_$1}"; mkdir -p "$OUT"   # $1: a tag (e.g. the KODR_BS_MODE of a tuning build)
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" \
    --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-encode-decode > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
# the grouped launches are gf_bs_kernel<KW, 0, true, N>
python3 "$R/tools/pmc_sq.py" "$OUT" ", true, " | tee "$OUT/summary.txt"

#!/bin/bash
# The clock a grouped bit-sliced launch runs at: GRBM_GUI_ACTIVE / duration
# (tools/clock_pmc.py) for the product build's B = 32 / 256 launches and the
# tuning build's no-row-stream bound (MODE 31, kodr_amd/tune_m/), one --pmc
# pass each (two GRBM counters, no tracing domains)
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT="$R/gpurun_out/${1:-clock}"; mkdir -p "$OUT"
cd /tmp
for v in prod:0 tune:31 tune:0; do
  lib=${v%%:*}; M=${v##*:}
  libp="$R/kodr_amd/libkodr_rlnc.so"; [ $lib = tune ] && libp="$R/kodr_amd/tune_m/libkodr_rlnc.so"
  KODR_BS_MODE=$M KODR_RLNC_LIB=$libp timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$OUT/${lib}_m$M" -o run --output-format csv -- python3 "$R/tools/group_bs_time.py" 32 256 \
    > "$OUT/${lib}_m$M.log" 2>&1 || { tail -5 "$OUT/${lib}_m$M.log"; exit 1; }
  echo "== $lib mode $M: $(grep -E "^(32|256) " "$OUT/${lib}_m$M.log" | sed 's/"single[^,]*, //; s/, "speedup[^}]*//' | tr "\n" " ")"
  python3 "$R/tools/clock_pmc.py" "$OUT/${lib}_m$M" | head -6
done

#!/bin/bash
# North-star grouped encode (one coded piece per 32 MiB/256 generation, G per
# launch): kernel trace, then separate FETCH_SIZE and WRITE_SIZE passes
# (MI355X_MICROARCH.md HBM section), summarised by tools/pmc_summary.py.
# usage: tools/pmc_group.sh [G] [COUNT]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export G="${1:-16}" COUNT="${2:-1}" TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_group_G${G}_c${COUNT}"
mkdir -p "$OUT"
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/tools/prof_group.py" > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; tail -5 "$OUT/trace.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
  python3 "$R/tools/prof_group.py" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -5 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
  python3 "$R/tools/prof_group.py" > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -5 "$OUT/write.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" "$COUNT" gf_gemm_kernel > "$OUT/summary.json"
cat "$OUT/summary.json" "$OUT/trace.log"

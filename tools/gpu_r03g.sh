#!/bin/bash
# Recode B = 32: where the time goes -- rocprof kernel durations with the
# side product (register / LDS-staged) and without (separate vector launch),
# beside encode B = 32 (tools/compact_time.py).
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/${1:-r03g}"; mkdir -p "$OUT"
export TMPDIR=/tmp
for V in "0 0" "1 0" "1 1"; do
  set -- $V
  KODR_REC_SIDE=$1 KODR_SIDE_STAGE=$2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/rec_s$1_t$2" -o run -- \
    python3 "$R/tools/recode_time.py" 32 > "$OUT/rec_s$1_t$2.log" 2>&1 || { tail -20 "$OUT/rec_s$1_t$2.log"; exit 1; }
  echo "side=$1 stage=$2 $(tail -1 "$OUT/rec_s$1_t$2.log")"
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/enc" -o run -- python3 "$R/tools/compact_time.py" > "$OUT/enc.log" 2>&1 || { tail -20 "$OUT/enc.log"; exit 1; }
tail -1 "$OUT/enc.log"
python3 "$R/tools/kernel_durations.py" "$OUT/rec_s0_t0" "$OUT/rec_s1_t0" "$OUT/rec_s1_t1" "$OUT/enc"

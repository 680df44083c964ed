#!/bin/bash
# Round-4 rocprof evidence (run on the GPU box; summaries copied into
# profiles/r04/ afterwards):
#   1. tools/profile_headline.sh: kernel trace of the driver's command
#      (bench.py --steps 20 --warmup 5) with the headline launches picked out,
#      then separate FETCH_SIZE / WRITE_SIZE passes over the headline alone;
#   2. a kernel trace of bench.py --no-extras (headline + encode_decode round
#      trip only), summarised per round-trip kernel by tools/prof_roundtrip.py;
#   3. tools/pmc_sq_group.sh: SQ counters of the headline launch.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-r04prof}"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
bash "$R/tools/profile_headline.sh" > "$OUT/headline.txt" 2>&1 || { tail -20 "$OUT/headline.txt"; exit 1; }
cat "$OUT/headline.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rt" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_rt.json" 2> "$OUT/rt.err" \
  || { tail -20 "$OUT/rt.err"; exit 1; }
python3 "$R/tools/prof_roundtrip.py" "$OUT/rt/run_kernel_trace.csv" "$OUT/bench_rt.json" --out "$OUT/roundtrip.json" \
  || exit 1
head -c 3000 "$OUT/roundtrip.json"; echo
bash "$R/tools/pmc_sq_group.sh" r04 > "$OUT/sq.txt" 2>&1 || { tail -20 "$OUT/sq.txt"; exit 1; }
cat "$OUT/sq.txt"

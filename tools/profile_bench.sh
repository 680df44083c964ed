#!/bin/bash
# rocprofv3 evidence for the headline bench command (run on the GPU box):
#   1. --kernel-trace --stats of `bench.py` (per-kernel average duration)
#   2. separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (no tracing
#      domains), summarised into HBM bytes per gf_gemm launch.
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}; B=${2:-8}
OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$R/bench.py" --no-cpu-baseline --no-extras --steps 100 --batch "$B")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${BENCH[@]}" \
  > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- "${BENCH[@]}" \
  > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || { tail -20 "$OUT/fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- "${BENCH[@]}" \
  > "$OUT/bench_write.json" 2> "$OUT/write.err" || { tail -20 "$OUT/write.err"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" "$B" > "$OUT/summary.json" && cat "$OUT/summary.json"

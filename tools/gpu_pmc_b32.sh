#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over the B = 32 encode leg alone (bench.py
# --no-encode-decode --no-extras), summarised per launch by pmc_summary.py
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-pmcb32}"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
HB=(python3 "$R/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-encode-decode)
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- "${HB[@]}" > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- "${HB[@]}" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || { tail -20 "$OUT/fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- "${HB[@]}" > "$OUT/bench_write.json" 2> "$OUT/write.err" || { tail -20 "$OUT/write.err"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" 32 "gf_bs_kernel<" 4096 headline > "$OUT/pmc_summary.json" && cat "$OUT/pmc_summary.json"

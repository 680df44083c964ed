#!/bin/bash
# rocprofv3 evidence for the headline, round 2 (grouped step):
#   1. --kernel-trace --stats of the driver's command (bench.py --steps 20
#      --warmup 5, extras included) + tools/prof_headline.py: the timed
#      launches' rocprof average against the bench line's HIP-event average;
#   2. separate --pmc FETCH_SIZE / WRITE_SIZE passes over the headline alone
#      (--no-extras), summarised per launch by tools/pmc_summary.py.
# Outputs under gpurun_out/profh/; the summaries are copied into profiles/.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/profh"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" \
  || { tail -20 "$OUT/trace.err"; exit 1; }
python3 "$R/tools/prof_headline.py" "$OUT/trace/run_kernel_trace.csv" "$OUT/bench_trace.json" \
  --out "$OUT/prof_headline.json" > /dev/null || exit 1
HB=(python3 "$R/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-encode-decode)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- "${HB[@]}" \
  > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || { tail -20 "$OUT/fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- "${HB[@]}" \
  > "$OUT/bench_write.json" 2> "$OUT/write.err" || { tail -20 "$OUT/write.err"; exit 1; }
# the headline launch's grid (threads): the most common gf_bs_kernel grid of the PMC runs
python3 "$R/tools/pmc_summary.py" "$OUT" 32 "gf_bs_kernel<" 4096 headline > "$OUT/pmc_summary.json" || exit 1
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
h = json.load(open(o + "/prof_headline.json"))
p = json.load(open(o + "/pmc_summary.json"))
print(json.dumps({k: h[k] for k in ("kernel", "grid", "timed_launches", "rocprof_avg_us", "bench_events_avg_launch_us",
                                    "events_over_rocprof", "bench_value", "hbm_frac_from_rocprof")}))
print(json.dumps(p))
PY

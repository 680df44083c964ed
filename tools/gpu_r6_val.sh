#!/bin/bash
# Round-6 validation on one lease: the GPU suite, smoke, the driver's bench
# command unprofiled, the same command under rocprofv3 --kernel-trace --stats
# (tools/prof_roundtrip.py: each leg's rocprof average against the bench
# line's HIP events), separate FETCH_SIZE / WRITE_SIZE passes for the round
# trip's encode launch (tools/pmc_roundtrip.py) and one SQ/GRBM pass for the
# VALU anchor of both gf_bs_kernel legs (tools/pmc_valu.py).
# usage: tools/gpu_r6_val.sh [tag]   (outputs under gpurun_out/<tag>/)
#   SKIP_TESTS=1: no suite/smoke; SKIP_PMC=1: no counter passes
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
OUT="$R/gpurun_out/${1:-r6val}"; mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  echo "tests: $(tail -1 "$OUT/pytest_gpu.log")"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "alone_us", d["roofline"].get("avg_launch_us"))
print("rt", d["roundtrip"])
print("encode", d["encode"]["value"], d["encode"]["ms_per_step"], d["encode"]["roofline"]["frac"])
legs = d["roofline"]["legs"]
print({k: (v.get("avg_us"), v.get("alone_us"), v.get("issue_frac"), v.get("valu")) for k, v in legs.items() if isinstance(v, dict)})
x = d.get("extras", {})
for key in ("c2_decode", "c2_decode_grouped", "c4_systematic_decode"):
    v = x.get(key)
    if isinstance(v, dict):
        print(key, {a: b for a, b in v.items() if not isinstance(b, (list, dict))})
PY
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" \
  || { tail -20 "$OUT/trace.err"; exit 1; }
python3 "$R/tools/prof_roundtrip.py" "$OUT/trace/run_kernel_trace.csv" "$OUT/bench_trace.json" \
  --out "$OUT/prof_driver.json" && cat "$OUT/prof_driver.json" || exit 1
[ -n "${SKIP_PMC:-}" ] && exit 0
HB=(python3 "$R/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline)
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- "${HB[@]}" \
  > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || { tail -20 "$OUT/fetch.err"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- "${HB[@]}" \
  > "$OUT/bench_write.json" 2> "$OUT/write.err" || { tail -20 "$OUT/write.err"; exit 1; }
python3 "$R/tools/pmc_roundtrip.py" "$OUT" "$OUT/bench_fetch.json" > "$OUT/pmc_roundtrip.json" && cat "$OUT/pmc_roundtrip.json"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/valu" -o run \
  --output-format csv -- "${HB[@]}" > "$OUT/bench_valu.json" 2> "$OUT/valu.err" || { tail -20 "$OUT/valu.err"; exit 1; }
python3 "$R/tools/pmc_valu.py" "$OUT/valu" "$OUT/bench_valu.json" > "$OUT/pmc_valu.json" && cat "$OUT/pmc_valu.json"

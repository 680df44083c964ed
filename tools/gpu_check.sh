#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; steps are chained so the first
# failure ends the session.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STAGE="${1:-all}"
run() { echo "== $*" >&2; "$@"; }
if [[ "$STAGE" == all || "$STAGE" == tests ]]; then
  run timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
if [[ "$STAGE" == all || "$STAGE" == bench ]]; then
  run timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
if [[ "$STAGE" == all || "$STAGE" == prof ]]; then
  cd /tmp
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 "$R/bench.py" --no-cpu-baseline --no-extras --steps 200 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
  find "$OUT/prof" -name "*stats*" | head
fi

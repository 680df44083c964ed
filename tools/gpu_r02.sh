#!/bin/bash
# Round-2 GPU session: new parity tests first, then the full -m gpu suite,
# the default bench, and the rocprofv3 kernel trace of the driver's exact
# bench command.  Each GPU step has its own time limit; the first failure ends
# the session.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
OUT="$R/gpurun_out/r02"
mkdir -p "$OUT"
export TMPDIR=/tmp
STAGES="${*:-new all bench prof}"
for st in $STAGES; do
  case "$st" in
    new)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
      tail -3 "$OUT/pytest_new.log" ;;
    all)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
        || { tail -30 "$OUT/bench_driver.err"; exit 1; }
      cat "$OUT/bench_driver.json" ;;
    prof)
      cd /tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
        || { tail -30 "$OUT/prof.err"; exit 1; }
      cd "$R"
      find "$OUT/prof" -name "*kernel_stats*" ;;
  esac
done

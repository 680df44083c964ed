#!/bin/bash
# Round 6: the twin copy's footprint beside the pipelined encode: the driver's
# bench command (--no-extras) on a -DKODR_TUNE build (kodr_amd/tune_cp) with
# KODR_COPY_WG_PER_CU = 16 (the shipped cap), 8, 4, 2, 1 workgroups per CU,
# two interleaved reps; kernel traces of the best and the shipped setting.
# First the co-residency tests (the hook runs once the work ahead is done).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coresidency.py \
  > $O/pytest.log 2>&1; ok $? pytest
grep -E "PASS|FAIL|SKIP" $O/pytest.log | cut -c1-150
for rep in 1 2; do
  for w in 16 8 4 2 1; do
    KODR_RLNC_LIB=kodr_amd/tune_cp/libkodr_rlnc.so KODR_COPY_WG_PER_CU=$w timeout -k 10 300 python -u bench.py \
      --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err
    ok $? bench_w$w
  done
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "ok", d["roundtrip"]["roundtrip_ok"],
          d["roundtrip"]["elimination_routes"])
PY
for w in 16 2; do
  KODR_RLNC_LIB=kodr_amd/tune_cp/libkodr_rlnc.so KODR_COPY_WG_PER_CU=$w timeout -k 10 300 rocprofv3 --kernel-trace \
    --stats -d $O/trace_w$w -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
    --no-cpu-baseline > $O/trace_w$w.json 2> $O/trace_w$w.err; ok $? trace_w$w
  echo "w=$w"; python3 tools/step_timeline.py $O/trace_w$w/run_kernel_trace.csv 10 2
done

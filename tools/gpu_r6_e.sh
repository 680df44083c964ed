#!/bin/bash
# Round 6: the pipelined round trip without the host wait before AddPiece
# (--overlap elim: the library calls the hook once the work ahead of the
# elimination is done) against the host-wait variant (--overlap elim_sync) and
# the serial round trip, three interleaved reps; the pipelined tests; a kernel
# trace of --overlap elim for tools/step_timeline.py.
# Continues past a failed test (exit 1); stops at anything else.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_headline.py::test_bench_roundtrip_pipelined_exact > $O/pytest.log 2>&1; ok $? pytest
grep -E "PASS|FAIL|ERROR" $O/pytest.log | cut -c1-160; tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in elim elim_sync serial; do
    a="--overlap $v"; [ $v = serial ] && a="--serial-roundtrip"
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline $a \
      > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; ok $? bench_$v
  done
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception as e:
        print(f, "no line", e); continue
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "routes",
          d["roundtrip"]["elimination_routes"], "ok", d["roundtrip"]["roundtrip_ok"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err
ok $? trace
python3 tools/step_timeline.py $O/trace/run_kernel_trace.csv 10 3

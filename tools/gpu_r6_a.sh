#!/bin/bash
# Round 6, first GPU lease: the pipelined round trip against the serial one
# (bench.py --serial-roundtrip), the round's new GPU tests, the C4-shape
# elimination A/B (host vs mc4 at k = 128 and 256, tools/elim_time.py), then the
# round-5 fault configuration in bounds-checked builds (tools/gpu_r6_fault.sh's
# two runs).  Continues past a failed test (exit 1); stops at anything else
# (a fault, an abort, a time limit).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; ok $? bench
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --serial-roundtrip --no-extras \
  > $O/bench_serial.json 2> $O/bench_serial.err; ok $? bench_serial
python3 - $O/bench.json $O/bench_serial.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception as e:
        print(f, "no line", e); continue
    legs = d["roofline"]["legs"]
    print(f, "value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "alone_us",
          d["roofline"].get("avg_launch_us"), "routes", d["roundtrip"]["elimination_routes"], "ok",
          d["roundtrip"]["roundtrip_ok"])
    print("  legs", {k: (v.get("avg_us"), v.get("alone_us")) for k, v in legs.items() if isinstance(v, dict)})
PY
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_headline.py::test_bench_roundtrip_pipelined_exact tests/test_gpu_headline.py::test_bench_roundtrip_step_exact \
  tests/test_gpu_coresidency.py tests/test_gpu_elim_route.py tests/test_gpu_destroy_async.py \
  tests/test_gpu_zz_session_coresidency.py > $O/pytest_new.log 2>&1; ok $? pytest
tail -3 $O/pytest_new.log
timeout -k 10 300 python -u tools/elim_time.py 128,256 1 131072 > $O/elim_c4.log 2>&1; ok $? elim_time
cat $O/elim_c4.log
O2=gpurun_out/r6_fault; mkdir -p $O2
KODR_RLNC_LIB=kodr_amd/chk_plain/libkodr_rlnc.so KODR_ELIM_MC=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
  -d $O2/plain_g8 -o run --output-format csv -- python3 tools/elim_time.py 256 8 256 > $O2/plain_g8.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "plain_g8 rc $rc"; tail -5 $O2/plain_g8.log; exit $rc; }
KODR_RLNC_LIB=kodr_amd/chk_probe/libkodr_rlnc.so KODR_ELIM_MC=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
  -d $O2/probe_g8 -o run --output-format csv -- python3 tools/elim_time.py 256 8 256 > $O2/probe_g8.log 2>&1
rc=$?
grep -h '^{' $O2/*.log | cut -c1-200
grep -c "KODR_MC_CHECK site" $O2/plain_g8.log $O2/probe_g8.log
exit $rc

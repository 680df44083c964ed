#!/bin/bash
# Round 6: stream priority range on the box; the round trip's pipelining A/B
# (bench.py --no-extras: --overlap elim / elim_only / --serial-roundtrip, two
# interleaved reps); the pipelined and co-residency tests; then the round-5
# fault configuration (mc4 forced, 8 decoders = 264 workgroups, launch cap
# raised to 1024) in bounds-checked builds, without and with the round-5 probe.
# Continues past a failed test (exit 1); stops at anything else.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 60 python3 -c "
import ctypes
l = ctypes.CDLL('tests/cpp/libkodr_occupy.so')
a, b = ctypes.c_int(), ctypes.c_int()
print('stream priority range (least, greatest):', l.kodr_test_stream_priority_range(0, ctypes.byref(a), ctypes.byref(b)), a.value, b.value)
" > $O/prio.log 2>&1; ok $? prio; cat $O/prio.log
for rep in 1 2; do
  for v in elim elim_only serial; do
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
    legs = d["roofline"]["legs"]
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "routes",
          d["roundtrip"]["elimination_routes"], "ok", d["roundtrip"]["roundtrip_ok"],
          "legs", {k: (v.get("avg_us"), v.get("alone_us")) for k, v in legs.items() if isinstance(v, dict)})
PY
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_headline.py::test_bench_roundtrip_pipelined_exact tests/test_gpu_coresidency.py \
  tests/test_gpu_zz_session_coresidency.py > $O/pytest_new.log 2>&1; ok $? pytest
grep -E "PASS|FAIL|ERROR|call " $O/pytest_new.log | cut -c1-200; tail -2 $O/pytest_new.log
O2=gpurun_out/r6_fault; mkdir -p $O2
KODR_RLNC_LIB=kodr_amd/chk_plain/libkodr_rlnc.so KODR_ELIM_MC=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
  -d $O2/plain_g8 -o run --output-format csv -- python3 tools/elim_time.py 256 8 256 > $O2/plain_g8.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "plain_g8 rc $rc"; tail -5 $O2/plain_g8.log; exit $rc; }
grep -h "KODR_MC_CHECK launch" $O2/plain_g8.log | sort | uniq -c | head -3
KODR_RLNC_LIB=kodr_amd/chk_probe/libkodr_rlnc.so KODR_ELIM_MC=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
  -d $O2/probe_g8 -o run --output-format csv -- python3 tools/elim_time.py 256 8 256 > $O2/probe_g8.log 2>&1
rc=$?
grep -h '^{' $O2/*.log | cut -c1-200
grep -c "KODR_MC_CHECK site" $O2/plain_g8.log $O2/probe_g8.log
grep -h "KODR_MC_CHECK launch" $O2/probe_g8.log | sort | uniq -c | head -3
grep -h "gf_elim" $O2/plain_g8/*kernel_stats.csv $O2/probe_g8/*kernel_stats.csv | cut -d, -f1-6 | cut -c1-160
exit $rc

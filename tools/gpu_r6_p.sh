#!/bin/bash
# Round 6: the mc2 chain waves' sleep between hand-off polls (agent-scope
# loads of every lane; s_sleep 2 shipped) beside the pipelined encode:
# A/B builds with -DKODR_MC2_POLL_SLEEP=8 / 32 (kodr_amd/ab_sl8, ab_sl32):
# the round-trip parity test on each, the driver's bench command
# (--no-extras) three interleaved reps, and the 16-decoder elimination alone
# (tools/elim_time.py 256 16, rocprof).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
for v in sl8 sl32; do
  KODR_RLNC_LIB=kodr_amd/ab_$v/libkodr_rlnc.so timeout -k 10 300 python -u -m pytest -q --timeout 200 \
    --timeout-method thread -m gpu "tests/test_gpu_headline.py::test_bench_roundtrip_pipelined_exact" \
    tests/test_gpu_elim_route.py > $O/pytest_$v.log 2>&1; ok $? pytest_$v
  tail -1 $O/pytest_$v.log
done
for rep in 1 2 3; do
  for v in ship sl8 sl32; do
    lib=kodr_amd/libkodr_rlnc.so; [ $v != ship ] && lib=kodr_amd/ab_$v/libkodr_rlnc.so
    KODR_RLNC_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; ok $? bench_$v
  done
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "ok", d["roundtrip"]["roundtrip_ok"],
          d["roundtrip"]["elimination_routes"], "serial add leg", d["roofline"]["legs"]["add_pieces_call"]["avg_us"])
PY
for v in ship sl8 sl32; do
  lib=kodr_amd/libkodr_rlnc.so; [ $v != ship ] && lib=kodr_amd/ab_$v/libkodr_rlnc.so
  KODR_RLNC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/elim_$v -o run --output-format csv -- \
    python3 tools/elim_time.py 256 16 131072 > $O/elim_$v.log 2>&1; ok $? elim_$v
  echo "$v: $(grep -h gf_elim_mc2 $O/elim_$v/run_kernel_stats.csv | cut -d, -f2-4)"
done

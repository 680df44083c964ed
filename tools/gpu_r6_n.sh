#!/bin/bash
# Round 6: the bit-sliced kernel's output rows stored with streaming
# (nontemporal) stores (-DKODR_BS_NT_STORE=1, kodr_amd/ab_nts) against the
# shipped build: the GPU headline tests on the A/B build, the driver's bench
# command (--no-extras), three interleaved reps, grouped launches at B = 258 /
# 256 / 32 (tools/group_bs_time.py, a first B = 16 absorbing the warm-up),
# and a kernel trace of each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
KODR_RLNC_LIB=kodr_amd/ab_nts/libkodr_rlnc.so timeout -k 10 300 python -u -m pytest -q --timeout 200 \
  --timeout-method thread -m gpu tests/test_gpu_headline.py > $O/pytest_nts.log 2>&1; ok $? pytest_nts
tail -1 $O/pytest_nts.log
for rep in 1 2 3; do
  for v in ship nts; do
    lib=kodr_amd/libkodr_rlnc.so; [ $v = nts ] && lib=kodr_amd/ab_nts/libkodr_rlnc.so
    KODR_RLNC_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; ok $? bench_$v
  done
done
for v in ship nts; do
  lib=kodr_amd/libkodr_rlnc.so; [ $v = nts ] && lib=kodr_amd/ab_nts/libkodr_rlnc.so
  KODR_RLNC_LIB=$lib timeout -k 10 200 python -u tools/group_bs_time.py 16 258 256 32 > $O/group_$v.log 2>&1; ok $? group_$v
  echo "group $v"; grep -v "^{" $O/group_$v.log
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "ok", d["roundtrip"]["roundtrip_ok"],
          "serial add leg", d["roofline"]["legs"]["add_pieces_call"]["avg_us"])
PY
for v in ship nts; do
  lib=kodr_amd/libkodr_rlnc.so; [ $v = nts ] && lib=kodr_amd/ab_nts/libkodr_rlnc.so
  KODR_RLNC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/trace_$v.json 2> $O/trace_$v.err
  ok $? trace_$v
  echo "$v"; python3 tools/step_timeline.py $O/trace_$v/run_kernel_trace.csv 10 2
done

#!/bin/bash
# Round 6: the elimination's register footprint beside the pipelined encode:
# gf_elim_mc2_kernel capped by amdgpu_waves_per_eu (tuning builds with
# -DKODR_MC2_WAVES_PER_EU=5: 96 VGPRs, kodr_amd/tune_w5; =6: 80 VGPRs,
# kodr_amd/tune_w6; =8, 64 VGPRs, measured slower: 159 spills), so that encode waves fit beside its workgroups, against
# the shipped build (128 VGPRs): the round-trip parity test on each, then the
# driver's bench command (--no-extras), three interleaved reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
for v in w5 w6; do
  KODR_RLNC_LIB=kodr_amd/tune_$v/libkodr_rlnc.so timeout -k 10 300 python -u -m pytest -q --timeout 200 \
    --timeout-method thread -m gpu "tests/test_gpu_headline.py::test_bench_roundtrip_pipelined_exact" \
    > $O/pytest_$v.log 2>&1; ok $? pytest_$v
  tail -1 $O/pytest_$v.log
done
for rep in 1 2 3; do
  for v in ship w5 w6; do
    lib=kodr_amd/libkodr_rlnc.so; [ $v != ship ] && lib=kodr_amd/tune_$v/libkodr_rlnc.so
    KODR_RLNC_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; ok $? bench_$v
  done
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    legs = d["roofline"]["legs"]
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "ok", d["roundtrip"]["roundtrip_ok"],
          d["roundtrip"]["elimination_routes"], "serial add leg", legs["add_pieces_call"]["avg_us"])
PY

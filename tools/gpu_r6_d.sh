#!/bin/bash
# Round 6: the split tail (k + 2 = 258 pieces: 256 bit-sliced + 2 on gf_gemm)
# in the grouped encode (tools/group_bs_time.py 258 256, tuning build
# kodr_amd/ab_modes with KODR_SPLIT_TAIL=0/1, interleaved); its parity tests;
# the round trip A/B (--overlap elim with the idle start / --serial-roundtrip,
# interleaved, product build).  Continues past a failed test (exit 1) only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_headline.py > $O/pytest_headline.log 2>&1; ok $? pytest
grep -E "FAIL|ERROR" $O/pytest_headline.log | head; tail -1 $O/pytest_headline.log
for s in 2 0 1 2 0 1; do
  KODR_RLNC_LIB=kodr_amd/ab_modes/libkodr_rlnc.so KODR_SPLIT_TAIL=$s timeout -k 10 200 python -u tools/group_bs_time.py 258 256 \
    > $O/split_$s.log 2>&1; ok $? split_$s
  echo "split $s: $(tail -1 $O/split_$s.log | cut -c1-300)"
done
for rep in 1 2; do
  for v in elim serial; do
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
          "legs", {k: v.get("avg_us") for k, v in legs.items() if isinstance(v, dict)},
          "pipe", legs.get("pipelined_in_step"))
PY

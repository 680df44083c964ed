#!/bin/bash
# Round 6: the bit-sliced kernel's block order past 32 row groups (bands of
# 32, gf_bs.hip) against the previous single cycle over all row groups
# (kodr_amd/ab_old_map): the encode / parity GPU tests on the new build, then
# grouped launches at B = 258 / 256 over 16 prepared 32 MiB/256 generations
# (tools/group_bs_time.py) and the driver's bench command (--no-extras), new
# and old interleaved, three reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r6k; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_headline.py \
  tests/test_gpu_parity.py > $O/pytest.log 2>&1; ok $? pytest
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in new old; do
    lib=kodr_amd/libkodr_rlnc.so; [ $v = old ] && lib=kodr_amd/ab_old_map/libkodr_rlnc.so
    KODR_RLNC_LIB=$lib timeout -k 10 200 python -u tools/group_bs_time.py 258 256 > $O/group_${v}_$rep.log 2>&1
    ok $? group_$v
    echo "group $v $rep: $(tail -1 $O/group_${v}_$rep.log | cut -c1-300)"
    KODR_RLNC_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; ok $? bench_$v
  done
done
python3 - $O/bench_*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"],
          "ok", d["roundtrip"]["roundtrip_ok"], d["roundtrip"]["elimination_routes"])
PY

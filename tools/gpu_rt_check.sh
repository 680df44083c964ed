#!/bin/bash
# Round-trip checks: the decode/elimination parity tests, the encode_decode
# step's host phases (tools/rt_phases.py, KODR_ADD_TIMING=1) and a kernel
# trace of bench.py --no-extras (headline + round trip) with per-kernel
# medians and the idle gaps of the round trip's last steps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rtcheck}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_group_decode.py tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py tests/test_gpu_headline.py -x -q -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
KODR_ADD_TIMING=1 timeout -k 10 200 python -u tools/rt_phases.py 4 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
grep "^step" $OUT/phases.log | tail -2
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/rt -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/bench_rt.json 2> $R/$OUT/rt.err || { tail -20 $R/$OUT/rt.err; exit 1; }
cd $R
python3 - $OUT <<'PY'
import csv, glob, json, statistics, sys, collections
o = sys.argv[1]
rows = sorted(csv.DictReader(open(glob.glob(f"{o}/rt/**/*kernel_trace.csv", recursive=True)[0])), key=lambda r: int(r["Start_Timestamp"]))
g = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0][-50:]
    g[(n, r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:7]:
    print(f"{sum(v) / 1e3:8.2f} ms n={len(v):4d} median {statistics.median(v):8.1f} us {k}")
d = json.loads([l for l in open(f"{o}/bench_rt.json") if l.startswith("{")][-1])
ed = d["encode_decode"]
print("encode_decode", ed["ms_per_step"], "ms/step", ed["us_per_generation"], "us/gen; headline", d["value"], d["ms_per_step"])
PY

#!/bin/bash
# Round-4 validation on one box: the whole GPU suite, smoke, the driver's
# bench command, and the N = 2 rehearsal of the multi-rank line (two ranks on
# device 0 over gloo, KODR_BENCH_REHEARSE=1: plumbing only, not scaling).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04val}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ed = d.get("encode_decode") or {}
x = d.get("extras", {})
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"])
print("encode_decode", {k: ed.get(k) for k in ("value", "ms_per_step", "us_per_generation", "roundtrip_ok")})
print("c2_decode", {k: x.get("c2_decode", {}).get(k) for k in ("s", "add_s", "get_s", "piecewise_s")})
print("cpu", (d.get("cpu_baseline") or {}).get("value"), (ed.get("cpu_baseline") or {}).get("value"))
PY
KODR_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 2 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { tail -30 $OUT/bench_n2.err; exit 1; }
python3 - $OUT/bench_n2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ed = d.get("encode_decode") or {}
print("N=2 rehearsal value", d["value"], "encode_decode", ed.get("value"), ed.get("n_gpus"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY

# round 5: the whole GPU suite, smoke, the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
echo "pytest exit $?"; tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "bench exit $?"
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r5b/bench.json").read().strip().splitlines()[-1])
ed=d.get("encode_decode") or {}
x=d.get("extras",{})
print("value",d["value"],"ms",d["ms_per_step"],"frac",d["roofline"]["frac"])
print("rt us/gen",ed.get("us_per_generation"),"ok",ed.get("roundtrip_ok"))
for key in ("c2_decode","c2_decode_grouped","batched_decode_elimination"):
    v=x.get(key)
    if isinstance(v,dict): print(key,{a:b for a,b in v.items() if not isinstance(b,(list,dict))})
PY

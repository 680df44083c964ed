# round 5: GPU suite (compact rows), the grouped-kernel bounds, the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
echo "pytest exit $?"; tail -3 $O/pytest_gpu.log
bash tools/gpu_bs_bound.sh r5c/bsbound || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "bench exit $?"
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r5c/bench.json").read().strip().splitlines()[-1])
print("value",d["value"],"ms",d["ms_per_step"],"frac",d["roofline"]["frac"], "rt", d["roundtrip"])
print("encode", d["encode"]["value"], d["encode"]["ms_per_step"], d["encode"]["roofline"]["frac"])
legs=d["roofline"]["legs"]; print({k:(v.get("avg_us"), v.get("issue_frac")) for k,v in legs.items() if isinstance(v,dict)})
x=d.get("extras",{})
for key in ("c2_decode","c2_decode_grouped","c4_systematic_decode"):
    v=x.get(key)
    if isinstance(v,dict): print(key,{a:b for a,b in v.items() if not isinstance(b,(list,dict))})
PY

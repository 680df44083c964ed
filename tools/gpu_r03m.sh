#!/bin/bash
# Session probes: one-launch 32 MiB read floor (shapes), RCCL ring shift with
# two ranks on one GPU, the headline step alone.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03m}; mkdir -p $OUT
timeout -k 10 120 ./tools/probe/read_floor > $OUT/read_floor.log 2>&1 || { cat $OUT/read_floor.log; exit 1; }
cat $OUT/read_floor.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_read -o run --output-format csv -- ./tools/probe/read_floor > $OUT/prof_read.log 2>&1 || { tail -20 $OUT/prof_read.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, statistics, sys, collections
o = sys.argv[1]
f = glob.glob(f"{o}/prof_read/**/*kernel_trace.csv", recursive=True)
d = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    d[(r["Kernel_Name"][:40], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for key, v in d.items():
    print("rocprof", key, f"n={len(v)} median {statistics.median(v) / 1e3:.2f} us")
PY
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/probe/rccl_same_gpu.py > $OUT/rccl.log 2>&1; echo "rccl rc=$?"; tail -5 $OUT/rccl.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-encode-decode > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench_headline.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"

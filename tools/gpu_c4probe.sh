#!/bin/bash
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/c4probe; mkdir -p $OUT
timeout -k 10 120 python3 $R/tools/c4_probe.py > $OUT/plain.json 2>&1 || { cat $OUT/plain.json; exit 1; }
cat $OUT/plain.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $OUT/prof -o run --output-format csv -- python3 $R/tools/c4_probe.py > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
grep add_get $OUT/prof.log

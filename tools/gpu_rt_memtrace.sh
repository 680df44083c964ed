#!/bin/bash
# kernel + memory-copy trace of the round trip (bench.py --no-extras): what
# sits between one step's GetPieces and the next step's encode
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rtmem}; mkdir -p $OUT
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$OUT/tr -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/b.json 2> $R/$OUT/b.err || { tail -20 $R/$OUT/b.err; exit 1; }
ls $R/$OUT/tr

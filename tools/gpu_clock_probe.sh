#!/bin/bash
# clocks and power under back-to-back grouped launches (tools/clock_probe.py):
# the product build at B = 32 and 256, the no-row-stream bound (tuning build
# MODE 31) at B = 32
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-clockprobe}; mkdir -p $OUT
timeout -k 10 120 python -u tools/clock_probe.py $OUT/prod.jsonl 32 256 > $OUT/prod.log 2>&1; echo "prod rc $?"; cat $OUT/prod.log | cut -c1-1600
KODR_BS_MODE=31 KODR_RLNC_LIB=kodr_amd/tune_m/libkodr_rlnc.so timeout -k 10 120 python -u tools/clock_probe.py $OUT/m31.jsonl 32 > $OUT/m31.log 2>&1; echo "m31 rc $?"; grep -v "first sample" $OUT/m31.log

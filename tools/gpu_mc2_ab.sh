#!/bin/bash
# gf_elim_mc2_kernel A/B: parity (elimination, lazy and grouped decode, the
# bench's round-trip step) under the default build, then one and 16
# decoders' batched AddPiece (tools/elim_time.py, k = 128 and 256) for
# KODR_ELIM_MC 0 / 1 / 2 and the mc2 variants (KODR_MC2_VARIANT bits:
# 1 split small products, 2 readlane pivot broadcast), two interleaved reps,
# then rocprof kernel durations of two of them and the phases of one call.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mc2ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py tests/test_gpu_group_decode.py tests/test_gpu_headline.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
CONFIGS=${CONFIGS:-"0:0 1:0 2:0 2:1 2:2 2:3"}
for rep in 1 2; do
  for C in $CONFIGS; do
    M=${C%%:*}; V=${C##*:}
    KODR_ELIM_MC=$M KODR_MC2_VARIANT=$V timeout -k 10 120 python -u tools/elim_time.py 128,256 1,16 > $OUT/e_${M}_${V}_r$rep.log 2>&1 || { tail -20 $OUT/e_${M}_${V}_r$rep.log; exit 1; }
    echo "mc=$M var=$V rep $rep: $(python3 -c "import json,sys; print(' '.join(f\"k{d['k']}G{d['G']} {d['gpu_us']}/{d['host_us']}\" for d in map(json.loads, open(sys.argv[1]))))" $OUT/e_${M}_${V}_r$rep.log)"
  done
done
KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/elim_time.py 256 1 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
tail -3 $OUT/phases.log
for V in ${PROF_VARIANTS:-0 3}; do
  KODR_MC2_VARIANT=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_v$V -o run --output-format csv -- python3 tools/elim_time.py 256 1,16 > $OUT/prof_v$V.log 2>&1 || { tail -20 $OUT/prof_v$V.log; exit 1; }
done
python3 - $OUT "${PROF_VARIANTS:-0 3}" <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for V in sys.argv[2].split():
    f = glob.glob(f"{o}/prof_v{V}/**/*kernel_trace.csv", recursive=True)
    d = {}
    for r in csv.DictReader(open(f[0])):
        if "elim" in r["Kernel_Name"]:
            d.setdefault((r["Kernel_Name"].split("(")[0][-30:], r["Grid_Size_Y"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in d.items():
        print(f"var={V} {n}: n={len(v)} min {min(v):.1f} median {statistics.median(v):.1f} max {max(v):.1f} us")
PY

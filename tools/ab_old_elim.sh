#!/bin/bash
# Batched elimination (k = 256, G = 1 / 4 / 16, L = 256) with earlier builds
# of the library (ab_old/<name>/libkodr_rlnc.so, built from older commits,
# not tracked) against the tree's, two interleaved reps (tools/elim_time.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abold}; mkdir -p $OUT
for rep in 1 2; do
  for lib in ab_old/*/libkodr_rlnc.so kodr_amd/libkodr_rlnc.so; do
    n=$(basename $(dirname $lib))
    KODR_RLNC_LIB=$PWD/$lib timeout -k 10 100 python -u tools/elim_time.py 256 1,4,16 256 > $OUT/${n}_$rep.log 2>&1 || { tail -5 $OUT/${n}_$rep.log; exit 1; }
  done
done
for f in $OUT/*.log; do echo "$f $(python3 -c "import json,sys; print(' '.join(f\"G{d['G']} {d['gpu_us']}/{d['host_us']}\" for d in map(json.loads, open(sys.argv[1]))))" $f)"; done

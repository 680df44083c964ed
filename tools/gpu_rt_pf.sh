#!/bin/bash
# the round trip with the vector download beside every launch (this tree)
# and only after a failure (KODR_VEC_PREFETCH=0, tuning build), and r5lib_pre
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  echo "new: $(timeout -k 10 200 python -u tools/rt_variants.py 20 1 2>&1 | grep async)"
  echo "nopf: $(KODR_VEC_PREFETCH=0 KODR_RLNC_LIB=kodr_amd/tune_c/libkodr_rlnc.so timeout -k 10 200 python -u tools/rt_variants.py 20 1 2>&1 | grep async)"
  echo "pre: $(KODR_RLNC_LIB=kodr_amd/r5lib_pre/libkodr_rlnc.so timeout -k 10 200 python -u tools/rt_variants.py 20 1 2>&1 | grep async)"
done

#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in new pre; do
  libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
  echo "== $v"; KODR_RLNC_LIB=$libp timeout -k 10 200 python -u tools/rt_variants.py 20 3 2>&1 | tail -6
done

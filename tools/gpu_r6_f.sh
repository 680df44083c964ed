#!/bin/bash
# Round 6: the elimination's 16 x 16 inversion with the guessed pivot
# (mc3_gj) against the previous library (kodr_amd/ab_v5, ballot on every
# step): the chain probe, C2's AddPiece per repetition (tools/c2_add_phases.py)
# and the mc4 / mc2 kernels under rocprof (tools/elim_time.py, 1 and 16
# decoders of k = 256), interleaved; then the elimination and round-trip
# GPU tests on the new library.  Stops at anything but a test failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc $rc at $2"; exit $rc; }; }
timeout -k 10 120 ./tools/probe/chain_probe 512 > $O/chain.log 2>&1; ok $? probe
cat $O/chain.log
for rep in 1 2; do
  for v in new old; do
    lib=kodr_amd/libkodr_rlnc.so; [ $v = old ] && lib=kodr_amd/ab_v5/libkodr_rlnc.so
    KODR_RLNC_LIB=$lib timeout -k 10 120 python3 tools/c2_add_phases.py 24 7 > $O/c2_${v}_$rep.log 2>&1; ok $? c2_$v
    KODR_RLNC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/elim_${v}_$rep -o run \
      --output-format csv -- python3 tools/elim_time.py 256 1,16 131072 > $O/elim_${v}_$rep.log 2>&1; ok $? elim_$v
  done
done
for f in $O/c2_*.log; do
  python3 - "$f" <<'PY'
import re, statistics, sys
v = [float(m.group(1)) for m in re.finditer(r"add\s+([0-9.]+) us", open(sys.argv[1]).read())][2:]
print(sys.argv[1].split("/")[-1], "add us: best %.1f median %.1f (%d reps)" % (min(v), statistics.median(v), len(v)))
PY
done
grep -h "gf_elim_mc" $O/elim_*/run_kernel_stats.csv | cut -d, -f1-8 | cut -c1-200
for f in $O/elim_*.log; do echo "$f: $(grep -h '^{' $f | cut -c1-300)"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_elim.py \
  tests/test_gpu_elim_route.py tests/test_gpu_lazy_decode.py tests/test_gpu_headline.py > $O/pytest.log 2>&1
ok $? pytest
tail -3 $O/pytest.log

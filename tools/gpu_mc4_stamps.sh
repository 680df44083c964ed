# round 5: mc4 timelines (KODR_ELIM_TIMING builds) of round 4's kernel and this tree's
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5stamps
mkdir -p $O
for rep in 1 2; do
for v in r4lib_t r5lib_t; do
  KODR_ELIM_DUMP=$O/$v.dump timeout -k 10 60 python3 tools/elim_ab.py kodr_amd/$v/libkodr_rlnc.so 256 1 256 5 > $O/$v.log 2>&1 || { echo fail $v; cat $O/$v.log; exit 1; }
  echo "== $v rep $rep"; python3 tools/elim_mc4_stamps.py $O/$v.dump 256
done
done

# round 5: KODR_ADD_TIMING phases of the 16-decoder batched AddPiece, r4 vs this tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5phases
mkdir -p $O
for v in r4lib new; do
  libp=kodr_amd/libkodr_rlnc.so; [ $v = r4lib ] && libp=kodr_amd/r4lib/libkodr_rlnc.so
  KODR_ADD_TIMING=1 timeout -k 10 120 python3 tools/elim_ab.py $libp 256 16 256 12 4 > $O/$v.log 2>&1 || { echo "fail $v"; exit 1; }
  echo "== $v"; tail -8 $O/$v.log
done

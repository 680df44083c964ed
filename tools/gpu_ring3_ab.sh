# round 5: three rows in flight for the direct grouped launch (MODE 33, map
# moved down: KODR_BS_ACC=4 build kodr_amd/tune_m4/) against two (MODE 0 of the
# same build and of the product build) and the no-row-stream bound (MODE 31),
# interleaved, tools/group_bs_time.py B = 32 and 256 over 16 generations
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ring3}; mkdir -p $OUT
for rep in 1 2; do
  for v in prod:0 m4:0 m4:33 m4:31; do
    lib=${v%%:*}; M=${v##*:}
    libp=kodr_amd/libkodr_rlnc.so; [ $lib = m4 ] && libp=kodr_amd/tune_m4/libkodr_rlnc.so
    KODR_BS_MODE=$M KODR_RLNC_LIB=$libp timeout -k 10 120 python -u tools/group_bs_time.py 32 256 \
      > $OUT/t_${lib}_m${M}_r$rep.log 2>&1 || { tail -20 $OUT/t_${lib}_m${M}_r$rep.log; exit 1; }
    echo "$lib mode $M rep $rep: $(grep -E "^(32|256) " $OUT/t_${lib}_m${M}_r$rep.log | sed 's/"single[^,]*, //; s/, "speedup[^}]*//' | tr "\n" " ")"
  done
done

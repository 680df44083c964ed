# round 5: what a load path could save in the grouped direct bit-sliced launch:
# tuning build (kodr_amd/tune_m/, -DKODR_TUNE_MODES) MODE 0 (product loop),
# 31 (no row stream), 30 (bodies inlined, no jumps), 32 (neither), interleaved,
# tools/group_bs_time.py over 16 prepared 32 MiB/256 generations
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-bsbound}; mkdir -p $OUT
for rep in 1 2; do
  for M in 0 31 30 32; do
    KODR_BS_MODE=$M KODR_RLNC_LIB=kodr_amd/tune_m/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 32 258 \
      > $OUT/t_m${M}_r$rep.log 2>&1 || { tail -20 $OUT/t_m${M}_r$rep.log; exit 1; }
    echo "mode $M rep $rep: $(grep -E "^(32|258) " $OUT/t_m${M}_r$rep.log | tr "\n" " ")"
  done
done

mkdir -p gpurun_out/gbs
for KW in 0 2 3 4 6 8 16; do
  if [ $KW = 0 ]; then env -u KODR_BS_KW KODR_RLNC_LIB=kodr_amd/tune_g/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 16 32 64 > gpurun_out/gbs/kw$KW.log 2>&1 || exit 1
  else KODR_BS_KW=$KW KODR_RLNC_LIB=kodr_amd/tune_g/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 16 32 64 > gpurun_out/gbs/kw$KW.log 2>&1 || exit 1; fi
  echo "KW $KW"; head -3 gpurun_out/gbs/kw$KW.log
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/gbs/bench.json 2> gpurun_out/gbs/bench.err || { tail gpurun_out/gbs/bench.err; exit 1; }
cut -c1-1500 gpurun_out/gbs/bench.json

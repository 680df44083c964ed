set -uo pipefail
T=$PWD/kodr_amd/tune/libkodr_rlnc.so
for m in 0 20 6 3; do bash tools/pmc_sq.sh 32 $T $m > gpurun_out/pmc_m$m.txt 2>&1 || { cat gpurun_out/pmc_m$m.txt; exit 1; }; done
for m in 0 20 6 3; do echo "== mode $m"; cat gpurun_out/pmc_m$m.txt; done

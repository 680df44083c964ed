set -uo pipefail
R=$PWD
bash tools/pmc_group.sh 16 1 || exit 1
mkdir -p gpurun_out/biggen
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/biggen/prof -o run --output-format csv -- python3 $R/tools/big_gen.py --shapes 64x128,64x128,64x128 > $R/gpurun_out/biggen/out.log 2>&1 || { tail -20 $R/gpurun_out/biggen/out.log; exit 1; }
cat $R/gpurun_out/biggen/out.log

# round 5: mc2 (16 decoders, seed 4: no decoder needs a second attempt), r4 vs this tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g16
mkdir -p $O
for v in r4lib new r4lib new; do
  libp=kodr_amd/libkodr_rlnc.so; [ $v = r4lib ] && libp=kodr_amd/r4lib/libkodr_rlnc.so
  rm -rf $O/$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 tools/elim_ab.py $libp 256 16 256 30 4 > $O/$v.log 2>&1 || { echo "fail $v"; exit 1; }
  grep "call median" $O/$v.log
  python3 -c "
import csv,glob
for f in glob.glob('$O/$v/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'elim' in r['Name']: print('$v', r['Calls'], 'avg_us', round(float(r['AverageNs'])/1e3,1))
"
done

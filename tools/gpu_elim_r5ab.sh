# round 5: the elimination kernels with attempts (this tree) against round 4's
# build (kodr_amd/r4lib), interleaved, kernel durations from rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ab
mkdir -p $O
for rep in 1; do
  for v in r4lib new; do
    libp=kodr_amd/libkodr_rlnc.so; [ $v = r4lib ] && libp=kodr_amd/r4lib/libkodr_rlnc.so
    for cfg in "256 1 256" "256 16 256" "256 1 131072"; do
      set -- $cfg
      tag=${v}_k$1_G$2_L$3_r$rep
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 tools/elim_ab.py $libp $1 $2 $3 30 > $O/$tag.log 2>&1 || { echo "fail $tag"; exit 1; }
      tail -1 $O/$tag.log
    done
  done
done
python3 - <<'PY'
import glob, csv, os
for f in sorted(glob.glob("gpurun_out/r5ab/*/**/run_kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "elim" in r["Name"] or "copy_bitslice" in r["Name"]:
            print(f.split("/")[2], r["Name"][:40], r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1),
                  "min_us", round(float(r["MinNs"]) / 1e3, 1))
PY

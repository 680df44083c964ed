set -uo pipefail
for G in 4 8 16 32; do
  G=$G COUNTS=1 AUXS=2 CFGS="1,16,2,8;1,4,1,8;1,8,1,8;1,1,1,16" timeout -k 10 200 python tools/group_sweep.py || exit 1
  G=$G COUNTS=2 AUXS=2 CFGS="2,16,2,8;2,4,1,8" timeout -k 10 200 python tools/group_sweep.py || exit 1
  G=$G COUNTS=4 AUXS=2 CFGS="4,8,2,4;4,4,1,8" timeout -k 10 200 python tools/group_sweep.py || exit 1
  G=$G COUNTS=8 AUXS=2 CFGS="8,16,2,2;8,4,1,8" timeout -k 10 200 python tools/group_sweep.py || exit 1
done

#!/bin/bash
# Host elimination of a k + 4 row coded batch (tools/core_time.py) on the box's
# CPU: kodr's route (KODR_FULL_SOLVE=0) vs the blocked full-batch solve.
for K in 96 128 192 256; do
  KODR_FULL_SOLVE=0 K=$K timeout -k 5 120 python tools/core_time.py | sed 's/^/route   /'
  K=$K timeout -k 5 120 python tools/core_time.py | sed "s/^/blocked /"
done
gcc -O2 -mavx512f -mavx512bw -mgfni -mavx512vl tools/probe/gfni_tput.c -o /tmp/gfni_tput && /tmp/gfni_tput
grep -m1 "model name" /proc/cpuinfo

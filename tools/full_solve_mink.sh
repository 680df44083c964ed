#!/bin/bash
# kodr's route vs the blocked solve below the default threshold (KODR_FULL_MIN_K)
for K in 64 96 128 160 192 224; do
  KODR_FULL_SOLVE=0 K=$K timeout -k 5 60 python tools/core_time.py | sed 's/^/route   /'
  KODR_FULL_MIN_K=2 K=$K timeout -k 5 60 python tools/core_time.py | sed "s/^/blocked /"
done

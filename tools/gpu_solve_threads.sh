#!/bin/bash
# Host-side: the threaded full-batch solve on the GPU box's CPU (no GPU work).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-solve_threads}; mkdir -p $OUT
lscpu | grep -E 'Model name|^CPU\(s\)|Thread|Core|Socket|NUMA node\(s\)' > $OUT/cpu.txt; cat $OUT/cpu.txt
for t in 1 2 3 4 6 8; do
  for g in 0 1000; do
    echo "threads $t $(KODR_SOLVE_THREADS=$t KODR_FULL_SOLVE=2 timeout -k 5 60 ./tools/probe/solve_threads $g 2>&1 | tail -2 | tr '\n' ' ')"
  done
done | tee $OUT/solve_threads.log

#!/bin/bash
# The N = 2 rehearsal's relay recode, split (tools/relay_n2_probe.py): two
# ranks on the one GPU, gloo.  Output: gpurun_out/relay_n2/.
set -o pipefail
mkdir -p gpurun_out/relay_n2
export KODR_BENCH_REHEARSE=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 tools/relay_n2_probe.py > gpurun_out/relay_n2/probe.log 2>&1
rc=$?
grep '^{' gpurun_out/relay_n2/probe.log > gpurun_out/relay_n2/probe.json
tail -3 gpurun_out/relay_n2/probe.log | cut -c1-1500
exit $rc

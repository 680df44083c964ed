mkdir -p gpurun_out/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
for rep in 1 2; do for g in 16 32; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --gens $g --no-extras --no-cpu-baseline --no-encode-decode > gpurun_out/final/g${g}_r$rep.json 2> gpurun_out/final/g${g}_r$rep.err || { tail -5 gpurun_out/final/g${g}_r$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/final/g${g}_r$rep.json').read().strip().splitlines()[-1]); print('G=$g rep $rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done; done

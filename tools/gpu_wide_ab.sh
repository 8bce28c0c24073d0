set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/wide
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or configs4" > gpurun_out/wide/tests.log 2>&1; echo "tests: $(tail -1 gpurun_out/wide/tests.log)"
for v in 1 0; do
  MV_MLPW32=$v timeout -k 10 300 python -u bench.py --workload synthetic.botnet.wide --n-gen 100 --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-generate > gpurun_out/wide/w$v.json 2> gpurun_out/wide/w$v.log
  python3 -c "import json;d=json.load(open('gpurun_out/wide/w$v.json'));print('MV_MLPW32=$v', round(d['value']/1e6,2), 'M evals/s', {k: round(v*1000,2) for k,v in d['kernels_avg_ms_per_generation'].items() if k!='dominant'}, d['kernels']['k_mlp']['kernel'], round(d['kernels']['k_mlp']['frac'],3))"
done

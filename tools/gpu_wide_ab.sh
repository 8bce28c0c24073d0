#!/bin/bash
# configs[4] (synthetic.botnet.wide) classifier A/B: the wide-net parity tests on the product
# build, then one 100-generation attack per library in LIBS (names as tools/gpu_libs.sh) and
# per classifier precision in DTYPES.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide; mkdir -p $O
L=moeva2-ijcai22-replication_amd/lib
path() { [ -z "$1" -o "$1" = main ] && echo $L/libmoeva_mi355x.so || echo $L/libmoeva_mi355x_$1.so; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-wide or configs4 or bf16}" > $O/tests.log 2>&1; echo "tests: $(tail -1 $O/tests.log)"
for d in ${DTYPES:-fp32 bf16}; do
  for n in ${LIBS:-main}; do
    MOEVA_MI355X_LIB=$(path $n) timeout -k 10 300 python -u bench.py --workload synthetic.botnet.wide --mlp-dtype $d --n-gen 100 --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-generate > $O/$d.$n.json 2> $O/$d.$n.log
    python3 -c "import json;d=json.load(open('$O/$d.$n.json'));print('$d [$n]', round(d['value']/1e6,2), 'M evals/s', {k: round(v*1000,2) for k,v in d['kernels_avg_ms_per_generation'].items() if not isinstance(v, str)}, d['kernels']['k_mlp']['kernel'], round(d['kernels']['k_mlp']['frac'],3))"
  done
done

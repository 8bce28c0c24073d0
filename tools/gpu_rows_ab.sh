#!/bin/bash
# k_genc rows-per-workgroup A/B: per setting of MV_VARY_ROWS, the bench's single-group event
# times (k_genc ms per generation) and the PMC FETCH_SIZE / WRITE_SIZE of k_genc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rows; mkdir -p $O
for r in ${ROWS:-32 10 12 16}; do
  MV_VARY_ROWS=$r timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 --groups 1 > $O/b$r.json 2> $O/b$r.log || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    MV_VARY_ROWS=$r timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc$r$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-gen 20 --groups 1 > $O/pmc$r$c.log 2>&1 || exit 1
  done
  python3 tools/pmc_traffic.py $O/traffic$r.json $(find $O/pmc${r}FETCH_SIZE $O/pmc${r}WRITE_SIZE -name '*counter_collection.csv') > /dev/null 2>&1
  echo "rows $r: $(python3 -c "import json;d=json.load(open('$O/b$r.json'));print(round(d['value']/1e6,1),'M evals/s', d['kernels_avg_ms_per_generation'])") traffic k_genc $(python3 -c "import json;d=json.load(open('$O/traffic$r.json'));print(round(d['k_genc']['traffic_bytes']/1e6,1),'MB fetch',round(2*d['k_genc']['fetch_kib']/1024,1),'write',round(d['k_genc']['write_kib']/1024,1))")"
done

cd $GRAFT_REPO_ROOT
for m in 0 1 2 4 8 16 31; do
  MV_DBG_VARY=$m timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 100 > gpurun_out/dbg_$m.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/dbg_$m.json')); print($m, d['kernels_avg_ms_per_generation'])"
done

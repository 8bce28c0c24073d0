cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for g in 1 2 3 4; do
  MV_GROUPS=$g timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --n-gen 200 > gpurun_out/b$g.json 2>/dev/null || exit 1
  echo "groups=$g"; python3 tools/show_bench.py gpurun_out/b$g.json | head -1
done

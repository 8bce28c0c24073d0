cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
python -c "import torch;p=torch.cuda.get_device_properties(0);print(p.name,p.multi_processor_count,getattr(p,'gcnArchName',''))"
for pz in none 255 127 0; do
  if [ $pz = none ]; then unset MV_POISON; else export MV_POISON=$pz; fi
  DET_OUT=gpurun_out/det_$pz.npy timeout -k 10 200 python -u tools/determinism.py --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
unset MV_POISON
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -v -s --timeout 180 --timeout-method thread 2>&1 | grep -E "o1..o7|passed|failed"

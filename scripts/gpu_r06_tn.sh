# round 6: mixed whole-tile + split-K TN launch -- GPU tests, per-shape times under held CUs, step A/B
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tn}; O=gpurun_out/r06/$T; mkdir -p $O
run_step r06/$T/pytest 600 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py tests/gpu/test_comm_emu_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 2 $O/pytest.log; grep -q " passed" $O/pytest.log || exit 3
WHAT=tn,flash run_step r06/$T/micro 400 python scripts/comm_gemm_micro.py
grep '^{' $O/micro.log | cut -c1-150
B="python bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARM:-3} --daemon-bench 0"
run_step r06/$T/base 300 $B; grep -o '"value": [0-9.]*' $O/base.log
for k in ${KS:-8 16}; do
  TH_COMM_EMU="cus=$k" TH_COMM_CUS=0 run_step r06/$T/k${k}_nofix 300 $B; grep -o '"value": [0-9.]*' $O/k${k}_nofix.log
  TH_COMM_EMU="cus=$k" run_step r06/$T/k${k}_fix 300 $B; grep -o '"value": [0-9.]*' $O/k${k}_fix.log
done

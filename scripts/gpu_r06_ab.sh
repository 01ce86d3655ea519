# round 6: same-box A/B of the step against the round-5 tree (_ab/r5, a git worktree of 152779d with its own
# libthk.so), TN per-shape times under held CUs, and the emulated-comm step without / with the fix
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-ab}; O=gpurun_out/r06/$T; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  run_step r06/$T/pytest 900 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py tests/gpu/test_comm_emu_gpu.py tests/gpu/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread
  tail -n 2 $O/pytest.log; grep -q " passed" $O/pytest.log || exit 3
fi
WHAT=${WHAT:-tn} run_step r06/$T/micro 400 python scripts/comm_gemm_micro.py
grep '^{' $O/micro.log | cut -c1-150
B="bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARM:-3} --daemon-bench 0"
for i in 1 2; do
  run_step r06/$T/new_$i 300 python $B; grep -o '"value": [0-9.]*' $O/new_$i.log
  (cd _ab/r5 && timeout -k 10 300 python $B > $R/$O/r5_$i.log 2>&1); echo "[step] r5_$i rc=$?"; grep -o '"value": [0-9.]*' $O/r5_$i.log
done
for k in ${KS:-16}; do
  TH_COMM_EMU="cus=$k" TH_COMM_CUS=0 run_step r06/$T/k${k}_nofix 300 python $B; grep -o '"value": [0-9.]*' $O/k${k}_nofix.log
  TH_COMM_EMU="cus=$k" run_step r06/$T/k${k}_fix 300 python $B; grep -o '"value": [0-9.]*' $O/k${k}_fix.log
done

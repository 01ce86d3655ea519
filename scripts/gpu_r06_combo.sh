# round 6: comm-emulator GPU tests, the forced-RCCL ZeRO-1 torchrun path, and the modelled 8-rank ZeRO-1 schedule
# (bucket mode now with the parameter all-gathers beside the next forward)
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-combo}; O=gpurun_out/r06/$T; mkdir -p $O
run_step r06/$T/pytest 300 python -u -m pytest tests/gpu/test_comm_emu_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 2 $O/pytest.log; grep -q " passed" $O/pytest.log || exit 3
bash scripts/gpu_r06_rccl.sh || exit 1
TAG=sweep5 SPECS="${SPECS:-cus=16,mode=bucket cus=32,mode=bucket}" bash scripts/gpu_r06_sweep.sh

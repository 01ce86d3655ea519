# round 5: attribution changes on the GPU box (forged task id, protection, HBM counters, remote
# telemetry, multi-tenant node) + the flash tests after the TH_KF_DIAG split
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-attr}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/pytest 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/gpu/test_forged_task_gpu.py tests/gpu/test_protection_gpu.py tests/gpu/test_hbm_counter_gpu.py \
  tests/gpu/test_remote_telemetry_gpu.py tests/gpu/test_multitenant_node_gpu.py tests/gpu/test_native_gpu.py \
  tests/gpu/test_flash_attn_gpu.py
tail -n 30 gpurun_out/r05/$T/pytest.log

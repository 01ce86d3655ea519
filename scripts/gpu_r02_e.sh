# RCCL one-rank collective path + LM-head chunk A/B (interleaved)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02e_ddp 400 python -u -m pytest tests/gpu/test_ddp_gpu.py -v -s --timeout 300 --timeout-method thread
for rep in 1 2; do
  for c in 4096 8192 16384; do
    TH_CE_CHUNK=$c run_step r02e_ce${c}_$rep 300 python bench.py --daemon-bench 0 --steps 5 --warmup 2
    tail -n 1 gpurun_out/r02e_ce${c}_$rep.log
  done
done

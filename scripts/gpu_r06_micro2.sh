# round 6: per-kernel times with emulated channel CUs held (scripts/comm_gemm_micro.py), fixed syncs
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-micro2}; O=gpurun_out/r06/$T; mkdir -p $O
WHAT=${WHAT:-tn,blas,flash} run_step r06/$T/micro 400 python scripts/comm_gemm_micro.py
grep '^{' $O/micro.log | cut -c1-150

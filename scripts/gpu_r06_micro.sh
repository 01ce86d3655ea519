# round 6: per-kernel cost of CUs held by an idle emulated channel kernel (scripts/comm_gemm_micro.py)
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-micro}; O=gpurun_out/r06/$T; mkdir -p $O
run_step r06/$T/micro 400 python scripts/comm_gemm_micro.py
cat $O/micro.log | grep '^{' | cut -c1-160
TAG=sk TENSILE_STREAMK_MAX_CUS=${SKCUS:-248} KS=${SKKS:-0,8} WHAT=blas run_step r06/$T/micro_sk 300 python scripts/comm_gemm_micro.py
grep '^{' $O/micro_sk.log

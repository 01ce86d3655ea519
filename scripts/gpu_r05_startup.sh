# round 5: what a queued job's 5.2 s startup is made of -- import torch, HIP init, first kernel -- with and
# without the in-task HBM counter tool (ROCP_TOOL_LIBRARIES=libthhbm) that th-run injects into every task
R=$GRAFT_REPO_ROOT; cd $R; T=${TAG:-startup}; mkdir -p gpurun_out/r05/$T
TOOL=$R/tensorhive_fixed_amd/native/lib/libthhbm.so
J='import time; t0=time.time(); import torch; t1=time.time(); x=torch.randn(8192,8192,device="cuda",dtype=torch.bfloat16); torch.cuda.synchronize(); t2=time.time(); print("import_s %.3f cuda_init_s %.3f" % (t1-t0, t2-t1), flush=True)'
for i in 1 2 3; do
  for mode in plain tool; do
    s=$(date +%s.%N)
    if [ $mode = tool ]; then ROCP_TOOL_LIBRARIES=$TOOL timeout -k 10 120 python -c "$J" > gpurun_out/r05/$T/$mode$i.log 2>&1 || exit 1
    else timeout -k 10 120 python -c "$J" > gpurun_out/r05/$T/$mode$i.log 2>&1 || exit 1; fi
    e=$(date +%s.%N)
    echo "$mode run $i wall $(python3 -c "print(round($e-$s,3))") $(grep import_s gpurun_out/r05/$T/$mode$i.log)"
  done
done | tee gpurun_out/r05/$T/summary.txt

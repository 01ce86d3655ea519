# round 5: does GPU visibility shrink rocprofiler-sdk's agent discovery (the in-task tool's startup cost)?
R=$GRAFT_REPO_ROOT; cd $R; T=${TAG:-startup5}; mkdir -p gpurun_out/r05/$T
{ echo "kfd topology nodes: $(ls /sys/class/kfd/kfd/topology/nodes | wc -l)"; env | grep -E "VISIBLE|ROCR|HIP_" | sort; } > gpurun_out/r05/$T/env.txt
cat gpurun_out/r05/$T/env.txt
J='import time; t0=time.time(); import torch; t1=time.time(); x=torch.randn(8192,8192,device="cuda",dtype=torch.bfloat16); torch.cuda.synchronize(); t2=time.time(); print("import_s %.3f cuda_init_s %.3f" % (t1-t0, t2-t1), flush=True)'
for i in 1 2; do
  for mode in plain p4 p4rocr0 lazyrocr0; do
    L=""; EXTRA=""
    case $mode in p4) L=$R/scripts/libprobetool4.so;; p4rocr0) L=$R/scripts/libprobetool4.so; EXTRA="ROCR_VISIBLE_DEVICES=0";;
      lazyrocr0) L=$R/tensorhive_fixed_amd/native/lib/libthhbm.so; EXTRA="ROCR_VISIBLE_DEVICES=0";; esac
    s=$(date +%s.%N)
    env $EXTRA ROCP_TOOL_LIBRARIES=$L timeout -k 10 120 python -c "$J" > gpurun_out/r05/$T/$mode$i.log 2>&1 || exit 1
    e=$(date +%s.%N)
    echo "$mode run $i wall $(python3 -c "print(round($e-$s,3))") $(grep import_s gpurun_out/r05/$T/$mode$i.log)"
  done
done | tee gpurun_out/r05/$T/summary.txt

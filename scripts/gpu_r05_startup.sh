# round 5: what a queued job's 5.2 s startup is made of -- import torch, HIP init, first kernel -- bare, with a
# do-nothing rocprofiler-sdk tool, with the in-task HBM counter tool as round 4 built it (counter enumeration
# inside tool_init) and as now (enumeration on the tool's own thread); then the HBM counter GPU tests
R=$GRAFT_REPO_ROOT; cd $R; T=${TAG:-startup}; mkdir -p gpurun_out/r05/$T
J='import time; t0=time.time(); import torch; t1=time.time(); x=torch.randn(8192,8192,device="cuda",dtype=torch.bfloat16); torch.cuda.synchronize(); t2=time.time(); print("import_s %.3f cuda_init_s %.3f" % (t1-t0, t2-t1), flush=True)'
for i in 1 2 3; do
  for mode in ${MODES:-plain null eager lazy}; do
    unset ROCPROFILER_METRICS_PATH
    case $mode in
      plain) L="";; null) L=$R/scripts/libnulltool.so;; eager) L=$R/scripts/libthhbm_eager.so;;
      lazy) L=$R/tensorhive_fixed_amd/native/lib/libthhbm.so;;  p1|p2|p3|p4|p5) L=$R/scripts/libprobetool${mode#p}.so;;
    esac
    s=$(date +%s.%N)
    ROCP_TOOL_LIBRARIES=$L timeout -k 10 120 python -c "$J" > gpurun_out/r05/$T/$mode$i.log 2>&1 || exit 1
    e=$(date +%s.%N)
    echo "$mode run $i wall $(python3 -c "print(round($e-$s,3))") $(grep import_s gpurun_out/r05/$T/$mode$i.log)"
  done
done | tee gpurun_out/r05/$T/summary.txt
[ -n "$NO_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/gpu/test_hbm_counter_gpu.py tests/gpu/test_remote_telemetry_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/$T/hbm_tests.log 2>&1; echo "hbm tests rc=$?"; tail -n 3 gpurun_out/r05/$T/hbm_tests.log

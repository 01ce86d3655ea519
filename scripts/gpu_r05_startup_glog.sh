# round 5: rocprofiler-sdk's own log around tool discovery (find_clients) for the probe tools
R=$GRAFT_REPO_ROOT; cd $R; T=${TAG:-startup9}; mkdir -p gpurun_out/r05/$T
for mode in ${MODES:-null p1 p4}; do
  case $mode in null) L=$R/scripts/libnulltool.so;; *) L=$R/scripts/libprobetool${mode#p}.so;; esac
  GLOG_v=3 GLOG_minloglevel=0 ROCPROFILER_LOG_LEVEL=info GLOG_logtostderr=1 ROCP_TOOL_LIBRARIES=$L timeout -k 10 120 python -c "import time; t0=time.time(); import torch; print('import_s %.3f' % (time.time()-t0), flush=True)" > gpurun_out/r05/$T/$mode.log 2>&1 || exit 1
  echo "$mode: $(grep import_s gpurun_out/r05/$T/$mode.log) $(grep -c 'searching' gpurun_out/r05/$T/$mode.log) searches; $(grep -m1 -o 'I[0-9]* [0-9:.]* [0-9]* registration.cpp:518' gpurun_out/r05/$T/$mode.log) -> $(grep -m1 -o 'I[0-9]* [0-9:.]* [0-9]* registration.cpp:475.*' gpurun_out/r05/$T/$mode.log)"
done | tee gpurun_out/r05/$T/summary.txt

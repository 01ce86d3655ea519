# round 3, verdict item 3: HBM bytes from counters.  The in-task rocprofiler tool (libthhbm)
# samples device counting INSIDE the load's process; compared against (a) the bytes the copy /
# add streams move by construction and (b) rocprofv3 dispatch-mode PMC of the same counters
# for the GEMM+SwiGLU mix (bytes per iteration).
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
O=gpurun_out/r03/hbm; mkdir -p $O
TOOL=$PWD/tensorhive_fixed_amd/native/lib/libthhbm.so
for k in add copy; do
  run_step r03/hbm/tool_$k 120 env ROCP_TOOL_LIBRARIES=$TOOL TH_HBM_OUT=$O/tool_$k.jsonl TH_HBM_APPEND=1 \
    TH_HBM_PERIOD_MS=500 python3 scripts/hbm_stream.py 4 $k
done
run_step r03/hbm/tool_mix 120 env ROCP_TOOL_LIBRARIES=$TOOL TH_HBM_OUT=$O/tool_mix.jsonl TH_HBM_APPEND=1 \
  TH_HBM_PERIOD_MS=500 python3 scripts/hbm_mix.py 4
run_step r03/hbm/plain_mix 120 python3 scripts/hbm_mix.py 4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run_step r03/hbm/pmc_mix 180 timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum \
  TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc_mix -o run --output-format csv -- python3 scripts/hbm_mix.py 2
run_step r03/hbm/pmc_add 180 timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum \
  TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc_add -o run --output-format csv -- python3 scripts/hbm_stream.py 1 add
for f in $O/*.jsonl; do echo "== $f"; head -c 1500 $f; done
cat gpurun_out/r03/hbm/*.log | grep '^{' ; find $O -name '*counter_collection*'

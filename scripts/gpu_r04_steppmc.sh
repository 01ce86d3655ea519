# round 4: MFMA busy per kernel inside the training step (dispatch PMC over bench.py --steps 2)
R=$GRAFT_REPO_ROOT; cd $R; T=${PMC_TAG:-steppmc}; mkdir -p gpurun_out/r04/$T
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/r04/$T/pmc -o run -- python3 $R/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $R/gpurun_out/r04/$T/pmc.log 2>&1 || exit 1
cd $R && python3 scripts/step_pmc_summary.py gpurun_out/r04/$T/pmc > gpurun_out/r04/$T/summary.txt && cat gpurun_out/r04/$T/summary.txt

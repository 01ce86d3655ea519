# kh probes under PMC: does the no-DMA probe's speed-up come with a higher clock?  One counter pass per
# library (GRBM_GUI_ACTIVE, MFMA busy, waits) with the kernel trace for wall times.
cd $GRAFT_REPO_ROOT; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03_khclock
cd /tmp && export TMPDIR=/tmp
for v in libthk_base kh_probe8; do
  export TH_KERNEL_LIB=$R/ab_libs/$v.so
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace \
    --output-format csv -d $R/gpurun_out/r03_khclock/$v -o run -- python3 $R/scripts/flash_pmc.py \
    > $R/gpurun_out/r03_khclock/$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $R/gpurun_out/r03_khclock/$v.log; exit 1; }
done
cd $R && python3 scripts/kh_clock_pmc.py gpurun_out/r03_khclock/libthk_base gpurun_out/r03_khclock/kh_probe8

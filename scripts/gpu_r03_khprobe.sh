# kh timing probes (results deliberately wrong): what the P-exchange barrier and the dV role's
# exponentials cost the backward.  probe0 = control built the same way as the probes.
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_khprobe
A=$PWD/ab_libs
AB_ROUNDS=16 AB_BASE_LIB=$A/libthk_base.so AB_VARIANTS="p8_nodma=$A/kh_probe8.so,p32_contig=$A/kh_probe32.so" \
  run_step r03_khprobe/contig 400 python scripts/lib_ab.py
grep op gpurun_out/r03_khprobe/contig.log

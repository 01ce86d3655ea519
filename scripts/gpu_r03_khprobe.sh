# kh timing probes (results deliberately wrong): what the P-exchange barrier and the dV role's
# exponentials cost the backward.  probe0 = control built the same way as the probes.
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_khprobe
A=$PWD/ab_libs
AB_ROUNDS=24 AB_BASE_LIB=$A/libthk_base.so AB_VARIANTS="s2=$A/kh_split2.so,s4=$A/kh_split4.so,s6=$A/kh_split6.so" \
  run_step r03_khprobe/split 400 python scripts/lib_ab.py
grep op gpurun_out/r03_khprobe/split.log

set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py > gpurun_out/fa_test.log 2>&1
for i in 1 2; do
 for v in old new; do
  if [ $v = old ]; then export TH_KERNEL_LIB=$R/tensorhive_fixed_amd/ops/_build/libthk_old.so; else unset TH_KERNEL_LIB; fi
  cd /tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fa_ab/$v$i -o run -- python3 $R/scripts/flash_pmc.py > $R/gpurun_out/fa_ab_$v$i.log 2>&1
  cd $R
 done
done
if [ "${FA_AB_BENCH:-0}" = 1 ]; then
 for v in new old; do
  if [ $v = old ]; then export TH_KERNEL_LIB=$R/tensorhive_fixed_amd/ops/_build/libthk_old.so; else unset TH_KERNEL_LIB; fi
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/fa_ab_bench_$v.json 2> gpurun_out/fa_ab_bench_$v.err
 done
fi

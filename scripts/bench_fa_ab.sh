set -e
cd $GRAFT_REPO_ROOT
for v in ${FA_AB_SET:-0 8 0 8}; do
  TH_FA_BWD_FLAGS=$v timeout -k 10 300 python bench.py --steps 6 --warmup 2 >> gpurun_out/bench_ab_$v.json 2>> gpurun_out/bench_ab.err
done

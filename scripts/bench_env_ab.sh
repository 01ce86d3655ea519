set -e
# alternating bench runs under two settings of one env var: AB_VAR=NAME AB_VALS="1 0 1 0"
cd $GRAFT_REPO_ROOT
for v in $AB_VALS; do
  env "$AB_VAR=$v" timeout -k 10 300 python bench.py --steps 6 --warmup 2 >> gpurun_out/bench_ab_${AB_VAR}_$v.json 2>> gpurun_out/bench_ab.err
done

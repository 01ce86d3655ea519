# round 6: hipBLASLt stream-K grid knobs vs held CUs (w13 input gradient is stream-K by default): idle and 8 CUs
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-skenv}; O=gpurun_out/r06/$T; mkdir -p $O
summ() { python3 -c '
import sys, json
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(" ".join("k%d=%s" % (r["k"], r["ms"]) for r in rows if r["kernel"] == "blas.w13.dgrad"))' "$1"; }
for e in ${ENVS:-TENSILE_STREAMK_DYNAMIC_GRID=0 TENSILE_STREAMK_DYNAMIC_GRID=1 TENSILE_STREAMK_DYNAMIC_GRID=2 TENSILE_STREAMK_DYNAMIC_GRID=3 TENSILE_STREAMK_GRID_MULTIPLIER=2 TENSILE_STREAMK_FIXED_GRID=512 TENSILE_STREAMK_FIXED_GRID=248 TENSILE_STREAMK_DATA_PARALLEL=1 TENSILE_STREAMK_FULL_TILES=0}; do
  n=$(echo $e | tr '=' '_')
  ( export $e; KS=0,8 WHAT=blas run_step r06/$T/$n 200 python scripts/comm_gemm_micro.py ) || exit 1
  echo "$e $(summ $O/$n.log)"
done

# hipBLASLt environment A/B over the step's GEMM shapes: one process per setting, baseline repeated
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; out=gpurun_out/hipblaslt_env.jsonl; : > $out
run() { local tag=$1; shift; env AB_TAG=$tag "$@" timeout -k 10 120 python scripts/bench_hipblaslt_env.py >> $out 2> gpurun_out/hipblaslt_env_$tag.err || { echo "[env] $tag failed rc=$?"; tail -3 gpurun_out/hipblaslt_env_$tag.err; }; }
run base
run rocroller HIPBLASLT_USE_ROCROLLER=1
run sk_dyn0 TENSILE_STREAMK_DYNAMIC_GRID=0
run sk_dyn1 TENSILE_STREAMK_DYNAMIC_GRID=1
run sk_mult2 TENSILE_STREAMK_GRID_MULTIPLIER=2
run sk_dp TENSILE_STREAMK_DATA_PARALLEL=1
run sk_full TENSILE_STREAMK_FULL_TILES=1
run wgm8 TENSILE_FIXED_WGM=8
run wgmxcc8 TENSILE_FIXED_WGMXCC=8
run nostagger TENSILE_DISABLE_STAGGERU=1
run base2
python3 -c "
import json
for l in open('$out'):
    r=json.loads(l); print(r['env'], r['per_step_ms'], r['avg_tflops'], ' '.join(str(s['tflops']) for s in r['shapes']))"

# hipBLASLt workspace size (torch's HIPBLASLT_WORKSPACE_SIZE, KiB) over the step's GEMM shapes, baseline repeated
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; out=gpurun_out/hipblaslt_ws.jsonl; : > $out
run() { local tag=$1; shift; env AB_TAG=$tag "$@" timeout -k 10 120 python scripts/bench_hipblaslt_env.py >> $out 2> gpurun_out/hipblaslt_ws_$tag.err || { echo "[env] $tag failed rc=$?"; tail -3 gpurun_out/hipblaslt_ws_$tag.err; exit 1; }; }
run base
run ws128m HIPBLASLT_WORKSPACE_SIZE=131072
run ws1g HIPBLASLT_WORKSPACE_SIZE=1048576
run base2
python3 -c "
import json
for l in open('$out'):
    r=json.loads(l); print(r['env'], r['per_step_ms'], r['avg_tflops'], ' '.join(str(s['tflops']) for s in r['shapes']))"

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_gputest.log 2>&1 && echo TESTS_OK && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python bench.py > gpurun_out/r02_bench.log 2>&1 && tail -1 gpurun_out/r02_bench.log

#!/bin/bash
# kf (one-wave-per-SIMD fused dK|dV) check + A/B against kh: flash GPU tests, then the backward timing
set -o pipefail
T=${KF_TAG:-kf1}
OUT=gpurun_out/r04/$T
mkdir -p $OUT
export PYTHONUNBUFFERED=1
[ -z "$KF_NOTEST" ] && { timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py \
 > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }; }
tail -3 $OUT/test.log
FA_FLAGS=${KF_FLAGS:-0,16,0,16} timeout -k 10 200 python -u scripts/fa_bwd_ab.py > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
cat $OUT/ab.log
if [ -n "$KF_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  FA_FLAGS=${KF_FLAGS:-0,16} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/fa_bwd_ab.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec head -12 {} \;
  FA_FLAGS=${KF_FLAGS:-0,16} timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/pmc -o run -- python3 scripts/fa_bwd_ab.py > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
  python3 scripts/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt; cat $OUT/pmc_summary.txt
fi
if [ -n "$KF_STAMPS" ]; then
  timeout -k 10 200 python -u scripts/kf_stamps.py > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
  cat $OUT/stamps.log
fi

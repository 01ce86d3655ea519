#!/usr/bin/env bash
# rocprofv3 PMC passes (no tracing domains in the same run) over a workload script; summaries to gpurun_out/pmc_*.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
W="${1:-scripts/flash_pmc.py}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_CYCLES SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/pmc_$i" -o run -- python3 "$R/$W" \
    > "$R/gpurun_out/pmc_$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$R/gpurun_out/pmc_$i.log"; exit 1; }
done
cd "$R" && python3 scripts/pmc_summary.py gpurun_out/pmc_*/

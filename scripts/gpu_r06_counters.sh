# round 6: which TCC / fabric counters exist on gfx950 (for the w13 band question, round-5 verdict weak #9)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r06/counters; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/r06/counters/list.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/r06/counters/list.txt 2>&1
grep -oE "TCC_[A-Z0-9_]+|MALL[A-Z0-9_]*|DF_[A-Z0-9_]+" $R/gpurun_out/r06/counters/list.txt | sort -u | tr '\n' ' ' | head -c 4000

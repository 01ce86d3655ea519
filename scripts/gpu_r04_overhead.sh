# round 4: what the shipped monitoring costs on the final tree (th-counters on by default since round 4)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r04/daemon
run_step r04/daemon/overhead 900 python -m tensorhive_fixed_amd.cli bench overhead
grep '^{' gpurun_out/r04/daemon/overhead.log | cut -c1-900

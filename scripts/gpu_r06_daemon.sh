# round 6: the daemon halves on the final tree (background attestation, private agent event sockets): the
# queue-scheduled Llama-3-8B run and the multi-tenant queue on the real node
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh; T=${TAG:-daemon}; O=gpurun_out/r06/$T; mkdir -p $O
run_step r06/$T/mt_bench 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
grep '^{' $O/mt_bench.log | cut -c1-900
run_step r06/$T/scheduled 900 python -m tensorhive_fixed_amd.cli bench scheduled
grep '^{' $O/scheduled.log | cut -c1-700

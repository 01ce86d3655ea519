# round 4: kf variants (kernel A/B + PMC), then the training step with kh and the best kf candidates,
# alternating (A B C A B C), 10 timed steps each
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${KF_TAG:-kfstep}; mkdir -p gpurun_out/r04/$T
export PYTHONUNBUFFERED=1
KF_NOTEST=1 KF_PROF=${KF_PROF:-} KF_TAG=$T KF_FLAGS=${KF_FLAGS:-0,3024,7120} bash scripts/gpu_r04_kf.sh || exit 1
for round in 1 2; do
  for f in ${STEP_FLAGS:-0 3024 7120}; do
    TH_FA_BWD_FLAGS=$f run_step r04/$T/step_f${f}_r$round 400 python bench.py --gpus 1 --steps 10 --warmup 3 --daemon-bench 0
    echo "flags=$f round=$round $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04/$T/step_f${f}_r$round.log)"
  done
done

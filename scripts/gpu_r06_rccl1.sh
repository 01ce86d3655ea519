#!/bin/bash
# Round 6: the driver's N > 1 launch shape on one GPU -- torchrun, RCCL one-rank group with every collective
# issued (TH_FORCE_COLLECTIVES=1), ZeRO-1 sharded optimizer -- on the final tree.
set -o pipefail
OUT=gpurun_out/r06/rccl1
mkdir -p $OUT
export TH_FORCE_COLLECTIVES=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29631 \
  bench.py --gpus 1 --steps 6 --warmup 3 --daemon-bench 0 --zero 1 > $OUT/zero1.log 2>&1; rc=$?
echo "zero1 rc=$rc"; grep '^{"metric"' $OUT/zero1.log | cut -c1-400; exit $rc

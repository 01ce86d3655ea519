"""N06 output contract on CPU: the JSON schema rccl-bench must print (both modes), checked by
core/rccl_bench.parse.  The GPU runs of both modes are in tests/gpu/test_native_gpu.py."""
import json

import pytest

from tensorhive_fixed_amd.core import rccl_bench as R


def _out(mode="per_rank", world=8, extra=None):
    head = {"rccl_bench": 1, "mode": mode, "world": world, "rccl_version": 22703, "env": {"NCCL_DEBUG": "WARN"}}
    rows = [{"op": "allreduce", "mode": mode, "gpus": world, "bytes": 1 << 28, "time_us": 1000.0,
             "algbw_GBps": 268.44, "busbw_GBps": round(268.44 * 2 * (world - 1) / world, 2)},
            {"op": "allgather", "mode": mode, "gpus": world, "bytes": 1 << 28, "time_us": 700.0,
             "algbw_GBps": 383.49, "busbw_GBps": round(383.49 * (world - 1) / world, 2)}]
    return "\n".join(json.dumps(x) for x in [head] + rows + (extra or [])) + "\n"


def test_valid_output_parses():
    doc = R.parse(_out())
    assert doc["header"]["mode"] == "per_rank" and len(doc["results"]) == 2


@pytest.mark.parametrize("bad", [
    {"op": "allreduce", "mode": "per_rank", "gpus": 8, "bytes": 1 << 20, "time_us": 10.0, "algbw_GBps": 100.0,
     "busbw_GBps": 100.0},                                               # wrong bus-bandwidth factor
    {"op": "allreduce", "mode": "single_process", "gpus": 8, "bytes": 1 << 20, "time_us": 10.0,
     "algbw_GBps": 100.0, "busbw_GBps": 175.0},                         # mode differs from the header
    {"op": "broadcast", "mode": "per_rank", "gpus": 8, "bytes": 1, "time_us": 1.0, "algbw_GBps": 0.0,
     "busbw_GBps": 0.0},                                                 # unknown op
    {"op": "allreduce", "mode": "per_rank", "gpus": 8, "bytes": 1 << 20, "time_us": 10.0},  # missing keys
])
def test_schema_violations_are_rejected(bad):
    with pytest.raises(R.SchemaError):
        R.parse(_out(extra=[bad]))


def test_header_is_required():
    with pytest.raises(R.SchemaError):
        R.parse(json.dumps({"op": "allreduce"}) + "\n")

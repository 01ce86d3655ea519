"""Training payload checkpoint/resume: a run interrupted after a checkpoint and resumed with
``--resume`` ends with bit-identical parameters, optimizer state and loss to an uninterrupted run
(tiny Llama on CPU; the same code path runs on the GPU)."""
import json

import torch

from tensorhive_fixed_amd.workloads import llama3_ddp


def _run(argv, capsys):
    assert llama3_ddp.main(argv) == 0
    lines = [json.loads(line) for line in capsys.readouterr().out.splitlines() if line.startswith("{")]
    return lines


def test_resume_is_bit_exact(tmp_path, capsys, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    base = ["--model", "tiny", "--seq-len", "32", "--micro-batch", "2", "--log-every", "100"]
    full = _run(base + ["--steps", "6", "--warmup", "0", "--ckpt-dir", str(tmp_path / "a"), "--ckpt-every", "6"],
                capsys)
    # interrupted: 3 steps with a checkpoint at step 3, then a fresh process continues to 6
    _run(base + ["--steps", "3", "--warmup", "0", "--ckpt-dir", str(tmp_path / "b"), "--ckpt-every", "3"], capsys)
    resumed = _run(base + ["--steps", "6", "--warmup", "0", "--ckpt-dir", str(tmp_path / "b"), "--ckpt-every", "6",
                           "--resume"], capsys)
    assert resumed[0] == {"event": "resumed", "step": 3}
    assert full[-1]["steps"] == resumed[-1]["steps"] == 6
    assert full[-1]["loss"] == resumed[-1]["loss"]
    a = torch.load(tmp_path / "a" / "ckpt.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "ckpt.pt", weights_only=True)
    for k in ("param_buf", "master", "exp_avg", "exp_avg_sq", "step", "data_drawn"):
        assert torch.equal(a[k], b[k]), k


def test_layout_mismatch_is_refused(tmp_path, capsys):
    import pytest

    _run(["--model", "tiny", "--seq-len", "16", "--micro-batch", "1", "--steps", "1", "--warmup", "0",
          "--ckpt-dir", str(tmp_path), "--ckpt-every", "1"], capsys)
    st = torch.load(tmp_path / "ckpt.pt", weights_only=True)
    st["names"] = "something.else"
    torch.save(st, tmp_path / "ckpt.pt")
    with pytest.raises(ValueError):
        llama3_ddp.main(["--model", "tiny", "--seq-len", "16", "--micro-batch", "1", "--steps", "2", "--warmup", "0",
                         "--ckpt-dir", str(tmp_path), "--resume"])

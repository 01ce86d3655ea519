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


def _free_ports(n):
    """n distinct ports the OS handed out, all bound at once (so none repeats) and then released."""
    import contextlib
    import socket

    with contextlib.ExitStack() as st:
        socks = [st.enter_context(socket.socket()) for _ in range(n)]
        for s in socks:
            s.bind(("127.0.0.1", 0))
        return [s.getsockname()[1] for s in socks]


def _zero_ckpt_rank(rank, world, ports, argv_list, out_dir):
    import contextlib
    import io
    import os

    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1")
    torch.set_num_threads(2)
    for i, argv in enumerate(argv_list):
        os.environ["MASTER_PORT"] = str(ports[i])  # one OS-assigned port per run (no port + i guesses)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert llama3_ddp.main(argv) == 0
        with open(f"{out_dir}/out{i}.rank{rank}.txt", "w") as f:
            f.write(buf.getvalue())


def test_zero1_sharded_resume_is_bit_exact(tmp_path):
    """2 gloo ranks with the sharded optimizer: each rank checkpoints its own optimizer slices."""
    import torch.multiprocessing as mp

    base = ["--model", "tiny", "--seq-len", "32", "--micro-batch", "2", "--log-every", "100", "--warmup", "0",
            "--zero", "1"]
    runs = [base + ["--steps", "4", "--ckpt-dir", str(tmp_path / "a"), "--ckpt-every", "4"],
            base + ["--steps", "2", "--ckpt-dir", str(tmp_path / "b"), "--ckpt-every", "2"],
            base + ["--steps", "4", "--ckpt-dir", str(tmp_path / "b"), "--ckpt-every", "4", "--resume"]]
    mp.start_processes(_zero_ckpt_rank, args=(2, _free_ports(len(runs)), runs, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    done = [json.loads(x) for x in (tmp_path / "out0.rank0.txt").read_text().splitlines() if x.startswith("{")]
    resumed = [json.loads(x) for x in (tmp_path / "out2.rank0.txt").read_text().splitlines() if x.startswith("{")]
    assert resumed[0] == {"event": "resumed", "step": 2}
    assert done[-1]["loss"] == resumed[-1]["loss"]
    a = torch.load(tmp_path / "a" / "ckpt.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "ckpt.pt", weights_only=True)
    assert int(a["zero_world"]) == 2 and "master" not in a
    assert torch.equal(a["param_buf"], b["param_buf"])
    for r in range(2):
        sa = torch.load(tmp_path / "a" / f"ckpt.pt.optim.{r}-of-2", weights_only=True)
        sb = torch.load(tmp_path / "b" / f"ckpt.pt.optim.{r}-of-2", weights_only=True)
        for k in ("master", "exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k], sb[k]), (r, k)

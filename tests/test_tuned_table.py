"""The shipped TunableOp table (ops/tuned): well-formed, made for this image's library versions, lookup-only
loading, and off without a GPU or with TH_GEMM_TUNED=0."""
import csv

import torch

from tensorhive_fixed_amd.ops import tuned


def test_table_is_well_formed_and_matches_this_image():
    rows = list(csv.reader(open(tuned.TABLE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["PT_VERSION"] == torch.__version__.split("+")[0]
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    ops = [r for r in rows if r[0] != "Validator"]
    assert ops and all(len(r) == 4 and r[0].startswith("GemmTunableOp_BFloat16_") for r in ops)
    # the 32768-token forward / input-gradient shapes of the Llama-3-8B step are covered
    sigs = {r[1] for r in ops}
    assert "tn_28672_32768_4096_ld_4096_4096_28672" in sigs  # gate|up forward
    # the w13 input-gradient entry stays on the library default (its tuned choice measured 1 % slower)
    assert any(r[1] == "tn_4096_32768_28672_ld_28672_28672_4096" and r[2] == "Default" for r in ops)


def test_loader_is_off_without_a_gpu_or_when_disabled(monkeypatch):
    monkeypatch.setenv("TH_GEMM_TUNED", "1")
    if not torch.cuda.is_available():
        assert tuned.load_gemm_table() is False
    monkeypatch.setenv("TH_GEMM_TUNED", "0")
    assert tuned.load_gemm_table() is False


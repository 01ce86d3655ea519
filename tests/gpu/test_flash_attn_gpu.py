"""HIP flash attention (fwd, dQ, dK/dV) vs an fp32 PyTorch reference, on the packed-qkv layout."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

# The launch flags the production library serves (csrc/flash_attn.hip flags_shipped, round 6): the default
# kf path, the paired kh kernel (also the automatic fallback when S % 64 != 0), the fused register-staged
# dK|dV kernel beside the DMA dQ kernel, and register-staged tiles throughout (the automatic fallback when
# 32-bit DMA offsets overflow).  The experiment variants live in the TH_FA_DIAG build only.
KF_DEFAULT = 16 | (7535 << 6) | (1 << 19)
PROD_FLAGS = [KF_DEFAULT, 1 << 19, 8 | (1 << 19), 32]
PROD_IDS = ["kf_default", "kh", "fused_dkv", "regstage"]


def _ref(qkv, B, S, Hq, Hkv, D, causal=True):
    from tensorhive_fixed_amd.ops.attention import _split, attention_reference
    q, k, v = _split(qkv, B, S, Hq, Hkv, D)
    return attention_reference(q, k, v, causal).reshape(B * S, Hq * D)


@pytest.mark.parametrize("bwd_flags", PROD_FLAGS, ids=PROD_IDS)
@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 128, 4, 1), (2, 200, 8, 2), (1, 1024, 32, 8), (1, 64, 2, 2), (3, 192, 4, 2)])
def test_flash_fwd_bwd_matches_reference(B, S, Hq, Hkv, bwd_flags):
    from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd
    torch.manual_seed(0)
    D = 128
    row = (Hq + 2 * Hkv) * D
    qkv = torch.randn(B * S, row, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    x = qkv.float().requires_grad_(True)
    ref = _ref(x, B, S, Hq, Hkv, D)
    err = (o.float() - ref).abs().max().item()
    assert err < 2e-2, f"fwd max err {err}"
    # LSE check (natural log of sum exp(scale * s))
    from tensorhive_fixed_amd.ops.attention import _split
    q, k, _ = _split(x.detach(), B, S, Hq, Hkv, D)
    rep = Hq // Hkv
    s = (q.transpose(1, 2) @ k.transpose(1, 2).repeat_interleave(rep, 1).transpose(-1, -2)) / math.sqrt(D)
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device="cuda").triu(1), float("-inf"))
    lse_ref = torch.logsumexp(s, -1)
    assert (lse - lse_ref).abs().max().item() < 1e-2
    do = torch.randn_like(o)
    ref.backward(do.float())
    dqkv = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=bwd_flags)
    g = x.grad
    for name, a, b in (("dq", dqkv[:, : Hq * D], g[:, : Hq * D]),
                       ("dk", dqkv[:, Hq * D:(Hq + Hkv) * D], g[:, Hq * D:(Hq + Hkv) * D]),
                       ("dv", dqkv[:, (Hq + Hkv) * D:], g[:, (Hq + Hkv) * D:])):
        rel = ((a.float() - b).norm() / (b.norm() + 1e-6)).item()
        assert rel < 2e-2, f"{name} rel err {rel}"


def test_qkv_attention_with_rope_matches_sdpa_path():
    from tensorhive_fixed_amd.ops.attention import qkv_attention
    torch.manual_seed(1)
    B, S, Hq, Hkv, D = 2, 256, 8, 2, 128
    base = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    a = base.clone().requires_grad_(True)
    b = base.clone().requires_grad_(True)
    oa = qkv_attention(a * 1, B, S, Hq, Hkv, D, 500000.0, backend="hip")
    ob = qkv_attention(b * 1, B, S, Hq, Hkv, D, 500000.0, backend="sdpa")
    assert (oa.float() - ob.float()).abs().max().item() < 2e-2
    g = torch.randn_like(oa)
    oa.backward(g)
    ob.backward(g)
    rel = ((a.grad.float() - b.grad.float()).norm() / b.grad.float().norm()).item()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("bwd_flags", PROD_FLAGS, ids=PROD_IDS)
@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 200, 8, 2), (1, 384, 4, 4), (2, 320, 6, 3)])
def test_flash_noncausal_bwd_matches_reference(B, S, Hq, Hkv, bwd_flags):
    from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd
    torch.manual_seed(1)
    D = 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D, causal=False)
    x = qkv.float().requires_grad_(True)
    ref = _ref(x, B, S, Hq, Hkv, D, causal=False)
    assert (o.float() - ref).abs().max().item() < 2e-2
    do = torch.randn_like(o)
    ref.backward(do.float())
    dqkv = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, causal=False, flags=bwd_flags)
    rel = ((dqkv.float() - x.grad).norm() / x.grad.norm()).item()
    assert rel < 2e-2, f"dqkv rel err {rel}"


def test_retired_forward_variants_are_rejected():
    """Production library: only the default forward (and its register-staged twin for offsets past 2^31)."""
    from tensorhive_fixed_amd.ops.attention import flash_fwd
    B, S, Hq, Hkv, D = 1, 128, 4, 2, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, _ = flash_fwd(qkv, B, S, Hq, Hkv, D, variant=15)
    ref = _ref(qkv.float(), B, S, Hq, Hkv, D)
    assert (o.float() - ref).abs().max().item() < 2e-2
    for v in (0, 1, 7, 8, 31):
        with pytest.raises(RuntimeError, match="bad shape"):
            flash_fwd(qkv, B, S, Hq, Hkv, D, variant=v)


@pytest.mark.parametrize("bwd_flags", [KF_DEFAULT, 1 << 19], ids=["kf_default", "kh"])
@pytest.mark.parametrize("S,Hq,Hkv", [(4096, 32, 8), (8192, 8, 2)], ids=["S4096_bench_heads", "S8192_model_max"])
def test_flash_long_sequences_match_fp32(S, Hq, Hkv, bwd_flags):
    """The training shapes: S = 4096 (the bench) with Llama-3-8B's 32/8 heads, and S = 8192 (the
    model's maximum) -- fp32 reference computed per head group in chunks to bound its memory."""
    from tensorhive_fixed_amd.ops.attention import _split, flash_bwd, flash_fwd
    torch.manual_seed(3)
    B, D = 1, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    do = torch.randn_like(o)
    dqkv = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=bwd_flags)
    rep = Hq // Hkv
    mask = torch.ones(S, S, dtype=torch.bool, device="cuda").triu(1)
    for kv in range(Hkv):  # one GQA group at a time: q heads kv*rep..(kv+1)*rep share k/v head kv
        x = qkv.float().requires_grad_(True)
        q, k, v = _split(x, B, S, Hq, Hkv, D)
        qg = q[:, :, kv * rep:(kv + 1) * rep].transpose(1, 2)  # [B, rep, S, D]
        kg, vg = k[:, :, kv:kv + 1].transpose(1, 2), v[:, :, kv:kv + 1].transpose(1, 2)
        s = (qg @ kg.transpose(-1, -2)) / math.sqrt(D)
        p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
        og = (p @ vg).transpose(1, 2).reshape(B * S, rep * D)
        sl = slice(kv * rep * D, (kv + 1) * rep * D)
        rel_o = ((o[:, sl].float() - og).norm() / og.norm()).item()
        assert rel_o < 1e-2, f"group {kv} fwd rel err {rel_o}"
        og.backward(do[:, sl].float())
        g = x.grad
        for name, cols in (("dq", sl), ("dk", slice((Hq + kv) * D, (Hq + kv + 1) * D)),
                           ("dv", slice((Hq + Hkv + kv) * D, (Hq + Hkv + kv + 1) * D))):
            ref = g[:, cols]
            rel = ((dqkv[:, cols].float() - ref).norm() / (ref.norm() + 1e-6)).item()
            assert rel < 2e-2, f"group {kv} {name} rel err {rel}"
        del x, q, k, v, s, p, og, g


@pytest.mark.parametrize("bwd_flags", [KF_DEFAULT, 1 << 19], ids=["kf_default", "kh"])
@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 256, 8, 2), (2, 200, 4, 4), (1, 4096, 32, 8)])
def test_rotary_backward_in_the_kernels_matches_the_separate_pass(B, S, Hq, Hkv, bwd_flags):
    """The rotary backward folded into the dQ / dK epilogues gives the dqkv of the flash backward
    followed by the separate in-place rope pass (dq, dk rotated; dv untouched)."""
    from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd
    from tensorhive_fixed_amd.ops.rope import rope_inplace, rope_tables

    torch.manual_seed(7)
    D = 128
    qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda") * 0.5).to(torch.bfloat16)
    rope_inplace(qkv, S, Hq + Hkv, D, 500000.0, 1.0)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    do = torch.randn_like(o)
    ref = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=bwd_flags)
    rope_inplace(ref, S, Hq + Hkv, D, 500000.0, -1.0)
    got = flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=bwd_flags,
                    rope=rope_tables(S, D, 500000.0, qkv.device))
    err = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
    assert err < 5e-3, err  # one bf16 rounding less on the fused path
    assert torch.equal(got[:, (Hq + Hkv) * D:], ref[:, (Hq + Hkv) * D:])  # dv is not rotated


def test_unknown_kf_variant_is_rejected_before_any_launch():
    """An unlisted kf variant (flags bits 6-18) fails loudly instead of running a different kernel."""
    from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd
    B, S, Hq, Hkv, D = 1, 128, 4, 2, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    with pytest.raises(RuntimeError, match="bad shape"):
        flash_bwd(torch.randn_like(o), qkv, o, lse, B, S, Hq, Hkv, D, flags=16 | (5 << 6))


@pytest.mark.parametrize("flags", [16 | (3439 << 6) | (1 << 19), 16 | (7535 << 6), 0, 1 | (1 << 19), 2 | (1 << 19)],
                         ids=["kf_v3439", "kf_no_dq_spread", "kh_plain_dq", "q_major_dq", "old_dkv_order"])
def test_retired_backward_flags_are_rejected(flags):
    from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd
    B, S, Hq, Hkv, D = 1, 128, 4, 2, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    with pytest.raises(RuntimeError, match="bad shape"):
        flash_bwd(torch.randn_like(o), qkv, o, lse, B, S, Hq, Hkv, D, flags=flags)


# The 8-wave ping-pong forward (flags bit 6) lost to the default kernel (profiles/r06_flash/) and lives in the
# diagnostic library only: its numerics run when TH_KERNEL_LIB points at one (scripts/build_variant_lib.sh
# fa_diag -DTH_FA_DIAG=1), and the production library must refuse the flag.
_DIAG_LIB = __import__("os").environ.get("TH_KERNEL_LIB", "").endswith("fa_diag.so")


@pytest.mark.skipif(not _DIAG_LIB, reason="ping-pong forward: diagnostic library only")
@pytest.mark.parametrize("causal", [True, False], ids=["causal", "full"])
@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 128, 4, 1), (2, 200, 8, 2), (1, 1024, 32, 8), (3, 192, 4, 2),
                                        (2, 320, 6, 3), (1, 4096, 32, 8), (1, 8192, 8, 2)])
def test_pingpong_forward_matches_default_and_fp32(B, S, Hq, Hkv, causal):
    """The 8-wave ping-pong forward (flags bit 6): same output as the default kernel, fp32 reference on one
    GQA group (chunked for the long shapes), S % 64 != 0 and non-causal included."""
    from tensorhive_fixed_amd.ops.attention import _split, flash_fwd
    torch.manual_seed(5)
    D = 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D, causal=causal, variant=64)
    o_d, lse_d = flash_fwd(qkv, B, S, Hq, Hkv, D, causal=causal)
    assert (o.float() - o_d.float()).abs().max().item() < 1e-2
    assert (lse - lse_d).abs().max().item() < 1e-4
    rep = Hq // Hkv
    kv = Hkv - 1  # last group: the highest query heads of the last workgroup pair
    q, k, v = _split(qkv.float(), B, S, Hq, Hkv, D)
    qg = q[:, :, kv * rep:(kv + 1) * rep].transpose(1, 2)
    kg, vg = k[:, :, kv:kv + 1].transpose(1, 2), v[:, :, kv:kv + 1].transpose(1, 2)
    s = (qg @ kg.transpose(-1, -2)) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device="cuda").triu(1), float("-inf"))
    og = (torch.softmax(s, -1) @ vg).transpose(1, 2).reshape(B * S, rep * D)
    sl = slice(kv * rep * D, (kv + 1) * rep * D)
    rel = ((o[:, sl].float() - og).norm() / og.norm()).item()
    assert rel < 1e-2, f"fwd rel err {rel}"
    lse_ref = torch.logsumexp(s, -1)  # [B, rep, S]
    assert (lse[:, kv * rep:(kv + 1) * rep] - lse_ref).abs().max().item() < 1e-2


def test_pingpong_forward_refused_by_production_or_odd_groups():
    """Production: flag 64 is refused outright; diagnostic library: refused for an odd GQA group."""
    from tensorhive_fixed_amd.ops.attention import flash_fwd
    B, S, D = 1, 128, 128
    for Hq, Hkv in ((3, 1),) + (() if _DIAG_LIB else ((4, 2),)):
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
        with pytest.raises(RuntimeError, match="bad shape"):
            flash_fwd(qkv, B, S, Hq, Hkv, D, variant=64)

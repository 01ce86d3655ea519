"""One full-width Llama-3-8B block at the bench sequence length against an fp32 reference
(round-1 verdict, weak item 12): d 4096, 32 query / 8 kv heads, FFN 14336, S 4096.  The GPU
model runs every gfx950 kernel of the training step (fused add-norm, packed-QKV flash attention
with RoPE, gate|up SwiGLU, TN weight-grad GEMMs, fused LM-head CE) in bf16; the reference is the
same module on the CPU in float32 (plain PyTorch ops).  Also checks the f32 gradient-buffer path
(``TH_GRAD_FP32``) of the AdamW kernel and of a training step."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_full_width_block_matches_fp32_at_s4096():
    from tensorhive_fixed_amd.models.llama3 import Llama, LlamaConfig

    torch.set_num_threads(16)
    cfg = LlamaConfig(vocab_size=4096, dim=4096, n_layers=1, n_heads=32, n_kv_heads=8, ffn_dim=14336,
                      ce_chunk=4096)
    ref = Llama(cfg, device="cpu", dtype=torch.float32, seed=3)
    gpu = Llama(cfg, device="cuda", dtype=torch.bfloat16, seed=3)
    with torch.no_grad():
        for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
            pg.copy_(pr.to(torch.bfloat16))
            pr.copy_(pg.float().cpu())  # both sides start from the same bf16-representable weights
    g = torch.Generator().manual_seed(1)
    tok = torch.randint(0, cfg.vocab_size, (1, 4096), generator=g)
    tgt = torch.randint(0, cfg.vocab_size, (1, 4096), generator=g)
    t0 = time.time()
    lg = gpu(tok.cuda(), tgt.cuda())
    lg.backward()
    torch.cuda.synchronize()
    t1 = time.time()
    lr = ref(tok, tgt)
    lr.backward()
    t2 = time.time()
    lg, lr = float(lg.detach()), float(lr.detach())
    print(f"loss gpu {lg:.5f} fp32 {lr:.5f}; gpu {t1 - t0:.2f} s, cpu fp32 {t2 - t1:.1f} s")
    assert abs(lg - lr) < 1e-2
    worst = {}
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        worst[n] = _rel(pg.grad, pr.grad)
    print("grad rel L2:", {k: round(v, 4) for k, v in worst.items()})
    assert max(worst.values()) < 3e-2, worst


@pytest.mark.parametrize("n", [4096, 1 << 20])
def test_adamw_flat_f32_gradients(n):
    from tensorhive_fixed_amd.ops.adamw import adamw_flat_, grad_sumsq_

    torch.manual_seed(7)
    p = torch.randn(n, device="cuda").to(torch.bfloat16)
    g32 = torch.randn(n, device="cuda") * 1e-3
    outs = []
    for g in (g32, g32.to(torch.bfloat16)):
        master = p.float().clone()
        m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        ns = torch.zeros(1, device="cuda")
        grad_sumsq_(g, ns)
        assert abs(float(ns) - float(g.float().pow(2).sum())) <= 1e-3 * float(g.float().pow(2).sum())
        pp = p.clone()
        adamw_flat_(pp, master, m, v, g, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=1,
                    grad_scale=1.0, norm_sq=None, clip=0.0)  # no clipping: m must be exactly 0.1 g
        outs.append((master, m))
    # f32 gradients: the moment is the exact f32 value (no bf16 rounding of the gradient)
    assert torch.allclose(outs[0][1], 0.1 * g32, rtol=1e-6, atol=0)
    assert _rel(outs[0][0], outs[1][0]) < 1e-3


def test_training_step_with_f32_gradient_buffer_matches_bf16():
    from tensorhive_fixed_amd.models.llama3 import Llama, LlamaConfig
    from tensorhive_fixed_amd.parallel.flat import FlatAdamW, FlatParamStore

    cfg = LlamaConfig.tiny()
    res = {}
    for gdt in (torch.bfloat16, torch.float32):
        m = Llama(cfg, device="cuda", dtype=torch.bfloat16, seed=0)
        store = FlatParamStore(m.params_in_backward_order(), torch.device("cuda"), grad_dtype=gdt)
        opt = FlatAdamW(store, lr=1e-3, overlap=False)
        g = torch.Generator(device="cuda").manual_seed(0)
        losses = []
        for step in range(3):
            for i in range(2):  # two accumulated micro-batches
                tok = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
                tgt = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
                store.begin_microbatch(accumulate=i > 0, sync=i == 1)
                loss = m(tok, tgt, n_valid=2 * 2 * 128)
                loss.backward()
                losses.append(float(loss))
            store.finish_grad_sync()
            opt.step()
        torch.cuda.synchronize()
        assert store.grad_buf.dtype == gdt
        res[gdt] = (losses, store.param_buf.float().clone())
    (lb, pb), (lf, pf) = res[torch.bfloat16], res[torch.float32]
    assert max(abs(a - b) for a, b in zip(lb, lf)) < 2e-2, (lb, lf)
    assert _rel(pb, pf) < 1e-2

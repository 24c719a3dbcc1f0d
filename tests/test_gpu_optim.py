"""FusedAdamW (multi-tensor lthm_adamw_multi) vs torch.optim.AdamW
(wrapper.py:263-275 hyper-parameters), fp32 elementwise: 1e-6 relative (torch
uses lerp for the first moment, the kernel the b1 m + (1 - b1) g form)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fused_adamw_multi_matches_torch(dev):
    from recommendations_amd.optim import FusedAdamW
    torch.manual_seed(0)
    shapes = [(0,)] + [(int(s),) for s in torch.randint(1, 5000, (55,))] + [(256, 768), (1024, 256), (3, 5, 7)]
    ps = [torch.randn(s) for s in shapes]
    mine = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
    ref = [torch.nn.Parameter(p.clone()) for p in ps]
    kw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=1e-3)
    o1, o2 = FusedAdamW(mine, **kw), torch.optim.AdamW(ref, **kw, foreach=False)
    for it in range(3):
        gs = [torch.randn(s) for s in shapes]
        for a, b, gr in zip(mine, ref, gs):
            a.grad, b.grad = gr.to(dev), gr.clone()
        if it == 1:  # a parameter without a gradient is skipped
            mine[5].grad = ref[5].grad = None
        o1.step()
        o2.step()
    for a, b in zip(mine, ref):
        d = (a.detach().cpu() - b.detach()).abs().max() if a.numel() else torch.tensor(0.0)
        assert float(d) <= 1e-6 * max(1.0, float(b.detach().abs().max()) if b.numel() else 1.0)
    st = o1.state[mine[5]]
    assert st["step"] == 2 and o1.state[mine[6]]["step"] == 3


def test_fused_adamw_keeps_bf16_shadows_current(dev):
    """The bf16 GEMM operands (kernels.bf16_shadow) are rewritten by the AdamW pass
    itself: after each step the shadow equals bf16(param) exactly and the forward
    gets the same buffer back without a cast; a torch in-place write to the
    parameter (version bump) makes the next request re-cast."""
    from recommendations_amd import kernels as K
    from recommendations_amd.optim import FusedAdamW
    torch.manual_seed(1)
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in [(256, 768), (37,), (1024, 256)]]
    sh = [K.bf16_shadow(p) for p in ps[:2]]  # the third parameter has no shadow
    opt = FusedAdamW(ps, lr=1e-2, betas=(0.9, 0.95), weight_decay=1e-3)
    for _ in range(3):
        for p in ps:
            p.grad = torch.randn_like(p)
        opt.step()
        for p, s in zip(ps[:2], sh):
            assert K.bf16_shadow(p) is s
            assert torch.equal(s, p.detach().to(torch.bfloat16))
    assert K.shadow_of(ps[2]) is None
    with torch.no_grad():
        ps[0].copy_(torch.randn_like(ps[0]))
    assert K.shadow_of(ps[0]) is None
    s0 = K.bf16_shadow(ps[0])
    assert s0 is not sh[0] and torch.equal(s0, ps[0].detach().to(torch.bfloat16))

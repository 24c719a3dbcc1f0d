import sys, torch
sys.path.insert(0, '.')
from recommendations_amd.commons.layers import MLP
from oracle import ref
torch.manual_seed(0)
for din, hid in [(4, 64), (8, 64), (4, 32), (12, 64), (24, 32)]:
    m = MLP(din, 1, [hid])
    x = torch.randn(3000, din)
    lins = [l for l in m.model if isinstance(l, torch.nn.Linear)]
    xc = x.clone().requires_grad_(True)
    ws = [l.weight.detach().clone().requires_grad_(True) for l in lins]; bs = [l.bias.detach().clone().requires_grad_(True) for l in lins]
    yc = ref.mlp_quickgelu(xc, ws, bs); g = torch.randn_like(yc); yc.backward(g)
    md = m.cuda(); xd = x.cuda().requires_grad_(True)
    yd = md(xd); yd.backward(g.cuda())
    def re(a, b): return float((a.detach().cpu().double() - b.detach().double()).norm() / b.detach().double().norm())
    print(din, hid, 'y', re(yd, yc), 'dx', re(xd.grad, xc.grad), 'dx col0', re(xd.grad[:, 0], xc.grad[:, 0]), 'dW0', re(md.model[0].weight.grad, ws[0].grad), 'dW1', re(lins[1].weight.grad if False else md.model[2].weight.grad, ws[1].grad))

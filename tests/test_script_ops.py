"""The scriptable boundary: TORCH_LIBRARY(lthm) ops (csrc/torch_ops/lthm_ops.cpp).

SURVEY §8(b): the reference scripts its item-embedding module and saves it
(embedding_module_gen.py:191-192); the LTHM encoder loads it back
(models/lthm/sequence/encoder.py:29).  CPU tests: the op library registers every
op with its schema, the modules script into graphs that call ``ops.lthm.*``, a
scripted module survives save/load, and a CPU tensor raises (no fallback).  GPU
tests: scripted and eager modules agree bit-exactly through the same kernels.
"""
import io

import pytest
import torch
import torch.nn as nn

from recommendations_amd import _lib

OPS = {
    "abi_version": "lthm::abi_version() -> int",
    "kshift": "lthm::kshift(Tensor ids, Tensor weight, int P, int K, int mode, int F=1, ScalarType? out_dtype=None)"
              " -> Tensor",
    "kshift_rows": "lthm::kshift_rows(Tensor ids, int P, int K) -> Tensor",
    "gather_pool": "lthm::gather_pool(Tensor rows, Tensor weight, int mode, ScalarType out_dtype=6) -> Tensor",
    "activation": "lthm::activation(Tensor x, int act) -> Tensor",
    "mlp_chain": "lthm::mlp_chain(Tensor x, Tensor[] weights, Tensor[] biases, int[] acts, bool out_f32=True)"
                 " -> Tensor",
    "item_artifact": "lthm::item_artifact(Tensor ids, Tensor weight, int K, int mode, Tensor mask_weight, int mask_K,"
                     " Tensor w1, Tensor b1, Tensor w2, Tensor b2, ScalarType out_dtype=6) -> Tensor",
}


def _wrapper(P=5000, D=32, Dm=4):
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    from recommendations_amd.embedding_module_gen import ModelWrapper
    torch.manual_seed(0)
    mask = nn.Sequential(KShiftEmbedding(P, Dm, num_shifts=16), MLP(Dm, 1, [Dm * 16]))
    return ModelWrapper(KShiftEmbedding(P, D, num_shifts=16, normalize_output=True), mask).eval()


def test_op_library_registers_every_op():
    _lib.load_torch_ops()
    for name, schema in OPS.items():
        assert str(getattr(torch.ops.lthm, name).default._schema) == schema
    with open(_lib.HEADER) as f:
        import re
        want = int(re.search(r"#define\s+LTHM_ABI_VERSION\s+(\d+)", f.read()).group(1))
    assert torch.ops.lthm.abi_version() == want


def test_cpu_tensor_raises():
    _lib.load_torch_ops()
    with pytest.raises(RuntimeError, match="MI355X"):
        torch.ops.lthm.kshift(torch.zeros(3, dtype=torch.int64), torch.zeros(10, 4), 10, 2, 0)
    with pytest.raises(RuntimeError):  # no CPU kernel registered: the dispatcher refuses
        torch.ops.lthm.kshift_rows(torch.zeros(3, dtype=torch.int64), 10, 2)


def test_modules_script_and_round_trip():
    """embedding_module_gen.py:189-192: torch.jit.script(ModelWrapper) + save; then load."""
    _lib.load_torch_ops()
    sw = torch.jit.script(_wrapper())
    graph = str(sw.inlined_graph)
    assert "lthm::kshift" in graph and "lthm::mlp_chain" in graph
    buf = io.BytesIO()
    torch.jit.save(sw, buf)
    buf.seek(0)
    lw = torch.jit.load(buf)
    assert set(dict(lw.named_parameters())) == set(dict(sw.named_parameters()))


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [False, True])
def test_scripted_kshift_matches_eager(dev, normalize):
    from recommendations_amd.commons.layers import KShiftEmbedding
    _lib.load_torch_ops()
    torch.manual_seed(1)
    m = KShiftEmbedding(100_003, 32, num_shifts=16, normalize_output=normalize).to(dev)
    sm = torch.jit.script(m)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (257, 31), dtype=torch.int64, device=dev)
    y = m(ids)
    ys = sm(ids)
    assert torch.equal(y, ys)
    dy = torch.randn_like(y)
    (g,) = torch.autograd.grad((y * dy).sum(), m.emb.weight)
    (gs,) = torch.autograd.grad((ys * dy).sum(), m.emb.weight)
    # same kernel; the f32 atomic adds of a hot row's blocks land in any order: 1e-5 of the
    # largest row gradient (the hot rows P-1.. collect ~half of all adds)
    torch.testing.assert_close(gs, g, rtol=1e-5, atol=1e-5 * float(g.abs().max()))
    rows = torch.ops.lthm.kshift_rows(ids, 100_003, 16)
    assert torch.equal(rows, torch.stack([m.get_row_idx(ids, c) for c in range(16)], -1))


@pytest.mark.gpu
def test_scripted_model_wrapper_matches_eager(dev):
    """The scripted, saved and reloaded item-embedding module (the artifact the
    reference's encoder torch.jit.loads) is bit-identical to the eager one."""
    _lib.load_torch_ops()
    w = _wrapper().to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (64, 50), dtype=torch.int64, device=dev)
    with torch.no_grad():
        want = w(ids)
        sw = torch.jit.script(w)
        got = sw(ids)
        buf = io.BytesIO()
        torch.jit.save(sw, buf)
        buf.seek(0)
        got2 = torch.jit.load(buf, map_location=dev)(ids)
    assert torch.equal(got, want) and torch.equal(got2, want)
    # the fused one-kernel artifact op over the same weights: its mask MLP runs in f32, the
    # module's MLP on bf16 MFMA operands (1e-5 vs the f32 oracle: test_gpu_embgen.py)
    mlp = w.mask_model[1].model
    fused = torch.ops.lthm.item_artifact(ids, w.model.emb.weight, 16, 1, w.mask_model[0].emb.weight, 16,
                                         mlp[0].weight, mlp[0].bias, mlp[2].weight.view(-1), mlp[2].bias,
                                         torch.float32)
    from parity import check, relerr
    check("fused item artifact vs scripted ModelWrapper", relerr(fused, want), 1e-3)


@pytest.mark.gpu
def test_scripted_mlp_grads_match_eager(dev):
    from recommendations_amd.commons.layers import MLP
    _lib.load_torch_ops()
    torch.manual_seed(3)
    m = MLP(48, 7, [96, 40]).to(dev)
    sm = torch.jit.script(m)
    x = torch.randn(3000, 48, device=dev, requires_grad=True)
    y = m(x)
    ys = sm(x)
    assert torch.equal(y, ys)
    dy = torch.randn_like(y)
    ps = [x] + list(m.parameters())
    g = torch.autograd.grad((y * dy).sum(), ps)
    gs = torch.autograd.grad((ys * dy).sum(), ps)
    for a, b in zip(g, gs):
        if a.dim() == 1:  # bias: lthm_colsum folds its row chunks with f32 atomics (any order)
            torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-6 * float(a.abs().max()))
        else:  # dgrad / split-K wgrad: fixed summation order
            assert torch.equal(a, b)

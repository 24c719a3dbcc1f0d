import os, sys, collections
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
from recommendations_amd import kernels as K
seen = collections.Counter()
orig = K.gemm
def spy(A, B, M, N, Kd, **kw):
    seen[(K._GEMM_TAG[-1] if K._GEMM_TAG else "", M, N, Kd, kw.get("a_kcontig", True), kw.get("b_kcontig", True),
          str(kw.get("out_dtype")), kw.get("act", 0), kw.get("bias") is not None, kw.get("res1") is not None,
          kw.get("ldc"), kw.get("splits", 1))] += 1
    return orig(A, B, M, N, Kd, **kw)
K.gemm = spy
dev = torch.device("cuda:0")
cfgd = dict(bench.CONFIGS["c2"])
cfg, model = bench.build(cfgd, dev)
opts = model.optimizers_for_param_groups(model.param_groups())
from recommendations_amd.data import synthetic_lthm_batch
batch = synthetic_lthm_batch(cfgd["B"], cfgd["T"], n_cat=cfgd["n_cat"], seed=1234, rank=0, device=dev)
for _ in range(2):
    seen.clear()
    out = model(batch); loss, _ = model.train_step(batch, out); loss.backward()
    for o in opts:
        o.step(); o.zero_grad(set_to_none=True)
torch.cuda.synchronize()
for k, v in sorted(seen.items(), key=lambda x: str(x[0])):
    if k[0] != "enc":
        print(v, k)

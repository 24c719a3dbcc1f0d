// TORCH_LIBRARY(lthm) — the scriptable op layer over the C ABI of include/lthm.h.
//
// the reference's boundary is the PyTorch module API, and its offline
// caller scripts the item-embedding module (embedding_module_gen.py:191-192,
// `torch.jit.script(final_model)`) and the LTHM encoder loads it again
// (models/lthm/sequence/encoder.py:29).  The ctypes path in kernels.py cannot be
// compiled by TorchScript; these dispatcher ops can.  Each op checks its operands on
// the host (TORCH_CHECK -> RuntimeError, the reference's error style), allocates its
// outputs through the torch caching allocator and launches the same gfx950 kernel the
// eager path launches, on torch's current HIP stream.  Only the CUDA (= HIP on ROCm)
// and Autograd dispatch keys are implemented: a CPU tensor raises (no CPU fallback).
//
//   lthm::kshift        KShiftEmbedding.forward     commons/layers.py:152-172 (+ dense backward)
//   lthm::kshift_rows   KShiftEmbedding.get_row_idx commons/layers.py:174-185
//   lthm::gather_pool   the C3 row-sharded pool     
//   lthm::mlp_chain     MLP + QuickGELU             commons/layers.py:65-81 (+ backward)
//   lthm::activation    QuickGELU / GELU(tanh)      commons/layers.py:9-11 (+ backward)
//   lthm::item_artifact ModelWrapper.forward        embedding_module_gen.py:32-41 (fused)
#include <ATen/hip/HIPContext.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <vector>

#include "../../../include/lthm.h"

namespace {

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::tensor_list;

void* cur_stream() { return reinterpret_cast<void*>(at::hip::getCurrentHIPStream().stream()); }

int32_t dcode(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return LTHM_F32;
  if (t.scalar_type() == at::kBFloat16) return LTHM_BF16;
  TORCH_CHECK(false, "lthm ops take float32 or bfloat16 tensors, got ", t.scalar_type());
}

void on_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "lthm ops run only on an MI355X (gfx950) device; ", name, " is on ", t.device(),
              ". The CPU restatement lives in oracle/ and is test infrastructure only.");
}

void hip_ok(int rc, const char* fn) { TORCH_CHECK(rc == 0, fn, " failed with hip error ", rc); }

const void* cptr(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }

Tensor cast_to(const Tensor& x, at::ScalarType dt) {
  if (x.scalar_type() == dt) return x;
  auto xc = x.contiguous();
  auto out = at::empty(xc.sizes(), xc.options().dtype(dt));
  hip_ok(lthm_cast(xc.data_ptr(), dcode(xc), out.data_ptr(), dcode(out), xc.numel(), cur_stream()), "lthm_cast");
  return out;
}

// ---------------------------------------------------------------- KShift
void check_kshift(const Tensor& ids, const Tensor& weight, int64_t P, int64_t K, int64_t F) {
  on_gpu(ids, "ids");
  on_gpu(weight, "weight");
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids must be int64, got ", ids.scalar_type());
  TORCH_CHECK(P > 0 && K > 0 && K <= 64 && F >= 1, "bad KShift config P=", P, " K=", K, " F=", F);
  TORCH_CHECK(weight.dim() == 2 && weight.size(0) == F * P, "weight must be [F*P, D] = [", F * P, ", D], got ",
              weight.sizes());
  TORCH_CHECK(ids.numel() % F == 0, "ids.numel()=", ids.numel(), " is not a multiple of F=", F);
  TORCH_CHECK(weight.is_contiguous(), "weight must be contiguous");
}

std::tuple<Tensor, Tensor> kshift_fwd_impl(const Tensor& ids_, const Tensor& weight, int64_t P, int64_t K,
                                           int64_t mode, int64_t F, c10::optional<at::ScalarType> out_dtype,
                                           bool want_norms) {
  check_kshift(ids_, weight, P, K, F);
  auto ids = ids_.contiguous();
  const int64_t D = weight.size(1);
  auto shape = ids.sizes().vec();
  shape.push_back(D);
  auto out = at::empty(shape, weight.options().dtype(out_dtype.value_or(weight.scalar_type())));
  Tensor norms;
  if (mode == LTHM_KSHIFT_NORMALIZE && want_norms) norms = at::empty(ids.sizes(), weight.options().dtype(at::kFloat));
  hip_ok(lthm_kshift_fwd_multi(ids.data_ptr<int64_t>(), ids.numel() / F, (int32_t)F, weight.data_ptr(), dcode(weight),
                               P, (int32_t)D, (int32_t)K, (int32_t)mode, out.data_ptr(), dcode(out),
                               norms.defined() ? norms.data_ptr<float>() : nullptr, cur_stream()),
         "lthm_kshift_fwd_multi");
  return {out, norms};
}

Tensor kshift_cuda(const Tensor& ids, const Tensor& weight, int64_t P, int64_t K, int64_t mode, int64_t F,
                   c10::optional<at::ScalarType> out_dtype) {
  return std::get<0>(kshift_fwd_impl(ids, weight, P, K, mode, F, out_dtype, false));
}

class KShiftFunction : public torch::autograd::Function<KShiftFunction> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& ids, const Tensor& weight, int64_t P, int64_t K,
                        int64_t mode, int64_t F, c10::optional<at::ScalarType> out_dtype) {
    at::AutoDispatchBelowADInplaceOrView guard;
    auto [out, norms] = kshift_fwd_impl(ids, weight, P, K, mode, F, out_dtype, true);
    ctx->save_for_backward({ids.contiguous(), mode == LTHM_KSHIFT_NORMALIZE ? out : Tensor(), norms});
    ctx->saved_data["P"] = P;
    ctx->saved_data["K"] = K;
    ctx->saved_data["mode"] = mode;
    ctx->saved_data["F"] = F;
    ctx->saved_data["rows"] = weight.size(0);
    ctx->saved_data["D"] = weight.size(1);
    ctx->saved_data["wdtype"] = weight.scalar_type();
    return out;
  }
  static tensor_list backward(AutogradContext* ctx, tensor_list grads) {
    auto saved = ctx->get_saved_variables();
    const Tensor& ids = saved[0];
    const Tensor& out = saved[1];
    const Tensor& norms = saved[2];
    const int64_t P = ctx->saved_data["P"].toInt(), K = ctx->saved_data["K"].toInt();
    const int64_t mode = ctx->saved_data["mode"].toInt(), F = ctx->saved_data["F"].toInt();
    const int64_t rows = ctx->saved_data["rows"].toInt(), D = ctx->saved_data["D"].toInt();
    const auto wdt = ctx->saved_data["wdtype"].toScalarType();
    auto gy = grads[0].contiguous();
    TORCH_CHECK(gy.numel() == ids.numel() * D, "grad has ", gy.numel(), " elements, expected ", ids.numel() * D);
    auto dW = at::empty({rows, D}, gy.options().dtype(at::kFloat));
    hip_ok(lthm_fill_f32(dW.data_ptr<float>(), 0.f, dW.numel(), cur_stream()), "lthm_fill_f32");
    hip_ok(lthm_kshift_bwd_dense(ids.data_ptr<int64_t>(), ids.numel() / F, (int32_t)F, gy.data_ptr(), dcode(gy),
                                 out.defined() ? out.data_ptr() : nullptr, out.defined() ? dcode(out) : LTHM_F32,
                                 norms.defined() ? norms.data_ptr<float>() : nullptr, P, (int32_t)D, (int32_t)K,
                                 (int32_t)mode, dW.data_ptr<float>(), cur_stream()),
           "lthm_kshift_bwd_dense");
    if (wdt != at::kFloat) dW = cast_to(dW, wdt);
    return {Tensor(), dW, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

Tensor kshift_autograd(const Tensor& ids, const Tensor& weight, int64_t P, int64_t K, int64_t mode, int64_t F,
                       c10::optional<at::ScalarType> out_dtype) {
  return KShiftFunction::apply(ids, weight, P, K, mode, F, out_dtype);
}

Tensor kshift_rows_cuda(const Tensor& ids_, int64_t P, int64_t K) {
  on_gpu(ids_, "ids");
  TORCH_CHECK(ids_.scalar_type() == at::kLong, "ids must be int64");
  TORCH_CHECK(P > 0 && K > 0 && K <= 64, "bad KShift config P=", P, " K=", K);
  auto ids = ids_.contiguous();
  auto shape = ids.sizes().vec();
  shape.push_back(K);
  auto rows = at::empty(shape, ids.options());
  hip_ok(lthm_kshift_rows(ids.data_ptr<int64_t>(), ids.numel(), P, (int32_t)K, rows.data_ptr<int64_t>(),
                          cur_stream()),
         "lthm_kshift_rows");
  return rows;
}

Tensor gather_pool_cuda(const Tensor& rows_, const Tensor& W, int64_t mode, at::ScalarType out_dtype) {
  on_gpu(rows_, "rows");
  on_gpu(W, "W");
  TORCH_CHECK(rows_.scalar_type() == at::kLong && rows_.dim() == 2, "rows must be int64 [n, K]");
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "W must be a contiguous [R, D] table");
  const int64_t n = rows_.size(0), K = rows_.size(1), D = W.size(1);
  TORCH_CHECK(K > 0 && K <= 64, "K must be in 1..64");
  auto rows = rows_.contiguous();
  auto out = at::empty({n, D}, W.options().dtype(out_dtype));
  hip_ok(lthm_gather_pool(rows.data_ptr<int64_t>(), n, (int32_t)K, W.data_ptr(), dcode(W), W.size(0), (int32_t)D,
                          (int32_t)mode, out.data_ptr(), dcode(out), nullptr, cur_stream()),
         "lthm_gather_pool");
  return out;
}

// ---------------------------------------------------------------- GEMM chain (MLP)
// split-K factor of kernels._splits_for (same kernel choice => same summation order as eager)
int64_t splits_for(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
  if (tiles >= 256 || K < 4096) return 1;
  const int64_t s = std::max<int64_t>(1, std::min<int64_t>(512 / tiles, K / 2048));
  const int64_t tiles256 = ((M + 255) / 256) * ((N + 255) / 256);
  return std::max(s, std::min<int64_t>(256 / tiles256, K / 256));
}

// C = epi(A . B) with A [M, K] (a_kc) or [K, M]; B [N, K] (b_kc) or [K, N]; all bf16, C out_dtype.
Tensor gemm(const Tensor& A, const Tensor& B, int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc,
            at::ScalarType out_dtype, const Tensor& bias, int32_t act, const Tensor& aux, const Tensor& aux_out,
            int64_t splits = 1) {
  auto C = at::empty({M, N}, A.options().dtype(out_dtype));
  lthm_gemm_desc d{};
  d.A = A.data_ptr();
  d.B = B.data_ptr();
  d.C = C.data_ptr();
  d.M = M;
  d.N = N;
  d.K = K;
  d.lda = a_kc ? K : M;
  d.ldb = b_kc ? K : N;
  d.ldc = N;
  d.sA = d.sB = 0;
  d.sC = M * N;
  d.batch = 1;
  d.a_kcontig = a_kc;
  d.b_kcontig = b_kc;
  d.out_dtype = dcode(C);
  d.alpha = 1.f;
  d.act = act;
  d.bias = bias.defined() ? bias.data_ptr<float>() : nullptr;
  d.aux = aux.defined() ? aux.data_ptr() : nullptr;
  d.aux_out = aux_out.defined() ? aux_out.data_ptr() : nullptr;
  d.ldaux = N;
  d.res1_dtype = d.res2_dtype = LTHM_F32;
  d.ldr1 = d.ldr2 = N;
  d.splits = (int32_t)splits;
  Tensor ws;
  if (splits > 1) {
    ws = at::empty({splits * M * N}, A.options().dtype(at::kFloat));
    d.workspace = ws.data_ptr<float>();
    d.workspace_bytes = (size_t)ws.numel() * 4;
  }
  d.ab_dtype = LTHM_BF16;
  hip_ok(lthm_gemm(&d, cur_stream()), "lthm_gemm");
  return C;
}

int32_t act_grad_of(int64_t act) {
  if (act == LTHM_ACT_GELU) return LTHM_ACT_GELU_GRAD;
  if (act == LTHM_ACT_QGELU) return LTHM_ACT_QGELU_GRAD;
  return LTHM_ACT_NONE;
}

void check_chain(const Tensor& x, const std::vector<Tensor>& ws, const std::vector<c10::optional<Tensor>>& bs,
                 const std::vector<int64_t>& acts) {
  on_gpu(x, "x");
  TORCH_CHECK(!ws.empty() && ws.size() == bs.size() && ws.size() == acts.size(),
              "mlp_chain: weights, biases and acts must have one entry per Linear");
  int64_t din = x.size(-1);
  for (size_t i = 0; i < ws.size(); ++i) {
    on_gpu(ws[i], "weight");
    TORCH_CHECK(ws[i].dim() == 2 && ws[i].size(1) == din, "Linear ", i, ": weight ", ws[i].sizes(),
                " does not take ", din, " inputs");
    if (bs[i].has_value() && bs[i]->defined())
      TORCH_CHECK(bs[i]->numel() == ws[i].size(0) && bs[i]->scalar_type() == at::kFloat, "Linear ", i,
                  ": bias must be f32 [", ws[i].size(0), "]");
    TORCH_CHECK(acts[i] == LTHM_ACT_NONE || acts[i] == LTHM_ACT_GELU || acts[i] == LTHM_ACT_QGELU,
                "mlp_chain: act must be none, GELU or QuickGELU");
    din = ws[i].size(0);
  }
}

// forward of kernels.MLPChainFn: bf16 operands, bias + act fused, last layer f32 (out_f32) or bf16
Tensor mlp_chain_fwd(const Tensor& x, const std::vector<Tensor>& ws, const std::vector<c10::optional<Tensor>>& bs,
                     const std::vector<int64_t>& acts, bool out_f32, std::vector<Tensor>* hs, std::vector<Tensor>* pres,
                     std::vector<Tensor>* wsb) {
  check_chain(x, ws, bs, acts);
  const int64_t din = x.size(-1), M = x.numel() / din;
  Tensor h = cast_to(x.contiguous().view({M, din}), at::kBFloat16);
  const size_t n = ws.size();
  for (size_t i = 0; i < n; ++i) {
    const bool last = i + 1 == n;
    Tensor wb = cast_to(ws[i].detach().contiguous(), at::kBFloat16);
    const int64_t N = wb.size(0), K = wb.size(1);
    Tensor pre;
    if (acts[i] != LTHM_ACT_NONE) pre = at::empty({M, N}, h.options().dtype(at::kBFloat16));
    Tensor b = (bs[i].has_value() && bs[i]->defined()) ? bs[i]->detach().contiguous() : Tensor();
    if (hs) hs->push_back(h);
    h = gemm(h, wb, M, N, K, true, true, (last && out_f32) ? at::kFloat : at::kBFloat16, b, (int32_t)acts[i],
             Tensor(), pre);
    if (pres) pres->push_back(pre);
    if (wsb) wsb->push_back(wb);
  }
  auto shape = x.sizes().vec();
  shape.back() = h.size(1);
  return h.view(shape);
}

std::vector<c10::optional<Tensor>> opt_list(at::TensorList biases) {
  std::vector<c10::optional<Tensor>> bs;
  for (const auto& b : biases) bs.push_back(b);
  return bs;
}

Tensor mlp_chain_cuda(const Tensor& x, at::TensorList weights, at::TensorList biases, at::IntArrayRef acts,
                      bool out_f32) {
  auto bs = opt_list(biases);
  return mlp_chain_fwd(x, weights.vec(), bs, acts.vec(), out_f32, nullptr, nullptr, nullptr);
}

class MLPChainFunction : public torch::autograd::Function<MLPChainFunction> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& x, at::TensorList weights, at::TensorList biases,
                        at::IntArrayRef acts, bool out_f32) {
    at::AutoDispatchBelowADInplaceOrView guard;
    auto bs = opt_list(biases);
    std::vector<Tensor> hs, pres, wsb;
    Tensor y = mlp_chain_fwd(x, weights.vec(), bs, acts.vec(), out_f32, &hs, &pres, &wsb);
    const size_t n = weights.size();
    std::vector<Tensor> save;
    for (auto& t : hs) save.push_back(t);
    for (auto& t : pres) save.push_back(t);
    for (auto& t : wsb) save.push_back(t);
    ctx->save_for_backward(save);
    std::vector<int64_t> has_b;
    for (auto& b : bs) has_b.push_back(b.has_value() && b->defined());
    ctx->saved_data["n"] = (int64_t)n;
    ctx->saved_data["acts"] = acts.vec();
    ctx->saved_data["has_b"] = has_b;
    ctx->saved_data["xdt"] = x.scalar_type();
    ctx->saved_data["xshape"] = x.sizes().vec();
    return y;
  }
  static tensor_list backward(AutogradContext* ctx, tensor_list grads) {
    auto saved = ctx->get_saved_variables();
    const int64_t n = ctx->saved_data["n"].toInt();
    const auto acts = ctx->saved_data["acts"].toIntVector();
    const auto has_b = ctx->saved_data["has_b"].toIntVector();
    const auto xdt = ctx->saved_data["xdt"].toScalarType();
    const auto xshape = ctx->saved_data["xshape"].toIntVector();
    std::vector<Tensor> hs(saved.begin(), saved.begin() + n), pres(saved.begin() + n, saved.begin() + 2 * n),
        wsb(saved.begin() + 2 * n, saved.begin() + 3 * n);
    Tensor g = grads[0].contiguous();
    const int64_t M = hs[0].size(0);
    Tensor gb = cast_to(g.view({M, g.size(-1)}), at::kBFloat16);
    std::vector<Tensor> dW(n), db(n);
    Tensor dx;
    for (int64_t i = n - 1; i >= 0; --i) {
      const int64_t N = wsb[i].size(0), K = wsb[i].size(1);
      // dW = gb^T h  (both K-strided over the M token rows), f32 [N, K]
      dW[i] = gemm(gb, hs[i], N, K, M, false, false, at::kFloat, Tensor(), LTHM_ACT_NONE, Tensor(), Tensor(),
                   splits_for(N, K, M));
      if (has_b[i]) {
        db[i] = at::empty({N}, gb.options().dtype(at::kFloat));
        hip_ok(lthm_colsum(gb.data_ptr(), LTHM_BF16, M, N, N, db[i].data_ptr<float>(), 0, cur_stream()),
               "lthm_colsum");
      }
      if (i > 0) {
        gb = gemm(gb, wsb[i], M, K, N, true, false, at::kBFloat16, Tensor(), act_grad_of(acts[i - 1]), pres[i - 1],
                  Tensor());
      } else {
        dx = gemm(gb, wsb[0], M, K, N, true, false, xdt == at::kFloat ? at::kFloat : at::kBFloat16, Tensor(),
                  LTHM_ACT_NONE, Tensor(), Tensor());
      }
    }
    // one gradient slot per input variable: x, each weight, each bias (TensorLists expand), acts, out_f32
    tensor_list out{dx.view(xshape)};
    for (auto& t : dW) out.push_back(t);
    for (int64_t i = 0; i < n; ++i) out.push_back(has_b[i] ? db[i] : Tensor());
    out.push_back(Tensor());
    out.push_back(Tensor());
    return out;
  }
};

Tensor mlp_chain_autograd(const Tensor& x, at::TensorList weights, at::TensorList biases, at::IntArrayRef acts,
                          bool out_f32) {
  return MLPChainFunction::apply(x, weights, biases, acts, out_f32);
}

// ---------------------------------------------------------------- elementwise activation (QuickGELU / GELU)
Tensor activation_impl(const Tensor& x_, const Tensor& dy_, int64_t act) {
  on_gpu(x_, "x");
  TORCH_CHECK(act == LTHM_ACT_GELU || act == LTHM_ACT_QGELU, "activation: act must be GELU (1) or QuickGELU (2)");
  auto x = x_.contiguous();
  Tensor dy = dy_.defined() ? cast_to(dy_.contiguous(), x.scalar_type()) : Tensor();
  auto y = at::empty_like(x);
  hip_ok(lthm_activation(x.data_ptr(), dy.defined() ? dy.data_ptr() : nullptr, y.data_ptr(), dcode(x), x.numel(),
                         (int32_t)act, cur_stream()),
         "lthm_activation");
  return y;
}

Tensor activation_cuda(const Tensor& x, int64_t act) { return activation_impl(x, Tensor(), act); }

class ActivationFunction : public torch::autograd::Function<ActivationFunction> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& x, int64_t act) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->save_for_backward({x});
    ctx->saved_data["act"] = act;
    return activation_impl(x, Tensor(), act);
  }
  static tensor_list backward(AutogradContext* ctx, tensor_list grads) {
    auto x = ctx->get_saved_variables()[0];
    return {activation_impl(x, grads[0], ctx->saved_data["act"].toInt()), Tensor()};
  }
};

Tensor activation_autograd(const Tensor& x, int64_t act) { return ActivationFunction::apply(x, act); }

// ---------------------------------------------------------------- fused item artifact (forward only)
Tensor item_artifact_cuda(const Tensor& ids_, const Tensor& W, int64_t K, int64_t mode, const Tensor& Wm, int64_t Km,
                          const Tensor& W1, const Tensor& b1, const Tensor& w2, const Tensor& b2,
                          at::ScalarType out_dtype) {
  for (auto* t : {&ids_, &W, &Wm, &W1, &b1, &w2, &b2}) on_gpu(*t, "operand");
  TORCH_CHECK(ids_.scalar_type() == at::kLong, "ids must be int64");
  TORCH_CHECK(W.dim() == 2 && Wm.dim() == 2 && W.is_contiguous() && Wm.is_contiguous(), "tables must be contiguous 2-D");
  TORCH_CHECK(Wm.scalar_type() == at::kFloat && W1.scalar_type() == at::kFloat && b1.scalar_type() == at::kFloat &&
                  w2.scalar_type() == at::kFloat && b2.scalar_type() == at::kFloat,
              "mask model tensors must be f32");
  const int64_t Dm = Wm.size(1), H1 = W1.size(0);
  TORCH_CHECK(Dm % 4 == 0 && Dm <= 16 && H1 <= 256 && W1.size(1) == Dm && b1.numel() == H1 && w2.numel() == H1 &&
                  b2.numel() == 1,
              "mask model must be KShift(Dm % 4 == 0, Dm <= 16) -> Linear(Dm, H1 <= 256) -> Linear(H1, 1)");
  TORCH_CHECK(K > 0 && K <= 64 && Km > 0 && Km <= 64, "num_shifts must be in 1..64");
  auto ids = ids_.contiguous();
  const int64_t D = W.size(1);
  auto shape = ids.sizes().vec();
  shape.push_back(D);
  auto out = at::empty(shape, W.options().dtype(out_dtype));
  auto W1c = W1.contiguous(), b1c = b1.contiguous(), w2c = w2.contiguous(), b2c = b2.contiguous();
  hip_ok(lthm_item_artifact_fwd(ids.data_ptr<int64_t>(), ids.numel(), W.data_ptr(), dcode(W), W.size(0), (int32_t)D,
                                (int32_t)K, (int32_t)mode, Wm.data_ptr<float>(), Wm.size(0), (int32_t)Dm, (int32_t)Km,
                                W1c.data_ptr<float>(), b1c.data_ptr<float>(), (int32_t)H1, w2c.data_ptr<float>(),
                                b2c.data_ptr<float>(), out.data_ptr(), dcode(out), cur_stream()),
         "lthm_item_artifact_fwd");
  return out;
}

int64_t abi_version() { return lthm_abi_version(); }
// the include/lthm.h this op library was compiled against (descriptor layouts)
int64_t built_abi_version() { return LTHM_ABI_VERSION; }

}  // namespace

TORCH_LIBRARY(lthm, m) {
  m.def("abi_version() -> int", &abi_version);
  m.def("built_abi_version() -> int", &built_abi_version);
  m.def("kshift(Tensor ids, Tensor weight, int P, int K, int mode, int F=1, ScalarType? out_dtype=None) -> Tensor");
  m.def("kshift_rows(Tensor ids, int P, int K) -> Tensor");
  m.def("gather_pool(Tensor rows, Tensor weight, int mode, ScalarType out_dtype=float) -> Tensor");
  m.def("activation(Tensor x, int act) -> Tensor");
  m.def("mlp_chain(Tensor x, Tensor[] weights, Tensor[] biases, int[] acts, bool out_f32=True) -> Tensor");
  m.def(
      "item_artifact(Tensor ids, Tensor weight, int K, int mode, Tensor mask_weight, int mask_K, Tensor w1, "
      "Tensor b1, Tensor w2, Tensor b2, ScalarType out_dtype=float) -> Tensor");
}

TORCH_LIBRARY_IMPL(lthm, CUDA, m) {
  m.impl("kshift", &kshift_cuda);
  m.impl("kshift_rows", &kshift_rows_cuda);
  m.impl("gather_pool", &gather_pool_cuda);
  m.impl("mlp_chain", &mlp_chain_cuda);
  m.impl("activation", &activation_cuda);
  m.impl("item_artifact", &item_artifact_cuda);
}

TORCH_LIBRARY_IMPL(lthm, Autograd, m) {
  m.impl("kshift", &kshift_autograd);
  m.impl("mlp_chain", &mlp_chain_autograd);
  m.impl("activation", &activation_autograd);
}

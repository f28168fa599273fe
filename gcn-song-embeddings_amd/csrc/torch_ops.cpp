// PyTorch-ROCm operator library (libpinsage_torch.so): the hot path's ops as
// torch.ops.pinsage.* (TORCH_LIBRARY schemas, HIP dispatch key), each a thin
// call into libpinsage_hip.so's C-ABI on the current HIP stream of the
// tensors' device.  Tensors are torch-owned (caching allocator), device inputs
// must be contiguous, every op returns fresh tensors and raises RuntimeError
// (TORCH_CHECK) with the library's message on failure.  Autograd formulas for
// the differentiable ops are registered from Python (pinsage_ops.py,
// torch.library.register_autograd) on the *_backward ops defined here.
//
// SURVEY.md §8(b2) schema set:
//   ppr_topk      sample_neighborhood_topt (pinsage_model.py:88-107), fused walk + count + top-k
//   frontier      relevant_nodes_per_layer_precomp's unique step (pinsage_model.py:166)
//   linear        nn.Linear on gathered rows (+ LeakyReLU), pinsage_model.py:196-201, 209
//   weighted_agg  (w[:, :, None] * q).sum(1) / w.sum(1), pinsage_model.py:202
//   gemm          the backward products (dW = dY^T X, dX = dY W), any operand layout
//   segment_wmean the transposed aggregation (and lib/gnns MEAN, GNNs_unsupervised.py:537-588)
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/pinsage_hip.h"

namespace {

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "pinsage::", what, ": ", pinsage_last_error());
}

void* stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// (w f64 [n, k], nodes i64 [n, k]) of the sources' top-k PPR neighbours, Philox
// stream (seed, absolute source position src_base + i)
std::tuple<at::Tensor, at::Tensor> ppr_topk(const at::Tensor& indptr, const at::Tensor& indices,
                                            const at::Tensor& sources, int64_t n_hops, double alpha,
                                            int64_t k, int64_t seed, int64_t src_base) {
  need(indptr, at::kLong, "indptr");
  need(indices, at::kInt, "indices");
  need(sources, at::kLong, "sources");
  c10::hip::HIPGuard guard(sources.device().index());
  const int64_t n = sources.numel(), n_all = indptr.numel() - 1;
  auto w = at::empty({n, k}, sources.options().dtype(at::kDouble));
  auto nb = at::empty({n, k}, sources.options().dtype(at::kLong));
  if (n == 0) return {w, nb};
  const int64_t need_ws = pinsage_ppr_topk_workspace(n, n_hops, 0);
  auto ws = at::empty({std::min<int64_t>(need_ws, int64_t(1) << 30)}, sources.options().dtype(at::kByte));
  check(pinsage_ppr_topk(indptr.data_ptr<int64_t>(), indices.data_ptr<int32_t>(), n_all,
                         sources.data_ptr<int64_t>(), n, n_hops, (float)alpha, k, nullptr, (uint64_t)seed, 0,
                         src_base, ws.data_ptr(), ws.numel(), w.data_ptr<double>(), nb.data_ptr<int64_t>(),
                         nullptr, nullptr, 0, stream_of(sources)),
        "ppr_topk");
  return {w, nb};
}

// sorted unique(cat(nb[nodeset, :T].flatten(), nodeset)) as int64
at::Tensor frontier(const at::Tensor& nodeset, const at::Tensor& nb_table, int64_t T, int64_t n_items) {
  need(nodeset, at::kLong, "nodeset");
  need(nb_table, at::kInt, "nb_table");
  c10::hip::HIPGuard guard(nodeset.device().index());
  const int64_t n = nodeset.numel();
  auto ws = at::empty({pinsage_frontier_workspace(n_items)}, nodeset.options().dtype(at::kByte));
  auto out = at::empty({std::max<int64_t>(1, std::min(n_items, n * (T + 1)))}, nodeset.options().dtype(at::kInt));
  auto cnt = at::zeros({1}, nodeset.options().dtype(at::kInt));
  check(pinsage_frontier_step(nodeset.data_ptr<int64_t>(), n, nb_table.data_ptr<int32_t>(), nb_table.size(1), T,
                              n_items, ws.data_ptr(), out.data_ptr<int32_t>(), cnt.data_ptr<int32_t>(),
                              stream_of(nodeset)),
        "frontier");
  return out.narrow(0, 0, cnt.item<int32_t>()).to(at::kLong);
}

// y = x[rows] W^T (+ b) (LeakyReLU 0.01 if lrelu); rows int32 or none
at::Tensor linear(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const at::Tensor& W,
                  const c10::optional<at::Tensor>& b, bool lrelu) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.stride(1) == 1, "x: f32 device rows");
  need(W, at::kFloat, "W");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t K = W.size(1), N = W.size(0);
  TORCH_CHECK(x.size(1) >= K, "x narrower than W's in_features");
  const int32_t* idx = nullptr;
  int64_t M = x.size(0);
  if (rows.has_value()) {
    need(*rows, at::kInt, "rows");
    idx = rows->data_ptr<int32_t>();
    M = rows->numel();
  }
  const float* bias = nullptr;
  if (b.has_value()) {
    need(*b, at::kFloat, "b");
    bias = b->data_ptr<float>();
  }
  auto y = at::empty({M, N}, x.options());
  if (M == 0) return y;
  check(pinsage_linear(x.data_ptr<float>(), x.stride(0), idx, M, K, W.data_ptr<float>(), bias, N, lrelu ? 1 : 0,
                       y.data_ptr<float>(), N, stream_of(x)),
        "linear");
  return y;
}

// C [M][N] = op(A) op(B): a_kmajor: A [M][K] (rows gathered by a_idx) else [K][M];
// b_kmajor: B [N][K] else [K][N] (k-rows gathered by b_idx)
at::Tensor gemm(const at::Tensor& A, bool a_kmajor, const c10::optional<at::Tensor>& a_idx, const at::Tensor& B,
                bool b_kmajor, const c10::optional<at::Tensor>& b_idx, int64_t M, int64_t N, int64_t K) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && A.stride(1) == 1, "A: f32 device rows");
  TORCH_CHECK(B.is_cuda() && B.scalar_type() == at::kFloat && B.stride(1) == 1, "B: f32 device rows");
  c10::hip::HIPGuard guard(A.device().index());
  const int32_t* ai = nullptr;
  const int32_t* bi = nullptr;
  if (a_idx.has_value()) {
    need(*a_idx, at::kInt, "a_idx");
    ai = a_idx->data_ptr<int32_t>();
  }
  if (b_idx.has_value()) {
    need(*b_idx, at::kInt, "b_idx");
    bi = b_idx->data_ptr<int32_t>();
  }
  auto C = at::empty({M, N}, A.options());
  if (M == 0) return C;
  if (K == 0) return C.zero_();
  check(pinsage_gemm_ex(M, N, K, a_kmajor ? 1 : 0, b_kmajor ? 1 : 0, A.data_ptr<float>(), A.stride(0), ai,
                        B.data_ptr<float>(), B.stride(0), bi, C.data_ptr<float>(), N, nullptr, 0, 0, 1, -1, 0,
                        stream_of(A)),
        "gemm");
  return C;
}

// agg[f] = sum_t w[f][t] q[loc[f][t]]  (w already normalised)
at::Tensor weighted_agg(const at::Tensor& q, const at::Tensor& loc, const at::Tensor& w) {
  need(q, at::kFloat, "q");
  need(loc, at::kInt, "loc");
  need(w, at::kFloat, "w");
  TORCH_CHECK(loc.sizes() == w.sizes() && loc.dim() == 2, "loc and w: [n, T]");
  c10::hip::HIPGuard guard(q.device().index());
  const int64_t n = loc.size(0), T = loc.size(1), hid = q.size(1);
  auto agg = at::empty({n, hid}, q.options());
  if (n == 0) return agg;
  check(pinsage_weighted_agg(q.data_ptr<float>(), hid, loc.data_ptr<int32_t>(), w.data_ptr<float>(), n, T,
                             agg.data_ptr<float>(), stream_of(q)),
        "weighted_agg");
  return agg;
}

// out[i] = sum_{j in [seg[i], seg[i+1])} w[j] h[cols[j]]  (/ sum |w| if normalize)
at::Tensor segment_wmean(const at::Tensor& h, const at::Tensor& seg, const at::Tensor& cols, const at::Tensor& w,
                         bool normalize) {
  TORCH_CHECK(h.is_cuda() && h.scalar_type() == at::kFloat && h.stride(1) == 1, "h: f32 device rows");
  need(seg, at::kLong, "seg");
  need(cols, at::kInt, "cols");
  need(w, at::kFloat, "w");
  c10::hip::HIPGuard guard(h.device().index());
  const int64_t n_seg = seg.numel() - 1, d = h.size(1);
  auto out = at::empty({n_seg, d}, h.options());
  if (n_seg <= 0) return out;
  check(pinsage_segment_wmean(h.data_ptr<float>(), h.stride(0), h.size(0), d, seg.data_ptr<int64_t>(),
                              cols.data_ptr<int32_t>(), w.data_ptr<float>(), n_seg, normalize ? 1 : 0,
                              out.data_ptr<float>(), d, stream_of(h)),
        "segment_wmean");
  return out;
}

// d q of weighted_agg: dq[u] = sum over the slots (f, t) with loc = u of w[f][t] dagg[f]
at::Tensor weighted_agg_backward(const at::Tensor& dagg, const at::Tensor& loc, const at::Tensor& w,
                                 int64_t n_q) {
  need(loc, at::kInt, "loc");
  need(w, at::kFloat, "w");
  const int64_t T = loc.size(1);
  auto flat = loc.reshape({-1}).to(at::kLong);
  auto order = std::get<1>(at::sort(flat, /*stable=*/true, 0, false));
  auto seg = at::zeros({n_q + 1}, flat.options());
  seg.narrow(0, 1, n_q).copy_(at::cumsum(at::bincount(flat, {}, n_q), 0));
  auto rows = at::floor_divide(order, T).to(at::kInt).contiguous();
  auto wT = w.reshape({-1}).index_select(0, order).contiguous();
  return segment_wmean(dagg.contiguous(), seg, rows, wT, false);
}

}  // namespace

TORCH_LIBRARY(pinsage, m) {
  m.def("ppr_topk(Tensor indptr, Tensor indices, Tensor sources, int n_hops, float alpha, int k, int seed, "
        "int src_base=0) -> (Tensor, Tensor)");
  m.def("frontier(Tensor nodeset, Tensor nb_table, int T, int n_items) -> Tensor");
  m.def("linear(Tensor x, Tensor? rows, Tensor W, Tensor? b, bool lrelu) -> Tensor");
  m.def("gemm(Tensor A, bool a_kmajor, Tensor? a_idx, Tensor B, bool b_kmajor, Tensor? b_idx, int M, int N, "
        "int K) -> Tensor");
  m.def("weighted_agg(Tensor q, Tensor loc, Tensor w) -> Tensor");
  m.def("weighted_agg_backward(Tensor dagg, Tensor loc, Tensor w, int n_q) -> Tensor");
  m.def("segment_wmean(Tensor h, Tensor seg, Tensor cols, Tensor w, bool normalize) -> Tensor");
}

TORCH_LIBRARY_IMPL(pinsage, CUDA, m) {
  m.impl("ppr_topk", &ppr_topk);
  m.impl("frontier", &frontier);
  m.impl("linear", &linear);
  m.impl("gemm", &gemm);
  m.impl("weighted_agg", &weighted_agg);
  m.impl("weighted_agg_backward", &weighted_agg_backward);
  m.impl("segment_wmean", &segment_wmean);
}

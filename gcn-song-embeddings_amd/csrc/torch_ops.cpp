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
//   walk          do_random_walks (pinsage_model.py:32-53), MT19937 (torch's generator) or Philox draws
//   ppr_topk      sample_neighborhood_topt (pinsage_model.py:88-107), fused walk + count + top-k
//   frontier      relevant_nodes_per_layer_precomp's unique step (pinsage_model.py:166)
//   linear        nn.Linear on gathered rows (+ LeakyReLU), pinsage_model.py:196-201, 209
//   weighted_agg  (w[:, :, None] * q).sum(1) / w.sum(1), pinsage_model.py:202
//   gemm          the backward products (dW = dY^T X, dX = dY W), any operand layout
//   segment_wmean the transposed aggregation (and lib/gnns MEAN, GNNs_unsupervised.py:537-588)
//   gather_rows / scatter_add_rows   get_embeddings' gather and its gradient (pinsage_model.py:21-23)
//   concat_linear_lrelu_l2norm (+ norm_lrelu_backward)   the W projection (pinsage_model.py:208-210)
#include <ATen/ATen.h>
#include <ATen/core/Generator.h>
#include <ATen/CPUGeneratorImpl.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <mutex>
#include <string>
#include <vector>

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

// The reference's global generator (torch.manual_seed / torch.get_rng_state:
// do_random_walks draws from it, pinsage_model.py:38-48) as a library MT19937
// state: loaded before an MT19937-mode call, written back after it.
struct TorchRng {
  at::Generator gen = at::detail::getDefaultCPUGenerator();
  std::lock_guard<std::mutex> lock{gen.mutex()};
  at::Tensor state = gen.get_state();
  std::vector<uint8_t> mt = std::vector<uint8_t>((size_t)pinsage_mt_state_bytes());
  TorchRng() {
    check(pinsage_mt_from_torch(mt.data(), state.data_ptr<uint8_t>(), state.numel()), "rng state");
  }
  void commit() {
    check(pinsage_mt_to_torch(mt.data(), state.data_ptr<uint8_t>(), state.numel()), "rng state");
    gen.set_state(state);
  }
};

bool mt_mode(const std::string& rng_mode) {
  TORCH_CHECK(rng_mode == "philox" || rng_mode == "mt19937", "rng_mode must be 'philox' or 'mt19937', got '",
              rng_mode, "'");
  return rng_mode == "mt19937";
}

void check_csr(const at::Tensor& indptr, const at::Tensor& indices, const at::Tensor& sources, bool mt) {
  need(indptr, at::kLong, "indptr");
  need(indices, at::kInt, "indices");
  need(sources, at::kLong, "sources");
  if (mt && indptr.numel() > 1) {  // torch.randint(n) draws two words from n >= 2^28 on: not restated
    const int64_t maxdeg = (indptr.narrow(0, 1, indptr.numel() - 1) - indptr.narrow(0, 0, indptr.numel() - 1))
                               .max()
                               .item<int64_t>();
    TORCH_CHECK(maxdeg < (int64_t(1) << 28), "degree >= 2^28: use rng_mode 'philox'");
  }
}

// int32 trace [n, n_hops] of do_random_walks (pinsage_model.py:32-53) on the device
at::Tensor walk_i32(const at::Tensor& indptr, const at::Tensor& indices, const at::Tensor& sources, int64_t n_hops,
                    double alpha, int64_t seed, int64_t offset, bool mt, int64_t src_base) {
  const int64_t n = sources.numel(), n_all = indptr.numel() - 1;
  auto trace = at::empty({n, n_hops}, sources.options().dtype(at::kInt));
  if (n == 0) return trace;
  if (mt) {
    const int64_t need_ws = pinsage_walk_mt_workspace(n, n_hops);
    auto ws = at::empty({std::min<int64_t>(need_ws, int64_t(2) << 30)}, sources.options().dtype(at::kByte));
    TorchRng rng;
    check(pinsage_walk_mt(indptr.data_ptr<int64_t>(), indices.data_ptr<int32_t>(), n_all,
                          sources.data_ptr<int64_t>(), n, n_hops, (float)alpha, rng.mt.data(), ws.data_ptr(),
                          ws.numel(), trace.data_ptr<int32_t>(), stream_of(sources)),
          "walk");
    rng.commit();
  } else {
    check(pinsage_walk_philox(indptr.data_ptr<int64_t>(), indices.data_ptr<int32_t>(), n_all,
                              sources.data_ptr<int64_t>(), n, n_hops, (float)alpha, (uint64_t)seed,
                              (uint32_t)offset, src_base, trace.data_ptr<int32_t>(), stream_of(sources)),
          "walk");
  }
  return trace;
}

// do_random_walks (pinsage_model.py:32-53): int64 trace [n, n_hops].
// rng_mode "mt19937": the reference's own draws from torch's global generator
// (3 words per hop, advanced exactly as the reference advances it); "philox":
// counter-based draws keyed by (seed, hop, src_base + i, offset), torch's
// generator untouched.
at::Tensor walk(const at::Tensor& indptr, const at::Tensor& indices, const at::Tensor& sources, int64_t n_hops,
                double alpha, int64_t seed, int64_t offset, const std::string& rng_mode, int64_t src_base) {
  const bool mt = mt_mode(rng_mode);
  check_csr(indptr, indices, sources, mt);
  TORCH_CHECK(n_hops > 0, "n_hops must be positive");
  c10::hip::HIPGuard guard(sources.device().index());
  return walk_i32(indptr, indices, sources, n_hops, alpha, seed, offset, mt, src_base).to(at::kLong);
}

// (w f64 [n, k], nodes i64 [n, k]) = visit_prob.topk(k, 1) of each source's
// walks (sample_neighborhood_topt, pinsage_model.py:88-107), libstdc++ tie
// order; rng_mode / seed / offset / src_base as in walk.  The partial_sort
// regime runs the fused walk + heap-select kernels (the trace never reaches
// HBM); tiny graphs (k * 64 > N_all, torch's nth_element regime) the walk +
// visit_topk kernels.
std::tuple<at::Tensor, at::Tensor> ppr_topk(const at::Tensor& indptr, const at::Tensor& indices,
                                            const at::Tensor& sources, int64_t n_hops, double alpha,
                                            int64_t k, int64_t seed, int64_t src_base, int64_t offset,
                                            const std::string& rng_mode) {
  const bool mt = mt_mode(rng_mode);
  check_csr(indptr, indices, sources, mt);
  TORCH_CHECK(n_hops > 0, "n_hops must be positive");
  c10::hip::HIPGuard guard(sources.device().index());
  const int64_t n = sources.numel(), n_all = indptr.numel() - 1;
  TORCH_CHECK(k >= 1 && k <= n_all, "selected index k out of range");
  auto w = at::empty({n, k}, sources.options().dtype(at::kDouble));
  auto nb = at::empty({n, k}, sources.options().dtype(at::kLong));
  if (n == 0) return {w, nb};
  if (k * 64 > n_all || n_hops + k >= 65536 || n_hops > 8192) {
    auto trace = walk_i32(indptr, indices, sources, n_hops, alpha, seed, offset, mt, src_base);
    const int64_t sb = pinsage_visit_topk_scratch(n, n_all, k);
    auto scratch = at::empty({std::max<int64_t>(sb, 1)}, sources.options().dtype(at::kByte));
    check(pinsage_visit_topk(trace.data_ptr<int32_t>(), sources.data_ptr<int64_t>(), n, n_hops, n_all, k,
                             sb ? scratch.data_ptr() : nullptr, w.data_ptr<double>(), nb.data_ptr<int64_t>(),
                             nullptr, nullptr, 0, stream_of(sources)),
          "ppr_topk");
    return {w, nb};
  }
  const int64_t need_ws = pinsage_ppr_topk_workspace(n, n_hops, mt ? 1 : 0);
  auto ws = at::empty({std::min<int64_t>(need_ws, int64_t(1) << 30)}, sources.options().dtype(at::kByte));
  auto run = [&](void* mtp) {
    check(pinsage_ppr_topk(indptr.data_ptr<int64_t>(), indices.data_ptr<int32_t>(), n_all,
                           sources.data_ptr<int64_t>(), n, n_hops, (float)alpha, k, mtp, (uint64_t)seed,
                           (uint32_t)offset, src_base, ws.data_ptr(), ws.numel(), w.data_ptr<double>(),
                           nb.data_ptr<int64_t>(), nullptr, nullptr, 0, stream_of(sources)),
          "ppr_topk");
  };
  if (mt) {
    TorchRng rng;
    run(rng.mt.data());
    rng.commit();
  } else {
    run(nullptr);
  }
  return {w, nb};
}

// One step of relevant_nodes_per_layer_precomp (pinsage_model.py:162-166):
// (uniq, local_idx) with uniq = sorted unique(cat(nb[nodeset, :T].flatten(),
// nodeset)) int64 and local_idx int32 [n, T], uniq[local_idx[f][t]] ==
// nb[nodeset[f]][t] (weighted_agg's slot rows).  nb_table int64 (the
// reference's table, precompute_neighborhoods_topt) or int32 [n_items][>= T];
// n_items -1 = nb_table's rows.
std::tuple<at::Tensor, at::Tensor> frontier(const at::Tensor& nodeset, const at::Tensor& nb_table, int64_t T,
                                            int64_t n_items) {
  need(nodeset, at::kLong, "nodeset");
  TORCH_CHECK(nb_table.is_cuda() && nb_table.dim() == 2 &&
                  (nb_table.scalar_type() == at::kLong || nb_table.scalar_type() == at::kInt),
              "nb_table: int64 or int32 device [n_items, >= T]");
  TORCH_CHECK(T >= 1 && T <= nb_table.size(1), "T must be in [1, nb_table columns]");
  c10::hip::HIPGuard guard(nodeset.device().index());
  if (n_items < 0) n_items = nb_table.size(0);
  TORCH_CHECK(n_items >= 1 && n_items <= nb_table.size(0), "n_items must be in [1, nb_table rows]");
  // (the kernels read 32-bit node ids; an int64 table narrows once, on the device)
  const at::Tensor nb32 = nb_table.scalar_type() == at::kInt ? nb_table.contiguous()
                                                              : nb_table.narrow(1, 0, T).to(at::kInt).contiguous();
  const int64_t n = nodeset.numel();
  auto ws = at::empty({pinsage_frontier_workspace(n_items)}, nodeset.options().dtype(at::kByte));
  auto out = at::empty({std::max<int64_t>(1, std::min(n_items, n * (T + 1)))}, nodeset.options().dtype(at::kInt));
  auto cnt = at::zeros({1}, nodeset.options().dtype(at::kInt));
  auto local_idx = at::empty({n, T}, nodeset.options().dtype(at::kInt));
  check(pinsage_frontier_step(nodeset.data_ptr<int64_t>(), n, nb32.data_ptr<int32_t>(), nb32.size(1), T, n_items,
                              ws.data_ptr(), out.data_ptr<int32_t>(), cnt.data_ptr<int32_t>(), stream_of(nodeset)),
        "frontier");
  check(pinsage_frontier_local_idx(nodeset.data_ptr<int64_t>(), n, nb32.data_ptr<int32_t>(), nb32.size(1), T,
                                   n_items, ws.data_ptr(), local_idx.data_ptr<int32_t>(), stream_of(nodeset)),
        "frontier");
  return {out.narrow(0, 0, cnt.item<int32_t>()).to(at::kLong), local_idx};
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

// get_embeddings (pinsage_model.py:21-23): h[idx, :width] (width -1 = all columns)
at::Tensor gather_rows(const at::Tensor& h, const at::Tensor& idx, int64_t width) {
  TORCH_CHECK(h.is_cuda() && h.scalar_type() == at::kFloat && h.dim() == 2 && h.stride(1) == 1,
              "h: f32 device rows");
  need(idx, at::kLong, "idx");
  c10::hip::HIPGuard guard(h.device().index());
  const int64_t d = width < 0 ? h.size(1) : width, n = idx.numel();
  TORCH_CHECK(d <= h.size(1), "width exceeds h's columns");
  auto out = at::empty({n, d}, h.options());
  if (n == 0) return out;
  const auto mm = at::aminmax(idx);
  TORCH_CHECK_INDEX(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < h.size(0),
                    "gather_rows: index out of range for h with ", h.size(0), " rows");
  check(pinsage_gather_rows(h.data_ptr<float>(), h.stride(0), h.size(0), d, idx.data_ptr<int64_t>(), n,
                            out.data_ptr<float>(), d, stream_of(h)),
        "gather_rows");
  return out;
}

// the transpose of gather_rows: out [n_rows, width] = 0; out[idx[i], :d] += grad[i]
// (index_add, as get_embeddings' backward), summed in position order per row
// (deterministic: the CSR of idx and one segmented sum, no float atomics)
at::Tensor scatter_add_rows(const at::Tensor& grad, const at::Tensor& idx, int64_t n_rows, int64_t width) {
  TORCH_CHECK(grad.is_cuda() && grad.scalar_type() == at::kFloat && grad.dim() == 2, "grad: f32 device rows");
  need(idx, at::kLong, "idx");
  TORCH_CHECK(idx.numel() == grad.size(0), "idx and grad rows differ");
  c10::hip::HIPGuard guard(grad.device().index());
  const int64_t d = grad.size(1), w = width < 0 ? d : width;
  TORCH_CHECK(w >= d, "width narrower than grad");
  auto out = at::zeros({n_rows, w}, grad.options());
  if (idx.numel() == 0 || n_rows == 0) return out;
  const auto mm = at::aminmax(idx);
  TORCH_CHECK_INDEX(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < n_rows,
                    "scatter_add_rows: index out of range for ", n_rows, " rows");
  auto order = std::get<1>(at::sort(idx, /*stable=*/true, 0, false));
  auto seg = at::zeros({n_rows + 1}, idx.options());
  seg.narrow(0, 1, n_rows).copy_(at::cumsum(at::bincount(idx, {}, n_rows), 0));
  auto cols = order.to(at::kInt).contiguous();
  auto ones = at::ones({idx.numel()}, grad.options());
  auto g = grad.contiguous();
  check(pinsage_segment_wmean(g.data_ptr<float>(), d, g.size(0), d, seg.data_ptr<int64_t>(),
                              cols.data_ptr<int32_t>(), ones.data_ptr<float>(), n_rows, 0, out.data_ptr<float>(),
                              w, stream_of(g)),
        "scatter_add_rows");
  return out;
}

// ConvLayer's W projection (pinsage_model.py:208-210): (y, norms) with
// y = normalize(lrelu([h[self_rows, :d] || agg] W^T + b)), d = W.size(1) - agg.size(1)
std::tuple<at::Tensor, at::Tensor> concat_linear_lrelu_l2norm(const at::Tensor& h,
                                                              const c10::optional<at::Tensor>& self_rows,
                                                              const at::Tensor& agg, const at::Tensor& W,
                                                              const at::Tensor& b) {
  TORCH_CHECK(h.is_cuda() && h.scalar_type() == at::kFloat && h.dim() == 2 && h.stride(1) == 1,
              "h: f32 device rows");
  TORCH_CHECK(agg.is_cuda() && agg.scalar_type() == at::kFloat && agg.dim() == 2 && agg.stride(1) == 1,
              "agg: f32 device rows");
  need(W, at::kFloat, "W");
  need(b, at::kFloat, "b");
  c10::hip::HIPGuard guard(h.device().index());
  const int64_t n = agg.size(0), hid = agg.size(1), out = W.size(0), d = W.size(1) - hid;
  TORCH_CHECK(d > 0 && d <= h.size(1), "W's in_features must be h's d + agg's width");
  TORCH_CHECK(b.numel() == out, "b: [out]");
  at::Tensor rows32;
  if (self_rows.has_value()) {
    need(*self_rows, at::kLong, "self_rows");
    TORCH_CHECK(self_rows->numel() == n, "self_rows and agg rows differ");
    if (n) {
      const auto mm = at::aminmax(*self_rows);
      TORCH_CHECK_INDEX(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < h.size(0),
                        "self_rows out of range of h");
    }
    rows32 = self_rows->to(at::kInt).contiguous();
  } else {
    TORCH_CHECK(h.size(0) >= n, "h has fewer rows than agg");
  }
  auto y = at::empty({n, out}, h.options());
  auto norms = at::empty({n}, h.options());
  if (n == 0) return {y, norms};
  check(pinsage_concat_linear_l2norm(h.data_ptr<float>(), h.stride(0),
                                     rows32.defined() ? rows32.data_ptr<int32_t>() : nullptr, n, d,
                                     agg.data_ptr<float>(), agg.stride(0), hid, W.data_ptr<float>(),
                                     b.data_ptr<float>(), out, y.data_ptr<float>(), norms.data_ptr<float>(),
                                     stream_of(h)),
        "concat_linear_lrelu_l2norm");
  return {y, norms};
}

// dp of y = lrelu(p) / ||lrelu(p)||
at::Tensor norm_lrelu_backward(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& norms) {
  need(y, at::kFloat, "y");
  need(norms, at::kFloat, "norms");
  TORCH_CHECK(dy.sizes() == y.sizes() && y.dim() == 2 && norms.numel() == y.size(0), "dy, y: [n, out]; norms: [n]");
  c10::hip::HIPGuard guard(y.device().index());
  auto g = dy.contiguous();
  auto dp = at::empty_like(y);
  if (y.size(0) == 0) return dp;
  check(pinsage_norm_lrelu_backward(y.data_ptr<float>(), norms.data_ptr<float>(), g.data_ptr<float>(), y.size(0),
                                    y.size(1), dp.data_ptr<float>(), stream_of(y)),
        "norm_lrelu_backward");
  return dp;
}

}  // namespace

TORCH_LIBRARY(pinsage, m) {
  // rng_mode defaults to the reference's own stream (do_random_walks draws
  // from torch's global MT19937 generator, pinsage_model.py:32-53)
  m.def("walk(Tensor indptr, Tensor indices, Tensor sources, int n_hops, float alpha, int seed=0, int offset=0, "
        "str rng_mode='mt19937', int src_base=0) -> Tensor");
  m.def("ppr_topk(Tensor indptr, Tensor indices, Tensor sources, int n_hops, float alpha, int k, int seed=0, "
        "int src_base=0, int offset=0, str rng_mode='mt19937') -> (Tensor, Tensor)");
  m.def("frontier(Tensor nodeset, Tensor nb_table, int T, int n_items=-1) -> (Tensor, Tensor)");
  m.def("linear(Tensor x, Tensor? rows, Tensor W, Tensor? b, bool lrelu) -> Tensor");
  m.def("gemm(Tensor A, bool a_kmajor, Tensor? a_idx, Tensor B, bool b_kmajor, Tensor? b_idx, int M, int N, "
        "int K) -> Tensor");
  m.def("weighted_agg(Tensor q, Tensor loc, Tensor w) -> Tensor");
  m.def("weighted_agg_backward(Tensor dagg, Tensor loc, Tensor w, int n_q) -> Tensor");
  m.def("segment_wmean(Tensor h, Tensor seg, Tensor cols, Tensor w, bool normalize) -> Tensor");
  m.def("gather_rows(Tensor h, Tensor idx, int width=-1) -> Tensor");
  m.def("scatter_add_rows(Tensor grad, Tensor idx, int n_rows, int width=-1) -> Tensor");
  m.def("concat_linear_lrelu_l2norm(Tensor h, Tensor? self_rows, Tensor agg, Tensor W, Tensor b) -> (Tensor, Tensor)");
  m.def("norm_lrelu_backward(Tensor dy, Tensor y, Tensor norms) -> Tensor");
}

TORCH_LIBRARY_IMPL(pinsage, CUDA, m) {
  m.impl("walk", &walk);
  m.impl("ppr_topk", &ppr_topk);
  m.impl("frontier", &frontier);
  m.impl("linear", &linear);
  m.impl("gemm", &gemm);
  m.impl("weighted_agg", &weighted_agg);
  m.impl("weighted_agg_backward", &weighted_agg_backward);
  m.impl("segment_wmean", &segment_wmean);
  m.impl("gather_rows", &gather_rows);
  m.impl("scatter_add_rows", &scatter_add_rows);
  m.impl("concat_linear_lrelu_l2norm", &concat_linear_lrelu_l2norm);
  m.impl("norm_lrelu_backward", &norm_lrelu_backward);
}

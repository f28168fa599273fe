/*
 * pinsage_hip.h -- C-ABI of the MI355X (gfx950) PinSage convolution engine.
 *
 * The reference (MatejBevec/gcn-song-embeddings) is pure Python; its train-step
 * path calls into DGL (g.successors) and ATen CPU ops.  These entry points are
 * what a maintainer binds (ctypes stub in INTEGRATION.md) to replace those
 * call sites.  Plain pointers and sizes only; every device pointer is HIP
 * device memory (e.g. a torch tensor's data_ptr()), every `stream` a
 * hipStream_t.  Functions return 0 on success or a negative pinsage_status;
 * pinsage_last_error() gives the message of the calling thread's last failure.
 * No call synchronises the stream unless its comment says so.
 */
#ifndef PINSAGE_HIP_H
#define PINSAGE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum pinsage_status {
  PINSAGE_OK = 0,
  PINSAGE_ERR_HIP = -1,
  PINSAGE_ERR_ARG = -2,
  PINSAGE_ERR_WORKSPACE = -3,
  PINSAGE_ERR_GRAPH = -4, /* zero-degree node met by a walk (reference: torch.randint(0) raises) */
  PINSAGE_ERR_INDEX = -5, /* id out of range (reference: IndexError in h[nodeset]) */
};

/* ------------------------------------------------------------------ library */
int pinsage_version(void);
const char* pinsage_last_error(void);
/* number of visible HIP devices (0 when none); never fails */
int pinsage_device_count(void);

/* ------------------------------------------------------------------ RNG (host, no GPU needed)
 * Opaque MT19937 state with torch's CPU-generator semantics.  Replaces the
 * global generator the reference draws from in pinsage_model.py:42,45,50 and
 * pinsage_training.py:58,74 (torch.randint / torch.rand / torch.randperm).
 * torch_state is torch.get_rng_state() (5056 bytes). */
int pinsage_mt_state_bytes(void);
int pinsage_mt_from_torch(void* mt, const uint8_t* torch_state, int64_t nbytes);
int pinsage_mt_to_torch(const void* mt, uint8_t* torch_state, int64_t nbytes);
int pinsage_mt_seed(void* mt, uint64_t seed);
int pinsage_mt_skip(void* mt, int64_t n_draws);
int pinsage_mt_draws(void* mt, uint32_t* out, int64_t n);
/* torch.randperm(n)[:k] (pinsage_training.py:58,74): writes the first k entries
 * of the Fisher-Yates permutation and advances mt by the full n-1 draws. */
int pinsage_mt_randperm_prefix(void* mt, int64_t n, int64_t k, int64_t* out);

/* sample_batch with easy negatives (pinsage_training.py:53-77, 89-97) on the
 * host: positives is [P][2] int64, batch_out is [B][3] int64 (query, positive,
 * negative).  Consumes exactly the draws the reference does.  nodeset_out
 * (nullable, capacity 3B) receives batch.flatten().unique() (sorted), its
 * length in *n_nodeset. */
int pinsage_sample_batch_easy(void* mt, const int64_t* positives, int64_t n_pos_pairs,
                              int64_t n_items, int64_t batch_size, int64_t* batch_out,
                              int64_t* nodeset_out, int64_t* n_nodeset);

/* Batch sampler runtime (native data loader for PinSage.train's batch loop).
 * Holds positives [P][2] int64 (must stay alive and unchanged) and draws the
 * batch that the torch CPU generator state `state` (torch.get_rng_state()
 * bytes) yields: batch_out [B][3], nodeset_out (nullable, capacity 3B) =
 * batch.flatten().unique(), state_after = the generator state after the
 * reference's draws.  With speculate != 0 the batch starting at state_after is
 * drawn next on a worker thread and used by the next call iff its state is
 * byte-identical -- results are always exactly pinsage_sample_batch_easy's.
 * Returns 1 when the speculative draw was used, 0 when drawn synchronously. */
typedef struct pinsage_batch_sampler pinsage_batch_sampler;
int pinsage_batch_sampler_create(const int64_t* positives, int64_t n_pos_pairs, int64_t n_items,
                                 int64_t batch_size, pinsage_batch_sampler** out);
void pinsage_batch_sampler_destroy(pinsage_batch_sampler* s);
int pinsage_batch_sampler_next(pinsage_batch_sampler* s, const uint8_t* state, int64_t nbytes,
                               int64_t* batch_out, int64_t* nodeset_out, int64_t* n_nodeset,
                               uint8_t* state_after, int speculate);
/* The batch the worker drew speculatively for the NEXT request (from the
 * generator state the last pinsage_batch_sampler_next handed back), without
 * consuming it: waits for the worker, copies rows x 3 int64 ids into
 * batch_out and returns rows (0 if there is no finished draw or it exceeds
 * max_rows).  The next request still verifies its start state; a caller that
 * acts on a peeked batch (the trainer computes that batch's frontier ahead)
 * must compare it with the batch it is finally given. */
int pinsage_batch_sampler_peek(pinsage_batch_sampler* h, int64_t* batch_out, int64_t max_rows);

/* ------------------------------------------------------------------ sampler (device)
 * do_random_walks (pinsage_model.py:32-53).  CSR: indptr int64 [n_all+1],
 * indices int32 [E], successors in edge-insertion order (DGL g.successors,
 * pinsage_model.py:41,44).  sources int64 [n_src], trace int32 [n_src][n_hops].
 *
 * MT mode: `mt` (host state) is advanced by exactly 3*n_hops*n_src draws, as
 * the reference consumes.  `ws` is device scratch of pinsage_walk_mt_workspace
 * bytes (the raw MT words of one round of sources; smaller workspaces run in
 * more rounds).  Synchronises the stream (host prepares each round's chunk
 * states while the previous round runs). */
int64_t pinsage_walk_mt_workspace(int64_t n_src, int64_t n_hops);
int pinsage_walk_mt(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                    const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha, void* mt,
                    void* ws, int64_t ws_bytes, int32_t* trace, void* stream);
/* Philox mode: draws for (source position src_base+i, hop j) = Philox4x32-10
 * (key=seed, counter={j, pos_lo, pos_hi, offset}).  Synchronises the stream to
 * check for zero-degree nodes. */
int pinsage_walk_philox(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                        const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha,
                        uint64_t seed, uint32_t offset, int64_t src_base, int32_t* trace,
                        void* stream);

/* visit_prob.topk(k, 1) on the walks (pinsage_model.py:96-107): counts visits
 * per source, zeroes the source's own column, selects the top k with the exact
 * libstdc++ tie order of torch's CPU topk.  Outputs (any may be null):
 *   w_out f64 [n_src][k] = count / n_hops, nb_out int64 [n_src][k]   (reference dtypes)
 *   wn_out f32 [n_src][t_norm], nb32_out int32 [n_src][t_norm]: the first
 *     t_norm columns with weights divided by their row sum (device table)
 * dense_scratch: device bytes >= pinsage_visit_topk_scratch(n_src, n_all, k). */
int64_t pinsage_visit_topk_scratch(int64_t n_src, int64_t n_all, int64_t k);
int pinsage_visit_topk(const int32_t* trace, const int64_t* sources, int64_t n_src,
                       int64_t n_hops, int64_t n_all, int64_t k, void* dense_scratch,
                       double* w_out, int64_t* nb_out, float* wn_out, int32_t* nb32_out,
                       int64_t t_norm, void* stream);
/* Fused walk + visit counting + top-k (the SURVEY's ppr_topk): replaces
 * do_random_walks -> sample_neighborhood -> visit_prob.topk(k, 1)
 * (pinsage_model.py:32-53, 88-107) in sample_neighborhood_topt and
 * precompute_neighborhoods_topt (:103-132), and PersPageRank.knn
 * (baselines.py:114-151).  The walk's trace stays in LDS (never in HBM); outputs
 * as pinsage_visit_topk.  mt != null: MT19937 mode (host state advanced by
 * 3*n_hops*n_src draws, exactly the reference's consumption); mt == null:
 * Philox mode keyed by (seed, hop, src_base + i, offset), the same draws as
 * pinsage_walk_philox.  Only the partial_sort regime (k * 64 <= n_all); the
 * nth_element regime of tiny graphs goes through pinsage_visit_topk.
 * ws: device bytes >= pinsage_ppr_topk_workspace(n_src, n_hops, mt != null)
 * (smaller workspaces run in rounds).  Synchronises the stream (zero-degree
 * check: the reference's torch.randint(0) raises). */
int64_t pinsage_ppr_topk_workspace(int64_t n_src, int64_t n_hops, int rng_mt);
int pinsage_ppr_topk(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                     const int64_t* sources, int64_t n_src, int64_t n_hops, float alpha, int64_t k,
                     void* mt, uint64_t seed, uint32_t offset, int64_t src_base, void* ws,
                     int64_t ws_bytes, double* w_out, int64_t* nb_out, float* wn_out,
                     int32_t* nb32_out, int64_t t_norm, void* stream);
/* pinsage_ppr_topk (Philox mode) over n_seg consecutive segments of sources in
 * one call: segment i = sources[seg_start[i] .. seg_start[i+1]) is keyed by
 * (seg_seed[i], hop, seg_base[i] + j, offset), so each segment draws exactly
 * what its own pinsage_ppr_topk call would.  Serves the train step's model
 * calls on the fly (pinsage_model.py:142-154, called at :183-185 once per
 * call), one walk per segment and one top-k pass and zero-degree check for
 * all.  seg_start / seg_seed / seg_base are host arrays (n_seg + 1, n_seg,
 * n_seg); ws >= pinsage_ppr_topk_workspace(seg_start[n_seg], n_hops, 0).
 * Synchronises the stream. */
int pinsage_ppr_topk_segments(const int64_t* indptr, const int32_t* indices, int64_t n_all,
                              const int64_t* sources, int64_t n_seg, const int64_t* seg_start,
                              const uint64_t* seg_seed, const int64_t* seg_base, int64_t n_hops,
                              float alpha, int64_t k, uint32_t offset, void* ws, int64_t ws_bytes,
                              double* w_out, int64_t* nb_out, float* wn_out, int32_t* nb32_out,
                              int64_t t_norm, void* stream);
/* ------------------------------------------------------------------ on-the-fly step (device)
 * relevant_nodes_per_layer (pinsage_model.py:142-154) for a train step's three
 * model calls (pinsage_training.py:183-185), all sizes on the device (no host
 * synchronisation: the on-the-fly step is captured whole).  Philox draws: call
 * c, fly layer k (0 = top) walks with key seeds[c * n_layers + k] and numbers
 * its sources from 0, as pinsage_ppr_topk_segments.  batch int64 [B][3]; call
 * c's node v is c * n + v in every table and position; tables nbt / wnt
 * (host arrays of n_layers device pointers, engine layer order: 0 = bottom)
 * [rows_cap >= 3 n + x_cap][T], rows of every layer's nodes written; virtual
 * nodes 3 n + j (j < *n_x <= x_cap, x_cap >= 3 B) are the earlier occurrences
 * of ids repeated inside a call (the last occurrence owns the id's row).
 * tab_ptrs: device array of 2 n_layers pointers (the nbt, then the wnt of
 * every engine layer).  pos_ids [3 B]: the engine's positions (3 i + c);
 * ids_xo [x_cap]: virtual node j's real node; fx (nullable) [3 n + x_cap][ld_x]:
 * the virtual rows j get feats[ids_xo[j] % n].  err[0] != 0x7f7f7f7f: a walk
 * met a zero-degree node; err[1] != 0: a drawn id >= n (the reference raises).
 * ws: pinsage_fly_workspace_bytes, initialised once by pinsage_fly_init_workspace. */
int64_t pinsage_fly_workspace_bytes(int64_t n, int64_t B, int64_t n_layers, int64_t T, int64_t n_hops);
int pinsage_fly_init_workspace(void* ws, int64_t n, int64_t B, int64_t n_layers, int64_t T, int64_t n_hops,
                               void* stream);
int pinsage_fly_sample(const int64_t* indptr, const int32_t* indices, int64_t n_all, const int64_t* batch,
                       int64_t B, int64_t n, int64_t n_layers, int64_t T, int64_t n_hops, float alpha,
                       const uint64_t* seeds, void* ws, int64_t ws_bytes, int32_t* const* nbt, float* const* wnt,
                       int32_t** tab_ptrs, int64_t rows_cap, int64_t* pos_ids, int* n_x, int64_t* ids_xo,
                       int64_t x_cap, const float* feats, int64_t ld_f, int64_t d, float* fx, int64_t ld_x,
                       int* err, void* stream);
/* The sampler's two error words into the host ring slot (*ctr % R) at err_off
 * (the captured on-the-fly step reports them there; the host reads them when
 * it next waits for that slot). */
int pinsage_fly_publish_err(const int* err, void* ring, int64_t slot_bytes, int64_t R, const int64_t* ctr,
                            int64_t err_off, void* stream);
/* Refuse the captured on-the-fly step's optimizer update when its sampling
 * failed (err[0] / err[1] as pinsage_fly_sample sets them): err[2] becomes a
 * sticky halt word (the host clears it after raising), and a halted step's
 * Adam coefficients get bc2 = coef[1] = 0, which every fused Adam kernel takes
 * as "leave parameters and moments untouched" -- the reference raises before
 * optimizer.step() (pinsage_model.py:25, pinsage_training.py:188-191). */
int pinsage_fly_gate_adam(int* err, float* coef, void* stream);
/* sample_neighborhood (pinsage_model.py:88-101): dense f64 [n_src][n_all]. */
int pinsage_visit_dense(const int32_t* trace, const int64_t* sources, int64_t n_src,
                        int64_t n_hops, int64_t n_all, double* dense, void* stream);

/* ------------------------------------------------------------------ frontier (device)
 * relevant_nodes_per_layer_precomp (pinsage_model.py:156-168) for the API:
 * one step nodes_out = unique(cat(nb[nodeset, :T].flatten(), nodeset)), sorted.
 * nb_table int32 [n_items][ld]; nodes_out int32 capacity >= n*(T+1) (and
 * <= n_items); *count_out (device int) receives the size.  ws: device bytes >=
 * pinsage_frontier_workspace(n_items). */
int64_t pinsage_frontier_workspace(int64_t n_items);
int pinsage_frontier_step(const int64_t* nodeset, int64_t n, const int32_t* nb_table, int64_t ld,
                          int64_t T, int64_t n_items, void* ws, int32_t* nodes_out,
                          int32_t* count_out, void* stream);
/* After pinsage_frontier_step on ws (same nodeset, table, T, n_items): the
 * index table local_idx int32 [n][T] with nodes_out[local_idx[f][t]] ==
 * nb[nodeset[f]][t] -- the rows of the unique set the convolution's slots
 * read (weighted_agg's loc), from the set's bitmap ranks. */
int pinsage_frontier_local_idx(const int64_t* nodeset, int64_t n, const int32_t* nb_table, int64_t ld, int64_t T,
                               int64_t n_items, const void* ws, int32_t* local_idx, void* stream);

/* ------------------------------------------------------------------ kernels exposed for tests
 * fp32 MFMA GEMM: C[M][N] = A[M][K] * W[N][K]^T (+bias) (leaky_relu if act),
 * A rows gathered by a_idx (nullable) -- nn.Linear on gathered rows
 * (pinsage_model.py:196,201). */
int pinsage_linear(const float* A, int64_t lda, const int32_t* a_idx, int64_t M, int64_t K,
                   const float* W, const float* bias, int64_t N, int act, float* C, int64_t ldc,
                   void* stream);
/* General form of the same GEMM, for per-configuration tests and
 * microbenchmarks: C = op(A) op(B) with A K-major ([M][K], rows gathered by
 * a_idx) or M-major ([K][M], k-rows gathered), B K-major ([N][K]) or N-major
 * ([K][N], k-rows gathered by b_idx); epi 0 store, 1 accumulate, 3 split-K
 * slabs C[splits][M][N]; cfg -1 picks the tile by size, 0..2 forces one;
 * stream_k -1 chooses by size, 0 disables, 1 forces the stream-K schedule
 * (in-launch combine of tiles cut between workgroups; scratch is owned by
 * the library). */
/* Weight gradient of an nn.Linear weight over a device-side row count
 * (the AddmmBackward of pinsage_model.py:196-201 / 208-210):
 *   dst[M][N] = A^T [B || B2]  (A [K][M] row-major; B rows gathered by b_idx
 *   when set, columns >= N1 from B2 -- torch.cat along N), dst_b[M] = column
 *   sums of A (nullable), K = *K_dev (nullable: K_max rows).  Long-K form
 *   (wgrad.hip): 64 x 64 tiles, K cut into `splits` runs (0: by size) that
 *   are combined inside the launch in a fixed order (deterministic); with
 *   adam_p set, torch.optim.Adam is applied to the slice (adam_* pointers in
 *   dst's layout, coef = {lr / (1 - b1^t), sqrt(1 - b2^t)} on the device).
 *   M, N, N1 multiples of 64.  scratch: pinsage_wgrad_scratch_bytes(M, N)
 *   bytes, zeroed once before the first call (its tickets reset themselves). */
int64_t pinsage_wgrad_scratch_bytes(int64_t M, int64_t N);
int pinsage_wgrad(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const float* A, int64_t lda,
                  const float* B, int64_t ldb, const int32_t* b_idx, int64_t N1, const float* B2, int64_t ldb2,
                  float* dst, int64_t ld_dst, float* dst_b, int splits, void* scratch, float* adam_p,
                  float* adam_m, float* adam_v, float* adam_pb, float* adam_mb, float* adam_vb,
                  const float* coef, double beta1, double beta2, float eps, void* stream);
/* The same weight gradient with both operands given as their hi / mid / lo
 * bf16 planes (pinsage_split_planes: A3 [3][K][M], B3 [3][rows][N] with plane
 * strides a3_ps / b3_ps and row strides lda / ldb elements, B rows gathered
 * by b_idx): no conversions in the k loop.  Weights are bitwise the fp32
 * form's 4-wave launch (PINSAGE_KW_WAVES=4) on the planes' source matrices;
 * dst_b sums the planes' value (H + M) + L.  The layer-0 Q weight gradient
 * (pinsage_model.py:201's AddmmBackward) in the engine. */
/* Measurement only (tools/wgrad_bench.py): the weight-gradient launch with a
 * timing-only k loop -- probe 1: the DMAs without the products, 2: the products
 * without the DMAs, 3: 2 without the split, 4: the k loop without the split.
 * The results are WRONG by construction; nothing in the engine calls it. */
int pinsage_wgrad_probe(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const float* A, const float* B,
                        const int32_t* b_idx, float* dst, float* dst_b, int splits, void* scratch, int probe,
                        void* stream);
int pinsage_wgrad_planes(int64_t M, int64_t N, const int* K_dev, int64_t K_max, const uint16_t* A3, int64_t a3_ps,
                         int64_t lda, const uint16_t* B3, int64_t b3_ps, int64_t ldb, const int32_t* b_idx,
                         float* dst, int64_t ld_dst, float* dst_b, int splits, void* scratch, void* stream);
int pinsage_gemm_ex(int64_t M, int64_t N, int64_t K, int a_kmajor, int b_kmajor, const float* A,
                    int64_t lda, const int32_t* a_idx, const float* B, int64_t ldb,
                    const int32_t* b_idx, float* C, int64_t ldc, const float* bias, int act,
                    int epi, int splits, int cfg, int stream_k, void* stream);
/* Product arithmetic of the fp32 GEMMs with K-major operands (the Q / W
 * projections of the forward, the kNN dot products): 0 = v_mfma_f32_32x32x2_f32
 * (exact fp32 FMA chains); 1 (default; PINSAGE_GEMM_PREC overrides at load) =
 * each fp32 operand split exactly into hi + mid + lo bf16 (|residual| <= 2^-26
 * |x|), the six products down to 2^-18 of hi*hi on v_mfma_f32_32x32x16_bf16
 * with fp32 accumulation: fp32-level error at 2.67x the fp32 MFMA rate.
 * Process-wide; other GEMMs always use fp32 MFMA. */
int pinsage_gemm_set_prec(int prec);
int pinsage_gemm_get_prec(void);
/* hi / mid / lo bf16 planes of a row-major fp32 matrix W[rows][cols] (row
 * stride ldw floats): out[3][rows][cols] as uint16 bf16 bits, the exact split
 * the split-bf16 GEMM does in registers (cols % 8 == 0, ldw % 4 == 0). */
int pinsage_split_planes(const float* W, int64_t rows, int64_t cols, int64_t ldw, uint16_t* out,
                         void* stream);
/* pinsage_linear's product (K-major A rows gathered by a_idx, W[N][K]) under
 * split-bf16 arithmetic with W given ALSO as its pre-split planes (from
 * pinsage_split_planes(W, N, K, ...): row stride ldws == K elements, plane
 * stride N*K; other strides are rejected): the kernel converts A only.
 * Bitwise equal to the in-register split for cfg 0 and 3 (other cfg values,
 * -1 included, may run the in-register form; the result is the same). */
int pinsage_linear_split_b(const float* A, int64_t lda, const int32_t* a_idx, int64_t M, int64_t K,
                           const float* W, const uint16_t* W_planes, int64_t ldws,
                           const float* bias, int64_t N, int act, float* C, int64_t ldc, int cfg,
                           void* stream);
/* max_margin_loss (pinsage_training.py:31-41) of outputs given per position,
 * Z f32 [3][B][d] (q, pos, neg calls; d <= 256 dividing 1024), with the train
 * step's own kernels and reduction order (pinsage_engine_loss): scal f32[4] =
 * {loss, 0, sum |z_q|^2, variance of the z_q}, G f32 [3][3B][d] = the loss
 * cotangent of position (c, b) at row G[c][c*B + b] (other rows zero).  Equal
 * rows give the step's loss bits.  scratch: pinsage_triplet_loss_scratch_bytes
 * bytes, 16-B aligned.  The micro-batched step's loss. */
int64_t pinsage_triplet_loss_scratch_bytes(int64_t B, int64_t d);
int pinsage_triplet_loss(const float* Z, int64_t B, int64_t d, float margin, float* G, void* scratch, float* scal,
                         void* stream);
/* Interleaved split-bf16 table of src[rows][K] (K % 16 == 0, ld % 4 == 0):
 * row r at out + r * ldo (bf16 elements, ldo % 8 == 0, ldo >= 3K) holds K/16
 * stages of six 16-B chunks -- hi, mid, lo bf16 of the stage's 16 values, 8
 * per chunk -- the exact split the GEMM does in registers.  The input feature
 * table is split once (features do not change during training), W_Q per step. */
int pinsage_split_ilv(const float* src, int64_t ld, int64_t rows, int64_t K, uint16_t* out, int64_t ldo,
                      void* stream);
/* C[m][0..N) = act(A[a_idx[m]] . W[n] + bias[n]) from an interleaved table of
 * A (rows gathered by a_idx) and W [N][K] either as its interleaved table
 * (W_ilv, pinsage_split_ilv) or, W_ilv null, fp32 split in registers: bitwise
 * pinsage_linear's split-bf16 product on the same 128 x 128 tiles, every
 * gathered row's 16-k stage one contiguous 96-B read.  M static or *M_dev <=
 * M_max.  The layer-0 Q projection (pinsage_model.py:201). */
int pinsage_linear_ilv(const uint16_t* A_ilv, int64_t lda_ilv, const int32_t* a_idx, int64_t M, const int* M_dev,
                       int64_t M_max, int64_t K, const float* W, const uint16_t* W_ilv, int64_t ldw_ilv,
                       const float* bias, int64_t N, int act, float* C, int64_t ldc, void* stream);
/* agg[f] = sum_t w[f][t] * q[loc[f][t]]  (weights already normalised;
 * pinsage_model.py:202). */
int pinsage_weighted_agg(const float* q, int64_t hid, const int32_t* loc, const float* w,
                         int64_t n_rows, int64_t T, float* agg, void* stream);

/* ConvLayer.forward after the Q projection (pinsage_model.py:195-210): for each
 * row f of n_rows,
 *   agg[f]  = sum_t w[f][t] * q[loc[f][t]]                     (:202, w normalised)
 *   y[f]    = normalize(lrelu([h[self_src[f]] || agg[f]] W^T + bias))   (:208-210)
 *   norms[f] = ||lrelu(.)||_2 (nullable)
 * the engine's kernel: the aggregate formed in registers and written out once,
 * the projection on split-bf16 MFMA.  h f32 [.][ldh], q f32 [q_rows][hid],
 * loc int32 / w f32 [n_rows][T], W f32 [out][d+hid], y f32 [n_rows][out],
 * agg f32 [n_rows][hid].  out == 128, 1 <= T <= 64, d + hid a multiple of 64,
 * d and hid multiples of 4.  W_planes (nullable device scratch of
 * 3 * out * (d + hid) uint16): where the 32-row tile runs (>= 16 rows per CU,
 * d + hid a multiple of 128, d a multiple of 32) W is split into it
 * (fragment-order bf16 planes) and the tile's gather runs pipelined against its
 * projection (the same y bitwise); null runs it unpipelined. */
int pinsage_conv_agg_project(const float* h, int64_t ldh, int64_t d, const int32_t* self_src,
                             const float* q, int64_t hid, int64_t q_rows, const int32_t* loc,
                             const float* w, int64_t n_rows, int64_t T, const float* W,
                             const float* bias, int64_t out, uint16_t* W_planes, float* y,
                             float* norms, float* agg, void* stream);

/* get_embeddings' row gather (pinsage_model.py:21-23): out[i][0..d) =
 * h[idx[i]][0..d), idx int64 (device).  Ids outside [0, n_h) give zero rows
 * (the reference raises IndexError: callers validate).  Its transpose
 * (the gradient, an index_add over repeated ids) is a pinsage_segment_wmean
 * over the CSR of idx, deterministic in summation order. */
int pinsage_gather_rows(const float* h, int64_t ldh, int64_t n_h, int64_t d, const int64_t* idx, int64_t n,
                        float* out, int64_t ldo, void* stream);
/* ConvLayer's W projection alone (pinsage_model.py:208-210):
 *   y[f] = normalize(lrelu([h[self_idx[f]][0..d) || agg[f]] W^T + bias)),
 *   norms[f] = ||lrelu(.)||_2
 * with the concat read in place (no concat buffer).  self_idx int32 nullable
 * (rows 0..n-1), W f32 [out][d+hid], d and hid multiples of 4.  out <= 128:
 * one launch (the GEMM's L2-norm epilogue); wider: the GEMM with bias +
 * LeakyReLU, then an in-place row normalisation. */
int pinsage_concat_linear_l2norm(const float* h, int64_t ldh, const int32_t* self_idx, int64_t n, int64_t d,
                                 const float* agg, int64_t ld_agg, int64_t hid, const float* W,
                                 const float* bias, int64_t out, float* y, float* norms, void* stream);
/* Backward of y = lrelu(p) / ||lrelu(p)|| (the autograd of pinsage_model.py:209-210):
 *   dp = lrelu'(y) * (dy - y (y . dy)) / norms     (y, dy, dp f32 [n][out]) */
int pinsage_norm_lrelu_backward(const float* y, const float* norms, const float* dy, int64_t n, int64_t out,
                                float* dp, void* stream);

/* ------------------------------------------------------------------ step hand-off
 * (PinSage.train_batch, pinsage_training.py:181-214, as ONE graph launch per step)
 * pinsage_step_stage: copy nbytes at src_off of slot (*ctr % R) of a pinned host
 * ring (slot_bytes each) to dst, and 8 bytes at coef_off to coef_dst (if set);
 * offsets and sizes multiples of 8.  pinsage_step_publish: ring_out[*ctr % R2]
 * [0..n) = scal[0..n) (n <= 64), then *ctr += 1.  Both read the counter on the
 * device, so a captured step graph stages and publishes the step the host
 * wrote, without copies between launches. */
int pinsage_step_stage(const void* ring, int64_t slot_bytes, int64_t R, const int64_t* ctr,
                       int64_t src_off, int64_t nbytes, void* dst, int64_t coef_off, void* coef_dst,
                       void* stream);
int pinsage_step_publish(const float* scal, int64_t n, float* ring_out, int64_t R2, int64_t* ctr,
                         void* stream);
/* Measurement only (bench.py's per-kernel timing pass): one wave that holds the
 * stream for `us` microseconds (0..1e6) of the constant 100 MHz clock, so the
 * launches the host queues behind it run back to back and events around them
 * time the kernels rather than the host's enqueue gaps. */
int pinsage_stream_hold(int64_t us, void* stream);

/* The host side of one captured train step (pinsage_training._FusedStep) in
 * one call -- the per-step work of pinsage_training.py:181-191's loop body
 * before the device runs it.  ring: the pinned hand-off ring [R][slot_bytes]
 * whose slot holds the step's ids (off_ids), the predicted next ids
 * (off_next) and the Adam coefficients (off_coef, 2 f32).  Per parity p
 * (workspace), three hipGraphExec_t of torch captures: gf (stage + frontier),
 * gm (the step), ga (the step + the next batch's frontier in the other
 * workspace).  pinsage_stepper_step: waits for the slot's previous step,
 * writes coef, launches gf unless the batch equals the ids whose frontier the
 * previous step computed ahead, then ga with `next` (the sampler's predicted
 * next batch, nullable) or gm, and records the slot's event.  batch / next:
 * n_ids int64 host ids (ids outside [0, n_items): kErrIndex, nothing
 * launched).  info (nullable) int64[2] = {ahead hit, step index}. */
typedef struct pinsage_stepper pinsage_stepper;
int pinsage_stepper_create(void* ring, int64_t R, int64_t slot_bytes, int64_t off_ids, int64_t off_next,
                           int64_t off_coef, int64_t max_ids, int64_t n_items, pinsage_stepper** out);
void pinsage_stepper_destroy(pinsage_stepper* s);
int pinsage_stepper_set_graphs(pinsage_stepper* s, int p, void* gf, void* gm, void* ga);
/* host nanoseconds spent blocked on ring slots so far (the device behind the host) */
int64_t pinsage_stepper_wait_ns(const pinsage_stepper* s);
/* out[0 .. n) of {ns blocked on ring slots, ns inside hipGraphLaunch, ns inside
 * pinsage_stepper_step, steps, ahead hits} (host accounting of the native path) */
int pinsage_stepper_stats(const pinsage_stepper* s, int64_t* out, int n);
/* resume from the trainer's eager path: next parity, step counter, no pending frontier */
int pinsage_stepper_sync_state(pinsage_stepper* s, int parity, int64_t nstep);
int pinsage_stepper_step(pinsage_stepper* s, const int64_t* batch, int64_t n_ids, const float* coef,
                         const int64_t* next, void* stream, int64_t* info);

/* ------------------------------------------------------------------ lib/gnns MEAN aggregator
 * GNN_model.aggregate, agg_func 'MEAN' (lib/gnns/GNNs_unsupervised.py:537-588):
 * mask.mm(embed_matrix) with the dense [F, U] mask kept as a CSR.  For each
 * segment i in [0, n_seg), entries j in [seg_ptr[i], seg_ptr[i+1]):
 *   out[i, :] = sum_j w[j] * h[cols[j], :] / den_i
 * den_i = max(sum_j |w[j]|, 1e-12) (F.normalize(p=1)) if normalize, else 1.
 * h f32 [n_h][ldh], out f32 [n_seg][ldo], seg_ptr int64 [n_seg + 1], cols int32,
 * w f32 (device).  Entries whose col is outside [0, n_h) are skipped (the
 * caller validates).  The backward (dH = mask^T dOut) is the same call over the
 * transposed CSR with pre-normalised weights and normalize = 0. */
int pinsage_segment_wmean(const float* h, int64_t ldh, int64_t n_h, int64_t d, const int64_t* seg_ptr,
                          const int32_t* cols, const float* w, int64_t n_seg, int normalize, float* out,
                          int64_t ldo, void* stream);

/* ------------------------------------------------------------------ cosine kNN
 * knn_from_emb (baselines.py:91-103) over cosine_sim_ab (baselines.py:69-77), the
 * evaluation consumer of the embeddings (eval.py:112-143 save_knn, k = 1000):
 * for each query row q (int64 ids in [0, n), validated by the caller)
 *   sim(q, j) = dot(emb[q], emb[j]) / (|emb[q]| |emb[j]| + eps), j in [0, n)
 * out_w f32 [nq][k] / out_n int64 [nq][k]: the k largest, sorted descending
 * (exact ties: lower index first).  The reference then drops column 0.
 * emb: f32 device rows of stride ld (d % 4 == 0); 1 <= k <= min(n, 4096).
 * scratch: device bytes >= pinsage_knn_scratch_bytes(n, rows) for some
 * batch of rows >= 1 (the dot products of one batch of queries live there;
 * larger scratch = fewer batches). */
int64_t pinsage_knn_scratch_bytes(int64_t n, int64_t batch_rows);
int pinsage_knn_cosine(const float* emb, int64_t n, int64_t d, int64_t ld, const int64_t* queries,
                       int64_t nq, int64_t k, float eps, void* scratch, int64_t scratch_bytes,
                       float* out_w, int64_t* out_n, void* stream);

/* ------------------------------------------------------------------ train-step engine
 * PinSageModel.forward / PinSage.train_batch (pinsage_model.py:246-265,
 * pinsage_training.py:181-214) with device-resident sizes.  Parameters live in
 * one flat fp32 buffer in state_dict order: conv_layers.{i}.Q.weight, Q.bias,
 * W.weight, W.bias (i = 0..n_layers-1), G1.weight, G1.bias, G2.weight; the
 * gradient and Adam buffers use the same layout. */
typedef struct pinsage_engine pinsage_engine;
typedef struct {
  int64_t n_items;  /* feature-table rows (tracks) */
  int64_t d_in;     /* feature dim (dimensions[0]) */
  int64_t hid;      /* hidden_dim (dimensions[1]) */
  int64_t out;      /* out_dim (dimensions[2], <= 128) */
  int64_t n_layers;
  int64_t T;        /* neighbourhood size used by the model */
  int64_t max_pos;  /* max ids per forward (3 * batch_size for a train step) */
} pinsage_engine_config;
typedef struct {
  int64_t ids, pos_rank, z, dz, scalars, n_layers;
  int64_t count_S[8], count_N[8], members_S[8], members_N[8], cap_S[8], cap_N[8], y[8];
  int64_t param_offsets[8];
  int64_t hinge; /* f32 [batch]: cos(q,n) - cos(q,p) + margin of each triple of the last loss */
} pinsage_engine_offsets_t;

int pinsage_engine_create(const pinsage_engine_config* cfg, pinsage_engine** out);
/* Makes no HIP call (safe inside a stream capture, e.g. a finaliser run by the
 * garbage collector while torch.cuda.graph captures): the engine's streams and
 * events are retired to a process-wide pool that later engines reuse. */
void pinsage_engine_destroy(pinsage_engine* e);
/* engines created and not yet destroyed (diagnostics / tests) */
int64_t pinsage_engine_live_count(void);
int64_t pinsage_engine_workspace_bytes(const pinsage_engine* e);
int64_t pinsage_engine_num_params(const pinsage_engine* e);
/* byte offsets of engine outputs inside a workspace (ids int64, pos_rank int32,
 * z/dz f32 [rows][out], scalars f32 {loss, node_feat_loss, sum|h_q|^2, variance}). */
int pinsage_engine_offsets(const pinsage_engine* e, pinsage_engine_offsets_t* out);
/* features f32 [n_items][ld_feats]; tables: nb int32 / normalised weights f32
 * [n_items][ld_table] (first T columns used); grads / adam buffers may be null
 * for inference. */
int pinsage_engine_set_tensors(pinsage_engine* e, const float* feats, int64_t ld_feats,
                               const int32_t* nb_table, const float* w_table, int64_t ld_table,
                               float* params, float* grads, float* adam_m, float* adam_v);
/* The input feature table's hi / mid / lo bf16 planes [3][n][d_in] (from
 * pinsage_split_planes(feats, n, d_in, ld_feats, planes); plane stride in
 * elements), or null: with them the layer-0 Q weight gradient
 * (pinsage_model.py:201's AddmmBackward) runs on pre-split operands -- the
 * transposed aggregation writes layer 0's dpq as planes too -- and does no
 * conversions; the result's weights are those of the fp32 form's 4-wave
 * launch.  The caller keeps the planes equal to the split of the features the
 * engine reads (pinsage_model.Runner.bind re-splits when the tensor's version
 * changes). */
int pinsage_engine_set_feature_planes(pinsage_engine* e, const uint16_t* planes, int64_t plane_stride);
/* on = 0: the engine's next pinsage_engine_frontier calls do not fork its
 * side stream (PINSAGE_CSR_FORK), e.g. while the caller captures them on a
 * branch of a graph (forking off a capture branch, not the capture's origin,
 * sent hipStreamEndCapture into unbounded recursion); 1 (default) restores. */
int pinsage_engine_set_frontier_fork(pinsage_engine* e, int on);
/* The input feature table's interleaved split-bf16 table [n][ld] (from
 * pinsage_split_ilv(feats, ld_feats, n, d_in, table, ld); ld % 8 == 0, ld >=
 * 3 d_in), or null: with it the layer-0 Q projection (pinsage_model.py:201)
 * reads each gathered row's 16-k stage as one 96-B piece and converts nothing
 * (Q0 is split per step into the workspace); bitwise the in-register split on
 * the same 128 x 128 tiles.  The caller keeps the table equal to the split of
 * the features the engine reads. */
int pinsage_engine_set_feature_ilv(pinsage_engine* e, const uint16_t* table, int64_t ld);
/* Zero the workspace regions the step kernels keep zero after use (loss
 * scatter targets, CSR counters).  Call once per new workspace, before its
 * first forward. */
int pinsage_engine_init_workspace(pinsage_engine* e, void* ws, void* stream);
/* forward of all ids (a train step passes the [B][3] batch flattened); ids must
 * lie in [0, n_items) -- the caller validates them (pinsage_model raises
 * IndexError like the reference's features[nodeset]). */
int pinsage_engine_forward(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                           void* stream);
/* The forward's two phases (pinsage_engine_forward = frontier, then layers).
 * The frontier phase (relevant_nodes_per_layer_precomp, pinsage_model.py:156-168,
 * plus every layer's index tables) reads only the ids and the neighbourhood
 * table -- no parameters -- so a trainer with two workspaces runs the next
 * step's frontier on a side stream while this step's layers and backward run
 * in the other workspace. */
/* pinsage_engine_forward without the backward's plan (the CSR transposes of the
 * neighbour slots): for outputs only (PinSage.embed, evaluation, the first pass
 * of the micro-batched step); no backward may follow on this workspace. */
int pinsage_engine_forward_inference(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                                     void* stream);
int pinsage_engine_frontier(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                            void* stream);
int pinsage_engine_forward_layers(pinsage_engine* e, void* ws, void* stream);
/* Until reset with side_stream = NULL: each pinsage_engine_forward_layers call
 * also runs pinsage_engine_frontier(ws_next, ids_next, n_ids) on side_stream,
 * forked (event) right after the layer-0 Q projection, so it overlaps the rest
 * of the step.  The caller joins side_stream back. */
int pinsage_engine_set_fork(pinsage_engine* e, void* ws_next, const int64_t* ids_next,
                            int64_t n_ids, void* side_stream);
int pinsage_engine_gather_output(pinsage_engine* e, void* ws, int64_t n_ids, float* out,
                                 void* stream);
/* max_margin_loss + monitors on the last forward of a [B][3] batch.  It
 * accumulates the loss cotangent into the workspace's per-row gradient
 * accumulators (the head backward forms dZ from them and re-zeroes them), so a
 * pinsage_engine_backward / _backward_adam MUST follow every loss call on a
 * workspace before its next loss call (an eval-only loss would leave them
 * dirty for the next step).
 * The monitor kernel (loss / node-feature loss / variance scalars, on an engine
 * side stream, dependent on this loss) is enqueued by the next engine call
 * that enqueues work (normally the backward, right behind its first kernel;
 * PINSAGE_DEFER_SIDE=0/1 enqueues it here) and joined at the backward's end. */
int pinsage_engine_loss(pinsage_engine* e, void* ws, int64_t batch_size, float margin,
                        int with_monitors, void* stream);
/* dZ from an upstream gradient of gather_output (single call, autograd path) */
int pinsage_engine_set_output_grad(pinsage_engine* e, void* ws, const float* dout, int64_t n_ids,
                                   void* stream);
/* all parameter gradients from dZ into the grad buffer (overwritten) */
int pinsage_engine_backward(pinsage_engine* e, void* ws, void* stream);
/* Re-arm a workspace whose backward has run for another backward of the same
 * forward (autograd's retain_graph=True: backward(retain_graph=True) then
 * backward again): zeroes the scatter-add targets the backward accumulates
 * into.  The forward's activations and plan are left as they are. */
int pinsage_engine_reset_backward(pinsage_engine* e, void* ws, void* stream);
/* the same backward in two calls, for data-parallel steps that all-reduce the
 * first call's gradients while the second runs (pinsage_training.py:188-191
 * under DP): stage 0 = the head and layers L-1 .. 1 (every gradient but layer
 * 0's is complete in stream order at the call's end), stage 1 = layer 0. */
int pinsage_engine_backward_stage(pinsage_engine* e, void* ws, int stage, void* stream);
/* torch.optim.Adam step over the flat buffers (pinsage_training.py:147,191).
 * coef: device f32[2] = {lr / (1 - beta1^t), sqrt(1 - beta2^t)} for this step
 * t, computed by the caller in double as torch does (kept in device memory so
 * a captured step graph picks up each step's values). */
int pinsage_engine_adam(pinsage_engine* e, const float* coef, double beta1, double beta2, float eps,
                        void* stream);
/* backward followed by that Adam step, scheduled off the critical path: the
 * last gradient (layer 0's Q) applies its own Adam step in the reduction that
 * produces it, and every other parameter is updated beside that reduction.
 * Gradients are still written to the grad buffer; the arithmetic is that of
 * pinsage_engine_backward + pinsage_engine_adam. */
int pinsage_engine_backward_adam(pinsage_engine* e, void* ws, const float* coef, double beta1,
                                 double beta2, float eps, void* stream);

/* Frontier sizes of the last forward in ws (synchronises the stream): S[l] =
 * |S_l| (nodes convolved at layer l), N[l] = |N_l| (distinct neighbours). */
int pinsage_engine_read_counts(const pinsage_engine* e, void* ws, int64_t* S, int64_t* N,
                               void* stream);
/* Expected frontier sizes (e.g. from read_counts): choose GEMM block tiles
 * that fill the chip; sizes stay device-side, hints only affect speed. */
int pinsage_engine_set_hints(pinsage_engine* e, const int64_t* S, const int64_t* N);
/* Layer `layer`'s own neighbourhood table (nb int32 / normalised weights f32,
 * [n_items][ld], first T columns, rows of the layer's nodes used) in place of
 * the engine-wide one from pinsage_engine_set_tensors: the on-the-fly sampler
 * (relevant_nodes_per_layer, pinsage_model.py:142-154) draws every layer's
 * neighbourhoods separately.  nb = wn = null restores the engine-wide table.
 * Read when a frontier is enqueued (pinsage_engine_forward / _frontier). */
/* Whether a GEMM site's last launch ran stream-K (1), a whole-K tile (0), or
 * is unknown (-1): the in-context tuner keeps a site's summation order. */
int pinsage_engine_site_stream_k(const pinsage_engine* e, const char* site);
int pinsage_engine_set_layer_table(pinsage_engine* e, int64_t layer, const int32_t* nb,
                                   const float* wn, int64_t ld);
/* The on-the-fly step's virtual nodes (pinsage_fly_sample): ids x0 .. x0 +
 * *n_x - 1 join every frontier's top set, and pinsage_engine_loss hands
 * virtual node j the summed output gradient of its real node xids[j] (call
 * xids[j] / unit), each occurrence's conv output with multiplicity 1
 * (index_put's backward, pinsage_model.py:257-265).  n_x = null: off. */
int pinsage_engine_set_fly(pinsage_engine* e, int64_t x0, const int* n_x, const int64_t* xids, int64_t unit,
                           int64_t x_cap);
/* Per-site GEMM choice (a tuner measures the sites in context and fixes them):
 * site names as the timing sites -- fwd.q_gemm.lN, fwd.w_gemm.lN, bwd.dcat.lN,
 * bwd.dh.lN (block tile config cfg 0..3, stream_k 0/1), bwd.w_wgrad.lN,
 * bwd.q_wgrad.lN, bwd.wgrad.g1, bwd.wgrad.g2 (cfg 0..3 and split-K count
 * splits >= 1).  -1 / 0 leave a field to the launcher's size model; all three
 * unset removes the site's entry.  Speed only: every choice computes the same
 * GEMM (summation order may differ). */
int pinsage_engine_set_gemm_choice(pinsage_engine* e, const char* site, int cfg, int stream_k,
                                   int splits);

/* Per-launch-site HIP-event timing on the launch stream (bench/profiling):
 * enable (also clears), collect after the work (synchronises the events), then
 * read site idx = 0.. until PINSAGE_ERR_ARG: name, total ms, number of calls. */
int pinsage_engine_timing(pinsage_engine* e, int enable);
int pinsage_engine_timing_collect(pinsage_engine* e);
int pinsage_engine_timing_get(const pinsage_engine* e, int idx, char* name, int64_t name_len,
                              double* ms, int64_t* calls);

#ifdef __cplusplus
}
#endif
#endif /* PINSAGE_HIP_H */

// PinSage train-step engine: sequences the frontier, convolution, head, loss,
// backward and Adam kernels on one HIP stream with every data-dependent size
// kept on the device, so a step needs no host synchronisation and can be
// captured into a hipGraph.
//
// Forward over the UNION of the calls in one launch sequence: the reference
// runs the model three times per step (pinsage_training.py:184-186) and each
// output row depends only on its own node's subtree, so computing every
// distinct frontier node once gives the same values.  The reference's gradient
// semantics for repeated batch ids (index_put backward hands each repeated
// output row the summed gradient, pinsage_model.py:29,265) are reproduced in
// the loss kernel per call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <atomic>
#include <string>
#include <vector>

#include "aggw.h"
#include "common.h"
#include "conv.h"
#include "gemm.h"
#include "wgrad.h"

namespace ps {

// launchers from frontier.hip / conv.hip
int64_t bitset_words(int64_t universe);
int64_t bitset_blocks(int64_t universe);
int launch_mark_i64(unsigned long long*, const int64_t*, int64_t, int64_t, int*, hipStream_t);
int launch_mark_table(unsigned long long*, const int32_t*, const int*, int64_t, const int32_t*,
                      int64_t, int, int64_t, hipStream_t);
bool mark_finalize_fits(int64_t universe);
int launch_mark_finalize(unsigned long long*, const int32_t*, const int*, int64_t, const int32_t*, int64_t, int,
                         int64_t, int*, uint32_t*, int32_t*, int*, unsigned long long*, const unsigned long long*,
                         uint32_t*, int32_t*, int*, hipStream_t);
int launch_set_finalize(unsigned long long*, const unsigned long long*, const unsigned long long*,
                        int64_t, uint32_t*, uint32_t*, int32_t*, int*, hipStream_t);
int launch_top_set(unsigned long long*, int64_t, unsigned long long*, const int64_t*, int64_t,
                   int64_t, uint32_t*, uint32_t*, int32_t*, int*, hipStream_t, int64_t x0 = 0,
                   const int* x_n = nullptr);
int launch_fly_fix(float*, int*, int64_t, int, const unsigned long long*, const uint32_t*, const int*, const int64_t*,
                   int64_t, int64_t, int64_t, const int*, float*, bool, hipStream_t);

int launch_agg(const float*, int, const int32_t*, const float*, int, const int*, int64_t, float*,
               hipStream_t);
int launch_csr_build(const int32_t*, const float*, const int*, int64_t, int, const int*, int64_t, int*, int*,
                     int*, int*, int*, int2*, int2*, int*, int2*, int*, float*, int, hipStream_t, int2*);
int64_t dq_chunk_capacity(int64_t, int, int64_t);
int64_t dq_split_capacity(int64_t, int);
int launch_dq_chunks(const int2*, const int*, int64_t, const int2*, const int*, int64_t, const int*,
                     const int2*, const float*, int64_t, const float*, int, float*, float*, hipStream_t,
                     const int32_t* q_src = nullptr, int32_t* csrc = nullptr, const int* cbase = nullptr,
                     int* tk = nullptr, uint16_t* dpq3 = nullptr, int64_t ps3 = 0);
int dq_tree_levels(int64_t max_chunks);
int launch_norm_lrelu_bwd(const float*, const float*, const float*, int, const int*, int64_t,
                          float*, float*, int, const int*, int*, int64_t, hipStream_t);
int launch_loss(const float*, int, const int32_t*, int, float, const float*, int64_t, int,
                const int64_t*, float*, int*, int64_t, const int*, float*, float*, float*, float*,
                float*, bool, bool, const int*, const int32_t*, float*, hipStream_t);
int launch_pos_csr(const int32_t*, int64_t, const int*, int*, int32_t*, hipStream_t);
int launch_loss_monitor(const float*, int, const float*, int, int, float*, hipStream_t);
int launch_adam(float*, const float*, float*, float*, int64_t, const float*, double, double, float,
                hipStream_t);
int csr_prepare();
int launch_reduce_slabs_2d(const float*, int, int64_t, int, int, float*, int64_t, const float*,
                           float*, const AdamSlice*, hipStream_t);
int launch_gather_out(const float*, int, const int32_t*, int64_t, float*, hipStream_t);
int launch_head_fwd(const float*, int, const int*, int64_t, const float*, const float*,
                    const float*, float*, float*, hipStream_t);
int launch_head_bwd(float*, int*, int64_t, float*, int, const int*, int64_t, const float*,
                    const float*, const float*, const float*, const float*, float*, float*,
                    const int*, const int32_t*, const float*, hipStream_t);
int launch_dz_from_dout(const float*, int, const int32_t*, int64_t, const int*, int64_t, float*,
                        int*, float*, bool, const int*, const int32_t*, float*, hipStream_t);

struct EngineConfig {
  int64_t n_items;   // rows of the feature table (track universe)
  int64_t d_in;      // feature dim
  int64_t hid;       // hidden_dim (Q output)
  int64_t out;       // out_dim
  int64_t n_layers;
  int64_t T;         // neighbourhood size used by the model
  int64_t max_pos;   // max ids per forward (e.g. 3 * batch_size)
};

struct SetBuf {
  int64_t cap = 0;
  int64_t hint = 0;  // expected size (from a previous step), picks GEMM tile configs
  size_t bits = 0, prefix = 0, members = 0, count = 0;
};

struct LayerBuf {
  SetBuf S, N;      // frontier S_l and its neighbour set N_l
  int64_t d = 0;    // input dim of the layer
  size_t self_src = 0, q_src = 0, loc = 0, wloc = 0;
  size_t q = 0, agg = 0, y = 0, nrm = 0;
  size_t wplanes = 0;  // the W weight's fragment-order bf16 planes (aggw.hip pipelined form)
  // backward
  size_t dY = 0, dp = 0, dagg = 0, dpq = 0, cnt = 0, bsum = 0, off = 0, cursor = 0, cbase = 0,
         occ2 = 0, occ2b = 0, chunks = 0, nchunks = 0, dqpart = 0, split = 0, nsplit = 0;
  size_t csrc = 0;  // chunk rows' source indices (bottom layer, Engine::dq_chunk_rows)
  int64_t max_chunks = 0, max_split = 0;
  size_t dqtk = 0;  // split-row tree tickets (dq_tree_levels x max_chunks ints, self-resetting)
  size_t dpq3 = 0;  // (layer 0, Engine::wgrad_planes) dpq as bf16 planes [3][N.cap][hid]
  int64_t dqtk_len = 0;
  // parameter offsets (floats) into the flat param / grad buffers
  int64_t pQw = 0, pQb = 0, pWw = 0, pWb = 0;
  // this layer's own neighbourhood table (pinsage_engine_set_layer_table: the
  // on-the-fly sampler gives every layer its own draws); null = the engine's
  const int32_t* nb_tab = nullptr;
  const float* wn_tab = nullptr;
  int64_t ld_tab = 0;
};

// Optional HIP-event timing of launch sites on the launch stream (bench only).
struct TimingSite {
  std::string name;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double ms = 0.0;
  int64_t calls = 0;
};

struct Engine {
  EngineConfig cfg{};
  bool timing = false;
  // (The weight gradients run beside the caller's stream on side[1]; keeping
  // them, the CSR work or layer 0's W gradient on the chain measured 0.611 to
  // 0.648 ms/step against 0.605-0.615 in round 2 -- the A/B knob is retired.)
  // The head as one fused forward / backward kernel (head.hip); the separate
  // GEMM launches remain for the unfused arithmetic (fused_head false is no
  // longer selectable: settled A/B).
  bool fused_head = true;
  // the fused head backward sums repeated batch nodes' loss rows itself (no
  // rep_sum launch between the loss and it); PINSAGE_HEAD_REP_SUM=0: rep_sum
  // launch (A/B; bitwise the same G rows)
  bool head_rep_sum = !getenv("PINSAGE_HEAD_REP_SUM") || atoi(getenv("PINSAGE_HEAD_REP_SUM")) != 0;
  // the fused head's forward inside the top layer's 16-row aggregation + W
  // tile (AggHead, aggw.h): one launch less; PINSAGE_HEAD_IN_AGGW=0: head_fwd launch
  bool head_in_aggw = !getenv("PINSAGE_HEAD_IN_AGGW") || atoi(getenv("PINSAGE_HEAD_IN_AGGW")) != 0;
  // the last enqueued G producer was the loss with rep_sum left to the head
  // (G's repeated ranks still in Gp, three groups); dz_from_dout clears it
  bool reps_in_gp = false;
  // PINSAGE_FUSED_AGGW=0: aggregation and W projection as two launches (A/B);
  // 1 (default): one launch (aggw.hip).  Experimental forms measured slower and
  // removed: register-pipelined split-bf16 (C2 layer 0 39.7 us),
  // warp-specialised on LDS-DMA (45.8) or on registers (41.4), against 36.5.
  int fused_aggw = getenv("PINSAGE_FUSED_AGGW") ? atoi(getenv("PINSAGE_FUSED_AGGW")) : 1;
  // The next layer's Q projection inside the 32-row aggregation + W kernel
  // (AggNextQ, aggw.h): one launch less per upper layer, at the price of the
  // products of every output row (not only the next layer's neighbours) and
  // a longer tile.  Default (-1): per layer, where agg_w_next_q_pays -- the
  // 32-row form's tiles fit one pass over the CUs.  Measured (one session,
  // ms/step, layer 0's kernel µs): C2 (179 tiles) 0.4248/0.4296 -> 0.4194/0.4217,
  // 36.7 -> 49.2 against the 16 µs Q GEMM it replaces; C4 (268 tiles, a second
  // pass) 0.4645 -> 0.4665, 50.5 -> 75.2.  PINSAGE_FUSED_NEXT_Q=0 / 1 forces
  // it off / on wherever the 32-row form runs.
  int fused_next_q = getenv("PINSAGE_FUSED_NEXT_Q") ? atoi(getenv("PINSAGE_FUSED_NEXT_Q")) : -1;
  // PINSAGE_DQ_CHUNK_ROWS=1: the bottom layer's Q weight gradient over dq
  // chunk rows (masked per-chunk partials, h gathered per chunk) instead of
  // combined dpq rows, so the combine launch leaves the chain.  Measured (one
  // session, ms/step, bwd.layer.l0 µs): C2 0.451 -> 0.454, 167 -> 169; C4
  // 0.483 -> 0.476, 183 -> 179 -- the GEMM's K grows by the split rows' extra
  // chunks (C2 Q0 wgrad 69 -> 79 µs) about as much as the combine saved.
  bool dq_chunk_rows = getenv("PINSAGE_DQ_CHUNK_ROWS") && atoi(getenv("PINSAGE_DQ_CHUNK_ROWS")) != 0;
  // PINSAGE_CSR_FORK: the frontier's CSR transposes with a fork onto side[0]
  // (engine_frontier): 1 = layer 0's CSR on side[0] beside the upper layers',
  // 2 = an empty branch (fork + join, no work); 0 (default) = one stream.
  // Either fork is joined back into the frontier's stream before
  // engine_frontier returns, so no engine call leaves a side stream unjoined
  // inside a caller's capture (tests/test_gpu_trainer.py)
  int csr_fork = getenv("PINSAGE_CSR_FORK") ? atoi(getenv("PINSAGE_CSR_FORK")) : 0;
  // which side stream the frontier forks: 2 (default, its own), or 0 (the
  // backward's side[0]: the round-5 shape, kept for tools/dbg reproduction)
  int csr_fork_stream = getenv("PINSAGE_CSR_FORK_STREAM") ? atoi(getenv("PINSAGE_CSR_FORK_STREAM")) : 2;
  // pinsage_engine_set_frontier_fork(e, 0): the next frontiers do not fork
  // (a caller running the frontier on a branch of a graph being captured:
  // forking the engine's stream off a capture branch -- not the capture's
  // origin -- made hipStreamEndCapture recurse without end, DESIGN.md §5
  // round 6; and a branch already off the critical path gains nothing from it)
  int frontier_fork_ok = 1;
  // PINSAGE_WGRAD_KW: weight gradients by the long-K kernel (wgrad.hip: 64 x 64
  // tiles, few splits combined inside the launch, Adam fused) instead of the
  // split-K GEMM + reduce_slabs_2d; 1 (default) every site it supports, 0 none
  int wgrad_kw = getenv("PINSAGE_WGRAD_KW") ? atoi(getenv("PINSAGE_WGRAD_KW")) : 1;
  // the side stream's long-K weight gradients run beside the chain's kernels:
  // PINSAGE_KW_SIDE_FORM 1 = the 64-KiB form (wgrad.hip), so a CU holding one
  // still takes the chain's workgroups; PINSAGE_KW_SIDE_WG = their grid target
  // (128: half the CUs, so the chain's dq / dY W launches beside them keep the
  // rest; C4 -4 us, C4 B 4096 -23 us, C2 / C3 even against 256)
  int kw_side_form = getenv("PINSAGE_KW_SIDE_FORM") ? atoi(getenv("PINSAGE_KW_SIDE_FORM")) : 0;
  int kw_side_wg = getenv("PINSAGE_KW_SIDE_WG") ? atoi(getenv("PINSAGE_KW_SIDE_WG")) : 128;
  // PINSAGE_DQ_TREE (default 1): rows of the transposed aggregation split over
  // several chunks are summed by their chunk waves as a fixed fan-in-8 tree
  // (conv.hip dq_tree_leaf) instead of by a dq_combine launch after them
  // (three interleaved pairs at C2, ms/step: 0.3949 / 0.3975 / 0.3985 with the
  // combine launch, 0.3872 / 0.3855 / 0.3939 without; C4 even)
  int dq_tree = getenv("PINSAGE_DQ_TREE") ? atoi(getenv("PINSAGE_DQ_TREE")) : 1;
  // the input feature table as hi / mid / lo bf16 planes [3][n][d_in]
  // (pinsage_engine_set_feature_planes; null: none): the layer-0 Q weight
  // gradient then runs on pre-split operands (wgrad_pl_kernel), the
  // transposed aggregation writing layer 0's dpq as planes too (lb.dpq3)
  const uint16_t* fplanes = nullptr;
  int64_t fplanes_ps = 0;
  // the input feature table as its interleaved split-bf16 table [n][ld >= 3
  // d_in] (pinsage_engine_set_feature_ilv; null: none): the layer-0 Q
  // projection then reads each gathered row's 16-k stage as one 96-B piece and
  // converts nothing (gemm.hip a_ilv), with Q0 split per step into the
  // workspace's table (qw_ilv) beside the W planes (fwd.wsplit)
  const uint16_t* f_ilv = nullptr;
  int64_t f_ilv_ld = 0;
  // PINSAGE_WGRAD_PLANES=1: carve layer 0's dpq planes buffer so the planes
  // form can run (default 0: measured no faster -- C2 dQ0 53.4 us fp32 8-wave
  // form vs 54.0 us on planes, tools/wgrad_bench.py, round 6: the 12-KiB
  // stages fit only 4 waves x 3 stages in LDS, and the 4-wave fp32 form is
  // 63.7 us; the split the planes save is ~10 us of it)
  int wgrad_planes = getenv("PINSAGE_WGRAD_PLANES") ? atoi(getenv("PINSAGE_WGRAD_PLANES")) : 0;
  // a deque: Timed scopes nest and hold pointers to their sites, which must
  // stay valid when an inner scope appends a new site
  std::deque<TimingSite> sites;
  // per-site GEMM tile / stream-K / split-K choices (pinsage_engine_set_gemm_choice:
  // set by the trainer's in-context tuner; absent = the launcher's size model)
  struct GemmChoice {
    int cfg = -1, stream_k = -1, splits = 0;
  };
  std::map<std::string, GemmChoice> choice;
  // per GEMM site: whether its last launch ran stream-K (the tuner keeps a
  // site's summation order: pinsage_engine_site_stream_k)
  std::map<std::string, int> sk_used;
  // pinsage_engine_set_fork: the next forward_layers call forks another
  // workspace's frontier onto `stream` right after the layer-0 Q projection
  struct Fork {
    hipStream_t stream = nullptr;
    void* ws = nullptr;
    const int64_t* ids = nullptr;
    int64_t n = 0;
  } fork;
  std::vector<LayerBuf> L;
  int64_t pG1w = 0, pG1b = 0, pG2w = 0, n_params = 0;
  // workspace layout
  size_t bits_begin = 0, bits_end = 0;  // all bitmaps contiguous (one memset)
  size_t tickets = 0;                    // (inside the bitmap region)
  size_t block_sums = 0, ids = 0, pos_rank = 0, H1 = 0, Z = 0, dZ = 0, dP1 = 0;
  size_t G = 0, Kc = 0, part = 0, scal = 0, slab = 0, bslab = 0, varpart = 0, hinge = 0;
  // the batch positions by top-set rank (pos_csr) and the deterministic
  // accumulation of repeated nodes' gradients (conv.hip det_put / rep_sum_kernel)
  size_t rank_off = 0, pos_sorted = 0, Gp = 0;
  size_t slab_main = 0, bslab_main = 0;  // split-K slabs of the main stream's weight gradient
  size_t qw_ilv = 0;                     // Q0's interleaved split table [hid][3 d_in] (f_ilv)
  int64_t slab_floats = 0;
  // stream-K scratch of the main stream's GEMMs (gemm.h)
  size_t sk_slab = 0, sk_cnt = 0;
  int64_t sk_cnt_len = 0;
  // long-K weight gradients' split tickets (wgrad.hip), per stream
  size_t kw_cnt_main = 0, kw_cnt_side = 0;
  int64_t kw_cnt_len = 0;
  size_t total = 0;
  int64_t max_bsum_blocks = 0;
  // external device pointers (owned by the caller)
  const float* feats = nullptr;
  int64_t ld_f = 0;
  const int32_t* nb = nullptr;
  const float* wn = nullptr;
  int64_t ldT = 0;
  float* params = nullptr;
  float* grads = nullptr;
  float* adam_m = nullptr;
  float* adam_v = nullptr;
  // backward side streams: [0] transposes (CSR) of the neighbour slots, [1]
  // weight gradients; forked from / joined to the caller's stream with events
  // [2]: the frontier's own fork (engine_frontier, PINSAGE_CSR_FORK): never
  // forked by the backward, so a step graph whose look-ahead branch holds the
  // next frontier does not fork one stream from two parallel branches
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  int side_dev = 0;  // the device side[] and ev were created on (the retired pool's key)
  std::vector<hipEvent_t> ev;
  int ev_next = 0;
  // PINSAGE_DEFER_SIDE bit 0: in the backward, a launch forked onto a side
  // stream is enqueued after the main chain's next launch (same dependences:
  // its wait binds to an event recorded at the fork point); bit 1: the loss
  // monitors likewise, after the head backward.  In a captured graph the
  // chain's child is then created before the side node, which keeps the chain
  // on one hardware queue instead of hopping at every fork.
  // Measured at C2 (bench.py, ms per step): 3 (default) 0.445-0.453, 1 0.456-0.461,
  // 0 (side launches before the chain's next launch) 0.498; the original order
  // (side launches after the chain's next launch, un-deferred only within the
  // backward's own code) 0.463.  Forking the monitors behind the head backward
  // instead of at the loss measured 0.483-0.491; fewer fork points (the head's
  // and each layer's W gradients forked together with the layer's Q gradient /
  // the optimizer pass) 0.454-0.467.
  // (round 6, with the long-K weight gradients: all side launches collected
  // behind ONE fork after layer 0's dcat launch measured slower -- C2 0.391-
  // 0.395 -> 0.424-0.425 ms, C4 0.422-0.429 -> 0.449-0.453: the side work
  // then ends after the chain)
  int defer_side = getenv("PINSAGE_DEFER_SIDE") ? atoi(getenv("PINSAGE_DEFER_SIDE")) : 3;
  std::vector<std::function<int()>> pend;  // deferred side launches, in order
  // PINSAGE_FORK_PLAN: every fork point on the chain costs the chain's next
  // launch ~5.5 us (the rocprofv3 step timeline: the node after a fork starts
  // late), so side launches are merged into fewer forks -- side work may
  // always start LATER than its inputs exist.  Bit 0: the loss monitors ride
  // on the head backward's fork instead of forking at the loss; bit 1: layer
  // l > 0's Q weight gradient rides on the next W-gradient fork (layer l-1's,
  // after its normalisation backward); bit 2: layer 0's W weight gradient (and
  // what rides with it) forks with the optimizer pass, after layer 0's dcat.
  int fork_plan = getenv("PINSAGE_FORK_PLAN") ? atoi(getenv("PINSAGE_FORK_PLAN")) : 0;
  // launches with no fork point of their own (fork_plan bit 0: the monitors),
  // enqueued on the side stream of the next fork, after its wait
  std::vector<std::function<int(hipStream_t)>> ride;
  hipStream_t ride_st = nullptr;  // the stream the riders are ordered behind
  // the on-the-fly step (pinsage_engine_set_fly, fly.hip): the virtual nodes
  // x0 .. x0 + *fly_nx - 1 join the top set, and the loss hands each the
  // summed G row of its real node fly_xids[j] (call fly_xids[j] / fly_unit)
  int64_t fly_x0 = 0, fly_unit = 1, fly_xcap = 0;
  const int* fly_nx = nullptr;
  const int64_t* fly_xids = nullptr;
  ~Engine();
};

// Streams and events of destroyed engines are retired to a process-wide pool
// and handed to the next engine that needs them, never released: a destroy
// may run while some stream of the process is being captured into a graph (a
// Python finaliser inside torch.cuda.graph), and releasing HIP streams /
// events there invalidates that capture (global capture mode).  An engine
// destroy therefore makes no HIP call at all.
// The pool is keyed by the device the streams and events were created on (an
// engine on another device must not inherit them).
static std::mutex g_retired_mu;
static std::map<int, std::vector<hipStream_t>> g_retired_streams;
static std::map<int, std::vector<hipEvent_t>> g_retired_events;
static std::atomic<int64_t> g_live_engines{0};

Engine::~Engine() {
  std::lock_guard<std::mutex> lk(g_retired_mu);
  for (auto& s : side)
    if (s) g_retired_streams[side_dev].push_back(s);
  for (auto& e : ev) g_retired_events[side_dev].push_back(e);
  // (timing events are bench-only: pinsage_engine_timing(e, 0) releases them)
  g_live_engines--;
}

// An event from the engine's pool (round-robin; a step records well under
// kEvents, and a wait binds to the record that precedes it on the host).
constexpr int kEvents = 32;
static int ensure_streams(Engine& E) {
  if (E.side[0]) return kOk;
  PS_TRY(csr_prepare());
  PS_CHECK_HIP(hipGetDevice(&E.side_dev));
  std::lock_guard<std::mutex> lk(g_retired_mu);
  auto& rs = g_retired_streams[E.side_dev];
  auto& re = g_retired_events[E.side_dev];
  for (auto& s : E.side) {
    if (!rs.empty()) {
      s = rs.back();
      rs.pop_back();
    } else {
      PS_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
  }
  E.ev.resize(kEvents);
  for (auto& e : E.ev) {
    if (!re.empty()) {
      e = re.back();
      re.pop_back();
    } else {
      PS_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
  }
  return kOk;
}
// `to` waits for everything enqueued so far on `from`
static int dep(Engine& E, hipStream_t from, hipStream_t to) {
  if (from == to) return kOk;
  hipEvent_t e = E.ev[(size_t)(E.ev_next++ % kEvents)];
  PS_CHECK_HIP(hipEventRecord(e, from));
  PS_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
  return kOk;
}

// Fork `fn` (launches on `to`) off `from` at this point: the wait on `to`
// binds to an event recorded on `from` now; with `defer` the launch itself
// waits in E.pend until run_pend (after the main chain's next launch).
static int fork_side(Engine& E, hipStream_t from, hipStream_t to, bool defer, std::function<int()> fn) {
  std::vector<std::function<int(hipStream_t)>> ride;
  if (from == E.ride_st) ride.swap(E.ride);  // (only a fork behind the riders' inputs)
  if (from == to) {
    for (auto& r : ride) PS_TRY(r(to));
    return fn();
  }
  hipEvent_t e = E.ev[(size_t)(E.ev_next++ % kEvents)];
  PS_CHECK_HIP(hipEventRecord(e, from));
  if (!defer) {
    PS_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
    for (auto& r : ride) PS_TRY(r(to));
    return fn();
  }
  E.pend.push_back([to, e, fn, ride]() -> int {
    PS_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
    for (auto& r : ride) PS_TRY(r(to));
    return fn();
  });
  return kOk;
}
// launches still riding (no fork has taken them): fork them now
static int flush_ride(Engine& E) {
  if (E.ride.empty()) return kOk;
  PS_TRY(ensure_streams(E));
  return fork_side(E, E.ride_st, E.side[0], false, []() -> int { return kOk; });
}
static int run_pend(Engine& E) {
  std::vector<std::function<int()>> v;
  v.swap(E.pend);
  for (auto& f : v) PS_TRY(f());
  return kOk;
}

struct Timed {
  Engine& E;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  TimingSite* site = nullptr;
  Timed(Engine& e, const std::string& name, hipStream_t s) : E(e), st(s) {
    if (!E.timing) return;
    for (auto& t : E.sites)
      if (t.name == name) site = &t;
    if (!site) {
      E.sites.push_back(TimingSite{name, {}, 0.0, 0});
      site = &E.sites.back();
    }
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, st);
  }
  void stop() {
    if (!site) return;
    (void)hipEventRecord(b, st);
    site->pending.emplace_back(a, b);
    site = nullptr;
  }
  ~Timed() { stop(); }
};

static std::string lname(const char* base, int l) { return std::string(base) + ".l" + std::to_string(l); }

// the tuner's choice for a GEMM site, if any
static void apply_choice(const Engine& E, const std::string& site, GemmParams& p) {
  auto it = E.choice.find(site);
  if (it == E.choice.end()) return;
  if (it->second.cfg >= 0) p.cfg = it->second.cfg;
  if (it->second.stream_k >= 0) p.stream_k = it->second.stream_k;
}

static size_t carve(size_t& cur, int64_t bytes) {
  cur = (size_t)align_up((int64_t)cur, 256);
  size_t at = cur;
  cur += (size_t)std::max<int64_t>(bytes, 0);
  return at;
}

// Split-K weight gradients (C[M][N] = A^T B over K data rows): pick the block
// tile and split count so that tiles x splits gives ~2 blocks per CU with >= 128
// rows per split (the slabs cost S*M*N*8 bytes of traffic, so no more splits than
// that); small outputs (128 x 128 head weights) fall back to 32 x 128 tiles.
constexpr int kMaxSplits = 64;
static void choose_wgrad(int64_t M, int64_t N, int64_t Kest, int* cfg, int* splits, int64_t target = 512) {
  static const int bm[3] = {128, 64, 32};
  for (int c = 0; c < 3; ++c) {
    const int64_t tiles = ((M + bm[c] - 1) / bm[c]) * ((N + 127) / 128);
    int64_t s = std::max<int64_t>(1, (target + tiles - 1) / tiles);
    s = std::min<int64_t>(s, std::max<int64_t>(1, Kest / 128));
    s = std::min<int64_t>(s, kMaxSplits);
    if (tiles * s >= 256 || c == 2) {
      *cfg = c;
      *splits = (int)s;
      return;
    }
  }
}

static void layout(Engine& E) {
  const EngineConfig& c = E.cfg;
  const int64_t n = c.n_items, Lc = c.n_layers, T = c.T;
  E.L.assign((size_t)Lc, LayerBuf());
  // capacities, top-down
  int64_t capS = std::min(n, c.max_pos);
  for (int64_t l = Lc - 1; l >= 0; --l) {
    LayerBuf& lb = E.L[(size_t)l];
    lb.d = (l == 0) ? c.d_in : c.out;
    lb.S.cap = capS;
    lb.N.cap = std::min(n, capS * T);
    capS = std::min(n, lb.N.cap + lb.S.cap);
  }
  // parameter offsets in state_dict order
  int64_t po = 0;
  for (int64_t l = 0; l < Lc; ++l) {
    LayerBuf& lb = E.L[(size_t)l];
    lb.pQw = po; po += c.hid * lb.d;
    lb.pQb = po; po += c.hid;
    lb.pWw = po; po += c.out * (lb.d + c.hid);
    lb.pWb = po; po += c.out;
  }
  E.pG1w = po; po += c.out * c.out;
  E.pG1b = po; po += c.out;
  E.pG2w = po; po += c.out * c.out;
  E.n_params = po;

  size_t cur = 0;
  const int64_t nw = bitset_words(n);
  E.max_bsum_blocks = bitset_blocks(n);
  E.bits_begin = carve(cur, 0);
  for (auto& lb : E.L) {
    lb.S.bits = carve(cur, nw * 8);
    lb.N.bits = carve(cur, nw * 8);
  }
  // the fused mark + finalise launches' tickets (zeroed with the bitmaps by
  // every step's first kernel, reset by their last blocks)
  E.tickets = carve(cur, std::max<int64_t>(Lc, 1) * 4);
  E.bits_end = carve(cur, 0);
  const int64_t scan_blocks = std::max<int64_t>(E.max_bsum_blocks, 1);
  E.block_sums = carve(cur, scan_blocks * 4);
  for (auto& lb : E.L) {
    for (SetBuf* sb : {&lb.S, &lb.N}) {
      sb->prefix = carve(cur, nw * 4);
      sb->members = carve(cur, sb->cap * 4);
      sb->count = carve(cur, 16);
    }
    const int64_t FS = lb.S.cap, FN = lb.N.cap;
    lb.self_src = carve(cur, FS * 4);
    lb.q_src = carve(cur, FN * 4);
    lb.loc = carve(cur, FS * T * 4);
    lb.wloc = carve(cur, FS * T * 4);
    lb.q = carve(cur, FN * c.hid * 4);
    lb.wplanes = carve(cur, agg_w_planes_bytes(lb.d, c.hid));
    lb.agg = carve(cur, FS * c.hid * 4);
    lb.y = carve(cur, FS * c.out * 4);
    lb.nrm = carve(cur, FS * 4);
    lb.dY = carve(cur, FS * c.out * 4);
    lb.dp = carve(cur, FS * c.out * 4);
    lb.dagg = carve(cur, FS * c.hid * 4);
    lb.dpq = carve(cur, FN * c.hid * 4);
    lb.cnt = carve(cur, (FN + 1) * 4);
    lb.bsum = carve(cur, (int64_t)ceil_div(FN + 1, 1024) * 8 + 16);
    lb.off = carve(cur, (FN + 1) * 4);
    lb.cursor = carve(cur, (FN + 1) * 4);
    lb.max_chunks = dq_chunk_capacity(FS, (int)T, FN);
    lb.cbase = carve(cur, (FN + 1) * 4);
    lb.occ2 = carve(cur, lb.max_chunks * 16 * 8);  // {row, weight} pairs, 16 per chunk
    lb.occ2b = carve(cur, lb.max_chunks * 16 * 8);  // (split rows' canonical reorder)
    lb.chunks = carve(cur, lb.max_chunks * 8);
    lb.nchunks = carve(cur, 16);
    lb.dqpart = carve(cur, lb.max_chunks * c.hid * 4);  // partials of split dq rows
    lb.csrc = carve(cur, lb.max_chunks * 4);
    lb.max_split = dq_split_capacity(FS, (int)T);
    lb.split = carve(cur, lb.max_split * 8);
    lb.nsplit = carve(cur, 16);
    lb.dqtk_len = (int64_t)dq_tree_levels(lb.max_chunks) * lb.max_chunks;
    lb.dqtk = carve(cur, lb.dqtk_len * 4);
    if (&lb == &E.L[0] && E.wgrad_planes) lb.dpq3 = carve(cur, 3 * FN * c.hid * 2);
  }
  const int64_t top = E.L.back().S.cap;
  E.qw_ilv = carve(cur, c.hid * 3 * E.L[0].d * 2);
  E.ids = carve(cur, c.max_pos * 8 + 16);  // + Adam coefficients staged behind the ids
  E.pos_rank = carve(cur, c.max_pos * 4);
  E.H1 = carve(cur, top * c.out * 4);
  E.Z = carve(cur, top * c.out * 4);
  E.dZ = carve(cur, top * c.out * 4);
  E.dP1 = carve(cur, top * c.out * 4);
  E.G = carve(cur, 3 * top * c.out * 4);
  E.Kc = carve(cur, 3 * top * 4);
  E.rank_off = carve(cur, (c.max_pos + 2) * 4);
  E.pos_sorted = carve(cur, c.max_pos * 4);
  E.Gp = carve(cur, c.max_pos * c.out * 4);
  E.part = carve(cur, (int64_t)(ceil_div(c.max_pos, 4) + 1) * 4 * 4);
  E.varpart = carve(cur, (int64_t)(ceil_div(c.max_pos, 4) + 1) * 2 * c.out * 4);  // (sum, M2)
  E.hinge = carve(cur, (c.max_pos / 3 + 1) * 4);  // per-triple hinge argument of the last loss
  E.scal = carve(cur, 64);
  // split-K slabs: any split count up to kMaxSplits (it is chosen from size hints)
  int64_t slab = kMaxSplits * c.out * c.out;
  for (auto& lb : E.L) {
    slab = std::max(slab, (int64_t)kMaxSplits * c.hid * lb.d);
    slab = std::max(slab, (int64_t)kMaxSplits * c.out * (lb.d + c.hid));  // merged [self || agg]
  }
  E.slab_floats = slab;
  E.slab = carve(cur, slab * 4);
  E.bslab = carve(cur, kMaxSplits * std::max(c.hid, c.out) * 4);
  E.slab_main = carve(cur, slab * 4);
  E.bslab_main = carve(cur, kMaxSplits * std::max(c.hid, c.out) * 4);
  {
    int64_t max_rows = 0, max_cols = std::max(c.hid, c.out);
    for (auto& lb : E.L) {
      max_rows = std::max({max_rows, lb.S.cap, lb.N.cap});
      max_cols = std::max(max_cols, lb.d + c.hid);
    }
    E.sk_cnt_len = ceil_div(max_rows, 32) * ceil_div(max_cols, 128);
    E.sk_cnt = carve(cur, E.sk_cnt_len * 4);
    E.sk_slab = carve(cur, gemm_sk_slab_floats() * 4);
    E.kw_cnt_len = (int64_t)ceil_div(std::max(c.hid, c.out), 64) * ceil_div(max_cols, 64);
    E.kw_cnt_main = carve(cur, E.kw_cnt_len * 4);
    E.kw_cnt_side = carve(cur, E.kw_cnt_len * 4);
  }
  E.total = (size_t)align_up((int64_t)cur, 256);
}

template <class T>
static inline T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

// main-stream GEMMs may run stream-K (launch_gemm decides by shape)
static inline void with_sk(const Engine& E, void* ws, GemmParams& p) {
  p.sk_slab = at<float>(ws, E.sk_slab);
  p.sk_cnt = at<int>(ws, E.sk_cnt);
  p.sk_cnt_len = E.sk_cnt_len;
}

// ---------------------------------------------------------------- forward
// The forward in two phases.  engine_frontier depends only on the ids and the
// neighbourhood table (never on parameters): the frontier sets of every layer
// and each layer's index tables (layer_prep, which also zeroes that step's dY
// scatter targets).  engine_layers runs the projections, aggregations and the
// head.  A trainer with two workspaces runs step i+1's frontier beside step
// i's backward (pinsage_training._FusedStep).
int engine_frontier(Engine& E, void* ws, const int64_t* ids_dev, int64_t n_pos, hipStream_t st,
                    bool with_csr = true) {
  const EngineConfig& c = E.cfg;
  PS_REQUIRE(E.feats && E.nb && E.wn && E.params, kErrArg, "engine: pointers not set");
  PS_REQUIRE(n_pos > 0 && n_pos <= c.max_pos, kErrArg, "engine: n_pos out of range");
  const int Lc = (int)c.n_layers, T = (int)c.T;
  const int64_t n = c.n_items;
  if (ids_dev != at<int64_t>(ws, E.ids))
    PS_CHECK_HIP(hipMemcpyAsync(at<int64_t>(ws, E.ids), ids_dev, (size_t)n_pos * 8,
                                hipMemcpyDeviceToDevice, st));
  const int64_t* ids = at<int64_t>(ws, E.ids);
  uint32_t* bsum = at<uint32_t>(ws, E.block_sums);
  auto bits = [&](const SetBuf& s) { return at<unsigned long long>(ws, s.bits); };
  auto pref = [&](const SetBuf& s) { return at<uint32_t>(ws, s.prefix); };
  auto mem = [&](const SetBuf& s) { return at<int32_t>(ws, s.members); };
  auto cnt = [&](const SetBuf& s) { return at<int>(ws, s.count); };

  // frontier, top-down
  LayerBuf& top = E.L[(size_t)Lc - 1];
  Timed t_front(E, "fwd.frontier", st);
  // One kernel zeroes all of the step's bitmaps, marks the ids (range-checked
  // by the caller) and finalises the top set.  Captured step graphs stay
  // kernel-only: a memset node at the head of a replayed graph was not ordered
  // behind the previous replay's kernels on this stack (back-to-back replays
  // faulted; synchronised ones did not).
  PS_TRY(launch_top_set(at<unsigned long long>(ws, E.bits_begin),
                        (int64_t)(E.bits_end - E.bits_begin) / 8, bits(top.S), ids, n_pos, n, bsum,
                        pref(top.S), mem(top.S), cnt(top.S), st, E.fly_x0, E.fly_nx));
  for (int l = Lc - 1; l >= 0; --l) {
    LayerBuf& lb = E.L[(size_t)l];
    const int32_t* nb_l = lb.nb_tab ? lb.nb_tab : E.nb;
    const int64_t ld_l = lb.nb_tab ? lb.ld_tab : E.ldT;
    if (mark_finalize_fits(n) && lb.S.cap > 0) {  // one launch: mark N_l, finalise N_l and S_{l-1}
      LayerBuf* lo = l > 0 ? &E.L[(size_t)l - 1] : nullptr;
      PS_TRY(launch_mark_finalize(bits(lb.N), mem(lb.S), cnt(lb.S), lb.S.cap, nb_l, ld_l, T, n,
                                  at<int>(ws, E.tickets) + l, pref(lb.N), mem(lb.N), cnt(lb.N),
                                  lo ? bits(lo->S) : nullptr, bits(lb.S), lo ? pref(lo->S) : nullptr,
                                  lo ? mem(lo->S) : nullptr, lo ? cnt(lo->S) : nullptr, st));
      continue;
    }
    PS_TRY(launch_mark_table(bits(lb.N), mem(lb.S), cnt(lb.S), lb.S.cap, nb_l, ld_l, T, n, st));
    PS_TRY(launch_set_finalize(bits(lb.N), bits(lb.N), nullptr, n, bsum, pref(lb.N), mem(lb.N),
                               cnt(lb.N), st));
    if (l > 0) {
      LayerBuf& lo = E.L[(size_t)l - 1];
      PS_TRY(launch_set_finalize(bits(lo.S), bits(lb.N), bits(lb.S), n, bsum, pref(lo.S), mem(lo.S),
                                 cnt(lo.S), st));
    }
  }
  // index tables of every layer, one launch
  {
    LayerPrep pp[kMaxPrepLayers];
    int64_t smax[kMaxPrepLayers], nmax[kMaxPrepLayers];
    PS_REQUIRE(Lc <= kMaxPrepLayers, kErrArg, "engine: at most 4 layers");
    for (int l = 0; l < Lc; ++l) {
      LayerBuf& lb = E.L[(size_t)l];
      const SetBuf* prev = l > 0 ? &E.L[(size_t)l - 1].S : nullptr;
      const bool is_top = l == Lc - 1;  // the top layer also ranks the batch positions
      LayerPrep& p = pp[l];
      p.S_mem = mem(lb.S);
      p.nS = cnt(lb.S);
      p.N_mem = mem(lb.N);
      p.nN = cnt(lb.N);
      p.N_bits = bits(lb.N);
      p.N_pref = pref(lb.N);
      p.P_bits = prev ? bits(*prev) : nullptr;
      p.P_pref = prev ? pref(*prev) : nullptr;
      p.nb = lb.nb_tab ? lb.nb_tab : E.nb;
      p.wn = lb.nb_tab ? lb.wn_tab : E.wn;
      p.ldT = lb.nb_tab ? lb.ld_tab : E.ldT;
      p.self_src = at<int32_t>(ws, lb.self_src);
      p.q_src = at<int32_t>(ws, lb.q_src);
      p.loc = at<int32_t>(ws, lb.loc);
      p.wloc = at<float>(ws, lb.wloc);
      p.S_bits = bits(top.S);
      p.S_pref = pref(top.S);
      p.ids = ids;
      p.n_ids = is_top ? n_pos : 0;
      p.pos_rank = at<int32_t>(ws, E.pos_rank);
      p.z = prev ? at<float>(ws, E.L[(size_t)l - 1].dY) : nullptr;
      p.z_n = (int)c.out;
      p.z_rows = prev ? cnt(*prev) : nullptr;
      smax[l] = lb.S.cap;
      nmax[l] = lb.N.cap;
    }
    PS_TRY(launch_layer_preps(pp, smax, nmax, Lc, T, st));
    PS_TRY(launch_pos_csr(at<int32_t>(ws, E.pos_rank), n_pos, cnt(top.S), at<int>(ws, E.rank_off),
                          at<int32_t>(ws, E.pos_sorted), st));
  }
  // the transposes of the neighbour slots (CSR of slot occurrences by q row,
  // the aggregation backward's plan) depend only on the frontier: built here,
  // on the frontier's stream -- for a trainer's look-ahead frontier that is
  // beside the previous step, so the backward never waits for them.  An
  // inference forward (no backward will follow) skips them.
  if (!with_csr) return kOk;
  PS_TRY(csr_prepare());
  // (PINSAGE_CSR_FORK) the fork's wait binds to an event recorded on st here,
  // after the index tables the CSR builds read; the join below is recorded on
  // side[0] after its last launch and waited on st before this call returns
  hipStream_t s_fk = st;
  const int csr_fork = E.frontier_fork_ok ? E.csr_fork : 0;
  if (csr_fork) {
    PS_TRY(ensure_streams(E));
    s_fk = E.side[std::min(std::max(E.csr_fork_stream, 0), 2)];
    PS_TRY(dep(E, st, s_fk));
  }
  for (int l = Lc - 1; l >= 0; --l) {
    LayerBuf& lb = E.L[(size_t)l];
    hipStream_t sl = (csr_fork == 1 && l == 0) ? s_fk : st;
    Timed tc(E, lname("fwd.csr", l), sl);
    PS_TRY(launch_csr_build(at<int32_t>(ws, lb.loc), at<float>(ws, lb.wloc), cnt(lb.S), lb.S.cap, T, cnt(lb.N),
                            lb.N.cap, at<int>(ws, lb.cnt), at<int>(ws, lb.bsum), at<int>(ws, lb.off),
                            at<int>(ws, lb.cursor), at<int>(ws, lb.cbase), at<int2>(ws, lb.occ2),
                            at<int2>(ws, lb.chunks), at<int>(ws, lb.nchunks), at<int2>(ws, lb.split),
                            at<int>(ws, lb.nsplit), at<float>(ws, lb.dpq), (int)c.hid, sl,
                            at<int2>(ws, lb.occ2b)));
  }
  if (csr_fork) PS_TRY(dep(E, s_fk, st));  // join: nothing of this call stays on side[0]
  return kOk;
}

int engine_layers(Engine& E, void* ws, hipStream_t st) {
  const EngineConfig& c = E.cfg;
  PS_REQUIRE(E.feats && E.nb && E.wn && E.params, kErrArg, "engine: pointers not set");
  const int Lc = (int)c.n_layers, T = (int)c.T;
  auto cnt = [&](const SetBuf& s) { return at<int>(ws, s.count); };
  LayerBuf& top = E.L[(size_t)Lc - 1];
  // W of every layer whose aggregation + W kernel runs pipelined split once
  // into its fragment-order bf16 planes
  std::vector<int> wp((size_t)Lc, 0), next_q((size_t)Lc, 0);
  for (int l = 0; E.fused_aggw && E.fused_next_q && l + 1 < Lc; ++l) {
    const LayerBuf& lb = E.L[(size_t)l];
    const int64_t S_est = lb.S.hint > 0 ? std::min(lb.S.hint, lb.S.cap) : lb.S.cap;
    next_q[(size_t)l] = E.fused_next_q > 0 || agg_w_next_q_pays(lb.d, c.hid, T, S_est);
  }
  if (E.fused_aggw) {
    Timed ts(E, "fwd.wsplit", st);
    for (int l = 0; l < Lc; ++l) {
      LayerBuf& lb = E.L[(size_t)l];
      const int64_t S_est = lb.S.hint > 0 ? std::min(lb.S.hint, lb.S.cap) : lb.S.cap;
      if (!agg_w_supported(lb.d, c.hid, c.out, T) || !agg_w_uses_planes(lb.d, c.hid, c.out, T, S_est)) continue;
      wp[(size_t)l] = 1;
      PS_TRY(launch_split_wplanes(E.params + lb.pWw, lb.d + c.hid, (int)(lb.d + c.hid), at<uint16_t>(ws, lb.wplanes),
                                  st));
    }
  }
  // Q0 on the feature table's interleaved split (f_ilv): Q0 split per step
  const bool q0_ilv = E.f_ilv && E.L[0].d % 16 == 0;
  if (q0_ilv) {
    Timed ts(E, "fwd.wsplit_q", st);
    PS_TRY(launch_split_ilv(E.params + E.L[0].pQw, E.L[0].d, c.hid, (int)E.L[0].d, at<uint16_t>(ws, E.qw_ilv),
                            3 * E.L[0].d, st));
  }
  int q_done = 0;  // this layer's q rows came out of the layer below's kernel (AggNextQ)
  int head_done = 0;  // the head ran inside the top layer's kernel (AggHead)
  for (int l = 0; l < Lc; ++l) {
    LayerBuf& lb = E.L[(size_t)l];
    const float* h = l == 0 ? E.feats : at<float>(ws, E.L[(size_t)l - 1].y);
    const int64_t ldh = l == 0 ? E.ld_f : c.out;
    // Q projection of the distinct neighbours: lrelu(h[u] Q^T + b)
    if (!q_done) {
    GemmParams q;
    q.M_dev = cnt(lb.N);
    q.M_hint = (int)lb.N.hint;
    q.M_max = (int)lb.N.cap;
    q.N = (int)c.hid;
    q.K = (int)lb.d;
    q.a = h;
    q.lda = ldh;
    q.a_idx = at<int32_t>(ws, lb.q_src);
    q.b = E.params + lb.pQw;
    q.ldb = lb.d;
    q.c = at<float>(ws, lb.q);
    q.ldc = c.hid;
    q.bias = E.params + lb.pQb;
    q.act = true;
    if (l == 0 && q0_ilv) {
      q.a_ilv = E.f_ilv;
      q.lda_ilv = E.f_ilv_ld;
      q.b_ilv = at<uint16_t>(ws, E.qw_ilv);
      q.ldb_ilv = 3 * lb.d;
    }
    {
      Timed tt(E, lname("fwd.q_gemm", l), st);
      with_sk(E, ws, q);
      apply_choice(E, lname("fwd.q_gemm", l), q);
      PS_TRY(launch_gemm(q, st));
      E.sk_used[lname("fwd.q_gemm", l)] = gemm_last_stream_k();
    }
    }
    q_done = 0;
    if (l == 0 && E.fork.stream) {  // the next batch's frontier beside the rest of the step
      PS_TRY(ensure_streams(E));
      PS_TRY(dep(E, st, E.fork.stream));
      const int ok = E.frontier_fork_ok;
      E.frontier_fork_ok = 0;  // (no fork off this branch: frontier_fork_ok)
      const int rc = engine_frontier(E, E.fork.ws, E.fork.ids, E.fork.n, E.fork.stream);
      E.frontier_fork_ok = ok;
      PS_TRY(rc);
    }
    if (E.fused_aggw && agg_w_supported(lb.d, c.hid, c.out, T)) {
      // aggregation + [h_self || agg] W^T + bias, lrelu, row L2 norm in one launch
      Timed taw(E, lname("fwd.aggw", l), st);
      const int64_t S_est = lb.S.hint > 0 ? std::min(lb.S.hint, lb.S.cap) : lb.S.cap;
      AggNextQ nx;
      if (next_q[(size_t)l]) {  // the next layer's neighbours are rows of this y
        const LayerBuf& nb = E.L[(size_t)l + 1];
        nx.S_mem = at<int32_t>(ws, lb.S.members);
        nx.bits = at<unsigned long long>(ws, nb.N.bits);
        nx.pref = at<uint32_t>(ws, nb.N.prefix);
        nx.Qw = E.params + nb.pQw;
        nx.Qb = E.params + nb.pQb;
        nx.q = at<float>(ws, nb.q);
        nx.hid = (int)c.hid;
      }
      AggHead hd;
      if (l == Lc - 1 && E.fused_head && E.head_in_aggw) {
        hd.G1w = E.params + E.pG1w;
        hd.G1b = E.params + E.pG1b;
        hd.G2w = E.params + E.pG2w;
        hd.H1 = at<float>(ws, E.H1);
        hd.Z = at<float>(ws, E.Z);
      }
      PS_TRY(launch_agg_w(h, ldh, (int)lb.d, at<int32_t>(ws, lb.self_src), at<float>(ws, lb.q),
                          (int)c.hid, at<int32_t>(ws, lb.loc), at<float>(ws, lb.wloc), T, cnt(lb.S), 0,
                          S_est, E.params + lb.pWw, E.params + lb.pWb, at<float>(ws, lb.y),
                          at<float>(ws, lb.nrm), at<float>(ws, lb.agg), st, nx.q ? &nx : nullptr, &q_done,
                          wp[(size_t)l] ? at<uint16_t>(ws, lb.wplanes) : nullptr, wp[(size_t)l],
                          hd.G1w ? &hd : nullptr, &head_done));
      continue;
    }
    Timed t_agg(E, lname("fwd.agg", l), st);
    PS_TRY(launch_agg(at<float>(ws, lb.q), (int)c.hid, at<int32_t>(ws, lb.loc),
                      at<float>(ws, lb.wloc), T, cnt(lb.S), lb.S.cap, at<float>(ws, lb.agg), st));
    t_agg.stop();
    // W projection of [h_self || agg] with bias, lrelu and row L2 norm fused
    GemmParams w;
    w.M_dev = cnt(lb.S);
    w.M_hint = (int)lb.S.hint;
    w.M_max = (int)lb.S.cap;
    w.N = (int)c.out;
    w.K = (int)(lb.d + c.hid);
    w.a = h;
    w.lda = ldh;
    w.a_idx = at<int32_t>(ws, lb.self_src);
    w.K1 = (int)lb.d;
    w.a2 = at<float>(ws, lb.agg);
    w.lda2 = c.hid;
    w.b = E.params + lb.pWw;
    w.ldb = lb.d + c.hid;
    w.c = at<float>(ws, lb.y);
    w.ldc = c.out;
    w.bias = E.params + lb.pWb;
    w.epi = kEpiL2Norm;
    w.norms = at<float>(ws, lb.nrm);
    Timed tw(E, lname("fwd.w_gemm", l), st);
    with_sk(E, ws, w);
    apply_choice(E, lname("fwd.w_gemm", l), w);
    PS_TRY(launch_gemm(w, st));
    E.sk_used[lname("fwd.w_gemm", l)] = gemm_last_stream_k();
  }
  // head: G2(lrelu(G1 y))
  if (head_done) return kOk;
  Timed t_head(E, "fwd.head", st);
  if (E.fused_head)
    return launch_head_fwd(at<float>(ws, top.y), (int)c.out, cnt(top.S), top.S.cap,
                           E.params + E.pG1w, E.params + E.pG1b, E.params + E.pG2w,
                           at<float>(ws, E.H1), at<float>(ws, E.Z), st);
  GemmParams g1;
  g1.M_dev = cnt(top.S);
  g1.M_hint = (int)top.S.hint;
  g1.M_max = (int)top.S.cap;
  g1.N = (int)c.out;
  g1.K = (int)c.out;
  g1.a = at<float>(ws, top.y);
  g1.lda = c.out;
  g1.b = E.params + E.pG1w;
  g1.ldb = c.out;
  g1.c = at<float>(ws, E.H1);
  g1.ldc = c.out;
  g1.bias = E.params + E.pG1b;
  g1.act = true;
  PS_TRY(launch_gemm(g1, st));
  GemmParams g2 = g1;
  g2.a = at<float>(ws, E.H1);
  g2.b = E.params + E.pG2w;
  g2.c = at<float>(ws, E.Z);
  g2.bias = nullptr;
  g2.act = false;
  return launch_gemm(g2, st);
}

int engine_forward(Engine& E, void* ws, const int64_t* ids_dev, int64_t n_pos, hipStream_t st,
                   bool with_csr = true) {
  PS_TRY(engine_frontier(E, ws, ids_dev, n_pos, st, with_csr));
  return engine_layers(E, ws, st);
}

// Weight gradient dst[M][N] = A^T [B || B2] over the device row count (split-K
// slabs + one reduction); B2 (columns >= N1) is torch.cat's second operand.  If
// dst_b is set, the bias gradient dst_b[M] = column sums of A comes out of the
// same GEMM (bias_part) and the same reduction.
struct WGrad {
  const float* A = nullptr;
  int64_t lda = 0;
  int M = 0;
  const float* B = nullptr;
  int64_t ldb = 0;
  const int32_t* b_idx = nullptr;
  int N1 = -1;
  const float* B2 = nullptr;
  int64_t ldb2 = 0;
  int N = 0;
  const int* K_dev = nullptr;
  int64_t K_max = 0, K_hint = 0;
  float* dst = nullptr;
  int64_t ld_dst = 0;
  float* dst_b = nullptr;
  // pre-split operands (wgrad.hip wgrad_pl_kernel): both set, or neither
  const uint16_t* A3 = nullptr;
  int64_t a3_ps = 0;
  const uint16_t* B3 = nullptr;
  int64_t b3_ps = 0;
};

// Adam applied by the gradient reductions (pinsage_engine_backward_adam)
struct AdamStep {
  const float* coef;
  double beta1, beta2;
  float eps;
};

// Adam slice of the parameter at flat offsets (w_off, b_off); b_off < 0: none
static AdamSlice adam_slice(const Engine& E, const AdamStep& a, int64_t w_off, int64_t b_off) {
  AdamSlice s;
  s.p = E.params + w_off;
  s.m = E.adam_m + w_off;
  s.v = E.adam_v + w_off;
  if (b_off >= 0) {
    s.pb = E.params + b_off;
    s.mb = E.adam_m + b_off;
    s.vb = E.adam_v + b_off;
  }
  s.coef = a.coef;
  s.beta1 = a.beta1;
  s.beta2 = a.beta2;
  s.eps = a.eps;
  return s;
}

// after_use: with Adam fused, the reduction (which updates the parameter)
// waits for this event, recorded behind the main stream's last read of it
// main: the launch runs on the main stream (its own slabs; the
// weight-gradient stream may be using the others meanwhile)
static int weight_grad(Engine& E, void* ws, const WGrad& w, hipStream_t st, const std::string& site,
                       const AdamSlice* adam = nullptr, hipEvent_t after_use = nullptr,
                       bool main = false, bool beside = false) {
  float* const slab = at<float>(ws, main ? E.slab_main : E.slab);
  float* const bslab = at<float>(ws, main ? E.bslab_main : E.bslab);
  if (E.wgrad_kw && wgrad_kw_supported(w.M, w.N, w.N1, w.B2 != nullptr) &&
      (int64_t)(w.M / 64) * (w.N / 64) <= E.kw_cnt_len) {
    // the long-K kernel: splits combined in the launch, Adam fused (no
    // reduce_slabs_2d launch, no slab round trip through a second kernel)
    KwParams k;
    k.A = w.A;
    k.lda = w.lda;
    k.M = w.M;
    k.B = w.B;
    k.ldb = w.ldb;
    k.b_idx = w.b_idx;
    if (w.B2) {
      k.N1 = w.N1;
      k.B2 = w.B2;
      k.ldb2 = w.ldb2;
    }
    k.N = w.N;
    k.K_dev = w.K_dev;
    k.K_max = (int)w.K_max;
    k.dst = w.dst;
    k.ld_dst = w.ld_dst;
    k.dst_b = w.dst_b;
    k.A3 = w.A3;
    k.a3_ps = w.a3_ps;
    k.B3 = w.B3;
    k.b3_ps = w.b3_ps;
    if (adam) k.ad = *adam;
    k.slab = slab;
    k.bslab = bslab;
    k.cnt = at<int>(ws, main ? E.kw_cnt_main : E.kw_cnt_side);
    k.form = main ? 0 : E.kw_side_form;  // (the main stream's dQ0 in the 64-KiB form: 0.391 -> 0.401 ms at C2)
    k.S = wgrad_kw_splits(w.M, w.N, w.K_hint > 0 ? std::min(w.K_hint, w.K_max) : w.K_max,
                          main ? 256 : E.kw_side_wg);
    PS_REQUIRE((int64_t)k.S * w.M * w.N <= E.slab_floats, kErrWorkspace, "engine: wgrad slab too small");
    if (adam && after_use) PS_CHECK_HIP(hipStreamWaitEvent(st, after_use, 0));
    return launch_wgrad_kw(k, st);
  }
  PS_REQUIRE(!w.A3 && !w.B3, kErrArg, "engine: pre-split operands need the long-K weight-gradient kernel");
  int cfg = 0, S = 1;
  // (a side-stream target of 256 workgroups measured faster at C2 and slower
  // at C4, 128 slower, and a grid cap on side launches even or slower: one
  // target for both)
  choose_wgrad(w.M, w.N, w.K_hint > 0 ? std::min(w.K_hint, w.K_max) : w.K_max, &cfg, &S);
  {
    auto it = E.choice.find(site);
    if (it != E.choice.end()) {
      if (it->second.cfg >= 0) cfg = it->second.cfg;
      if (it->second.splits > 0) S = std::min(it->second.splits, kMaxSplits);
    }
  }
  GemmParams p;
  p.cfg = cfg;
  p.M = w.M;
  p.N = w.N;
  p.K_dev = w.K_dev;
  p.K_max = (int)w.K_max;
  p.a_kmajor = false;
  p.a = w.A;
  p.lda = w.lda;
  p.b_kmajor = false;
  p.b = w.B;
  p.ldb = w.ldb;
  p.b_idx = w.b_idx;
  if (w.B2) {
    p.N1 = w.N1;
    p.b2 = w.B2;
    p.ldb2 = w.ldb2;
  }
  p.c = slab;
  p.ldc = w.N;
  p.epi = kEpiPartial;
  p.splits = S;
  p.bias_part = w.dst_b ? bslab : nullptr;
  PS_REQUIRE((int64_t)S * w.M * w.N <= E.slab_floats, kErrWorkspace, "engine: split-K slab too small");
  PS_TRY(launch_gemm(p, st));
  if (adam && after_use) PS_CHECK_HIP(hipStreamWaitEvent(st, after_use, 0));
  return launch_reduce_slabs_2d(slab, S, (int64_t)w.M * w.N, w.M, w.N, w.dst,
                                w.ld_dst, p.bias_part, w.dst_b, adam, st);
}

// ---------------------------------------------------------------- backward
// Starts from dZ (gradient of the head output rows of the unique top nodes).
// The last gradient, dQ of layer 0, depends on the end of the main chain, so
// it runs on the main stream itself (no cross-queue hop at the step's tail).
// adam != nullptr: the step ends with torch.optim.Adam: Q0's reduction applies
// Q0's Adam itself, and the weight-gradient stream updates every other
// parameter (contiguous behind Q0 in the flat layout) once the main stream has
// read W0 for the last time -- the optimizer pass is off the critical path.
// stage -1: the whole backward; 0: the head and layers L-1 .. 1 (every
// gradient but layer 0's is complete when the call's stream reaches its end);
// 1: layer 0 (after a stage-0 call on the same workspace).  A data-parallel
// step all-reduces stage 0's gradients while stage 1 runs.
int engine_backward(Engine& E, void* ws, hipStream_t st, const AdamStep* adam, int stage = -1) {
  const EngineConfig& c = E.cfg;
  PS_REQUIRE(E.grads, kErrArg, "engine: grad buffer not set");
  PS_REQUIRE(!adam || (E.adam_m && E.adam_v), kErrArg, "engine: optimizer state not set");
  const LayerBuf& l0 = E.L[0];
  PS_REQUIRE(!adam || (l0.pQw == 0 && l0.pQb == l0.pQw + c.hid * l0.d && l0.pWw == l0.pQb + c.hid),
             kErrArg, "engine: Q0 must lead the flat parameter layout");
  const int Lc = (int)c.n_layers;
  auto cnt = [&](const SetBuf& s) { return at<int>(ws, s.count); };
  LayerBuf& top = E.L[(size_t)Lc - 1];
  const int o = (int)c.out, hd = (int)c.hid;
  float* gr = E.grads;
  PS_TRY(ensure_streams(E));
  hipStream_t s_csr = E.side[0], s_wg = E.side[1];
  hipStream_t s_wg0 = s_wg;
  // the CSR transposes were built with the frontier (engine_frontier)
  // weight gradients run on s_wg, each forked once its inputs exist on st
  const bool dfr = (E.defer_side & 1) != 0;
  PS_REQUIRE(stage < 0 || !adam, kErrArg, "engine: a staged backward runs without the fused optimizer");
  // side launches waiting for a later fork (E.fork_plan bits 1, 2): every
  // fork_late takes them along, ahead of its own launch
  std::vector<std::function<int()>> late;
  auto fork_late = [&](hipStream_t to, std::function<int()> fn) -> int {
    std::vector<std::function<int()>> v;
    v.swap(late);
    if (v.empty()) return fork_side(E, st, to, dfr, fn);
    return fork_side(E, st, to, dfr, [v, fn]() -> int {
      for (auto& f : v) PS_TRY(f());
      return fn();
    });
  };
  if (stage <= 0) {
  Timed t_hb(E, "bwd.head", st);
  auto wgrad_g2 = [&]() -> int {  // dG2 = dZ^T H1 beside the chain
    Timed tw(E, "bwd.wgrad.g2", s_wg);
    WGrad w;
    w.A = at<float>(ws, E.dZ);
    w.lda = o;
    w.M = o;
    w.B = at<float>(ws, E.H1);
    w.ldb = o;
    w.N = o;
    w.K_dev = cnt(top.S);
    w.K_max = top.S.cap;
    w.K_hint = top.S.hint;
    w.dst = gr + E.pG2w;
    w.ld_dst = o;
    return weight_grad(E, ws, w, s_wg, "bwd.wgrad.g2", nullptr, nullptr, false, s_wg != st);
  };
  if (!E.fused_head) {  // dZ exists (dz_combine): fork dG2 before the head backward
    PS_TRY(dep(E, st, s_wg));
    PS_TRY(wgrad_g2());
  }
  // dP1 = (dZ G2) * lrelu'(H1), dY_top = dP1 G1 and the top layer's
  // normalisation backward (dp_top) in one kernel, which also zeroes the
  // loss's multiplicity counters (the dY scatter-add targets of the layers
  // below were zeroed by the forward's layer_prep)
  if (E.fused_head) {
    // the head backward forms dZ = sum_c K[c] G[c] from the loss's
    // accumulators as it loads its rows (and zeroes them), writing dZ for dG2
    PS_TRY(launch_head_bwd(at<float>(ws, E.G), at<int>(ws, E.Kc), top.S.cap, at<float>(ws, E.dZ), o,
                           cnt(top.S), top.S.cap, at<float>(ws, E.H1), E.params + E.pG1w,
                           E.params + E.pG2w, at<float>(ws, top.y), at<float>(ws, top.nrm),
                           at<float>(ws, E.dP1), at<float>(ws, top.dp), at<int>(ws, E.rank_off),
                           at<int32_t>(ws, E.pos_sorted), E.reps_in_gp ? at<float>(ws, E.Gp) : nullptr, st));
    PS_TRY(run_pend(E));  // the loss monitors (PINSAGE_DEFER_SIDE bit 1)
    PS_TRY(fork_late(s_wg, wgrad_g2));
  } else {
    GemmParams p;  // dP1 = (dZ G2) * lrelu'(H1)
    p.M_dev = cnt(top.S);
    p.M_hint = (int)top.S.hint;
    p.M_max = (int)top.S.cap;
    p.N = o;
    p.K = o;
    p.a = at<float>(ws, E.dZ);
    p.lda = o;
    p.b_kmajor = false;
    p.b = E.params + E.pG2w;
    p.ldb = o;
    p.c = at<float>(ws, E.dP1);
    p.ldc = o;
    p.mask = at<float>(ws, E.H1);
    p.ldm = o;
    PS_TRY(launch_gemm(p, st));
    PS_TRY(run_pend(E));
    GemmParams q = p;  // dY_top = dP1 G1
    q.a = at<float>(ws, E.dP1);
    q.b = E.params + E.pG1w;
    q.c = at<float>(ws, top.dY);
    q.mask = nullptr;
    PS_TRY(launch_gemm(q, st));
    PS_TRY(launch_norm_lrelu_bwd(at<float>(ws, top.y), at<float>(ws, top.nrm),
                                 at<float>(ws, top.dY), o, cnt(top.S), top.S.cap,
                                 at<float>(ws, top.dp), nullptr, o, nullptr, at<int>(ws, E.Kc),
                                 3 * top.S.cap, st));
  }
  {
    WGrad w;  // dG1 and db1
    w.A = at<float>(ws, E.dP1);
    w.lda = o;
    w.M = o;
    w.B = at<float>(ws, top.y);
    w.ldb = o;
    w.N = o;
    w.K_dev = cnt(top.S);
    w.K_max = top.S.cap;
    w.K_hint = top.S.hint;
    w.dst = gr + E.pG1w;
    w.ld_dst = o;
    w.dst_b = gr + E.pG1b;
    PS_TRY(fork_late(s_wg, [&E, ws, w, s_wg, st]() -> int {
      Timed tw(E, "bwd.wgrad.g1", s_wg);
      return weight_grad(E, ws, w, s_wg, "bwd.wgrad.g1", nullptr, nullptr, false, s_wg != st);
    }));
  }
  t_hb.stop();
  }
  for (int l = Lc - 1; l >= 0; --l) {
    if ((stage == 0 && l == 0) || (stage == 1 && l != 0)) continue;
    Timed tb(E, lname("bwd.layer", l), st);
    LayerBuf& lb = E.L[(size_t)l];
    const int d = (int)lb.d;
    const float* h = l == 0 ? E.feats : at<float>(ws, E.L[(size_t)l - 1].y);
    const int64_t ldh = l == 0 ? E.ld_f : c.out;
    float* dp = at<float>(ws, lb.dp);
    float* dYprev = l > 0 ? at<float>(ws, E.L[(size_t)l - 1].dY) : nullptr;
    // dp = d(normalize(lrelu(.))); the top layer's came out of the head backward
    if (l < Lc - 1)
      PS_TRY(launch_norm_lrelu_bwd(at<float>(ws, lb.y), at<float>(ws, lb.nrm), at<float>(ws, lb.dY),
                                   o, cnt(lb.S), lb.S.cap, dp, nullptr, o, nullptr, nullptr, 0, st));
    hipStream_t s_w = l == 0 ? s_wg0 : s_wg;
    if (l < Lc - 1) PS_TRY(run_pend(E));  // behind the normalisation backward
    WGrad w_wgrad;
    {
      WGrad w;  // dW = dp^T [h_self || agg], dWb = colsum(dp)
      w.A = dp;
      w.lda = o;
      w.M = o;
      w.B = h;
      w.ldb = ldh;
      w.b_idx = at<int32_t>(ws, lb.self_src);
      w.N1 = d;
      w.B2 = at<float>(ws, lb.agg);
      w.ldb2 = hd;
      w.N = d + hd;
      w.K_dev = cnt(lb.S);
      w.K_max = lb.S.cap;
      w.K_hint = lb.S.hint;
      w.dst = gr + lb.pWw;
      w.ld_dst = d + hd;
      w.dst_b = gr + lb.pWb;
      w_wgrad = w;
    }
    {
      // [d_self || d_agg] = dp W: columns < d scatter-add into the rows of
      // layer l-1 (l > 0), columns >= d go to dagg
      GemmParams p;
      p.M_dev = cnt(lb.S);
      p.M_hint = (int)lb.S.hint;
      p.M_max = (int)lb.S.cap;
      p.K = o;
      p.a = dp;
      p.lda = o;
      p.b_kmajor = false;
      p.ldb = d + hd;
      if (l > 0) {
        p.N = d + hd;
        p.b = E.params + lb.pWw;
        p.c = dYprev;
        p.ldc = o;
        p.c_idx = at<int32_t>(ws, lb.self_src);
        p.epi = kEpiAccum;
        p.N1 = d;
        p.c2 = at<float>(ws, lb.dagg);
        p.ldc2 = hd;
      } else {
        p.N = hd;
        p.b = E.params + lb.pWw + d;
        p.c = at<float>(ws, lb.dagg);
        p.ldc = hd;
      }
      with_sk(E, ws, p);
      apply_choice(E, lname("bwd.dcat", l), p);
      // the W gradient forks before this launch (it reads dp), enqueued after it
      auto wfn = [&E, ws, w_wgrad, s_w, st, l]() -> int {
        Timed tw(E, lname("bwd.w_wgrad", l), s_w);
        return weight_grad(E, ws, w_wgrad, s_w, lname("bwd.w_wgrad", l), nullptr, nullptr, false, s_w != st);
      };
      if (l == 0 && (E.fork_plan & 4)) late.push_back(wfn);  // (forked with the optimizer pass)
      else PS_TRY(fork_late(s_w, wfn));
      Timed td(E, lname("bwd.dcat", l), st);
      PS_TRY(launch_gemm(p, st));
      E.sk_used[lname("bwd.dcat", l)] = gemm_last_stream_k();
    }
    PS_TRY(run_pend(E));
    if (adam && l == 0) {  // every gradient but Q0's exists on s_w; W0 was read last
      const int64_t off = l0.pWw, n = E.n_params - l0.pWw;
      const AdamStep a = *adam;
      PS_TRY(fork_late(s_w, [&E, s_w, off, n, a]() -> int {
        Timed ta(E, "adam", s_w);
        return launch_adam(E.params + off, E.grads + off, E.adam_m + off, E.adam_v + off, n, a.coef,
                           a.beta1, a.beta2, a.eps, s_w);
      }));
    } else if (l == 0 && !late.empty()) {
      PS_TRY(fork_late(s_w, []() -> int { return kOk; }));
    }
    const bool chunk_rows = l == 0 && E.dq_chunk_rows;
    // layer 0 on pre-split operands: dpq written as planes, the Q weight
    // gradient on them and on the feature table's planes (wgrad_pl_kernel)
    const bool planes = l == 0 && E.fplanes && lb.dpq3 && E.dq_tree && !chunk_rows && hd <= 512 && E.wgrad_kw &&
                        wgrad_kw_supported(hd, d, -1, false) && (int64_t)(hd / 64) * (d / 64) <= E.kw_cnt_len;
    PS_TRY(launch_dq_chunks(at<int2>(ws, lb.chunks), at<int>(ws, lb.nchunks), lb.max_chunks,
                            at<int2>(ws, lb.split), at<int>(ws, lb.nsplit), lb.max_split,
                            at<int>(ws, lb.off), at<int2>(ws, lb.occ2),
                            at<float>(ws, lb.dagg), hd, at<float>(ws, lb.q), hd, at<float>(ws, lb.dpq),
                            at<float>(ws, lb.dqpart), st, at<int32_t>(ws, lb.q_src),
                            chunk_rows ? at<int32_t>(ws, lb.csrc) : nullptr,
                            E.dq_tree ? at<int>(ws, lb.cbase) : nullptr, E.dq_tree ? at<int>(ws, lb.dqtk) : nullptr,
                            planes ? at<uint16_t>(ws, lb.dpq3) : nullptr, lb.N.cap * hd));
    PS_TRY(run_pend(E));
    WGrad q_wgrad;
    {
      // dQ = dpq^T h[q_src], dQb = colsum(dpq); chunk rows: the same sums over
      // the masked chunk partials, h gathered through csrc
      WGrad w;
      w.A = at<float>(ws, chunk_rows ? lb.dqpart : lb.dpq);
      w.lda = hd;
      w.M = hd;
      w.B = h;
      w.ldb = ldh;
      w.b_idx = at<int32_t>(ws, chunk_rows ? lb.csrc : lb.q_src);
      w.N = d;
      w.K_dev = chunk_rows ? at<int>(ws, lb.nchunks) : cnt(lb.N);
      w.K_max = chunk_rows ? lb.max_chunks : lb.N.cap;
      w.K_hint = lb.N.hint;
      w.dst = gr + lb.pQw;
      w.ld_dst = d;
      w.dst_b = gr + lb.pQb;
      if (planes) {
        w.A3 = at<uint16_t>(ws, lb.dpq3);
        w.a3_ps = lb.N.cap * hd;
        w.B3 = E.fplanes;
        w.b3_ps = E.fplanes_ps;
        w.ldb = d;
      }
      q_wgrad = w;
    }
    if (l > 0) {
      // dQ of this layer beside the chain, forked here (dpq complete), enqueued
      // after the dh launch
      auto qfn = [&E, ws, q_wgrad, s_wg, st, l]() -> int {
        Timed tq(E, lname("bwd.q_wgrad", l), s_wg);
        return weight_grad(E, ws, q_wgrad, s_wg, lname("bwd.q_wgrad", l), nullptr, nullptr, false,
                           s_wg != st);
      };
      if (E.fork_plan & 2) late.push_back(qfn);  // (rides on the next W-gradient fork)
      else PS_TRY(fork_late(s_wg, qfn));
      GemmParams p;  // dh = dpq Q  -> scatter-add into the rows of layer l-1
      p.M_dev = cnt(lb.N);
      p.M_hint = (int)lb.N.hint;
      p.M_max = (int)lb.N.cap;
      p.N = d;
      p.K = hd;
      p.a = at<float>(ws, lb.dpq);
      p.lda = hd;
      p.b_kmajor = false;
      p.b = E.params + lb.pQw;
      p.ldb = d;
      p.c = dYprev;
      p.ldc = o;
      p.c_idx = at<int32_t>(ws, lb.q_src);
      p.epi = kEpiAccum;
      with_sk(E, ws, p);
      apply_choice(E, lname("bwd.dh", l), p);
      Timed tdh(E, lname("bwd.dh", l), st);
      PS_TRY(launch_gemm(p, st));
      E.sk_used[lname("bwd.dh", l)] = gemm_last_stream_k();
    }
    PS_TRY(run_pend(E));
    if (l == 0) {  // dQ0 ends the chain, on the main stream
      AdamSlice q0;
      if (adam) q0 = adam_slice(E, *adam, lb.pQw, lb.pQb);
      Timed tq(E, lname("bwd.q_wgrad", l), st);
      PS_TRY(weight_grad(E, ws, q_wgrad, st, lname("bwd.q_wgrad", l), adam ? &q0 : nullptr, nullptr, true,
                         false));
    }
  }
  if (!late.empty()) PS_TRY(fork_late(s_wg, []() -> int { return kOk; }));  // (a stage-0 call)
  PS_TRY(flush_ride(E));
  PS_TRY(run_pend(E));
  // every gradient is written once the side streams drain into st (side[0]
  // also carries the loss monitors, pinsage_engine_loss)
  PS_TRY(dep(E, E.side[0], st));
  PS_TRY(dep(E, s_csr, st));
  PS_TRY(dep(E, s_wg, st));
  if (s_wg0 != s_wg) PS_TRY(dep(E, s_wg0, st));
  return kOk;
}

// Zero the regions that kernels keep zero after use (loss G / Kc, CSR counts,
// stream-K tickets):
// once per workspace, before its first step.
int engine_init_workspace(Engine& E, void* ws, hipStream_t st) {
  const EngineConfig& c = E.cfg;
  // the side streams and events now, outside any capture (a stream or event
  // created while a graph is being captured would invalidate that capture)
  PS_TRY(ensure_streams(E));
  const int64_t top = E.L.back().S.cap;
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.G), 0, (size_t)(3 * top * c.out) * 4, st));
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.Kc), 0, (size_t)(3 * top) * 4, st));
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.rank_off), 0xff, 4, st));  // (no positions yet)
  for (auto& lb : E.L) {
    PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, lb.cnt), 0, (size_t)(lb.N.cap + 1) * 4, st));
    PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, lb.dqtk), 0, (size_t)lb.dqtk_len * 4, st));
  }
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.sk_cnt), 0, (size_t)E.sk_cnt_len * 4, st));
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.kw_cnt_main), 0, (size_t)E.kw_cnt_len * 4, st));
  PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E.kw_cnt_side), 0, (size_t)E.kw_cnt_len * 4, st));
  return kOk;
}

}  // namespace ps

// ============================================================================ C-ABI
#include "../../include/pinsage_hip.h"

using namespace ps;

extern "C" {

int pinsage_engine_create(const pinsage_engine_config* cfg, pinsage_engine** out) {
  if (!cfg || !out) {
    set_error("engine_create: null argument");
    return kErrArg;
  }
  if (cfg->n_items <= 0 || cfg->d_in <= 0 || cfg->hid <= 0 || cfg->out <= 0 || cfg->n_layers <= 0 ||
      cfg->T <= 0 || cfg->max_pos <= 0) {
    set_error("engine_create: all sizes must be positive");
    return kErrArg;
  }
  if (cfg->d_in % 4 || cfg->hid % 4 || cfg->out % 4) {
    set_error("engine_create: d_in, hidden_dim and out_dim must be multiples of 4");
    return kErrArg;
  }
  if (cfg->out > 128) {
    set_error("engine_create: out_dim > 128 is not supported by the fused L2-norm epilogue");
    return kErrArg;
  }
  if (cfg->d_in < cfg->out) {
    // put_embeddings pads the conv output to the feature width (pinsage_model.py:27-29)
    set_error("engine_create: d_in < out_dim (the reference fails in put_embeddings)");
    return kErrArg;
  }
  auto* E = new Engine();
  g_live_engines++;
  E->cfg = EngineConfig{cfg->n_items, cfg->d_in, cfg->hid, cfg->out, cfg->n_layers, cfg->T,
                        cfg->max_pos};
  layout(*E);
  *out = reinterpret_cast<pinsage_engine*>(E);
  return kOk;
}

// capture-safe: no HIP call (the engine's streams and events are retired for
// reuse, see Engine::~Engine)
void pinsage_engine_destroy(pinsage_engine* e) { delete reinterpret_cast<Engine*>(e); }

int64_t pinsage_engine_live_count(void) { return g_live_engines.load(); }

int64_t pinsage_engine_workspace_bytes(const pinsage_engine* e) {
  return (int64_t) reinterpret_cast<const Engine*>(e)->total;
}

int64_t pinsage_engine_num_params(const pinsage_engine* e) {
  return reinterpret_cast<const Engine*>(e)->n_params;
}

int pinsage_engine_set_tensors(pinsage_engine* e, const float* feats, int64_t ld_feats,
                               const int32_t* nb_table, const float* w_table, int64_t ld_table,
                               float* params, float* grads, float* adam_m, float* adam_v) {
  Engine* E = reinterpret_cast<Engine*>(e);
  if (ld_table < E->cfg.T || ld_feats < E->cfg.d_in) {
    set_error("engine_set_tensors: leading dimension too small");
    return kErrArg;
  }
  E->feats = feats;
  E->ld_f = ld_feats;
  E->nb = nb_table;
  E->wn = w_table;
  E->ldT = ld_table;
  E->params = params;
  E->grads = grads;
  E->adam_m = adam_m;
  E->adam_v = adam_v;
  return kOk;
}

int pinsage_engine_offsets(const pinsage_engine* e, pinsage_engine_offsets_t* o) {
  const Engine* E = reinterpret_cast<const Engine*>(e);
  o->ids = (int64_t)E->ids;
  o->pos_rank = (int64_t)E->pos_rank;
  o->z = (int64_t)E->Z;
  o->dz = (int64_t)E->dZ;
  o->scalars = (int64_t)E->scal;
  o->hinge = (int64_t)E->hinge;
  o->n_layers = E->cfg.n_layers;
  for (int64_t l = 0; l < E->cfg.n_layers && l < 8; ++l) {
    o->count_S[l] = (int64_t)E->L[(size_t)l].S.count;
    o->count_N[l] = (int64_t)E->L[(size_t)l].N.count;
    o->members_S[l] = (int64_t)E->L[(size_t)l].S.members;
    o->members_N[l] = (int64_t)E->L[(size_t)l].N.members;
    o->cap_S[l] = E->L[(size_t)l].S.cap;
    o->cap_N[l] = E->L[(size_t)l].N.cap;
    o->y[l] = (int64_t)E->L[(size_t)l].y;
  }
  for (int l = 0; l < 8; ++l) o->param_offsets[l] = 0;
  return kOk;
}

int pinsage_engine_timing(pinsage_engine* e, int enable) {
  Engine* E = reinterpret_cast<Engine*>(e);
  for (auto& t : E->sites)
    for (auto& pr : t.pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  E->sites.clear();
  E->timing = enable != 0;
  return kOk;
}

int pinsage_engine_timing_collect(pinsage_engine* e) {
  Engine* E = reinterpret_cast<Engine*>(e);
  for (auto& t : E->sites) {
    for (auto& pr : t.pending) {
      PS_CHECK_HIP(hipEventSynchronize(pr.second));
      float ms = 0.f;
      PS_CHECK_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
      t.ms += ms;
      t.calls += 1;
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    t.pending.clear();
  }
  return kOk;
}

int pinsage_engine_timing_get(const pinsage_engine* e, int idx, char* name, int64_t name_len,
                              double* ms, int64_t* calls) {
  const Engine* E = reinterpret_cast<const Engine*>(e);
  if (idx < 0 || idx >= (int)E->sites.size()) return kErrArg;
  const TimingSite& t = E->sites[(size_t)idx];
  std::strncpy(name, t.name.c_str(), (size_t)name_len - 1);
  name[name_len - 1] = 0;
  *ms = t.ms;
  *calls = t.calls;
  return kOk;
}

int pinsage_engine_read_counts(const pinsage_engine* e, void* ws, int64_t* S, int64_t* N,
                               void* stream) {
  const Engine* E = reinterpret_cast<const Engine*>(e);
  PS_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
  for (size_t l = 0; l < E->L.size(); ++l) {
    int v = 0;
    PS_CHECK_HIP(hipMemcpy(&v, at<int>(ws, E->L[l].S.count), 4, hipMemcpyDeviceToHost));
    S[l] = v;
    PS_CHECK_HIP(hipMemcpy(&v, at<int>(ws, E->L[l].N.count), 4, hipMemcpyDeviceToHost));
    N[l] = v;
  }
  return kOk;
}

int pinsage_engine_set_feature_ilv(pinsage_engine* e, const uint16_t* table, int64_t ld) {
  if (!e || (table && (ld % 8 != 0 || ld < 3 * reinterpret_cast<Engine*>(e)->cfg.d_in))) {
    set_error("engine_set_feature_ilv: bad argument (ld a multiple of 8, >= 3 d_in)");
    return kErrArg;
  }
  Engine* E = reinterpret_cast<Engine*>(e);
  E->f_ilv = table;
  E->f_ilv_ld = table ? ld : 0;
  return kOk;
}

int pinsage_engine_set_frontier_fork(pinsage_engine* e, int on) {
  if (!e) {
    set_error("engine_set_frontier_fork: null engine");
    return kErrArg;
  }
  reinterpret_cast<Engine*>(e)->frontier_fork_ok = on != 0;
  return kOk;
}

int pinsage_engine_set_feature_planes(pinsage_engine* e, const uint16_t* planes, int64_t plane_stride) {
  if (!e || (planes && plane_stride <= 0)) {
    set_error("engine_set_feature_planes: bad argument");
    return kErrArg;
  }
  Engine* E = reinterpret_cast<Engine*>(e);
  E->fplanes = planes;
  E->fplanes_ps = planes ? plane_stride : 0;
  return kOk;
}

int pinsage_engine_set_gemm_choice(pinsage_engine* e, const char* site, int cfg, int stream_k,
                                   int splits) {
  Engine* E = reinterpret_cast<Engine*>(e);
  if (!E || !site) {
    set_error("engine_set_gemm_choice: null argument");
    return kErrArg;
  }
  if (cfg < -1 || cfg > 5 || stream_k < -1 || stream_k > 1 || splits < 0 || splits > kMaxSplits) {
    set_error("engine_set_gemm_choice: cfg in [-1, 5], stream_k in [-1, 1], splits in [0, 64]");
    return kErrArg;
  }
  if (cfg < 0 && stream_k < 0 && splits == 0) E->choice.erase(site);
  else E->choice[site] = Engine::GemmChoice{cfg, stream_k, splits};
  return kOk;
}

int pinsage_engine_site_stream_k(const pinsage_engine* e, const char* site) {
  const Engine* E = reinterpret_cast<const Engine*>(e);
  if (!E || !site) return -1;
  auto it = E->sk_used.find(site);
  return it == E->sk_used.end() ? -1 : it->second;
}

int pinsage_engine_set_layer_table(pinsage_engine* e, int64_t layer, const int32_t* nb,
                                   const float* wn, int64_t ld) {
  Engine* E = reinterpret_cast<Engine*>(e);
  if (!E || layer < 0 || layer >= E->cfg.n_layers || ((nb == nullptr) != (wn == nullptr)) ||
      (nb && ld < E->cfg.T)) {
    set_error("engine_set_layer_table: bad argument");
    return kErrArg;
  }
  LayerBuf& lb = E->L[(size_t)layer];
  lb.nb_tab = nb;
  lb.wn_tab = wn;
  lb.ld_tab = ld;
  return kOk;
}

int pinsage_engine_set_hints(pinsage_engine* e, const int64_t* S, const int64_t* N) {
  Engine* E = reinterpret_cast<Engine*>(e);
  for (size_t l = 0; l < E->L.size(); ++l) {
    E->L[l].S.hint = S ? S[l] : 0;
    E->L[l].N.hint = N ? N[l] : 0;
  }
  return kOk;
}

int pinsage_engine_init_workspace(pinsage_engine* e, void* ws, void* stream) {
  if (!e || !ws) {
    set_error("engine_init_workspace: null argument");
    return kErrArg;
  }
  return engine_init_workspace(*reinterpret_cast<Engine*>(e), ws, (hipStream_t)stream);
}

int pinsage_engine_forward(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                           void* stream) {
  PS_TRY(flush_ride(*reinterpret_cast<Engine*>(e)));
  PS_TRY(run_pend(*reinterpret_cast<Engine*>(e)));
  return engine_forward(*reinterpret_cast<Engine*>(e), ws, ids, n_ids, (hipStream_t)stream);
}

int pinsage_engine_forward_inference(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                                     void* stream) {
  PS_TRY(flush_ride(*reinterpret_cast<Engine*>(e)));
  PS_TRY(run_pend(*reinterpret_cast<Engine*>(e)));
  return engine_forward(*reinterpret_cast<Engine*>(e), ws, ids, n_ids, (hipStream_t)stream, false);
}

int pinsage_engine_frontier(pinsage_engine* e, void* ws, const int64_t* ids, int64_t n_ids,
                            void* stream) {
  PS_TRY(flush_ride(*reinterpret_cast<Engine*>(e)));
  PS_TRY(run_pend(*reinterpret_cast<Engine*>(e)));
  return engine_frontier(*reinterpret_cast<Engine*>(e), ws, ids, n_ids, (hipStream_t)stream);
}

int pinsage_engine_forward_layers(pinsage_engine* e, void* ws, void* stream) {
  PS_TRY(flush_ride(*reinterpret_cast<Engine*>(e)));
  PS_TRY(run_pend(*reinterpret_cast<Engine*>(e)));
  return engine_layers(*reinterpret_cast<Engine*>(e), ws, (hipStream_t)stream);
}

int pinsage_engine_set_fork(pinsage_engine* e, void* ws_next, const int64_t* ids_next,
                            int64_t n_ids, void* side_stream) {
  Engine* E = reinterpret_cast<Engine*>(e);
  if (side_stream && (!ws_next || !ids_next || n_ids <= 0 || n_ids > E->cfg.max_pos)) {
    set_error("engine_set_fork: bad argument");
    return kErrArg;
  }
  E->fork = Engine::Fork{(hipStream_t)side_stream, ws_next, ids_next, n_ids};
  return kOk;
}

int pinsage_engine_gather_output(pinsage_engine* e, void* ws, int64_t n_ids, float* out,
                                 void* stream) {
  Engine* E = reinterpret_cast<Engine*>(e);
  PS_TRY(flush_ride(*E));
  PS_TRY(run_pend(*E));
  return launch_gather_out(at<float>(ws, E->Z), (int)E->cfg.out, at<int32_t>(ws, E->pos_rank), n_ids,
                           out, (hipStream_t)stream);
}

int pinsage_engine_loss(pinsage_engine* e, void* ws, int64_t batch_size, float margin,
                        int with_monitors, void* stream) {
  Engine* E = reinterpret_cast<Engine*>(e);
  const EngineConfig& c = E->cfg;
  if (3 * batch_size > c.max_pos || batch_size < 2) {
    set_error("engine_loss: batch_size out of range (the reference needs B >= 2)");
    return kErrArg;
  }
  LayerBuf& top = E->L.back();
  hipStream_t st = (hipStream_t)stream;
  PS_TRY(flush_ride(*E));  // (an earlier loss's monitors read what this one rewrites)
  {
    Timed t(*E, "loss", st);
    // (on the fly the repeated ranks are summed in the loss launch: the
    // virtual nodes copy the summed rows)
    const bool fly = E->fly_nx != nullptr;
    E->reps_in_gp = E->fused_head && E->head_rep_sum && !fly;
    PS_TRY(launch_loss(at<float>(ws, E->Z), (int)c.out, at<int32_t>(ws, E->pos_rank), (int)batch_size,
                       margin, with_monitors ? E->feats : nullptr, E->ld_f, (int)c.d_in,
                       at<int64_t>(ws, E->ids), at<float>(ws, E->G), at<int>(ws, E->Kc), top.S.cap,
                       at<int>(ws, top.S.count), at<float>(ws, E->dZ), at<float>(ws, E->part),
                       at<float>(ws, E->varpart), at<float>(ws, E->scal), at<float>(ws, E->hinge),
                       !E->fused_head && !fly, !E->fused_head || !E->head_rep_sum || fly, at<int>(ws, E->rank_off),
                       at<int32_t>(ws, E->pos_sorted), at<float>(ws, E->Gp), st));
    if (fly)
      PS_TRY(launch_fly_fix(at<float>(ws, E->G), at<int>(ws, E->Kc), top.S.cap, (int)c.out,
                            at<unsigned long long>(ws, top.S.bits), at<uint32_t>(ws, top.S.prefix), E->fly_nx,
                            E->fly_xids, E->fly_x0, E->fly_unit, E->fly_xcap, at<int>(ws, top.S.count),
                            at<float>(ws, E->dZ), !E->fused_head, st));
  }
  // the monitors (loss, node-feature loss, variance scalars) beside the
  // backward, on side stream 0, joined at the backward's end (with
  // PINSAGE_DEFER_SIDE bit 1 enqueued behind the head backward's launch, or
  // by the next engine call that enqueues work)
  PS_TRY(ensure_streams(*E));
  PS_TRY(run_pend(*E));
  float* part = at<float>(ws, E->part);
  float* varpart = at<float>(ws, E->varpart);
  float* scal = at<float>(ws, E->scal);
  const int nb4 = (int)ceil_div(batch_size, 4), out = (int)c.out, B = (int)batch_size;
  hipStream_t s0 = E->side[0];
  auto mon = [E, part, varpart, scal, nb4, out, B](hipStream_t s) -> int {
    Timed tm(*E, "loss.monitor", s);
    return launch_loss_monitor(part, nb4, varpart, out, B, scal, s);
  };
  if (E->fork_plan & 1) {  // no fork at the loss: the head backward's fork takes them
    E->ride.push_back(mon);
    E->ride_st = st;
    return kOk;
  }
  return fork_side(*E, st, s0, (E->defer_side & 2) != 0, [mon, s0]() -> int { return mon(s0); });
}

int pinsage_engine_set_fly(pinsage_engine* e, int64_t x0, const int* n_x, const int64_t* xids, int64_t unit,
                           int64_t x_cap) {
  if (!e || (n_x && (!xids || unit <= 0 || x0 < 0 || x_cap < 0))) {
    set_error("engine_set_fly: bad argument");
    return kErrArg;
  }
  Engine* E = reinterpret_cast<Engine*>(e);
  E->fly_x0 = n_x ? x0 : 0;
  E->fly_nx = n_x;
  E->fly_xids = n_x ? xids : nullptr;
  E->fly_unit = n_x ? unit : 1;
  E->fly_xcap = n_x ? x_cap : 0;
  return kOk;
}

int pinsage_engine_set_output_grad(pinsage_engine* e, void* ws, const float* dout, int64_t n_ids,
                                   void* stream) {
  Engine* E = reinterpret_cast<Engine*>(e);
  PS_TRY(flush_ride(*E));
  PS_TRY(run_pend(*E));
  LayerBuf& top = E->L.back();
  E->reps_in_gp = false;
  return launch_dz_from_dout(dout, (int)E->cfg.out, at<int32_t>(ws, E->pos_rank), n_ids,
                             at<int>(ws, top.S.count), top.S.cap, at<float>(ws, E->G),
                             at<int>(ws, E->Kc), at<float>(ws, E->dZ), !E->fused_head,
                             at<int>(ws, E->rank_off), at<int32_t>(ws, E->pos_sorted), at<float>(ws, E->Gp),
                             (hipStream_t)stream);
}

int pinsage_engine_reset_backward(pinsage_engine* e, void* ws, void* stream) {
  if (!e || !ws) {
    set_error("engine_reset_backward: null argument");
    return kErrArg;
  }
  Engine* E = reinterpret_cast<Engine*>(e);
  PS_TRY(flush_ride(*E));
  PS_TRY(run_pend(*E));
  // the dY scatter-add targets of the layers below the top (the forward's
  // layer_prep zeroed them; a backward accumulates into them)
  for (size_t l = 0; l + 1 < E->L.size(); ++l)
    PS_CHECK_HIP(hipMemsetAsync(at<char>(ws, E->L[l].dY), 0, (size_t)(E->L[l].S.cap * E->cfg.out) * 4,
                                (hipStream_t)stream));
  return kOk;
}

int pinsage_engine_backward(pinsage_engine* e, void* ws, void* stream) {
  return engine_backward(*reinterpret_cast<Engine*>(e), ws, (hipStream_t)stream, nullptr);
}

int pinsage_engine_backward_stage(pinsage_engine* e, void* ws, int stage, void* stream) {
  if (stage != 0 && stage != 1) {
    set_error("engine_backward_stage: stage 0 (head and layers L-1 .. 1) or 1 (layer 0)");
    return kErrArg;
  }
  return engine_backward(*reinterpret_cast<Engine*>(e), ws, (hipStream_t)stream, nullptr, stage);
}

int pinsage_engine_backward_adam(pinsage_engine* e, void* ws, const float* coef, double beta1,
                                 double beta2, float eps, void* stream) {
  if (!coef) {
    set_error("engine_backward_adam: null coefficients");
    return kErrArg;
  }
  const AdamStep a{coef, beta1, beta2, eps};
  return engine_backward(*reinterpret_cast<Engine*>(e), ws, (hipStream_t)stream, &a);
}

int pinsage_engine_adam(pinsage_engine* e, const float* coef, double beta1, double beta2, float eps,
                        void* stream) {
  Engine* E = reinterpret_cast<Engine*>(e);
  PS_TRY(flush_ride(*E));
  PS_TRY(run_pend(*E));
  Timed t(*E, "adam", (hipStream_t)stream);
  if (!E->adam_m || !E->adam_v) {
    set_error("engine_adam: optimizer state not set");
    return kErrArg;
  }
  return launch_adam(E->params, E->grads, E->adam_m, E->adam_v, E->n_params, coef, beta1, beta2, eps,
                     (hipStream_t)stream);
}

}  // extern "C"

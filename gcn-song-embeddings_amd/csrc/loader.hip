// Batch sampler runtime: reference-exact training batches (easy negatives,
// pinsage_training.py:53-77, 89-97) with the next batches drawn speculatively
// on a native worker thread.
//
// The reference draws each batch from torch's global CPU generator; the O(P)
// part is torch.randperm(P) consuming P-1 draws of which only the first B
// matter.  After serving the batch that starts at generator state s_i, the
// worker draws the batch that starts at s_{i+1} (the state just handed back)
// into a private buffer.  The next request uses it only if its start state is
// byte-identical to s_{i+1}; anything else (another torch RNG user in between,
// a reseed) is drawn synchronously.  Results are therefore exactly the
// reference's, and the randperm skip leaves the training loop's critical path.
// Pure host code; no GPU calls.
#include <condition_variable>
#include <deque>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pinsage_hip.h"
#include "common.h"
#include "mt19937.h"

namespace ps {

int sample_batch_easy(MTState& g, const int64_t* positives, int64_t P, int64_t n_items,
                      int64_t batch_size, int64_t* batch_out, int64_t* nodeset_out,
                      int64_t* n_nodeset);

namespace {

struct Draw {
  std::vector<uint8_t> start, after;  // torch generator state before / after the batch
  std::vector<int64_t> batch, nodeset;
  int rc = kOk;
  std::string err;
};

struct BatchSampler {
  const int64_t* pos = nullptr;
  int64_t P = 0, n_items = 0, B = 0;

  // The worker draws a chain of batches ahead: the batch starting at the state
  // the last request handed back, then the one after it, ... up to kDepth
  // finished draws (so a caller that peeks at the next batch right after a
  // request finds it drawn during the previous step).  A request whose start
  // state is not the chain's next one discards the chain.
  static constexpr int kDepth = 2;
  std::mutex mu;
  std::condition_variable cv;
  std::thread worker;
  bool stop = false;
  bool running = false;          // the worker is drawing from run_start
  uint64_t generation = 0;       // bumped when the chain is discarded
  std::vector<uint8_t> chain;    // start state of the next draw (empty: none)
  std::vector<uint8_t> run_start;
  std::deque<Draw> ready;        // finished draws, in chain order

  void draw(Draw& d) const {
    MTState g;
    d.rc = kOk;
    d.err.clear();
    if (!g.from_torch(d.start.data(), (int64_t)d.start.size())) {
      d.rc = kErrArg;
      d.err = "batch_sampler: not a valid torch CPU generator state";
      return;
    }
    const int64_t b = std::min(B, P);
    d.batch.resize((size_t)(3 * b));
    d.nodeset.resize((size_t)(3 * b));
    int64_t n = 0;
    d.rc = sample_batch_easy(g, pos, P, n_items, B, d.batch.data(), d.nodeset.data(), &n);
    if (d.rc != kOk) {
      d.err = last_error();
      return;
    }
    d.nodeset.resize((size_t)n);
    d.after = d.start;
    g.to_torch(d.after.data());
  }

  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || (!chain.empty() && (int)ready.size() < kDepth); });
      if (stop) return;
      Draw d;
      d.start = chain;
      run_start = chain;
      running = true;
      const uint64_t gen = generation;
      lk.unlock();
      draw(d);
      lk.lock();
      running = false;
      if (gen == generation) {
        if (d.rc == kOk) {
          chain = d.after;
          ready.push_back(std::move(d));
        } else {
          chain.clear();  // a failing draw fails again synchronously, with its message
        }
      }
      cv.notify_all();
    }
  }

  static bool same(const std::vector<uint8_t>& a, const uint8_t* b, int64_t nbytes) {
    return (int64_t)a.size() == nbytes && std::memcmp(a.data(), b, (size_t)nbytes) == 0;
  }

  // The chain's draw for this start state, if it is the chain's next one
  // (waiting for it if the worker is on it); otherwise discard the chain.
  bool take(const uint8_t* state, int64_t nbytes, Draw& out) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (!ready.empty()) {
        if (same(ready.front().start, state, nbytes)) {
          out = std::move(ready.front());
          ready.pop_front();
          cv.notify_all();
          return true;
        }
        break;
      }
      // the worker is on it, or about to start it
      if ((running && same(run_start, state, nbytes)) ||
          (!running && same(chain, state, nbytes))) {
        cv.wait(lk, [&] { return !ready.empty() || (!running && chain.empty()); });
        if (ready.empty()) break;
        continue;
      }
      break;
    }
    ready.clear();
    chain.clear();
    ++generation;
    return false;
  }

  // The next draw of the chain (the batch the next request will get if it
  // starts where the last one ended), waiting for the worker if needed.
  bool peek(std::vector<int64_t>& batch) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return !ready.empty() || (!running && chain.empty()) || stop; });
    if (ready.empty()) return false;
    batch = ready.front().batch;
    return true;
  }

  // Start the chain at this state unless it already runs past it (a hit).
  void submit(const std::vector<uint8_t>& start) {
    std::lock_guard<std::mutex> lk(mu);
    if (!chain.empty()) return;
    chain = start;
    cv.notify_all();
  }

  ~BatchSampler() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
      cv.notify_all();
    }
    if (worker.joinable()) worker.join();
  }
};

}  // namespace
}  // namespace ps

using namespace ps;

extern "C" {

int pinsage_batch_sampler_create(const int64_t* positives, int64_t n_pos_pairs, int64_t n_items,
                                 int64_t batch_size, pinsage_batch_sampler** out) {
  if (!out || (!positives && n_pos_pairs > 0) || n_pos_pairs < 0 || n_items <= 0 ||
      batch_size <= 0) {
    set_error("batch_sampler_create: bad argument");
    return kErrArg;
  }
  auto* s = new BatchSampler();
  s->pos = positives;
  s->P = n_pos_pairs;
  s->n_items = n_items;
  s->B = batch_size;
  s->worker = std::thread([s] { s->loop(); });
  *out = reinterpret_cast<pinsage_batch_sampler*>(s);
  return kOk;
}

void pinsage_batch_sampler_destroy(pinsage_batch_sampler* s) {
  delete reinterpret_cast<BatchSampler*>(s);
}

int pinsage_batch_sampler_next(pinsage_batch_sampler* h, const uint8_t* state, int64_t nbytes,
                               int64_t* batch_out, int64_t* nodeset_out, int64_t* n_nodeset,
                               uint8_t* state_after, int speculate) {
  auto* s = reinterpret_cast<BatchSampler*>(h);
  if (!s || !state || !batch_out || !state_after || nbytes <= 0) {
    set_error("batch_sampler_next: bad argument");
    return kErrArg;
  }
  Draw d;
  const bool hit = s->take(state, nbytes, d);
  if (!hit) {
    d.start.assign(state, state + nbytes);
    s->draw(d);
  }
  if (d.rc != kOk) {
    set_error(d.err);
    return d.rc;
  }
  std::memcpy(batch_out, d.batch.data(), d.batch.size() * sizeof(int64_t));
  if (nodeset_out) std::memcpy(nodeset_out, d.nodeset.data(), d.nodeset.size() * sizeof(int64_t));
  if (n_nodeset) *n_nodeset = (int64_t)d.nodeset.size();
  std::memcpy(state_after, d.after.data(), (size_t)nbytes);
  if (speculate) s->submit(d.after);
  return hit ? 1 : kOk;
}

int pinsage_batch_sampler_peek(pinsage_batch_sampler* h, int64_t* batch_out, int64_t max_rows) {
  auto* s = reinterpret_cast<BatchSampler*>(h);
  if (!s || !batch_out || max_rows < 0) {
    set_error("batch_sampler_peek: bad argument");
    return kErrArg;
  }
  std::vector<int64_t> b;
  if (!s->peek(b) || (int64_t)b.size() > 3 * max_rows) return 0;
  std::memcpy(batch_out, b.data(), b.size() * sizeof(int64_t));
  return (int)(b.size() / 3);
}

}  // extern "C"

// Replays the stream / event / capture call sequence of a traced process
// (AMD_LOG_LEVEL=3 AMD_LOG_MASK=1 API log, reduced to ops by hand into
// tools/dbg/fork_crash_ops.txt) with a one-thread kernel standing in for every
// launch, to find which part of the sequence hipStreamEndCapture cannot take
// (VERDICT r05 item 6).  Ops: "B s mode" begin capture, "E s" end capture (+
// instantiate), "R e s" record, "W s e" wait, "K s" launch, "D e" destroy
// event, "S" device sync, "Y s" stream sync, "G" destroy the last
// instantiated graph's template (torch does, right after instantiating), "X"
// destroy the oldest live graph exec, "Q s" query the stream's capture state.  Handles are the traced ones,
// mapped to fresh streams / events on first sight (<null>: the null stream).
// argv[2] (optional): a number n -- skip the first n captures' ops (everything
// before the n-th begin is replayed eagerly without the captures' ops).
// Build: hipcc --offload-arch=gfx950 -O1 -o capture_replay capture_replay.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <deque>
#include <string>

__global__ void tick(int* p) { if (threadIdx.x == 0) p[0] += 1; }

int main(int argc, char** argv) {
  std::ifstream in(argc > 1 ? argv[1] : "fork_crash_ops.txt");
  int* d = nullptr;
  hipMalloc(&d, 64);
  std::map<std::string, hipStream_t> S;
  std::map<std::string, hipEvent_t> Ev;
  auto st = [&](const std::string& h) -> hipStream_t {
    if (h == "<null>" || h == "None") return nullptr;
    auto it = S.find(h);
    if (it != S.end()) return it->second;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    S[h] = s;
    return s;
  };
  auto ev = [&](const std::string& h) -> hipEvent_t {
    auto it = Ev.find(h);
    if (it != Ev.end()) return it->second;
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    Ev[h] = e;
    return e;
  };
  std::string line;
  int n = 0, cap = 0;
  bool capturing = false;
  hipGraph_t last_g = nullptr;
  std::deque<hipGraphExec_t> execs;
  while (std::getline(in, line)) {
    ++n;
    std::istringstream is(line);
    std::string op, a, b;
    is >> op >> a >> b;
    hipError_t r = hipSuccess;
    if (op == "B") {
      r = hipStreamBeginCapture(st(a), hipStreamCaptureModeGlobal);
      capturing = true;
      printf("[%d] begin capture %d on %s: %s\n", n, cap, a.c_str(), hipGetErrorName(r));
    } else if (op == "E") {
      hipGraph_t g = nullptr;
      printf("[%d] end capture %d ...\n", n, cap);
      fflush(stdout);
      r = hipStreamEndCapture(st(a), &g);
      printf("[%d] end capture %d: %s\n", n, cap, hipGetErrorName(r));
      fflush(stdout);
      if (r == hipSuccess && g) {
        hipGraphExec_t x;
        r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
        printf("[%d] instantiate %d: %s\n", n, cap, hipGetErrorName(r));
        if (r == hipSuccess) execs.push_back(x);
        last_g = g;
      }
      capturing = false;
      ++cap;
    } else if (op == "R") {
      r = hipEventRecord(ev(a), st(b));
    } else if (op == "W") {
      r = hipStreamWaitEvent(st(a), ev(b), 0);
    } else if (op == "K") {
      if (capturing && (a == "<null>")) continue;
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, st(a), d);
      r = hipGetLastError();
    } else if (op == "D") {
      auto it = Ev.find(a);
      if (it != Ev.end()) {
        r = hipEventDestroy(it->second);
        Ev.erase(it);
      }
    } else if (op == "G") {
      if (last_g) r = hipGraphDestroy(last_g);
      last_g = nullptr;
    } else if (op == "X") {
      if (!execs.empty()) {
        r = hipGraphExecDestroy(execs.front());
        execs.pop_front();
      }
    } else if (op == "Q") {
      hipStreamCaptureStatus cs;
      r = hipStreamIsCapturing(st(a), &cs);
    } else if (op == "S") {
      if (!capturing) r = hipDeviceSynchronize();
    } else if (op == "Y") {
      if (!capturing) r = hipStreamSynchronize(st(a));
    }
    if (r != hipSuccess) printf("[%d] %s -> %s\n", n, line.c_str(), hipGetErrorName(r));
    fflush(stdout);
  }
  printf("replayed %d ops, %d captures\n", n, cap);
  return 0;
}

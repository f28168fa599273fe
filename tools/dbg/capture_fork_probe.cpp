// Which forked-stream shapes does hipStreamEndCapture accept?  (VERDICT r05
// item 6: the step capture died with SIGSEGV inside hipStreamEndCapture when
// the layer-0 CSR build was forked onto an engine side stream.)  Each case
// runs in its own child process (a crash is reported, not inherited):
//   joined        fork A -> B (event), kernel on B, join B -> A, end capture
//   joined_empty  fork + join with no node on B
//   unjoined      fork, kernel on B, end capture without the join
//   unjoined_empty fork only (B holds no node), end capture
//   create_inside create a stream and an event while A captures (global mode)
//   err_then_end  a failing call inside the capture (invalidates it), then end
//   reuse_after_unjoined_empty  an unjoined empty fork of B, end capture (HIP
//                 accepts it), then a second capture that forks B again and
//                 joins it properly, then an eager launch on B
//   reuse_after_joined  the same with the first fork joined (control)
// Build: hipcc --offload-arch=gfx950 -O1 -o capture_fork_probe capture_fork_probe.cpp
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

__global__ void tick(int* p) { if (threadIdx.x == 0) p[0] += 1; }

static int run_reuse(const std::string& c) {
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipMemset(d, 0, 64);
  hipStream_t A, B;
  hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  hipEvent_t e1, e2;
  hipEventCreateWithFlags(&e1, hipEventDisableTiming);
  hipEventCreateWithFlags(&e2, hipEventDisableTiming);
  const bool join1 = c == "reuse_after_joined";
  for (int cap = 0; cap < 2; ++cap) {
    hipGraph_t g = nullptr;
    hipError_t r = hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
    printf("[%s] capture %d begin %s\n", c.c_str(), cap, hipGetErrorName(r));
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    r = hipEventRecord(e1, A);
    printf("[%s] capture %d record %s\n", c.c_str(), cap, hipGetErrorName(r));
    r = hipStreamWaitEvent(B, e1, 0);
    printf("[%s] capture %d wait %s\n", c.c_str(), cap, hipGetErrorName(r));
    if (cap == 1) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 4);
    if (cap == 1 || join1) {
      r = hipEventRecord(e2, B);
      printf("[%s] capture %d join record %s\n", c.c_str(), cap, hipGetErrorName(r));
      r = hipStreamWaitEvent(A, e2, 0);
      printf("[%s] capture %d join wait %s\n", c.c_str(), cap, hipGetErrorName(r));
    }
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    fflush(stdout);
    r = hipStreamEndCapture(A, &g);
    printf("[%s] capture %d end %s graph %p\n", c.c_str(), cap, hipGetErrorName(r), (void*)g);
    fflush(stdout);
    if (r == hipSuccess && g) {
      hipGraphExec_t x;
      r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
      if (r == hipSuccess) r = hipGraphLaunch(x, A);
      r = hipStreamSynchronize(A);
      printf("[%s] capture %d replay %s\n", c.c_str(), cap, hipGetErrorName(r));
    }
  }
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 8);
  hipError_t r = hipStreamSynchronize(B);
  int hv[16];
  hipMemcpy(hv, d, 64, hipMemcpyDeviceToHost);
  printf("[%s] eager on B %s counters A %d B-captured %d B-eager %d\n", c.c_str(), hipGetErrorName(r), hv[0], hv[4],
         hv[8]);
  fflush(stdout);
  return 0;
}

// The shape of the trainer's look-ahead step graph (pinsage_training
// _capture_graphs, graph `ga`): the origin stream A forks a branch S (the
// next batch's frontier); inside that branch the engine forks its side stream
// B off S and joins it back into S (nested_*: B empty or with a kernel); then
// the main chain on A forks the SAME side stream B again (the backward's
// monitors / weight gradients) and joins it into A; S is joined into A last.
// nested_separate: the branch's fork uses a third stream C instead of B.
static int run_nested(const std::string& c) {
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipMemset(d, 0, 64);
  hipStream_t A, S, B, C;
  for (hipStream_t* x : {&A, &S, &B, &C}) hipStreamCreateWithFlags(x, hipStreamNonBlocking);
  hipEvent_t e[8];
  for (auto& x : e) hipEventCreateWithFlags(&x, hipEventDisableTiming);
  hipStream_t F = c == "nested_separate" ? C : B;  // the stream the branch forks
  // *_tail: nothing runs on S after F's join (the branch ends with the wait,
  // as engine_frontier's join is the branch's last call before the trainer
  // joins S into A)
  const bool tail = c.find("tail") != std::string::npos;
  hipGraph_t g = nullptr;
  hipError_t r = hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  hipEventRecord(e[0], A);
  hipStreamWaitEvent(S, e[0], 0);                 // branch S off A
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, S, d + 4);
  hipEventRecord(e[1], S);
  r = hipStreamWaitEvent(F, e[1], 0);             // F off S
  printf("[%s] fork F off S %s\n", c.c_str(), hipGetErrorName(r));
  if (c.find("empty") == std::string::npos) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, F, d + 8);
  hipEventRecord(e[2], F);
  r = hipStreamWaitEvent(S, e[2], 0);             // F joined into S
  printf("[%s] join F into S %s\n", c.c_str(), hipGetErrorName(r));
  if (!tail) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, S, d + 4);
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  hipEventRecord(e[3], A);
  r = hipStreamWaitEvent(B, e[3], 0);             // B off A (again, for nested_*)
  printf("[%s] fork B off A %s\n", c.c_str(), hipGetErrorName(r));
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 12);
  hipEventRecord(e[4], B);
  hipStreamWaitEvent(A, e[4], 0);                 // B joined into A
  hipEventRecord(e[5], S);
  hipStreamWaitEvent(A, e[5], 0);                 // S joined into A
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  fflush(stdout);
  r = hipStreamEndCapture(A, &g);
  printf("[%s] end capture %s graph %p\n", c.c_str(), hipGetErrorName(r), (void*)g);
  fflush(stdout);
  if (r == hipSuccess && g) {
    hipGraphExec_t x;
    r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (r == hipSuccess) r = hipGraphLaunch(x, A);
    hipStreamSynchronize(A);
    int h[16];
    hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
    printf("[%s] replay %s counters A %d S %d F %d B %d\n", c.c_str(), hipGetErrorName(r), h[0], h[4], h[8], h[12]);
  }
  fflush(stdout);
  return 0;
}

// The trainer's capture ORDER (pinsage_training._capture_graphs): graph gf
// (the frontier on the origin stream A forks the side stream B and joins it),
// then graph ga (the origin forks a branch S; the frontier on S forks the
// SAME B and joins it into S; S joins A).  reuse_nested_fresh: ga's branch
// forks a stream no earlier capture used.
static int run_reuse_nested(const std::string& c) {
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipMemset(d, 0, 64);
  hipStream_t A, S, B, C;
  for (hipStream_t* x : {&A, &S, &B, &C}) hipStreamCreateWithFlags(x, hipStreamNonBlocking);
  hipEvent_t e[8];
  for (auto& x : e) hipEventCreateWithFlags(&x, hipEventDisableTiming);
  const bool empty = c.find("empty") != std::string::npos;
  hipStream_t F = c == "reuse_nested_fresh" ? C : B;
  for (int cap = 0; cap < 2; ++cap) {
    hipGraph_t g = nullptr;
    hipError_t r = hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    hipStream_t from = A, fk = B;
    if (cap == 1) {  // the look-ahead branch
      hipEventRecord(e[0], A);
      hipStreamWaitEvent(S, e[0], 0);
      from = S;
      fk = F;
    }
    hipEventRecord(e[1], from);
    r = hipStreamWaitEvent(fk, e[1], 0);
    printf("[%s] capture %d fork %s\n", c.c_str(), cap, hipGetErrorName(r));
    if (!empty) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, fk, d + 8);
    hipEventRecord(e[2], fk);
    r = hipStreamWaitEvent(from, e[2], 0);
    printf("[%s] capture %d join %s\n", c.c_str(), cap, hipGetErrorName(r));
    if (cap == 1) {
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, S, d + 4);
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
      hipEventRecord(e[3], S);
      hipStreamWaitEvent(A, e[3], 0);
    }
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    fflush(stdout);
    r = hipStreamEndCapture(A, &g);
    printf("[%s] capture %d end %s graph %p\n", c.c_str(), cap, hipGetErrorName(r), (void*)g);
    fflush(stdout);
    if (r == hipSuccess && g) {
      hipGraphExec_t x;
      r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
      if (r == hipSuccess) r = hipGraphLaunch(x, A);
      hipStreamSynchronize(A);
      printf("[%s] capture %d replay %s\n", c.c_str(), cap, hipGetErrorName(r));
    }
  }
  fflush(stdout);
  return 0;
}

// A side stream's captured history outliving its graph: capture 0 puts a
// kernel on B (B's last captured node lives in graph 0), graph 0 and its
// exec are destroyed and the host heap is churned, then capture 1 forks B
// again -- empty (stale_empty: wait + record with no node of B's own) or with
// a kernel (stale_kernel).  An empty fork's join records B's dependency set.
static int run_stale(const std::string& c) {
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipMemset(d, 0, 64);
  hipStream_t A, B;
  hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  hipEvent_t e[4];
  for (auto& x : e) hipEventCreateWithFlags(&x, hipEventDisableTiming);
  for (int cap = 0; cap < 4; ++cap) {
    hipGraph_t g = nullptr;
    hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    hipEventRecord(e[0], A);
    hipStreamWaitEvent(B, e[0], 0);
    if (cap == 0 || c == "stale_kernel") hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 8);
    hipEventRecord(e[1], B);
    hipStreamWaitEvent(A, e[1], 0);
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    fflush(stdout);
    hipError_t r = hipStreamEndCapture(A, &g);
    printf("[%s] capture %d end %s\n", c.c_str(), cap, hipGetErrorName(r));
    fflush(stdout);
    if (r != hipSuccess || !g) return 0;
    hipGraphExec_t x;
    r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (r == hipSuccess) r = hipGraphLaunch(x, A);
    hipStreamSynchronize(A);
    printf("[%s] capture %d replay %s\n", c.c_str(), cap, hipGetErrorName(r));
    hipGraphExecDestroy(x);
    hipGraphDestroy(g);
    for (int i = 0; i < 2000; ++i) {  // churn the host heap over the freed graph
      volatile char* q = static_cast<char*>(malloc(64 + (i % 7) * 64));
      memset((void*)q, 0xa5, 64);
      if (i % 3) free((void*)q);
    }
  }
  fflush(stdout);
  return 0;
}

// The join of a fork AFTER the origin advanced (engine_frontier with
// PINSAGE_CSR_FORK=2: fork, the CSR builds on the origin, then the empty
// side joined back -- the join adds an edge from an ancestor of the origin's
// last node).  nested_advanced_*: the same inside a branch S of A.
static int run_advanced(const std::string& c) {
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipMemset(d, 0, 64);
  hipStream_t A, S, B;
  for (hipStream_t* x : {&A, &S, &B}) hipStreamCreateWithFlags(x, hipStreamNonBlocking);
  hipEvent_t e[6];
  for (auto& x : e) hipEventCreateWithFlags(&x, hipEventDisableTiming);
  const bool nested = c.rfind("nested", 0) == 0, empty = c.find("empty") != std::string::npos;
  hipGraph_t g = nullptr;
  hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  hipStream_t O = A;
  if (nested) {
    hipEventRecord(e[0], A);
    hipStreamWaitEvent(S, e[0], 0);
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, S, d + 4);
    O = S;
  }
  hipEventRecord(e[1], O);
  hipStreamWaitEvent(B, e[1], 0);
  if (!empty) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 8);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, O, d + 4);
  hipEventRecord(e[2], B);
  hipError_t r = hipStreamWaitEvent(O, e[2], 0);
  printf("[%s] join %s\n", c.c_str(), hipGetErrorName(r));
  if (c.find("tail") == std::string::npos) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, O, d + 4);
  if (nested) {
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
    hipEventRecord(e[3], S);
    hipStreamWaitEvent(A, e[3], 0);
  }
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  fflush(stdout);
  r = hipStreamEndCapture(A, &g);
  printf("[%s] end capture %s graph %p\n", c.c_str(), hipGetErrorName(r), (void*)g);
  fflush(stdout);
  if (r == hipSuccess && g) {
    hipGraphExec_t x;
    r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    printf("[%s] instantiate %s\n", c.c_str(), hipGetErrorName(r));
    if (r == hipSuccess) r = hipGraphLaunch(x, A);
    hipStreamSynchronize(A);
    int h[16];
    hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
    printf("[%s] replay %s counters %d %d %d\n", c.c_str(), hipGetErrorName(r), h[0], h[4], h[8]);
  }
  fflush(stdout);
  return 0;
}

static int run_case(const std::string& c) {
  if (c.find("advanced") != std::string::npos) return run_advanced(c);
  if (c.rfind("stale", 0) == 0) return run_stale(c);
  if (c.rfind("reuse_nested", 0) == 0) return run_reuse_nested(c);
  if (c.rfind("nested", 0) == 0) return run_nested(c);
  if (c.rfind("reuse", 0) == 0) return run_reuse(c);
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 90;
  hipStream_t A, B;
  hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  hipEvent_t e1, e2;
  hipEventCreateWithFlags(&e1, hipEventDisableTiming);
  hipEventCreateWithFlags(&e2, hipEventDisableTiming);
  hipGraph_t g = nullptr;
  hipError_t r = hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
  printf("[%s] begin %s\n", c.c_str(), hipGetErrorName(r));
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  const bool fork = c != "create_inside" && c != "err_then_end";
  if (fork) {
    r = hipEventRecord(e1, A);
    printf("[%s] record %s\n", c.c_str(), hipGetErrorName(r));
    r = hipStreamWaitEvent(B, e1, 0);
    printf("[%s] wait %s\n", c.c_str(), hipGetErrorName(r));
    if (c == "joined" || c == "unjoined") hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, B, d + 4);
    if (c == "joined" || c == "joined_empty") {
      hipEventRecord(e2, B);
      hipStreamWaitEvent(A, e2, 0);
    }
  }
  if (c == "create_inside") {
    hipStream_t S;
    hipEvent_t E;
    r = hipStreamCreateWithFlags(&S, hipStreamNonBlocking);
    printf("[%s] stream create %s\n", c.c_str(), hipGetErrorName(r));
    r = hipEventCreateWithFlags(&E, hipEventDisableTiming);
    printf("[%s] event create %s\n", c.c_str(), hipGetErrorName(r));
  }
  if (c == "err_then_end") {
    r = hipMemcpy(d, d + 8, 4, hipMemcpyDeviceToDevice);  // synchronous: not capturable
    printf("[%s] sync memcpy %s\n", c.c_str(), hipGetErrorName(r));
  }
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, A, d);
  fflush(stdout);
  r = hipStreamEndCapture(A, &g);
  printf("[%s] end capture %s graph %p\n", c.c_str(), hipGetErrorName(r), (void*)g);
  if (r == hipSuccess && g) {
    hipGraphExec_t x;
    r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    printf("[%s] instantiate %s\n", c.c_str(), hipGetErrorName(r));
    if (r == hipSuccess) {
      r = hipGraphLaunch(x, A);
      hipStreamSynchronize(A);
      int h[2] = {0, 0};
      hipMemcpy(h, d, 4, hipMemcpyDeviceToHost);
      hipMemcpy(h + 1, d + 4, 4, hipMemcpyDeviceToHost);
      printf("[%s] replay %s counters %d %d\n", c.c_str(), hipGetErrorName(r), h[0], h[1]);
    }
  }
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const char* cases[] = {"joined",        "joined_empty", "unjoined",
                         "unjoined_empty", "create_inside", "err_then_end",
                         "reuse_after_joined", "reuse_after_unjoined_empty",
                         "nested_separate", "nested_kernel", "nested_empty",
                         "reuse_nested_kernel", "reuse_nested_empty", "reuse_nested_fresh",
                         "nested_empty_tail", "nested_kernel_tail", "stale_kernel", "stale_empty",
                         "advanced_empty", "advanced_kernel", "nested_advanced_empty", "nested_advanced_kernel",
                         "nested_advanced_empty_tail", "nested_advanced_kernel_tail"};
  if (argc > 1) return run_case(argv[1]);
  for (const char* c : cases) {
    fflush(stdout);
    pid_t pid = fork();
    if (pid == 0) {
      alarm(30);
      execl(argv[0], argv[0], c, (char*)nullptr);  // (a fresh process: nothing HIP-initialised here yet)
      _exit(99);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    if (WIFSIGNALED(st)) printf("[%s] CHILD KILLED BY SIGNAL %d (%s)\n", c, WTERMSIG(st), strsignal(WTERMSIG(st)));
    else printf("[%s] child exit %d\n", c, WEXITSTATUS(st));
    fflush(stdout);
  }
  return 0;
}

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
// Build: hipcc --offload-arch=gfx950 -O1 -o capture_fork_probe capture_fork_probe.cpp
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>

__global__ void tick(int* p) { if (threadIdx.x == 0) p[0] += 1; }

static int run_case(const std::string& c) {
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
  const char* cases[] = {"joined", "joined_empty", "unjoined", "unjoined_empty", "create_inside", "err_then_end"};
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

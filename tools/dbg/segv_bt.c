/* SIGSEGV diagnostics for a host crash inside a library call (the forked-
 * frontier capture crash in hipStreamEndCapture): install()
 * registers a handler that prints the native backtrace (glibc backtrace) of
 * the faulting thread to stderr, then restores the default action and
 * re-raises.  Loaded with ctypes by the test when PINSAGE_SEGV_BT=1.
 * Build: gcc -shared -fPIC -O1 -g -rdynamic -o segv_bt.so segv_bt.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static void on_segv(int sig, siginfo_t* si, void* ctx) {
  void* frames[64];
  const char hdr[] = "\n[segv_bt] native backtrace:\n";
  write(2, hdr, sizeof(hdr) - 1);
  char addr[64];
  int n = 0;
  unsigned long a = (unsigned long)si->si_addr;
  const char pre[] = "[segv_bt] fault address 0x";
  write(2, pre, sizeof(pre) - 1);
  for (int i = 60; i >= 0; i -= 4) addr[n++] = "0123456789abcdef"[(a >> i) & 15];
  addr[n++] = '\n';
  write(2, addr, n);
  {  /* the faulting thread's stack pointer (a fault just below it: overflow) */
    const ucontext_t* uc = (const ucontext_t*)ctx;
    unsigned long sp = (unsigned long)uc->uc_mcontext.gregs[REG_RSP];
    const char p2[] = "[segv_bt] rsp 0x";
    write(2, p2, sizeof(p2) - 1);
    n = 0;
    for (int i = 60; i >= 0; i -= 4) addr[n++] = "0123456789abcdef"[(sp >> i) & 15];
    addr[n++] = '\n';
    write(2, addr, n);
  }
  int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

/* the handler runs on its own stack, so a fault that is a stack overflow
 * (deep recursion inside the library) still gets its backtrace printed */
static char g_alt[1 << 16];
int install(void) {
  stack_t ss;
  memset(&ss, 0, sizeof(ss));
  ss.ss_sp = g_alt;
  ss.ss_size = sizeof(g_alt);
  if (sigaltstack(&ss, 0) != 0) return -1;
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND | SA_ONSTACK;
  return sigaction(SIGSEGV, &sa, 0);
}

/* Host-side SIGSEGV reporter for diagnosing a crash inside a runtime library: prints the native
   backtrace (backtrace_symbols_fd: module + offset per frame) and the fault address to stderr, then
   re-raises with the default action.  Loaded with ctypes and armed by rgbd_segv_install(); touches
   no GPU state.  Build: gcc -O1 -g -shared -fPIC segv_bt.c -o segv_bt.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <dlfcn.h>

static void report(int sig, siginfo_t* si, void* uctx) {
  (void)uctx;
  char line[256];
  int n = snprintf(line, sizeof line, "\n[segv_bt] signal %d, fault address %p\n", sig, si ? si->si_addr : 0);
  if (n > 0) write(2, line, (size_t)n);
  void* frames[96];
  const int nf = backtrace(frames, 96);
  for (int i = 0; i < nf; ++i) {
    Dl_info di;
    if (dladdr(frames[i], &di) && di.dli_fname) {
      n = snprintf(line, sizeof line, "[segv_bt] #%d %s +0x%lx (%s)\n", i, di.dli_fname,
                   (unsigned long)((char*)frames[i] - (char*)di.dli_fbase), di.dli_sname ? di.dli_sname : "?");
    } else {
      n = snprintf(line, sizeof line, "[segv_bt] #%d %p\n", i, frames[i]);
    }
    if (n > 0) write(2, line, (size_t)n);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int rgbd_segv_install(void) {
  static char stack[1 << 16];
  stack_t ss;
  ss.ss_sp = stack;
  ss.ss_size = sizeof stack;
  ss.ss_flags = 0;
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = report;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, 0) | sigaction(SIGBUS, &sa, 0);
}

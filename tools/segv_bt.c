// Debug aid: a SIGSEGV handler that prints the native backtrace (loaded with
// ctypes.CDLL by a test process; no effect until a segmentation fault).
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <stdlib.h>
#include <unistd.h>

static void on_segv(int sig) {
  static void* frames[256];
  int n = backtrace(frames, 256);
  const char msg[] = "native backtrace (SIGSEGV):\n";
  if (write(2, msg, sizeof(msg) - 1) < 0) return;
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void segv_bt_install(void) {
  stack_t ss;
  ss.ss_sp = malloc(1 << 20);
  ss.ss_size = 1 << 20;
  ss.ss_flags = 0;
  sigaltstack(&ss, 0);   // a handler for a stack overflow needs a stack of its own
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_segv;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
}

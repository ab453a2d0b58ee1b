// Debug aid: on SIGSEGV / SIGBUS / SIGABRT print the native call stack as "library+offset [symbol]" lines
// (symbolise the offsets here with llvm-symbolizer against the same image's libraries), then die with
// the default action.  Loaded with ctypes by tools/x3_capture_diag.py --bt; never preloaded.
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig) {
  static void* pcs[4096];
  int n = backtrace(pcs, 4096);
  char line[512];
  int len = snprintf(line, sizeof line, "[segv_bt] signal %d, %d frames\n", sig, n);
  write(2, line, len);
  for (int i = 0; i < n; ++i) {
    if (i == 40 && n > 80) i = n - 40;  // the innermost and outermost 40 frames
    Dl_info info;
    memset(&info, 0, sizeof info);
    if (dladdr(pcs[i], &info) && info.dli_fname) {
      len = snprintf(line, sizeof line, "[segv_bt] #%d %s+0x%lx %s\n", i, info.dli_fname,
                     (unsigned long)((char*)pcs[i] - (char*)info.dli_fbase), info.dli_sname ? info.dli_sname : "?");
    } else {
      len = snprintf(line, sizeof line, "[segv_bt] #%d %p\n", i, pcs[i]);
    }
    write(2, line, len);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

extern "C" int segv_bt_install() {
  // an alternate stack: a stack overflow (deep recursion) must still reach the handler
  static char alt[1 << 20];
  stack_t ss;
  ss.ss_sp = alt;
  ss.ss_size = sizeof alt;
  ss.ss_flags = 0;
  sigaltstack(&ss, nullptr);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = handler;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  sigaction(SIGABRT, &sa, nullptr);
  return 0;
}

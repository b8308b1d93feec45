/* segv_trace.c — a diagnostic: loaded into a process (ctypes.CDLL), its constructor installs a
 * SIGSEGV/SIGBUS/SIGABRT handler that prints the native backtrace (libraries and offsets) to stderr
 * and exits 139. Used by tools/capture_tiles.py to name the faulting frame of a host crash.
 *   gcc -O1 -g -shared -fPIC -o tools/libsegv_trace.so tools/segv_trace.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
  static const char msg[] = "\n*** segv_trace: fatal signal, native backtrace:\n";
  void* frames[64];
  (void)!write(2, msg, sizeof(msg) - 1);
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

/* (re)install: torch installs fatal-signal handlers of its own when it is imported, so the caller
 * calls this again right before the code under test */
void segv_trace_install(void) {
  /* an alternate stack: a stack overflow (deep recursion) must still reach the handler */
  static char alt[1 << 16];
  stack_t ss;
  memset(&ss, 0, sizeof(ss));
  ss.ss_sp = alt;
  ss.ss_size = sizeof(alt);
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_fault;
  sa.sa_flags = SA_RESETHAND | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
}

__attribute__((constructor)) static void install_at_load(void) { segv_trace_install(); }

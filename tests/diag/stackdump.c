/* stackdump.c — TEST DIAGNOSTICS ONLY: native stacks of a hung test process's threads. A test driver's
 * watchdog installs the handler (sd_install) and signals each thread in turn (sd_signal); the handler
 * writes that thread's return addresses to stderr (backtrace_symbols_fd: "lib.so(+0xOFFSET)"), which
 * `addr2line -f -C -e <lib> 0xOFFSET` resolves against the same .so files in this tree. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

static void sd_handler(int sig) {
  (void)sig;
  void *b[64];
  char hdr[80];
  const int n = backtrace(b, 64);
  const int len = snprintf(hdr, sizeof hdr, "--- native stack of tid %ld\n", (long)syscall(SYS_gettid));
  if (len > 0) (void)!write(2, hdr, (size_t)len);
  backtrace_symbols_fd(b, n, 2);
}

int sd_install(int sig) {
  void *warm[2];
  (void)backtrace(warm, 2); /* loads the unwinder now, not inside the handler */
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = sd_handler;
  sa.sa_flags = SA_RESTART;
  sigemptyset(&sa.sa_mask);
  return sigaction(sig, &sa, NULL);
}

int sd_signal(int tid, int sig) { return (int)syscall(SYS_tgkill, getpid(), tid, sig); }

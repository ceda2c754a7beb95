/* tools/segv_bt.c -- diagnostic: a SIGSEGV/SIGBUS handler that prints the native
 * backtrace of the faulting thread (backtrace_symbols_fd) and the faulting
 * address, then dies with the default action.  Loaded by a probe script with
 * ctypes (its constructor installs the handler); never part of the product.
 *   gcc -O1 -g -shared -fPIC tools/segv_bt.c -o build/libsegv_bt.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t *si, void *uc) {
  (void)uc;
  char msg[128];
  int n = snprintf(msg, sizeof(msg), "\n*** signal %d at address %p; native backtrace:\n", sig, si->si_addr);
  write(2, msg, (size_t)n);
  void *frames[64];
  int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
}

/* Debug aid (not shipped): linked into a host binary, prints a backtrace on SIGSEGV / SIGABRT. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
static void on_fault(int sig) {
    void* b[64];
    int n = backtrace(b, 64);
    backtrace_symbols_fd(b, n, 2);
    _exit(128 + sig);
}
__attribute__((constructor)) static void install(void) {
    signal(SIGSEGV, on_fault);
    signal(SIGABRT, on_fault);
}

/* Diagnostic only (never loaded by the product): a SIGSEGV / SIGBUS / SIGABRT handler that
 * writes the faulting address and the native backtrace (library + offset per frame) to stderr,
 * so a crash inside the HIP runtime (libamdhip64, stripped: offsets are resolved offline against
 * the same image's library) is located.  Built by tools/crash_probe.py with gcc. */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig, siginfo_t *si, void *uc) {
    (void)uc;
    void *buf[96];
    char msg[160];
    int n = backtrace(buf, 96);
    int len = snprintf(msg, sizeof msg, "crashtrace: signal %d, fault address %p, %d frames\n", sig, si->si_addr, n);
    if (write(2, msg, (size_t)len) < 0) {}
    backtrace_symbols_fd(buf, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

void crashtrace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGBUS, &sa, 0);
    sigaction(SIGABRT, &sa, 0);
}

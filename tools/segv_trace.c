/* Native stack on a fatal signal, for exit-path probes (tools/tab_exit_probe.py
 * with PROBE_SEGV=1): backtrace() of the faulting thread with the library of
 * every frame (backtrace_symbols_fd), the faulting address, then the default
 * action.  Diagnostics only, built by hand:
 *   gcc -shared -fPIC -O1 -g tools/segv_trace.c -o tools/libsegv_trace.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void on_fatal(int sig, siginfo_t* si, void* uc) {
    (void)uc;
    char buf[128];
    int n = snprintf(buf, sizeof buf, "\n[segv_trace] signal %d at address %p; native stack:\n", sig, si->si_addr);
    if (n > 0) (void)!write(2, buf, (size_t)n);
    void* frames[64];
    const int k = backtrace(frames, 64);
    backtrace_symbols_fd(frames, k, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_fatal;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);
    sigaction(SIGABRT, &sa, NULL);
    return 0;
}

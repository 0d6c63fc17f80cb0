// stackdump.c -- diagnostics (not product code): a native backtrace of every
// thread of the calling process (SIGUSR2 to each thread in turn,
// backtrace_symbols_fd in the handler), for a process whose stuck call a
// Python-level watchdog cannot see into (scripts/probe/watchdog_run.py).
//   gcc -O1 -fPIC -shared scripts/probe/stackdump.c -o build/libstackdump.so
#define _GNU_SOURCE
#include <dirent.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

static int g_fd = 2;
static volatile int g_done = 0;

static void handler(int sig) {
    (void)sig;
    void* fr[64];
    int n = backtrace(fr, 64);
    char hdr[64];
    int l = snprintf(hdr, sizeof hdr, "--- thread %ld\n", (long)syscall(SYS_gettid));
    if (l > 0) (void)!write(g_fd, hdr, (size_t)l);
    backtrace_symbols_fd(fr, n, g_fd);
    __atomic_add_fetch(&g_done, 1, __ATOMIC_RELEASE);
}

int sd_backtraces(int fd) {
    struct sigaction sa, old;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = handler;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESTART;
    void* warm[4];
    (void)backtrace(warm, 4);
    g_fd = fd;
    if (sigaction(SIGUSR2, &sa, &old) != 0) return -1;
    long self = (long)syscall(SYS_gettid);
    int answered = 0;
    DIR* d = opendir("/proc/self/task");
    if (d) {
        struct dirent* e;
        while ((e = readdir(d))) {
            long tid = atol(e->d_name);
            if (tid <= 0 || tid == self) continue;
            int before = __atomic_load_n(&g_done, __ATOMIC_ACQUIRE);
            if (syscall(SYS_tgkill, getpid(), tid, SIGUSR2) != 0) continue;
            for (int i = 0; i < 200 && __atomic_load_n(&g_done, __ATOMIC_ACQUIRE) == before; ++i) usleep(1000);
            if (__atomic_load_n(&g_done, __ATOMIC_ACQUIRE) != before) ++answered;
            else dprintf(fd, "--- thread %ld: no answer\n", tid);
        }
        closedir(d);
    }
    sigaction(SIGUSR2, &old, NULL);
    return answered;
}

// Wall-clock sampling of ONE thread (the caller of sampler_start): a CLOCK_MONOTONIC POSIX timer delivers SIGPROF to
// that thread only (SIGEV_THREAD_ID) every period; the handler stores the interrupted instruction pointer. Used by
// scripts/host_sample.py to see where SNARK::prove's calling thread spends its time (host work on the critical
// path, spin waits, HIP calls). Not part of the product.
// gcc -O2 -shared -fPIC -o scripts/micro/libsampler.so scripts/micro/sampler.c -lrt
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

enum { kScan = 60 };  // stack words copied per sample (the main thread's stack is deep: Python below)
static uint64_t* buf;
static volatile size_t n, cap;
static timer_t tid;
static int armed;

// each sample: the interrupted RIP and up to 3 return addresses from the frame-pointer chain (0 where the chain
// ends or leaves the stack window above RSP; libraries built without frame pointers give meaningless callers)
static void on_prof(int sig, siginfo_t* si, void* ucv) {
  (void)sig;
  (void)si;
  ucontext_t* uc = (ucontext_t*)ucv;
  if (n + 4 + kScan > cap) return;
  uint64_t* o = buf + n;
  o[0] = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
  uint64_t rsp = (uint64_t)uc->uc_mcontext.gregs[REG_RSP], fp = (uint64_t)uc->uc_mcontext.gregs[REG_RBP];
  for (int k = 1; k < 4; k++) {
    o[k] = 0;
    if (fp < rsp || fp > rsp + (8u << 20) || (fp & 7)) continue;
    const uint64_t* f = (const uint64_t*)fp;
    o[k] = f[1];
    if (f[0] <= fp) fp = 0;
    else fp = f[0];
  }
  // the top of the stack, for callers through frames without frame pointers (libc, the HIP runtime): the
  // analysis takes the first word that is a return address into libspg
  const uint64_t* st = (const uint64_t*)rsp;
  for (int k = 0; k < kScan; k++) o[4 + k] = st[k];
  n += 4 + kScan;
}

int sampler_start(size_t capacity, long period_ns) {
  if (armed) return -1;
  buf = (uint64_t*)malloc(capacity * sizeof(uint64_t));
  if (!buf) return -2;
  cap = capacity;
  n = 0;
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, NULL)) return -3;
  struct sigevent sev;
  memset(&sev, 0, sizeof(sev));
  sev.sigev_notify = SIGEV_THREAD_ID;
  sev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
  sev.sigev_signo = SIGPROF;
  if (timer_create(CLOCK_MONOTONIC, &sev, &tid)) return -4;
  struct itimerspec its;
  its.it_interval.tv_sec = 0;
  its.it_interval.tv_nsec = period_ns;
  its.it_value = its.it_interval;
  if (timer_settime(tid, 0, &its, NULL)) return -5;
  armed = 1;
  return 0;
}

size_t sampler_stop(uint64_t* out, size_t out_cap) {
  if (!armed) return 0;
  struct itimerspec its;
  memset(&its, 0, sizeof(its));
  timer_settime(tid, 0, &its, NULL);
  timer_delete(tid);
  armed = 0;
  signal(SIGPROF, SIG_IGN);
  size_t k = n < out_cap ? n : out_cap;
  memcpy(out, buf, k * sizeof(uint64_t));
  free(buf);
  buf = NULL;
  return k;
}

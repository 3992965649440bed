#include <map>
#include <thread>
#include <mutex>
#include <condition_variable>
#include <algorithm>
#include <chrono>
#include <string.h>
// spg — context management for the C-ABI (include/spg.h).
#include <ctype.h>
#include <stdio.h>
#include <string.h>

#include "comm.hpp"
#include "ctx.hpp"
#include "hpool.hpp"

namespace spg {

int set_err(spg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = c->ws_violation.empty() ? msg : c->ws_violation + " (then: " + msg + ")";
  return code;
}

void* pinned_get(spg_ctx* c, size_t bytes) {
  if (bytes <= c->pinned_bytes) return c->pinned;
  if (c->pinned) {
    hipStreamSynchronize(c->stream);  // the old staging may still be the source or target of a copy
    hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_bytes = 0;
  }
  size_t sz = std::max<size_t>((bytes + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1), 1 << 20);
  if (hipHostMalloc(&c->pinned, sz) != hipSuccess) {
    c->pinned = nullptr;
    return nullptr;
  }
  c->pinned_bytes = sz;
  return c->pinned;
}

void* enc_stage_get(spg_ctx* c, size_t bytes) {
  if (bytes <= c->enc_stage_bytes) return c->enc_stage;
  if (c->enc_stage) hipHostFree(c->enc_stage);
  c->enc_stage = nullptr;
  c->enc_stage_bytes = 0;
  const size_t sz = std::max<size_t>((bytes + (1 << 16) - 1) & ~(size_t)((1 << 16) - 1), 1 << 16);
  if (hipHostMalloc(&c->enc_stage, sz) != hipSuccess) {
    c->enc_stage = nullptr;
    return nullptr;
  }
  c->enc_stage_bytes = sz;
  return c->enc_stage;
}

// ---- streamed uploads (h2d_stream): T workers, each with its own copy stream and two page-locked chunk slots. A
// call hands every worker its chunks (k, k + T, ..) under one generation number and waits until all of them have
// copied their last chunk out of the caller's buffer and queued its DMA.
static constexpr size_t kUpChunk = (size_t)4 << 20;

struct Uploader {
  struct Lane {
    hipStream_t s = nullptr;
    void* slot[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int u = 0;
  };
  std::vector<Lane> lanes;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  uint64_t gen = 0;
  int remaining = 0, err = 0;
  bool quit = false;
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  size_t bytes = 0, ch = kUpChunk;  // this call's chunk size (<= kUpChunk: smaller uploads use every worker)

  int start(int device, int T) {
    lanes.resize(T);
    for (auto& L : lanes) {
      if (hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking) != hipSuccess) return SPG_E_HIP;
      for (int u = 0; u < 2; u++) {
        if (hipHostMalloc(&L.slot[u], kUpChunk) != hipSuccess) return SPG_E_NOMEM;
        if (hipEventCreateWithFlags(&L.ev[u], hipEventDisableTiming) != hipSuccess) return SPG_E_HIP;
      }
    }
    for (int k = 0; k < T; k++) th.emplace_back([this, device, k] { worker(device, k); });
    return SPG_OK;
  }
  void worker(int device, int k) {
    hipSetDevice(device);
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
      }
      Lane& L = lanes[k];
      int e = 0;
      const size_t T = lanes.size();
      for (size_t c = k; c * ch < bytes && !e; c += T) {
        const size_t off = c * ch, len = std::min(ch, bytes - off);
        if (L.used[L.u] && hipEventSynchronize(L.ev[L.u]) != hipSuccess) e = SPG_E_HIP;  // the slot's last DMA read it
        if (e) break;
        memcpy(L.slot[L.u], src + off, len);
        if (hipMemcpyAsync(dst + off, L.slot[L.u], len, hipMemcpyHostToDevice, L.s) != hipSuccess ||
            hipEventRecord(L.ev[L.u], L.s) != hipSuccess)
          e = SPG_E_HIP;
        L.used[L.u] = true;
        L.u ^= 1;
      }
      std::lock_guard<std::mutex> lk(mu);
      if (e && !err) err = e;
      if (--remaining == 0) done_cv.notify_all();
    }
  }
  int run(uint8_t* d, const uint8_t* s, size_t n) {
    std::unique_lock<std::mutex> lk(mu);
    dst = d;
    src = s;
    bytes = n;
    // about two chunks per worker, 256 KB .. 4 MB, 64 KB multiples
    static const size_t fixed = getenv("SPG_H2D_CHUNK_KB") ? (size_t)atol(getenv("SPG_H2D_CHUNK_KB")) << 10 : 0;
    const size_t want = (n / (2 * lanes.size()) + 65535) & ~(size_t)65535;
    ch = fixed ? std::min(kUpChunk, fixed) : std::min(kUpChunk, std::max<size_t>((size_t)256 << 10, want));
    err = 0;
    remaining = (int)lanes.size();
    gen++;
    cv.notify_all();
    done_cv.wait(lk, [&] { return remaining == 0; });
    return err;
  }
  void sync() {
    for (auto& L : lanes) hipStreamSynchronize(L.s);
  }
  ~Uploader() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
    for (auto& L : lanes) {
      if (L.s) {
        hipStreamSynchronize(L.s);
        hipStreamDestroy(L.s);
      }
      for (int u = 0; u < 2; u++) {
        if (L.slot[u]) hipHostFree(L.slot[u]);
        if (L.ev[u]) hipEventDestroy(L.ev[u]);
      }
    }
  }
};

int h2d_stream(spg_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!bytes) return 0;
  // default: one pageable hipMemcpyAsync (HIP stages it through its own page-locked buffers at ~56 GB/s on the box, and
  // returns once the caller's bytes are staged). SPG_H2D=1: the upload workers below -- as fast when they run, but 8 more
  // busy threads beside the pool's spinning workers pass the job's CPU quota and the process is throttled for ~9 ms at
  // a time (scripts/upload_probe.py, profiles/r06_upload_probe.txt: 268 MB in 4.7 ms either way, 13-80 ms with stalls)
  static const bool on = getenv("SPG_H2D") && atoi(getenv("SPG_H2D")) != 0;
  if (!on) {
    SPG_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return 0;
  }
  if (!c->up) {
    // 8 workers (measured best on the box: 4 / 8 / 16 -> 44 / 50 / 45 GB/s), fewer under a smaller CPU share
    static const int T0 = getenv("SPG_H2D_THREADS") ? atoi(getenv("SPG_H2D_THREADS")) : 8;
    const int T = std::max(1, std::min(T0, usable_cpus()));
    c->up = new Uploader();
    if (int rc = c->up->start(c->device, T)) {
      delete c->up;
      c->up = nullptr;
      return set_err(c, rc, "upload workers");
    }
  }
  static const bool trace = getenv("SPG_H2D_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  if (int rc = c->up->run((uint8_t*)dst, (const uint8_t*)src, bytes)) return set_err(c, rc, "streamed upload");
  if (trace)
    fprintf(stderr, "[spg h2d] %zu bytes, chunk %zu, %d workers: %.1f us\n", bytes, c->up->ch, (int)c->up->lanes.size(),
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  // the context stream waits for every worker's last DMA
  for (auto& L : c->up->lanes)
    if (L.used[L.u ^ 1]) SPG_HIP(c, hipStreamWaitEvent(c->stream, L.ev[L.u ^ 1], 0));
  return 0;
}

void h2d_sync(spg_ctx* c) {
  if (c->up) c->up->sync();
}

static constexpr size_t kDevCacheBlocks = 4;
static constexpr size_t kDevCacheBytes = (size_t)2 << 30;

static void dev_cache_trim(spg_ctx* c, size_t keep_blocks, size_t keep_bytes) {
  size_t tot = 0;
  for (auto& b : c->dcache) tot += b.second;
  while (!c->dcache.empty() && (c->dcache.size() > keep_blocks || tot > keep_bytes)) {
    tot -= c->dcache.front().second;
    hipFree(c->dcache.front().first);
    c->dcache.erase(c->dcache.begin());
  }
}

void* dev_cache_get(spg_ctx* c, size_t bytes) {
  int best = -1;
  for (size_t i = 0; i < c->dcache.size(); i++) {
    const size_t b = c->dcache[i].second;
    if (b >= bytes && b <= 2 * bytes && (best < 0 || b < c->dcache[best].second)) best = (int)i;
  }
  if (best >= 0) {
    void* p = c->dcache[best].first;
    c->dcache.erase(c->dcache.begin() + best);
    return p;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) == hipSuccess) return p;
  (void)hipGetLastError();
  dev_cache_trim(c, 0, 0);
  if (hipMalloc(&p, bytes) == hipSuccess) return p;
  (void)hipGetLastError();
  return nullptr;
}

void dev_cache_put(spg_ctx* c, void* p, size_t bytes) {
  if (!p) return;
  if (bytes > kDevCacheBytes) {
    hipFree(p);
    return;
  }
  c->dcache.push_back({p, bytes});
  dev_cache_trim(c, kDevCacheBlocks, kDevCacheBytes);
}

void* mapped_get(spg_ctx* c, size_t bytes, void** dev) {
  static const bool on = !getenv("SPG_MAPPED_BUCKETS") || atoi(getenv("SPG_MAPPED_BUCKETS")) != 0;
  if (!on) return nullptr;
  if (bytes > c->mapped_bytes) {
    if (c->mapped) {
      hipStreamSynchronize(c->stream);
      hipHostFree(c->mapped);
      c->mapped = c->d_mapped = nullptr;
      c->mapped_bytes = 0;
    }
    size_t sz = std::max<size_t>((bytes + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1), 1 << 20);
    void* h = nullptr;
    if (hipHostMalloc(&h, sz, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
    if (hipHostGetDevicePointer(&c->d_mapped, h, 0) != hipSuccess) {
      hipHostFree(h);
      return nullptr;
    }
    c->mapped = h;
    c->mapped_bytes = sz;
  }
  *dev = c->d_mapped;
  return c->mapped;
}

void* ws_get(spg_ctx* c, size_t slot, size_t bytes) {
  std::vector<spg_ctx::Slot>& space = c->stream2 && c->stream == c->stream2 ? c->ws2 : c->ws;
  if (space.size() <= slot) space.resize(slot + 1);
  spg_ctx::Slot& s = space[slot];
#ifdef SPG_CHECKED
  // two streams of one context must never share a slot while the previous owner may still read or write it (the
  // commit queue's side stream once did: the bench's repeated proves saw different bytes)
  if (s.p && s.owner && s.owner != c->stream && hipStreamQuery(s.owner) == hipErrorNotReady) {
    char m[160];
    snprintf(m, sizeof m, "workspace slot %zu taken by stream %p while stream %p still has work queued on it", slot,
             (void*)c->stream, (void*)s.owner);
    fprintf(stderr, "[spg checked] %s\n", m);
    if (c->ws_violation.empty()) c->ws_violation = m;
    return nullptr;
  }
#endif
  if (s.p && s.bytes >= bytes) {
    s.owner = c->stream;
    return s.p;
  }
  if (s.p) {
    hipStreamSynchronize(c->stream);
    if (s.owner && s.owner != c->stream) hipStreamSynchronize(s.owner);
    hipFree(s.p);
    s.p = nullptr;
    s.bytes = 0;
  }
  s.owner = c->stream;
  size_t want = bytes < 256 ? 256 : bytes;
  want += want / 4;  // headroom so repeated slightly-larger calls do not reallocate
  if (hipMalloc(&s.p, want) != hipSuccess) {
    s.p = nullptr;
    return nullptr;
  }
  s.bytes = want;
  return s.p;
}

bool failpoint(const spg_ctx* c, const char* site) {
  static const char* fp = getenv("SPG_FAILPOINT");
  static const int fr = getenv("SPG_FAILPOINT_RANK") ? atoi(getenv("SPG_FAILPOINT_RANK")) : 0;
  return fp && strcmp(fp, site) == 0 && c->rank == fr;
}

int mbox_wait(spg_ctx* ctx, uint32_t seq, Fq* out, int n) {
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t it = 0;; it++) {
    if (__atomic_load_n(ctx->mbox, __ATOMIC_ACQUIRE) == seq) break;
    if ((it & 1023) == 1023) {
      hipError_t e = hipStreamQuery(ctx->stream);
      if (e != hipSuccess && e != hipErrorNotReady) return set_err(ctx, SPG_E_HIP, "mailbox: stream failed");
      if (e == hipSuccess && __atomic_load_n(ctx->mbox, __ATOMIC_ACQUIRE) != seq)
        return set_err(ctx, SPG_E_HIP, "mailbox: kernel finished without posting");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
        return set_err(ctx, SPG_E_HIP, "mailbox: timed out");
    }
  }
  // the posted scalars: their cache lines were written by the device (snooped out of this core's caches), so each is a
  // miss; touch every line first so the misses overlap (one DRAM latency for the lot instead of one per line: a layer's
  // last round posts up to ~300 scalars), then copy. The acquire load of the sequence number above orders these reads
  // after the device's stores; the page does not change again before the next launch.
  const uint8_t* src = (const uint8_t*)(ctx->mbox + 8);
  const size_t bytes = (size_t)n * sizeof(Fq);
  for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(src + o, 0, 0);
  memcpy(out, src, bytes);
  return 0;
}

void down_post(spg_ctx* ctx, uint32_t seq, const Fq& r) {
  for (int i = 0; i < 8; i++) ctx->down[8 + i] = r.l[i];
  __atomic_store_n(ctx->down, seq, __ATOMIC_RELEASE);
}

struct SegArgs {
  const Fq* p[kSegMax];
  uint32_t off[kSegMax + 1];
  int k;
};

// thread i copies scalar i of the concatenated ranges into the result page (plain stores to coherent host memory;
// the stream synchronisation after the launch makes them visible)
__global__ void __launch_bounds__(256) k_gather_res(SegArgs a, Fq* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.off[a.k]) return;
  int j = 0;
  while (i >= a.off[j + 1]) j++;
  const uint4* src = (const uint4*)(a.p[j] + (i - a.off[j]));
  uint4* dst = (uint4*)(out + i);
  dst[0] = src[0];
  dst[1] = src[1];
}

int d2h_multi(spg_ctx* ctx, const FqSeg* segs, int k, Fq* h) {
  size_t total = 0;
  for (int j = 0; j < k; j++) total += segs[j].n;
  if (total == 0) return 0;
  if (k > kSegMax || total > kResScalars) {  // larger downloads: one copy per range through pinned staging
    for (int j = 0; j < k; j++) {
      Fq* st = (Fq*)pinned_get(ctx, segs[j].n * sizeof(Fq));
      if (!st) return set_err(ctx, SPG_E_NOMEM, "download staging");
      SPG_HIP(ctx, hipMemcpyAsync(st, segs[j].d, segs[j].n * sizeof(Fq), hipMemcpyDeviceToHost, ctx->stream));
      SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
      memcpy(h, st, segs[j].n * sizeof(Fq));
      h += segs[j].n;
    }
    return 0;
  }
  SegArgs a;
  a.k = k;
  a.off[0] = 0;
  for (int j = 0; j < k; j++) {
    a.p[j] = segs[j].d;
    a.off[j + 1] = a.off[j] + (uint32_t)segs[j].n;
  }
  hipLaunchKernelGGL(k_gather_res, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, ctx->stream, a, ctx->d_res);
  SPG_HIP(ctx, hipGetLastError());
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (size_t o = 0; o < total * sizeof(Fq); o += 64) __builtin_prefetch((const uint8_t*)ctx->res + o, 0, 0);  // (mbox_wait)
  memcpy(h, ctx->res, total * sizeof(Fq));
  return 0;
}

// ---- host thread placement -------------------------------------------------------------------------------------
static std::vector<int> parse_cpulist(const std::string& path) {
  std::vector<int> out;
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return out;
  char line[8192] = {0};
  if (fgets(line, sizeof(line), f)) {
    char* save = nullptr;
    for (char* tok = strtok_r(line, ",\n", &save); tok; tok = strtok_r(nullptr, ",\n", &save)) {
      int x = 0, y = 0;
      if (sscanf(tok, "%d-%d", &x, &y) == 2)
        for (int k = x; k <= y; k++) out.push_back(k);
      else if (sscanf(tok, "%d", &x) == 1)
        out.push_back(x);
    }
  }
  fclose(f);
  return out;
}
// busy jiffies per CPU from /proc/stat
static std::map<int, unsigned long long> cpu_busy() {
  std::map<int, unsigned long long> m;
  FILE* f = fopen("/proc/stat", "r");
  if (!f) return m;
  char line[512];
  while (fgets(line, sizeof(line), f)) {
    int cpu;
    unsigned long long u, n, sy, id, io, irq, sirq, st;
    if (sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, &u, &n, &sy, &id, &io, &irq, &sirq, &st) == 9)
      m[cpu] = u + n + sy + irq + sirq + st;
  }
  fclose(f);
  return m;
}
// The prover's host side is a chain of short bursts between Fiat-Shamir challenges: the calling thread, the pool
// workers and the mailbox spin exchange cache lines every few microseconds. Unplaced, those threads land on any
// of the machine's CPUs (two sockets, 16 L3 domains on the MI355X hosts), and every hand-off crosses dies. This
// picks the physical cores of one L3 domain on the GPU's NUMA node — the least busy one over a 20 ms sample — so
// the caller and the workers share an L3 next to the GPU's PCIe root.
std::vector<int> choose_pool_cpus(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return {};
  for (char* q = bus; *q; q++) *q = (char)tolower(*q);
  std::vector<int> local = parse_cpulist(std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist");
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return {};
  // L3 domains of the allowed, GPU-local physical cores (first SMT sibling only)
  std::map<std::string, std::vector<int>> doms;
  for (int c : local) {
    if (c < 0 || c >= CPU_SETSIZE || !CPU_ISSET(c, &allowed)) continue;
    const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(c);
    std::vector<int> sib = parse_cpulist(base + "/topology/thread_siblings_list");
    if (!sib.empty() && sib[0] != c) continue;
    std::vector<int> l3 = parse_cpulist(base + "/cache/index3/shared_cpu_list");
    std::string key;
    for (int x : l3) key += std::to_string(x) + ",";
    doms[key].push_back(c);
  }
  const size_t want = (size_t)pool_threads() + 1;  // the caller and the workers (the pool is not started yet)
  std::map<int, unsigned long long> b0 = cpu_busy();
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  std::map<int, unsigned long long> b1 = cpu_busy();
  std::vector<std::pair<double, std::vector<int>>> cand;  // (busy jiffies, cores) per domain
  for (auto& kv : doms) {
    if (kv.second.size() < want) continue;
    double load = 0;
    for (int c : kv.second) {
      const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(c);
      for (int x : parse_cpulist(base + "/topology/thread_siblings_list")) load += (double)(b1[x] - b0[x]);
    }
    cand.push_back({load, std::vector<int>(kv.second.begin(), kv.second.begin() + want)});
  }
  if (cand.empty()) return {};
  // one process alone: the least busy domain first. Several processes of one node started together (torchrun,
  // LOCAL_WORLD_SIZE > 1) would sample each other's start-up load, so they order the domains by core number
  // instead, which every process sees alike, and each takes the entry at its local rank: distinct domains
  const char* lws = getenv("LOCAL_WORLD_SIZE");
  if (lws && atoi(lws) > 1)
    std::stable_sort(cand.begin(), cand.end(), [](const std::pair<double, std::vector<int>>& a,
                                                  const std::pair<double, std::vector<int>>& b) { return a.second[0] < b.second[0]; });
  else
    std::stable_sort(cand.begin(), cand.end(), [](const std::pair<double, std::vector<int>>& a,
                                                  const std::pair<double, std::vector<int>>& b) { return a.first < b.first; });
  // torchrun: one process per GPU, or several sharing one in rehearsals. Without LOCAL_RANK the least busy domain:
  // a prover started next to a running one sees that one's spinning workers in the sample and goes elsewhere
  const char* lr = getenv("LOCAL_RANK");
  const size_t slot = lr ? (size_t)atoi(lr) : 0;
  return cand[slot % cand.size()].second;
}

static std::map<std::string, long>& copy_counts() {
  static std::map<std::string, long> m;
  return m;
}
void print_copy_counts() {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  std::vector<std::pair<long, std::string>> v;
  for (auto& kv : copy_counts()) v.push_back({kv.second, kv.first});
  std::sort(v.rbegin(), v.rend());
  for (auto& p : v) fprintf(stderr, "[spg] copies %8ld  %s\n", p.first, p.second.c_str());
  copy_counts().clear();
}
hipError_t memcpy_traced(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s, const char* file,
                         int line) {
  static const bool on = getenv("SPG_COPY_TRACE") && atoi(getenv("SPG_COPY_TRACE")) != 0;
  if (on) {
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const char* f = strrchr(file, '/');
    copy_counts()[std::string(f ? f + 1 : file) + ":" + std::to_string(line)]++;
  }
  return (hipMemcpyAsync)(dst, src, n, k, s);
}

void timer_start(spg_ctx* c) { hipEventRecord(c->ev0, c->stream); }
void timer_stop(spg_ctx* c) { hipEventRecord(c->ev1, c->stream); }

static hipEvent_t pool_event(spg_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

KScope::KScope(spg_ctx* ctx, const char* name, double bytes, double ops, double fqm) : c(ctx), idx(-1) {
  if (!c->prof_on) return;
  spg_ctx::ProfRec r;
  r.name = name;
  r.bytes = bytes;
  r.ops = ops;
  r.fqm = fqm;
  r.a = pool_event(c);
  r.b = pool_event(c);
  hipEventRecord(r.a, c->stream);
  c->prof_pending.push_back(r);
  idx = (int)c->prof_pending.size() - 1;
}
KScope::~KScope() {
  if (idx >= 0) hipEventRecord(c->prof_pending[idx].b, c->stream);
}

}  // namespace spg

extern "C" int spg_init(int device, spg_ctx** out) {
  if (!out) return SPG_E_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return SPG_E_NODEVICE;
  if (device < 0 || device >= count) return SPG_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SPG_E_NODEVICE;
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) return SPG_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return SPG_E_HIP;
  // SPG_PIN (default on): the host pool's workers (created on first use) on one L3 domain (CCD) local to the GPU, the
  // least busy one (spg::choose_pool_cpus); the calling thread joins them only inside prover calls (spg::HostPin)
  // and keeps its own affinity otherwise
  const char* pin = getenv("SPG_PIN");
  if ((!pin || atoi(pin) != 0) && spg::pool_cpus().empty()) {
    std::vector<int> cpus = spg::choose_pool_cpus(device);
    if (!cpus.empty()) spg::pool_cpus() = cpus;
  }
  spg_ctx* c = new spg_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_cx, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pre, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&c->d_counter, 64) != hipSuccess ||
      hipMemset(c->d_counter, 0, 64) != hipSuccess) {
    delete c;
    return SPG_E_HIP;
  }
  void* mb = nullptr;
  if (hipHostMalloc(&mb, 2 * spg::kMboxBytes + 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->d_mbox, mb, 0) != hipSuccess) {
    delete c;
    return SPG_E_HIP;
  }
  memset(mb, 0, 2 * spg::kMboxBytes + 4096);
  c->mbox = (volatile uint32_t*)mb;
  c->res = (spg::Fq*)((uint8_t*)mb + spg::kMboxBytes);
  c->d_res = (spg::Fq*)((uint8_t*)c->d_mbox + spg::kMboxBytes);
  c->down = (volatile uint32_t*)((uint8_t*)mb + 2 * spg::kMboxBytes);
  c->d_down = (uint32_t*)((uint8_t*)c->d_mbox + 2 * spg::kMboxBytes);
  *out = c;
  return SPG_OK;
}

extern "C" int spg_free(spg_ctx* c) {
  if (!c) return SPG_OK;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  if (c->stream2) hipStreamSynchronize(c->stream2);
  if (c->comm_owned_free) c->comm_owned_free(c->comm_owned);
  if (c->wt_cache) spg_r1cs_witness_free(c, c->wt_cache);
  spg::dev_cache_trim(c, 0, 0);
  for (auto* space : {&c->ws, &c->ws2})
    for (auto& s : *space)
      if (s.p) hipFree(s.p);
  if (c->up) delete c->up;  // joins the upload workers after their streams drain
  if (c->pinned) hipHostFree(c->pinned);
  if (c->enc_stage) hipHostFree(c->enc_stage);
  if (c->mapped) hipHostFree(c->mapped);
  if (c->mbox) hipHostFree((void*)c->mbox);
  if (c->d_counter) hipFree(c->d_counter);
  hipEventDestroy(c->ev0);
  hipEventDestroy(c->ev1);
  if (c->ev_cx) hipEventDestroy(c->ev_cx);
  if (c->ev_pre) hipEventDestroy(c->ev_pre);
  if (c->ev_side) hipEventDestroy(c->ev_side);
  if (c->stream2) {
    hipStreamSynchronize(c->stream2);
    hipStreamDestroy(c->stream2);
  }
  hipStreamDestroy(c->stream);
  delete c;
  return SPG_OK;
}

extern "C" const char* spg_last_error(const spg_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" double spg_last_kernel_us(const spg_ctx* c) { return c ? c->last_us : 0.0; }

extern "C" int spg_set_comm(spg_ctx* c, int rank, int nranks, spg_allgather_fn fn, void* user) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return SPG_E_ARG;
  if (c->comm_owned_free) c->comm_owned_free(c->comm_owned);
  c->comm_owned = nullptr;
  c->comm_owned_free = nullptr;
  c->rank = rank;
  c->nranks = nranks;
  c->allgather = fn;
  c->comm_user = user;
  return SPG_OK;
}

namespace spg {

int comm_allgather(spg_ctx* c, const Shard& sh, int status, const void* send, size_t bytes, std::vector<uint8_t>& recv) {
  if (sh.n == 1) {
    recv.assign((const uint8_t*)send, (const uint8_t*)send + bytes);
    return status;
  }
  if (!c->allgather) return set_err(c, SPG_E_ARG, "no communicator set (spg_set_comm)");
  // a caller transcript that failed on this rank is this rank's failure (TrFailScope)
  if (!status && c->tr_failed && *c->tr_failed) status = set_err(c, SPG_E_CALLBACK, "transcript callback failed");
  int64_t first = 0;
  if (allgather_with_status(c->allgather, c->comm_user, sh.n, status, send, bytes, recv, &first) != 0)
    return set_err(c, SPG_E_HIP, "allgather failed");
  if (status) return status;
  if (first) return set_err(c, (int)first, "a peer rank failed (status " + std::to_string(first) + ")");
  return 0;
}

int comm_sum_fq(spg_ctx* c, const Shard& sh, int status, Fq* v, size_t n) {
  if (sh.n == 1) return status;
  std::vector<uint8_t> r;
  int rc = comm_allgather(c, sh, status, v, n * sizeof(Fq), r);
  if (rc) return rc;
  sum_over_ranks(r.data(), sh.n, n, v);
  return 0;
}

}  // namespace spg

extern "C" int spg_prof_enable(spg_ctx* c, int on) {
  if (!c) return SPG_E_ARG;
  c->prof_on = on != 0;
  return SPG_OK;
}

// Resolves pending kernel timings; writes up to `max` (name, launches, total_us, bytes, ops, fq products) records.
// names: max x 32 chars (NUL-terminated). Returns the number of records, or a negative error.
extern "C" int spg_prof_read3(spg_ctx* c, char* names, long* launches, double* total_us, double* bytes, double* ops,
                              double* fqm, int max, int reset) {
  if (!c) return SPG_E_ARG;
  hipStreamSynchronize(c->stream);
  hipStreamSynchronize(c->stream2);
  // device busy time = the union of the timed intervals (kernels on the second stream overlap the main one's).
  // A resident launch (scope name ending in "_persist") spans the host's answers between its rounds, so it is left
  // out of "(device_busy)" and counted only in "(device_busy_resident)", the union over every launch.
  if (!c->prof_pending.empty()) {
    std::vector<std::pair<float, float>> iv, iv_all;
    const hipEvent_t base = c->prof_pending.front().a;
    for (auto& r : c->prof_pending) {
      float s = 0.f, e = 0.f;
      if (hipEventElapsedTime(&s, base, r.a) == hipSuccess && hipEventElapsedTime(&e, base, r.b) == hipSuccess) {
        iv_all.push_back({s, e});
        const size_t n = r.name.size();
        if (!(n >= 8 && r.name.compare(n - 8, 8, "_persist") == 0)) iv.push_back({s, e});
      }
    }
    auto union_ms = [](std::vector<std::pair<float, float>>& v) {
      std::sort(v.begin(), v.end());
      double busy = 0, lo = 0, hi = 0;
      bool open = false;
      for (auto& x : v) {
        if (open && x.first <= hi) {
          hi = std::max<double>(hi, x.second);
          continue;
        }
        if (open) busy += hi - lo;
        lo = x.first;
        hi = x.second;
        open = true;
      }
      if (open) busy += hi - lo;
      return busy;
    };
    c->prof_acc["(device_busy)"].us += union_ms(iv) * 1000.0;
    c->prof_acc["(device_busy_resident)"].us += union_ms(iv_all) * 1000.0;
  }
  for (auto& r : c->prof_pending) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, r.a, r.b);
    auto& acc = c->prof_acc[r.name];
    acc.launches += 1;
    acc.us += ms * 1000.0;
    acc.bytes += r.bytes;
    acc.ops += r.ops;
    acc.fqm += r.fqm;
    c->ev_pool.push_back(r.a);
    c->ev_pool.push_back(r.b);
  }
  c->prof_pending.clear();
  int k = 0;
  for (auto& kv : c->prof_acc) {
    if (k >= max) break;
    if (names) {
      strncpy(names + 32 * k, kv.first.c_str(), 31);
      names[32 * k + 31] = 0;
    }
    if (launches) launches[k] = kv.second.launches;
    if (total_us) total_us[k] = kv.second.us;
    if (bytes) bytes[k] = kv.second.bytes;
    if (ops) ops[k] = kv.second.ops;
    if (fqm) fqm[k] = kv.second.fqm;
    k++;
  }
  if (reset) c->prof_acc.clear();
  return k;
}
extern "C" int spg_prof_read2(spg_ctx* c, char* names, long* launches, double* total_us, double* bytes, double* ops,
                              int max, int reset) {
  return spg_prof_read3(c, names, launches, total_us, bytes, ops, nullptr, max, reset);
}
extern "C" int spg_prof_read(spg_ctx* c, char* names, long* launches, double* total_us, double* bytes, int max,
                             int reset) {
  return spg_prof_read2(c, names, launches, total_us, bytes, nullptr, max, reset);
}

// ---- device-resident scalar vectors ----
extern "C" int spg_buf_upload(spg_ctx* c, const uint64_t* host, size_t n, spg_buf** out) {
  if (!c || !out || (!host && n)) return SPG_E_ARG;
  spg_buf* b = new spg_buf();
  b->n = n;
  if (hipMalloc(&b->d, (n ? n : 1) * sizeof(spg::Fq)) != hipSuccess) {
    delete b;
    return spg::set_err(c, SPG_E_NOMEM, "spg_buf_upload");
  }
  if (n) SPG_HIP(c, hipMemcpyAsync(b->d, host, n * sizeof(spg::Fq), hipMemcpyHostToDevice, c->stream));
  SPG_HIP(c, hipStreamSynchronize(c->stream));
  *out = b;
  return SPG_OK;
}
extern "C" int spg_buf_download(spg_ctx* c, const spg_buf* b, uint64_t* host) {
  if (!c || !b || !host) return SPG_E_ARG;
  SPG_HIP(c, hipMemcpyAsync(host, b->d, b->n * sizeof(spg::Fq), hipMemcpyDeviceToHost, c->stream));
  SPG_HIP(c, hipStreamSynchronize(c->stream));
  return SPG_OK;
}
extern "C" size_t spg_buf_len(const spg_buf* b) { return b ? b->n : 0; }
extern "C" int spg_buf_free(spg_ctx* c, spg_buf* b) {
  (void)c;
  if (!b) return SPG_OK;
  if (b->d) hipFree(b->d);
  delete b;
  return SPG_OK;
}

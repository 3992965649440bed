// Microbenchmark: what one transcript-sequential round costs under different ways of getting the round's kernel onto
// the GPU (VERDICT r4 "next round" item 1). A round = the host learns the previous round's result from the mailbox
// (coherent mapped host page), draws a "challenge", the device runs a one-workgroup kernel that consumes it and posts
// its result + sequence number to the mailbox. Modes:
//   hip       hipLaunchKernel per round, challenge in the kernel arguments (what libspg does today)
//   aql_sys   our own HSA queue, the host writes one AQL dispatch packet per round (challenge in a kernarg ring in
//             coherent host memory) and rings the doorbell; system-scope acquire / release fences in the header
//   aql_agt   the same with agent-scope fences
//   gate_and  every round's packet pair queued AHEAD of time: a barrier-AND packet on a per-round HSA signal, then the
//             dispatch; the host writes the challenge to a host slot and sets the round's signal to 0
//   armed     the next round's kernel launched (HIP) before the challenge exists; its lane 0 polls the host slot
// each at two kernel sizes: `tiny` (post only) and `work` (~3 us of dependent 64-bit products + 256 KB written).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o aql_dispatch aql_dispatch.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

struct Args {
  const uint32_t* slot;  // gate / armed: host slot [0] = round number, [8..15] challenge
  uint32_t* mb;          // mailbox: [0] = sequence number, [8..15] result
  uint32_t* dirty;       // device buffer the `work` kernel writes
  uint32_t seq;
  uint32_t chal[8];      // hip / aql: the challenge
  int mode;              // 0: challenge in args; 1: wait for slot[0] == seq, then read the slot
  int work;              // product iterations
  int dirty_words;
};

__device__ __forceinline__ uint32_t round_body(const Args& A, const uint32_t* c) {
  uint64_t x = c[0] | ((uint64_t)c[1] << 32);
  for (int i = 0; i < A.work; i++) x = x * 0x9E3779B97F4A7C15ull + (x >> 17);
  for (int i = threadIdx.x; i < A.dirty_words; i += 256) A.dirty[i] = (uint32_t)x + i;
  return (uint32_t)x;
}

extern "C" __global__ void __launch_bounds__(256) k_round(Args A) {
  __shared__ uint32_t c[8];
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    if (A.mode == 1) {
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(A.slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != A.seq) {
        if (wall_clock64() - t0 > 200000000ull) {  // 2 s
          ok = 0;
          break;
        }
      }
      for (int j = 0; j < 8; j++) c[j] = __hip_atomic_load(A.slot + 8 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      for (int j = 0; j < 8; j++) c[j] = A.chal[j];
    }
  }
  __syncthreads();
  if (!ok) return;
  const uint32_t v = round_body(A, c);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(A.mb + 8, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

#define HC(x)                                                                      \
  do {                                                                             \
    hsa_status_t s_ = (x);                                                         \
    if (s_ != HSA_STATUS_SUCCESS) {                                                \
      const char* m_ = nullptr;                                                    \
      hsa_status_string(s_, &m_);                                                  \
      fprintf(stderr, "%s:%d %s -> %d %s\n", __FILE__, __LINE__, #x, s_, m_ ? m_ : ""); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

struct KInfo {
  uint64_t obj = 0;
  uint32_t karg = 0, group = 0, priv = 0;
  hsa_agent_t agent{};
  std::string name;
};

static hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
  KInfo* k = (KInfo*)d;
  hsa_symbol_kind_t kind;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind);
  if (kind != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
  uint32_t n = 0;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &n);
  std::string nm(n, '\0');
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &nm[0]);
  if (nm != k->name && nm != k->name + ".kd") return HSA_STATUS_SUCCESS;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->obj);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->karg);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv);
  return HSA_STATUS_INFO_BREAK;
}
static hsa_status_t exe_cb(hsa_executable_t e, void* d) {
  KInfo* k = (KInfo*)d;
  hsa_executable_iterate_agent_symbols(e, k->agent, sym_cb, d);
  return k->obj ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}
static hsa_status_t gpu_cb(hsa_agent_t a, void* d) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) {
    *(hsa_agent_t*)d = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

struct Host {
  volatile uint32_t* mb;  // mailbox (host view)
  uint32_t* mb_dev;
  volatile uint32_t* slot;
  uint32_t* slot_dev;
  uint32_t* dirty;
};

static bool wait_mb(const Host& h, uint32_t seq) {
  const auto t0 = clk::now();
  while (__atomic_load_n(h.mb, __ATOMIC_ACQUIRE) != seq)
    if (us_since(t0) > 2e6) return false;
  return true;
}
// ~1 us of "transcript" work between rounds
static void host_work(uint32_t* c, uint32_t v) {
  const auto t0 = clk::now();
  uint64_t x = v;
  while (us_since(t0) < 1.0) x = x * 6364136223846793005ull + 1;
  for (int j = 0; j < 8; j++) c[j] = (uint32_t)(x >> (j * 4)) ^ j;
}

static const int R = 400;

static double run_hip(Host& h, hipStream_t st, Args A, uint32_t& seq) {
  uint32_t c[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  A.mode = 0;
  const auto t0 = clk::now();
  for (int i = 0; i < R; i++) {
    A.seq = ++seq;
    memcpy(A.chal, c, 32);
    hipLaunchKernelGGL(k_round, dim3(1), dim3(256), 0, st, A);
    if (!wait_mb(h, A.seq)) return -1;
    host_work(c, h.mb[8]);
  }
  const double r = us_since(t0) / R;
  hipStreamSynchronize(st);
  return r;
}

static double run_armed(Host& h, hipStream_t st, Args A, uint32_t& seq) {
  uint32_t c[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  A.mode = 1;
  const uint32_t s0 = seq + 1;
  A.seq = s0;
  hipLaunchKernelGGL(k_round, dim3(1), dim3(256), 0, st, A);
  const auto t0 = clk::now();
  for (int i = 0; i < R; i++) {
    const uint32_t s = s0 + i;
    for (int j = 0; j < 8; j++) h.slot[8 + j] = c[j];
    __atomic_store_n(h.slot, s, __ATOMIC_RELEASE);
    if (i + 1 < R) {
      A.seq = s + 1;
      hipLaunchKernelGGL(k_round, dim3(1), dim3(256), 0, st, A);
    }
    if (!wait_mb(h, s)) return -1;
    host_work(c, h.mb[8]);
  }
  const double r = us_since(t0) / R;
  seq = s0 + R - 1;
  hipStreamSynchronize(st);
  return r;
}

struct Aql {
  hsa_queue_t* q;
  KInfo k;
  uint8_t* kargs;  // ring of 512-byte kernarg slots (coherent host memory, or device memory the host writes over BAR)
  uint8_t* kargs_host;
  uint8_t* kargs_dev;
  int nk;
};
// explicit arguments, then the code object v5 hidden arguments at their metadata offsets (llvm-readelf --notes):
// block_count xyz (u32) +0, group_size xyz (u16) +12, remainder xyz (u16) +18, global_offset xyz (u64) +40, grid_dims +64
static Args* put_karg(Aql& a, int slot, const Args& A) {
  uint8_t* k = a.kargs + (size_t)(slot % a.nk) * 512;
  uint8_t buf[512];
  memset(buf, 0, sizeof buf);
  memcpy(buf, &A, sizeof A);
  uint8_t* h = buf + 72;
  const uint32_t bc[3] = {1, 1, 1};
  const uint16_t gs[3] = {256, 1, 1};
  memcpy(h, bc, 12);
  memcpy(h + 12, gs, 6);
  const uint16_t dims = 1;
  memcpy(h + 64, &dims, 2);
  memcpy(k, buf, 328);
  if (a.kargs == a.kargs_dev) (void)*(volatile uint8_t*)(k + 327);  // read back: the BAR writes have landed
  return (Args*)k;
}

static void write_dispatch(Aql& a, uint64_t idx, Args* karg, int scope) {
  hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)a.q->base_address + (idx & (a.q->size - 1));
  memset(((uint8_t*)p) + 4, 0, 60);
  p->workgroup_size_x = 256;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->grid_size_x = 256;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = a.k.priv;
  p->group_segment_size = a.k.group;
  p->kernel_object = a.k.obj;
  p->kernarg_address = karg;
  const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                       (scope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                       (scope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n((uint32_t*)p, hdr | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
}
static void write_barrier(Aql& a, uint64_t idx, hsa_signal_t dep) {
  hsa_barrier_and_packet_t* p = (hsa_barrier_and_packet_t*)a.q->base_address + (idx & (a.q->size - 1));
  memset(((uint8_t*)p) + 4, 0, 60);
  p->dep_signal[0] = dep;
  const uint16_t hdr = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                       (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                       (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  __atomic_store_n((uint32_t*)p, (uint32_t)hdr, __ATOMIC_RELEASE);
}

static double run_aql(Host& h, Aql& a, Args A, uint32_t& seq, int scope) {
  uint32_t c[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  A.mode = 0;
  const auto t0 = clk::now();
  for (int i = 0; i < R; i++) {
    A.seq = ++seq;
    memcpy(A.chal, c, 32);
    Args* ka = put_karg(a, i, A);
    const uint64_t idx = hsa_queue_add_write_index_relaxed(a.q, 1);
    write_dispatch(a, idx, ka, scope);
    hsa_signal_store_screlease(a.q->doorbell_signal, idx);
    if (!wait_mb(h, A.seq)) return -1;
    host_work(c, h.mb[8]);
  }
  return us_since(t0) / R;
}

static double run_gate(Host& h, Aql& a, Args A, uint32_t& seq, int scope, bool value_pkt) {
  uint32_t c[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  A.mode = 1;
  const int G = std::min<int>(R, a.nk);
  std::vector<hsa_signal_t> sig(G);
  for (int i = 0; i < G; i++) HC(hsa_signal_create(1, 0, nullptr, &sig[i]));
  const uint32_t s0 = seq + 1;
  // queue every round ahead: gate i, dispatch i
  uint64_t idx = hsa_queue_add_write_index_relaxed(a.q, 2 * G);
  for (int i = 0; i < G; i++) {
    Args Ai = A;
    Ai.seq = s0 + i;
    Args* ka = put_karg(a, i, Ai);
    if (value_pkt) {
      hsa_amd_barrier_value_packet_t* p =
          (hsa_amd_barrier_value_packet_t*)a.q->base_address + ((idx + 2 * i) & (a.q->size - 1));
      memset(((uint8_t*)p) + 4, 0, 60);
      p->signal = sig[i];
      p->value = 0;
      p->mask = ~0ll;
      p->cond = HSA_SIGNAL_CONDITION_EQ;
      const uint16_t hdr = (HSA_PACKET_TYPE_VENDOR_SPECIFIC << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER);
      __atomic_store_n((uint32_t*)p, (uint32_t)hdr | ((uint32_t)HSA_AMD_PACKET_TYPE_BARRIER_VALUE << 16), __ATOMIC_RELEASE);
    } else {
      write_barrier(a, idx + 2 * i, sig[i]);
    }
    write_dispatch(a, idx + 2 * i + 1, ka, scope);
  }
  hsa_signal_store_screlease(a.q->doorbell_signal, idx + 2 * G - 1);
  const auto t0 = clk::now();
  for (int i = 0; i < G; i++) {
    const uint32_t s = s0 + i;
    for (int j = 0; j < 8; j++) h.slot[8 + j] = c[j];
    __atomic_store_n(h.slot, s, __ATOMIC_RELEASE);
    hsa_signal_store_screlease(sig[i], 0);
    if (!wait_mb(h, s)) {
      for (int k = i + 1; k < G; k++) hsa_signal_store_screlease(sig[k], 0);
      return -1;
    }
    host_work(c, h.mb[8]);
  }
  const double r = us_since(t0) / G;
  seq = s0 + G - 1;
  const auto tq = clk::now();
  while (hsa_queue_load_read_index_scacquire(a.q) < idx + 2 * G)
    if (us_since(tq) > 2e6) {
      fprintf(stderr, "queue did not drain\n");
      exit(1);
    }
  for (auto& s : sig) hsa_signal_destroy(s);
  return r;
}

int main(int argc, char** argv) {
  hipSetDevice(0);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  Host h;
  void *mbh, *slh;
  hipHostMalloc(&mbh, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostMalloc(&slh, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&h.mb_dev, mbh, 0);
  hipHostGetDevicePointer((void**)&h.slot_dev, slh, 0);
  h.mb = (volatile uint32_t*)mbh;
  h.slot = (volatile uint32_t*)slh;
  memset(mbh, 0, 4096);
  memset(slh, 0, 4096);
  hipMalloc(&h.dirty, 1 << 20);
  Args A{};
  A.slot = h.slot_dev;
  A.mb = h.mb_dev;
  A.dirty = h.dirty;
  // one HIP launch so that HIP has loaded the code object; then find it through the loader's executables
  A.seq = 0;
  hipLaunchKernelGGL(k_round, dim3(1), dim3(256), 0, st, A);
  hipStreamSynchronize(st);

  HC(hsa_init());
  Aql a;
  a.k.name = "k_round";
  HC(hsa_iterate_agents(gpu_cb, &a.k.agent) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
  hsa_ven_amd_loader_1_03_pfn_t ld;
  HC(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ld), &ld));
  ld.hsa_ven_amd_loader_iterate_executables(exe_cb, &a.k);
  if (!a.k.obj) {
    fprintf(stderr, "kernel object not found through the loader\n");
    return 1;
  }
  printf("k_round: object %#lx kernarg %u group %u private %u (sizeof Args %zu)\n", a.k.obj, a.k.karg, a.k.group,
         a.k.priv, sizeof(Args));
  HC(hsa_queue_create(a.k.agent, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &a.q));
  a.nk = 2048;
  hipHostMalloc((void**)&a.kargs_host, (size_t)a.nk * 512, hipHostMallocCoherent | hipHostMallocMapped);
  a.kargs = a.kargs_host;
  {  // kernargs in HBM, written by the host through the BAR (what HIP does with HIP_FORCE_DEV_KERNARG)
    struct PoolFind {
      hsa_amd_memory_pool_t pool{};
      bool ok = false;
    } pf;
    HC(hsa_amd_agent_iterate_memory_pools(
        a.k.agent,
        [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
          hsa_amd_segment_t seg;
          hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
          uint32_t fl = 0;
          hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
          if (seg == HSA_AMD_SEGMENT_GLOBAL && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
            ((PoolFind*)d)->pool = p;
            ((PoolFind*)d)->ok = true;
            return HSA_STATUS_INFO_BREAK;
          }
          return HSA_STATUS_SUCCESS;
        },
        &pf) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
    HC(hsa_amd_memory_pool_allocate(pf.pool, (size_t)a.nk * 512, 0, (void**)&a.kargs_dev));
    hsa_agent_t cpu{};
    HC(hsa_iterate_agents(
        [](hsa_agent_t ag, void* d) -> hsa_status_t {
          hsa_device_type_t t;
          hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t);
          if (t == HSA_DEVICE_TYPE_CPU) {
            *(hsa_agent_t*)d = ag;
            return HSA_STATUS_INFO_BREAK;
          }
          return HSA_STATUS_SUCCESS;
        },
        &cpu) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
    HC(hsa_amd_agents_allow_access(1, &cpu, nullptr, a.kargs_dev));
  }
  // device-memory kernargs variant: the host writes the kernarg ring through hipMemcpy ahead of time (gate mode only)
  uint32_t seq = 100;
  for (int rep = 0; rep < 3; rep++) {
    for (int sz = 0; sz < 2; sz++) {
      A.work = sz ? 100 : 0;
      A.dirty_words = sz ? 65536 : 0;
      const char* nm = sz ? "work" : "tiny";
      const double t_hip = run_hip(h, st, A, seq);
      a.kargs = a.kargs_host;
      const double t_sys = run_aql(h, a, A, seq, HSA_FENCE_SCOPE_SYSTEM);
      const double t_agt = run_aql(h, a, A, seq, HSA_FENCE_SCOPE_AGENT);
      a.kargs = a.kargs_dev;
      const double t_sys_d = run_aql(h, a, A, seq, HSA_FENCE_SCOPE_SYSTEM);
      const double t_agt_d = run_aql(h, a, A, seq, HSA_FENCE_SCOPE_AGENT);
      const double t_gand = run_gate(h, a, A, seq, HSA_FENCE_SCOPE_AGENT, false);
      a.kargs = a.kargs_host;
      printf("rep %d %-4s: us/round hip %.2f | host kernargs: aql_sys %.2f aql_agt %.2f | device kernargs: aql_sys %.2f "
             "aql_agt %.2f gate_and %.2f  (1 us host work included)\n",
             rep, nm, t_hip, t_sys, t_agt, t_sys_d, t_agt_d, t_gand);
      if (t_hip < 0 || t_sys < 0 || t_agt < 0 || t_sys_d < 0 || t_agt_d < 0 || t_gand < 0) return 1;
      fflush(stdout);
    }
  }
  // kernel-only time of each size, back to back on the HIP stream (events)
  for (int sz = 0; sz < 2; sz++) {
    A.work = sz ? 100 : 0;
    A.dirty_words = sz ? 65536 : 0;
    A.mode = 0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    for (int i = 0; i < 200; i++) {
      A.seq = ++seq;
      hipLaunchKernelGGL(k_round, dim3(1), dim3(256), 0, st, A);
    }
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%s: back-to-back %.2f us per kernel (events)\n", sz ? "work" : "tiny", ms * 1000 / 200);
  }
  hsa_queue_destroy(a.q);
  return 0;
}

// spg — per-context state: device, stream, error text, timing events and a growable HBM workspace.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spg.h"
#include "curve.hpp"

namespace spg {
struct Uploader;  // api.hip
}

struct spg_ctx {
  int device = -1;
  // spg_set_comb(ctx, 0): this context's MSMs skip the comb tables (comb.hip) and run the bucket pipelines, for an
  // A/B against the fixed-base precomputation (bench.py config 2's no-table leg)
  bool comb_off = false;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_cx = nullptr;  // DotProductProofLog: the Cx MSM's completion, ahead of Bullet round 0 on the stream
  // second stream: SNARK::prove's latency-path witness commits run on it beside the early block_vars MSM on `stream`;
  // ev_pre marks the point of `stream` they follow (everything queued before that MSM)
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_pre = nullptr;
  // R1CS proof: the Z table's fill on `stream2` (beside Az/Bz/Cz and phase 1 on `stream`); phase 2 waits on it
  hipEvent_t ev_side = nullptr;
  void* pinned = nullptr;          // page-locked host staging (pinned_get), grown on demand
  size_t pinned_bytes = 0;
  void* enc_stage = nullptr;       // page-locked staging of points encoded on the host (enc_stage_get)
  size_t enc_stage_bytes = 0;
  // streamed uploads of caller host data (h2d_stream, api.hip): upload workers, each with its own copy stream and two
  // page-locked chunk slots (created on first use, joined by spg_free)
  spg::Uploader* up = nullptr;
  // device blocks of freed witnesses kept for the next upload (dev_cache_get / dev_cache_put)
  std::vector<std::pair<void*, size_t>> dcache;
  // fine-grained (coherent, mapped) host buffer that latency-path kernels write their bucket sums into
  // directly (mapped_get): the host reads them after the stream synchronisation, no D2H copy launch
  void* mapped = nullptr;
  void* d_mapped = nullptr;
  size_t mapped_bytes = 0;
  unsigned* d_counter = nullptr;   // grid-reduction ticket (zero between launches)
  // mailbox in fine-grained (coherent, mapped) host memory: a kernel's last block posts a round's scalars
  // and a sequence number with system-scope stores; the host spins on the number instead of a D2H copy +
  // stream synchronisation (spg::mbox_wait)
  volatile uint32_t* mbox = nullptr;
  uint32_t* d_mbox = nullptr;
  uint32_t mbox_seq = 0;
  // the reverse direction (coherent, mapped host memory after the result page): the host answers a persistent
  // kernel's posted round with the round's challenge and the round's sequence number (spg::down_post); the kernel's
  // workgroups poll word 0 (layer.hpp, k_layer_persist)
  volatile uint32_t* down = nullptr;
  uint32_t* d_down = nullptr;
  // result page (coherent, mapped host memory next to the mailbox): d2h_multi's gather kernel writes the
  // scalars the host needs there, so a download is one small kernel + a stream synchronisation, no blit copy
  spg::Fq* res = nullptr;
  spg::Fq* d_res = nullptr;
  // multi-process proving (spg_set_comm): this process' rank and an allgather provided by the caller
  int rank = 0, nranks = 1;
  spg_allgather_fn allgather = nullptr;
  void* comm_user = nullptr;
  // a transport the library owns (spg_set_comm_rccl), released by the next spg_set_comm* or spg_free
  void* comm_owned = nullptr;
  void (*comm_owned_free)(void*) = nullptr;
  // SNARK::prove's per-prove witness sections (pairwise / perm-root R1CSProofs): kept between proves, refilled in
  // place, so a prove allocates and frees no device memory (a hipFree synchronises the device: ~0.2 ms)
  spg_r1cs_witness* wt_cache = nullptr;
  double last_us = 0.0;
  std::string err;
  // workspace slots: grown on demand, reused across calls (no allocation in steady state). Each stream has its own
  // slot space (ws for `stream`, ws2 for `stream2`), so work queued on the two streams at once can never share a
  // buffer by slot number. `owner` records the stream that took the slot; the checked build (make checked,
  // -DSPG_CHECKED) refuses a slot that another stream still has work queued on.
  struct Slot {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t owner = nullptr;
  };
  std::vector<Slot> ws, ws2;
  std::string ws_violation;  // checked build: the first cross-stream slot conflict (prefixed to the error text)
  // the transcript of the prove in progress when it forwards to caller callbacks (TrCallbacks::failed): every
  // cross-rank exchange carries its failure as this rank's status, so all ranks fail together
  const int* tr_failed = nullptr;
  // optional per-kernel timing (spg_prof_enable): event pairs resolved lazily in spg_prof_read
  bool prof_on = false;
  struct ProfRec {
    std::string name;
    hipEvent_t a, b;
    double bytes;  // algorithmic HBM bytes of the launch (0 = not modelled)
    double ops;    // algorithmic VALU work of the launch in curve mixed additions (0 = not modelled)
    double fqm;    // algorithmic VALU work of the launch in Fq (scalar-field) products (0 = not modelled)
  };
  struct ProfAcc {
    long launches = 0;
    double us = 0.0, bytes = 0.0, ops = 0.0, fqm = 0.0;
  };
  std::vector<ProfRec> prof_pending;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, ProfAcc> prof_acc;  // name -> totals
};

struct spg_buf {  // device-resident scalar vector (Montgomery Fq)
  size_t n = 0;
  spg::Fq* d = nullptr;
};

struct spg_gens {
  size_t n = 0;                  // number of G points; h is point n
  spg::Niels* niels = nullptr;   // n+1 affine Niels points (device)
  spg::Niels* table = nullptr;   // [254][n+1] : table[k][i] = 2^k * P_i (device)
  uint8_t* compressed = nullptr; // (n+1) x 32 host copy
  // comb.hip: a table of small multiples of generators [0, slots) and of generator h, built on first use under
  // comb_mu (contexts on several threads may share one gens). A published table is never freed while the gens
  // lives -- a context may still have launches reading it queued: a wider table replaces it for new launches and
  // the old one waits in comb_retired until spg_gens_free.
  struct Comb {
    spg::Niels* p = nullptr;
    size_t slots = 0, bytes = 0;
    int h = -1;
    int c = 12;  // window width: 253 / c + 1 windows of 2^(c-1) multiples per generator
    int st = 3;  // entry stride in 32-byte coordinates: 3 (96-byte Niels) or 4 (padded to one 128-byte line)
  };
  mutable std::mutex comb_mu;
  mutable Comb comb;
  mutable std::vector<Comb> comb_retired;
};

namespace spg {

// SPG_COPY_TRACE=1: count hipMemcpyAsync calls per source line (printed at exit); every async copy is a blit
// kernel on the stream, so the per-round ones cost a dispatch each
hipError_t memcpy_traced(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s, const char* file, int line);
void print_copy_counts();  // and reset

static const int kTableRows = 254;  // bit offsets 0..253 cover every window of a 253-bit scalar

int set_err(spg_ctx* c, int code, const std::string& msg);
// test failpoint: true when SPG_FAILPOINT names `site` and SPG_FAILPOINT_RANK (default 0) is this context's rank
// (tests/test_gpu_dist.py injects a failure on one rank of a sharded proof this way; unset in production)
bool failpoint(const spg_ctx* c, const char* site);

#define SPG_HIP(ctx, call)                                                                     \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return spg::set_err(ctx, SPG_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define SPG_CHECK(ctx, cond, msg) \
  do {                            \
    if (!(cond)) return spg::set_err(ctx, SPG_E_ARG, msg); \
  } while (0)

// returns a device buffer of at least `bytes` for workspace slot `slot` (contents undefined)
void* ws_get(spg_ctx* c, size_t slot, size_t bytes);

// page-locked host staging of at least `bytes` (contents undefined; valid until the next larger request,
// which synchronises the stream before freeing the old buffer)
void* pinned_get(spg_ctx* c, size_t bytes);
void* enc_stage_get(spg_ctx* c, size_t bytes);  // callers synchronise before returning: no copy is ever in flight
// bytes of caller host memory (pageable) to device memory: the upload workers copy 4 MB chunks (worker k: chunks k,
// k + T, ..) into their own page-locked slots and DMA each on their own stream, so host copies and DMAs of different
// chunks overlap (scripts/micro/h2d_upload.hip on the box: 8 workers ~2.7 ms for 134 MB, 50 GB/s, against 4.5 ms for one
// pageable hipMemcpyAsync). Returns once every byte has left `src` (the caller's buffer is free again); the last DMAs may
// still be in flight, and the context stream waits for them (work queued on it afterwards, and on stream2 behind it, sees
// the data). Default (SPG_H2D unset or 0): one pageable hipMemcpyAsync on the context stream instead, which returns
// once HIP has staged the bytes (measured as fast, and no extra threads; api.hip). Returns 0 or an SPG error code.
int h2d_stream(spg_ctx* c, void* dst, const void* src, size_t bytes);
// waits for every streamed upload of the context (before device memory they target is freed)
void h2d_sync(spg_ctx* c);
// device memory for per-call uploads (witnesses): a block freed earlier by dev_cache_put when one fits (at most twice
// the size asked for), else hipMalloc (after releasing the cached blocks if the first attempt fails); nullptr on failure.
// dev_cache_put keeps a block for reuse (up to 4 blocks / 2 GiB per context; the oldest are freed). A per-prove
// upload of the same shape then skips hipMalloc / hipFree of 10^8-byte buffers.
void* dev_cache_get(spg_ctx* c, size_t bytes);
void dev_cache_put(spg_ctx* c, void* p, size_t bytes);

// coherent mapped host memory of at least `bytes`: host pointer returned, device alias in *dev (contents
// undefined; a larger request synchronises the stream before freeing the old buffer). Null when
// SPG_MAPPED_BUCKETS=0 or on failure: callers then take the device buffer + copy path.
void* mapped_get(spg_ctx* c, size_t bytes, void** dev);

// timing bracket on the context stream
void timer_start(spg_ctx* c);
void timer_stop(spg_ctx* c);

// B fixed-base MSMs of n scalars (device pointers) against generator table g; scalar i of MSM b uses
// generator d_idx[b*n+i] when d_idx is given, else gen_offset + i; d_blinds (B) multiply generator
// h_index (-1: g->n). d_out: B x 32 compressed bytes (device). Stream-ordered, no host sync.
// comb.hip: batches of row MSMs from per-generator-set comb tables (kCombSkip: not applicable, use the buckets)
static const int kCombSkip = -1;
// halve: every scalar times 2^-1 mod l (the points are P / 2, for the host's batched encoding of doubles,
// hcurve.hpp hext_double_and_compress_batch; d_out must then be null)
int msm_comb(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
             const Fq* d_blinds, uint8_t* d_out, int h_index, Ext* ext, bool halve = false);
void comb_free(const spg_gens* g);
// g's comb table covering generators [0, need) (built on first use): 0 with *out set, 1 when the comb does not
// apply (disabled, too wide, over the memory cap), or an SPG error code
int comb_get(spg_ctx* ctx, const spg_gens* g, size_t need, spg_gens::Comb* out);
int msm_batch_device(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                     const Fq* d_blinds, uint8_t* d_out, const uint32_t* d_idx, long h_index, Ext* d_ext = nullptr);
// the same rows (gen_offset 0) with their 32-byte encodings on the host in out (msm.hip: halved comb points encoded as
// doubles on the host pool where the comb applies); synchronous. timed: record the context's stop event right after
// the device work (before the download and the host encodings), for spg_last_kernel_us
int msm_rows_host_enc(spg_ctx* ctx, const spg_gens* g, const Fq* d_scalars, size_t n, size_t B, const Fq* d_blinds,
                      long h_index, uint8_t* out, bool timed = false);

// latency path for small batches (B * n up to a few thousand): same inputs, results left in extended
// coordinates in d_out (B x Ext, device); the caller encodes them (host).
int msm_small_device(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                     const Fq* d_blinds, Ext* d_out, const uint32_t* d_idx, long h_index);

// bucket stage of the latency path only (d_buckets: B x NB Ext); *nb_out = NB
int msm_small_buckets(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                      const Fq* d_blinds, const uint32_t* d_idx, long h_index, Ext* d_buckets, int* nb_out);
// the latency path for many small rows (Hyrax rows of <= ~1K scalars): compressed outputs, d_out: B x 32 (device)
int msm_small_compressed(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                         uint8_t* d_out);
// n extended points (device) -> n x 32 encoded bytes (device), one lane per point, stream-ordered
int compress_ext_device(spg_ctx* ctx, const Ext* d_ext, size_t n, uint8_t* d_out);

// one Bullet round (msm.hip k_bullet_round_q): applies round k-1's fold with (u, uinv) to the device state
// (aa: Montgomery, cw: plain integers; in -> out, double-buffered), then the bucket sums of the round's L and
// R MSMs (2 x (64 + 1) Ext: buckets 1..64, then the top window's carries) into d_buckets; completion is
// posted to the mailbox with *seq_out
int bullet_round_device(spg_ctx* ctx, const spg_gens* g, const Fq* aa_in, const Fq* cw_in, Fq* aa_out, Fq* cw_out,
                        const uint32_t* gidx, const Fq& u, const Fq& uinv, int k, int n, int nk, Ext* d_buckets,
                        uint32_t* seq_out);
static const int kBulletNB = 64;  // buckets per MSM of bullet_round_device (c = 7)
// the comb form of a Bullet round (bullet.hpp k_bullet_comb): partial points of the L and R MSMs, 2 x *per_msm Ext
// into d_parts (at most kBulletPartsMax per MSM), completion posted to the mailbox with *seq_out; the host adds each
// MSM's parts. Returns 1 when g has no comb table for these generators (the caller takes the bucket form).
static const int kBulletPartsMax = 512;
// B MSMs of n Montgomery scalars over generators d_idx[b n + i] (< gmax) from g's comb table, as B x *per_msm partial
// points into d_parts (stream-ordered, no completion post); 1 when the comb does not apply
int comb_msm_parts(spg_ctx* ctx, const spg_gens* g, const Fq* d_scalars, const uint32_t* d_idx, size_t gmax, int n,
                   int B, Ext* d_parts, int* per_msm);
// out[j] = d cw_j (j odd ? u : u^-1) as Montgomery scalars, from the device Bullet rounds' cw (plain integers)
int bullet_delta_scalars(spg_ctx* ctx, const Fq* cw, int n, const Fq& d, const Fq& u, const Fq& uinv, Fq* out);
int bullet_round_comb(spg_ctx* ctx, const spg_gens* g, const Fq* aa_in, const Fq* cw_in, Fq* aa_out, Fq* cw_out,
                      const uint32_t* gidx, size_t gmax, const Fq& u, const Fq& uinv, int k, int n, int nk,
                      Ext* d_parts, uint32_t* seq_out, int* per_msm);

// the mailbox page: sequence number (word 0), then up to kMboxScalars scalars from word 8
static const size_t kMboxBytes = 65536;
static const size_t kMboxScalars = (kMboxBytes - 32) / 32;
static const size_t kResScalars = kMboxBytes / sizeof(Fq);
// a few device scalar ranges downloaded at once: one gather launch into the result page, one synchronisation
struct FqSeg {
  const Fq* d;
  size_t n;
};
static const int kSegMax = 16;
int d2h_multi(spg_ctx* ctx, const FqSeg* segs, int k, Fq* h);
inline int d2h_multi(spg_ctx* ctx, std::initializer_list<FqSeg> segs, Fq* h) {
  return d2h_multi(ctx, segs.begin(), (int)segs.size(), h);
}
// waits (spinning, bounded) until the mailbox carries sequence number `seq`, then copies n scalars out
int mbox_wait(spg_ctx* ctx, uint32_t seq, Fq* out, int n);
// the host's answer to a persistent kernel: r in words 8..15, then (x86 stores are ordered) seq in word 0
static const uint32_t kDownAbort = 0xffffffffu;
void down_post(spg_ctx* ctx, uint32_t seq, const Fq& r);

// agent-scope write-through (sc1) accesses of HBM scalars handed from one workgroup to another inside a launch
// (MI355X_MICROARCH hand-off table, row 1: sc1 stores, each storing wave drained before its signal, sc1 loads)
typedef __attribute__((address_space(1))) uint64_t gu64_t;  // global (not flat) accesses
__device__ __forceinline__ Fq ld_sc1(const Fq* p) {
  Fq r;
  gu64_t* w = (gu64_t*)p;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t v = __hip_atomic_load(w + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r.l[2 * i] = (uint32_t)v;
    r.l[2 * i + 1] = (uint32_t)(v >> 32);
  }
  return r;
}
__device__ __forceinline__ void st_sc1(Fq* p, const Fq& v) {
  gu64_t* w = (gu64_t*)p;
#pragma unroll
  for (int i = 0; i < 4; i++)
    __hip_atomic_store(w + i, (uint64_t)v.l[2 * i] | ((uint64_t)v.l[2 * i + 1] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// A scalar into coherent (fine-grained) host memory as two plain 16-byte stores, made visible by the system-scope
// release fence that every post puts before its sequence number. Per-word system-scope atomic stores (what the posts
// used through round 4) go out as one host write transaction per 4-byte word, serialised at ~45 ns each: a round's 3
// scalars cost 2.2 us more from launch to host-visible, a layer's 147 posted entries 53 us
// (scripts/micro/mbox_post.hip, profiles/r05_mbox_post.txt). Addresses are 32-byte aligned (mailbox slots).
__device__ __forceinline__ void host_put(uint32_t* p, const Fq& v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4* q = (u32x4*)p;
  q[0] = u32x4{v.l[0], v.l[1], v.l[2], v.l[3]};
  q[1] = u32x4{v.l[4], v.l[5], v.l[6], v.l[7]};
}
// device side of the mailbox: the scalars, then (after a system-scope release fence) the sequence number
__device__ __forceinline__ void mbox_post(uint32_t* mb, uint32_t seq, const Fq* v, int n) {
  for (int k = 0; k < n; k++) host_put(mb + 8 + 8 * k, v[k]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// three scalars (a sumcheck round's e0, e2, e3) without a local array: the array form's runtime-indexed loop put it
// in scratch memory, and a kernel with a private segment costs more to dispatch
__device__ __forceinline__ void mbox_post3(uint32_t* mb, uint32_t seq, const Fq& a, const Fq& b, const Fq& c) {
  host_put(mb + 8, a);
  host_put(mb + 16, b);
  host_put(mb + 24, c);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- multi-process collectives (spg_set_comm) -----------------------------------------------------------
// One shard of an SPMD call: rank `rank` of `n` processes (n == 1: this process alone, no communication).
struct Shard {
  int rank = 0, n = 1;
};
inline Shard ctx_shard(const spg_ctx* c) { return Shard{c->rank, c->nranks}; }
// balanced split of [0, n) into `parts`: part r is [shard_begin(n, parts, r), shard_begin(n, parts, r + 1)),
// the first n % parts parts one longer
inline size_t shard_begin(size_t n, int parts, int r) {
  return (size_t)r * (n / (size_t)parts) + std::min((size_t)r, n % (size_t)parts);
}
// allgather through the context's callback, carrying every rank's status: recv holds rank 0's `bytes`, then
// rank 1's, ...; returns 0 only when every rank's status is 0 (a failure on any rank fails all of them alike,
// so no rank is left blocked in a later collective). sh.n == 1: a local copy.
int comm_allgather(spg_ctx* c, const Shard& sh, int status, const void* send, size_t bytes, std::vector<uint8_t>& recv);
// v[0..n) summed mod q over the ranks (in place), with the same status rule
int comm_sum_fq(spg_ctx* c, const Shard& sh, int status, Fq* v, size_t n);

// per-kernel profiling scope (no-op unless spg_prof_enable(ctx, 1))
struct KScope {
  spg_ctx* c;
  int idx;
  KScope(spg_ctx* ctx, const char* name, double bytes = 0.0, double ops = 0.0, double fqm = 0.0);
  ~KScope();
};

}  // namespace spg

#ifndef SPG_NO_COPY_TRACE
#define hipMemcpyAsync(d, src, n, k, st) spg::memcpy_traced(d, src, n, k, st, __FILE__, __LINE__)
#endif

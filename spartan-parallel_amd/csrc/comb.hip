// spg — comb tables for batches of Hyrax row commitments (DensePolynomial::commit_inner, src/dense_mlpoly.rs:184-212,
// through Commitments::commit, src/commitments.rs:69-92).
//
// A batch of B row MSMs over the SAME R <= 1024 generators (every Hyrax row of a polynomial, every polynomial of a
// commit-queue group) is the prover's biggest latency item at the start of SNARK::prove: the 2 x 512 x 1024 block
// witness is 1024 rows of 1024 scalars. The bucket pipeline (msm.hip) sorts 25 M signed digits into 1024 x 1024
// buckets and then reduces 2 M buckets with running sums. Here the generators' small multiples are precomputed
// instead, once per generator set, in HBM (288 GB per GPU leaves room for it):
//   comb[w][s][m - 1] = m * 2^(c w) * G_s   (affine Niels, 96 B),  m = 1 .. 2^(c-1), w < W = 253 / c + 1,
// s < R and one more slot for h. A signed c-bit digit d of scalar i in window w is then ONE table entry
// +-comb[w][i][|d| - 1], and a row commitment is a plain sum of n W points: no digit sort, no buckets, no running
// sums. With c = 12 (W = 22, 2048 multiples) the table is 22 x 1025 x 2048 x 96 B = 4.4 GB for R = 1024 and a row
// costs 22 mixed additions per scalar (the bucket path: 24 at c = 11, plus its bucket reduction).
//   k_comb_build : one lane per run of 64 consecutive multiples of one (w, s): the first by double-and-add, the
//                  rest by repeated mixed addition; one batched inversion (Montgomery's trick over the run, Z
//                  through a global scratch) to affine Niels.
//   k_comb_accum : 256-thread workgroups, S per row (S = 2 for 1024 rows of 1024): every lane recodes its scalars
//                  into signed digits (staged in LDS) and adds their entries in one-lane mixed additions; the lane
//                  sums meet per quad (DPP) and in a 6-level LDS quad tree (quad.hpp); k_comb_join adds a row's S parts.
// The points are the group elements the bucket path computes, so the encodings (k_compress_ext) are identical.
#include <string.h>

#include <atomic>
#include <chrono>

#include "ctx.hpp"
#include "hcurve.hpp"
#include "hvec.hpp"
#include "hpool.hpp"
#include "lds.hpp"
#include "quad.hpp"

namespace spg {

// window width of the tables up to kCombSmall generators: 13 (20 windows, 4096 multiples: 10.7 GB at 1024 generators
// with 128-byte entries; the 1024 x 1024 row batch 1.02 -> 0.93 ms against 12, profiles/r05_ab_comb_c13.txt); of the
// tables between that and kCombWide: 12 (config 5's ops / memory tables: at 13 they crowd its 2^14-generator derefs
// table out of the memory cap, which then falls back to 12-bit windows, 183 -> 189 ms per proof). SPG_COMB_C = 10 .. 13
// sets both.
static constexpr size_t kCombSmall = 1024;
static int comb_c(size_t slots) {
  static const int c = getenv("SPG_COMB_C") ? std::max(10, std::min(13, atoi(getenv("SPG_COMB_C")))) : 0;
  return c ? c : (slots <= kCombSmall ? 13 : 12);
}
static constexpr int kCombRun = 64;                 // multiples per build lane
static constexpr size_t kCombMaxR = 65536;          // most generators a table covers
static constexpr size_t kCombWide = 16384;          // tables past this many generators take the narrow window
static constexpr size_t kCombBig = 16384;           // tables of this many generators take the big window when it fits
// wider tables take c = 9 (SPG_COMB_C_WIDE: 9 or 10): 2^16 generators are 29 x 65537 x 256 x 96 B = 47 GB, where
// c = 12 would need 283 GB. Tables of exactly kCombBig generators (the SPARK derefs rows of 2^14 at 2^24 nonzeros)
// take c = 13 (SPG_COMB_C_BIG: 12 or 13): 20 windows instead of 22, so 9 % fewer mixed additions per scalar, for a
// 129 GB table instead of 70 GB; where that does not fit (cap, free HBM) the table falls back to c = 12
static int comb_c_for(size_t slots) {
  static const int cw = getenv("SPG_COMB_C_WIDE") ? std::max(9, std::min(10, atoi(getenv("SPG_COMB_C_WIDE")))) : 9;
  static const int cb = getenv("SPG_COMB_C_BIG") ? std::max(12, std::min(13, atoi(getenv("SPG_COMB_C_BIG")))) : 13;
  if (slots > kCombWide) return cw;
  if (slots == kCombBig && !getenv("SPG_COMB_C")) return cb;
  return comb_c(slots);
}

// lane L = ((w * NS + s) * runs + k): multiples k * Run + 1 .. (k + 1) * Run of 2^(c w) G_gen, gen = s (s < NS - 1)
// or hgen (s = NS - 1)
// (lanes lane0 .. lane0 + chunk of the whole table per launch: the Z scratch covers one chunk)
template <int C>
__global__ void __launch_bounds__(64) k_comb_build(const Niels* __restrict__ tab, int n1, int NS, int hgen,
                                                   Niels* __restrict__ comb, Fp* __restrict__ zs, size_t lanes,
                                                   size_t lane0, int st) {
  constexpr int NB = 1 << (C - 1);
  const size_t L = lane0 + (size_t)blockIdx.x * 64 + threadIdx.x;
  if (L >= lanes) return;
  constexpr int runs = NB / kCombRun;
  const int k = (int)(L % runs);
  const size_t ws = L / runs;
  const int s = (int)(ws % NS), w = (int)(ws / NS);
  const int gen = s == NS - 1 ? hgen : s;
  const Niels bn = tab[(size_t)(w * C) * n1 + gen];
  // (k Run + 1) * base, most significant bit first
  const uint32_t m0 = (uint32_t)k * kCombRun + 1u;
  Ext P = niels_to_ext(bn);
  for (int b = 30 - __builtin_clz(m0); b >= 0; b--) {
    P = ext_dbl(P);
    if ((m0 >> b) & 1u) P = ext_madd(P, bn, false);
  }
  // entry j of the run: coordinates out[j * st + 0..2] (ypx, ymx, t2d; st = 4 leaves a pad coordinate)
  Fp* out = reinterpret_cast<Fp*>(comb) + (ws * NB + (size_t)k * kCombRun) * st;
  Fp* z = zs + (L - lane0) * kCombRun;
  // forward: X, Y parked in the entry, the prefix product of the Z's in its third field, Z in the scratch
  Fp pp = fp_one();
  for (int j = 0; j < kCombRun; j++) {
    if (j) P = ext_madd(P, bn, false);
    pp = fp_mul(pp, P.Z);
    out[j * st] = P.X;
    out[j * st + 1] = P.Y;
    out[j * st + 2] = pp;
    z[j] = P.Z;
  }
  // backward: 1/Z_j = (1 / prod_{i <= j} Z_i) * prod_{i < j} Z_i
  Fp inv = fp_inv(pp);
  for (int j = kCombRun - 1; j >= 0; j--) {
    const Fp zi = j ? fp_mul(inv, out[(j - 1) * st + 2]) : inv;
    if (j) inv = fp_mul(inv, z[j]);
    const Fp x = fp_mul(out[j * st], zi), y = fp_mul(out[j * st + 1], zi);
    out[j * st] = fp_canon(fp_add(y, x));
    out[j * st + 1] = fp_canon(fp_sub(y, x));
    out[j * st + 2] = fp_canon(fp_mul(fp_mul(x, y), c_d2()));
    if (st == 4) out[j * st + 3] = fp_zero();
  }
}

// workgroup (row b, part h) of S per row, G window groups per scalar: wave v of the workgroup takes window group
// j = v mod G (uniform per wave, so no divergence) of its 64 scalars (v / G) * 64 + lane of the workgroup's 256 / G;
// part h covers scalars h * 256/G + i_local + k * S * 256/G of the row (+ blind_b h as scalar n). A lane recomputes
// the signed-digit carry into its group from the lower windows, stages its group's digits in LDS and adds their
// entries in one-lane mixed additions; the lane sums meet per quad by DPP broadcasts (no LDS), then in a 6-level
// LDS quad tree, one point per workgroup into part[b S + h]. G > 1 gives few rows (a SPARK derefs commit: 128 x 256)
// more lanes, so each lane's chain of dependent additions is W / G long; with G = 1 and S = 2 the 1024-row block
// witness fills the chip with 2048 workgroups (~8 per CU: LDS is the tree's 8 KB plus <= 11 KB of digits)
template <int C, int G>
__global__ void __launch_bounds__(256) k_comb_accum(const Fq* __restrict__ scalars, const Fq* __restrict__ blinds,
                                                    int n, int gen_offset, const Niels* __restrict__ comb, int NS,
                                                    int S, Ext* __restrict__ part, int st, Fq mulc) {
  constexpr int W = 253 / C + 1, NB = 1 << (C - 1), WG = (W + G - 1) / G, SPW = 256 / G;
  constexpr uint32_t MASK = (1u << C) - 1u;
  __shared__ int16_t dg[WG * 256];  // this lane's digits of its group (lane-major: a lane reads its own)
  __shared__ uint32_t pts[soa_words<Ext, 64>()];
  const int b = blockIdx.x / S, h = blockIdx.x % S, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int wave = t >> 6, j = wave % G, w0 = j * WG, nx = W - w0 < WG ? W - w0 : WG;
  const int per = n + (blinds ? 1 : 0);
  const size_t wstride = (size_t)NS * NB;
  Ext P = ext_identity();
  for (int i = h * SPW + (wave / G) * 64 + (t & 63); i < per; i += SPW * S) {
    Fq sm;
    int s;
    if (i < n) {
      sm = scalars[(size_t)b * n + i];
      s = gen_offset + i;
    } else {
      sm = blinds[b];
      s = NS - 1;
    }
    const Fq k = fq_mul(sm, mulc);  // out of Montgomery form (mulc = 1), halved on the way (mulc = (l + 1) / 2)
    int carry = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      if (w >= w0 + WG) break;  // uniform per wave
      const int bit = w * C;
      const int li = bit >> 5, of = bit & 31;
      uint32_t v = k.l[li] >> of;
      if (of + C > 32 && li + 1 < 8) v |= k.l[li + 1] << (32 - of);
      int d = (int)(v & MASK) + carry;
      carry = d > NB ? 1 : 0;
      d -= carry << C;
      if (w >= w0) dg[(w - w0) * 256 + t] = (int16_t)d;
    }
    const size_t e0 = (size_t)s * NB + (size_t)w0 * wstride;  // entry index of window w0, multiple 1
    const Fp* cf = reinterpret_cast<const Fp*>(comb);
#pragma unroll 1
    for (int x = 0; x < nx; x++) {
      const int d = dg[x * 256 + t];
      if (d) {
        const Fp* c = cf + (e0 + (size_t)x * wstride + (d < 0 ? -d : d) - 1) * st;
        Niels ne;
        ne.ypx = c[0];
        ne.ymx = c[1];
        ne.t2d = c[2];
        P = ext_madd(P, ne, d < 0);
      }
    }
  }
  // the quad's four lane sums, broadcast to the quad one after another
  Ext acc;
  acc.X = fp_qbcast<0>(P.X);
  acc.Y = fp_qbcast<0>(P.Y);
  acc.Z = fp_qbcast<0>(P.Z);
  acc.T = fp_qbcast<0>(P.T);
  {
    Ext o;
    o.X = fp_qbcast<1>(P.X), o.Y = fp_qbcast<1>(P.Y), o.Z = fp_qbcast<1>(P.Z), o.T = fp_qbcast<1>(P.T);
    acc = quad_add(acc, o, q);
    o.X = fp_qbcast<2>(P.X), o.Y = fp_qbcast<2>(P.Y), o.Z = fp_qbcast<2>(P.Z), o.T = fp_qbcast<2>(P.T);
    acc = quad_add(acc, o, q);
    o.X = fp_qbcast<3>(P.X), o.Y = fp_qbcast<3>(P.Y), o.Z = fp_qbcast<3>(P.Z), o.T = fp_qbcast<3>(P.T);
    acc = quad_add(acc, o, q);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<64>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<64>(pts, slot, q), q);
    __syncthreads();
  }
  if (t == 0) part[blockIdx.x] = acc;
}

// one quad per row: out[b] = sum of the row's S parts
__global__ void __launch_bounds__(256) k_comb_join(const Ext* __restrict__ part, int B, int S, Ext* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x, q = t & 3, b = t >> 2;
  if (b >= B) return;  // whole quads exit together (B quads, 4 lanes each)
  Ext acc = part[(size_t)b * S];
  for (int h = 1; h < S; h++) acc = quad_add(acc, part[(size_t)b * S + h], q);
  if (q == 0) out[b] = acc;
}

// comb tables of all live generator sets of this process, against the process-wide cap (SPG_COMB_GB, default 96 GiB;
// a table replaced by a wider one stays allocated until spg_gens_free, see spg_gens::comb_retired)
static std::atomic<size_t> g_comb_bytes{0};
// tables built by this process and their summed build time (spg_comb_stats: the precomputation the bench discloses)
static std::atomic<int> g_comb_built{0};
static std::atomic<uint64_t> g_comb_build_ns{0};

void comb_free(const spg_gens* g) {
  if (!g) return;
  std::lock_guard<std::mutex> lk(g->comb_mu);
  g->comb_retired.push_back(g->comb);
  for (auto& c : g->comb_retired) {
    if (!c.p) continue;
    hipFree(c.p);
    g_comb_bytes -= c.bytes;
  }
  g->comb_retired.clear();
  g->comb = spg_gens::Comb();
}

static bool comb_enabled() {
  static const bool on = !getenv("SPG_COMB") || atoi(getenv("SPG_COMB")) != 0;
  return on;
}

// returns 0 with *use = a table covering generators [0, need) and h = hgen (hgen < 0: no blinds, any h slot); 1 when
// the comb path does not apply here (disabled, too wide, over the memory cap, allocation refused, or a table for
// another h exists: blinded rows on a second h take the bucket path rather than rebuilding gigabytes), or an SPG
// error code. *use stays valid until the gens is freed.
static int comb_ensure(spg_ctx* ctx, const spg_gens* g, size_t need, int hgen, spg_gens::Comb* use) {
  if (!comb_enabled() || ctx->comb_off || need > kCombMaxR) return 1;
  std::lock_guard<std::mutex> lk(g->comb_mu);
  const spg_gens::Comb cur = g->comb;
  if (cur.p && hgen >= 0 && cur.h != hgen) return 1;
  if (cur.p && cur.slots >= need) {
    *use = cur;
    return 0;
  }
  if (hgen < 0) hgen = cur.p ? cur.h : (int)g->n;
  // a rebuild only ever grows (never below the table it replaces)
  size_t cn = std::max<size_t>(256, cur.slots);
  while (cn < need) cn *= 2;
  cn = std::min(cn, g->n);
  if (cn < need || hgen < 0 || (size_t)hgen > g->n) return 1;
  const int NS = (int)cn + 1;
  // the cap is per process (SPG_COMB_GB, default 144 GiB); without an explicit setting a table is also built only when
  // the device keeps kCombHeadroom free beside it, so co-located provers (several processes on one GPU) cannot starve
  // each other's workspaces into SPG_E_NOMEM: a table that does not fit at the preferred width tries 12,
  // and one that does not fit at all leaves the rows on the buckets
  static const bool cap_set = getenv("SPG_COMB_GB") != nullptr;
  static const size_t cap = (size_t)(cap_set ? atof(getenv("SPG_COMB_GB")) : 144.0) * (1ull << 30);
  // entries padded to one 128-byte line each (SPG_COMB_PAD, default on) where the padded table fits: a 96-byte entry
  // gathered at random straddles two lines two times in three (~2x the algorithmic bytes, PMC-measured)
  // Padded tables up to SPG_COMB_PAD_GB (default 64: the 1024-generator tables, 5.9 GB, and config 2's 2^16-generator
  // one, 62 GB); larger ones stay packed -- the config-5 derefs tables run at the madd peak already, and a 93 GB padded
  // 12-bit fallback beside another process's table left two ranks sharing one GPU without room for their workspaces
  static const bool pad_on = !getenv("SPG_COMB_PAD") || atoi(getenv("SPG_COMB_PAD")) != 0;
  static const size_t pad_max = (size_t)(getenv("SPG_COMB_PAD_GB") ? atof(getenv("SPG_COMB_PAD_GB")) : 64.0) * (1ull << 30);
  auto table_bytes = [&](int c, int st) { return (size_t)(253 / c + 1) * NS * ((size_t)1 << (c - 1)) * 32 * st; };
  auto fits = [&](size_t bytes) {
    if (g_comb_bytes.load() + bytes > cap) return false;
    if (cap_set) return true;
    static const size_t kCombHeadroom = (size_t)24 << 30;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return bytes + kCombHeadroom <= free_b;
  };
  // the preferred width padded, then packed; then 12-bit windows padded, then packed
  const int C0 = comb_c_for(cn);
  int C = 0, st = 0;
  const int cands[4][2] = {{C0, 4}, {C0, 3}, {12, 4}, {12, 3}};
  for (int i = 0; i < (C0 > 12 ? 4 : 2) && !st; i++)
    if ((cands[i][1] == 3 || (pad_on && table_bytes(cands[i][0], 4) <= pad_max)) && fits(table_bytes(cands[i][0], cands[i][1]))) {
      C = cands[i][0];
      st = cands[i][1];
    }
  if (!st) return 1;
  const size_t entries = (size_t)(253 / C + 1) * NS * ((size_t)1 << (C - 1)), bytes = table_bytes(C, st);
  const auto t_build = std::chrono::steady_clock::now();
  Niels* comb = nullptr;
  Fp* zs = nullptr;
  const size_t lanes = entries / kCombRun;
  // built a window at a time: the Z scratch holds one window's entries (107 MB at 2^14 generators, not 23 GB)
  const size_t chunk = lanes / (size_t)(253 / C + 1);
  if (hipMalloc(&comb, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  if (hipMalloc(&zs, chunk * kCombRun * sizeof(Fp)) != hipSuccess) {
    (void)hipGetLastError();
    hipFree(comb);
    return 1;
  }
  const dim3 gb((unsigned)((chunk + 63) / 64)), tb(64);
  for (size_t l0 = 0; l0 < lanes; l0 += chunk) {
    if (C == 9)
      hipLaunchKernelGGL(k_comb_build<9>, gb, tb, 0, ctx->stream, g->table, (int)(g->n + 1), NS, hgen, comb, zs, lanes, l0, st);
    else if (C == 10)
      hipLaunchKernelGGL(k_comb_build<10>, gb, tb, 0, ctx->stream, g->table, (int)(g->n + 1), NS, hgen, comb, zs, lanes, l0, st);
    else if (C == 11)
      hipLaunchKernelGGL(k_comb_build<11>, gb, tb, 0, ctx->stream, g->table, (int)(g->n + 1), NS, hgen, comb, zs, lanes, l0, st);
    else if (C == 13)
      hipLaunchKernelGGL(k_comb_build<13>, gb, tb, 0, ctx->stream, g->table, (int)(g->n + 1), NS, hgen, comb, zs, lanes, l0, st);
    else
      hipLaunchKernelGGL(k_comb_build<12>, gb, tb, 0, ctx->stream, g->table, (int)(g->n + 1), NS, hgen, comb, zs, lanes, l0, st);
  }
  const hipError_t e = hipGetLastError();
  const hipError_t e2 = hipStreamSynchronize(ctx->stream);
  hipFree(zs);
  if (e != hipSuccess || e2 != hipSuccess) {
    hipFree(comb);
    return set_err(ctx, SPG_E_HIP, "comb table build");
  }
  if (cur.p) g->comb_retired.push_back(cur);
  g->comb = spg_gens::Comb{comb, cn, bytes, hgen, C, st};
  g_comb_bytes += bytes;
  g_comb_built++;
  g_comb_build_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now() - t_build).count();
  *use = g->comb;
  return 0;
}

int comb_get(spg_ctx* ctx, const spg_gens* g, size_t need, spg_gens::Comb* out) {
  return comb_ensure(ctx, g, need, -1, out);
}

}  // namespace spg

extern "C" int spg_set_comb(spg_ctx* ctx, int on) {
  if (!ctx) return SPG_E_ARG;
  ctx->comb_off = !on;
  return SPG_OK;
}

namespace spg {
extern std::atomic<size_t> g_gens_table_bytes;  // msm.hip
}

extern "C" int spg_comb_stats(uint64_t* bytes, int* tables_built, double* build_seconds, uint64_t* gens_table_bytes) {
  if (bytes) *bytes = spg::g_comb_bytes.load();
  if (gens_table_bytes) *gens_table_bytes = spg::g_gens_table_bytes.load();
  if (tables_built) *tables_built = spg::g_comb_built.load();
  if (build_seconds) *build_seconds = (double)spg::g_comb_build_ns.load() * 1e-9;
  return SPG_OK;
}

namespace spg {

// B row MSMs of n contiguous generators from gen_offset (+ blinds on h): SPG_OK with the rows' points in ext
// (B Ext, device) and, when d_out is set, their encodings; kCombSkip when the comb does not apply (the caller
// runs the bucket pipeline); or an SPG error code
// the plain (not Montgomery) multiplier that takes a Montgomery scalar to its canonical value (1) or to half of it
static Fq comb_mulc(bool halve) {
  Fq c = fq_zero();
  if (!halve) {
    c.l[0] = 1;
    return c;
  }
  // (l + 1) / 2
  const uint32_t h[8] = {0x2e7ae9f7u, 0x2c09318du, 0x517bce6bu, 0x0a6f7cefu, 0u, 0u, 0u, 0x08000000u};
  for (int i = 0; i < 8; i++) c.l[i] = h[i];
  return c;
}

int msm_comb(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
             const Fq* d_blinds, uint8_t* d_out, int h_index, Ext* ext, bool halve) {
  if (halve && d_out) return set_err(ctx, SPG_E_ARG, "msm_comb: halved points have no device encoding");
  spg_gens::Comb cb;
  const int rc = comb_ensure(ctx, g, gen_offset + n, h_index, &cb);
  if (rc == 1) return kCombSkip;
  if (rc) return rc;
  const size_t per = n + (d_blinds ? 1 : 0);
  static const size_t want = getenv("SPG_COMB_WGS") ? (size_t)atol(getenv("SPG_COMB_WGS")) : 2048;
  // window groups per scalar: few rows get up to 4 lanes per scalar (>= 2^17 lanes when there are that few)
  static const size_t gmax = getenv("SPG_COMB_GMAX") ? (size_t)atol(getenv("SPG_COMB_GMAX")) : 4;
  static const size_t gmin = getenv("SPG_COMB_GMIN") ? (size_t)atol(getenv("SPG_COMB_GMIN")) : 1;
  size_t G = gmin == 2 || gmin == 4 ? gmin : 1;
  while (G < gmax && G < 4 && B * per * G < ((size_t)1 << 17)) G *= 2;
  const size_t spw = 256 / G;
  const size_t S = std::max<size_t>(1, std::min((want + B - 1) / B, (per + spw - 1) / spw));
  Ext* part = ext;
  if (S > 1) {
    // the commit queue's second stream runs row commits while the main stream's block-witness commit is in flight:
    // ws_get gives each stream its own slot space
    part = (Ext*)ws_get(ctx, 25, B * S * sizeof(Ext) + 64);
    if (!part) return set_err(ctx, SPG_E_NOMEM, "comb parts");
  }
  {
    const int C = cb.c;
    KScope ks(ctx, "msm_comb", 0.0, (double)B * per * (253 / C + 1) * (1.0 - 1.0 / (double)(1 << C)));
    const dim3 ga((unsigned)(B * S)), ta(256);
    const int NS = (int)cb.slots + 1;
#define SPG_COMB_LAUNCH(CC, GG)                                                                                  \
  hipLaunchKernelGGL((k_comb_accum<CC, GG>), ga, ta, 0, ctx->stream, d_scalars, d_blinds, (int)n, (int)gen_offset, \
                     cb.p, NS, (int)S, part, cb.st, comb_mulc(halve))
    const int key = C * 8 + (int)G;
    switch (key) {
      case 9 * 8 + 1: SPG_COMB_LAUNCH(9, 1); break;
      case 9 * 8 + 2: SPG_COMB_LAUNCH(9, 2); break;
      case 9 * 8 + 4: SPG_COMB_LAUNCH(9, 4); break;
      case 10 * 8 + 1: SPG_COMB_LAUNCH(10, 1); break;
      case 10 * 8 + 2: SPG_COMB_LAUNCH(10, 2); break;
      case 10 * 8 + 4: SPG_COMB_LAUNCH(10, 4); break;
      case 11 * 8 + 1: SPG_COMB_LAUNCH(11, 1); break;
      case 11 * 8 + 2: SPG_COMB_LAUNCH(11, 2); break;
      case 11 * 8 + 4: SPG_COMB_LAUNCH(11, 4); break;
      case 12 * 8 + 1: SPG_COMB_LAUNCH(12, 1); break;
      case 12 * 8 + 2: SPG_COMB_LAUNCH(12, 2); break;
      case 13 * 8 + 1: SPG_COMB_LAUNCH(13, 1); break;
      case 13 * 8 + 2: SPG_COMB_LAUNCH(13, 2); break;
      case 13 * 8 + 4: SPG_COMB_LAUNCH(13, 4); break;
      default: SPG_COMB_LAUNCH(12, 4); break;
    }
#undef SPG_COMB_LAUNCH
    if (S > 1)
      hipLaunchKernelGGL(k_comb_join, dim3((unsigned)((4 * B + 255) / 256)), dim3(256), 0, ctx->stream, part, (int)B,
                         (int)S, ext);
  }
  if (d_out) return compress_ext_device(ctx, ext, B, d_out);
  SPG_HIP(ctx, hipGetLastError());
  return SPG_OK;
}

// One large MSM from the comb table: the rows kernel with B = 1 and S workgroups, whose S partial points go to mapped
// host memory and are added on the host pool (k_comb_join would add them on one quad, a chain of S additions)
int msm_single_comb(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n,
                    const Fq* d_blind, h::HExt* out) {
  spg_gens::Comb cb;
  const int rc = comb_ensure(ctx, g, gen_offset + n, d_blind ? (int)g->n : -1, &cb);
  if (rc) return rc;
  const size_t per = n + (d_blind ? 1 : 0);
  // window groups per scalar (a lane's chain is W / G mixed additions) and workgroups: ~4 waves per SIMD
  static const size_t gsel = getenv("SPG_BIG_COMB_G") ? (size_t)atol(getenv("SPG_BIG_COMB_G")) : 2;
  const size_t G = gsel == 1 || gsel == 2 ? gsel : 4, spw = 256 / G;
  const size_t S = std::max<size_t>(1, (per + spw - 1) / spw);
  void* d_map = nullptr;
  Ext* parts = (Ext*)mapped_get(ctx, S * sizeof(Ext), &d_map);
  if (!parts) return 1;
  const int C = cb.c, NS = (int)cb.slots + 1;
  {
    KScope ks(ctx, "msm_comb_single", 0.0, (double)per * (253 / C + 1) * (1.0 - 1.0 / (double)(1 << C)));
    const dim3 ga((unsigned)S), ta(256);
#define SPG_CS(CC, GG)                                                                                          \
  hipLaunchKernelGGL((k_comb_accum<CC, GG>), ga, ta, 0, ctx->stream, d_scalars, d_blind, (int)n, (int)gen_offset, \
                     cb.p, NS, (int)S, (Ext*)d_map, cb.st, comb_mulc(false))
    const int key = C * 8 + (int)G;
    switch (key) {
      case 9 * 8 + 1: SPG_CS(9, 1); break;
      case 9 * 8 + 2: SPG_CS(9, 2); break;
      case 9 * 8 + 4: SPG_CS(9, 4); break;
      case 10 * 8 + 1: SPG_CS(10, 1); break;
      case 10 * 8 + 2: SPG_CS(10, 2); break;
      case 10 * 8 + 4: SPG_CS(10, 4); break;
      case 11 * 8 + 1: SPG_CS(11, 1); break;
      case 11 * 8 + 2: SPG_CS(11, 2); break;
      case 11 * 8 + 4: SPG_CS(11, 4); break;
      case 12 * 8 + 1: SPG_CS(12, 1); break;
      case 12 * 8 + 2: SPG_CS(12, 2); break;
      case 13 * 8 + 1: SPG_CS(13, 1); break;
      case 13 * 8 + 2: SPG_CS(13, 2); break;
      case 13 * 8 + 4: SPG_CS(13, 4); break;
      default: SPG_CS(12, 4); break;
    }
#undef SPG_CS
  }
  SPG_HIP(ctx, hipGetLastError());
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // the S parts over the pool: contiguous chunks (8-lane IFMA sums where the CPU has them), then their sums here
  static const bool vec = h::ifma_on() && !(getenv("SPG_VEC_MIN") && atol(getenv("SPG_VEC_MIN")) == 0);
  const int K = (int)std::max<size_t>(1, std::min<size_t>(S / (vec ? 64 : 16), (size_t)pool().size() + 1));
  std::vector<h::HExt> part(K);
  pool().parallel_for(K, [&](int c) {
    const size_t lo = S * c / K, hi = S * (c + 1) / K;
    for (const uint8_t* q = (const uint8_t*)(parts + lo); q < (const uint8_t*)(parts + hi); q += 64)
      __builtin_prefetch(q, 0, 0);
    if (vec && hi - lo >= 16) {
      std::vector<h::HExt> hx(hi - lo);
      for (size_t i = lo; i < hi; i++) hx[i - lo] = h::hext_from_dev(parts[i]);
      part[c] = h::ext_sum8(hx.data(), hi - lo);
      return;
    }
    h::HExt acc = h::hext_from_dev(parts[lo]);
    for (size_t i = lo + 1; i < hi; i++) acc = h::hext_add(acc, h::hext_from_dev(parts[i]));
    part[c] = acc;
  });
  h::HExt sum = part[0];
  for (int c = 1; c < K; c++) sum = h::hext_add(sum, part[c]);
  *out = sum;
  return 0;
}

}  // namespace spg

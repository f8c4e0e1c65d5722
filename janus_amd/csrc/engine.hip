// Host side of the prio3gpu C ABI (include/prio3gpu.h): contexts, batch states, aggregates,
// kernel launches and the RCCL merge.  One HIP stream per context.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <string>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "../../include/prio3gpu.h"
#include "../../include/prio3gpu_test.h"
#include "errors.h"
#include "prio3_kernels.h"
#include "fpvec_kernels.h"
#include "wires_mfma.h"
#include "fpvec_mfma.h"
#include "fpvec_pair.h"

using namespace p3g;

namespace {
thread_local std::string g_err;
}  // namespace

void p3g::set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

namespace {

#define set_err p3g::set_error

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return PRIO3GPU_E_HIP;                                                      \
    }                                                                             \
  } while (0)

#define RCCLCHK(x)                                                                  \
  do {                                                                              \
    ncclResult_t e_ = (x);                                                          \
    if (e_ != ncclSuccess) {                                                        \
      set_err("%s failed: %s (%s:%d)", #x, ncclGetErrorString(e_), __FILE__, __LINE__); \
      return PRIO3GPU_E_RCCL;                                                       \
    }                                                                               \
  } while (0)

#define CHK(x)                   \
  do {                           \
    int rc_ = (x);               \
    if (rc_ != 0) return rc_;    \
  } while (0)

typedef unsigned __int128 u128;

// ---- host modular arithmetic for table setup only ---------------------------------------------
u128 addmod(u128 x, u128 y, u128 p) {
  u128 s = x + y;
  if (s < x || s >= p) s -= p;
  return s;
}
u128 mulmod(u128 a, u128 b, u128 p) {
  u128 r = 0;
  a %= p;
  while (b) {
    if (b & 1) r = addmod(r, a, p);
    a = addmod(a, a, p);
    b >>= 1;
  }
  return r;
}
u128 powmod(u128 a, u128 e, u128 p) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = mulmod(r, a, p);
    a = mulmod(a, a, p);
    e >>= 1;
  }
  return r;
}
const u128 P128 = ((u128)0xFFFFFFFFFFFFFFE4ull << 64) | 1u;
const u128 P64 = (u128)0xFFFFFFFF00000001ull;

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

uint32_t next_pow2(uint32_t x) {
  uint32_t r = 1;
  while (r < x) r <<= 1;
  return r;
}
uint32_t ilog2(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) ++l;
  return l;
}

// Grow-only device buffer; owns its allocation (freed on destruction, never copied).  Every
// per-state buffer is sized by prio3gpu_state_create, so a call on a state never grows one (a
// hipFree inside a call would wait for the whole device); the context-level scratch grows to the
// largest batch it has seen.  An allocation the device cannot hold is PRIO3GPU_E_CAPACITY, with
// the HIP error cleared so the next launch check of the same context does not report it.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    cap = 0;
    const size_t want = bytes ? bytes : 16;
    const hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      size_t fr = 0, tot = 0;
      (void)hipMemGetInfo(&fr, &tot);
      set_err("device allocation of %zu bytes failed: %s (%zu of %zu bytes free)", want,
              hipGetErrorString(e), fr, tot);
      return e == hipErrorOutOfMemory ? PRIO3GPU_E_CAPACITY : PRIO3GPU_E_HIP;
    }
    cap = bytes;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

// One id per kernel, named exactly as rocprofv3 reports it (kernel-trace names are the
// template-stripped function names), so the bench's HIP-event table and the profiles agree.
enum KernelId {
  KID_QUERY = 0, KID_EXPAND, KID_HELPER_XOF, KID_JR, KID_FLP_WEIGHTS, KID_FLP_WIRES,
  KID_FPV_WEIGHTS, KID_FPV_WIRES0, KID_FPV_WIRES1, KID_FPV_FINAL, KID_DECIDE, KID_FPV_DECIDE,
  KID_PNEXT, KID_ACC_PART, KID_ACC_SPEC, KID_ACC_MERGE, KID_OUT, KID_MERGE, KID_SHARD_SEEDS,
  KID_SHARD_MEAS, KID_SHARD_JR, KID_PROVE, KID_SHARD_PROOF, KID_REPORT_META, KID_REPORT_META_FOLD,
  KID_SHARD_NORM, KID_JR_RING, KID_FLP_QUERY_LANE, KID_FLP_WIRES_COLS, KID_FLP_WIRES_MFMA,
  KID_FPV_REGEN, KID_COUNT
};
const char* const kKernelNames[KID_COUNT] = {
    "k_query_rand", "k_expand", "k_helper_xof", "k_jr", "k_flp_weights", "k_flp_wires",
    "k_fpv_weights", "k_fpv_wires0", "k_fpv_wires1", "k_fpv_finalize", "k_decide", "k_fpv_decide",
    "k_prepare_next", "k_accum_partial", "k_accum_spec", "k_accum_merge", "k_out_shares", "k_merge",
    "k_shard_seeds", "k_shard_meas", "k_shard_jr", "k_flp_prove", "k_shard_proof", "k_report_meta",
    "k_report_meta_fold", "k_shard_norm", "k_jr_ring", "k_flp_query_lane", "k_flp_wires_cols",
    "k_flp_wires_mfma", "k_fpv_regen"};

// Per-kernel HIP-event timing on the context's stream (opt-in; used by bench.py).
struct Prof {
  bool on = false;
  struct Rec {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
};

}  // namespace

struct prio3gpu_ctx {
  Cfg cfg{};
  prio3gpu_sizes sz{};
  uint8_t vk[16];
  int device = 0;
  hipStream_t stream = nullptr;
  // snapshot-mode helper query: k_fpv_regen of the next half-chunk runs on `aux` beside the
  // current half-chunk's query on `stream` (created on first use); aux_ev[0..1] regenerated,
  // aux_ev[2..3] read, per scratch half
  hipStream_t aux = nullptr;
  hipEvent_t aux_ev[4] = {};
  DevBuf twiddles, twiddles1, twiddles2;
  // generic staging (inputs given as host pointers) and scratch
  DevBuf io[6];
  DevBuf perm, chunks, partials, pcounts, spec_idx;
  std::vector<uint32_t> h_perm, h_chunk_begin, h_chunk_slot;
  // Engine options (prio3gpu_ctx_set_option; include/prio3gpu.h lists them).  The defaults are the
  // measured-fastest paths; every alternative is parity-tested against the oracle.
  bool speculate = true;     // "speculate": accumulation from k_jr's column sums (0: direct)
  bool fused_helper = true;  // "fused_helper": FixedPoint helper via k_helper_xof (0: two-pass)
  // "helper_snap": FixedPoint helper states keep sponge snapshots instead of the expanded share
  // (k_fpv_regen rewrites it per chunk); read when a state is created
  bool helper_snap = true;
  uint32_t snap_chunk = 512;  // "snap_chunk": reports per FixedPoint query / regeneration chunk
  bool spread = true;        // "spread": one CU per workgroup for latency-bound sponge launches
  // "spread_lds": the dynamic LDS such a workgroup requests (96 KB: one per CU; <= 80 KB lets a
  // leader and a helper workgroup share a CU when both aggregators run on one GPU)
  size_t spread_lds = 96 * 1024;
  bool jr_ring = true;       // "jr_ring": FixedPoint leader joint-rand part via k_jr_ring
  // "chain_pairs": 64-report chains per k_helper_xof / k_jr_ring workgroup (0: auto -- 1 while the
  // launch takes at most half the CUs, else 2, so a leader and a helper launch side by side
  // still give every sponge wave its own SIMD)
  uint32_t chain_pairs = 0;
  // "pair_chains": the FixedPoint chains with each sponge state on a lane pair (fpvec_pair.h:
  // k_helper_xof_pair, k_jr_ring_pair; half the instructions on the latency-bound chain)
  bool pair_chains = true;
  // "query_overlap": snapshot-mode helper query regenerates half-chunk i+1 on a second stream
  // while half-chunk i is queried (two scratch halves; the default since the lane-pair chains:
  // config E 1,232 -> 1,200 ms per step at 10,240 reports, profiles/r05/pair/r5_pair8, r5_pair9;
  // with the one-lane chains it measured 1,773 vs 1,765 ms, the regeneration starving the wires)
  bool query_overlap = true;
  bool wires_mfma = true;    // "wires_mfma": SumVec chunk > 64 wire pass on the matrix cores
  bool wires_cols = true;    // "wires_cols": chunk <= 64 lane-per-column wire pass
  size_t expand_lds = 0;     // "expand_lds": dynamic LDS per k_expand block (occupancy cap)
  size_t jr_lds = 0;         // "jr_lds": dynamic LDS per k_jr block (occupancy cap)
  uint32_t cus = 0;          // compute units of the device
  DevBuf fallback;           // k_helper_xof's non-canonical-element counter
  Prof prof;
  // async mode (prio3gpu_ctx_set_async): calls whose buffers are all device memory return once
  // their work is queued; cross-context order via prio3gpu_ctx_wait
  bool async_mode = false;
  static constexpr int kMarks = 16;
  hipEvent_t ev[kMarks] = {};  // ring of marks (prio3gpu_ctx_mark)
  uint32_t ev_gen[kMarks] = {};  // generation of each ring slot: a mark = gen * kMarks + slot
  int ev_next = 0;
  uint32_t gen_next = 1;
  hipEvent_t wait_ev = nullptr;  // prio3gpu_ctx_wait: recorded on the other context, not a mark
  int wait_ev_dev = -1;          // device wait_ev was created on (the other context's)
  std::mutex mark_mu;            // ev_next / ev_gen / wait_ev
  // the device-side accumulation plan of the last call (single slot, no per-report slots):
  // reused while (n, speculative layout, slot count) are unchanged -- no host planning, no upload
  bool plan_valid = false;
  size_t plan_n = 0;
  uint32_t plan_slots = 0, plan_nd = 0, plan_e0 = 0, plan_e1 = 0;
  bool plan_spec = false;
  uint32_t plan_ndir = 0, plan_nspec = 0, plan_nch = 0, plan_tiles = 0, plan_epb = 0;
};

namespace {
struct ProfScope {
  prio3gpu_ctx* c;
  int kid;
  hipEvent_t a{}, b{};
  hipStream_t s;
  ProfScope(prio3gpu_ctx* c_, int kid_, hipStream_t s_ = nullptr)
      : c(c_), kid(kid_), s(s_ ? s_ : c_->stream) {
    if (c->prof.on) {
      a = c->prof.get();
      b = c->prof.get();
      (void)hipEventRecord(a, s);
    }
  }
  ~ProfScope() {
    if (c->prof.on) {
      (void)hipEventRecord(b, s);
      c->prof.recs.push_back({kid, a, b});
    }
  }
};
}  // namespace
#define PROF(kid) ProfScope prof_scope_##kid(c, kid)
#define PROF_ON(kid, strm) ProfScope prof_scope_##kid(c, kid, strm)

struct prio3gpu_state {
  prio3gpu_ctx* ctx = nullptr;
  int agg_id = 0;
  size_t cap = 0;
  size_t n = 0;
  size_t in_pitch = 0;  // row pitch of the caller's input shares (0: packed, the share length)
  DevBuf t, jr, part, seed, meas, proof, prep, msg, status, nonces, pub, input, w;
  DevBuf fpart, flags;  // FixedPointBoundedL2VecSum: wire partials per row group, query flags
  size_t fpart_rows = 0;  // reports fpart holds (the query runs in chunks of at most this many)
  // FixedPoint helper, snapshot mode (helper_snap): k_helper_xof's sponge snapshots of every
  // report; `scratch` holds one chunk of regenerated measurement-share rows.  snap_active: the
  // prepared batch's share exists only as snapshots (the fused path ran), so every reader of
  // meas_rows goes through regen_rows.
  DevBuf snaps, scratch;
  bool snap = false, snap_active = false;
  bool snap_pair = false;  // the snapshots were written by k_helper_xof_pair (dword-pair halves)
  CRows meas_rows{nullptr, 0};  // measurement shares of the prepared batch
  CRows proof_rows{nullptr, 0};  // proof shares (prepare_init_xof -> prepare_init_query)
  bool xof_done = false;         // the XOF phase ran; the query phase is due
  bool weights_done = false;     // ParallelSum: k_flp_weights of the query phase ran already
  bool query_done = false;       // Count: the XOF phase ran the whole query (fused query rand)
  // speculative accumulation: per-wave column sums of meas-share words, written by k_jr
  DevBuf spec_lo, spec_cy;
  bool spec_ok = false;
  size_t spec_n = 0;
  uint32_t spec_nd = 0, spec_e0 = 0, spec_e1 = 0;
};

struct prio3gpu_agg {
  prio3gpu_ctx* ctx = nullptr;
  uint32_t slots = 0;
  DevBuf share;   // slots x out_len x ES
  DevBuf counts;  // slots x u64
  DevBuf meta;    // slots x SlotMeta: report-ID checksum + client timestamp interval
  DevBuf wmeta;   // per-wave partials of k_report_meta
};

struct prio3gpu_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  // all-gather scratch, shared by every context that flushes through this communicator
  DevBuf gather, cgather, mgather;
  // Flushes through one communicator are serialised: the host issues one at a time (mu), and each
  // flush's collectives wait on `done`, recorded after the previous flush's k_merge_ranks, so an
  // async context's collectives never overwrite scratch another context's merge still reads.
  std::mutex mu;
  hipEvent_t done = nullptr;
  bool done_valid = false;
};

namespace {

// prio `optimal_chunk_length` (src/vdaf/prio3.rs, ext): among gadget_calls = 2^k - 1,
// k = round(log2(len + 1)) .. 1, the chunk length minimising the ParallelSum(Mul) proof length
// 2 chunk + 2 ((1 + calls).next_power_of_two() - 1) + 1; the first minimum (largest k) wins.
uint32_t optimal_chunk_length(uint32_t len) {
  if (len <= 1) return 1;
  const int max_log2 = (int)std::lround(std::log2((double)len + 1.0));
  uint64_t best_cost = ~0ull;
  uint32_t best = 1;
  for (int k = max_log2; k >= 1; --k) {
    const uint64_t calls = (1ull << k) - 1;
    const uint64_t chunk = (len + calls - 1) / calls;
    const uint64_t cost = 2 * chunk + 2 * (next_pow2((uint32_t)(1 + calls)) - 1) + 1;
    if (cost < best_cost) {
      best_cost = cost;
      best = (uint32_t)chunk;
    }
  }
  return best;
}

// FLP tables of one gadget (Montgomery form), 3m + 1 entries:
//   [0, m)        alpha_m^k
//   m             1/m
//   [m+1, 2m+1)   S_i = sum_{k=1..calls} alpha_m^(ik)   (gadget-output sum as a dot product)
//   [2m+1, 3m+1)  alpha_m^k / m                          (Lagrange weight scale)
int upload_tables(DevBuf& buf, uint32_t m, uint32_t calls, uint32_t es) {
  const u128 p = (es == 16) ? P128 : P64;
  const u128 R = (es == 16) ? (u128)0 - P128 /* 2^128 mod p */ : ((u128)1 << 64) % P64;
  const u128 alpha = powmod(7, (p - 1) / m, p);
  const u128 inv_m = p - (p - 1) / m;
  std::vector<u128> tv(3 * (size_t)m + 1);
  u128 a = 1;
  for (uint32_t k = 0; k < m; ++k) {
    tv[k] = a;
    tv[2 * m + 1 + k] = mulmod(a, inv_m, p);
    a = mulmod(a, alpha, p);
  }
  tv[m] = inv_m;
  for (uint32_t i = 0; i < m; ++i) {
    const u128 x = tv[i];  // alpha^i
    u128 y = x, acc = 0;
    for (uint32_t k = 1; k <= calls; ++k) {
      acc = addmod(acc, y, p);
      y = mulmod(y, x, p);
    }
    tv[m + 1 + i] = acc;
  }
  std::vector<uint8_t> tw(tv.size() * es);
  for (size_t k = 0; k < tv.size(); ++k) {
    const u128 mv = mulmod(tv[k], R, p);
    for (uint32_t b = 0; b < es; ++b) tw[k * es + b] = (uint8_t)(mv >> (8 * b));
  }
  CHK(buf.ensure(tw.size()));
  HIPCHK(hipMemcpy(buf.p, tw.data(), tw.size(), hipMemcpyHostToDevice));
  return 0;
}

int setup_cfg(prio3gpu_ctx* c, int kind, uint32_t bits, uint32_t length, uint32_t chunk) {
  Cfg& g = c->cfg;
  g.kind = (uint32_t)kind;
  g.wave_prio = 1u;
  // VDAF-07 algorithm IDs: Count 0, Sum 1, SumVec 2, Histogram 3; FixedPoint L2 0xFFFF0000
  g.algo_id = kind == PRIO3GPU_FPVEC ? 0xFFFF0000u : (uint32_t)kind;
  g.qr_len = kind == PRIO3GPU_FPVEC ? 2u : 1u;
  uint32_t calls = 0, arity = 0, prove_rand = 0;
  switch (kind) {
    case PRIO3GPU_COUNT:
      g.es = 8;
      g.meas_len = 1;
      g.out_len = 1;
      g.jr_len = 0;
      calls = 1;
      arity = 2;
      prove_rand = 2;
      break;
    case PRIO3GPU_SUM:
      if (bits == 0 || bits > 64) {
        set_err("Prio3Sum: bits must be in 1..64");
        return PRIO3GPU_E_ARG;
      }
      g.es = 16;
      g.meas_len = bits;
      g.out_len = 1;
      g.jr_len = 1;
      calls = bits;
      arity = 1;
      prove_rand = 1;
      break;
    case PRIO3GPU_SUMVEC:
      if (bits == 0 || bits > 64 || length == 0 || chunk == 0) {
        set_err("Prio3SumVec: bad parameters");
        return PRIO3GPU_E_ARG;
      }
      g.es = 16;
      g.meas_len = bits * length;
      g.out_len = length;
      g.jr_len = 1;
      calls = (g.meas_len + chunk - 1) / chunk;
      arity = 2 * chunk;
      prove_rand = 2 * chunk;
      break;
    case PRIO3GPU_HISTOGRAM:
      if (length == 0 || chunk == 0) {
        set_err("Prio3Histogram: bad parameters");
        return PRIO3GPU_E_ARG;
      }
      g.es = 16;
      g.meas_len = length;
      g.out_len = length;
      g.jr_len = 2;
      calls = (length + chunk - 1) / chunk;
      arity = 2 * chunk;
      prove_rand = 2 * chunk;
      break;
    case PRIO3GPU_FPVEC:
      if ((bits != 16 && bits != 32 && bits != 64) || length == 0) {
        set_err("Prio3FixedPointBoundedL2VecSum: bits must be 16, 32 or 64 and length >= 1");
        return PRIO3GPU_E_ARG;
      }
      g.es = 16;
      g.meas_len = bits * length + 2 * bits - 2;  // entry bits || norm bits
      g.out_len = length;
      g.jr_len = 2;
      chunk = optimal_chunk_length(g.meas_len);
      calls = (g.meas_len + chunk - 1) / chunk;
      arity = 2 * chunk;
      g.chunk1 = optimal_chunk_length(length);
      g.calls1 = (length + g.chunk1 - 1) / g.chunk1;
      prove_rand = 2 * chunk + g.chunk1;
      break;
    default:
      set_err("unknown kind %d", kind);
      return PRIO3GPU_E_ARG;
  }
  g.bits = bits;
  g.length = length;
  g.chunk =
      (kind == PRIO3GPU_SUMVEC || kind == PRIO3GPU_HISTOGRAM || kind == PRIO3GPU_FPVEC) ? chunk : 0;
  g.calls = calls;
  g.arity = arity;
  g.prove_rand_len = prove_rand;
  g.m = next_pow2(1 + calls);
  g.logm = ilog2(g.m);
  if (g.m > 4096) {
    set_err("gadget too large (m = %u)", g.m);
    return PRIO3GPU_E_ARG;
  }
  g.gp_len = 2 * (g.m - 1) + 1;  // every gadget here has degree 2
  g.proof_len = arity + g.gp_len;
  g.verifier_len = 1 + arity + 1;
  if (kind == PRIO3GPU_FPVEC) {
    g.m1 = next_pow2(1 + g.calls1);
    g.logm1 = ilog2(g.m1);
    g.gp_len1 = 2 * (g.m1 - 1) + 1;
    g.proof_len += g.chunk1 + g.gp_len1;
    g.verifier_len += g.chunk1 + 1;
    // k_fpv_weights keeps three m-entry tables and an r-power table in LDS
    if (g.m > 2048 || g.chunk + 1 > 4096 ||
        (size_t)16 * (3 * (size_t)g.m + g.chunk + 1 + 12) + 16 > 160 * 1024) {
      set_err("FixedPointBoundedL2VecSum: length %u too large (m = %u, chunk = %u)", length, g.m,
              g.chunk);
      return PRIO3GPU_E_ARG;
    }
  }
  const uint32_t es = g.es;
  g.leader_share_len = es * (g.meas_len + g.proof_len) + (g.jr_len ? 16 : 0);
  g.helper_share_len = g.jr_len ? 48 : 32;
  g.public_share_len = g.jr_len ? 32 : 0;
  g.prep_share_len = es * g.verifier_len + (g.jr_len ? 16 : 0);
  g.prep_msg_len = g.jr_len ? 16 : 0;

  prio3gpu_sizes& s = c->sz;
  s.field_size = es;
  s.meas_len = g.meas_len;
  s.proof_len = g.proof_len;
  s.verifier_len = g.verifier_len;
  s.joint_rand_len = g.jr_len;
  s.output_len = g.out_len;
  s.leader_input_share = g.leader_share_len;
  s.helper_input_share = g.helper_share_len;
  s.public_share = g.public_share_len;
  s.prep_share = g.prep_share_len;
  s.prep_msg = g.prep_msg_len;
  s.aggregate_share = g.out_len * es;

  CHK(upload_tables(c->twiddles, g.m, g.calls, es));
  g.twiddles = c->twiddles.u8();
  g.twiddles1 = nullptr;
  if (kind == PRIO3GPU_FPVEC) {
    CHK(upload_tables(c->twiddles1, g.m1, g.calls1, es));
    g.twiddles1 = c->twiddles1.u8();
  }
  // prover table: w^k (k < 2m, w = primitive 2m-th root), 1/m, 1/(2m); Montgomery
  {
    const u128 p = (es == 16) ? P128 : P64;
    const u128 R = (es == 16) ? (u128)0 - P128 /* 2^128 mod p */ : ((u128)1 << 64) % P64;
    const uint32_t m2 = 2 * g.m;
    const u128 w = powmod(7, (p - 1) / m2, p);
    std::vector<uint8_t> t2((size_t)(m2 + 2) * es);
    u128 x = 1;
    for (uint32_t k = 0; k < m2 + 2; ++k) {
      u128 v = k < m2 ? x : (k == m2 ? p - (p - 1) / g.m : p - (p - 1) / m2);
      u128 mv = mulmod(v, R, p);
      for (uint32_t b = 0; b < es; ++b) t2[(size_t)k * es + b] = (uint8_t)(mv >> (8 * b));
      x = mulmod(x, w, p);
    }
    CHK(c->twiddles2.ensure(t2.size()));
    HIPCHK(hipMemcpy(c->twiddles2.p, t2.data(), t2.size(), hipMemcpyHostToDevice));
  }
  return 0;
}

// Make `src` (host or device, `bytes`) available on device; returns the device pointer.
int stage_in(prio3gpu_ctx* c, DevBuf& buf, const void* src, size_t bytes, const uint8_t** out) {
  if (!src || bytes == 0) {
    *out = static_cast<const uint8_t*>(src);
    return 0;
  }
  if (is_device_ptr(src)) {
    *out = static_cast<const uint8_t*>(src);
    return 0;
  }
  CHK(buf.ensure(bytes));
  HIPCHK(hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, c->stream));
  *out = buf.u8();
  return 0;
}

int copy_out(prio3gpu_ctx* c, void* dst, const void* dev_src, size_t bytes) {
  if (!dst || bytes == 0 || dst == dev_src) return 0;
  HIPCHK(hipMemcpyAsync(dst, dev_src, bytes, hipMemcpyDefault, c->stream));
  return 0;
}

dim3 grid1(size_t n, uint32_t tpb) { return dim3((unsigned)((n + tpb - 1) / tpb)); }

// Spreading: a workgroup requests c->spread_lds of dynamic LDS, so no second one fits its CU.
bool spread_ok(const prio3gpu_ctx* c, uint32_t blocks) { return c->spread && blocks <= c->cus; }

// 64-report chains per FixedPoint chain workgroup (option chain_pairs).
uint32_t chain_pairs(const prio3gpu_ctx* c, size_t n) {
  if (c->chain_pairs) return c->chain_pairs;
  return (n + 63) / 64 > std::max<uint32_t>(1u, c->cus / 2) ? 2u : 1u;
}

// Measurement-share words that k_jr absorbs through its LDS window ("fast" blocks 1..lf cover
// words [16, 21 (lf+1) - 5)); elements [e0, e1) lie entirely inside.  Field128 types with JR only.
bool spec_range(const Cfg& g, uint32_t& nd, uint32_t& e0, uint32_t& e1) {
  if (g.es != 16 || g.jr_len == 0) return false;
  const int64_t nbytes = (int64_t)g.meas_len * 16;
  const int64_t ndw = nbytes / 8, padw = (42 + nbytes) >> 3;
  auto is_fast = [&](int64_t b) { return b >= 1 && 21 * b + 15 < ndw && 21 * b + 20 < padw; };
  int64_t lf = 0;
  while (is_fast(lf + 1)) ++lf;
  if (lf < 1) return false;
  const int64_t f1 = (21 * (lf + 1) - 5) & ~(int64_t)1;
  nd = (uint32_t)ndw;
  e0 = 8;
  e1 = (uint32_t)(f1 / 2);
  return e1 > e0;
}

// Snapshot mode: the helper's expanded measurement shares of reports [r0, r0 + nr) rewritten
// from k_helper_xof's sponge snapshots into rows 0..nr-1 of `dst` (default st->scratch, which is
// then sized for them), on `strm` (default the context's stream) (k_fpv_regen).
int regen_rows(prio3gpu_ctx* c, prio3gpu_state* st, size_t r0, size_t nr, uint8_t* dst = nullptr,
               hipStream_t strm = nullptr) {
  const Cfg& g = c->cfg;
  const size_t row = (size_t)g.meas_len * g.es;
  if (!dst) {
    CHK(st->scratch.ensure(nr * row));
    dst = st->scratch.u8();
  }
  if (!strm) strm = c->stream;
  const uint64_t lanes = (uint64_t)nr * snap_count(g);
  PROF_ON(KID_FPV_REGEN, strm);
  hipLaunchKernelGGL(st->snap_pair ? k_fpv_regen<true> : k_fpv_regen<false>,
                     dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, strm, g,
                     (uint32_t)nr, (uint32_t)r0, reinterpret_cast<const uint64_t*>(st->snaps.p),
                     Rows{dst, row});
  HIPCHK(hipGetLastError());
  return 0;
}

// The context's auxiliary stream and its four events (created on first use).
int ensure_aux(prio3gpu_ctx* c) {
  if (!c->aux) HIPCHK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
  for (auto& e : c->aux_ev)
    if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return 0;
}

// Reports per FixedPoint query / regeneration chunk.
size_t fpv_chunk(const prio3gpu_ctx* c, const prio3gpu_state* st, size_t n) {
  return std::max<size_t>(1, std::min<size_t>({n, (size_t)c->snap_chunk, st->fpart_rows}));
}

// FixedPointBoundedL2VecSum FLP query (fpvec_kernels.h), first part: the report flags and
// k_fpv_weights (Lagrange weights, p(t), gadget-output sums: the proof share and the randomness
// only, no measurement row) for the whole batch, so the chunked wire passes do not wait for it.
int launch_fpv_weights(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, CRows proof,
                       uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const FpvW W = fpv_w_layout(g);
  Rows wrows{st->w.u8(), (size_t)W.len * 16};
  Rows prep{st->prep.u8(), g.prep_share_len};
  uint32_t* flags = reinterpret_cast<uint32_t*>(st->flags.p);
  HIPCHK(hipMemsetAsync(flags, 0, n * 4, c->stream));
  const size_t lds = (size_t)16 * (3 * (size_t)g.m + g.chunk + 1 + 12) + 16;
  PROF(KID_FPV_WEIGHTS);
  hipLaunchKernelGGL(k_fpv_weights, dim3((uint32_t)n, 2), dim3(256), lds, c->stream, g,
                     (uint32_t)n, proof, CRows{st->t.u8(), 32}, CRows{st->jr.u8(), 32}, prep,
                     d_status, wrows, flags);
  HIPCHK(hipGetLastError());
  return 0;
}

// Second part: wire passes and finalize over reports [r0, r0 + n) (rows 0..n-1 of `meas`; the
// state's per-report arrays at r0; d_status at r0).
int launch_fpv_query_rows(prio3gpu_ctx* c, prio3gpu_state* st, size_t r0, size_t n, CRows meas,
                          uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const uint32_t N = (uint32_t)n;
  const uint32_t H = fpv_rows(g);
  const FpvW W = fpv_w_layout(g);
  Rows wrows{st->w.u8() + r0 * (size_t)W.len * 16, (size_t)W.len * 16};
  Rows prep{st->prep.u8() + r0 * g.prep_share_len, g.prep_share_len};
  uint32_t* flags = reinterpret_cast<uint32_t*>(st->flags.p) + r0;
  const CRows jr{st->jr.u8() + r0 * 32, 32};
  const CRows part{st->part.u8() + r0 * 16, 16};
  // matrix-core wire passes (fpvec_mfma.h) unless the option is off or the digit windows of a
  // call range would not fit 64 KB of LDS; gadget 1 on them for 16- and 32-bit entries
  const bool m0 = c->wires_mfma && fpv_w0m_lds(g) <= 64 * 1024 && H >= kFpvMfmaH;
  const bool m1 = c->wires_mfma && fpv_w1m_bits_ok(g.bits) && fpv_w1m_lds(g) <= 64 * 1024;
  const uint32_t H0 = m0 ? kFpvMfmaH : H;  // partial row groups k_fpv_finalize folds
  {
    PROF(KID_FPV_WIRES0);
    if (m0)
      hipLaunchKernelGGL(k_fpv_wires0_mfma, dim3(kFpvMfmaH, N), dim3(256), fpv_w0m_lds(g),
                         c->stream, g, N, meas, CRows{wrows.base, wrows.stride}, d_status,
                         st->fpart.u8(), flags);
    else
      hipLaunchKernelGGL(k_fpv_wires0, dim3((g.chunk + 255) / 256, H, N), dim3(256), 0, c->stream,
                         g, N, H, meas, CRows{wrows.base, wrows.stride}, d_status, st->fpart.u8(),
                         flags);
  }
  {
    PROF(KID_FPV_WIRES1);
    if (m1)
      // tile groups per report: enough blocks to fill the chip at small chunks
      hipLaunchKernelGGL(k_fpv_wires1_mfma,
                         dim3(N, std::max<uint32_t>(1u, std::min<uint32_t>(
                                     4u, (g.bits * g.chunk1 + 127u) / 128u))),
                         dim3(256), fpv_w1m_lds(g), c->stream, g, N, meas,
                         CRows{wrows.base, wrows.stride}, prep, d_status);
    else
      hipLaunchKernelGGL(k_fpv_wires1, dim3((g.chunk1 + 255) / 256, N), dim3(256), 0, c->stream, g,
                         N, meas, CRows{wrows.base, wrows.stride}, prep, d_status);
  }
  {
    PROF(KID_FPV_FINAL);
    hipLaunchKernelGGL(k_fpv_finalize, dim3((g.chunk + 255) / 256, N), dim3(256), 0, c->stream, g,
                       N, H0, meas, CRows{wrows.base, wrows.stride}, jr, part, st->fpart.u8(), prep,
                       d_status, flags);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// The query over the whole batch in chunks of fpv_chunk reports (the wire partials `fpart` hold
// one chunk); a snapshot-mode helper batch regenerates each chunk's shares first.
int launch_fpv_query(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, CRows meas, CRows proof,
                     uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const size_t ch = fpv_chunk(c, st, n);
  CHK(launch_fpv_weights(c, st, n, proof, d_status));
  if (st->snap_active && c->query_overlap && n > 1) {
    // Half-chunks through two scratch halves: k_fpv_regen of half-chunk i + 1 (aux stream, a
    // VALU-bound sponge pass) runs beside the query of half-chunk i (HBM-bound wire passes).
    // regen(i) waits for query(i - 2), which read the same half; query(i) waits for regen(i).
    const size_t hc = std::max<size_t>(1, (ch + 1) / 2), row = (size_t)g.meas_len * g.es;
    CHK(st->scratch.ensure(2 * hc * row));
    CHK(ensure_aux(c));
    HIPCHK(hipEventRecord(c->aux_ev[2], c->stream));  // the snapshots are written
    HIPCHK(hipStreamWaitEvent(c->aux, c->aux_ev[2], 0));
    for (size_t i = 0, r0 = 0; r0 < n; ++i, r0 += hc) {
      const size_t nr = std::min(hc, n - r0), h = i & 1;
      uint8_t* buf = st->scratch.u8() + h * hc * row;
      if (i >= 2) HIPCHK(hipStreamWaitEvent(c->aux, c->aux_ev[2 + h], 0));
      CHK(regen_rows(c, st, r0, nr, buf, c->aux));
      HIPCHK(hipEventRecord(c->aux_ev[h], c->aux));
      HIPCHK(hipStreamWaitEvent(c->stream, c->aux_ev[h], 0));
      CHK(launch_fpv_query_rows(c, st, r0, nr, CRows{buf, row}, d_status + r0));
      HIPCHK(hipEventRecord(c->aux_ev[2 + h], c->stream));
    }
    return 0;
  }
  for (size_t r0 = 0; r0 < n; r0 += ch) {
    const size_t nr = std::min(ch, n - r0);
    CRows m{meas.base + r0 * meas.stride, meas.stride};
    if (st->snap_active) {
      CHK(regen_rows(c, st, r0, nr));
      m = CRows{st->scratch.u8(), (size_t)g.meas_len * g.es};
    }
    CHK(launch_fpv_query_rows(c, st, r0, nr, m, d_status + r0));
  }
  return 0;
}

template <class FO>
int launch_prep_query(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, uint8_t* d_status,
                      bool weights_only = false);

// Row pitch of a state's input shares: the caller's (prio3gpu_state_set_input_pitch) or packed.
size_t input_pitch(const prio3gpu_state* st) {
  const Cfg& g = st->ctx->cfg;
  return st->in_pitch ? st->in_pitch : (st->agg_id == 0 ? g.leader_share_len : g.helper_share_len);
}

// prepare_init, first phase: query randomness, (helper) share expansion, joint randomness.
template <class FO>
int launch_prep_xof(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* d_nonces,
                    const uint8_t* d_pub, const uint8_t* d_in, uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const uint32_t es = g.es;
  const uint32_t N = (uint32_t)n;
  const uint32_t TPB = 256;
  uint64_t vk_lo, vk_hi;
  memcpy(&vk_lo, c->vk, 8);
  memcpy(&vk_hi, c->vk + 8, 8);
  CRows nonces{d_nonces, 16};
  CRows pub{d_pub, g.public_share_len};
  Rows t_rows{st->t.u8(), (size_t)16 * g.qr_len};
  st->query_done = false;
  if (g.kind == KIND_COUNT) {
    // Count: one kernel derives t and runs the whole FLP query (k_flp_query_lane with the nonces):
    // the short Keccak and the latency-bound query share the launch, and the query phase is empty
    const size_t in_pitch = input_pitch(st);
    CRows meas{d_in, in_pitch}, proof{d_in + (size_t)g.meas_len * es, in_pitch};
    if (st->agg_id != 0) {
      Rows mo{st->meas.u8(), (size_t)g.meas_len * es};
      Rows po{st->proof.u8(), (size_t)g.proof_len * es};
      {
        PROF(KID_EXPAND);
        hipLaunchKernelGGL(k_expand<FO>, grid1(n, TPB), dim3(TPB), c->expand_lds, c->stream, g, N,
                           (uint32_t)st->agg_id, CRows{d_in, in_pitch}, mo, po, d_status);
      }
      meas = CRows{mo.base, mo.stride};
      proof = CRows{po.base, po.stride};
    }
    {
      PROF(KID_FLP_QUERY_LANE);
      hipLaunchKernelGGL(k_flp_query_lane<FO>, grid1(n, 256), dim3(256), 0, c->stream, g, N, meas,
                         proof, CRows{st->t.u8(), 16}, CRows{st->jr.u8(), 16},
                         CRows{st->part.u8(), 16}, Rows{st->prep.u8(), g.prep_share_len}, d_status,
                         d_nonces, vk_lo, vk_hi);
    }
    HIPCHK(hipGetLastError());
    st->meas_rows = meas;
    st->proof_rows = proof;
    st->n = n;
    st->xof_done = true;
    st->weights_done = false;
    st->query_done = true;
    return 0;
  }
  {
    PROF(KID_QUERY);
    hipLaunchKernelGGL(k_query_rand<FO>, grid1(n, TPB), dim3(TPB), 0, c->stream, g, N, vk_lo, vk_hi,
                       nonces, t_rows, d_status);
  }
  st->spec_ok = false;
  uint64_t* spec_lo = nullptr;
  uint8_t* spec_cy = nullptr;
  uint32_t snd = 0, se0 = 0, se1 = 0;
  if (g.jr_len > 0 && c->speculate && spec_range(g, snd, se0, se1)) {
    // sized by prio3gpu_state_create for the state's capacity (no growth inside a call)
    spec_lo = reinterpret_cast<uint64_t*>(st->spec_lo.p);
    spec_cy = st->spec_cy.u8();
    st->spec_ok = true;
    st->spec_n = n;
    st->spec_nd = snd;
    st->spec_e0 = se0;
    st->spec_e1 = se1;
  }
  CRows meas, proof, blinds;
  const size_t in_pitch = input_pitch(st);
  if (st->agg_id == 0) {
    meas = CRows{d_in, in_pitch};
    proof = CRows{d_in + (size_t)g.meas_len * es, in_pitch};
    blinds = CRows{d_in + (size_t)(g.meas_len + g.proof_len) * es, in_pitch};
  } else {
    Rows mo{st->meas.u8(), (size_t)g.meas_len * es};
    Rows po{st->proof.u8(), (size_t)g.proof_len * es};
    bool fused_done = false;
    if constexpr (FO::ES == 16) {
      // Few huge reports: the two helper sponges (expansion, joint-rand part) in lockstep.
      if (g.kind == KIND_FPVEC && c->fused_helper && !g.exact_squeeze && g.jr_len > 0) {
        CHK(c->fallback.ensure(4));
        uint32_t* fb = reinterpret_cast<uint32_t*>(c->fallback.p);
        HIPCHK(hipMemsetAsync(fb, 0, 4, c->stream));
        st->snap_pair = c->pair_chains;
        if (c->pair_chains) {
          // 64 reports per workgroup: two producer, two consumer sponge waves and a storer
          PROF(KID_HELPER_XOF);
          const uint32_t blocks = (N + kHxRows - 1) / kHxRows;
          const size_t lds = std::max<size_t>(kHxPairLds, spread_ok(c, blocks) ? c->spread_lds : 0);
          hipLaunchKernelGGL(k_helper_xof_pair<kHxDepth>, dim3(blocks), dim3(5 * kHxRows), lds,
                             c->stream, g, N, CRows{d_in, in_pitch}, nonces, pub, mo, po,
                             Rows{st->part.u8(), 16}, Rows{st->seed.u8(), 16},
                             Rows{st->jr.u8(), (size_t)g.jr_len * es}, d_status, fb,
                             spec_lo, spec_cy,
                             st->snap ? reinterpret_cast<uint64_t*>(st->snaps.p) : nullptr);
        } else {
          PROF(KID_HELPER_XOF);
          const uint32_t P = chain_pairs(c, n), rows = P * kHxRows;
          const uint32_t blocks = (N + rows - 1) / rows;
          const size_t lds = std::max<size_t>(P * kHxRingBytes,
                                              spread_ok(c, blocks) ? c->spread_lds : 0);
          auto kern = P == 2 ? k_helper_xof<kHxDepth, 2> : k_helper_xof<kHxDepth, 1>;
          hipLaunchKernelGGL(kern, dim3(blocks), dim3(3 * rows), lds, c->stream, g, N,
                             CRows{d_in, in_pitch}, nonces, pub, mo, po,
                             Rows{st->part.u8(), 16}, Rows{st->seed.u8(), 16},
                             Rows{st->jr.u8(), (size_t)g.jr_len * es}, d_status, fb,
                             spec_lo, spec_cy,
                             st->snap ? reinterpret_cast<uint64_t*>(st->snaps.p) : nullptr);
        }
        uint32_t h_fb = 0;
        HIPCHK(hipMemcpyAsync(&h_fb, fb, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        fused_done = h_fb == 0;  // else: a non-canonical element; redo the exact two-pass path
      }
    }
    if (fused_done) {  // the storer wave wrote the speculative column sums
      st->snap_active = st->snap;
      if (st->snap_active && st->spec_ok) {
        // the storer summed EVERY word of the share: the column sums cover all elements, so no
        // edge element is read from rows that only exist as snapshots
        st->spec_e0 = 0;
        st->spec_e1 = g.meas_len;
      }
      st->meas_rows = CRows{mo.base, mo.stride};
      st->proof_rows = CRows{po.base, po.stride};
      st->n = n;
      st->xof_done = true;
      st->weights_done = false;
      return 0;
    }
    st->snap_active = false;
    if (st->snap) {  // the exact path (non-canonical element, or fused path off) stores the rows
      CHK(st->meas.ensure(n * (size_t)g.meas_len * es));
      mo = Rows{st->meas.u8(), (size_t)g.meas_len * es};
    }
    {
      PROF(KID_EXPAND);
      // c->expand_lds (PRIO3GPU_EXPAND_LDS, A/B knob): unused dynamic LDS that caps the blocks
      // per CU, i.e. k_expand's occupancy
      hipLaunchKernelGGL(k_expand<FO>, grid1(n, TPB), dim3(TPB), c->expand_lds, c->stream, g, N,
                         (uint32_t)st->agg_id, CRows{d_in, in_pitch}, mo, po, d_status);
    }
    meas = CRows{mo.base, mo.stride};
    proof = CRows{po.base, po.stride};
    blinds = CRows{d_in + 32, in_pitch};
  }
  bool ring_done = false;
  if constexpr (FO::ES == 16) {
    // few huge FixedPoint reports: sponge wave + loader wave per CU (k_jr_ring)
    const uint32_t P = chain_pairs(c, n), rows = P * kHxRows;
    const uint32_t blocks = (N + rows - 1) / rows;
    const uint32_t pblocks = (N + 2 * kHxRows - 1) / (2 * kHxRows);
    if (g.jr_len > 0 && g.kind == KIND_FPVEC && c->jr_ring && c->jr_lds == 0 && c->pair_chains &&
        spread_ok(c, pblocks)) {
      // 128 reports per workgroup: four sponge waves (a lane pair per report) and two loaders
      PROF(KID_JR_RING);
      const size_t lds = std::max<size_t>(kJrPairLds, c->spread_lds);
      hipLaunchKernelGGL(k_jr_ring_pair, dim3(pblocks), dim3(6 * kHxRows), lds, c->stream,
                         g, N, (uint32_t)st->agg_id, nonces, pub, blinds, meas,
                         Rows{st->part.u8(), 16}, Rows{st->seed.u8(), 16},
                         Rows{st->jr.u8(), (size_t)g.jr_len * es}, d_status, spec_lo, spec_cy);
      ring_done = true;
    } else if (g.jr_len > 0 && g.kind == KIND_FPVEC && c->jr_ring && c->jr_lds == 0 &&
               spread_ok(c, blocks)) {
      PROF(KID_JR_RING);
      const size_t lds = std::max<size_t>(P * kHxRingBytes, c->spread_lds);
      auto kern = P == 2 ? k_jr_ring<2> : k_jr_ring<1>;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(2 * rows), lds, c->stream,
                         g, N, (uint32_t)st->agg_id, nonces, pub, blinds, meas,
                         Rows{st->part.u8(), 16}, Rows{st->seed.u8(), 16},
                         Rows{st->jr.u8(), (size_t)g.jr_len * es}, d_status, spec_lo, spec_cy);
      ring_done = true;
    }
  }
  if (g.jr_len > 0 && !ring_done) {
    {
      PROF(KID_JR);
      // a wave per CU when there are few (see spread_ok); otherwise 4-wave blocks
      const bool sp = c->jr_lds == 0 && spread_ok(c, (N + 63) / 64);
      const uint32_t tpb = sp ? 64u : TPB;
      const size_t jr_lds = sp ? c->spread_lds
                               : std::max<size_t>((TPB / 64) * kJrWaveLds,
                                                  std::min<size_t>(c->jr_lds, 160 * 1024));
      hipLaunchKernelGGL(k_jr<FO>, grid1(n, tpb), dim3(tpb), jr_lds, c->stream, g, N,
                         (uint32_t)st->agg_id, nonces, pub, blinds, meas, Rows{st->part.u8(), 16},
                         Rows{st->seed.u8(), 16}, Rows{st->jr.u8(), (size_t)g.jr_len * es}, d_status,
                         spec_lo, spec_cy);
    }
  }
  HIPCHK(hipGetLastError());
  st->meas_rows = meas;
  st->proof_rows = proof;
  st->n = n;
  st->xof_done = true;
  st->weights_done = false;
  return 0;
}

// ParallelSum types (SumVec, Histogram, Field128): the FLP query in two kernels -- the Lagrange
// weights and the rest of the verifier except the wires (k_flp_weights: lane per report,
// latency-bound), then the wire pass over the measurement share (HBM streaming).
// weight rows (row-major), then k_flp_weights' element-major scratch (block prefix products)
WMat psum_wrows(const prio3gpu_state* st) {
  const Cfg& g = st->ctx->cfg;
  return WMat{st->w.u8(), (size_t)flp_w_len(g) * g.es, (size_t)g.es};
}

int launch_psum_weights(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, CRows proof,
                        uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const uint32_t N = (uint32_t)n;
  uint8_t* wscr = st->w.u8() + (size_t)N * flp_w_len(g) * g.es;
  PROF(KID_FLP_WEIGHTS);
  hipLaunchKernelGGL(k_flp_weights, grid1(n, kFwThreads), dim3(kFwThreads), 0, c->stream, g, N,
                     proof, CRows{st->t.u8(), 16}, CRows{st->jr.u8(), (size_t)g.jr_len * g.es},
                     CRows{st->part.u8(), 16}, Rows{st->prep.u8(), g.prep_share_len}, d_status,
                     psum_wrows(st), wscr);
  HIPCHK(hipGetLastError());
  st->weights_done = true;
  return 0;
}

int launch_psum_query(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, CRows meas, CRows proof,
                      uint8_t* d_status) {
  const Cfg& g = c->cfg;
  const uint32_t es = g.es;
  const uint32_t N = (uint32_t)n;
  if (!st->weights_done) CHK(launch_psum_weights(c, st, n, proof, d_status));
  st->weights_done = false;
  const WMat wrows = psum_wrows(st);
  const CRows jr{st->jr.u8(), (size_t)g.jr_len * es};
  const Rows prep{st->prep.u8(), g.prep_share_len};
  if (g.chunk <= 64 && c->wires_cols) {
    // G = next_pow2(chunk) lanes per report, lane = column (Histogram, small SumVec/CountVec)
    uint32_t lg = 0;
    while ((1u << lg) < g.chunk) ++lg;
    PROF(KID_FLP_WIRES_COLS);
    hipLaunchKernelGGL(k_flp_wires_cols, grid1((size_t)N << lg, 256), dim3(256), 0, c->stream, g, N,
                       lg, meas, proof, wrows, jr, prep, d_status);
  } else if (c->wires_mfma && g.kind == KIND_SUMVEC && g.chunk > 64 && g.calls <= kWmMaxCalls &&
             wires_mfma_e_bytes(g.calls) + 16 <= 64 * 1024) {
    // byte-limb convolution on v_mfma_i32_32x32x32_i8 (wires_mfma.h): a wave per 32 columns
    const uint32_t nwv = std::min(4u, (g.chunk + 31) / 32);
    PROF(KID_FLP_WIRES_MFMA);
    hipLaunchKernelGGL(k_flp_wires_mfma, dim3(N), dim3(64 * nwv), wires_mfma_e_bytes(g.calls) + 16,
                       c->stream, g, N, meas, proof, wrows, prep, d_status);
  } else {
    // the VALU wire pass: block per report, (column, row group) slots; short reports get >= 4
    // rows per thread (Histogram256: H 16 -> 4 took 18.0 -> 6.1 ms/step,
    // profiles/r02/ab_hist_slots*.log)
    constexpr uint32_t kSlots = 256;
    FlpDims dims;
    uint32_t nthr;
    dims.rp_len = std::max(g.chunk, g.calls) + 1;
    dims.cols = g.chunk;
    if (g.chunk <= kSlots) {
      dims.H = std::min(kSlots / g.chunk, std::max(1u, g.calls / 4));
      nthr = ((dims.H * g.chunk + 63) / 64) * 64;
    } else {
      dims.H = 1;
      nthr = 256;
    }
    size_t lds2 = (size_t)16 * (2 * (size_t)g.calls + 2 * (size_t)dims.H * dims.cols + nthr) + 16;
    lds2 = (lds2 + 15) & ~(size_t)15;
    if (lds2 > 160 * 1024) {
      set_err("FLP wire pass LDS requirement %zu too large", lds2);
      return PRIO3GPU_E_ARG;
    }
    PROF(KID_FLP_WIRES);
    hipLaunchKernelGGL(k_flp_wires<Field128Ops>, dim3(N), dim3(nthr), lds2, c->stream, g, N, dims,
                       meas, proof, wrows, jr, prep, d_status);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// prepare_init, second phase: the FLP query over the shares the first phase left in the state.
template <class FO>
int launch_prep_query(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, uint8_t* d_status,
                      bool weights_only) {
  const Cfg& g = c->cfg;
  const uint32_t es = g.es;
  const uint32_t N = (uint32_t)n;
  const CRows meas = st->meas_rows, proof = st->proof_rows;
  if (!st->xof_done || st->n != n) {
    set_err("prepare_init query phase without its XOF phase over the same %zu reports", n);
    return PRIO3GPU_E_ARG;
  }
  const bool psum = (g.kind == KIND_SUMVEC || g.kind == KIND_HISTOGRAM);
  if (weights_only) {  // the latency-bound first half of a ParallelSum query; others: nothing yet
    if constexpr (FO::ES == 16) {
      if (psum && !st->weights_done) CHK(launch_psum_weights(c, st, n, proof, d_status));
    }
    return 0;
  }
  st->xof_done = false;
  if (st->query_done) {  // Count: ran in the XOF phase
    st->query_done = false;
    return 0;
  }
  if constexpr (FO::ES == 16) {
    if (g.kind == KIND_FPVEC) {
      CHK(launch_fpv_query(c, st, n, meas, proof, d_status));
      return 0;
    }
  }
  // FLP query: block per report.  ParallelSum types (SumVec, Histogram) split it in two: the
  // weights (power tables, NTTs, gadget outputs; latency-bound, 2 waves) and the wire pass over
  // the measurement share (HBM streaming, many blocks in flight).
  if constexpr (FO::ES == 16) {
    if (psum) return launch_psum_query(c, st, n, meas, proof, d_status);
  }
  if (g.kind != KIND_COUNT && g.kind != KIND_SUM) {
    set_err("no FLP query for VDAF kind %u", g.kind);
    return PRIO3GPU_E_ARG;
  }
  {
    PROF(KID_FLP_QUERY_LANE);
    hipLaunchKernelGGL(k_flp_query_lane<FO>, grid1(n, 256), dim3(256),
                       flpq_pair(g) ? kFlpqPairLds : 0u, c->stream, g, N, meas,
                       proof, CRows{st->t.u8(), 16}, CRows{st->jr.u8(), (size_t)g.jr_len * es},
                       CRows{st->part.u8(), 16}, Rows{st->prep.u8(), g.prep_share_len}, d_status,
                       nullptr, 0ull, 0ull);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

template <class FO>
int launch_prepare_init(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* d_nonces,
                        const uint8_t* d_pub, const uint8_t* d_in, uint8_t* d_status) {
  CHK(launch_prep_xof<FO>(c, st, n, d_nonces, d_pub, d_in, d_status));
  return launch_prep_query<FO>(c, st, n, d_status);
}

template <class FO>
int launch_decide(prio3gpu_ctx* c, size_t n, const uint8_t* d_l, const uint8_t* d_h,
                  uint8_t* d_msg, uint8_t* d_status) {
  const Cfg& g = c->cfg;
  if (g.kind == KIND_FPVEC) {
    PROF(KID_FPV_DECIDE);
    hipLaunchKernelGGL(k_fpv_decide, dim3((unsigned)n), dim3(256), 0, c->stream, g, (uint32_t)n,
                       CRows{d_l, g.prep_share_len}, CRows{d_h, g.prep_share_len},
                       Rows{d_msg, g.prep_msg_len}, d_status);
    HIPCHK(hipGetLastError());
    return 0;
  }
  {
    PROF(KID_DECIDE);
    hipLaunchKernelGGL(k_decide<FO>, grid1(n, 256), dim3(256), 0, c->stream, g, (uint32_t)n,
                       CRows{d_l, g.prep_share_len}, CRows{d_h, g.prep_share_len},
                       Rows{d_msg, g.prep_msg_len ? g.prep_msg_len : 16}, d_status);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// Segmented accumulation of the batch's output shares into agg slots.
template <class FO>
int launch_accumulate(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint32_t* slots,
                      const uint8_t* d_status, prio3gpu_agg* agg) {
  const Cfg& g = c->cfg;
  const uint32_t S = agg->slots;
  const bool spec = st->spec_ok && st->spec_n == n && FO::ES == 16;
  const uint32_t epb = std::min<uint32_t>(256, std::max<uint32_t>(1, g.meas_len));
  const uint32_t tiles = (g.meas_len + epb - 1) / epb;
  // One batch slot and the same batch shape as the last call: the plan on the device still holds
  // (no host planning, no upload, no stream synchronisation).
  const bool reuse = !slots && c->plan_valid && c->plan_n == n && c->plan_slots == S &&
                     c->plan_spec == spec &&
                     (!spec || (c->plan_nd == st->spec_nd && c->plan_e0 == st->spec_e0 &&
                                c->plan_e1 == st->spec_e1));
  if (!reuse) {
    c->plan_valid = false;
    std::vector<uint32_t> hslots;
    const uint32_t* sl = slots;
    if (slots && is_device_ptr(slots)) {
      hslots.resize(n);
      HIPCHK(hipMemcpyAsync(hslots.data(), slots, n * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      sl = hslots.data();
    }
    for (size_t r = 0; r < n; ++r) {
      const uint32_t s = sl ? sl[r] : 0;
      if (s >= S) {
        set_err("batch slot %u out of range (%u slots)", s, S);
        return PRIO3GPU_E_ARG;
      }
    }
    auto slot_of = [&](size_t r) -> uint32_t { return sl ? sl[r] : 0u; };
    // Chunks (runs of reports of one slot, contiguous per slot in chunk order) of two kinds:
    //  * direct: k_accum_partial sums every measurement element of the chunk's reports;
    //  * speculative (whole waves of 64 reports whose slots agree, when k_jr left column sums):
    //    k_accum_spec folds the per-wave sums of elements [e0, e1) and corrects the rejected
    //    rows, k_accum_partial adds the few edge elements outside that range.
    const size_t nw = (n + 63) / 64;
    std::vector<std::vector<uint32_t>> spec_w(S), direct_r(S);
    if (spec) {
      for (size_t w = 0; w < nw; ++w) {
        const size_t r0 = 64 * w, r1 = std::min(n, r0 + 64);
        const uint32_t s = slot_of(r0);
        bool uni = true;
        for (size_t r = r0 + 1; r < r1 && uni; ++r) uni = slot_of(r) == s;
        if (uni) {
          spec_w[s].push_back((uint32_t)w);
        } else {
          for (size_t r = r0; r < r1; ++r) direct_r[slot_of(r)].push_back((uint32_t)r);
        }
      }
    } else {
      for (size_t r = 0; r < n; ++r) direct_r[slot_of(r)].push_back((uint32_t)r);
    }
    const uint32_t G = 256 / epb;
    const size_t target_chunks = std::max<size_t>(1, 2048 / tiles);
    const size_t CH = std::max<size_t>((size_t)G * 4, (n + target_chunks - 1) / target_chunks);
    const size_t WCH = 32;  // waves per speculative chunk
    auto& perm = c->h_perm;
    auto& cb = c->h_chunk_begin;
    auto& cs = c->h_chunk_slot;
    perm.clear();
    cb.clear();
    cs.clear();
    std::vector<uint32_t> dir_ids, spec_ids, swb, wl;
    for (uint32_t s = 0; s < S; ++s) {
      const auto& sw = spec_w[s];
      for (size_t i = 0; i < sw.size(); i += WCH) {
        spec_ids.push_back((uint32_t)cs.size());
        cb.push_back((uint32_t)perm.size());
        cs.push_back(s);
        swb.push_back((uint32_t)wl.size());
        for (size_t q = i; q < std::min(sw.size(), i + WCH); ++q) {
          wl.push_back(sw[q]);
          for (size_t r = 64 * (size_t)sw[q]; r < std::min(n, 64 * (size_t)sw[q] + 64); ++r)
            perm.push_back((uint32_t)r);
        }
      }
      const auto& dr = direct_r[s];
      for (size_t i = 0; i < dr.size(); i += CH) {
        dir_ids.push_back((uint32_t)cs.size());
        cb.push_back((uint32_t)perm.size());
        cs.push_back(s);
        perm.insert(perm.end(), dr.begin() + i, dr.begin() + std::min(dr.size(), i + CH));
      }
    }
    const uint32_t nch = (uint32_t)cs.size();
    if (nch == 0) return 0;
    cb.push_back((uint32_t)perm.size());
    swb.push_back((uint32_t)wl.size());
    const uint32_t ndir = (uint32_t)dir_ids.size(), nspec = (uint32_t)spec_ids.size();
    CHK(c->perm.ensure(std::max<size_t>(1, perm.size()) * 4));
    CHK(c->chunks.ensure((size_t)(2 * nch + 1) * 4));
    CHK(c->partials.ensure((size_t)nch * g.meas_len * g.es));
    CHK(c->pcounts.ensure((size_t)nch * 4));
    CHK(c->spec_idx.ensure((size_t)(ndir + 2 * nspec + 1 + wl.size() + 1) * 4));
    HIPCHK(hipMemcpyAsync(c->perm.p, perm.data(), perm.size() * 4, hipMemcpyHostToDevice, c->stream));
    uint32_t* d_cb = reinterpret_cast<uint32_t*>(c->chunks.p);
    uint32_t* d_cs = d_cb + nch + 1;
    HIPCHK(hipMemcpyAsync(d_cb, cb.data(), (nch + 1) * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_cs, cs.data(), nch * 4, hipMemcpyHostToDevice, c->stream));
    uint32_t* d_dir = reinterpret_cast<uint32_t*>(c->spec_idx.p);
    uint32_t* d_sid = d_dir + ndir;
    uint32_t* d_swb = d_sid + nspec;
    uint32_t* d_wl = d_swb + nspec + 1;
    if (ndir) HIPCHK(hipMemcpyAsync(d_dir, dir_ids.data(), ndir * 4, hipMemcpyHostToDevice, c->stream));
    if (nspec) {
      HIPCHK(hipMemcpyAsync(d_sid, spec_ids.data(), nspec * 4, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(d_swb, swb.data(), (nspec + 1) * 4, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(d_wl, wl.data(), wl.size() * 4, hipMemcpyHostToDevice, c->stream));
    }
    // the host vectors must outlive the async copies (and a later re-plan rewrites them)
    HIPCHK(hipStreamSynchronize(c->stream));
    c->plan_ndir = ndir;
    c->plan_nspec = nspec;
    c->plan_nch = nch;
    c->plan_valid = !slots;
    c->plan_n = n;
    c->plan_slots = S;
    c->plan_spec = spec;
    c->plan_nd = st->spec_nd;
    c->plan_e0 = st->spec_e0;
    c->plan_e1 = st->spec_e1;
  }
  const uint32_t ndir = c->plan_ndir, nspec = c->plan_nspec, nch = c->plan_nch;
  const uint32_t* d_cb = reinterpret_cast<const uint32_t*>(c->chunks.p);
  const uint32_t* d_cs = d_cb + nch + 1;
  const uint32_t* d_dir = reinterpret_cast<const uint32_t*>(c->spec_idx.p);
  const uint32_t* d_sid = d_dir + ndir;
  const uint32_t* d_swb = d_sid + nspec;
  const uint32_t* d_wl = d_swb + nspec + 1;
  const uint32_t* d_perm = reinterpret_cast<const uint32_t*>(c->perm.p);
  uint32_t* d_pc = reinterpret_cast<uint32_t*>(c->pcounts.p);
  const size_t red_lds = 256 * sizeof(typename FO::T) + 16;
  if (ndir) {
    PROF(KID_ACC_PART);
    hipLaunchKernelGGL(k_accum_partial<FO>, dim3(ndir, tiles), dim3(256), red_lds, c->stream, g,
                       st->meas_rows, d_perm, d_cb, d_status, epb, c->partials.u8(), d_pc, d_dir,
                       g.meas_len, g.meas_len);
  }
  if (nspec) {
    const uint32_t e0 = st->spec_e0, e1 = st->spec_e1;
    const uint32_t nedge = e0 + (g.meas_len - e1);
    const uint32_t epb_e = std::min<uint32_t>(256, std::max<uint32_t>(1, nedge));
    // at least one tile: its first row of blocks also counts each chunk's accepted reports (a
    // snapshot-mode batch has no edge elements -- its column sums cover every element)
    const uint32_t tiles_e = std::max<uint32_t>(1, (nedge + epb_e - 1) / epb_e);
    {
      PROF(KID_ACC_PART);
      hipLaunchKernelGGL(k_accum_partial<FO>, dim3(nspec, tiles_e), dim3(256), red_lds, c->stream, g,
                         st->meas_rows, d_perm, d_cb, d_status, epb_e, c->partials.u8(), d_pc, d_sid,
                         e0, e1);
    }
    {
      PROF(KID_ACC_SPEC);
      hipLaunchKernelGGL(k_accum_spec<FO>, dim3(nspec, (e1 - e0 + 127) / 128), dim3(256), 0,
                         c->stream, g, (uint32_t)n, st->meas_rows, d_sid, d_swb, d_wl,
                         reinterpret_cast<const uint64_t*>(st->spec_lo.p), st->spec_cy.u8(),
                         st->spec_nd, e0, e1, d_status, c->partials.u8());
    }
  }
  {
    PROF(KID_ACC_MERGE);
    const uint32_t bpe =
        (g.kind == KIND_SUMVEC || g.kind == KIND_SUM || g.kind == KIND_FPVEC) ? g.bits : 1u;
    hipLaunchKernelGGL(k_accum_merge<FO>, grid1(g.out_len, 256 / bpe), dim3(256), 0, c->stream, g, nch,
                       d_cs, c->partials.u8(), reinterpret_cast<const uint32_t*>(c->pcounts.p),
                       agg->share.u8(), reinterpret_cast<unsigned long long*>(agg->counts.p));
  }
  HIPCHK(hipGetLastError());
  return 0;
}

template <class FO>
int launch_out_shares(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* d_status,
                      uint8_t* d_out) {
  const Cfg& g = c->cfg;
  dim3 grid((g.out_len + 255) / 256, (unsigned)n);
  {
    PROF(KID_OUT);
    hipLaunchKernelGGL(k_out_shares<FO>, grid, dim3(256), 0, c->stream, g, (uint32_t)n,
                       st->meas_rows, Rows{d_out, (size_t)g.out_len * g.es}, d_status);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// Accumulation of a prepared batch.  A snapshot-mode helper batch (its shares exist only as
// snapshots) takes the speculative column sums as they are when they are exact without any row:
// every report accepted, whole waves, one batch slot (the storer summed every element of every
// row).  Otherwise its rows are regenerated chunk by chunk and summed directly.
template <class FO>
int accumulate_batch(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint32_t* slots,
                     uint8_t* d_status, prio3gpu_agg* agg) {
  if (!st->snap_active) return launch_accumulate<FO>(c, st, n, slots, d_status, agg);
  const Cfg& g = c->cfg;
  bool whole = st->spec_ok && st->spec_n == n && !slots && n % 64 == 0;
  if (whole) {
    std::vector<uint8_t> hs(n);
    HIPCHK(hipMemcpyAsync(hs.data(), d_status, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (size_t r = 0; r < n && whole; ++r) whole = hs[r] == 0;
  }
  if (whole) return launch_accumulate<FO>(c, st, n, nullptr, d_status, agg);
  const bool spec = st->spec_ok;
  const CRows rows = st->meas_rows;
  st->spec_ok = false;
  const size_t ch = fpv_chunk(c, st, n);
  int rc = 0;
  for (size_t r0 = 0; r0 < n && rc == 0; r0 += ch) {
    const size_t nr = std::min(ch, n - r0);
    rc = regen_rows(c, st, r0, nr);
    st->meas_rows = CRows{st->scratch.u8(), (size_t)g.meas_len * g.es};
    if (rc == 0)
      rc = launch_accumulate<FO>(c, st, nr, slots ? slots + r0 : nullptr, d_status + r0, agg);
    // the next chunk's regeneration overwrites the scratch rows only after this chunk's sums
    // (same stream)
  }
  st->spec_ok = spec;
  st->meas_rows = rows;
  return rc;
}

// Output shares of a prepared batch (a snapshot-mode helper batch: regenerated chunk by chunk).
template <class FO>
int out_shares_batch(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* d_status,
                     uint8_t* d_out) {
  if (!st->snap_active) return launch_out_shares<FO>(c, st, n, d_status, d_out);
  const Cfg& g = c->cfg;
  const CRows rows = st->meas_rows;
  const size_t ch = fpv_chunk(c, st, n), out_row = (size_t)g.out_len * g.es;
  int rc = 0;
  for (size_t r0 = 0; r0 < n && rc == 0; r0 += ch) {
    const size_t nr = std::min(ch, n - r0);
    rc = regen_rows(c, st, r0, nr);
    st->meas_rows = CRows{st->scratch.u8(), (size_t)g.meas_len * g.es};
    if (rc == 0) rc = launch_out_shares<FO>(c, st, nr, d_status + r0, d_out + r0 * out_row);
  }
  st->meas_rows = rows;
  return rc;
}

bool is_f64(const prio3gpu_ctx* c) { return c->cfg.es == 8; }


int check_state(prio3gpu_ctx* c, prio3gpu_state* st, size_t n) {
  if (!c || !st || st->ctx != c) {
    set_err("bad context/state");
    return PRIO3GPU_E_ARG;
  }
  if (n > st->cap) {
    set_err("batch of %zu reports exceeds state capacity %zu", n, st->cap);
    return PRIO3GPU_E_CAPACITY;
  }
  return 0;
}

// status: stage in (host or device) into st->status
int stage_status(prio3gpu_ctx* c, DevBuf& buf, uint8_t* status, size_t n, uint8_t** d_status) {
  if (!status) {
    set_err("status array is required");
    return PRIO3GPU_E_ARG;
  }
  if (is_device_ptr(status)) {
    *d_status = status;
    return 0;
  }
  CHK(buf.ensure(n));
  HIPCHK(hipMemcpyAsync(buf.p, status, n, hipMemcpyHostToDevice, c->stream));
  *d_status = buf.u8();
  return 0;
}

// End of an ABI call: wait for the context's stream unless the context is in async mode and every
// buffer the call touched is device memory (host inputs are staged by async copies and host
// outputs are written by them: those need the wait).
int finish_call(prio3gpu_ctx* c, std::initializer_list<const void*> bufs) {
  bool host = !c->async_mode;
  for (const void* b : bufs)
    if (b && !is_device_ptr(b)) host = true;
  if (host) HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

}  // namespace

// =================================================================================================
// C ABI
// =================================================================================================
// Build identity: janus_amd/_lib.py passes the SHA-256 of the sources, headers and flags it
// compiled; it is kept as a searchable marker so a stale or foreign library is detected without
// loading it.
#ifndef PRIO3GPU_BUILD_HASH
#define PRIO3GPU_BUILD_HASH "unhashed"
#endif
extern "C" __attribute__((used)) const char prio3gpu_build_id[] =
    "PRIO3GPU_BUILD_HASH=" PRIO3GPU_BUILD_HASH;

extern "C" {

const char* prio3gpu_last_error(void) { return g_err.c_str(); }

const char* prio3gpu_build_hash(void) { return prio3gpu_build_id + 20; }

int prio3gpu_ctx_create(int kind, uint32_t bits, uint32_t length, uint32_t chunk_length,
                        const uint8_t verify_key[16], int device, prio3gpu_ctx** out) {
  return prio3gpu_ctx_create2(kind, bits, length, chunk_length, verify_key, device,
                              PRIO3GPU_XOF_SHAKE128, out);
}

int prio3gpu_ctx_create2(int kind, uint32_t bits, uint32_t length, uint32_t chunk_length,
                         const uint8_t verify_key[16], int device, int xof, prio3gpu_ctx** out) {
  if (!out || !verify_key) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  if (xof != PRIO3GPU_XOF_SHAKE128 && xof != PRIO3GPU_XOF_TURBOSHAKE128) {
    set_err("unknown XOF %d", xof);
    return PRIO3GPU_E_ARG;
  }
  *out = nullptr;
  HIPCHK(hipSetDevice(device));
  auto* c = new prio3gpu_ctx();
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
      cu = 0;  // unknown: no spreading
    c->cus = (uint32_t)cu;
  }
  c->device = device;
  memcpy(c->vk, verify_key, 16);
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    set_err("hipStreamCreate: %s", hipGetErrorString(e));
    delete c;
    return PRIO3GPU_E_HIP;
  }
  int rc = setup_cfg(c, kind, bits, length, chunk_length);
  if (!rc) rc = c->fallback.ensure(4);  // k_helper_xof's counter: no allocation inside a call
  if (rc) {
    prio3gpu_ctx_destroy(c);
    return rc;
  }
  c->cfg.xof = xof == PRIO3GPU_XOF_TURBOSHAKE128 ? kXofTurboShake128 : kXofShake128;
  *out = c;
  return 0;
}

int prio3gpu_ctx_destroy(prio3gpu_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->twiddles.release();
  c->twiddles1.release();
  c->twiddles2.release();
  for (auto& b : c->io) b.release();
  c->perm.release();
  c->chunks.release();
  c->partials.release();
  c->pcounts.release();
  for (auto& r : c->prof.recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto ev : c->prof.pool) (void)hipEventDestroy(ev);
  for (auto ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->wait_ev) (void)hipEventDestroy(c->wait_ev);
  if (c->aux) (void)hipStreamSynchronize(c->aux);
  for (auto ev : c->aux_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int prio3gpu_ctx_sizes(const prio3gpu_ctx* c, prio3gpu_sizes* out) {
  if (!c || !out) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  *out = c->sz;
  return 0;
}

int prio3gpu_ctx_sync(prio3gpu_ctx* c) {
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

void* prio3gpu_ctx_stream(prio3gpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

int prio3gpu_state_create(prio3gpu_ctx* c, int agg_id, size_t capacity, prio3gpu_state** out) {
  if (!c || !out || (agg_id != 0 && agg_id != 1) || capacity == 0) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  auto* st = new prio3gpu_state();
  st->ctx = c;
  st->agg_id = agg_id;
  st->cap = capacity;
  const Cfg& g = c->cfg;
  const size_t N = capacity;
  // Every buffer a call on this state may touch, sized for `capacity` reports, so no call grows
  // one; the sum is checked against the device's free memory before anything is allocated.
  struct Want {
    DevBuf* b;
    size_t bytes;
  };
  std::vector<Want> plan;
  auto want = [&](DevBuf& b, size_t bytes) { plan.push_back({&b, bytes}); };
  want(st->t, N * 16 * g.qr_len);
  want(st->jr, N * 16 * std::max<uint32_t>(1, g.jr_len));
  want(st->part, N * 16);
  want(st->seed, N * 16);
  want(st->prep, N * g.prep_share_len);
  want(st->msg, N * 16);
  want(st->status, N);
  if (g.kind == KIND_SUMVEC || g.kind == KIND_HISTOGRAM)
    want(st->w, N * (size_t)(flp_w_len(g) + flp_scratch_len(g)) * g.es);  // rows + scratch
  if (g.kind == KIND_FPVEC) {
    want(st->w, N * (size_t)fpv_w_layout(g).len * 16);
    st->fpart_rows = std::min<size_t>(N, c->snap_chunk);
    want(st->fpart, st->fpart_rows * (size_t)fpv_rows(g) * g.chunk * 32);
    want(st->flags, N * 4);
  }
  {  // speculative column sums (k_jr, the FixedPoint storer waves), one row per 64 reports
    uint32_t snd = 0, se0 = 0, se1 = 0;
    if (g.jr_len > 0 && spec_range(g, snd, se0, se1)) {
      const size_t nw = (N + 63) / 64;
      want(st->spec_lo, nw * snd * 8);
      want(st->spec_cy, nw * snd);
    }
  }
  st->snap = g.kind == KIND_FPVEC && agg_id == 1 && c->helper_snap;
  if (agg_id == 1) {
    const size_t row = (size_t)g.meas_len * g.es;
    if (st->snap) {
      // the expanded shares live as snapshots; the regenerated rows of one query chunk (two
      // half-chunks with query_overlap) are the only full-size scratch.  The full rows exist only
      // on the exact path (a non-canonical element), which allocates them when it runs.
      want(st->snaps, N * (size_t)snap_count(g) * kSnapBytes);
      want(st->scratch, 2 * ((st->fpart_rows + 1) / 2) * row);
    } else {
      want(st->meas, N * row);
    }
    want(st->proof, N * (size_t)g.proof_len * g.es);
  }
  size_t need = 0;
  for (const Want& w : plan) need += w.bytes ? w.bytes : 16;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    fr = tot = 0;
  }
  if (tot != 0 && need > fr) {
    set_err("a %s state of %zu reports needs %zu bytes of device memory; %zu of %zu bytes are free",
            agg_id == 0 ? "leader" : "helper", N, need, fr, tot);
    delete st;
    return PRIO3GPU_E_CAPACITY;
  }
  for (const Want& w : plan) {
    const int rc = w.b->ensure(w.bytes);
    if (rc) {
      delete st;  // DevBuf destructors free what was allocated
      return rc;
    }
  }
  *out = st;
  return 0;
}

int prio3gpu_state_set_input_pitch(prio3gpu_state* st, size_t pitch) {
  if (!st) {
    set_err("null state");
    return PRIO3GPU_E_ARG;
  }
  const Cfg& g = st->ctx->cfg;
  const size_t len = st->agg_id == 0 ? g.leader_share_len : g.helper_share_len;
  if (pitch != 0 && (pitch < len || pitch % 16 != 0)) {
    set_err("input pitch %zu: must be 0 or a multiple of 16 that is >= the input share (%zu B)",
            pitch, len);
    return PRIO3GPU_E_ARG;
  }
  st->in_pitch = pitch;
  return 0;
}

int prio3gpu_state_destroy(prio3gpu_state* st) {
  if (!st) return 0;
  if (st->ctx) (void)hipStreamSynchronize(st->ctx->stream);
  for (DevBuf* b : {&st->t, &st->jr, &st->part, &st->seed, &st->meas, &st->proof, &st->prep,
                    &st->msg, &st->status, &st->nonces, &st->pub, &st->input, &st->w,
                    &st->spec_lo, &st->spec_cy})
    b->release();
  delete st;
  return 0;
}

int prio3gpu_agg_create(prio3gpu_ctx* c, uint32_t num_slots, prio3gpu_agg** out) {
  if (!c || !out || num_slots == 0) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  auto* a = new prio3gpu_agg();
  a->ctx = c;
  a->slots = num_slots;
  if (a->share.ensure((size_t)num_slots * c->cfg.out_len * c->cfg.es) ||
      a->counts.ensure((size_t)num_slots * 8) ||
      a->meta.ensure((size_t)num_slots * sizeof(SlotMeta))) {
    prio3gpu_agg_destroy(a);
    return PRIO3GPU_E_HIP;
  }
  *out = a;
  return prio3gpu_agg_reset(a);
}

int prio3gpu_agg_destroy(prio3gpu_agg* a) {
  if (!a) return 0;
  a->share.release();
  a->counts.release();
  a->meta.release();
  a->wmeta.release();
  delete a;
  return 0;
}

int prio3gpu_agg_reset(prio3gpu_agg* a) {
  HIPCHK(hipMemsetAsync(a->share.p, 0, (size_t)a->slots * a->ctx->cfg.out_len * a->ctx->cfg.es,
                        a->ctx->stream));
  HIPCHK(hipMemsetAsync(a->counts.p, 0, (size_t)a->slots * 8, a->ctx->stream));
  {
    std::vector<SlotMeta> m(a->slots);
    for (auto& x : m) {
      memset(x.ck, 0, sizeof x.ck);
      x.tmin = ~0ull;
      x.tmax = 0ull;
    }
    HIPCHK(hipMemcpyAsync(a->meta.p, m.data(), m.size() * sizeof(SlotMeta),
                          hipMemcpyHostToDevice, a->ctx->stream));
    HIPCHK(hipStreamSynchronize(a->ctx->stream));
  }
  HIPCHK(hipStreamSynchronize(a->ctx->stream));
  return 0;
}

int prio3gpu_agg_read(prio3gpu_agg* a, uint32_t slot, uint8_t* out_share, uint64_t* out_count) {
  if (!a || slot >= a->slots) {
    set_err("bad slot");
    return PRIO3GPU_E_ARG;
  }
  prio3gpu_ctx* c = a->ctx;
  const size_t bytes = (size_t)c->cfg.out_len * c->cfg.es;
  if (out_share)
    HIPCHK(hipMemcpyAsync(out_share, a->share.u8() + slot * bytes, bytes, hipMemcpyDefault,
                          c->stream));
  if (out_count)
    HIPCHK(hipMemcpyAsync(out_count, a->counts.u8() + (size_t)slot * 8, 8, hipMemcpyDefault,
                          c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// Collector::unshard (collector/src/lib.rs:539; prio Prio3::unshard): sum the aggregate shares
// mod p, then decode_result: integers for Count/Sum/SumVec/Histogram (16-byte LE each), or
// d * 2^(1-bits) - num_measurements per entry for the fixed-point vector (prio to_float_bits).
int prio3gpu_unshard(const prio3gpu_ctx* c, const uint8_t* agg_shares, size_t num_shares,
                     uint64_t num_measurements, uint8_t* out_u128, double* out_f64) {
  if (!c || !agg_shares || num_shares == 0) {
    set_err("unshard: bad argument");
    return PRIO3GPU_E_ARG;
  }
  const Cfg& g = c->cfg;
  const uint32_t es = g.es;
  const u128 p = es == 16 ? P128 : P64;
  const size_t share_len = (size_t)g.out_len * es;
  const bool fp = g.kind == KIND_FPVEC;
  if ((fp && !out_f64) || (!fp && !out_u128)) {
    set_err("unshard: %s output required", fp ? "f64" : "u128");
    return PRIO3GPU_E_ARG;
  }
  for (uint32_t e = 0; e < g.out_len; ++e) {
    u128 acc = 0;
    for (size_t k = 0; k < num_shares; ++k) {
      u128 x = 0;
      const uint8_t* src = agg_shares + k * share_len + (size_t)e * es;
      for (uint32_t b = 0; b < es; ++b) x |= (u128)src[b] << (8 * b);
      if (x >= p) {
        set_err("unshard: aggregate share element out of range");
        return PRIO3GPU_E_ARG;
      }
      acc = addmod(acc, x, p);
    }
    if (fp) {
      out_f64[e] = std::ldexp((double)acc, 1 - (int)g.bits) - (double)num_measurements;
    } else {
      for (uint32_t b = 0; b < 16; ++b) out_u128[(size_t)e * 16 + b] = (uint8_t)(acc >> (8 * b));
    }
  }
  return 0;
}

int prio3gpu_agg_update_reports(prio3gpu_agg* a, size_t n, const uint8_t* report_ids,
                                const uint64_t* times, const uint8_t* status,
                                const uint32_t* batch_slots) {
  if (!a || (n && (!report_ids || !times))) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  if (n == 0) return 0;
  prio3gpu_ctx* c = a->ctx;
  HIPCHK(hipSetDevice(c->device));
  const uint8_t *d_ids, *d_times, *d_st = nullptr, *d_slots = nullptr;
  CHK(stage_in(c, c->io[0], report_ids, n * 16, &d_ids));
  CHK(stage_in(c, c->io[1], times, n * 8, &d_times));
  if (status) CHK(stage_in(c, c->io[2], status, n, &d_st));
  if (batch_slots) CHK(stage_in(c, c->io[3], batch_slots, n * 4, &d_slots));
  const uint32_t nwaves = (uint32_t)((n + 255) / 256 * 4);
  CHK(a->wmeta.ensure((size_t)nwaves * sizeof(WaveMeta)));
  {
    PROF(KID_REPORT_META);
    hipLaunchKernelGGL(k_report_meta, grid1(n, 256), dim3(256), 0, c->stream, (uint32_t)n,
                       CRows{d_ids, 16}, reinterpret_cast<const uint64_t*>(d_times), d_st,
                       reinterpret_cast<const uint32_t*>(d_slots), a->slots,
                       reinterpret_cast<SlotMeta*>(a->meta.p),
                       reinterpret_cast<WaveMeta*>(a->wmeta.p));
  }
  {
    PROF(KID_REPORT_META_FOLD);
    // a column of blocks per slot, ~2K wave partials each (one block walking 65K partials of a
    // 4M-report batch was latency-bound: 0.13 ms)
    const uint32_t ny = std::max(1u, std::min(64u, (uint32_t)((nwaves + 2047) / 2048)));
    hipLaunchKernelGGL(k_report_meta_fold, dim3(a->slots, ny), dim3(256), 0, c->stream, nwaves,
                       reinterpret_cast<const WaveMeta*>(a->wmeta.p),
                       reinterpret_cast<SlotMeta*>(a->meta.p));
  }
  HIPCHK(hipGetLastError());
  // every staged host buffer (ids, times, status, slots) must outlive its copy: the async rule
  return finish_call(c, {report_ids, times, status, batch_slots});
}

int prio3gpu_agg_read_reports(prio3gpu_agg* a, uint32_t slot, uint8_t* out_checksum,
                              uint64_t* out_interval_start, uint64_t* out_interval_duration) {
  if (!a || slot >= a->slots) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  prio3gpu_ctx* c = a->ctx;
  HIPCHK(hipSetDevice(c->device));
  SlotMeta m;
  HIPCHK(hipMemcpyAsync(&m, a->meta.u8() + (size_t)slot * sizeof(SlotMeta), sizeof m,
                        hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (out_checksum)
    for (int i = 0; i < 8; ++i)
      for (int b = 0; b < 4; ++b) out_checksum[4 * i + b] = (uint8_t)(m.ck[i] >> (24 - 8 * b));
  const bool empty = m.tmin > m.tmax;
  if (out_interval_start) *out_interval_start = empty ? 0 : m.tmin;
  if (out_interval_duration) *out_interval_duration = empty ? 0 : m.tmax - m.tmin + 1;
  return 0;
}

int prio3gpu_agg_merge_bytes(prio3gpu_agg* a, uint32_t slot, const uint8_t* share,
                             uint64_t count) {
  if (!a || slot >= a->slots || !share) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  prio3gpu_ctx* c = a->ctx;
  const size_t nel = c->cfg.out_len;
  const size_t bytes = nel * c->cfg.es;
  const uint8_t* d_src;
  CHK(stage_in(c, c->io[0], share, bytes, &d_src));
  uint8_t* dst = a->share.u8() + slot * bytes;
  if (is_f64(c))
    {
      PROF(KID_MERGE);
      hipLaunchKernelGGL(k_merge<Field64Ops>, grid1(nel, 256), dim3(256), 0, c->stream, dst, d_src, nel);
    }
  else
    {
      PROF(KID_MERGE);
      hipLaunchKernelGGL(k_merge<Field128Ops>, grid1(nel, 256), dim3(256), 0, c->stream, dst, d_src, nel);
    }
  HIPCHK(hipGetLastError());
  uint64_t cur = 0;
  HIPCHK(hipMemcpyAsync(&cur, a->counts.u8() + (size_t)slot * 8, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  cur += count;
  HIPCHK(hipMemcpyAsync(a->counts.u8() + (size_t)slot * 8, &cur, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int prio3gpu_prepare_init(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                          const uint8_t* public_shares, const uint8_t* input_shares,
                          uint8_t* out_prep_shares, uint8_t* status) {
  CHK(check_state(c, st, n));
  if (n == 0) return 0;
  if (!nonces || !input_shares || (c->cfg.jr_len && !public_shares)) {
    set_err("null input");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  const uint8_t *d_nonces, *d_pub, *d_in;
  CHK(stage_in(c, st->nonces, nonces, n * 16, &d_nonces));
  CHK(stage_in(c, st->pub, public_shares, n * g.public_share_len, &d_pub));
  const size_t in_len = st->agg_id == 0 ? g.leader_share_len : g.helper_share_len;
  CHK(stage_in(c, st->input, input_shares, (n - 1) * input_pitch(st) + in_len, &d_in));
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  if (is_f64(c))
    CHK(launch_prepare_init<Field64Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  else
    CHK(launch_prepare_init<Field128Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  CHK(copy_out(c, out_prep_shares, st->prep.p, n * g.prep_share_len));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {nonces, public_shares, input_shares, out_prep_shares, status});
}

int prio3gpu_prepare_init_xof(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                              const uint8_t* public_shares, const uint8_t* input_shares,
                              uint8_t* status) {
  CHK(check_state(c, st, n));
  if (n == 0) return 0;
  if (!nonces || !input_shares || (c->cfg.jr_len && !public_shares)) {
    set_err("null input");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  const uint8_t *d_nonces, *d_pub, *d_in;
  CHK(stage_in(c, st->nonces, nonces, n * 16, &d_nonces));
  CHK(stage_in(c, st->pub, public_shares, n * g.public_share_len, &d_pub));
  const size_t in_len = st->agg_id == 0 ? g.leader_share_len : g.helper_share_len;
  CHK(stage_in(c, st->input, input_shares, (n - 1) * input_pitch(st) + in_len, &d_in));
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  if (is_f64(c))
    CHK(launch_prep_xof<Field64Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  else
    CHK(launch_prep_xof<Field128Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {nonces, public_shares, input_shares, status});
}

int prio3gpu_prepare_init_query(prio3gpu_ctx* c, prio3gpu_state* st, size_t n,
                                uint8_t* out_prep_shares, uint8_t* status) {
  CHK(check_state(c, st, n));
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(c->device));
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  if (is_f64(c))
    CHK(launch_prep_query<Field64Ops>(c, st, n, d_status));
  else
    CHK(launch_prep_query<Field128Ops>(c, st, n, d_status));
  CHK(copy_out(c, out_prep_shares, st->prep.p, n * c->cfg.prep_share_len));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {out_prep_shares, status});
}

int prio3gpu_prepare_init_weights(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, uint8_t* status) {
  CHK(check_state(c, st, n));
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(c->device));
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  if (is_f64(c))
    CHK(launch_prep_query<Field64Ops>(c, st, n, d_status, true));
  else
    CHK(launch_prep_query<Field128Ops>(c, st, n, d_status, true));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {status});
}

int prio3gpu_ctx_set_async(prio3gpu_ctx* c, int on) {
  if (!c) return PRIO3GPU_E_ARG;
  c->async_mode = on != 0;
  return 0;
}

int prio3gpu_ctx_set_option(prio3gpu_ctx* c, const char* name, int64_t value) {
  if (!c || !name) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  const std::string k(name);
  const bool on = value != 0;
  if (k == "speculate") {
    c->speculate = on;
  } else if (k == "fused_helper") {
    c->fused_helper = on;
  } else if (k == "spread_lds") {
    if (value < 16 * 1024 || value > 160 * 1024) {
      set_err("option spread_lds: %lld bytes is outside [16384, 163840]", (long long)value);
      return PRIO3GPU_E_ARG;
    }
    c->spread_lds = (size_t)value;
  } else if (k == "helper_snap") {
    c->helper_snap = on;
  } else if (k == "snap_chunk") {
    if (value < 1 || value > 65536) {
      set_err("option snap_chunk: %lld is outside [1, 65536]", (long long)value);
      return PRIO3GPU_E_ARG;
    }
    c->snap_chunk = (uint32_t)value;
  } else if (k == "spread") {
    c->spread = on;
  } else if (k == "jr_ring") {
    c->jr_ring = on;
  } else if (k == "query_overlap") {
    c->query_overlap = on;
  } else if (k == "chain_pairs") {
    if (value < 0 || value > 2) {
      set_err("option chain_pairs: %lld is not 0 (auto), 1 or 2", (long long)value);
      return PRIO3GPU_E_ARG;
    }
    c->chain_pairs = (uint32_t)value;
  } else if (k == "pair_chains") {
    c->pair_chains = on;
  } else if (k == "wires_mfma") {
    c->wires_mfma = on;
  } else if (k == "wires_cols") {
    c->wires_cols = on;

  } else if (k == "expand_lds" || k == "jr_lds") {
    if (value < 0 || value > 160 * 1024) {
      set_err("option %s: %lld bytes is outside [0, 163840]", name, (long long)value);
      return PRIO3GPU_E_ARG;
    }
    (k == "expand_lds" ? c->expand_lds : c->jr_lds) = (size_t)value;
  } else if (k == "wave_prio") {
    if (value < 0 || value > 2) {
      set_err("option wave_prio: %lld is not 0, 1 or 2", (long long)value);
      return PRIO3GPU_E_ARG;
    }
    c->cfg.wave_prio = (uint32_t)value;
  } else if (k == "exact_squeeze") {
    // every XOF squeeze takes the exact per-element rejection path (test switch); the FixedPoint
    // helper then runs its exact two-pass XOF
    c->cfg.exact_squeeze = on ? 1u : 0u;
  } else {
    set_err("unknown engine option \"%s\"", name);
    return PRIO3GPU_E_ARG;
  }
  c->plan_valid = false;
  return 0;
}

int prio3gpu_ctx_mark(prio3gpu_ctx* c, int* out_mark) {
  if (!c || !out_mark) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  constexpr int K = prio3gpu_ctx::kMarks;
  std::lock_guard<std::mutex> lk(c->mark_mu);
  const int k = c->ev_next;
  if (!c->ev[k]) HIPCHK(hipEventCreateWithFlags(&c->ev[k], hipEventDisableTiming));
  HIPCHK(hipEventRecord(c->ev[k], c->stream));
  c->ev_next = (k + 1) % K;
  const uint32_t gen = c->gen_next;
  c->gen_next = (gen + 1) & 0x07FFFFFFu ? (gen + 1) & 0x07FFFFFFu : 1u;  // mark stays a positive int
  c->ev_gen[k] = gen;
  *out_mark = (int)(gen * (uint32_t)K + (uint32_t)k);
  return 0;
}

int prio3gpu_ctx_wait_mark(prio3gpu_ctx* c, prio3gpu_ctx* other, int mark) {
  constexpr int K = prio3gpu_ctx::kMarks;
  if (!c || !other || mark < K) {
    set_err("bad mark");
    return PRIO3GPU_E_ARG;
  }
  const int k = mark % K;
  const uint32_t gen = (uint32_t)(mark / K);
  std::lock_guard<std::mutex> lk(other->mark_mu);
  if (!other->ev[k] || other->ev_gen[k] != gen) {
    set_err("stale mark %d: its ring slot was re-marked (more than %d newer marks)", mark, K);
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamWaitEvent(c->stream, other->ev[k], 0));
  return 0;
}

int prio3gpu_ctx_wait(prio3gpu_ctx* c, prio3gpu_ctx* other) {
  if (!c || !other) {
    set_err("null context");
    return PRIO3GPU_E_ARG;
  }
  if (c == other) return 0;
  // a private event of the waiting context, recorded on the other stream: the other context's
  // mark ring (marks its caller may still hold) is not touched.  An event can only be recorded on
  // a stream of its own device, so it lives on the other context's device (re-created when the
  // other context sits on a different device than last time); the wait itself works across devices.
  std::lock_guard<std::mutex> lk(c->mark_mu);
  if (c->wait_ev && c->wait_ev_dev != other->device) {
    (void)hipEventDestroy(c->wait_ev);
    c->wait_ev = nullptr;
  }
  HIPCHK(hipSetDevice(other->device));
  if (!c->wait_ev) {
    HIPCHK(hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming));
    c->wait_ev_dev = other->device;
  }
  HIPCHK(hipEventRecord(c->wait_ev, other->stream));
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamWaitEvent(c->stream, c->wait_ev, 0));
  return 0;
}

int prio3gpu_prepare_shares_to_prepare_message(prio3gpu_ctx* c, size_t n,
                                               const uint8_t* leader_prep_shares,
                                               const uint8_t* helper_prep_shares,
                                               uint8_t* out_prep_msgs, uint8_t* status) {
  if (!c || !leader_prep_shares || !helper_prep_shares) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  const uint8_t *d_l, *d_h;
  CHK(stage_in(c, c->io[0], leader_prep_shares, n * g.prep_share_len, &d_l));
  CHK(stage_in(c, c->io[1], helper_prep_shares, n * g.prep_share_len, &d_h));
  uint8_t* d_status;
  CHK(stage_status(c, c->io[2], status, n, &d_status));
  uint8_t* d_msg;
  if (out_prep_msgs && is_device_ptr(out_prep_msgs)) {
    d_msg = out_prep_msgs;
  } else {
    CHK(c->io[3].ensure(n * 16));
    d_msg = c->io[3].u8();
  }
  if (is_f64(c))
    CHK(launch_decide<Field64Ops>(c, n, d_l, d_h, d_msg, d_status));
  else
    CHK(launch_decide<Field128Ops>(c, n, d_l, d_h, d_msg, d_status));
  CHK(copy_out(c, out_prep_msgs, d_msg, n * g.prep_msg_len));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {leader_prep_shares, helper_prep_shares, out_prep_msgs, status});
}

int prio3gpu_prepare_next(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* prep_msgs,
                          uint8_t* status, uint8_t* out_output_shares, const uint32_t* batch_slots,
                          prio3gpu_agg* agg) {
  CHK(check_state(c, st, n));
  if (n == 0) return 0;
  if (n != st->n) {
    set_err("prepare_next over %zu reports but %zu were prepared", n, st->n);
    return PRIO3GPU_E_ARG;
  }
  if (agg && agg->ctx != c) {
    set_err("aggregate belongs to another context");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  if (g.jr_len) {
    if (!prep_msgs) {
      set_err("prep messages required");
      return PRIO3GPU_E_ARG;
    }
    const uint8_t* d_msgs;
    CHK(stage_in(c, c->io[4], prep_msgs, n * 16, &d_msgs));
    {
      PROF(KID_PNEXT);
      hipLaunchKernelGGL(k_prepare_next, grid1(n, 256), dim3(256), 0, c->stream, g, (uint32_t)n,
                         CRows{d_msgs, 16}, CRows{st->seed.u8(), 16}, d_status);
    }
    HIPCHK(hipGetLastError());
  }
  if (out_output_shares) {
    const size_t bytes = n * (size_t)g.out_len * g.es;
    uint8_t* d_out;
    if (is_device_ptr(out_output_shares)) {
      d_out = out_output_shares;
    } else {
      CHK(c->io[5].ensure(bytes));
      d_out = c->io[5].u8();
    }
    if (is_f64(c))
      CHK(out_shares_batch<Field64Ops>(c, st, n, d_status, d_out));
    else
      CHK(out_shares_batch<Field128Ops>(c, st, n, d_status, d_out));
    CHK(copy_out(c, out_output_shares, d_out, bytes));
  }
  if (agg) {
    if (is_f64(c))
      CHK(accumulate_batch<Field64Ops>(c, st, n, batch_slots, d_status, agg));
    else
      CHK(accumulate_batch<Field128Ops>(c, st, n, batch_slots, d_status, agg));
  }
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {prep_msgs, status, out_output_shares, batch_slots});
}

int prio3gpu_helper_init(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                         const uint8_t* public_shares, const uint8_t* helper_input_shares,
                         const uint8_t* leader_prep_shares, const uint32_t* batch_slots,
                         uint8_t* out_prep_msgs, uint8_t* status, prio3gpu_agg* agg) {
  CHK(check_state(c, st, n));
  if (st->agg_id != 1) {
    set_err("helper_init needs a helper (agg_id 1) state");
    return PRIO3GPU_E_ARG;
  }
  if (n == 0) return 0;
  if (!nonces || !helper_input_shares || !leader_prep_shares || (c->cfg.jr_len && !public_shares)) {
    set_err("null input");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  const uint8_t *d_nonces, *d_pub, *d_in, *d_lps;
  CHK(stage_in(c, st->nonces, nonces, n * 16, &d_nonces));
  CHK(stage_in(c, st->pub, public_shares, n * g.public_share_len, &d_pub));
  CHK(stage_in(c, st->input, helper_input_shares, (n - 1) * input_pitch(st) + g.helper_share_len,
               &d_in));
  CHK(stage_in(c, c->io[0], leader_prep_shares, n * g.prep_share_len, &d_lps));
  uint8_t* d_status;
  CHK(stage_status(c, st->status, status, n, &d_status));
  const bool f64 = is_f64(c);
  if (f64)
    CHK(launch_prepare_init<Field64Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  else
    CHK(launch_prepare_init<Field128Ops>(c, st, n, d_nonces, d_pub, d_in, d_status));
  uint8_t* d_msg = st->msg.u8();
  if (f64)
    CHK(launch_decide<Field64Ops>(c, n, d_lps, st->prep.u8(), d_msg, d_status));
  else
    CHK(launch_decide<Field128Ops>(c, n, d_lps, st->prep.u8(), d_msg, d_status));
  if (g.jr_len) {
    {
      PROF(KID_PNEXT);
      hipLaunchKernelGGL(k_prepare_next, grid1(n, 256), dim3(256), 0, c->stream, g, (uint32_t)n,
                         CRows{d_msg, 16}, CRows{st->seed.u8(), 16}, d_status);
    }
    HIPCHK(hipGetLastError());
  }
  if (agg) {
    if (f64)
      CHK(accumulate_batch<Field64Ops>(c, st, n, batch_slots, d_status, agg));
    else
      CHK(accumulate_batch<Field128Ops>(c, st, n, batch_slots, d_status, agg));
  }
  CHK(copy_out(c, out_prep_msgs, d_msg, n * g.prep_msg_len));
  CHK(copy_out(c, status, d_status, n));
  return finish_call(c, {nonces, public_shares, helper_input_shares, leader_prep_shares,
                         batch_slots, out_prep_msgs, status});
}

int prio3gpu_random_size(const prio3gpu_ctx* c) {
  if (!c) return PRIO3GPU_E_ARG;
  return 16 * (3 + (c->cfg.jr_len ? 2 : 0));
}

}  // extern "C"

namespace {
template <class FO>
int launch_shard(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* d_nonces,
                 const uint64_t* d_meas, uint32_t mw, const uint8_t* d_rand, uint8_t* d_pub,
                 uint8_t* d_leader, uint8_t* d_helper) {
  const Cfg& g = c->cfg;
  const uint32_t N = (uint32_t)n, es = g.es;
  const size_t rs = (size_t)prio3gpu_random_size(c);
  // scratch: helper meas/proof (state), proof + prove rand + jr (state buffers reused)
  CHK(st->meas.ensure(n * (size_t)g.meas_len * es));  // a snapshot-mode state has no rows yet
  st->snap_active = false;
  CHK(st->prep.ensure(n * (size_t)g.proof_len * es));       // full proof
  CHK(st->jr.ensure(n * (size_t)std::max<uint32_t>(g.prove_rand_len, 1) * es + n * 32));
  uint8_t* d_proof = st->prep.u8();
  uint8_t* d_prand = st->jr.u8();
  uint8_t* d_jr = d_prand + n * (size_t)std::max<uint32_t>(g.prove_rand_len, 1) * es;
  Rows helper{d_helper, g.helper_share_len}, leader{d_leader, g.leader_share_len};
  {
    PROF(KID_SHARD_SEEDS);
    hipLaunchKernelGGL(k_shard_seeds, grid1(n, 256), dim3(256), 0, c->stream, g, N,
                       CRows{d_rand, rs}, helper, leader);
  }
  Rows hm{st->meas.u8(), (size_t)g.meas_len * es}, hp{st->proof.u8(), (size_t)g.proof_len * es};
  {
    PROF(KID_EXPAND);
    hipLaunchKernelGGL(k_expand<FO>, grid1(n, 256), dim3(256), 0, c->stream, g, N, 1u,
                       CRows{d_helper, g.helper_share_len}, hm, hp, (const uint8_t*)nullptr);
  }
  uint64_t* d_norms = nullptr;  // FixedPointBoundedL2VecSum: squared norm per measurement
  if (g.kind == KIND_FPVEC) {
    CHK(c->io[5].ensure(n * 16));
    d_norms = reinterpret_cast<uint64_t*>(c->io[5].p);
    PROF(KID_SHARD_NORM);
    hipLaunchKernelGGL(k_shard_norm, dim3(N), dim3(256), 0, c->stream, g, N, d_meas, d_norms);
  }
  {
    PROF(KID_SHARD_MEAS);
    hipLaunchKernelGGL(k_shard_meas<FO>, dim3((g.meas_len + 255) / 256, N), dim3(256), 0,
                       c->stream, g, N, d_meas, mw, CRows{hm.base, hm.stride}, leader, d_norms);
  }
  {
    PROF(KID_SHARD_JR);
    hipLaunchKernelGGL(k_shard_jr<FO>, grid1(n, 256), dim3(256), 0, c->stream, g, N,
                       CRows{d_nonces, 16}, CRows{d_rand, rs}, CRows{hm.base, hm.stride},
                       CRows{d_leader, g.leader_share_len}, Rows{d_pub, g.public_share_len},
                       Rows{d_jr, 32}, Rows{d_prand, (size_t)std::max<uint32_t>(g.prove_rand_len, 1) * es});
  }
  {
    PROF(KID_PROVE);
    const uint32_t cc =
        (g.kind == KIND_SUMVEC || g.kind == KIND_HISTOGRAM || g.kind == KIND_FPVEC) ? g.chunk : 1u;
    const size_t lds = sizeof(typename FO::T) * (6 * (size_t)g.m + cc + 1 + g.calls + 1) + 16;
    if (lds > 160 * 1024) {
      set_err("prove LDS requirement %zu too large", lds);
      return PRIO3GPU_E_ARG;
    }
    hipLaunchKernelGGL(k_flp_prove<FO>, dim3(N), dim3(256), lds, c->stream, g, N,
                       c->twiddles2.u8(), d_meas, mw,
                       CRows{d_prand, (size_t)std::max<uint32_t>(g.prove_rand_len, 1) * es},
                       CRows{d_jr, 32}, Rows{d_proof, (size_t)g.proof_len * es}, d_norms);
  }
  {
    PROF(KID_SHARD_PROOF);
    hipLaunchKernelGGL(k_shard_proof<FO>, dim3((g.proof_len + 255) / 256, N), dim3(256), 0,
                       c->stream, g, N, CRows{d_proof, (size_t)g.proof_len * es},
                       CRows{hp.base, hp.stride}, leader);
  }
  HIPCHK(hipGetLastError());
  return 0;
}
}  // namespace

extern "C" {

int prio3gpu_shard(prio3gpu_ctx* c, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                   const uint64_t* measurements, const uint8_t* rand, uint8_t* out_public,
                   uint8_t* out_leader, uint8_t* out_helper) {
  CHK(check_state(c, st, n));
  if (st->agg_id != 1) {
    set_err("shard needs a helper-shaped (agg_id 1) state for scratch");
    return PRIO3GPU_E_ARG;
  }
  if (n == 0) return 0;
  if (!nonces || !measurements || !rand || !out_leader || !out_helper ||
      (c->cfg.jr_len && !out_public)) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  const uint32_t mw = (g.kind == KIND_SUMVEC || g.kind == KIND_FPVEC) ? g.length : 1u;
  const size_t rs = (size_t)prio3gpu_random_size(c);
  const uint8_t *d_nonces, *d_meas, *d_rand;
  CHK(stage_in(c, st->nonces, nonces, n * 16, &d_nonces));
  CHK(stage_in(c, st->pub, measurements, n * (size_t)mw * 8, &d_meas));
  CHK(stage_in(c, st->input, rand, n * rs, &d_rand));
  // outputs: device pointers written in place, host pointers staged
  uint8_t* d_out[3];
  void* host_out[3] = {out_public, out_leader, out_helper};
  const size_t out_len[3] = {n * g.public_share_len, n * (size_t)g.leader_share_len,
                             n * (size_t)g.helper_share_len};
  for (int i = 0; i < 3; ++i) {
    if (!host_out[i] || out_len[i] == 0) {
      d_out[i] = nullptr;
      continue;
    }
    if (is_device_ptr(host_out[i])) {
      d_out[i] = static_cast<uint8_t*>(host_out[i]);
    } else {
      CHK(c->io[i].ensure(out_len[i]));
      d_out[i] = c->io[i].u8();
    }
  }
  int rc;
  if (is_f64(c))
    rc = launch_shard<Field64Ops>(c, st, n, d_nonces, reinterpret_cast<const uint64_t*>(d_meas),
                                  mw, d_rand, d_out[0], d_out[1], d_out[2]);
  else
    rc = launch_shard<Field128Ops>(c, st, n, d_nonces, reinterpret_cast<const uint64_t*>(d_meas),
                                   mw, d_rand, d_out[0], d_out[1], d_out[2]);
  if (rc) return rc;
  for (int i = 0; i < 3; ++i)
    if (d_out[i] && d_out[i] != host_out[i]) CHK(copy_out(c, host_out[i], d_out[i], out_len[i]));
  HIPCHK(hipStreamSynchronize(c->stream));
  st->n = 0;  // scratch was used for sharding, not a prepared batch
  return 0;
}

int prio3gpu_comm_unique_id(uint8_t out_id[128]) {
  ncclUniqueId id;
  RCCLCHK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "unique id size");
  memcpy(out_id, &id, 128);
  return 0;
}

int prio3gpu_comm_init(const uint8_t id[128], int nranks, int rank, int device,
                       prio3gpu_comm** out) {
  HIPCHK(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, 128);
  auto* cm = new prio3gpu_comm();
  cm->nranks = nranks;
  cm->rank = rank;
  cm->device = device;
  if (hipEventCreateWithFlags(&cm->done, hipEventDisableTiming) != hipSuccess) {
    set_err("hipEventCreate failed");
    delete cm;
    return PRIO3GPU_E_HIP;
  }
  ncclResult_t e = ncclCommInitRank(&cm->comm, nranks, uid, rank);
  if (e != ncclSuccess) {
    set_err("ncclCommInitRank: %s", ncclGetErrorString(e));
    (void)hipEventDestroy(cm->done);
    delete cm;
    return PRIO3GPU_E_RCCL;
  }
  *out = cm;
  return 0;
}

int prio3gpu_comm_destroy(prio3gpu_comm* cm) {
  if (!cm) return 0;
  (void)hipSetDevice(cm->device);
  {
    std::lock_guard<std::mutex> lk(cm->mu);
    if (cm->done_valid) (void)hipEventSynchronize(cm->done);  // the last merge has read the scratch
  }
  cm->gather.release();
  cm->cgather.release();
  cm->mgather.release();
  if (cm->done) (void)hipEventDestroy(cm->done);
  if (cm->comm) ncclCommDestroy(cm->comm);
  delete cm;
  return 0;
}

int prio3gpu_agg_allreduce(prio3gpu_comm* cm, prio3gpu_ctx* c, prio3gpu_agg* local,
                           prio3gpu_agg* total) {
  if (!cm || !c || !local || local->ctx != c || (total && (total->ctx != c ||
                                                           total->slots != local->slots))) {
    set_err("bad argument");
    return PRIO3GPU_E_ARG;
  }
  if (c->device != cm->device) {
    set_err("context on device %d, communicator on device %d", c->device, cm->device);
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  std::lock_guard<std::mutex> lk(cm->mu);
  // the previous flush (any context) must have finished reading the shared scratch
  if (cm->done_valid) HIPCHK(hipStreamWaitEvent(c->stream, cm->done, 0));
  const size_t nel = (size_t)local->slots * c->cfg.out_len;
  const size_t bytes = nel * c->cfg.es;
  CHK(cm->gather.ensure(bytes * cm->nranks));
  CHK(cm->cgather.ensure((size_t)local->slots * 8));
  // all-gather the raw LE field-element bytes; counts: uint64 sum
  RCCLCHK(ncclAllGather(local->share.p, cm->gather.p, bytes, ncclUint8, cm->comm, c->stream));
  RCCLCHK(ncclAllReduce(local->counts.p, cm->cgather.p, local->slots, ncclUint64, ncclSum, cm->comm,
                        c->stream));
  // report-ID checksums (XOR) and client-timestamp intervals (min/max): RCCL has neither
  // reduction, so all-gather the slot meta and fold it in k_merge_ranks below
  const size_t mbytes = (size_t)local->slots * sizeof(SlotMeta);
  CHK(cm->mgather.ensure(mbytes * cm->nranks));
  RCCLCHK(ncclAllGather(local->meta.p, cm->mgather.p, mbytes, ncclUint8, cm->comm, c->stream));
  prio3gpu_agg* dst = total ? total : local;
  // ONE stream-ordered launch folds every rank, in rank order (identical on every rank; mod-p
  // addition is exact): dst = (total ? dst : 0) + sum_r share_r, counts likewise, and the slot
  // meta = BatchAggregation::merged_with's checksum XOR + interval union
  // (models.rs:962-991; core/src/time.rs:289-302).  No host round trip: in async mode the call
  // returns once queued, like every other all-device call.
  {
    PROF(KID_MERGE);
    const uint32_t nb = (uint32_t)std::min<size_t>((nel + 255) / 256, 4096);
    if (is_f64(c))
      hipLaunchKernelGGL(k_merge_ranks<Field64Ops>, dim3(nb + 1), dim3(256), 0, c->stream,
                         dst->share.u8(), cm->gather.u8(), nel, (uint32_t)cm->nranks,
                         total ? 1u : 0u, reinterpret_cast<unsigned long long*>(dst->counts.p),
                         reinterpret_cast<const unsigned long long*>(cm->cgather.p),
                         reinterpret_cast<SlotMeta*>(dst->meta.p),
                         reinterpret_cast<const SlotMeta*>(cm->mgather.p), local->slots, nb);
    else
      hipLaunchKernelGGL(k_merge_ranks<Field128Ops>, dim3(nb + 1), dim3(256), 0, c->stream,
                         dst->share.u8(), cm->gather.u8(), nel, (uint32_t)cm->nranks,
                         total ? 1u : 0u, reinterpret_cast<unsigned long long*>(dst->counts.p),
                         reinterpret_cast<const unsigned long long*>(cm->cgather.p),
                         reinterpret_cast<SlotMeta*>(dst->meta.p),
                         reinterpret_cast<const SlotMeta*>(cm->mgather.p), local->slots, nb);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(cm->done, c->stream));
  cm->done_valid = true;
  if (total) {  // the local partial has been merged: reset it for the next job (flush semantics)
    HIPCHK(hipMemsetAsync(local->share.p, 0, bytes, c->stream));
    HIPCHK(hipMemsetAsync(local->counts.p, 0, (size_t)local->slots * 8, c->stream));
    hipLaunchKernelGGL(k_meta_reset, dim3((local->slots + 255) / 256), dim3(256), 0, c->stream,
                       reinterpret_cast<SlotMeta*>(local->meta.p), local->slots);
    HIPCHK(hipGetLastError());
  }
  return finish_call(c, {});
}

int prio3gpu_agg_epoch_merge(prio3gpu_comm* cm, prio3gpu_ctx* c, prio3gpu_agg* local,
                             const uint32_t* slot_map, uint32_t union_slots, prio3gpu_agg* total) {
  if (!cm || !c || !local || !total || local->ctx != c || total->ctx != c ||
      total->slots != union_slots || union_slots == 0 || !slot_map) {
    set_err("epoch merge: bad argument");
    return PRIO3GPU_E_ARG;
  }
  std::vector<uint8_t> seen(union_slots, 0);
  for (uint32_t s = 0; s < local->slots; ++s) {
    if (slot_map[s] == PRIO3GPU_SLOT_UNUSED) continue;
    if (slot_map[s] >= union_slots || seen[slot_map[s]]++) {
      set_err("epoch merge: slot_map[%u] = %u is out of range or repeated", s, slot_map[s]);
      return PRIO3GPU_E_ARG;
    }
  }
  HIPCHK(hipSetDevice(c->device));
  // the partial laid out by the epoch's union slot table, identical on every rank
  prio3gpu_agg* stage = nullptr;
  CHK(prio3gpu_agg_create(c, union_slots, &stage));
  DevBuf dmap;
  int rc = dmap.ensure((size_t)local->slots * 4);
  if (rc == 0) rc = hipMemcpyAsync(dmap.p, slot_map, (size_t)local->slots * 4,
                                   hipMemcpyHostToDevice, c->stream) == hipSuccess
                        ? 0 : PRIO3GPU_E_HIP;
  if (rc == 0) {
    const size_t row_words = (size_t)c->cfg.out_len * c->cfg.es / 8;
    const uint32_t bx = (uint32_t)std::min<size_t>((row_words + 255) / 256, 64);
    hipLaunchKernelGGL(k_agg_scatter, dim3(bx, local->slots), dim3(256), 0, c->stream,
                       reinterpret_cast<uint64_t*>(stage->share.p),
                       reinterpret_cast<unsigned long long*>(stage->counts.p),
                       reinterpret_cast<SlotMeta*>(stage->meta.p),
                       reinterpret_cast<const uint64_t*>(local->share.p),
                       reinterpret_cast<const unsigned long long*>(local->counts.p),
                       reinterpret_cast<const SlotMeta*>(local->meta.p),
                       reinterpret_cast<const uint32_t*>(dmap.p), row_words);
    rc = hipGetLastError() == hipSuccess ? 0 : PRIO3GPU_E_HIP;
  }
  if (rc == 0) rc = prio3gpu_agg_allreduce(cm, c, stage, total);  // total += sum_r stage_r
  if (rc == 0) rc = prio3gpu_agg_reset(local);  // the epoch's partial is flushed
  // the staging buffers are freed only after the stream has used them
  const bool synced = hipStreamSynchronize(c->stream) == hipSuccess;
  prio3gpu_agg_destroy(stage);
  if (rc == 0 && !synced) {
    set_err("epoch merge: stream synchronisation failed");
    rc = PRIO3GPU_E_HIP;
  }
  return rc;
}

}  // extern "C"

namespace {
// Test-only: the XOF squeeze (SqueezeVec, the code every XOF kernel runs) over caller-crafted rate
// blocks -- blocks[25 i .. 25 i + 25) is the state after the i-th "permutation" -- so the exact
// rejection branches (non-canonical elements, the element straddling two Field128 blocks) run on
// inputs that real SHAKE128 output reaches with probability 28 / 2^64 per element.  One lane.
template <class FO>
__global__ void k_test_squeeze(const uint64_t* blocks, uint32_t nblocks, uint32_t n, uint8_t* out,
                               uint32_t exact, uint32_t* overrun) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t s[25];
  for (int i = 0; i < 25; ++i) s[i] = blocks[i];
  uint32_t b = 0;
  SqueezeVec<FO>::run(s, n, out, exact != 0u, [&](uint64_t st[25]) {
    ++b;
    const bool have = b < nblocks;
    for (int i = 0; i < 25; ++i) st[i] = have ? blocks[25 * (size_t)b + i] : 0ull;
    if (!have) *overrun = 1u;
  });
}
}  // namespace

extern "C" {

int prio3gpu_test_squeeze(int field_size, const uint64_t* blocks, size_t nblocks, uint32_t n,
                          uint8_t* out, int exact) {
  if ((field_size != 8 && field_size != 16) || !blocks || nblocks == 0 || (n && !out)) {
    set_err("test_squeeze: bad argument");
    return PRIO3GPU_E_ARG;
  }
  if (n == 0) return 0;
  void *d_blocks = nullptr, *d_out = nullptr, *d_over = nullptr;
  const size_t bb = nblocks * 25 * 8, ob = (size_t)n * field_size;
  int rc = 0;
  uint32_t over = 0;
  if (hipMalloc(&d_blocks, bb) != hipSuccess || hipMalloc(&d_out, ob) != hipSuccess ||
      hipMalloc(&d_over, 4) != hipSuccess) {
    set_err("test_squeeze: hipMalloc failed");
    rc = PRIO3GPU_E_HIP;
  }
  if (!rc && (hipMemcpy(d_blocks, blocks, bb, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemset(d_over, 0, 4) != hipSuccess || hipMemset(d_out, 0, ob) != hipSuccess)) {
    set_err("test_squeeze: copy failed");
    rc = PRIO3GPU_E_HIP;
  }
  if (!rc) {
    if (field_size == 16)
      hipLaunchKernelGGL(k_test_squeeze<Field128Ops>, dim3(1), dim3(64), 0, nullptr,
                         static_cast<const uint64_t*>(d_blocks), (uint32_t)nblocks, n,
                         static_cast<uint8_t*>(d_out), (uint32_t)(exact != 0),
                         static_cast<uint32_t*>(d_over));
    else
      hipLaunchKernelGGL(k_test_squeeze<Field64Ops>, dim3(1), dim3(64), 0, nullptr,
                         static_cast<const uint64_t*>(d_blocks), (uint32_t)nblocks, n,
                         static_cast<uint8_t*>(d_out), (uint32_t)(exact != 0),
                         static_cast<uint32_t*>(d_over));
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, d_out, ob, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&over, d_over, 4, hipMemcpyDeviceToHost) != hipSuccess) {
      set_err("test_squeeze: kernel failed");
      rc = PRIO3GPU_E_HIP;
    }
  }
  if (!rc && over) {
    set_err("test_squeeze: the squeeze needed more blocks than supplied");
    rc = PRIO3GPU_E_ARG;
  }
  if (d_blocks) (void)hipFree(d_blocks);
  if (d_out) (void)hipFree(d_out);
  if (d_over) (void)hipFree(d_over);
  return rc;
}

// Test-only: the FLP query phase of prepare_init over caller-supplied randomness.  Real query and
// joint randomness come out of SHAKE128, so the branches for a query point that is a root of unity
// (prio's "invalid query randomness", a VdafPrepError) and for a joint-rand element r with
// r^m == 1 (the closed-form gadget sum's degenerate case in k_flp_query_lane) are unreachable
// with real inputs; this entry runs launch_prep_query on crafted values so tests can compare them
// with the oracle's direct flp_query.
int prio3gpu_test_flp_query(prio3gpu_ctx* c, size_t n, const uint8_t* leader_input_shares,
                            const uint8_t* query_rand, const uint8_t* joint_rand,
                            const uint8_t* own_parts, uint8_t* out_prep_shares, uint8_t* status) {
  if (!c || !leader_input_shares || !query_rand || !own_parts || !status || n == 0 ||
      (c->cfg.jr_len && !joint_rand)) {
    set_err("test_flp_query: bad argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const Cfg& g = c->cfg;
  prio3gpu_state* st = nullptr;
  CHK(prio3gpu_state_create(c, 0, n, &st));
  int rc = 0;
  auto run = [&]() -> int {
    const size_t qr = (size_t)g.qr_len * g.es;
    CHK(st->input.ensure(n * g.leader_share_len));
    HIPCHK(hipMemcpyAsync(st->input.p, leader_input_shares, n * g.leader_share_len,
                          hipMemcpyDefault, c->stream));
    // query randomness rows have a 16-byte slot per element (k_query_rand's layout)
    std::vector<uint8_t> t(n * 16 * g.qr_len, 0);
    for (size_t r = 0; r < n; ++r)
      for (uint32_t i = 0; i < g.qr_len; ++i)
        memcpy(&t[r * 16 * g.qr_len + (size_t)i * g.es], query_rand + r * qr + (size_t)i * g.es,
               g.es);
    HIPCHK(hipMemcpyAsync(st->t.p, t.data(), t.size(), hipMemcpyHostToDevice, c->stream));
    if (g.jr_len)
      HIPCHK(hipMemcpyAsync(st->jr.p, joint_rand, n * (size_t)g.jr_len * g.es, hipMemcpyDefault,
                            c->stream));
    HIPCHK(hipMemcpyAsync(st->part.p, own_parts, n * 16, hipMemcpyDefault, c->stream));
    HIPCHK(hipMemcpyAsync(st->status.p, status, n, hipMemcpyDefault, c->stream));
    st->meas_rows = CRows{st->input.u8(), g.leader_share_len};
    st->proof_rows = CRows{st->input.u8() + (size_t)g.meas_len * g.es, g.leader_share_len};
    st->n = n;
    st->xof_done = true;
    if (is_f64(c))
      CHK(launch_prep_query<Field64Ops>(c, st, n, st->status.u8()));
    else
      CHK(launch_prep_query<Field128Ops>(c, st, n, st->status.u8()));
    CHK(copy_out(c, out_prep_shares, st->prep.p, n * g.prep_share_len));
    CHK(copy_out(c, status, st->status.p, n));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
  };
  rc = run();
  prio3gpu_state_destroy(st);
  return rc;
}

int prio3gpu_prof_enable(prio3gpu_ctx* c, int on) {
  if (!c) {
    set_err("null context");
    return PRIO3GPU_E_ARG;
  }
  c->prof.on = on != 0;
  return 0;
}

int prio3gpu_prof_read(prio3gpu_ctx* c, double* ms, uint64_t* launches, int max_kernels) {
  if (!c || !ms || !launches) {
    set_err("null argument");
    return PRIO3GPU_E_ARG;
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int i = 0; i < max_kernels; ++i) {
    ms[i] = 0.0;
    launches[i] = 0;
  }
  for (auto& r : c->prof.recs) {
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
    if (r.kid < max_kernels) {
      ms[r.kid] += t;
      launches[r.kid] += 1;
    }
    c->prof.pool.push_back(r.a);
    c->prof.pool.push_back(r.b);
  }
  c->prof.recs.clear();
  return std::min<int>(KID_COUNT, max_kernels);
}

const char* prio3gpu_prof_kernel_name(int kid) {
  return (kid >= 0 && kid < KID_COUNT) ? kKernelNames[kid] : "";
}

int prio3gpu_dev_alloc(prio3gpu_ctx* c, size_t bytes, void** out) {
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMalloc(out, bytes ? bytes : 16));
  return 0;
}
int prio3gpu_dev_free(prio3gpu_ctx* c, void* p) {
  (void)c;
  HIPCHK(hipFree(p));
  return 0;
}
int prio3gpu_memcpy(prio3gpu_ctx* c, void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"

/*
 * prio3gpu.h -- C ABI of the MI355X (gfx950) batched Prio3 preparation + aggregation engine.
 *
 * This is the drop-in boundary for Janus's leader/helper aggregate-init hot path.  The reference
 * (Janus 0.6, DAP-07) calls prio 0.15.1's `prio::vdaf::Aggregator` trait ONE REPORT AT A TIME:
 *
 *   trait Aggregator<16, 16>            (prio 0.15.1 src/vdaf.rs; surface mirrored by the fake VDAF
 *                                        at core/src/test_util/dummy_vdaf.rs:80-141)
 *     prepare_init(verify_key, agg_id, &(), nonce, public_share, input_share)
 *         -> (PrepareState, PrepareShare)                       -> prio3gpu_prepare_init
 *     prepare_shares_to_prepare_message(&(), [PrepareShare; 2])
 *         -> PrepareMessage                                     -> prio3gpu_prepare_shares_to_prepare_message
 *     prepare_next(PrepareState, PrepareMessage)
 *         -> PrepareTransition::Finish(OutputShare)             -> prio3gpu_prepare_next
 *     aggregate(&(), impl IntoIterator<OutputShare>) -> AggregateShare
 *   Aggregatable::{merge, accumulate}  (dummy_vdaf.rs:230-242)  -> prio3gpu_prepare_next(agg != NULL),
 *                                                                  prio3gpu_agg_merge_bytes
 *   Collector::unshard (collector/src/lib.rs:539)               -> prio3gpu_agg_read + host sum
 *
 * called from
 *   helper  aggregator/src/aggregator.rs:1775-1797   helper_initialized + evaluate + accumulate
 *                                                    -> prio3gpu_helper_init (fused, whole job)
 *   leader  aggregator/src/aggregator/aggregation_job_driver.rs:362-380   leader_initialized
 *                                                    -> prio3gpu_prepare_init(agg_id = 0)
 *           aggregation_job_driver.rs:579-627         leader_continued + accumulate
 *                                                    -> prio3gpu_prepare_next(agg != NULL)
 *   accumulate aggregator/src/aggregator/accumulator.rs:76-122  (per batch identifier)
 *   VDAF construction aggregator/src/aggregator.rs:797-840 (TaskAggregator::new)
 *                                                    -> prio3gpu_ctx_create
 *
 * Every batch entry point takes n reports.  Buffers hold the DAP/VDAF little-endian encodings,
 * report-major (report r at base + r * <len>).  They may be HOST or DEVICE pointers (detected);
 * device pointers avoid all PCIe traffic.  Errors never fail a whole batch for one report:
 * per-report status bytes mirror DAP `PrepareError` (messages/src/lib.rs:2288-2298):
 *   0 = ok, 3 = HpkeUnknownConfigId, 4 = HpkeDecryptError (HPKE stage), 5 = VdafPrepError,
 *   8 = InvalidMessage.  A report whose status is non-zero on entry to
 * a later stage is skipped by that stage (its outputs are left as zeros).
 * Return codes: 0 = ok, < 0 = API error (bad argument, HIP failure).
 *
 * Thread safety: one context may be used by one thread at a time; create one context per
 * concurrent job driver (each context owns its own HIP stream).
 */
#ifndef PRIO3GPU_H
#define PRIO3GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* VDAF kinds (VdafInstance, core/src/task.rs:24-59).  Prio3CountVec{length} is
 * SUMVEC with bits = 1 (aggregator.rs:805-813). */
enum prio3gpu_kind {
  PRIO3GPU_COUNT = 0,     /* Prio3Count                     Field64  */
  PRIO3GPU_SUM = 1,       /* Prio3Sum { bits }               Field128 */
  PRIO3GPU_SUMVEC = 2,    /* Prio3SumVec { bits, length, chunk_length }  Field128 */
  PRIO3GPU_HISTOGRAM = 3, /* Prio3Histogram { length, chunk_length }     Field128 */
  /* Prio3FixedPoint{16,32,64}BitBoundedL2VecSum { length } (core/src/task.rs:24-59,
   * aggregator.rs:839-861): bits = 16/32/64 (FixedI16<U15>/FixedI32<U31>/FixedI64<U63>),
   * length = entries; chunk_length is ignored (prio picks both gadgets' chunk lengths with
   * optimal_chunk_length).  Field128, algorithm ID 0xFFFF0000.  prio3gpu_shard takes the raw
   * two's-complement entries (see there). */
  PRIO3GPU_FPVEC = 4
};

enum prio3gpu_status {
  PRIO3GPU_OK = 0,
  PRIO3GPU_HPKE_UNKNOWN_CONFIG_ID = 3,
  PRIO3GPU_HPKE_DECRYPT_ERROR = 4,
  PRIO3GPU_VDAF_PREP_ERROR = 5,
  PRIO3GPU_INVALID_MESSAGE = 8
};

enum prio3gpu_err {
  PRIO3GPU_E_OK = 0,
  PRIO3GPU_E_ARG = -1,
  PRIO3GPU_E_HIP = -2,
  PRIO3GPU_E_RCCL = -3,
  PRIO3GPU_E_CAPACITY = -4,
  PRIO3GPU_E_HPKE = -5,        /* HPKE open/seal failed (bad key, tag mismatch) */
  PRIO3GPU_E_UNSUPPORTED = -6, /* HPKE suite not supported */
  /* The whole request is invalid (DAP "invalidMessage" for the request, not one report):
   * duplicate report IDs (aggregator.rs:1588-1598), an aggregation parameter that is not
   * Prio3's empty `()` (aggregator.rs:1605). */
  PRIO3GPU_E_INVALID_MESSAGE = -7
};

typedef struct prio3gpu_ctx prio3gpu_ctx;
typedef struct prio3gpu_state prio3gpu_state;
typedef struct prio3gpu_agg prio3gpu_agg;
typedef struct prio3gpu_comm prio3gpu_comm;

/* Sizes of the encodings for a configured context. */
typedef struct prio3gpu_sizes {
  uint32_t field_size;          /* 8 (Field64) or 16 (Field128) */
  uint32_t meas_len;            /* measurement-share length (field elements) */
  uint32_t proof_len;           /* proof-share length */
  uint32_t verifier_len;
  uint32_t joint_rand_len;
  uint32_t output_len;
  uint32_t leader_input_share;  /* bytes: meas || proof || [blind] */
  uint32_t helper_input_share;  /* bytes: meas seed || proof seed || [blind] */
  uint32_t public_share;        /* bytes: [part_0 || part_1] */
  uint32_t prep_share;          /* bytes: verifier || [part] */
  uint32_t prep_msg;            /* bytes: [joint rand seed] */
  uint32_t aggregate_share;     /* bytes: output_len * field_size */
} prio3gpu_sizes;

/* Prio3::new_{count,sum,sum_vec,histogram,fixedpoint_boundedl2_vec_sum}(2, ...) + verify key
 * (aggregator.rs:797-861).
 * `bits`, `length`, `chunk_length` are ignored where the kind does not use them.
 * `device` = HIP device ordinal. */
int prio3gpu_ctx_create(int kind, uint32_t bits, uint32_t length, uint32_t chunk_length,
                        const uint8_t verify_key[16], int device, prio3gpu_ctx** out);
/* The XOF behind every Prio3 stream of a context.  PRIO3GPU_XOF_SHAKE128 is prio 0.15.1's
 * XofShake128 (VDAF-07; what Janus 0.6 runs, aggregator/src/aggregator.rs:73) and the default of
 * prio3gpu_ctx_create.  PRIO3GPU_XOF_TURBOSHAKE128 is draft-irtf-cfrg-vdaf-08+'s
 * XofTurboShake128 (Keccak-p[1600, 12], domain byte 0x01) over the same message framing, with the
 * rest of Prio3 unchanged: a forward-compatibility mode, parity unpinned (no reference vectors). */
#define PRIO3GPU_XOF_SHAKE128 0
#define PRIO3GPU_XOF_TURBOSHAKE128 1
int prio3gpu_ctx_create2(int kind, uint32_t bits, uint32_t length, uint32_t chunk_length,
                         const uint8_t verify_key[16], int device, int xof, prio3gpu_ctx** out);
int prio3gpu_ctx_destroy(prio3gpu_ctx* ctx);
int prio3gpu_ctx_sizes(const prio3gpu_ctx* ctx, prio3gpu_sizes* out);
/* Wait for all work queued on the context's stream. */
int prio3gpu_ctx_sync(prio3gpu_ctx* ctx);
/* Async mode (default off): a call whose buffers are ALL device memory returns once its work is
 * queued on the context's stream instead of waiting for it (calls with any host buffer still
 * wait: their staging copies / results need it).  Lets a job driver queue job k+1 behind job k
 * (Janus runs aggregation jobs concurrently, aggregator/src/binary_utils/job_driver.rs:119-216);
 * order work across contexts with prio3gpu_ctx_wait and finish with prio3gpu_ctx_sync. */
int prio3gpu_ctx_set_async(prio3gpu_ctx* ctx, int on);
/* Engine options of a context (all default to the measured-fastest path; each alternative is
 * parity-tested against the oracle; value 0/1 for switches):
 *   "speculate"     1: accumulate from k_jr's per-wave column sums; 0: direct accumulation
 *   "wires_mfma"    1: SumVec (chunk > 64) wire pass on the matrix cores; 0: VALU k_flp_wires
 *   "wires_cols"    1: chunk <= 64 lane-per-column wire pass; 0: VALU k_flp_wires
 *   "fused_helper"  1: FixedPoint helper XOF pipeline (k_helper_xof); 0: exact two-pass path
 *   "helper_snap"   1: FixedPoint helper states (created after the call) keep 200-B sponge
 *                   snapshots of every 64th block instead of the expanded measurement share
 *                   (1/54 of its HBM); its rows are regenerated per chunk where they are read
 *                   (FLP query, accumulation past the column sums, output shares); 0: full rows
 *   "snap_chunk"    reports per FixedPoint query / regeneration chunk (default 512; the
 *                   regenerated rows of one chunk are the only full-size helper scratch)
 *   "query_overlap" 1 (default): the snapshot-mode helper query regenerates half-chunk i + 1 on a
 *                   second stream while half-chunk i is queried (two scratch halves); 0: in turn
 *   "wave_prio"     1: FixedPoint chain waves (k_helper_xof, k_jr_ring; the lane-pair kernels'
 *                   sponge waves only) issue at s_setprio 3 and the FixedPoint matrix-core wire
 *                   passes at 2 over co-running waves; 2: also the lane-pair kernels' storer /
 *                   loader waves; 0: all at 0
 *   "jr_ring"       1: FixedPoint leader joint-rand part via k_jr_ring; 0: k_jr
 *   "pair_chains"   1: the FixedPoint chains (k_helper_xof_pair, k_jr_ring_pair) keep each
 *                   sponge state on a lane pair, bit-interleaved (half the instructions on the
 *                   latency-bound chain; 64 / 128 reports per workgroup); 0: one lane per state
 *   "chain_pairs"   (pair_chains 0) 64-report chains per k_helper_xof / k_jr_ring workgroup: 1, 2, or 0 (auto,
 *                   default: 2 once the launch would take more than half the CUs, so a leader's
 *                   and a helper's launches side by side keep one sponge wave per SIMD)
 *   "spread"        1: latency-bound sponge launches take one CU per workgroup
 *   "spread_lds"    the dynamic LDS bytes that spreading requests (default 98304 = one workgroup
 *                   per CU; <= 81920 lets two, e.g. a leader's and a helper's, share a CU)
 *   "expand_lds", "jr_lds"  dynamic LDS bytes per k_expand / k_jr block (0 = none): caps those
 *                   kernels' occupancy so another context's kernels fit beside them
 *   "exact_squeeze" test switch: every XOF squeeze takes the exact per-element rejection path
 * The engine reads no environment variables.  PRIO3GPU_E_ARG for an unknown name. */
int prio3gpu_ctx_set_option(prio3gpu_ctx* ctx, const char* name, int64_t value);
/* Work queued on `ctx` from now on starts only after all work queued on `other` so far. */
int prio3gpu_ctx_wait(prio3gpu_ctx* ctx, prio3gpu_ctx* other);
/* The same in two steps: mark what is queued on `ctx` now; later make another context wait for
 * that mark.  Marks live in a ring of 16 per context, each carrying a generation: waiting on a mark
 * after 16 newer ones were taken fails with PRIO3GPU_E_ARG ("stale mark") instead of waiting on
 * newer work.  prio3gpu_ctx_wait uses a private event and takes no mark.  Marking and waiting are
 * thread-safe per context. */
int prio3gpu_ctx_mark(prio3gpu_ctx* ctx, int* out_mark);
int prio3gpu_ctx_wait_mark(prio3gpu_ctx* ctx, prio3gpu_ctx* other, int mark);
/* The context's HIP stream (hipStream_t), for callers that interoperate (e.g. bench timing). */
void* prio3gpu_ctx_stream(prio3gpu_ctx* ctx);

/* Preparation state + device scratch for up to `capacity` reports of one aggregator
 * (Prio3PrepareState for a whole batch).  Every buffer a call on the state can use is allocated
 * here, after checking the total against the device's free memory: a state the device cannot
 * hold is PRIO3GPU_E_CAPACITY (the message gives the bytes needed and free) with nothing
 * allocated, and calls on a created state do not allocate (except the FixedPoint helper's exact
 * path after a non-canonical squeezed element in snapshot mode, which allocates the full rows and
 * also reports a failure as PRIO3GPU_E_CAPACITY). */
int prio3gpu_state_create(prio3gpu_ctx* ctx, int agg_id, size_t capacity, prio3gpu_state** out);
int prio3gpu_state_destroy(prio3gpu_state* st);
/* Row pitch of the input shares this state's prepare_init / prepare_init_xof / helper_init calls
 * read: report i's input share at input_shares + i * pitch (0 = packed, the default: pitch = the
 * input share length).  A non-zero pitch is a multiple of 16 and >= the share length.  A caller
 * that decodes leader input shares (134,944 B for SumVec(8,1000)) into 128-B-aligned rows
 * (pitch 135,040) gives k_jr's LDS-DMA windows and the FLP wire pass line-aligned rows
 * (aggregator_core/src/datastore.rs:1298-1304 decodes each LeaderStoredReport's share). */
int prio3gpu_state_set_input_pitch(prio3gpu_state* st, size_t pitch);

/* Aggregate shares: `num_slots` batch identifiers (caller maps BatchIdentifier -> slot). */
int prio3gpu_agg_create(prio3gpu_ctx* ctx, uint32_t num_slots, prio3gpu_agg** out);
int prio3gpu_agg_destroy(prio3gpu_agg* agg);
int prio3gpu_agg_reset(prio3gpu_agg* agg);
/* Read one slot's aggregate share (aggregate_share bytes) and report count. */
int prio3gpu_agg_read(prio3gpu_agg* agg, uint32_t slot, uint8_t* out_share, uint64_t* out_count);
/* Aggregatable::merge: slot += share (aggregate_share bytes, host or device), count += count. */
int prio3gpu_agg_merge_bytes(prio3gpu_agg* agg, uint32_t slot, const uint8_t* share,
                             uint64_t count);

/* Accumulator::update's report bookkeeping (accumulator.rs:76-122): for every report whose status
 * is 0, slot checksum ^= SHA-256(report_id) (ReportIdChecksum, core/src/report_id.rs:18-44) and
 * the slot's client_timestamp_interval is merged with [time, time + 1) (core/src/time.rs:289-312).
 * report_ids n x 16, times n x u64 (seconds), status / batch_slots may be NULL (all ok / slot 0);
 * host or device pointers.  Call with the final statuses (after prepare_next / helper_init). */
int prio3gpu_agg_update_reports(prio3gpu_agg* agg, size_t n, const uint8_t* report_ids,
                                const uint64_t* times, const uint8_t* status,
                                const uint32_t* batch_slots);
/* The slot's ReportIdChecksum (32 bytes) and interval (start, duration; 0, 0 when empty). */
int prio3gpu_agg_read_reports(prio3gpu_agg* agg, uint32_t slot, uint8_t* out_checksum,
                              uint64_t* out_interval_start, uint64_t* out_interval_duration);

/* Collector::unshard (collector/src/lib.rs:539): sum `num_shares` aggregate shares
 * (num_shares x aggregate_share bytes, host) mod p and decode the aggregate result:
 *   Count / Sum / SumVec / Histogram -> out_u128: output_len x 16-byte LE integers;
 *   FixedPoint vectors               -> out_f64:  d * 2^(1-bits) - num_measurements per entry
 *                                                 (prio to_float_bits; interop FP16 KAT). */
int prio3gpu_unshard(const prio3gpu_ctx* ctx, const uint8_t* agg_shares, size_t num_shares,
                     uint64_t num_measurements, uint8_t* out_u128, double* out_f64);

/* prepare_init for n reports with the state's agg_id (0 = leader, 1 = helper).
 *   nonces          n x 16          (report IDs)
 *   public_shares   n x public_share
 *   input_shares    n x (agg_id == 0 ? leader_input_share : helper_input_share)
 *   out_prep_shares n x prep_share   (may be NULL: kept only inside the state)
 *   status          n bytes, in/out (initialise to 0)
 * The leader's input shares must stay valid (unchanged) until prio3gpu_prepare_next on the same
 * state when they are DEVICE pointers; host inputs are copied into the state. */
int prio3gpu_prepare_init(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                          const uint8_t* public_shares, const uint8_t* input_shares,
                          uint8_t* out_prep_shares, uint8_t* status);
/* prio3gpu_prepare_init in two phases over the same state and n: the XOF phase (query and joint
 * randomness, the helper's share expansion; VALU-bound Keccak) and the FLP-query phase (weights +
 * one HBM pass over the measurement shares).  prepare_init == xof then query.  Split so a driver
 * can overlap one batch's HBM-bound query with another batch's Keccak on a second context.  The
 * input buffers must stay valid until the query phase.  Count has no HBM-bound half: its XOF phase
 * runs the whole query (one kernel derives t and evaluates the FLP), and its query phase only
 * copies the prep shares out. */
int prio3gpu_prepare_init_xof(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n,
                              const uint8_t* nonces, const uint8_t* public_shares,
                              const uint8_t* input_shares, uint8_t* status);
/* Optional step between the two: the latency-bound first half of the FLP query (ParallelSum types:
 * k_flp_weights -- Lagrange weights, gadget poly at t, circuit output), so a scheduler can keep it
 * out from under another context's sponge kernels and overlap only the HBM-bound wire pass
 * (prio3gpu_prepare_init_query then runs just that).  A no-op for Count / Sum / FixedPoint. */
int prio3gpu_prepare_init_weights(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n, uint8_t* status);
int prio3gpu_prepare_init_query(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n,
                                uint8_t* out_prep_shares, uint8_t* status);

/* prepare_shares_to_prepare_message for n reports (leader share, helper share) -> prep msg. */
int prio3gpu_prepare_shares_to_prepare_message(prio3gpu_ctx* ctx, size_t n,
                                               const uint8_t* leader_prep_shares,
                                               const uint8_t* helper_prep_shares,
                                               uint8_t* out_prep_msgs, uint8_t* status);

/* prepare_next for the n reports prepared in `st`: check prep msg == corrected joint-rand seed;
 * optionally write output shares (n x aggregate_share bytes) and/or accumulate into `agg` at
 * `batch_slots[r]` (NULL slots = slot 0).  Reports with non-zero status are not accumulated. */
int prio3gpu_prepare_next(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n, const uint8_t* prep_msgs,
                          uint8_t* status, uint8_t* out_output_shares, const uint32_t* batch_slots,
                          prio3gpu_agg* agg);

/* Helper aggregate-init, fused (aggregator.rs:1613-1848 for a whole job): prepare_init(1) +
 * prepare_shares_to_prepare_message(leader share, own share) + prepare_next + accumulate.
 * Writes the prep msg each report's Finish message carries. */
int prio3gpu_helper_init(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                         const uint8_t* public_shares, const uint8_t* helper_input_shares,
                         const uint8_t* leader_prep_shares, const uint32_t* batch_slots,
                         uint8_t* out_prep_msgs, uint8_t* status, prio3gpu_agg* agg);

/* Client::shard for n reports (prio 0.15.1 shard_with_random; SURVEY §8(f) #1: batched client
 * shard + FLP prove, used to generate inputs at scale).
 *   measurements  n x (SUMVEC or FPVEC ? length : 1) u64 (Count 0/1, Sum value, SumVec entries,
 *                 Histogram bucket index, FixedPoint raw two's-complement entries whose L2 norm
 *                 is < 1 -- prio's shard rejects others; here they yield reports that fail
 *                 verification; client/src/lib.rs:212-258)
 *   rand          n x prio3gpu_random_size() bytes, prio order:
 *                 k_meas, k_proof, [blind_helper, blind_leader], k_prove
 *   outputs       public shares, leader input shares, helper input shares (DAP encodings)
 * `st` must be a helper (agg_id 1) state of sufficient capacity; it is used as scratch. */
int prio3gpu_random_size(const prio3gpu_ctx* ctx);
int prio3gpu_shard(prio3gpu_ctx* ctx, prio3gpu_state* st, size_t n, const uint8_t* nonces,
                   const uint64_t* measurements, const uint8_t* rand, uint8_t* out_public,
                   uint8_t* out_leader, uint8_t* out_helper);

/* BatchAggregation::merged_with (aggregator_core/src/datastore/models.rs:962-991) on host
 * buffers: the merge Janus applies to the batch-aggregation shards of a batch at collection
 * (aggregate_share.rs:47-65) and prio3gpu_agg_allreduce applies to the per-GPU partials.
 *   aggregate_share  dst += src elementwise mod p (Aggregatable::merge); output_len elements of
 *                    field_size (8: Field64, 16: Field128) canonical LE bytes; both NULL: skipped
 *   report_count     dst += src
 *   checksum         dst ^= src (ReportIdChecksum::combined_with, core/src/report_id.rs:18-44)
 *   interval         Interval::merge (core/src/time.rs:289-302): a zero-duration interval is
 *                    empty and yields the other; else [min start, max end).
 * Host only (no GPU).  PRIO3GPU_E_ARG on a non-canonical share element or interval overflow. */
typedef struct prio3gpu_batch_aggregation {
  uint8_t* aggregate_share;
  uint64_t report_count;
  uint8_t checksum[32];
  uint64_t interval_start, interval_duration;
} prio3gpu_batch_aggregation;
int prio3gpu_batch_aggregation_merge(uint32_t field_size, size_t output_len,
                                     prio3gpu_batch_aggregation* dst,
                                     const prio3gpu_batch_aggregation* src);

/* Multi-GPU merge of per-GPU partial aggregates (one process per GPU).  RCCL all-gather of the
 * raw field-element bytes over xGMI, then a mod-p add kernel (RCCL sum is neither modular nor
 * 128-bit).  Counts are summed with an RCCL uint64 all-reduce.
 * agg_allreduce: total += sum over ranks of local, then local is reset (the per-GPU partial of one
 * aggregation job is flushed into the running aggregate, like Accumulator::flush_to_datastore,
 * accumulator.rs:133-215).  With total == NULL, local is replaced by the sum over ranks.
 * agg_allreduce is a collective per call: every rank must issue its flushes on a communicator in
 * the same order with the same slot count.  Within a process the communicator serialises
 * concurrent contexts, but across processes nothing orders them -- concurrent job workers that
 * flush per job need one communicator each (or prio3gpu_agg_epoch_merge below, which keeps the
 * partials across jobs and merges once per epoch). */
int prio3gpu_comm_unique_id(uint8_t out_id[128]);
int prio3gpu_comm_init(const uint8_t id[128], int nranks, int rank, int device,
                       prio3gpu_comm** out);
int prio3gpu_comm_destroy(prio3gpu_comm* comm);
int prio3gpu_agg_allreduce(prio3gpu_comm* comm, prio3gpu_ctx* ctx, prio3gpu_agg* local,
                           prio3gpu_agg* total);

/* Epoch merge: the multi-GPU contract for independent job drivers.  Each GPU keeps its partial
 * aggregate across ANY number of jobs (its own slots, keyed by the batch identifiers it saw) and
 * the ranks merge once per epoch -- a collection boundary, as aggregate_share.rs:44-66 merges the
 * batch-aggregation shards -- instead of in lockstep per job:
 *   slot_map[s]   for each of local's slots, its index in the epoch's union slot table
 *                 (union_slots entries: the sorted union of every rank's batch identifiers,
 *                 agreed over the caller's host channel, the same on every rank); injective,
 *                 < union_slots, or PRIO3GPU_SLOT_UNUSED for a slot no job of the epoch used
 *   total         union_slots slots; total[slot_map[s]] += sum over ranks of local[s] (mod p,
 *                 counts, checksum XOR, interval union, folded in rank order), then local is reset
 * Ordering contract: a collective over `comm`.  Every rank calls it once per epoch with epochs in
 * the same order, from ONE thread per communicator, and no other flush (agg_allreduce) is in
 * flight on that communicator -- give each merger (task x aggregator role) its own communicator
 * or serialise them.  Synchronous: returns after the merge has completed on this rank. */
#define PRIO3GPU_SLOT_UNUSED 0xFFFFFFFFu
int prio3gpu_agg_epoch_merge(prio3gpu_comm* comm, prio3gpu_ctx* ctx, prio3gpu_agg* local,
                             const uint32_t* slot_map, uint32_t union_slots, prio3gpu_agg* total);

/* Per-kernel timing with HIP events on the context's stream (opt-in; bench.py uses it for the
 * live roofline numbers).  prof_read returns min(kernel ids, max_kernels) and fills, per kernel id,
 * the summed milliseconds and launch count since the last read. */
int prio3gpu_prof_enable(prio3gpu_ctx* ctx, int on);
int prio3gpu_prof_read(prio3gpu_ctx* ctx, double* ms, uint64_t* launches, int max_kernels);
const char* prio3gpu_prof_kernel_name(int kernel_id);

/* ---- DAP codec edge (host-only; janus_amd/csrc/codec.cpp) ------------------------------------
 * Batched decode/encode of the aggregate-init messages around the engine,
 * replacing the per-report Decode/Encode calls of the helper and leader loops:
 *   helper  AggregationJobInitializeReq::get_decoded   aggregator.rs:1561-1612 (request body)
 *           PlaintextInputShare::get_decoded + InputShare/PublicShare::get_decoded_with_param
 *                                                        aggregator.rs:1702-1768
 *           AggregationJobResp::get_encoded             aggregator.rs:1811-1848
 *   leader  AggregationJobInitializeReq::new + encode   aggregation_job_driver.rs:329-437
 *           AggregationJobResp::get_decoded             aggregation_job_driver.rs:530-600
 * Message layouts: messages/src/lib.rs (see codec.cpp).  Offsets are byte offsets into `msg`.
 * query_type: 1 = TimeInterval, 2 = FixedSize (lib.rs:2024-2028). */
typedef struct prio3gpu_prepare_init_view {
  uint64_t report_id_off;    /* 16-byte ReportId (= VDAF nonce) */
  uint64_t time;             /* ReportMetadata time, seconds since the epoch */
  uint64_t public_share_off;
  uint64_t enc_off;          /* HpkeCiphertext encapsulated key */
  uint64_t payload_off;      /* HpkeCiphertext payload */
  uint64_t prep_share_off;   /* PingPongMessage Initialize/Continue prep share */
  uint64_t prep_msg_off;     /* PingPongMessage Continue/Finish prep msg */
  uint32_t public_share_len, enc_len, payload_len, prep_share_len, prep_msg_len;
  uint8_t hpke_config_id;
  uint8_t message_type;      /* 0 Initialize, 1 Continue, 2 Finish */
} prio3gpu_prepare_init_view;

typedef struct prio3gpu_prepare_resp_view {
  uint64_t report_id_off;
  uint64_t prep_share_off, prep_msg_off;
  uint32_t prep_share_len, prep_msg_len;
  uint8_t result;            /* PrepareStepResult: 0 Continue, 1 Finished, 2 Reject */
  uint8_t message_type;      /* Continue: PingPongMessage type */
  uint8_t error;             /* Reject: PrepareError */
} prio3gpu_prepare_resp_view;

/* AggregationJobInitializeReq -> one view per PrepareInit.  views == NULL counts only.
 * out_agg_param (may be NULL) = {offset, length}; out_batch_id (FixedSize, may be NULL) 32 bytes.
 * A malformed request is PRIO3GPU_E_ARG (Janus rejects the whole request,
 * AggregationJobInitializeReq::get_decoded at aggregator.rs:1586). */
int prio3gpu_decode_agg_init_req(const uint8_t* msg, size_t len, int query_type,
                                 uint8_t* out_batch_id, uint64_t* out_agg_param,
                                 prio3gpu_prepare_init_view* views, size_t max_views,
                                 size_t* out_n);
/* Helper: the request-level checks handle_aggregate_init_generic makes after decoding, each
 * PRIO3GPU_E_INVALID_MESSAGE for the whole request:
 *   two PrepareInits with the same report ID           (aggregator.rs:1588-1598)
 *   an aggregation parameter other than Prio3's `()`   (aggregator.rs:1605: non-empty bytes). */
int prio3gpu_check_agg_init_req(const uint8_t* msg, const prio3gpu_prepare_init_view* views,
                                size_t n, uint64_t agg_param_len);
/* Helper: pack the engine inputs of n PrepareInits (nonces n x 16, public shares, leader prep
 * shares) and record each report's structural fault WITHOUT touching its status:
 *   faults[i] = 8 InvalidMessage  public share of the wrong length        (aggregator.rs:1755-1768)
 *             = 5 VdafPrepError   not Initialize{prep share of the right length}
 *                                 (ping-pong, aggregator.rs:1775-1797 / error.rs:240-300)
 *             = 0                 none.
 * Janus reaches these checks only after HPKE open (3 / 4) and the plaintext / input-share decode
 * (8) succeeded, so the caller applies faults to the reports whose status is still 0 after those
 * stages (prio3gpu_apply_faults).  Rows of faulty reports are zeroed. */
int prio3gpu_gather_prepare_inits(const prio3gpu_sizes* sizes, const uint8_t* msg,
                                  const prio3gpu_prepare_init_view* views, size_t n,
                                  uint8_t* nonces, uint8_t* public_shares,
                                  uint8_t* leader_prep_shares, uint8_t* faults);
/* status[i] = faults[i] for every report whose status is 0 (the precedence of the helper loop,
 * aggregator.rs:1663-1797: HPKE config / decrypt, plaintext + input-share decode, public-share
 * decode, ping-pong). */
int prio3gpu_apply_faults(size_t n, const uint8_t* faults, uint8_t* status);
/* HPKE-opened PlaintextInputShares (report i = plaintexts[offsets[i] .. offsets[i+1])) ->
 * n x input share (agg_id 0: leader, 1: helper).  Undecodable, duplicate extensions or wrong
 * payload length -> InvalidMessage.  status in/out. */
int prio3gpu_decode_plaintext_input_shares(const prio3gpu_sizes* sizes, const uint8_t* plaintexts,
                                           const uint64_t* offsets, size_t n, int agg_id,
                                           uint8_t* out_input_shares, uint8_t* status);
/* Helper: AggregationJobResp from the batch outputs: status 0 -> Continue{Finish{prep msg}},
 * otherwise Reject(status).  out == NULL (or too small) reports the length in out_len. */
int prio3gpu_encode_agg_job_resp(const uint8_t* nonces, const uint8_t* prep_msgs,
                                 uint32_t prep_msg_len, const uint8_t* status, size_t n,
                                 uint8_t* out, size_t cap, size_t* out_len);
/* Leader: AggregationJobInitializeReq for the reports whose status is 0 (status may be NULL):
 * ReportShare{id, time, public share, HpkeCiphertext{config id, enc, payload}} +
 * Initialize{leader prep share}.  Variable-length enc/payload use offset arrays (n + 1). */
int prio3gpu_encode_agg_init_req(int query_type, const uint8_t* batch_id, const uint8_t* agg_param,
                                 uint32_t agg_param_len, size_t n, const uint8_t* nonces,
                                 const uint64_t* times, const uint8_t* public_shares,
                                 uint32_t public_share_len, const uint8_t* hpke_config_ids,
                                 const uint8_t* encs, const uint64_t* enc_offsets,
                                 const uint8_t* payloads, const uint64_t* payload_offsets,
                                 const uint8_t* prep_shares, uint32_t prep_share_len,
                                 const uint8_t* status, uint8_t* out, size_t cap,
                                 size_t* out_len);
/* AggregationJobResp -> one view per PrepareResp (views == NULL counts only). */
int prio3gpu_decode_agg_job_resp(const uint8_t* msg, size_t len,
                                 prio3gpu_prepare_resp_view* views, size_t max_views,
                                 size_t* out_n);
/* Leader: match the helper's responses to the n reports it sent (status 0 ones, in order):
 * Continue{Finish{prep msg}} -> prep msg; Reject(e) -> status e; anything else -> VdafPrepError.
 * A response for an unexpected report ID is an API error (the job fails). */
int prio3gpu_gather_helper_resps(const prio3gpu_sizes* sizes, const uint8_t* msg,
                                 const prio3gpu_prepare_resp_view* views, size_t n_views,
                                 const uint8_t* nonces, size_t n, uint8_t* prep_msgs,
                                 uint8_t* status);

/* ---- HPKE open on host threads (janus_amd/csrc/hpke.cpp) -------------------
 * RFC 9180 base mode, single shot, as core/src/hpke.rs:158-202 (hpke::seal / hpke::open).
 * Suites: KEM 0x20 X25519HkdfSha256 | 0x10 P256HkdfSha256; KDF 1/2/3 HkdfSha256/384/512;
 * AEAD 1/2/3 Aes128Gcm/Aes256Gcm/ChaCha20Poly1305.  Keys are the RFC 9180 serializations
 * (X25519: 32 B; P-256: 32-B scalar, 65-B uncompressed point).
 * Returns 0, PRIO3GPU_E_HPKE (decryption / key failure), PRIO3GPU_E_UNSUPPORTED (suite),
 * PRIO3GPU_E_CAPACITY (out buffer too small; the needed length is stored), PRIO3GPU_E_ARG. */
typedef struct prio3gpu_hpke_keypair {  /* HpkeKeypair (core/src/hpke.rs:233-255) */
  uint8_t config_id;
  uint16_t kem_id, kdf_id, aead_id;
  const uint8_t* public_key;
  uint32_t public_key_len;
  const uint8_t* private_key;
  uint32_t private_key_len;
} prio3gpu_hpke_keypair;

int prio3gpu_hpke_open(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id, const uint8_t* sk,
                       size_t sk_len, const uint8_t* pk, size_t pk_len, const uint8_t* enc,
                       size_t enc_len, const uint8_t* info, size_t info_len, const uint8_t* aad,
                       size_t aad_len, const uint8_t* ct, size_t ct_len, uint8_t* pt, size_t cap,
                       size_t* pt_len);
/* sk_e = ephemeral private key (NULL: fresh random; fixed keys are for tests). */
int prio3gpu_hpke_seal(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id, const uint8_t* pk,
                       size_t pk_len, const uint8_t* sk_e, size_t sk_e_len, const uint8_t* info,
                       size_t info_len, const uint8_t* aad, size_t aad_len, const uint8_t* pt,
                       size_t pt_len, uint8_t* enc, size_t enc_cap, size_t* enc_len, uint8_t* ct,
                       size_t ct_cap, size_t* ct_len);
/* SerializePublicKey(pk(sk)) -- key generation (generate_hpke_config_and_private_key,
 * core/src/hpke.rs:204-231); PRIO3GPU_E_HPKE if sk is not a valid private key. */
int prio3gpu_hpke_public_key(uint16_t kem_id, const uint8_t* sk, size_t sk_len, uint8_t* pk,
                             size_t cap, size_t* pk_len);
/* out[i] = X25519(sk, points[i]) (RFC 7748 §5; the DH of the DHKEM Decap inside hpke::open,
 * core/src/hpke.rs:184-200) for n 32-byte points under ONE private key.  simd != 0 runs groups of
 * eight in the AVX-512 IFMA ladder the batched open uses (PRIO3GPU_E_UNSUPPORTED if the host CPU
 * lacks IFMA); simd == 0 is the scalar ladder.  Exposed so tests can check one against the other. */
int prio3gpu_x25519_batch(const uint8_t* sk, const uint8_t* points, size_t n, uint8_t* out,
                          int simd);
/* Helper: open the n encrypted input shares of a decoded AggregationJobInitializeReq on
 * `threads` host threads (<= 0: all cores), replacing the per-report hpke::open of
 * aggregator.rs:1634-1700: keypair by config id (task keys first, global keys on decryption
 * failure), info = "dap-07 input share" || sender_role || recipient_role, aad = InputShareAad
 * (task_id[32], report metadata, public share).  Unknown config id -> status 3
 * (HpkeUnknownConfigId), failure -> 4 (HpkeDecryptError); reports with status != 0 on entry are
 * skipped.  offsets (n + 1) are always filled: report i's plaintext (a PlaintextInputShare for
 * prio3gpu_decode_plaintext_input_shares) is plaintexts[offsets[i] .. offsets[i+1]);
 * plaintexts == NULL is a sizing call. */
int prio3gpu_hpke_open_report_shares(const uint8_t* task_id, const prio3gpu_hpke_keypair* task_keys,
                                     size_t n_task_keys, const prio3gpu_hpke_keypair* global_keys,
                                     size_t n_global_keys, uint8_t sender_role,
                                     uint8_t recipient_role, const uint8_t* msg,
                                     const prio3gpu_prepare_init_view* views, size_t n,
                                     uint8_t* plaintexts, uint64_t* offsets, uint8_t* status,
                                     int threads);

/* Last error message for this thread (static storage). */
const char* prio3gpu_last_error(void);
/* Build identity: the SHA-256 (hex) of the sources, headers and compiler flags the library was
 * built from ("unhashed" for a build outside janus_amd/_lib.py).  A caller (the Rust build.rs,
 * janus_amd/_lib.py) rejects a library whose hash is not that of the sources it ships with. */
const char* prio3gpu_build_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* PRIO3GPU_H */

//! Raw FFI to the MI355X batched Prio3 engine (`include/prio3gpu.h`, built by `build.rs` into
//! `libprio3gpu.so`).  Every `extern "C"` item here mirrors one declaration of the header, in the
//! header's order; `tests/test_rust_ffi.py` checks names, argument counts and the pointer /
//! integer width of every argument against the header mechanically.
//!
//! Replaces, per aggregation job (not per report), the `prio::vdaf::Aggregator` calls Janus makes
//! in its hot loops (prio 0.15.1, ext):
//!   helper  aggregator/src/aggregator.rs:1775-1797   -> prio3gpu_helper_init
//!   leader  aggregator/src/aggregator/aggregation_job_driver.rs:362-380 -> prio3gpu_prepare_init
//!           aggregation_job_driver.rs:579-627         -> prio3gpu_prepare_next
//!   accumulate aggregator/src/aggregator/accumulator.rs:76-122 (per batch identifier slot)
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

// ---- enums (header `enum prio3gpu_kind`, `prio3gpu_status`, `prio3gpu_err`) -------------------
/// VdafInstance (core/src/task.rs:24-59); Prio3CountVec{length} is SUMVEC with bits = 1.
pub const PRIO3GPU_COUNT: c_int = 0;
pub const PRIO3GPU_SUM: c_int = 1;
pub const PRIO3GPU_SUMVEC: c_int = 2;
pub const PRIO3GPU_HISTOGRAM: c_int = 3;
pub const PRIO3GPU_FPVEC: c_int = 4;

/// Per-report status bytes = DAP PrepareError (messages/src/lib.rs:2288-2298) + 0 = ok.
pub const PRIO3GPU_OK: u8 = 0;
pub const PRIO3GPU_HPKE_UNKNOWN_CONFIG_ID: u8 = 3;
pub const PRIO3GPU_HPKE_DECRYPT_ERROR: u8 = 4;
pub const PRIO3GPU_VDAF_PREP_ERROR: u8 = 5;
pub const PRIO3GPU_INVALID_MESSAGE: u8 = 8;

pub const PRIO3GPU_E_OK: c_int = 0;
pub const PRIO3GPU_E_ARG: c_int = -1;
pub const PRIO3GPU_E_HIP: c_int = -2;
pub const PRIO3GPU_E_RCCL: c_int = -3;
pub const PRIO3GPU_E_CAPACITY: c_int = -4;
pub const PRIO3GPU_E_HPKE: c_int = -5;
pub const PRIO3GPU_E_UNSUPPORTED: c_int = -6;
pub const PRIO3GPU_E_INVALID_MESSAGE: c_int = -7;

pub const PRIO3GPU_XOF_SHAKE128: c_int = 0;
pub const PRIO3GPU_XOF_TURBOSHAKE128: c_int = 1;
pub const PRIO3GPU_SLOT_UNUSED: u32 = 0xFFFF_FFFF;

// ---- opaque handles --------------------------------------------------------------------------
#[repr(C)]
pub struct prio3gpu_ctx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct prio3gpu_state {
    _p: [u8; 0],
}
#[repr(C)]
pub struct prio3gpu_agg {
    _p: [u8; 0],
}
#[repr(C)]
pub struct prio3gpu_comm {
    _p: [u8; 0],
}

// ---- structs ---------------------------------------------------------------------------------
#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct prio3gpu_sizes {
    pub field_size: u32,
    pub meas_len: u32,
    pub proof_len: u32,
    pub verifier_len: u32,
    pub joint_rand_len: u32,
    pub output_len: u32,
    pub leader_input_share: u32,
    pub helper_input_share: u32,
    pub public_share: u32,
    pub prep_share: u32,
    pub prep_msg: u32,
    pub aggregate_share: u32,
}

/// BatchAggregation::merged_with's operands (aggregator_core/src/datastore/models.rs:962-991).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct prio3gpu_batch_aggregation {
    pub aggregate_share: *mut u8,
    pub report_count: u64,
    pub checksum: [u8; 32],
    pub interval_start: u64,
    pub interval_duration: u64,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct prio3gpu_prepare_init_view {
    pub report_id_off: u64,
    pub time: u64,
    pub public_share_off: u64,
    pub enc_off: u64,
    pub payload_off: u64,
    pub prep_share_off: u64,
    pub prep_msg_off: u64,
    pub public_share_len: u32,
    pub enc_len: u32,
    pub payload_len: u32,
    pub prep_share_len: u32,
    pub prep_msg_len: u32,
    pub hpke_config_id: u8,
    pub message_type: u8,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct prio3gpu_prepare_resp_view {
    pub report_id_off: u64,
    pub prep_share_off: u64,
    pub prep_msg_off: u64,
    pub prep_share_len: u32,
    pub prep_msg_len: u32,
    pub result: u8,
    pub message_type: u8,
    pub error: u8,
}

/// HpkeKeypair (core/src/hpke.rs:233-255), borrowed key bytes.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct prio3gpu_hpke_keypair {
    pub config_id: u8,
    pub kem_id: u16,
    pub kdf_id: u16,
    pub aead_id: u16,
    pub public_key: *const u8,
    pub public_key_len: u32,
    pub private_key: *const u8,
    pub private_key_len: u32,
}

extern "C" {
    // -- context ------------------------------------------------------------------------------
    pub fn prio3gpu_ctx_create(kind: c_int, bits: u32, length: u32, chunk_length: u32,
                               verify_key: *const u8, device: c_int,
                               out: *mut *mut prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_ctx_create2(kind: c_int, bits: u32, length: u32, chunk_length: u32,
                                verify_key: *const u8, device: c_int, xof: c_int,
                                out: *mut *mut prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_ctx_destroy(ctx: *mut prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_ctx_sizes(ctx: *const prio3gpu_ctx, out: *mut prio3gpu_sizes) -> c_int;
    pub fn prio3gpu_ctx_sync(ctx: *mut prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_ctx_set_async(ctx: *mut prio3gpu_ctx, on: c_int) -> c_int;
    pub fn prio3gpu_ctx_set_option(ctx: *mut prio3gpu_ctx, name: *const c_char, value: i64)
                                   -> c_int;
    pub fn prio3gpu_ctx_wait(ctx: *mut prio3gpu_ctx, other: *mut prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_ctx_mark(ctx: *mut prio3gpu_ctx, out_mark: *mut c_int) -> c_int;
    pub fn prio3gpu_ctx_wait_mark(ctx: *mut prio3gpu_ctx, other: *mut prio3gpu_ctx,
                                  mark: c_int) -> c_int;
    pub fn prio3gpu_ctx_stream(ctx: *mut prio3gpu_ctx) -> *mut c_void;

    // -- preparation state and aggregates -----------------------------------------------------
    pub fn prio3gpu_state_create(ctx: *mut prio3gpu_ctx, agg_id: c_int, capacity: usize,
                                 out: *mut *mut prio3gpu_state) -> c_int;
    pub fn prio3gpu_state_destroy(st: *mut prio3gpu_state) -> c_int;
    pub fn prio3gpu_state_set_input_pitch(st: *mut prio3gpu_state, pitch: usize) -> c_int;
    pub fn prio3gpu_agg_create(ctx: *mut prio3gpu_ctx, num_slots: u32,
                               out: *mut *mut prio3gpu_agg) -> c_int;
    pub fn prio3gpu_agg_destroy(agg: *mut prio3gpu_agg) -> c_int;
    pub fn prio3gpu_agg_reset(agg: *mut prio3gpu_agg) -> c_int;
    pub fn prio3gpu_agg_read(agg: *mut prio3gpu_agg, slot: u32, out_share: *mut u8,
                             out_count: *mut u64) -> c_int;
    pub fn prio3gpu_agg_merge_bytes(agg: *mut prio3gpu_agg, slot: u32, share: *const u8,
                                    count: u64) -> c_int;
    pub fn prio3gpu_agg_update_reports(agg: *mut prio3gpu_agg, n: usize, report_ids: *const u8,
                                       times: *const u64, status: *const u8,
                                       batch_slots: *const u32) -> c_int;
    pub fn prio3gpu_agg_read_reports(agg: *mut prio3gpu_agg, slot: u32, out_checksum: *mut u8,
                                     out_interval_start: *mut u64,
                                     out_interval_duration: *mut u64) -> c_int;
    pub fn prio3gpu_unshard(ctx: *const prio3gpu_ctx, agg_shares: *const u8, num_shares: usize,
                            num_measurements: u64, out_u128: *mut u8, out_f64: *mut f64) -> c_int;

    // -- the Aggregator trait, batched ----------------------------------------------------------
    pub fn prio3gpu_prepare_init(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                                 nonces: *const u8, public_shares: *const u8,
                                 input_shares: *const u8, out_prep_shares: *mut u8,
                                 status: *mut u8) -> c_int;
    pub fn prio3gpu_prepare_init_xof(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                                     nonces: *const u8, public_shares: *const u8,
                                     input_shares: *const u8, status: *mut u8) -> c_int;
    pub fn prio3gpu_prepare_init_weights(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                                         status: *mut u8) -> c_int;
    pub fn prio3gpu_prepare_init_query(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state,
                                       n: usize, out_prep_shares: *mut u8,
                                       status: *mut u8) -> c_int;
    pub fn prio3gpu_prepare_shares_to_prepare_message(ctx: *mut prio3gpu_ctx, n: usize,
                                                      leader_prep_shares: *const u8,
                                                      helper_prep_shares: *const u8,
                                                      out_prep_msgs: *mut u8,
                                                      status: *mut u8) -> c_int;
    pub fn prio3gpu_prepare_next(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                                 prep_msgs: *const u8, status: *mut u8,
                                 out_output_shares: *mut u8, batch_slots: *const u32,
                                 agg: *mut prio3gpu_agg) -> c_int;
    pub fn prio3gpu_helper_init(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                                nonces: *const u8, public_shares: *const u8,
                                helper_input_shares: *const u8, leader_prep_shares: *const u8,
                                batch_slots: *const u32, out_prep_msgs: *mut u8,
                                status: *mut u8, agg: *mut prio3gpu_agg) -> c_int;

    // -- client shard (input generation at scale) ---------------------------------------------
    pub fn prio3gpu_random_size(ctx: *const prio3gpu_ctx) -> c_int;
    pub fn prio3gpu_shard(ctx: *mut prio3gpu_ctx, st: *mut prio3gpu_state, n: usize,
                          nonces: *const u8, measurements: *const u64, rand: *const u8,
                          out_public: *mut u8, out_leader: *mut u8, out_helper: *mut u8) -> c_int;

    // -- batch aggregation merge (host) and the multi-GPU merge --------------------------------
    pub fn prio3gpu_batch_aggregation_merge(field_size: u32, output_len: usize,
                                            dst: *mut prio3gpu_batch_aggregation,
                                            src: *const prio3gpu_batch_aggregation) -> c_int;
    pub fn prio3gpu_comm_unique_id(out_id: *mut u8) -> c_int;
    pub fn prio3gpu_comm_init(id: *const u8, nranks: c_int, rank: c_int, device: c_int,
                              out: *mut *mut prio3gpu_comm) -> c_int;
    pub fn prio3gpu_comm_destroy(comm: *mut prio3gpu_comm) -> c_int;
    pub fn prio3gpu_agg_allreduce(comm: *mut prio3gpu_comm, ctx: *mut prio3gpu_ctx,
                                  local: *mut prio3gpu_agg, total: *mut prio3gpu_agg) -> c_int;
    pub fn prio3gpu_agg_epoch_merge(comm: *mut prio3gpu_comm, ctx: *mut prio3gpu_ctx,
                                    local: *mut prio3gpu_agg, slot_map: *const u32,
                                    union_slots: u32, total: *mut prio3gpu_agg) -> c_int;

    // -- profiling (the test hooks of include/prio3gpu_test.h are not bound) -------------------
    pub fn prio3gpu_prof_enable(ctx: *mut prio3gpu_ctx, on: c_int) -> c_int;
    pub fn prio3gpu_prof_read(ctx: *mut prio3gpu_ctx, ms: *mut f64, launches: *mut u64,
                              max_kernels: c_int) -> c_int;
    pub fn prio3gpu_prof_kernel_name(kernel_id: c_int) -> *const c_char;

    // -- DAP codec edge (host) ----------------------------------------------------------------
    pub fn prio3gpu_decode_agg_init_req(msg: *const u8, len: usize, query_type: c_int,
                                        out_batch_id: *mut u8, out_agg_param: *mut u64,
                                        views: *mut prio3gpu_prepare_init_view,
                                        max_views: usize, out_n: *mut usize) -> c_int;
    pub fn prio3gpu_check_agg_init_req(msg: *const u8, views: *const prio3gpu_prepare_init_view,
                                       n: usize, agg_param_len: u64) -> c_int;
    pub fn prio3gpu_gather_prepare_inits(sizes: *const prio3gpu_sizes, msg: *const u8,
                                         views: *const prio3gpu_prepare_init_view, n: usize,
                                         nonces: *mut u8, public_shares: *mut u8,
                                         leader_prep_shares: *mut u8, faults: *mut u8) -> c_int;
    pub fn prio3gpu_apply_faults(n: usize, faults: *const u8, status: *mut u8) -> c_int;
    pub fn prio3gpu_decode_plaintext_input_shares(sizes: *const prio3gpu_sizes,
                                                  plaintexts: *const u8, offsets: *const u64,
                                                  n: usize, agg_id: c_int,
                                                  out_input_shares: *mut u8,
                                                  status: *mut u8) -> c_int;
    pub fn prio3gpu_encode_agg_job_resp(nonces: *const u8, prep_msgs: *const u8,
                                        prep_msg_len: u32, status: *const u8, n: usize,
                                        out: *mut u8, cap: usize, out_len: *mut usize) -> c_int;
    pub fn prio3gpu_encode_agg_init_req(query_type: c_int, batch_id: *const u8,
                                        agg_param: *const u8, agg_param_len: u32, n: usize,
                                        nonces: *const u8, times: *const u64,
                                        public_shares: *const u8, public_share_len: u32,
                                        hpke_config_ids: *const u8, encs: *const u8,
                                        enc_offsets: *const u64, payloads: *const u8,
                                        payload_offsets: *const u64, prep_shares: *const u8,
                                        prep_share_len: u32, status: *const u8, out: *mut u8,
                                        cap: usize, out_len: *mut usize) -> c_int;
    pub fn prio3gpu_decode_agg_job_resp(msg: *const u8, len: usize,
                                        views: *mut prio3gpu_prepare_resp_view,
                                        max_views: usize, out_n: *mut usize) -> c_int;
    pub fn prio3gpu_gather_helper_resps(sizes: *const prio3gpu_sizes, msg: *const u8,
                                        views: *const prio3gpu_prepare_resp_view,
                                        n_views: usize, nonces: *const u8, n: usize,
                                        prep_msgs: *mut u8, status: *mut u8) -> c_int;

    // -- HPKE on host threads -----------------------------------------------------------------
    pub fn prio3gpu_hpke_open(kem_id: u16, kdf_id: u16, aead_id: u16, sk: *const u8,
                              sk_len: usize, pk: *const u8, pk_len: usize, enc: *const u8,
                              enc_len: usize, info: *const u8, info_len: usize, aad: *const u8,
                              aad_len: usize, ct: *const u8, ct_len: usize, pt: *mut u8,
                              cap: usize, pt_len: *mut usize) -> c_int;
    pub fn prio3gpu_hpke_seal(kem_id: u16, kdf_id: u16, aead_id: u16, pk: *const u8,
                              pk_len: usize, sk_e: *const u8, sk_e_len: usize, info: *const u8,
                              info_len: usize, aad: *const u8, aad_len: usize, pt: *const u8,
                              pt_len: usize, enc: *mut u8, enc_cap: usize, enc_len: *mut usize,
                              ct: *mut u8, ct_cap: usize, ct_len: *mut usize) -> c_int;
    pub fn prio3gpu_hpke_public_key(kem_id: u16, sk: *const u8, sk_len: usize, pk: *mut u8,
                                    cap: usize, pk_len: *mut usize) -> c_int;
    pub fn prio3gpu_x25519_batch(sk: *const u8, points: *const u8, n: usize, out: *mut u8,
                                 simd: c_int) -> c_int;
    pub fn prio3gpu_hpke_open_report_shares(task_id: *const u8,
                                            task_keys: *const prio3gpu_hpke_keypair,
                                            n_task_keys: usize,
                                            global_keys: *const prio3gpu_hpke_keypair,
                                            n_global_keys: usize, sender_role: u8,
                                            recipient_role: u8, msg: *const u8,
                                            views: *const prio3gpu_prepare_init_view, n: usize,
                                            plaintexts: *mut u8, offsets: *mut u64,
                                            status: *mut u8, threads: c_int) -> c_int;

    // -- errors and build identity ------------------------------------------------------------
    pub fn prio3gpu_last_error() -> *const c_char;
    pub fn prio3gpu_build_hash() -> *const c_char;
}

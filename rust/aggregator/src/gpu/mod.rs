//! `aggregator/src/gpu`: the MI355X engine behind Janus's Prio3 aggregate-init path.
//!
//! Not compiled in this image (no cargo/rustc); written against `include/prio3gpu.h` through
//! `ffi.rs`, whose declarations `tests/test_rust_ffi.py` checks against the header.  This module
//! is what the `mi355x` cargo feature adds to Janus 0.6:
//!
//! * `GpuPrio3` -- one engine context (= one HIP stream) per concurrent job-driver worker
//!   (aggregator/src/binary_utils/job_driver.rs:119-216 runs jobs concurrently; a context is used
//!   by one thread at a time).
//! * `GpuVdafOps::Prio3SumVec` -- the batched arm next to `VdafOps::Prio3SumVec`
//!   (aggregator/src/aggregator.rs:1040-1065): where `handle_aggregate_init_generic`
//!   (aggregator.rs:1561-2045) calls `vdaf.helper_initialized(..).evaluate(vdaf)` once per report
//!   (:1775-1797) and then `accumulator.update` (:1811-1819), the arm makes ONE
//!   `prio3gpu_helper_init` call for the whole job, then one `prio3gpu_agg_update_reports`.
//!   The leader's `step_aggregation_job_aggregate_init` (aggregation_job_driver.rs:290-437) and
//!   `process_response_from_helper` (:530-727) become one `prio3gpu_prepare_init` and one
//!   `prio3gpu_prepare_next` per job.
//! * Per-report errors keep Janus's mapping (error.rs:240-300): status 5 -> VdafPrepError,
//!   8 -> InvalidMessage, 3/4 -> the HPKE errors; a batch call never fails a job for one report.
pub mod ffi;

use std::ffi::CStr;
use std::ptr;

/// An engine error (an API failure, not a per-report status).
#[derive(Debug, Clone)]
pub struct GpuError {
    pub code: i32,
    pub message: String,
}

fn check(rc: i32) -> Result<(), GpuError> {
    if rc == 0 {
        return Ok(());
    }
    // SAFETY: prio3gpu_last_error returns a NUL-terminated thread-local string.
    let message = unsafe { CStr::from_ptr(ffi::prio3gpu_last_error()) }
        .to_string_lossy()
        .into_owned();
    Err(GpuError { code: rc, message })
}

/// The library this binary links must be the one built from the sources it ships with.
pub fn check_build(expected_hash: &str) -> Result<(), GpuError> {
    // SAFETY: static NUL-terminated string.
    let got = unsafe { CStr::from_ptr(ffi::prio3gpu_build_hash()) }.to_string_lossy();
    if got != expected_hash {
        return Err(GpuError { code: ffi::PRIO3GPU_E_ARG,
                              message: format!("libprio3gpu build {got} != {expected_hash}") });
    }
    Ok(())
}

/// One engine context: the Prio3 instance of a task (`Prio3::new_*(2, ..)` + verify key,
/// TaskAggregator::new, aggregator.rs:797-861) on one GPU and one HIP stream.
pub struct GpuPrio3 {
    ctx: *mut ffi::prio3gpu_ctx,
    pub sizes: ffi::prio3gpu_sizes,
}

// A context is moved between tokio blocking threads but never used by two at once.
unsafe impl Send for GpuPrio3 {}

impl GpuPrio3 {
    /// Prio3SumVec { bits, length, chunk_length } (core/src/task.rs:24-59; chunk_length =
    /// VdafInstance::chunk_size(bits * length), core/src/task.rs:84-86).
    pub fn new_sum_vec(bits: u32, length: u32, chunk_length: u32, verify_key: &[u8; 16],
                       device: i32) -> Result<Self, GpuError> {
        Self::new(ffi::PRIO3GPU_SUMVEC, bits, length, chunk_length, verify_key, device)
    }

    pub fn new(kind: i32, bits: u32, length: u32, chunk_length: u32, verify_key: &[u8; 16],
               device: i32) -> Result<Self, GpuError> {
        let mut ctx = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_ctx_create(kind, bits, length, chunk_length,
                                                verify_key.as_ptr(), device, &mut ctx) })?;
        let mut sizes = ffi::prio3gpu_sizes::default();
        check(unsafe { ffi::prio3gpu_ctx_sizes(ctx, &mut sizes) })?;
        Ok(Self { ctx, sizes })
    }

    pub fn new_state(&self, agg_id: i32, capacity: usize) -> Result<PrepareState, GpuError> {
        let mut st = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_state_create(self.ctx, agg_id, capacity, &mut st) })?;
        Ok(PrepareState { st })
    }

    /// One aggregate per batch identifier of the job (Accumulator's
    /// HashMap<BatchIdentifier, BatchAggregation>, accumulator.rs:26-122).
    pub fn new_aggregate(&self, slots: u32) -> Result<AggregateShares, GpuError> {
        let mut agg = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_agg_create(self.ctx, slots, &mut agg) })?;
        Ok(AggregateShares { agg, share_len: self.sizes.aggregate_share as usize })
    }

    /// Helper aggregate-init for a whole job (aggregator.rs:1613-1848): prepare_init(1) +
    /// prepare_shares_to_prepare_message + prepare_next + accumulate into `agg`, then the
    /// report-ID checksum / client-timestamp interval bookkeeping of Accumulator::update.
    /// `status` arrives holding the HPKE / decode outcomes (0 = ok) and leaves with the final
    /// per-report PrepareError codes.  Returns the prep messages of the Finish replies.
    #[allow(clippy::too_many_arguments)]
    pub fn helper_init(&self, st: &mut PrepareState, nonces: &[u8], public_shares: &[u8],
                       helper_input_shares: &[u8], leader_prep_shares: &[u8],
                       report_times: &[u64], batch_slots: &[u32], status: &mut [u8],
                       agg: &mut AggregateShares) -> Result<Vec<u8>, GpuError> {
        let n = status.len();
        assert_eq!(nonces.len(), n * 16);
        assert_eq!(public_shares.len(), n * self.sizes.public_share as usize);
        assert_eq!(helper_input_shares.len(), n * self.sizes.helper_input_share as usize);
        assert_eq!(leader_prep_shares.len(), n * self.sizes.prep_share as usize);
        assert!(batch_slots.len() == n && report_times.len() == n);
        let mut msgs = vec![0u8; n * self.sizes.prep_msg as usize];
        check(unsafe {
            ffi::prio3gpu_helper_init(self.ctx, st.st, n, nonces.as_ptr(), public_shares.as_ptr(),
                                      helper_input_shares.as_ptr(), leader_prep_shares.as_ptr(),
                                      batch_slots.as_ptr(), msgs.as_mut_ptr(), status.as_mut_ptr(),
                                      agg.agg)
        })?;
        check(unsafe {
            ffi::prio3gpu_agg_update_reports(agg.agg, n, nonces.as_ptr(), report_times.as_ptr(),
                                             status.as_ptr(), batch_slots.as_ptr())
        })?;
        Ok(msgs)
    }

    /// Leader `leader_initialized` for a whole job (aggregation_job_driver.rs:329-402): the prep
    /// shares for the PingPongMessage::Initialize messages; the state stays on the GPU until
    /// `leader_continued`.
    pub fn leader_init(&self, st: &mut PrepareState, nonces: &[u8], public_shares: &[u8],
                       leader_input_shares: &[u8], status: &mut [u8])
                       -> Result<Vec<u8>, GpuError> {
        let n = status.len();
        assert_eq!(leader_input_shares.len(), n * self.sizes.leader_input_share as usize);
        let mut prep = vec![0u8; n * self.sizes.prep_share as usize];
        check(unsafe {
            ffi::prio3gpu_prepare_init(self.ctx, st.st, n, nonces.as_ptr(), public_shares.as_ptr(),
                                       leader_input_shares.as_ptr(), prep.as_mut_ptr(),
                                       status.as_mut_ptr())
        })?;
        Ok(prep)
    }

    /// Leader `leader_continued` + accumulate (aggregation_job_driver.rs:566-686) once the
    /// helper's Finish{prep_msg} replies are gathered (prio3gpu_gather_helper_resps).
    pub fn leader_finish(&self, st: &mut PrepareState, prep_msgs: &[u8], nonces: &[u8],
                         report_times: &[u64], batch_slots: &[u32], status: &mut [u8],
                         agg: &mut AggregateShares) -> Result<(), GpuError> {
        let n = status.len();
        check(unsafe {
            ffi::prio3gpu_prepare_next(self.ctx, st.st, n, prep_msgs.as_ptr(), status.as_mut_ptr(),
                                       ptr::null_mut(), batch_slots.as_ptr(), agg.agg)
        })?;
        check(unsafe {
            ffi::prio3gpu_agg_update_reports(agg.agg, n, nonces.as_ptr(), report_times.as_ptr(),
                                             status.as_ptr(), batch_slots.as_ptr())
        })
    }
}

impl Drop for GpuPrio3 {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_ctx_destroy(self.ctx) };
    }
}

/// Prio3PrepareState of a whole job (device scratch: the helper's expanded shares, the
/// verifier pieces, the corrected joint-rand seeds).  Reused across jobs: creating one allocates
/// device memory.
pub struct PrepareState {
    st: *mut ffi::prio3gpu_state,
}
unsafe impl Send for PrepareState {}
impl Drop for PrepareState {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_state_destroy(self.st) };
    }
}

/// Per-slot aggregate shares + BatchAggregation bookkeeping of a job, flushed like
/// `Accumulator::flush_to_datastore` (accumulator.rs:133-215).
pub struct AggregateShares {
    agg: *mut ffi::prio3gpu_agg,
    share_len: usize,
}
unsafe impl Send for AggregateShares {}

/// One slot as Janus stores it in `batch_aggregations` (models.rs:843-991).
pub struct SlotAggregation {
    pub aggregate_share: Vec<u8>,
    pub report_count: u64,
    pub checksum: [u8; 32],
    pub interval_start: u64,
    pub interval_duration: u64,
}

impl AggregateShares {
    pub fn read(&self, slot: u32) -> Result<SlotAggregation, GpuError> {
        let mut s = SlotAggregation { aggregate_share: vec![0u8; self.share_len], report_count: 0,
                                      checksum: [0u8; 32], interval_start: 0,
                                      interval_duration: 0 };
        check(unsafe { ffi::prio3gpu_agg_read(self.agg, slot, s.aggregate_share.as_mut_ptr(),
                                              &mut s.report_count) })?;
        check(unsafe { ffi::prio3gpu_agg_read_reports(self.agg, slot, s.checksum.as_mut_ptr(),
                                                      &mut s.interval_start,
                                                      &mut s.interval_duration) })?;
        Ok(s)
    }

    pub fn reset(&mut self) -> Result<(), GpuError> {
        check(unsafe { ffi::prio3gpu_agg_reset(self.agg) })
    }
}
impl Drop for AggregateShares {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_agg_destroy(self.agg) };
    }
}

/// The batched arm a Janus build with the `mi355x` feature adds beside `VdafOps`
/// (aggregator.rs:1040-1065).  `TaskAggregator::new` (aggregator.rs:797-900) builds it next to
/// the CPU `Prio3SumVecMultithreaded`; `VdafOps::handle_aggregate_init` (aggregator.rs:1230-1274)
/// routes `VdafInstance::Prio3SumVec { .. }` here when a GPU is configured, everything else keeps
/// the reference's per-report path.
pub enum GpuVdafOps {
    Prio3SumVec { engine: std::sync::Mutex<GpuPrio3>, state: std::sync::Mutex<PrepareState> },
}

/// What `handle_aggregate_init_generic` needs from one job, after it has decoded the request,
/// checked it (duplicate IDs, aggregation parameter: aggregator.rs:1588-1605), opened the HPKE
/// ciphertexts and decoded the plaintext input shares (:1634-1768) -- all on CPU threads.
pub struct HelperJob<'a> {
    pub nonces: &'a [u8],
    pub public_shares: &'a [u8],
    pub helper_input_shares: &'a [u8],
    pub leader_prep_shares: &'a [u8],
    pub report_times: &'a [u64],
    /// index of `Q::to_batch_identifier(..)` per report (aggregator.rs:1615-1631)
    pub batch_slots: &'a [u32],
    pub slot_count: u32,
}

impl GpuVdafOps {
    /// The per-report loop of aggregator.rs:1613-1848 for a whole job.  Returns the prep messages
    /// (status 0 -> PrepareStepResult::Continue{Finish{prep_msg}}, else Reject(status)) and the
    /// per-slot aggregations the datastore transaction (:1889-2044) writes.
    pub fn helper_aggregate_init(&self, job: &HelperJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, Vec<SlotAggregation>), GpuError> {
        match self {
            GpuVdafOps::Prio3SumVec { engine, state } => {
                let engine = engine.lock().unwrap();
                let mut state = state.lock().unwrap();
                let mut agg = engine.new_aggregate(job.slot_count)?;
                let msgs = engine.helper_init(&mut state, job.nonces, job.public_shares,
                                              job.helper_input_shares, job.leader_prep_shares,
                                              job.report_times, job.batch_slots, status,
                                              &mut agg)?;
                let slots = (0..job.slot_count).map(|s| agg.read(s))
                    .collect::<Result<Vec<_>, _>>()?;
                Ok((msgs, slots))
            }
        }
    }
}

//! `aggregator/src/gpu`: the MI355X engine behind Janus's Prio3 aggregate-init path.
//!
//! Not compiled in this image (no cargo/rustc); written against `include/prio3gpu.h` through
//! `ffi.rs`, whose declarations `tests/test_rust_ffi.py` checks against the header (and this
//! file's `ffi::` calls against the header's argument counts).  This module is what the `mi355x`
//! cargo feature adds to Janus 0.6:
//!
//! * `GpuPrio3` -- one engine context (= one HIP stream) of a task's Prio3 instance on one GPU.
//! * `GpuTask` -- a pool of contexts, one per concurrent job-driver worker
//!   (aggregator/src/binary_utils/job_driver.rs:119-216 runs jobs concurrently), each with its
//!   preparation states and aggregates allocated once and reused: creating a state or aggregate
//!   allocates device memory, and freeing it (`hipFree`) waits for the whole device.
//! * `GpuVdafOps` -- the batched arms next to `VdafOps` (aggregator/src/aggregator.rs:1040-1065),
//!   one per Prio3 instance Janus dispatches (Count, CountVec, Sum, SumVec, Histogram,
//!   FixedPoint{16,32,64}BitBoundedL2VecSum); Poplar1 and the fake VDAFs keep the reference's
//!   per-report path.
//!   - helper: where `handle_aggregate_init_generic` (aggregator.rs:1561-2045) calls
//!     `vdaf.helper_initialized(..).evaluate(vdaf)` once per report (:1775-1797) and then
//!     `accumulator.update` (:1811-1819), the arm makes ONE `prio3gpu_helper_init` call for the
//!     whole job, then one `prio3gpu_agg_update_reports`;
//!   - leader: `step_aggregation_job_aggregate_init` (aggregation_job_driver.rs:290-437) becomes
//!     one `prio3gpu_prepare_init(agg_id 0)` per job, returning a `LeaderPending` that holds the
//!     job's device state across the HTTP round trip; `process_response_from_helper`
//!     (:530-727) becomes one `prio3gpu_prepare_next` + accumulate on it.
//! * Per-report errors keep Janus's mapping (error.rs:240-300): status 5 -> VdafPrepError,
//!   8 -> InvalidMessage, 3/4 -> the HPKE errors; a batch call never fails a job for one report.
//!
//! The Janus call sites themselves (construction in `TaskAggregator`, the helper's loop, the
//! leader's job driver, the `gpu:` config sections) are `rust/patches/janus-0.6-mi355x.patch`; the
//! adapters they use (`GpuConfig`, `HelperBatch`, `LeaderBatch`, `LeaderFinishBatch`, `SlotMap`,
//! `GpuTaskCache`, `status_of` / `prepare_error`) are at the end of this file.
pub mod ffi;

use std::collections::HashMap;
use std::ffi::{c_int, CStr};
use std::hash::Hash;
use std::ptr;
use std::sync::atomic::{AtomicUsize, Ordering};
use std::sync::{Arc, Mutex, MutexGuard};

use janus_core::task::VdafInstance;
use janus_messages::PrepareError;
use prio::topology::ping_pong::PingPongMessage;
use serde::{Deserialize, Serialize};

/// An engine error (an API failure, not a per-report status).
#[derive(Debug, Clone)]
pub struct GpuError {
    pub code: i32,
    pub message: String,
}

impl std::fmt::Display for GpuError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "mi355x engine error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for GpuError {}

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

fn arg_error(message: String) -> GpuError {
    GpuError { code: ffi::PRIO3GPU_E_ARG, message }
}

/// The library this binary links must be the one built from the sources it ships with
/// (`env!("PRIO3GPU_BUILD_HASH")`, set by build.rs).
pub fn check_build(expected_hash: &str) -> Result<(), GpuError> {
    // SAFETY: static NUL-terminated string.
    let got = unsafe { CStr::from_ptr(ffi::prio3gpu_build_hash()) }.to_string_lossy();
    if got != expected_hash {
        return Err(arg_error(format!("libprio3gpu build {got} != {expected_hash}")));
    }
    Ok(())
}

/// The engine's parameters of a Prio3 instance: `prio3gpu_ctx_create`'s (kind, bits, length,
/// chunk_length), chosen exactly as `TaskAggregator::new` constructs the CPU VDAF
/// (aggregator.rs:797-861; chunk length `VdafInstance::chunk_size`, core/src/task.rs:84-86).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct EngineParams {
    pub kind: c_int,
    pub bits: u32,
    pub length: u32,
    pub chunk_length: u32,
}

/// `None` for the instances the engine does not run (Poplar1, the fake VDAFs): those keep the
/// reference's per-report path.
pub fn engine_params(vdaf: &VdafInstance) -> Option<EngineParams> {
    let p = |kind, bits: usize, length: usize, chunk: usize| EngineParams {
        kind,
        bits: bits as u32,
        length: length as u32,
        chunk_length: chunk as u32,
    };
    match vdaf {
        VdafInstance::Prio3Count => Some(p(ffi::PRIO3GPU_COUNT, 0, 0, 0)),
        // Prio3::new_sum_vec_multithreaded(2, 1, length, chunk_size(length)) (aggregator.rs:805-813)
        VdafInstance::Prio3CountVec { length } => Some(p(
            ffi::PRIO3GPU_SUMVEC,
            1,
            *length,
            VdafInstance::chunk_size(*length),
        )),
        VdafInstance::Prio3Sum { bits } => Some(p(ffi::PRIO3GPU_SUM, *bits, 0, 0)),
        VdafInstance::Prio3SumVec { bits, length } => Some(p(
            ffi::PRIO3GPU_SUMVEC,
            *bits,
            *length,
            VdafInstance::chunk_size(*bits * *length),
        )),
        VdafInstance::Prio3Histogram { length } => Some(p(
            ffi::PRIO3GPU_HISTOGRAM,
            0,
            *length,
            VdafInstance::chunk_size(*length),
        )),
        // new_fixedpoint_boundedl2_vec_sum_multithreaded(2, length) over FixedI16<U15> /
        // FixedI32<U31> / FixedI64<U63> (aggregator.rs:839-861); the engine picks both gadgets'
        // chunk lengths like prio's optimal_chunk_length
        #[cfg(feature = "fpvec_bounded_l2")]
        VdafInstance::Prio3FixedPoint16BitBoundedL2VecSum { length } => {
            Some(p(ffi::PRIO3GPU_FPVEC, 16, *length, 0))
        }
        #[cfg(feature = "fpvec_bounded_l2")]
        VdafInstance::Prio3FixedPoint32BitBoundedL2VecSum { length } => {
            Some(p(ffi::PRIO3GPU_FPVEC, 32, *length, 0))
        }
        #[cfg(feature = "fpvec_bounded_l2")]
        VdafInstance::Prio3FixedPoint64BitBoundedL2VecSum { length } => {
            Some(p(ffi::PRIO3GPU_FPVEC, 64, *length, 0))
        }
        _ => None,
    }
}

/// One engine context: the Prio3 instance of a task (`Prio3::new_*(2, ..)` + verify key,
/// TaskAggregator::new, aggregator.rs:797-861) on one GPU and one HIP stream.
pub struct GpuPrio3 {
    ctx: *mut ffi::prio3gpu_ctx,
    pub sizes: ffi::prio3gpu_sizes,
    kind: c_int,
}

// A context is moved between tokio blocking threads but never used by two at once (GpuTask
// hands each out behind a Mutex).
unsafe impl Send for GpuPrio3 {}

impl GpuPrio3 {
    pub fn new(params: EngineParams, verify_key: &[u8; 16], device: i32) -> Result<Self, GpuError> {
        let mut ctx = ptr::null_mut();
        check(unsafe {
            ffi::prio3gpu_ctx_create(params.kind, params.bits, params.length, params.chunk_length,
                                     verify_key.as_ptr(), device, &mut ctx)
        })?;
        let mut sizes = ffi::prio3gpu_sizes::default();
        if let Err(e) = check(unsafe { ffi::prio3gpu_ctx_sizes(ctx, &mut sizes) }) {
            unsafe { ffi::prio3gpu_ctx_destroy(ctx) };
            return Err(e);
        }
        Ok(Self { ctx, sizes, kind: params.kind })
    }

    /// `Collector::unshard` (collector/src/lib.rs:539-543): the sum of the aggregators' aggregate
    /// shares mod p, decoded as the instance's aggregate result -- integers for Count, Sum, SumVec
    /// and Histogram, `d * 2^(1-bits) - num_measurements` per entry for the fixed-point vectors.
    pub fn unshard(&self, aggregate_shares: &[&[u8]], num_measurements: u64)
                   -> Result<AggregateResult, GpuError> {
        let len = self.sizes.aggregate_share as usize;
        if aggregate_shares.is_empty() || aggregate_shares.iter().any(|a| a.len() != len) {
            return Err(arg_error(format!("unshard: {} shares of {len} bytes expected",
                                         aggregate_shares.len())));
        }
        let joined = aggregate_shares.concat();
        let out_len = self.sizes.output_len as usize;
        if self.kind == ffi::PRIO3GPU_FPVEC {
            let mut out = vec![0f64; out_len];
            check(unsafe {
                ffi::prio3gpu_unshard(self.ctx, joined.as_ptr(), aggregate_shares.len(),
                                      num_measurements, ptr::null_mut(), out.as_mut_ptr())
            })?;
            Ok(AggregateResult::FixedPoint(out))
        } else {
            let mut out = vec![0u8; out_len * 16];
            check(unsafe {
                ffi::prio3gpu_unshard(self.ctx, joined.as_ptr(), aggregate_shares.len(),
                                      num_measurements, out.as_mut_ptr(), ptr::null_mut())
            })?;
            Ok(AggregateResult::Integers(
                out.chunks_exact(16).map(|c| u128::from_le_bytes(c.try_into().unwrap())).collect(),
            ))
        }
    }

    pub fn new_state(&self, agg_id: i32, capacity: usize) -> Result<PrepareState, GpuError> {
        let mut st = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_state_create(self.ctx, agg_id, capacity, &mut st) })?;
        Ok(PrepareState { st, capacity })
    }

    /// One aggregate slot per batch identifier of the job (Accumulator's
    /// HashMap<BatchIdentifier, BatchAggregation>, accumulator.rs:26-122).
    pub fn new_aggregate(&self, slots: u32) -> Result<AggregateShares, GpuError> {
        let mut agg = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_agg_create(self.ctx, slots, &mut agg) })?;
        Ok(AggregateShares { agg, slots, share_len: self.sizes.aggregate_share as usize })
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
        let s = &self.sizes;
        if nonces.len() != n * 16
            || public_shares.len() != n * s.public_share as usize
            || helper_input_shares.len() != n * s.helper_input_share as usize
            || leader_prep_shares.len() != n * s.prep_share as usize
            || batch_slots.len() != n
            || report_times.len() != n
        {
            return Err(arg_error("helper_init: buffer lengths do not match the job".into()));
        }
        st.fits(n)?;
        agg.fits(batch_slots)?;
        let mut msgs = vec![0u8; n * s.prep_msg as usize];
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
    /// shares for the PingPongMessage::Initialize messages; the state (output shares, corrected
    /// joint-rand seeds) stays on the GPU until `leader_finish`.
    pub fn leader_init(&self, st: &mut PrepareState, nonces: &[u8], public_shares: &[u8],
                       leader_input_shares: &[u8], status: &mut [u8])
                       -> Result<Vec<u8>, GpuError> {
        let n = status.len();
        let s = &self.sizes;
        if nonces.len() != n * 16
            || public_shares.len() != n * s.public_share as usize
            || leader_input_shares.len() != n * s.leader_input_share as usize
        {
            return Err(arg_error("leader_init: buffer lengths do not match the job".into()));
        }
        st.fits(n)?;
        let mut prep = vec![0u8; n * s.prep_share as usize];
        check(unsafe {
            ffi::prio3gpu_prepare_init(self.ctx, st.st, n, nonces.as_ptr(), public_shares.as_ptr(),
                                       leader_input_shares.as_ptr(), prep.as_mut_ptr(),
                                       status.as_mut_ptr())
        })?;
        Ok(prep)
    }

    /// Leader `leader_continued` + accumulate (aggregation_job_driver.rs:566-686) once the
    /// helper's Finish{prep_msg} replies are gathered (prio3gpu_gather_helper_resps, which also
    /// folds the helper's Reject codes into `status`).
    #[allow(clippy::too_many_arguments)]
    pub fn leader_finish(&self, st: &mut PrepareState, prep_msgs: &[u8], nonces: &[u8],
                         report_times: &[u64], batch_slots: &[u32], status: &mut [u8],
                         agg: &mut AggregateShares) -> Result<(), GpuError> {
        let n = status.len();
        if prep_msgs.len() != n * self.sizes.prep_msg as usize
            || nonces.len() != n * 16
            || report_times.len() != n
            || batch_slots.len() != n
        {
            return Err(arg_error("leader_finish: buffer lengths do not match the job".into()));
        }
        agg.fits(batch_slots)?;
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
/// verifier pieces, the corrected joint-rand seeds).  Pooled by GpuTask.
pub struct PrepareState {
    st: *mut ffi::prio3gpu_state,
    capacity: usize,
}
unsafe impl Send for PrepareState {}
impl PrepareState {
    fn fits(&self, n: usize) -> Result<(), GpuError> {
        if n > self.capacity {
            return Err(arg_error(format!("job of {n} reports > state capacity {}", self.capacity)));
        }
        Ok(())
    }
}
impl Drop for PrepareState {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_state_destroy(self.st) };
    }
}

/// Per-slot aggregate shares + BatchAggregation bookkeeping of a job, flushed like
/// `Accumulator::flush_to_datastore` (accumulator.rs:133-215).  Pooled by GpuTask: `reset`
/// after the slots are read.
pub struct AggregateShares {
    agg: *mut ffi::prio3gpu_agg,
    slots: u32,
    share_len: usize,
}
unsafe impl Send for AggregateShares {}

/// One slot as Janus stores it in `batch_aggregations` (models.rs:843-991).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct SlotAggregation {
    pub aggregate_share: Vec<u8>,
    pub report_count: u64,
    pub checksum: [u8; 32],
    pub interval_start: u64,
    pub interval_duration: u64,
}

impl AggregateShares {
    fn fits(&self, batch_slots: &[u32]) -> Result<(), GpuError> {
        match batch_slots.iter().max() {
            Some(&m) if m >= self.slots => {
                Err(arg_error(format!("batch slot {m} >= the aggregate's {} slots", self.slots)))
            }
            _ => Ok(()),
        }
    }

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

    /// The job's slots, then zeroed for the next job (one flush per job, accumulator.rs:133-215).
    pub fn take(&mut self, slot_count: u32) -> Result<Vec<SlotAggregation>, GpuError> {
        let out = (0..slot_count).map(|s| self.read(s)).collect::<Result<Vec<_>, _>>()?;
        self.reset()?;
        Ok(out)
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

/// One job-driver worker's engine: a context plus its pooled device objects.
struct Worker {
    engine: GpuPrio3,
    helper_state: Option<PrepareState>,
    /// free leader states; one is lent to each `LeaderPending` in flight
    leader_states: Vec<PrepareState>,
    agg: Option<AggregateShares>,
}

/// The worker's pooled aggregate, grown (re-created) only when a job has more batch slots than
/// any before it.
fn pooled_aggregate<'a>(engine: &GpuPrio3, agg: &'a mut Option<AggregateShares>, slot_count: u32)
                        -> Result<&'a mut AggregateShares, GpuError> {
    if agg.as_ref().map_or(true, |a| a.slots < slot_count) {
        *agg = None;
        *agg = Some(engine.new_aggregate(slot_count.max(1))?);
    }
    Ok(agg.as_mut().unwrap())
}

/// The engines of one task: `workers` contexts on `device` (one per concurrent aggregation-job
/// worker, `max_concurrent_job_workers`, aggregator/src/bin/aggregation_job_driver.rs:97-103), each
/// with states sized for `max_job_size` reports (`max_aggregation_job_size`,
/// docs/samples/basic_config/aggregation_job_creator.yaml:19-22).
pub struct GpuTask {
    pub params: EngineParams,
    pub sizes: ffi::prio3gpu_sizes,
    max_job_size: usize,
    workers: Vec<Mutex<Worker>>,
    next: AtomicUsize,
}

impl GpuTask {
    pub fn new(params: EngineParams, verify_key: &[u8; 16], device: i32, workers: usize,
               max_job_size: usize) -> Result<Arc<Self>, GpuError> {
        if workers == 0 || max_job_size == 0 {
            return Err(arg_error("a GpuTask needs at least one worker and job size > 0".into()));
        }
        let mut ws = Vec::with_capacity(workers);
        for _ in 0..workers {
            let engine = GpuPrio3::new(params, verify_key, device)?;
            ws.push(Mutex::new(Worker { engine, helper_state: None, leader_states: Vec::new(),
                                        agg: None }));
        }
        let sizes = ws[0].lock().unwrap().engine.sizes;
        Ok(Arc::new(Self { params, sizes, max_job_size, workers: ws, next: AtomicUsize::new(0) }))
    }

    /// A free worker (round robin, then wait on one): at most `workers` jobs use the GPU at once.
    fn acquire(&self) -> (usize, MutexGuard<'_, Worker>) {
        let n = self.workers.len();
        let start = self.next.fetch_add(1, Ordering::Relaxed) % n;
        for i in 0..n {
            let w = (start + i) % n;
            if let Ok(g) = self.workers[w].try_lock() {
                return (w, g);
            }
        }
        (start, self.workers[start].lock().unwrap())
    }

    fn check_job(&self, n: usize) -> Result<(), GpuError> {
        if n == 0 || n > self.max_job_size {
            return Err(arg_error(format!("job of {n} reports (max {})", self.max_job_size)));
        }
        Ok(())
    }

    /// The per-report loop of aggregator.rs:1613-1848 for a whole job.  Returns the prep messages
    /// (status 0 -> PrepareStepResult::Continue{Finish{prep_msg}}, else Reject(status)) and the
    /// per-slot aggregations the datastore transaction (:1889-2044) writes.  The leader picks the
    /// job size, so a job larger than the pooled state runs as consecutive engine calls into the
    /// same aggregate.
    pub fn helper_aggregate_init(&self, job: &HelperJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, Vec<SlotAggregation>), GpuError> {
        let n = status.len();
        if n == 0 {
            return Err(arg_error("empty helper job".into()));
        }
        let (_, mut guard) = self.acquire();
        let Worker { engine, helper_state, agg, .. } = &mut *guard;
        if helper_state.is_none() {
            *helper_state = Some(engine.new_state(1, self.max_job_size)?);
        }
        let agg = pooled_aggregate(engine, agg, job.slot_count)?;
        let s = self.sizes;
        let (ps, hs, lp) = (s.public_share as usize, s.helper_input_share as usize,
                            s.prep_share as usize);
        let mut run = || -> Result<(Vec<u8>, Vec<SlotAggregation>), GpuError> {
            let mut msgs = Vec::with_capacity(n * s.prep_msg as usize);
            let mut lo = 0;
            while lo < n {
                let hi = (lo + self.max_job_size).min(n);
                msgs.extend(engine.helper_init(
                    helper_state.as_mut().unwrap(), &job.nonces[16 * lo..16 * hi],
                    &job.public_shares[ps * lo..ps * hi],
                    &job.helper_input_shares[hs * lo..hs * hi],
                    &job.leader_prep_shares[lp * lo..lp * hi], &job.report_times[lo..hi],
                    &job.batch_slots[lo..hi], &mut status[lo..hi], agg)?);
                lo = hi;
            }
            Ok((msgs, agg.take(job.slot_count)?))
        };
        let res = run();
        if res.is_err() {
            // a failed call may have accumulated part of the job: the pooled aggregate starts clean
            let _ = agg.reset();
        }
        res
    }

    /// `step_aggregation_job_aggregate_init` (aggregation_job_driver.rs:290-437) for a whole job:
    /// the leader prep shares of the AggregationJobInitializeReq, and the job's device state,
    /// held until the helper's response arrives.
    pub fn leader_aggregate_init(self: &Arc<Self>, job: &LeaderInitJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, LeaderPending), GpuError> {
        let n = status.len();
        self.check_job(n)?;
        let (wi, mut guard) = self.acquire();
        let w = &mut *guard;
        let mut state = match w.leader_states.pop() {
            Some(s) => s,
            None => w.engine.new_state(0, self.max_job_size)?,
        };
        match w.engine.leader_init(&mut state, job.nonces, job.public_shares,
                                   job.leader_input_shares, status) {
            Ok(prep) => Ok((prep, LeaderPending { task: Arc::clone(self), worker: wi, n,
                                                  state: Some(state) })),
            Err(e) => {
                w.leader_states.push(state);
                Err(e)
            }
        }
    }

    /// `process_response_from_helper` (aggregation_job_driver.rs:530-727): `leader_continued`
    /// with the helper's prep messages, accumulation, and the per-slot aggregations the
    /// transaction (:698-720) writes.  The pending state returns to its worker's pool.
    pub fn leader_process_response(&self, mut pending: LeaderPending, job: &LeaderFinishJob,
                                   status: &mut [u8]) -> Result<Vec<SlotAggregation>, GpuError> {
        if !ptr::eq(Arc::as_ptr(&pending.task), self) || status.len() != pending.n {
            return Err(arg_error("leader response does not belong to this pending job".into()));
        }
        let mut guard = self.workers[pending.worker].lock().unwrap();
        let Worker { engine, agg, leader_states, .. } = &mut *guard;
        let mut state = pending.state.take().unwrap();
        let res = pooled_aggregate(engine, agg, job.slot_count).and_then(|agg| {
            engine.leader_finish(&mut state, job.prep_msgs, job.nonces, job.report_times,
                                 job.batch_slots, status, agg)?;
            agg.take(job.slot_count)
        });
        leader_states.push(state);
        res
    }
}

/// What `handle_aggregate_init_generic` needs from one job, after it has decoded the request,
/// checked it (duplicate IDs, aggregation parameter: aggregator.rs:1588-1605), opened the HPKE
/// ciphertexts and decoded the plaintext input shares (:1634-1768) -- all on CPU threads
/// (prio3gpu_decode_agg_init_req, prio3gpu_hpke_open_report_shares,
/// prio3gpu_decode_plaintext_input_shares).
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

/// The leader's decoded `LeaderStoredReport`s of one job (aggregation_job_driver.rs:329-402;
/// shares decoded by aggregator_core/src/datastore.rs:1298-1304).
pub struct LeaderInitJob<'a> {
    pub nonces: &'a [u8],
    pub public_shares: &'a [u8],
    pub leader_input_shares: &'a [u8],
}

/// The helper's AggregationJobResp, gathered per report (prio3gpu_decode_agg_job_resp +
/// prio3gpu_gather_helper_resps), plus the accumulation keys (aggregation_job_driver.rs:566-686).
pub struct LeaderFinishJob<'a> {
    pub prep_msgs: &'a [u8],
    pub nonces: &'a [u8],
    pub report_times: &'a [u64],
    pub batch_slots: &'a [u32],
    pub slot_count: u32,
}

/// A leader job between its AggregationJobInitializeReq and the helper's response: the job's
/// device state, lent from its worker's pool (returned by `leader_process_response`, or on drop
/// when the job is abandoned, e.g. the helper request failed and the lease will be retried).
pub struct LeaderPending {
    task: Arc<GpuTask>,
    worker: usize,
    n: usize,
    state: Option<PrepareState>,
}

impl Drop for LeaderPending {
    fn drop(&mut self) {
        if let Some(st) = self.state.take() {
            if let Ok(mut w) = self.task.workers[self.worker].lock() {
                w.leader_states.push(st);
            }
        }
    }
}

/// The batched arms a Janus build with the `mi355x` feature adds beside `VdafOps`
/// (aggregator.rs:1040-1065), one per Prio3 variant.  `TaskAggregator::new`
/// (aggregator.rs:797-900) builds it next to the CPU VDAF with `GpuVdafOps::new`;
/// `VdafOps::handle_aggregate_init` (aggregator.rs:1230-1274) routes the job here when the task
/// has one, and the leader's job driver (aggregation_job_driver.rs:102-119) likewise.
pub enum GpuVdafOps {
    Prio3Count(Arc<GpuTask>),
    Prio3CountVec(Arc<GpuTask>),
    Prio3Sum(Arc<GpuTask>),
    Prio3SumVec(Arc<GpuTask>),
    Prio3Histogram(Arc<GpuTask>),
    #[cfg(feature = "fpvec_bounded_l2")]
    Prio3FixedPoint16BitBoundedL2VecSum(Arc<GpuTask>),
    #[cfg(feature = "fpvec_bounded_l2")]
    Prio3FixedPoint32BitBoundedL2VecSum(Arc<GpuTask>),
    #[cfg(feature = "fpvec_bounded_l2")]
    Prio3FixedPoint64BitBoundedL2VecSum(Arc<GpuTask>),
}

impl GpuVdafOps {
    /// `None` when the instance stays on the CPU path (Poplar1, the fake VDAFs).
    pub fn new(vdaf: &VdafInstance, verify_key: &[u8; 16], device: i32, workers: usize,
               max_job_size: usize) -> Option<Result<Self, GpuError>> {
        let params = engine_params(vdaf)?;
        let task = match GpuTask::new(params, verify_key, device, workers, max_job_size) {
            Ok(t) => t,
            Err(e) => return Some(Err(e)),
        };
        Some(Ok(match vdaf {
            VdafInstance::Prio3Count => GpuVdafOps::Prio3Count(task),
            VdafInstance::Prio3CountVec { .. } => GpuVdafOps::Prio3CountVec(task),
            VdafInstance::Prio3Sum { .. } => GpuVdafOps::Prio3Sum(task),
            VdafInstance::Prio3SumVec { .. } => GpuVdafOps::Prio3SumVec(task),
            VdafInstance::Prio3Histogram { .. } => GpuVdafOps::Prio3Histogram(task),
            #[cfg(feature = "fpvec_bounded_l2")]
            VdafInstance::Prio3FixedPoint16BitBoundedL2VecSum { .. } => {
                GpuVdafOps::Prio3FixedPoint16BitBoundedL2VecSum(task)
            }
            #[cfg(feature = "fpvec_bounded_l2")]
            VdafInstance::Prio3FixedPoint32BitBoundedL2VecSum { .. } => {
                GpuVdafOps::Prio3FixedPoint32BitBoundedL2VecSum(task)
            }
            #[cfg(feature = "fpvec_bounded_l2")]
            VdafInstance::Prio3FixedPoint64BitBoundedL2VecSum { .. } => {
                GpuVdafOps::Prio3FixedPoint64BitBoundedL2VecSum(task)
            }
            _ => unreachable!("engine_params returned Some"),
        }))
    }

    /// The engine kind behind each arm (include/prio3gpu.h `enum prio3gpu_kind`).
    pub fn kind(&self) -> c_int {
        match self {
            GpuVdafOps::Prio3Count(_) => ffi::PRIO3GPU_COUNT,
            GpuVdafOps::Prio3CountVec(_) => ffi::PRIO3GPU_SUMVEC,
            GpuVdafOps::Prio3Sum(_) => ffi::PRIO3GPU_SUM,
            GpuVdafOps::Prio3SumVec(_) => ffi::PRIO3GPU_SUMVEC,
            GpuVdafOps::Prio3Histogram(_) => ffi::PRIO3GPU_HISTOGRAM,
            #[cfg(feature = "fpvec_bounded_l2")]
            GpuVdafOps::Prio3FixedPoint16BitBoundedL2VecSum(_)
            | GpuVdafOps::Prio3FixedPoint32BitBoundedL2VecSum(_)
            | GpuVdafOps::Prio3FixedPoint64BitBoundedL2VecSum(_) => ffi::PRIO3GPU_FPVEC,
        }
    }

    pub fn task(&self) -> &Arc<GpuTask> {
        match self {
            GpuVdafOps::Prio3Count(t)
            | GpuVdafOps::Prio3CountVec(t)
            | GpuVdafOps::Prio3Sum(t)
            | GpuVdafOps::Prio3SumVec(t)
            | GpuVdafOps::Prio3Histogram(t) => t,
            #[cfg(feature = "fpvec_bounded_l2")]
            GpuVdafOps::Prio3FixedPoint16BitBoundedL2VecSum(t)
            | GpuVdafOps::Prio3FixedPoint32BitBoundedL2VecSum(t)
            | GpuVdafOps::Prio3FixedPoint64BitBoundedL2VecSum(t) => t,
        }
    }

    /// Helper: `handle_aggregate_init_generic`'s per-report loop for a whole job.
    pub fn helper_aggregate_init(&self, job: &HelperJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, Vec<SlotAggregation>), GpuError> {
        self.task().helper_aggregate_init(job, status)
    }

    /// Leader: `step_aggregation_job_aggregate_init`'s per-report loop for a whole job.
    pub fn leader_aggregate_init(&self, job: &LeaderInitJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, LeaderPending), GpuError> {
        self.task().leader_aggregate_init(job, status)
    }

    /// Leader: `process_response_from_helper`'s per-report loop for a whole job.
    pub fn leader_process_response(&self, pending: LeaderPending, job: &LeaderFinishJob,
                                   status: &mut [u8]) -> Result<Vec<SlotAggregation>, GpuError> {
        self.task().leader_process_response(pending, job, status)
    }
}

/// The per-process RCCL communicator for merging per-GPU partial aggregates (one rank per GPU;
/// the engine serialises flushes of all contexts through it).  Janus-native alternative: write
/// each GPU's partial as its own batch-aggregation shard (`ord`, accumulator.rs:92) and let
/// collection merge them (aggregate_share.rs:47-65).
pub struct GpuComm {
    comm: *mut ffi::prio3gpu_comm,
}
unsafe impl Send for GpuComm {}
unsafe impl Sync for GpuComm {}

impl GpuComm {
    pub fn unique_id() -> Result<[u8; 128], GpuError> {
        let mut id = [0u8; 128];
        check(unsafe { ffi::prio3gpu_comm_unique_id(id.as_mut_ptr()) })?;
        Ok(id)
    }

    pub fn new(id: &[u8; 128], nranks: i32, rank: i32, device: i32) -> Result<Self, GpuError> {
        let mut comm = ptr::null_mut();
        check(unsafe { ffi::prio3gpu_comm_init(id.as_ptr(), nranks, rank, device, &mut comm) })?;
        Ok(Self { comm })
    }

    /// total += sum over ranks of `local` (mod p, counts, checksum XOR, interval union); `local`
    /// is reset.  Every rank calls it with the same slot count, in the same order: a per-job
    /// lockstep flush, only for drivers that step jobs in lockstep across GPUs.
    pub fn allreduce(&self, engine: &GpuPrio3, local: &mut AggregateShares,
                     total: &mut AggregateShares) -> Result<(), GpuError> {
        check(unsafe { ffi::prio3gpu_agg_allreduce(self.comm, engine.ctx, local.agg, total.agg) })
    }

    /// The epoch merge for independent job drivers (prio3gpu_agg_epoch_merge): `local` is this
    /// GPU's partial over any number of jobs, its slot i holding batch identifier `keys[i]`;
    /// `union` is the epoch's sorted union of every rank's keys (agreed over the host channel,
    /// identical on every rank).  Returns the totals, one slot per union key; `local` is reset.
    /// Every rank calls it once per epoch, epochs in the same order, one merger per communicator.
    pub fn epoch_merge<K: Eq + Hash>(&self, engine: &GpuPrio3, local: &mut AggregateShares,
                                     keys: &[K], union: &[K])
                                     -> Result<AggregateShares, GpuError> {
        let index: HashMap<&K, u32> = union.iter().enumerate().map(|(i, k)| (k, i as u32)).collect();
        let mut slot_map = vec![ffi::PRIO3GPU_SLOT_UNUSED; local.slots as usize];
        if keys.len() > slot_map.len() {
            return Err(arg_error("epoch merge: more keys than local slots".into()));
        }
        for (s, k) in keys.iter().enumerate() {
            slot_map[s] = *index
                .get(k)
                .ok_or_else(|| arg_error("epoch merge: a local key is not in the union".into()))?;
        }
        let mut total = engine.new_aggregate(union.len() as u32)?;
        check(unsafe {
            ffi::prio3gpu_agg_epoch_merge(self.comm, engine.ctx, local.agg, slot_map.as_ptr(),
                                          union.len() as u32, total.agg)
        })?;
        Ok(total)
    }
}

impl Drop for GpuComm {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_comm_destroy(self.comm) };
    }
}

/// `Collector::unshard`'s aggregate result: `u64` / `u128` / `Vec<u128>` for the integer Prio3
/// types (Count and Sum have one entry), `Vec<f64>` for the fixed-point vectors.
#[derive(Debug, Clone, PartialEq)]
pub enum AggregateResult {
    Integers(Vec<u128>),
    FixedPoint(Vec<f64>),
}

/// The collection-time merge of batch-aggregation shards (aggregate_share.rs:44-66,
/// `BatchAggregation::merged_with`, models.rs:962-991): `acc` += `src` -- mod-p share sum, count
/// sum, checksum XOR, interval union.  Host only.
pub fn merge_slot_aggregations(field_size: u32, acc: &mut SlotAggregation, src: &SlotAggregation)
                               -> Result<(), GpuError> {
    if acc.aggregate_share.len() != src.aggregate_share.len() || field_size == 0
        || acc.aggregate_share.len() % field_size as usize != 0
    {
        return Err(arg_error("merge: aggregate shares of different lengths".into()));
    }
    let mut src_share = src.aggregate_share.clone();
    let mut dst = ffi::prio3gpu_batch_aggregation {
        aggregate_share: acc.aggregate_share.as_mut_ptr(), report_count: acc.report_count,
        checksum: acc.checksum, interval_start: acc.interval_start,
        interval_duration: acc.interval_duration,
    };
    let from = ffi::prio3gpu_batch_aggregation {
        aggregate_share: src_share.as_mut_ptr(), report_count: src.report_count,
        checksum: src.checksum, interval_start: src.interval_start,
        interval_duration: src.interval_duration,
    };
    check(unsafe {
        ffi::prio3gpu_batch_aggregation_merge(field_size,
                                              acc.aggregate_share.len() / field_size as usize,
                                              &mut dst, &from)
    })?;
    acc.report_count = dst.report_count;
    acc.checksum = dst.checksum;
    acc.interval_start = dst.interval_start;
    acc.interval_duration = dst.interval_duration;
    Ok(())
}

// ------------------------------------------------------------------------------------------------
// Janus call-site adapters: what rust/patches/janus-0.6-mi355x.patch calls from
// handle_aggregate_init_generic (aggregator.rs:1613-1848) and the aggregation job driver
// (aggregation_job_driver.rs:290-437, :530-727).
// ------------------------------------------------------------------------------------------------

/// The `gpu:` section of the aggregator and aggregation-job-driver configs.  One process per GPU:
/// `device` is the HIP ordinal this process drives.
#[derive(Debug, Clone, Copy, PartialEq, Eq, Serialize, Deserialize)]
pub struct GpuConfig {
    pub device: i32,
    /// Engine contexts (HIP streams) per task = aggregation jobs on the GPU at once; the job
    /// driver's `max_concurrent_job_workers` is the natural value.
    pub workers: usize,
    /// Reports per job each pooled state holds.  The leader's `max_aggregation_job_size` must not
    /// exceed it; the helper splits larger jobs into consecutive calls.
    pub max_job_size: usize,
}

impl GpuConfig {
    /// The task's batched arms (`TaskAggregator::new`, aggregator.rs:797-900), or `None` when the
    /// VDAF stays on the per-report CPU path (Poplar1, the fake VDAFs) or the verify key is not
    /// the 16 bytes Prio3 takes.
    pub fn ops_for(&self, vdaf: &VdafInstance, verify_key: &[u8])
                   -> Option<Result<GpuVdafOps, GpuError>> {
        let vk: &[u8; 16] = verify_key.try_into().ok()?;
        GpuVdafOps::new(vdaf, vk, self.device, self.workers, self.max_job_size)
    }
}

/// Engine status of `PrepareError::BatchCollected` (its DAP code, 0, is the engine's "ok").
const STATUS_BATCH_COLLECTED: u8 = 0xFE;

/// A report's `PrepareError` as the engine's status byte; a non-zero status makes every engine
/// call skip the report and leave its status as it is.
pub fn status_of(error: PrepareError) -> u8 {
    match error {
        PrepareError::BatchCollected => STATUS_BATCH_COLLECTED,
        e => e as u8,
    }
}

/// The `PrepareError` of a non-zero status.  The engine itself only writes VdafPrepError (5;
/// every ping-pong failure maps there, error.rs:240-300) and InvalidMessage (8, a non-canonical
/// element or share length); the other codes come back as the caller set them.
pub fn prepare_error(status: u8) -> PrepareError {
    match status {
        STATUS_BATCH_COLLECTED => PrepareError::BatchCollected,
        1 => PrepareError::ReportReplayed,
        2 => PrepareError::ReportDropped,
        3 => PrepareError::HpkeUnknownConfigId,
        4 => PrepareError::HpkeDecryptError,
        6 => PrepareError::BatchSaturated,
        7 => PrepareError::TaskExpired,
        8 => PrepareError::InvalidMessage,
        _ => PrepareError::VdafPrepError,
    }
}

/// A job's batch identifiers in first-seen order, numbered as the engine's aggregate slots
/// (`Accumulator`'s HashMap<BatchIdentifier, BatchData>, accumulator.rs:26-122).
pub struct SlotMap<K> {
    keys: Vec<K>,
    index: HashMap<K, u32>,
}

impl<K: Clone + Eq + Hash> Default for SlotMap<K> {
    fn default() -> Self {
        Self { keys: Vec::new(), index: HashMap::new() }
    }
}

impl<K: Clone + Eq + Hash> SlotMap<K> {
    pub fn new() -> Self {
        Self::default()
    }

    pub fn slot_of(&mut self, key: &K) -> u32 {
        if let Some(&s) = self.index.get(key) {
            return s;
        }
        let s = self.keys.len() as u32;
        self.keys.push(key.clone());
        self.index.insert(key.clone(), s);
        s
    }

    pub fn len(&self) -> u32 {
        self.keys.len() as u32
    }

    pub fn is_empty(&self) -> bool {
        self.keys.is_empty()
    }

    pub fn into_keys(self) -> Vec<K> {
        self.keys
    }
}

/// Per-report results of one engine call plus the per-slot aggregations, keyed by batch
/// identifier.
pub struct JobOutcome<K> {
    pub status: Vec<u8>,
    report_ids: Vec<u8>,
    batch_slots: Vec<u32>,
    prep_msg_len: usize,
    prep_msgs: Vec<u8>,
    pub slots: Vec<(K, SlotAggregation)>,
}

impl<K> JobOutcome<K> {
    /// Helper: report `i`'s `PrepareStepResult` payload -- `Continue{Finish{prep_msg}}` (Prio3 is
    /// one round: the helper finishes in its first step, aggregator.rs:1811-1826) or
    /// `Reject(error)`.
    pub fn result(&self, i: usize) -> Result<PingPongMessage, PrepareError> {
        match self.status[i] {
            0 => Ok(PingPongMessage::Finish {
                prep_msg: self.prep_msgs[i * self.prep_msg_len..(i + 1) * self.prep_msg_len]
                    .to_vec(),
            }),
            s => Err(prepare_error(s)),
        }
    }

    /// Leader: report `i`'s final state -- `Ok` = Finished and accumulated, else Failed(error).
    pub fn finished(&self, i: usize) -> Result<(), PrepareError> {
        match self.status[i] {
            0 => Ok(()),
            s => Err(prepare_error(s)),
        }
    }

    /// The report IDs accumulated into `slot` (status 0): `BatchData::included_report_ids`, which
    /// `flush_to_datastore` reports back as unmergeable when the batch was collected meanwhile.
    pub fn slot_report_ids(&self, slot: usize) -> Vec<[u8; 16]> {
        (0..self.status.len())
            .filter(|&i| self.status[i] == 0 && self.batch_slots[i] as usize == slot)
            .map(|i| self.report_ids[16 * i..16 * i + 16].try_into().unwrap())
            .collect()
    }
}

/// One helper aggregation job gathered for ONE engine call: `handle_aggregate_init_generic`
/// (aggregator.rs:1613-1848) keeps its per-report HPKE open and decoding, pushes each report
/// here instead of calling `helper_initialized(..).evaluate(..)` (:1775-1797), and after the loop
/// runs the job (`prio3gpu_helper_init` + `prio3gpu_agg_update_reports`).
pub struct HelperBatch<K> {
    sizes: ffi::prio3gpu_sizes,
    slots: SlotMap<K>,
    nonces: Vec<u8>,
    public_shares: Vec<u8>,
    helper_input_shares: Vec<u8>,
    leader_prep_shares: Vec<u8>,
    report_times: Vec<u64>,
    batch_slots: Vec<u32>,
    status: Vec<u8>,
}

impl<K: Clone + Eq + Hash> HelperBatch<K> {
    pub fn new(ops: &GpuVdafOps, capacity: usize) -> Self {
        let s = ops.task().sizes;
        Self {
            sizes: s,
            slots: SlotMap::new(),
            nonces: Vec::with_capacity(16 * capacity),
            public_shares: Vec::with_capacity(s.public_share as usize * capacity),
            helper_input_shares: Vec::with_capacity(s.helper_input_share as usize * capacity),
            leader_prep_shares: Vec::with_capacity(s.prep_share as usize * capacity),
            report_times: Vec::with_capacity(capacity),
            batch_slots: Vec::with_capacity(capacity),
            status: Vec::with_capacity(capacity),
        }
    }

    /// The aggregate slot of a report's batch identifier (`Q::to_batch_identifier`, :1615-1619).
    pub fn slot_of(&mut self, batch_identifier: &K) -> u32 {
        self.slots.slot_of(batch_identifier)
    }

    /// One report, in request order.  `shares`: the encoded public share and the decrypted
    /// helper input share (`PlaintextInputShare::payload`), or the `PrepareError` the CPU stages
    /// gave the report (HPKE, decoding: :1633-1770).  `leader_message` must be
    /// `Initialize{prep_share}`; anything else is a ping-pong mismatch, VdafPrepError.
    pub fn push(&mut self, report_id: &[u8; 16], time: u64, slot: u32,
                shares: Result<(&[u8], &[u8]), PrepareError>, leader_message: &PingPongMessage) {
        let s = &self.sizes;
        let (pl, hl, ll) = (s.public_share as usize, s.helper_input_share as usize,
                            s.prep_share as usize);
        let mut st = 0u8;
        let (public_share, input_share) = match shares {
            Ok((p, h)) if p.len() == pl && h.len() == hl => (p, h),
            Ok(_) => {
                st = status_of(PrepareError::InvalidMessage);
                (&[][..], &[][..])
            }
            Err(e) => {
                st = status_of(e);
                (&[][..], &[][..])
            }
        };
        let prep_share = match leader_message {
            PingPongMessage::Initialize { prep_share } if prep_share.len() == ll => {
                Some(prep_share.as_slice())
            }
            _ => None,
        };
        if st == 0 && prep_share.is_none() {
            st = status_of(PrepareError::VdafPrepError);
        }
        let fill = |v: &mut Vec<u8>, b: &[u8], len: usize| {
            if st == 0 {
                v.extend_from_slice(b);
            } else {
                v.resize(v.len() + len, 0);
            }
        };
        self.nonces.extend_from_slice(report_id);
        fill(&mut self.public_shares, public_share, pl);
        fill(&mut self.helper_input_shares, input_share, hl);
        fill(&mut self.leader_prep_shares, prep_share.unwrap_or(&[]), ll);
        self.report_times.push(time);
        self.batch_slots.push(slot);
        self.status.push(st);
    }

    pub fn len(&self) -> usize {
        self.status.len()
    }

    pub fn is_empty(&self) -> bool {
        self.status.is_empty()
    }

    /// The job on the GPU: per-report results and the per-batch-identifier aggregations.
    pub fn run(mut self, ops: &GpuVdafOps) -> Result<JobOutcome<K>, GpuError> {
        let prep_msg_len = self.sizes.prep_msg as usize;
        let (prep_msgs, slots) = if self.status.is_empty() {
            (Vec::new(), Vec::new())
        } else {
            let job = HelperJob {
                nonces: &self.nonces, public_shares: &self.public_shares,
                helper_input_shares: &self.helper_input_shares,
                leader_prep_shares: &self.leader_prep_shares, report_times: &self.report_times,
                batch_slots: &self.batch_slots, slot_count: self.slots.len(),
            };
            ops.helper_aggregate_init(&job, &mut self.status)?
        };
        Ok(JobOutcome {
            status: self.status, report_ids: self.nonces, batch_slots: self.batch_slots,
            prep_msg_len, prep_msgs, slots: self.slots.into_keys().into_iter().zip(slots).collect(),
        })
    }
}

/// The leader's job between `prepare_init` and the helper's response: the prep shares that go
/// into the `PrepareInit` messages and the job's device state.
pub struct LeaderInitOutcome {
    status: Vec<u8>,
    report_ids: Vec<u8>,
    report_times: Vec<u64>,
    prep_share_len: usize,
    prep_shares: Vec<u8>,
    /// `None` for a job with no report left after the per-report checks
    pending: Option<LeaderPending>,
}

impl LeaderInitOutcome {
    /// Report `i`'s `PingPongMessage::Initialize` for the AggregationJobInitializeReq
    /// (aggregation_job_driver.rs:381-394), or the PrepareError it failed with (:395-400).
    pub fn message(&self, i: usize) -> Result<PingPongMessage, PrepareError> {
        match self.status[i] {
            0 => Ok(PingPongMessage::Initialize {
                prep_share: self.prep_shares[i * self.prep_share_len..(i + 1) * self.prep_share_len]
                    .to_vec(),
            }),
            s => Err(prepare_error(s)),
        }
    }
}

/// The leader's `step_aggregation_job_aggregate_init` loop (aggregation_job_driver.rs:329-402):
/// the reports that passed the per-report checks, then ONE `prio3gpu_prepare_init(agg_id 0)`.
pub struct LeaderBatch {
    sizes: ffi::prio3gpu_sizes,
    nonces: Vec<u8>,
    public_shares: Vec<u8>,
    leader_input_shares: Vec<u8>,
    report_times: Vec<u64>,
}

impl LeaderBatch {
    pub fn new(ops: &GpuVdafOps, capacity: usize) -> Self {
        let s = ops.task().sizes;
        Self {
            sizes: s,
            nonces: Vec::with_capacity(16 * capacity),
            public_shares: Vec::with_capacity(s.public_share as usize * capacity),
            leader_input_shares: Vec::with_capacity(s.leader_input_share as usize * capacity),
            report_times: Vec::with_capacity(capacity),
        }
    }

    /// One stored client report: its public share and leader input share as the datastore holds
    /// them (`RawLeaderStoredReport`, read by the patch's `get_client_report_raw` without the
    /// `get_decoded_with_param` of aggregator_core/src/datastore.rs:1297-1304).  The engine
    /// validates the encodings per report: a share of the wrong length (here) or a
    /// non-canonical field element (`prio3gpu_prepare_init`) fails that report alone with
    /// InvalidMessage.
    pub fn push(&mut self, report_id: &[u8; 16], time: u64, public_share: &[u8],
                leader_input_share: &[u8]) {
        let s = &self.sizes;
        let ok = public_share.len() == s.public_share as usize
            && leader_input_share.len() == s.leader_input_share as usize;
        self.nonces.extend_from_slice(report_id);
        if ok {
            self.public_shares.extend_from_slice(public_share);
            self.leader_input_shares.extend_from_slice(leader_input_share);
        } else {
            // an all-zero leader share is never a valid report: the engine rejects it, and
            // `run` marks it InvalidMessage first
            let (pl, ll) = (s.public_share as usize, s.leader_input_share as usize);
            self.public_shares.resize(self.public_shares.len() + pl, 0);
            self.leader_input_shares.resize(self.leader_input_shares.len() + ll, 0);
        }
        self.report_times.push(if ok { time } else { u64::MAX });
    }

    pub fn len(&self) -> usize {
        self.report_times.len()
    }

    pub fn is_empty(&self) -> bool {
        self.report_times.is_empty()
    }

    pub fn run(self, ops: &GpuVdafOps) -> Result<LeaderInitOutcome, GpuError> {
        let mut status: Vec<u8> = self
            .report_times
            .iter()
            .map(|&t| if t == u64::MAX { status_of(PrepareError::InvalidMessage) } else { 0 })
            .collect();
        let (prep_shares, pending) = if status.is_empty() {
            (Vec::new(), None)
        } else {
            let job = LeaderInitJob {
                nonces: &self.nonces, public_shares: &self.public_shares,
                leader_input_shares: &self.leader_input_shares,
            };
            let (prep, pending) = ops.leader_aggregate_init(&job, &mut status)?;
            (prep, Some(pending))
        };
        Ok(LeaderInitOutcome {
            status, report_ids: self.nonces, report_times: self.report_times,
            prep_share_len: self.sizes.prep_share as usize, prep_shares, pending,
        })
    }
}

/// `process_response_from_helper` (aggregation_job_driver.rs:530-727) for a GPU-initialised
/// job: the helper's `PrepareResp`s gathered per report, then ONE `prio3gpu_prepare_next` +
/// accumulate + report bookkeeping.
pub struct LeaderFinishBatch<K> {
    init: LeaderInitOutcome,
    prep_msg_len: usize,
    prep_msgs: Vec<u8>,
    batch_slots: Vec<u32>,
    slots: SlotMap<K>,
}

impl<K: Clone + Eq + Hash> LeaderFinishBatch<K> {
    pub fn new(ops: &GpuVdafOps, init: LeaderInitOutcome) -> Self {
        let n = init.status.len();
        let pm = ops.task().sizes.prep_msg as usize;
        Self { init, prep_msg_len: pm, prep_msgs: vec![0u8; n * pm], batch_slots: vec![0; n],
               slots: SlotMap::new() }
    }

    /// The helper's answer for report `i` (an index into the init batch): `Ok(message)` for
    /// `PrepareStepResult::Continue{message}` -- a Prio3 helper answers Finish{prep_msg}; any
    /// other message is a ping-pong mismatch (VdafPrepError) -- or the error the caller mapped
    /// (`Reject(err)` -> err; `Finished` while the leader is still continued -> VdafPrepError,
    /// :632-664).  `batch_identifier`: `Q::to_batch_identifier` of the report's time.
    pub fn push(&mut self, i: usize, batch_identifier: &K,
                helper_message: Result<&PingPongMessage, PrepareError>) {
        self.batch_slots[i] = self.slots.slot_of(batch_identifier);
        if self.init.status[i] != 0 {
            return;
        }
        let pm = self.prep_msg_len;
        self.init.status[i] = match helper_message {
            Ok(PingPongMessage::Finish { prep_msg }) if prep_msg.len() == pm => {
                self.prep_msgs[i * pm..(i + 1) * pm].copy_from_slice(prep_msg);
                0
            }
            Ok(_) => status_of(PrepareError::VdafPrepError),
            Err(e) => status_of(e),
        };
    }

    /// Reports of the init batch (pushed or not: a report that failed at init, and so was not
    /// sent, keeps its status).
    pub fn len(&self) -> usize {
        self.init.status.len()
    }

    pub fn is_empty(&self) -> bool {
        self.init.status.is_empty()
    }

    pub fn run(self, ops: &GpuVdafOps) -> Result<JobOutcome<K>, GpuError> {
        let Self { init, prep_msg_len, prep_msgs, batch_slots, slots } = self;
        let LeaderInitOutcome { mut status, report_ids, report_times, pending, .. } = init;
        let aggs = match pending {
            None => Vec::new(),
            Some(pending) => {
                let job = LeaderFinishJob {
                    prep_msgs: &prep_msgs, nonces: &report_ids, report_times: &report_times,
                    batch_slots: &batch_slots, slot_count: slots.len().max(1),
                };
                ops.leader_process_response(pending, &job, &mut status)?
            }
        };
        Ok(JobOutcome {
            status, report_ids, batch_slots, prep_msg_len, prep_msgs,
            slots: slots.into_keys().into_iter().zip(aggs).collect(),
        })
    }
}

/// The aggregation job driver's engines, one `GpuVdafOps` per (task, verify key), created on
/// first use (the driver has no `TaskAggregator` cache; aggregation_job_driver.rs:102-119 builds
/// the VDAF per job).
pub struct GpuTaskCache {
    cfg: GpuConfig,
    tasks: Mutex<HashMap<(Vec<u8>, Vec<u8>), Option<Arc<GpuVdafOps>>>>,
}

impl GpuTaskCache {
    pub fn new(cfg: GpuConfig) -> Self {
        Self { cfg, tasks: Mutex::new(HashMap::new()) }
    }

    /// `None` for VDAFs that stay on the CPU path.  An engine failure is returned, not cached.
    pub fn ops_for(&self, task_id: &[u8], vdaf: &VdafInstance, verify_key: &[u8])
                   -> Result<Option<Arc<GpuVdafOps>>, GpuError> {
        let key = (task_id.to_vec(), verify_key.to_vec());
        let mut tasks = self.tasks.lock().unwrap();
        if let Some(ops) = tasks.get(&key) {
            return Ok(ops.clone());
        }
        let ops = match self.cfg.ops_for(vdaf, verify_key) {
            None => None,
            Some(Ok(ops)) => Some(Arc::new(ops)),
            Some(Err(e)) => return Err(e),
        };
        tasks.insert(key, ops.clone());
        Ok(ops)
    }
}

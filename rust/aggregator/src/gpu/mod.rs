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
pub mod ffi;

use std::ffi::{c_int, CStr};
use std::ptr;
use std::sync::atomic::{AtomicUsize, Ordering};
use std::sync::{Arc, Mutex, MutexGuard};

use janus_core::task::VdafInstance;

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
        Ok(Self { ctx, sizes })
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
    /// per-slot aggregations the datastore transaction (:1889-2044) writes.
    pub fn helper_aggregate_init(&self, job: &HelperJob, status: &mut [u8])
                                 -> Result<(Vec<u8>, Vec<SlotAggregation>), GpuError> {
        self.check_job(status.len())?;
        let (_, mut guard) = self.acquire();
        let Worker { engine, helper_state, agg, .. } = &mut *guard;
        if helper_state.is_none() {
            *helper_state = Some(engine.new_state(1, self.max_job_size)?);
        }
        let agg = pooled_aggregate(engine, agg, job.slot_count)?;
        let msgs = engine.helper_init(helper_state.as_mut().unwrap(), job.nonces,
                                      job.public_shares, job.helper_input_shares,
                                      job.leader_prep_shares, job.report_times, job.batch_slots,
                                      status, agg)?;
        let slots = agg.take(job.slot_count)?;
        Ok((msgs, slots))
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
    /// is reset.  Every rank calls it with the same slot count, in the same order.
    pub fn allreduce(&self, engine: &GpuPrio3, local: &mut AggregateShares,
                     total: &mut AggregateShares) -> Result<(), GpuError> {
        check(unsafe { ffi::prio3gpu_agg_allreduce(self.comm, engine.ctx, local.agg, total.agg) })
    }
}

impl Drop for GpuComm {
    fn drop(&mut self) {
        unsafe { ffi::prio3gpu_comm_destroy(self.comm) };
    }
}

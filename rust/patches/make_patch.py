#!/usr/bin/env python3
"""Generate rust/patches/janus-0.6-mi355x.patch: the reference-side edits that put Janus 0.6's
Prio3 aggregate-init path behind the MI355X engine (`mi355x` cargo feature).

    python rust/patches/make_patch.py [--reference /root/reference] [--check]

Each edit below is an anchored replacement that must match the reference file exactly once; the
edited text is diffed against the original (difflib, 3 lines of context) into one unified diff
with git's a/ b/ prefixes.  `--check` regenerates and compares with the committed patch.

To apply (a Janus checkout at the 0.6 tag):

    cp -r rust/aggregator/src/gpu  <janus>/aggregator/src/gpu
    cp rust/aggregator/build.rs    <janus>/aggregator/build.rs
    git -C <janus> apply rust/patches/janus-0.6-mi355x.patch
    cargo build -p janus_aggregator --features mi355x

What the patch does (call sites by reference file:line):
  * aggregator/Cargo.toml:15-17  the `mi355x` feature;
  * aggregator/src/lib.rs:7      `#[cfg(feature = "mi355x")] pub mod gpu;`
  * aggregator/src/aggregator.rs
      :186-218   `Config::gpu` (`GpuConfig`: device, workers, max_job_size), default None;
      :622-624   `task_aggregator_for` attaches the engine (`TaskAggregator::with_gpu`);
      :785-900   `TaskAggregator::gpu_ops` built from the task's VdafInstance + verify key;
      :937-957, :1230-1274  the arms are passed down to `handle_aggregate_init_generic`;
      :1561-1848 the helper loop keeps HPKE open + decoding per report, pushes each report into
                 a `gpu::HelperBatch` instead of helper_initialized(..).evaluate(..) (:1775-1797),
                 and after the loop runs the job as ONE engine call, maps statuses to
                 PrepareStepResult::{Continue{Finish}, Reject} and feeds the per-batch-identifier
                 aggregations to `Accumulator::update_aggregated`;
  * aggregator/src/aggregator/accumulator.rs:76-122  `update_aggregated` (a pre-aggregated
      BatchAggregation merged as `update` merges one report's);
  * aggregator_core/Cargo.toml, aggregator_core/src/datastore.rs:1160-1199  the `mi355x`
      feature and `get_client_report_raw` / `RawLeaderStoredReport`: a client report's public
      share and leader input share as stored, not decoded (:1297-1304 decode them);
  * aggregator/src/aggregator/aggregation_job_driver.rs
      :47-100   `AggregationJobDriver::with_gpu` (a `gpu::GpuTaskCache`);
      :141-232  the engine's tasks read their START reports through `get_client_report_raw`;
      :317-437  the leader loop's per-report checks stay (missing report, repeated extensions);
                leader_initialized (:362-401) becomes one `gpu::LeaderBatch` call for the job,
                fed the stored encodings; the response goes to
                `process_response_from_helper_gpu` (one prepare_next + accumulate);
      :688-726  the storage tail of process_response_from_helper becomes `write_step_results`,
                shared by both paths;
  * aggregator/src/bin/{aggregator,aggregation_job_driver}.rs  the `gpu:` config section.
"""
import argparse
import difflib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PATCH = os.path.join(HERE, "janus-0.6-mi355x.patch")

AGG = "aggregator/src/aggregator.rs"
DRV = "aggregator/src/aggregator/aggregation_job_driver.rs"
ACC = "aggregator/src/aggregator/accumulator.rs"
DS = "aggregator_core/src/datastore.rs"

EDITS = [
    # ---------------------------------------------------------------- Cargo feature, module
    ("aggregator/Cargo.toml",
     'fpvec_bounded_l2 = ["dep:fixed", "janus_core/fpvec_bounded_l2"]\n',
     'fpvec_bounded_l2 = ["dep:fixed", "janus_core/fpvec_bounded_l2"]\n'
     '# Prio3 aggregate-init on the MI355X engine (src/gpu; build.rs compiles and links it)\n'
     'mi355x = ["janus_aggregator_core/mi355x"]\n'),
    ("aggregator_core/Cargo.toml",
     'test-util = ["dep:hex", "dep:sqlx", "dep:testcontainers", "janus_core/test-util", "janus_messages/test-util"]\n',
     'test-util = ["dep:hex", "dep:sqlx", "dep:testcontainers", "janus_core/test-util", "janus_messages/test-util"]\n'
     '# the undecoded client-report read of the MI355X leader feed (janus_aggregator/mi355x)\n'
     'mi355x = []\n'),
    ("aggregator/src/lib.rs",
     "pub mod config;\n",
     "pub mod config;\n#[cfg(feature = \"mi355x\")]\npub mod gpu;\n"),

    # ---------------------------------------------------------------- aggregator.rs: config
    (AGG,
     """    pub global_hpke_configs_refresh_interval: StdDuration,

    pub taskprov_config: TaskprovConfig,
}
""",
     """    pub global_hpke_configs_refresh_interval: StdDuration,

    pub taskprov_config: TaskprovConfig,

    /// The MI355X engine for Prio3 aggregate-init (`mi355x` feature); `None` keeps every task on
    /// the per-report CPU path.
    #[cfg(feature = "mi355x")]
    pub gpu: Option<crate::gpu::GpuConfig>,
}
"""),
    (AGG,
     """            taskprov_config: TaskprovConfig::default(),
        }
    }
}

impl<C: Clock> Aggregator<C> {
""",
     """            taskprov_config: TaskprovConfig::default(),
            #[cfg(feature = "mi355x")]
            gpu: None,
        }
    }
}

impl<C: Clock> Aggregator<C> {
"""),
    (AGG,
     """                let task_agg =
                    Arc::new(TaskAggregator::new(task, Arc::clone(&self.report_writer))?);
""",
     """                let task_agg = TaskAggregator::new(task, Arc::clone(&self.report_writer))?;
                #[cfg(feature = "mi355x")]
                let task_agg = task_agg.with_gpu(self.cfg.gpu.as_ref())?;
                let task_agg = Arc::new(task_agg);
"""),

    # ---------------------------------------------------------------- TaskAggregator
    (AGG,
     """    /// Report writer, with support for batching.
    report_writer: Arc<ReportWriteBatcher<C>>,
}

impl<C: Clock> TaskAggregator<C> {
""",
     """    /// Report writer, with support for batching.
    report_writer: Arc<ReportWriteBatcher<C>>,
    /// The task's MI355X arms (`mi355x` feature): a Prio3 aggregate-init job runs as one engine
    /// call instead of the per-report loop.
    #[cfg(feature = "mi355x")]
    gpu_ops: Option<Arc<crate::gpu::GpuVdafOps>>,
}

impl<C: Clock> TaskAggregator<C> {
"""),
    (AGG,
     """        Ok(Self {
            task: Arc::new(task),
            vdaf_ops,
            report_writer,
        })
    }
""",
     """        Ok(Self {
            task: Arc::new(task),
            vdaf_ops,
            report_writer,
            #[cfg(feature = "mi355x")]
            gpu_ops: None,
        })
    }

    /// Attach the MI355X engine (the `gpu:` config section) when the task's VDAF runs on it.
    #[cfg(feature = "mi355x")]
    fn with_gpu(mut self, cfg: Option<&crate::gpu::GpuConfig>) -> Result<Self, Error> {
        if let Some(cfg) = cfg.filter(|_| crate::gpu::engine_params(self.task.vdaf()).is_some()) {
            let verify_key = self.task.primary_vdaf_verify_key::<VERIFY_KEY_LENGTH>()?;
            self.gpu_ops = cfg
                .ops_for(self.task.vdaf(), verify_key.as_bytes())
                .transpose()
                .map_err(|error| Error::Internal(error.to_string()))?
                .map(Arc::new);
        }
        Ok(self)
    }

    fn gpu_ops(&self) -> GpuOps<'_> {
        #[cfg(feature = "mi355x")]
        return self.gpu_ops.as_deref();
        #[cfg(not(feature = "mi355x"))]
        None
    }
"""),
    (AGG,
     """        self.vdaf_ops
            .handle_aggregate_init(
                datastore,
                global_hpke_keypairs,
                aggregate_step_failure_counter,
                Arc::clone(&self.task),
                batch_aggregation_shard_count,
                aggregation_job_id,
                req_bytes,
            )
            .await
""",
     """        self.vdaf_ops
            .handle_aggregate_init(
                datastore,
                global_hpke_keypairs,
                aggregate_step_failure_counter,
                Arc::clone(&self.task),
                batch_aggregation_shard_count,
                aggregation_job_id,
                req_bytes,
                self.gpu_ops(),
            )
            .await
"""),
    (AGG,
     """/// VdafOps stores VDAF-specific operations for a TaskAggregator in a non-generic way.
""",
     """/// A task's MI355X arms (`mi355x` feature); `None` keeps the per-report CPU path.
#[cfg(feature = "mi355x")]
type GpuOps<'a> = Option<&'a crate::gpu::GpuVdafOps>;
#[cfg(not(feature = "mi355x"))]
type GpuOps<'a> = Option<&'a std::convert::Infallible>;

/// VdafOps stores VDAF-specific operations for a TaskAggregator in a non-generic way.
"""),

    # ---------------------------------------------------------------- VdafOps::handle_aggregate_init
    (AGG,
     """        aggregation_job_id: &AggregationJobId,
        req_bytes: &[u8],
    ) -> Result<AggregationJobResp, Error> {
        match task.query_type() {
""",
     """        aggregation_job_id: &AggregationJobId,
        req_bytes: &[u8],
        gpu: GpuOps<'_>,
    ) -> Result<AggregationJobResp, Error> {
        match task.query_type() {
"""),
    (AGG,
     """                    Self::handle_aggregate_init_generic::<VERIFY_KEY_LENGTH, TimeInterval, VdafType, _>(
                        datastore,
                        global_hpke_keypairs,
                        vdaf,
                        aggregate_step_failure_counter,
                        task,
                        batch_aggregation_shard_count,
                        aggregation_job_id,
                        verify_key,
                        req_bytes,
                    )
""",
     """                    Self::handle_aggregate_init_generic::<VERIFY_KEY_LENGTH, TimeInterval, VdafType, _>(
                        datastore,
                        global_hpke_keypairs,
                        vdaf,
                        aggregate_step_failure_counter,
                        task,
                        batch_aggregation_shard_count,
                        aggregation_job_id,
                        verify_key,
                        req_bytes,
                        gpu,
                    )
"""),
    (AGG,
     """                    Self::handle_aggregate_init_generic::<VERIFY_KEY_LENGTH, FixedSize, VdafType, _>(
                        datastore,
                        global_hpke_keypairs,
                        vdaf,
                        aggregate_step_failure_counter,
                        task,
                        batch_aggregation_shard_count,
                        aggregation_job_id,
                        verify_key,
                        req_bytes,
                    )
""",
     """                    Self::handle_aggregate_init_generic::<VERIFY_KEY_LENGTH, FixedSize, VdafType, _>(
                        datastore,
                        global_hpke_keypairs,
                        vdaf,
                        aggregate_step_failure_counter,
                        task,
                        batch_aggregation_shard_count,
                        aggregation_job_id,
                        verify_key,
                        req_bytes,
                        gpu,
                    )
"""),

    # ---------------------------------------------------------------- helper loop
    (AGG,
     """    async fn handle_aggregate_init_generic<const SEED_SIZE: usize, Q, A, C>(
""",
     """    #[cfg_attr(not(feature = "mi355x"), allow(unused_variables))]
    async fn handle_aggregate_init_generic<const SEED_SIZE: usize, Q, A, C>(
"""),
    (AGG,
     """        verify_key: &VerifyKey<SEED_SIZE>,
        req_bytes: &[u8],
    ) -> Result<AggregationJobResp, Error>
    where
        Q: AccumulableQueryType,
""",
     """        verify_key: &VerifyKey<SEED_SIZE>,
        req_bytes: &[u8],
        gpu: GpuOps<'_>,
    ) -> Result<AggregationJobResp, Error>
    where
        Q: AccumulableQueryType,
"""),
    (AGG,
     """            agg_param.clone(),
        );

        for (ord, prepare_init) in req.prepare_inits().iter().enumerate() {
            // Compute intervals for each batch identifier included in this aggregation job.
            let batch_identifier = Q::to_batch_identifier(
                &task,
                req.batch_selector().batch_identifier(),
                prepare_init.report_share().metadata().time(),
            )?;
""",
     """            agg_param.clone(),
        );
        // MI355X: the loop gathers the job's reports; the VDAF steps run after it as ONE engine
        // call.
        #[cfg(feature = "mi355x")]
        let mut gpu_batch =
            gpu.map(|ops| crate::gpu::HelperBatch::new(ops, req.prepare_inits().len()));

        for (ord, prepare_init) in req.prepare_inits().iter().enumerate() {
            // Compute intervals for each batch identifier included in this aggregation job.
            let batch_identifier = Q::to_batch_identifier(
                &task,
                req.batch_selector().batch_identifier(),
                prepare_init.report_share().metadata().time(),
            )?;
            #[cfg(feature = "mi355x")]
            let gpu_slot = gpu_batch
                .as_mut()
                .map_or(0, |batch| batch.slot_of(&batch_identifier));
"""),
    (AGG,
     """            let input_share = plaintext_input_share.and_then(|plaintext_input_share| {
""",
     """            #[cfg(feature = "mi355x")]
            let gpu_payload = match (&gpu_batch, &plaintext_input_share) {
                (Some(_), Ok(plaintext_input_share)) => plaintext_input_share.payload().to_vec(),
                _ => Vec::new(),
            };

            let input_share = plaintext_input_share.and_then(|plaintext_input_share| {
"""),
    (AGG,
     """            let shares = input_share.and_then(|input_share| Ok((public_share?, input_share)));
""",
     """            let shares = input_share.and_then(|input_share| Ok((public_share?, input_share)));

            #[cfg(feature = "mi355x")]
            if let Some(batch) = gpu_batch.as_mut() {
                batch.push(
                    prepare_init.report_share().metadata().id().as_ref(),
                    prepare_init
                        .report_share()
                        .metadata()
                        .time()
                        .as_seconds_since_epoch(),
                    gpu_slot,
                    shares.map(|_| {
                        (
                            prepare_init.report_share().public_share(),
                            gpu_payload.as_slice(),
                        )
                    }),
                    prepare_init.message(),
                );
                continue;
            }
"""),
    (AGG,
     """            ));
        }

        // Store data to datastore.
""",
     """            ));
        }

        #[cfg(feature = "mi355x")]
        if let (Some(batch), Some(ops)) = (gpu_batch, gpu) {
            let outcome = batch
                .run(ops)
                .map_err(|error| Error::Internal(error.to_string()))?;
            for (ord, prepare_init) in req.prepare_inits().iter().enumerate() {
                let (report_aggregation_state, prepare_step_result) = match outcome.result(ord) {
                    Ok(message) => (
                        ReportAggregationState::Finished,
                        PrepareStepResult::Continue { message },
                    ),
                    Err(prepare_error) => (
                        ReportAggregationState::Failed(prepare_error),
                        PrepareStepResult::Reject(prepare_error),
                    ),
                };
                report_share_data.push(ReportShareData::new(
                    prepare_init.report_share().clone(),
                    ReportAggregation::<SEED_SIZE, A>::new(
                        *task.id(),
                        *aggregation_job_id,
                        *prepare_init.report_share().metadata().id(),
                        *prepare_init.report_share().metadata().time(),
                        ord.try_into()?,
                        Some(PrepareResp::new(
                            *prepare_init.report_share().metadata().id(),
                            prepare_step_result,
                        )),
                        report_aggregation_state,
                    ),
                ));
            }
            for (slot, (batch_identifier, aggregation)) in outcome.slots.iter().enumerate() {
                if aggregation.report_count == 0 {
                    continue;
                }
                accumulator.update_aggregated(
                    batch_identifier.clone(),
                    A::AggregateShare::get_decoded_with_param(
                        &(vdaf, &agg_param),
                        &aggregation.aggregate_share,
                    )?,
                    aggregation.report_count,
                    Interval::new(
                        janus_messages::Time::from_seconds_since_epoch(aggregation.interval_start),
                        Duration::from_seconds(aggregation.interval_duration),
                    )?,
                    ReportIdChecksum::from(aggregation.checksum),
                    outcome
                        .slot_report_ids(slot)
                        .into_iter()
                        .map(janus_messages::ReportId::from),
                )?;
            }
        }

        // Store data to datastore.
"""),

    # ---------------------------------------------------------------- accumulator
    (ACC,
     """    /// Write the accumulated aggregate shares, report counts and checksums to the datastore. If a
""",
     """    /// Merge a batch identifier's pre-aggregated share -- the MI355X engine's aggregate of a whole
    /// job's reports in one batch -- exactly as `update` merges one report's output share.
    #[cfg(feature = "mi355x")]
    pub fn update_aggregated(
        &mut self,
        batch_identifier: Q::BatchIdentifier,
        aggregate_share: A::AggregateShare,
        report_count: u64,
        client_timestamp_interval: Interval,
        checksum: ReportIdChecksum,
        report_ids: impl IntoIterator<Item = ReportId>,
    ) -> Result<(), datastore::Error> {
        let batch_aggregation = BatchAggregation::new(
            *self.task.id(),
            batch_identifier.clone(),
            self.aggregation_parameter.clone(),
            thread_rng().gen_range(0..self.shard_count),
            BatchAggregationState::Aggregating,
            Some(aggregate_share),
            report_count,
            client_timestamp_interval,
            checksum,
        );
        match self.aggregations.entry(batch_identifier) {
            std::collections::hash_map::Entry::Occupied(mut entry) => {
                let data = entry.get_mut();
                data.batch_aggregation = batch_aggregation.merged_with(&data.batch_aggregation)?;
                data.included_report_ids.extend(report_ids);
            }
            std::collections::hash_map::Entry::Vacant(entry) => {
                entry.insert(BatchData {
                    batch_aggregation,
                    included_report_ids: report_ids.into_iter().collect(),
                });
            }
        }
        Ok(())
    }

    /// Write the accumulated aggregate shares, report counts and checksums to the datastore. If a
"""),

    # ---------------------------------------------------------------- leader job driver
    (DRV,
     """    #[derivative(Debug = "ignore")]
    http_request_duration_histogram: Histogram<f64>,
}
""",
     """    #[derivative(Debug = "ignore")]
    http_request_duration_histogram: Histogram<f64>,
    /// The MI355X engines of the tasks this driver steps (`mi355x` feature).
    #[cfg(feature = "mi355x")]
    #[derivative(Debug = "ignore")]
    gpu: Option<Arc<crate::gpu::GpuTaskCache>>,
}
"""),
    (DRV,
     """            job_retry_counter,
            http_request_duration_histogram,
        }
    }
""",
     """            job_retry_counter,
            http_request_duration_histogram,
            #[cfg(feature = "mi355x")]
            gpu: None,
        }
    }

    /// Step Prio3 aggregate-init jobs on the MI355X engine (the `gpu:` config section).
    #[cfg(feature = "mi355x")]
    pub fn with_gpu(mut self, cfg: Option<crate::gpu::GpuConfig>) -> Self {
        self.gpu = cfg.map(|cfg| Arc::new(crate::gpu::GpuTaskCache::new(cfg)));
        self
    }
"""),
    (DRV,
     """                matches!(report_aggregation.state(), &ReportAggregationState::Start)
            })
            .collect();

        // Compute report shares to send to helper, and decrypt our input shares & initialize
        // preparation state.
        let mut report_aggregations_to_write = Vec::new();
        let mut prepare_inits = Vec::new();
        let mut stepped_aggregations = Vec::new();
""",
     """                matches!(report_aggregation.state(), &ReportAggregationState::Start)
            })
            .collect();

        // MI355X: the reports that pass the checks below are gathered and initialised by ONE
        // engine call after the loop.
        #[cfg(feature = "mi355x")]
        let gpu = match &self.gpu {
            Some(cache) => cache.ops_for(task.id().as_ref(), task.vdaf(), verify_key.as_bytes())?,
            None => None,
        };
        #[cfg(feature = "mi355x")]
        let mut gpu_batch = gpu
            .as_deref()
            .map(|ops| crate::gpu::LeaderBatch::new(ops, report_aggregations.len()));
        #[cfg(feature = "mi355x")]
        let (mut gpu_reports, mut gpu_stepped) = (Vec::new(), Vec::new());

        // Compute report shares to send to helper, and decrypt our input shares & initialize
        // preparation state.
        let mut report_aggregations_to_write = Vec::new();
        let mut prepare_inits = Vec::new();
        let mut stepped_aggregations = Vec::new();
"""),
    (DRV,
     """        for report_aggregation in report_aggregations {
            // Look up report.
            let report = if let Some(report) = client_reports.get(report_aggregation.report_id()) {
""",
     """        for report_aggregation in report_aggregations {
            // MI355X: the report as stored (undecoded, `get_client_report_raw`) goes into the
            // job's engine batch after the same per-report checks as below; the engine validates
            // the encodings itself (a non-canonical element fails that report: InvalidMessage)
            #[cfg(feature = "mi355x")]
            if let Some(batch) = gpu_batch.as_mut() {
                let report = match raw_reports.remove(report_aggregation.report_id()) {
                    Some(report) => report,
                    None => {
                        info!(report_id = %report_aggregation.report_id(), "Attempted to aggregate missing report (most likely garbage collected)");
                        self.aggregate_step_failure_counter
                            .add(1, &[KeyValue::new("type", "missing_client_report")]);
                        report_aggregations_to_write.push(report_aggregation.with_state(
                            ReportAggregationState::Failed(PrepareError::ReportDropped),
                        ));
                        continue;
                    }
                };
                let mut extension_types = HashSet::new();
                if !report
                    .extensions
                    .iter()
                    .all(|extension| extension_types.insert(extension.extension_type()))
                {
                    info!(report_id = %report_aggregation.report_id(), "Received report with duplicate extensions");
                    self.aggregate_step_failure_counter
                        .add(1, &[KeyValue::new("type", "duplicate_extension")]);
                    report_aggregations_to_write.push(report_aggregation.with_state(
                        ReportAggregationState::Failed(PrepareError::InvalidMessage),
                    ));
                    continue;
                }
                batch.push(
                    report.metadata.id().as_ref(),
                    report.metadata.time().as_seconds_since_epoch(),
                    &report.public_share,
                    &report.leader_input_share,
                );
                gpu_reports.push((report_aggregation, report));
                continue;
            }

            // Look up report.
            let report = if let Some(report) = client_reports.get(report_aggregation.report_id()) {
"""),
    (DRV,
     """        // Construct request, send it to the helper, and process the response.
        // TODO(#235): abandon work immediately on "terminal" failures from helper, or other
        // unexpected cases such as unknown/unexpected content type.
        let req = AggregationJobInitializeReq::<Q>::new(
""",
     """        #[cfg(feature = "mi355x")]
        let gpu_init = match (gpu_batch, gpu.as_deref()) {
            (Some(batch), Some(ops)) => {
                let init = batch.run(ops)?;
                for (i, (report_aggregation, report)) in gpu_reports.into_iter().enumerate() {
                    match init.message(i) {
                        Ok(ping_pong_message) => {
                            prepare_inits.push(PrepareInit::new(
                                ReportShare::new(
                                    report.metadata,
                                    report.public_share,
                                    report.helper_encrypted_input_share,
                                ),
                                ping_pong_message,
                            ));
                            gpu_stepped.push((i, report_aggregation));
                        }
                        Err(prep_error) => report_aggregations_to_write.push(
                            report_aggregation
                                .with_state(ReportAggregationState::Failed(prep_error)),
                        ),
                    }
                }
                Some(init)
            }
            _ => None,
        };

        // Construct request, send it to the helper, and process the response.
        // TODO(#235): abandon work immediately on "terminal" failures from helper, or other
        // unexpected cases such as unknown/unexpected content type.
        let req = AggregationJobInitializeReq::<Q>::new(
"""),
    (DRV,
     """        let resp = AggregationJobResp::get_decoded(&resp_bytes)?;

        self.process_response_from_helper(
            datastore,
            vdaf,
            lease,
            task,
            aggregation_job,
            &stepped_aggregations,
            report_aggregations_to_write,
            resp.prepare_resps(),
        )
        .await
    }

    async fn step_aggregation_job_aggregate_continue<
""",
     """        let resp = AggregationJobResp::get_decoded(&resp_bytes)?;

        #[cfg(feature = "mi355x")]
        if let (Some(init), Some(ops)) = (gpu_init, gpu.as_deref()) {
            return self
                .process_response_from_helper_gpu(
                    datastore,
                    vdaf,
                    lease,
                    task,
                    aggregation_job,
                    ops,
                    init,
                    gpu_stepped,
                    report_aggregations_to_write,
                    resp.prepare_resps(),
                )
                .await;
        }

        self.process_response_from_helper(
            datastore,
            vdaf,
            lease,
            task,
            aggregation_job,
            &stepped_aggregations,
            report_aggregations_to_write,
            resp.prepare_resps(),
        )
        .await
    }

    async fn step_aggregation_job_aggregate_continue<
"""),
    (DRV,
     """        // Write everything back to storage.
        let mut aggregation_job_writer = AggregationJobWriter::new(Arc::clone(&task));
""",
     """        self.write_step_results(
            datastore,
            vdaf,
            lease,
            task,
            aggregation_job,
            report_aggregations_to_write,
            accumulator,
        )
        .await
    }

    /// `process_response_from_helper` for a job the MI355X engine initialised: the helper's
    /// answers checked and mapped per report as above, then ONE `prepare_next` + accumulate +
    /// report bookkeeping for the job.
    #[cfg(feature = "mi355x")]
    #[allow(clippy::too_many_arguments)]
    async fn process_response_from_helper_gpu<
        const SEED_SIZE: usize,
        C: Clock,
        Q: CollectableQueryType,
        A: vdaf::Aggregator<SEED_SIZE, 16> + Send + Sync + 'static,
    >(
        &self,
        datastore: &Datastore<C>,
        vdaf: Arc<A>,
        lease: Arc<Lease<AcquiredAggregationJob>>,
        task: Arc<Task>,
        aggregation_job: AggregationJob<SEED_SIZE, Q, A>,
        gpu: &crate::gpu::GpuVdafOps,
        init: crate::gpu::LeaderInitOutcome,
        stepped: Vec<(usize, ReportAggregation<SEED_SIZE, A>)>,
        mut report_aggregations_to_write: Vec<ReportAggregation<SEED_SIZE, A>>,
        helper_prep_resps: &[PrepareResp],
    ) -> Result<()>
    where
        A: 'static,
        A::AggregationParam: Send + Sync + Eq + PartialEq,
        A::AggregateShare: Send + Sync,
        A::OutputShare: Send + Sync,
        A::PrepareMessage: Send + Sync,
        A::PrepareShare: Send + Sync,
        A::PrepareState: Send + Sync + Encode,
    {
        if stepped.len() != helper_prep_resps.len() {
            return Err(anyhow!(
                "missing, duplicate, out-of-order, or unexpected prepare steps in response"
            ));
        }
        let mut finish = crate::gpu::LeaderFinishBatch::new(gpu, init);
        for ((i, report_aggregation), helper_prep_resp) in stepped.iter().zip(helper_prep_resps) {
            if helper_prep_resp.report_id() != report_aggregation.report_id() {
                return Err(anyhow!(
                    "missing, duplicate, out-of-order, or unexpected prepare steps in response"
                ));
            }
            let helper_message = match helper_prep_resp.result() {
                PrepareStepResult::Continue { message } => Ok(message),
                PrepareStepResult::Finished => {
                    warn!(
                        report_id = %report_aggregation.report_id(),
                        "Helper finished but Leader did not",
                    );
                    self.aggregate_step_failure_counter
                        .add(1, &[KeyValue::new("type", "finish_mismatch")]);
                    Err(PrepareError::VdafPrepError)
                }
                PrepareStepResult::Reject(err) => {
                    info!(
                        report_id = %report_aggregation.report_id(),
                        helper_error = ?err,
                        "Helper couldn't step report aggregation",
                    );
                    self.aggregate_step_failure_counter
                        .add(1, &[KeyValue::new("type", "helper_step_failure")]);
                    Err(*err)
                }
            };
            let batch_identifier = Q::to_batch_identifier(
                &task,
                aggregation_job.partial_batch_identifier(),
                report_aggregation.time(),
            )?;
            finish.push(*i, &batch_identifier, helper_message);
        }
        let outcome = finish.run(gpu)?;

        let mut accumulator = Accumulator::<SEED_SIZE, Q, A>::new(
            Arc::clone(&task),
            self.batch_aggregation_shard_count,
            aggregation_job.aggregation_parameter().clone(),
        );
        for (slot, (batch_identifier, aggregation)) in outcome.slots.iter().enumerate() {
            if aggregation.report_count == 0 {
                continue;
            }
            accumulator.update_aggregated(
                batch_identifier.clone(),
                A::AggregateShare::get_decoded_with_param(
                    &(vdaf.as_ref(), aggregation_job.aggregation_parameter()),
                    &aggregation.aggregate_share,
                )?,
                aggregation.report_count,
                janus_messages::Interval::new(
                    janus_messages::Time::from_seconds_since_epoch(aggregation.interval_start),
                    janus_messages::Duration::from_seconds(aggregation.interval_duration),
                )?,
                janus_messages::ReportIdChecksum::from(aggregation.checksum),
                outcome
                    .slot_report_ids(slot)
                    .into_iter()
                    .map(ReportId::from),
            )?;
        }
        for (i, report_aggregation) in stepped {
            let new_state = match outcome.finished(i) {
                Ok(()) => ReportAggregationState::Finished,
                Err(prepare_error) => ReportAggregationState::Failed(prepare_error),
            };
            report_aggregations_to_write.push(report_aggregation.with_state(new_state));
        }

        self.write_step_results(
            datastore,
            vdaf,
            lease,
            task,
            aggregation_job,
            report_aggregations_to_write,
            accumulator,
        )
        .await
    }

    /// Write a stepped job's report aggregations, batch aggregations and lease release back to
    /// storage: the tail of `process_response_from_helper`, shared with the MI355X path.
    #[allow(clippy::too_many_arguments)]
    async fn write_step_results<
        const SEED_SIZE: usize,
        C: Clock,
        Q: CollectableQueryType,
        A: vdaf::Aggregator<SEED_SIZE, 16> + Send + Sync + 'static,
    >(
        &self,
        datastore: &Datastore<C>,
        vdaf: Arc<A>,
        lease: Arc<Lease<AcquiredAggregationJob>>,
        task: Arc<Task>,
        aggregation_job: AggregationJob<SEED_SIZE, Q, A>,
        report_aggregations_to_write: Vec<ReportAggregation<SEED_SIZE, A>>,
        accumulator: Accumulator<SEED_SIZE, Q, A>,
    ) -> Result<()>
    where
        A: 'static,
        A::AggregationParam: Send + Sync + Eq + PartialEq,
        A::AggregateShare: Send + Sync,
        A::OutputShare: Send + Sync,
        A::PrepareMessage: Send + Sync,
        A::PrepareShare: Send + Sync,
        A::PrepareState: Send + Sync + Encode,
    {
        // Write everything back to storage.
        let mut aggregation_job_writer = AggregationJobWriter::new(Arc::clone(&task));
"""),

    # ---------------------------------------------------------------- binaries: gpu config
    ("aggregator/src/bin/aggregator.rs",
     """    #[serde(default)]
    global_hpke_configs_refresh_interval: Option<u64>,
}
""",
     """    #[serde(default)]
    global_hpke_configs_refresh_interval: Option<u64>,

    /// The MI355X engine for Prio3 aggregate-init (`mi355x` feature): `device`, `workers`,
    /// `max_job_size`.  Absent: the CPU path.
    #[cfg(feature = "mi355x")]
    #[serde(default)]
    gpu: Option<janus_aggregator::gpu::GpuConfig>,
}
"""),
    ("aggregator/src/bin/aggregator.rs",
     """                None => GlobalHpkeKeypairCache::DEFAULT_REFRESH_INTERVAL,
            },
        }
    }
}
""",
     """                None => GlobalHpkeKeypairCache::DEFAULT_REFRESH_INTERVAL,
            },
            #[cfg(feature = "mi355x")]
            gpu: self.gpu,
        }
    }
}
"""),
    ("aggregator/src/bin/aggregator.rs",
     """            global_hpke_configs_refresh_interval: None,
        })
""",
     """            global_hpke_configs_refresh_interval: None,
            #[cfg(feature = "mi355x")]
            gpu: None,
        })
"""),
    ("aggregator/src/bin/aggregation_job_driver.rs",
     """        let aggregation_job_driver = Arc::new(AggregationJobDriver::new(
            reqwest::Client::builder()
                .user_agent(CLIENT_USER_AGENT)
                .build()
                .context("couldn't create HTTP client")?,
            &ctx.meter,
            ctx.config.batch_aggregation_shard_count,
        ));
""",
     """        let aggregation_job_driver = AggregationJobDriver::new(
            reqwest::Client::builder()
                .user_agent(CLIENT_USER_AGENT)
                .build()
                .context("couldn't create HTTP client")?,
            &ctx.meter,
            ctx.config.batch_aggregation_shard_count,
        );
        #[cfg(feature = "mi355x")]
        let aggregation_job_driver = aggregation_job_driver.with_gpu(ctx.config.gpu);
        let aggregation_job_driver = Arc::new(aggregation_job_driver);
"""),
    ("aggregator/src/bin/aggregation_job_driver.rs",
     """    /// the cost of collection.
    batch_aggregation_shard_count: u64,
}
""",
     """    /// the cost of collection.
    batch_aggregation_shard_count: u64,

    /// The MI355X engine for Prio3 aggregate-init (`mi355x` feature): `device`, `workers` (set it
    /// to `max_concurrent_job_workers`), `max_job_size` (>= the jobs' size).  Absent: the CPU
    /// path.
    #[cfg(feature = "mi355x")]
    #[serde(default)]
    gpu: Option<janus_aggregator::gpu::GpuConfig>,
}
"""),
    ("aggregator/src/bin/aggregation_job_driver.rs",
     """            batch_aggregation_shard_count: 32,
            taskprov_config: TaskprovConfig::default(),
        })
""",
     """            batch_aggregation_shard_count: 32,
            taskprov_config: TaskprovConfig::default(),
            #[cfg(feature = "mi355x")]
            gpu: None,
        })
"""),
    # ---------------------------------------------------------------- datastore: raw leader read
    (DS,
     """use tracing::error;
use url::Url;
""",
     """use tracing::error;
use url::Url;

/// A leader's client report as stored, its VDAF shares NOT decoded (`mi355x` feature): the
/// MI355X engine takes the encodings as they are and validates them per report, so the leader
/// skips `get_decoded_with_param` (a range check and Montgomery conversion of every field
/// element) and the re-encoding the engine call would otherwise need.
#[cfg(feature = "mi355x")]
#[derive(Clone, Debug)]
pub struct RawLeaderStoredReport {
    pub metadata: ReportMetadata,
    pub extensions: Vec<Extension>,
    /// `client_reports.public_share`, as stored
    pub public_share: Vec<u8>,
    /// `client_reports.leader_input_share`, as stored
    pub leader_input_share: Vec<u8>,
    pub helper_encrypted_input_share: HpkeCiphertext,
}
"""),
    (DS,
     """        .map(|row| Self::client_report_from_row(vdaf, *task_id, *report_id, row))
        .transpose()
    }
""",
     """        .map(|row| Self::client_report_from_row(vdaf, *task_id, *report_id, row))
        .transpose()
    }

    /// `get_client_report` for the MI355X leader feed (`mi355x` feature): the same row, with the
    /// public share and leader input share returned as stored instead of decoded
    /// (`client_report_from_row` decodes them).  The extensions and the helper's ciphertext are
    /// decoded as before: the driver checks the one and forwards the other.
    #[cfg(feature = "mi355x")]
    #[tracing::instrument(skip(self), err)]
    pub async fn get_client_report_raw(
        &self,
        task_id: &TaskId,
        report_id: &ReportId,
    ) -> Result<Option<RawLeaderStoredReport>, Error> {
        let stmt = self
            .prepare_cached(
                "SELECT
                    client_reports.client_timestamp,
                    client_reports.extensions,
                    client_reports.public_share,
                    client_reports.leader_input_share,
                    client_reports.helper_encrypted_input_share
                FROM client_reports
                JOIN tasks ON tasks.id = client_reports.task_id
                WHERE tasks.task_id = $1
                  AND client_reports.report_id = $2
                  AND client_reports.client_timestamp >= COALESCE($3::TIMESTAMP - tasks.report_expiry_age * '1 second'::INTERVAL, '-infinity'::TIMESTAMP)",
            )
            .await?;
        self.query_opt(
            &stmt,
            &[
                /* task_id */ &task_id.as_ref(),
                /* report_id */ &report_id.as_ref(),
                /* now */ &self.clock.now().as_naive_date_time()?,
            ],
        )
        .await?
        .map(|row| {
            let time = Time::from_naive_date_time(&row.get("client_timestamp"));
            let encoded_extensions: Vec<u8> = row.get("extensions");
            let extensions: Vec<Extension> =
                decode_u16_items(&(), &mut Cursor::new(&encoded_extensions))?;
            let encoded_helper_input_share: Vec<u8> = row.get("helper_encrypted_input_share");
            Ok(RawLeaderStoredReport {
                metadata: ReportMetadata::new(*report_id, time),
                extensions,
                public_share: row.get("public_share"),
                leader_input_share: row.get("leader_input_share"),
                helper_encrypted_input_share: HpkeCiphertext::get_decoded(
                    &encoded_helper_input_share,
                )?,
            })
        })
        .transpose()
    }
"""),

    # ---------------------------------------------------------------- driver: raw leader read
    (DRV,
     """use super::error::handle_ping_pong_error;
""",
     """use super::error::handle_ping_pong_error;

/// The undecoded client reports of a job whose VDAF the MI355X engine runs (`mi355x` feature;
/// `()` without it, so the default build carries nothing).
#[cfg(feature = "mi355x")]
type RawReports = HashMap<ReportId, janus_aggregator_core::datastore::RawLeaderStoredReport>;
#[cfg(not(feature = "mi355x"))]
type RawReports = ();
"""),
    (DRV,
     """        // Read all information about the aggregation job.
        let (task, aggregation_job, report_aggregations, client_reports, verify_key) = datastore
            .run_tx_with_name("step_aggregation_job_1", |tx| {
""",
     """        // MI355X: a task whose VDAF the engine runs reads its reports undecoded (raw_reports)
        #[cfg(feature = "mi355x")]
        let gpu_wanted =
            self.gpu.is_some() && crate::gpu::engine_params(lease.leased().vdaf()).is_some();

        // Read all information about the aggregation job.
        let (task, aggregation_job, report_aggregations, client_reports, raw_reports, verify_key) =
            datastore
            .run_tx_with_name("step_aggregation_job_1", |tx| {
"""),
    (DRV,
     """                    // Read client reports, but only for report aggregations in state START.
                    // TODO(#224): create "get_client_reports_for_aggregation_job" datastore
                    // operation to avoid needing to join many futures?
                    let client_reports: HashMap<_, _> =
                        try_join_all(report_aggregations.iter().filter_map(|report_aggregation| {
""",
     """                    // MI355X: the engine's tasks (Prio3, 16-byte verify keys: exactly those
                    // `GpuTaskCache::ops_for` gives arms) read their START reports undecoded and
                    // leave the decoded map empty
                    #[cfg(feature = "mi355x")]
                    let raw = gpu_wanted && verify_key.as_bytes().len() == 16;
                    #[cfg(not(feature = "mi355x"))]
                    let raw = false;
                    #[cfg(feature = "mi355x")]
                    let raw_reports: RawReports = if raw {
                        try_join_all(
                            report_aggregations
                                .iter()
                                .filter(|report_aggregation| {
                                    matches!(
                                        report_aggregation.state(),
                                        &ReportAggregationState::Start
                                    )
                                })
                                .map(|report_aggregation| {
                                    tx.get_client_report_raw(
                                        lease.leased().task_id(),
                                        report_aggregation.report_id(),
                                    )
                                    .map(|rslt| {
                                        rslt.map(|report| {
                                            report.map(|report| {
                                                (*report_aggregation.report_id(), report)
                                            })
                                        })
                                    })
                                }),
                        )
                        .await?
                        .into_iter()
                        .flatten()
                        .collect()
                    } else {
                        HashMap::new()
                    };
                    #[cfg(not(feature = "mi355x"))]
                    let raw_reports: RawReports = ();

                    // Read client reports, but only for report aggregations in state START.
                    // TODO(#224): create "get_client_reports_for_aggregation_job" datastore
                    // operation to avoid needing to join many futures?
                    let client_reports: HashMap<_, _> = if raw { HashMap::new() } else {
                        try_join_all(report_aggregations.iter().filter_map(|report_aggregation| {
"""),
    (DRV,
     """                        .flatten()
                        .collect();

                    Ok((
                        Arc::new(task),
                        aggregation_job,
                        report_aggregations,
                        client_reports,
                        verify_key,
                    ))
""",
     """                        .flatten()
                        .collect()
                    };

                    Ok((
                        Arc::new(task),
                        aggregation_job,
                        report_aggregations,
                        client_reports,
                        raw_reports,
                        verify_key,
                    ))
"""),
    (DRV,
     """                    report_aggregations,
                    client_reports,
                    verify_key,
                )
                .await
""",
     """                    report_aggregations,
                    client_reports,
                    raw_reports,
                    verify_key,
                )
                .await
"""),
    (DRV,
     """        client_reports: HashMap<ReportId, LeaderStoredReport<SEED_SIZE, A>>,
        verify_key: VerifyKey<SEED_SIZE>,
    ) -> Result<()>
""",
     """        client_reports: HashMap<ReportId, LeaderStoredReport<SEED_SIZE, A>>,
        #[allow(unused_mut, unused_variables)] mut raw_reports: RawReports,
        verify_key: VerifyKey<SEED_SIZE>,
    ) -> Result<()>
"""),
]


def build(reference):
    files = {}
    for path, old, new in EDITS:
        if path not in files:
            with open(os.path.join(reference, path)) as f:
                files[path] = [f.read(), None]
        cur = files[path][1] if files[path][1] is not None else files[path][0]
        n = cur.count(old)
        if n != 1:
            raise SystemExit(f"{path}: anchor matches {n} times:\n{old}")
        files[path][1] = cur.replace(old, new)
    out = []
    for path in sorted(files):
        a, b = files[path]
        out.extend(difflib.unified_diff(a.splitlines(keepends=True), b.splitlines(keepends=True),
                                        f"a/{path}", f"b/{path}", n=3))
    return "".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    text = build(a.reference)
    if a.check:
        with open(PATCH) as f:
            if f.read() != text:
                print("janus-0.6-mi355x.patch is stale: rerun make_patch.py", file=sys.stderr)
                return 1
        return 0
    with open(PATCH, "w") as f:
        f.write(text)
    print(f"wrote {PATCH}: {text.count(chr(10))} lines")
    return 0


if __name__ == "__main__":
    sys.exit(main())

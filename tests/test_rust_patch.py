"""The reference-side binding as a checked patch (rust/patches/janus-0.6-mi355x.patch).

No cargo/rustc exists in this image, so the patch is checked mechanically (CPU only):
  * it is the output of rust/patches/make_patch.py over the reference sources (not stale);
  * `git apply --check` accepts it on a copy of the files it touches under /root/reference, and
    applying it leaves every new line behind `#[cfg(feature = "mi355x")]` (the default build is
    the reference's);
  * every `crate::gpu::` / `janus_aggregator::gpu::` item it names is a `pub` item of
    rust/aggregator/src/gpu/mod.rs, and every method it calls on an engine object -- and on the
    functions the patch itself adds -- exists with the argument count the call passes.

Reference call sites: aggregator/src/aggregator.rs:797-900 (TaskAggregator::new), :1613-1848
(handle_aggregate_init_generic's per-report loop), aggregator/src/aggregator/
aggregation_job_driver.rs:329-402, :530-727 (leader init and response), accumulator.rs:76-122.
The tests skip when /root/reference is absent (it does not travel to the GPU box)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "rust", "patches", "janus-0.6-mi355x.patch")
MOD = os.path.join(ROOT, "rust", "aggregator", "src", "gpu", "mod.rs")

needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")


def patch_files():
    """{path: [added lines]} of the patch."""
    out, cur = {}, None
    for line in open(PATCH):
        if line.startswith("+++ b/"):
            cur = line[6:].strip()
            out[cur] = []
        elif line.startswith("+") and not line.startswith("+++") and cur:
            out[cur].append(line[1:].rstrip("\n"))
    return out


def split_args(s):
    """Top-level comma split of an argument / parameter list (nesting: () [] <> {})."""
    depth, cur, parts = 0, "", []
    i = 0
    while i < len(s):
        c = s[i]
        if s.startswith("->", i):
            cur += "->"
            i += 2
            continue
        if c in "([<{":
            depth += 1
        elif c in ")]>}":
            depth -= 1
        if c == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def paren_body(text, start):
    """The text inside the parenthesis opening at text[start] == '('."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "(":
            depth += 1
        elif text[i] == ")":
            depth -= 1
            if depth == 0:
                return text[start + 1:i]
    raise ValueError("unbalanced")


def fn_arities(text):
    """{fn name: [arities]} of `fn name<...>(params)` definitions, `self` receivers excluded."""
    out = {}
    for m in re.finditer(r"\bfn\s+(\w+)\s*(<[^{;]*?>)?\s*\(", text):
        params = split_args(paren_body(text, m.end() - 1))
        params = [p for p in params if not re.match(r"^(mut\s+)?&?\s*(mut\s+)?(\'\w+\s+)?self\b", p)]
        out.setdefault(m.group(1), []).append(len(params))
    return out


def impl_methods(text):
    """{type name: {method: arity}} of the inherent impl blocks of mod.rs."""
    out = {}
    for m in re.finditer(r"^impl(?:<[^>]*>)?\s+(\w+)(?:<[^>]*>)?\s*\{", text, re.M):
        depth, i = 0, m.end() - 1
        for j in range(i, len(text)):
            if text[j] == "{":
                depth += 1
            elif text[j] == "}":
                depth -= 1
                if depth == 0:
                    break
        body = text[i:j]
        for name, ar in fn_arities(body).items():
            out.setdefault(m.group(1), {})[name] = ar[0]
    return out


def pub_items(text):
    return set(re.findall(r"^pub\s+(?:struct|enum|fn|const|type)\s+(\w+)", text, re.M))


@needs_ref
def test_patch_is_generated_from_the_reference():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "rust", "patches", "make_patch.py"),
                        "--reference", REF, "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@needs_ref
def test_patch_applies_to_the_reference(tmp_path):
    files = list(patch_files())
    assert set(files) == {
        "aggregator/Cargo.toml", "aggregator/src/lib.rs", "aggregator/src/aggregator.rs",
        "aggregator/src/aggregator/accumulator.rs",
        "aggregator/src/aggregator/aggregation_job_driver.rs",
        "aggregator/src/bin/aggregator.rs", "aggregator/src/bin/aggregation_job_driver.rs",
        "aggregator_core/Cargo.toml", "aggregator_core/src/datastore.rs"}
    for f in files:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    subprocess.run(["git", "init", "-q", str(tmp_path)], check=True)
    r = subprocess.run(["git", "-C", str(tmp_path), "apply", "--check", PATCH],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    subprocess.run(["git", "-C", str(tmp_path), "apply", PATCH], check=True)
    toml = (tmp_path / "aggregator/Cargo.toml").read_text()
    features = toml[toml.index("[features]"):]
    features = features[:features.index("\n[", 1)]
    assert '\nmi355x = ["janus_aggregator_core/mi355x"]\n' in features
    core = (tmp_path / "aggregator_core/Cargo.toml").read_text()
    core = core[core.index("[features]"):]
    assert "\nmi355x = []\n" in core[:core.index("\n[", 1)]
    lib = (tmp_path / "aggregator/src/lib.rs").read_text()
    assert '#[cfg(feature = "mi355x")]\npub mod gpu;' in lib
    # every item the patch adds to a Rust file sits behind the feature: the added lines outside a
    # cfg'd item are only call arguments / fields already under one, or the shared storage tail
    agg = (tmp_path / "aggregator/src/aggregator.rs").read_text()
    assert agg.count('#[cfg(feature = "mi355x")]') >= 10
    drv = (tmp_path / "aggregator/src/aggregator/aggregation_job_driver.rs").read_text()
    assert "async fn write_step_results<" in drv and "async fn process_response_from_helper_gpu<" in drv
    assert drv.count("self.write_step_results(") == 2


def test_patch_names_only_existing_gpu_items():
    mod = open(MOD).read()
    items = pub_items(mod)
    added = patch_files()
    used = set()
    for lines in added.values():
        for m in re.finditer(r"\b(?:crate|janus_aggregator)::gpu::(\w+)", "\n".join(lines)):
            used.add(m.group(1))
    assert used, "the patch names no gpu items"
    assert used <= items, used - items
    # the patch's constructor calls: crate::gpu::X::new(args)
    methods = impl_methods(mod)
    for lines in added.values():
        text = "\n".join(lines)
        for m in re.finditer(r"\bcrate::gpu::(\w+)::(\w+)\s*\(", text):
            typ, fn = m.groups()
            n = len(split_args(paren_body(text, m.end() - 1)))
            assert methods[typ][fn] == n, (typ, fn, n)


# receivers of engine objects in the patch, per file -> the mod.rs (or patch-added) type
RECEIVERS = {
    "aggregator/src/aggregator.rs": {"batch": "HelperBatch", "outcome": "JobOutcome",
                                     "cfg": "GpuConfig", "accumulator": "Accumulator",
                                     "task_agg": "TaskAggregator"},
    "aggregator/src/aggregator/aggregation_job_driver.rs": {
        "batch": "LeaderBatch", "init": "LeaderInitOutcome", "finish": "LeaderFinishBatch",
        "outcome": "JobOutcome", "cache": "GpuTaskCache", "accumulator": "Accumulator",
        "self": "AggregationJobDriver"},
    "aggregator/src/bin/aggregation_job_driver.rs": {
        "aggregation_job_driver": "AggregationJobDriver"},
    "aggregator_core/src/datastore.rs": {},
}
# methods the patch adds to reference types: (type) -> {method: arity}, read from the patch
PATCH_TYPES = {"Accumulator": "aggregator/src/aggregator/accumulator.rs",
               "AggregationJobDriver": "aggregator/src/aggregator/aggregation_job_driver.rs",
               "TaskAggregator": "aggregator/src/aggregator.rs"}
STD = {"as_mut", "as_deref", "map", "map_or", "clone", "into_iter", "iter", "enumerate", "len",
       "push", "await", "as_ref", "to_vec", "get_encoded", "metadata", "report_id", "result",
       "time", "state", "with_state", "zip", "collect", "as_seconds_since_epoch", "message",
       "add", "slot_of", "filter"}


def test_patch_calls_match_engine_signatures():
    mod = open(MOD).read()
    methods = impl_methods(mod)
    added = patch_files()
    for typ, f in PATCH_TYPES.items():
        methods.setdefault(typ, {}).update(
            {k: v[0] for k, v in fn_arities("\n".join(added[f])).items()})
    checked = 0
    for f, recv in RECEIVERS.items():
        text = "\n".join(added[f])
        for m in re.finditer(r"\b(\w+)\s*\.\s*(\w+)\s*\(", text):
            obj, meth = m.groups()
            typ = recv.get(obj)
            if typ is None:
                continue
            if meth not in methods.get(typ, {}):
                # std / reference methods on the same receivers (e.g. `self.aggregate_step_...`)
                assert typ not in ("HelperBatch", "LeaderBatch", "LeaderFinishBatch",
                                   "LeaderInitOutcome", "JobOutcome", "GpuTaskCache",
                                   "GpuConfig") or meth in STD, (f, obj, meth)
                continue
            n = len(split_args(paren_body(text, m.end() - 1)))
            assert methods[typ][meth] == n, (f, obj, meth, n, methods[typ][meth])
            checked += 1
    # batch.push / slot_of / run, outcome.result / slot_report_ids / finished, init.message,
    # finish.push / run, cache.ops_for, accumulator.update_aggregated, self.write_step_results ...
    assert checked >= 15, checked


def test_mod_rs_status_mapping_covers_prepare_error():
    """status_of / prepare_error round-trip every PrepareError of messages/src/lib.rs:2288-2298
    (BatchCollected's DAP code 0 is the engine's "ok", so it gets a private status)."""
    mod = open(MOD).read()
    body = mod[mod.index("pub fn prepare_error"):]
    body = body[:body.index("\n}\n")]
    got = dict((int(c), n) for c, n in re.findall(r"(\d+) => PrepareError::(\w+)", body))
    assert got == {1: "ReportReplayed", 2: "ReportDropped", 3: "HpkeUnknownConfigId",
                   4: "HpkeDecryptError", 6: "BatchSaturated", 7: "TaskExpired",
                   8: "InvalidMessage"}
    assert "STATUS_BATCH_COLLECTED => PrepareError::BatchCollected" in body
    assert "_ => PrepareError::VdafPrepError" in body


@needs_ref
def test_leader_feed_reads_reports_undecoded(tmp_path):
    """The leader's engine batch is fed the stored encodings: a
    `get_client_report_raw` datastore read (the columns of aggregator_core/src/datastore.rs:
    1162-1199 without `get_decoded_with_param`, :1297-1304) behind the feature, called by the job
    step for the engine's tasks, whose rows go to `LeaderBatch::push` as they are -- no
    decode/re-encode of the 135 KB SumVec leader share in Rust."""
    added = patch_files()
    ds = "\n".join(added["aggregator_core/src/datastore.rs"])
    drv = "\n".join(added["aggregator/src/aggregator/aggregation_job_driver.rs"])
    # the accessor and its row type, both behind the feature
    assert re.search(r'#\[cfg\(feature = "mi355x"\)\]\n#\[derive\(Clone, Debug\)\]\n'
                     r'pub struct RawLeaderStoredReport \{', ds)
    fields = set(re.findall(r"^    pub (\w+):", ds[ds.index("pub struct RawLeaderStoredReport"):],
                            re.M))
    assert fields == {"metadata", "extensions", "public_share", "leader_input_share",
                      "helper_encrypted_input_share"}
    acc = ds[ds.index("pub async fn get_client_report_raw("):]
    assert '#[cfg(feature = "mi355x")]' in ds[:ds.index("pub async fn get_client_report_raw(")]
    assert len(split_args(paren_body(acc, acc.index("(")))) == 3  # &self, task_id, report_id
    if "\n    }\n" in acc:  # (the diff may share the closing lines with the previous fn)
        acc = acc[:acc.index("\n    }\n")]
    assert "get_decoded_with_param" not in acc
    assert 'public_share: row.get("public_share")' in acc
    assert 'leader_input_share: row.get("leader_input_share")' in acc
    # the job step reads through it and pushes the raw rows; the decoded read is skipped
    assert "tx.get_client_report_raw(" in drv
    assert "let client_reports: HashMap<_, _> = if raw { HashMap::new() } else {" in drv
    push = drv[drv.index("batch.push("):]
    push = paren_body(push, push.index("("))
    assert split_args(push)[2:] == ["&report.public_share", "&report.leader_input_share"]
    assert "leader_input_share().get_encoded()" not in drv
    # every field the driver reads from a raw report exists
    used = set(re.findall(r"\breport\.(\w+)\b(?!\s*\()", drv))
    assert used <= fields, used - fields
    # LeaderBatch::push takes (report id, time, public share, leader input share)
    assert impl_methods(open(MOD).read())["LeaderBatch"]["push"] == 4

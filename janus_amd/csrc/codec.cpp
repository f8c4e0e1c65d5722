// DAP-07 codec edge of the aggregate-init path: batched decode of
// AggregationJobInitializeReq / PlaintextInputShare / AggregationJobResp straight into the
// engine's report-major input arrays, and encode of the messages built from its outputs.
// Host code (no GPU), part of libprio3gpu.so; C ABI in include/prio3gpu.h.
//
// Wire formats (Janus 0.6 messages/src/lib.rs; TLS-style big-endian lengths, u32/u16-prefixed
// byte lists whose prefix is the BYTE length of the encoded items):
//   AggregationJobInitializeReq  u32 opaque agg_param | PartialBatchSelector | u32 PrepareInit list
//                                (lib.rs:2432-2500)
//   PartialBatchSelector         u8 query type (1 TimeInterval, 2 FixedSize + BatchId[32])
//                                (lib.rs:1562-1620, query type codes lib.rs:2024-2028)
//   PrepareInit                  ReportShare | PingPongMessage (lib.rs:2139-2185)
//   ReportShare                  ReportId[16] | Time u64 | u32 opaque public share |
//                                HpkeCiphertext{u8 config id, u16 opaque enc, u32 opaque payload}
//                                (lib.rs:2068-2135, :915-990, :1209-1250)
//   PingPongMessage              u8 type: 0 Initialize{u32 prep_share} | 1 Continue{u32 prep_msg,
//                                u32 prep_share} | 2 Finish{u32 prep_msg} (lib.rs:4094-4267 KATs)
//   PlaintextInputShare          u16 list of Extension{u16 type, u16 opaque data} | u32 payload
//                                (lib.rs:1253-1300, :837-880)
//   AggregationJobResp           u32 PrepareResp list (lib.rs:2619-2660)
//   PrepareResp                  ReportId[16] | u8 result: 0 Continue{PingPongMessage} |
//                                1 Finished | 2 Reject{u8 PrepareError} (lib.rs:2187-2317)
// Per-report error mapping follows the helper loop (aggregator/src/aggregator.rs:1702-1797):
// undecodable plaintext / duplicate extensions / undecodable input or public share ->
// InvalidMessage (8); a peer prep share the VDAF cannot decode or an unexpected ping-pong message
// -> VdafPrepError (5) (handle_ping_pong_error, aggregator/error.rs:240-300).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/prio3gpu.h"
#include "errors.h"

namespace {

struct Reader {
  const uint8_t* p;
  size_t len, off = 0;
  bool ok = true;
  Reader(const uint8_t* p_, size_t l) : p(p_), len(l) {}
  bool need(size_t n) {
    if (!ok || len - off < n) ok = false;
    return ok;
  }
  uint64_t be(int nbytes) {
    if (!need((size_t)nbytes)) return 0;
    uint64_t v = 0;
    for (int i = 0; i < nbytes; ++i) v = (v << 8) | p[off + i];
    off += (size_t)nbytes;
    return v;
  }
  // skip an opaque byte string with a `nbytes`-wide length prefix; returns its offset
  size_t opaque(int nbytes, uint32_t* out_len) {
    const uint64_t n = be(nbytes);
    const size_t at = off;
    if (!need((size_t)n)) return 0;
    off += (size_t)n;
    *out_len = (uint32_t)n;
    return at;
  }
  size_t fixed(size_t n) {
    const size_t at = off;
    if (need(n)) off += n;
    return at;
  }
};

struct Writer {
  uint8_t* p;
  size_t cap, off = 0;
  Writer(uint8_t* p_, size_t c) : p(p_), cap(c) {}
  void be(uint64_t v, int nbytes) {
    for (int i = nbytes - 1; i >= 0; --i) {
      if (p && off < cap) p[off] = (uint8_t)(v >> (8 * i));
      ++off;
    }
  }
  void bytes(const uint8_t* b, size_t n) {
    if (p && off + n <= cap && n) memcpy(p + off, b, n);
    off += n;
  }
};

bool parse_ping_pong(Reader& r, uint8_t* type, uint64_t* share_off, uint32_t* share_len,
                     uint64_t* msg_off, uint32_t* msg_len) {
  *type = (uint8_t)r.be(1);
  *share_len = *msg_len = 0;
  *share_off = *msg_off = 0;
  switch (*type) {
    case 0: *share_off = r.opaque(4, share_len); break;
    case 1:
      *msg_off = r.opaque(4, msg_len);
      *share_off = r.opaque(4, share_len);
      break;
    case 2: *msg_off = r.opaque(4, msg_len); break;
    default: return false;
  }
  return r.ok;
}

}  // namespace

extern "C" {

int prio3gpu_decode_agg_init_req(const uint8_t* msg, size_t len, int query_type,
                                 uint8_t* out_batch_id, uint64_t* out_agg_param,
                                 prio3gpu_prepare_init_view* views, size_t max_views,
                                 size_t* out_n) {
  if (!msg || !out_n || (query_type != 1 && query_type != 2)) return PRIO3GPU_E_ARG;
  Reader r(msg, len);
  uint32_t ap_len = 0;
  const size_t ap_off = r.opaque(4, &ap_len);
  if (out_agg_param) {
    out_agg_param[0] = ap_off;
    out_agg_param[1] = ap_len;
  }
  if ((int)r.be(1) != query_type) return PRIO3GPU_E_ARG;
  if (query_type == 2) {
    const size_t b = r.fixed(32);
    if (r.ok && out_batch_id) memcpy(out_batch_id, msg + b, 32);
  }
  const uint64_t list_len = r.be(4);
  if (!r.need((size_t)list_len)) return PRIO3GPU_E_ARG;
  const size_t end = r.off + (size_t)list_len;
  if (end != len) return PRIO3GPU_E_ARG;  // get_decoded: no trailing bytes
  size_t n = 0;
  Reader q(msg, end);
  q.off = r.off;
  while (q.ok && q.off < end) {
    prio3gpu_prepare_init_view v{};
    v.report_id_off = q.fixed(16);
    v.time = q.be(8);
    v.public_share_off = q.opaque(4, &v.public_share_len);
    v.hpke_config_id = (uint8_t)q.be(1);
    v.enc_off = q.opaque(2, &v.enc_len);
    v.payload_off = q.opaque(4, &v.payload_len);
    if (!parse_ping_pong(q, &v.message_type, &v.prep_share_off, &v.prep_share_len,
                         &v.prep_msg_off, &v.prep_msg_len))
      return PRIO3GPU_E_ARG;
    if (views) {
      if (n >= max_views) return PRIO3GPU_E_CAPACITY;
      views[n] = v;
    }
    ++n;
  }
  if (!q.ok || q.off != end) return PRIO3GPU_E_ARG;
  *out_n = n;
  return 0;
}

int prio3gpu_check_agg_init_req(const uint8_t* msg, const prio3gpu_prepare_init_view* views,
                                size_t n, uint64_t agg_param_len) {
  if (n && (!msg || !views)) return PRIO3GPU_E_ARG;
  // Duplicate report IDs abort the whole request (aggregator.rs:1588-1598).  Sorting the IDs as
  // big-endian 128-bit keys is O(n log n) whatever IDs an adversarial leader picks.
  std::vector<std::pair<uint64_t, uint64_t>> ids(n);
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* id = msg + views[i].report_id_off;
    uint64_t hi = 0, lo = 0;
    for (int b = 0; b < 8; ++b) hi = (hi << 8) | id[b];
    for (int b = 8; b < 16; ++b) lo = (lo << 8) | id[b];
    ids[i] = {hi, lo};
  }
  std::sort(ids.begin(), ids.end());
  for (size_t i = 1; i < n; ++i) {
    if (ids[i] == ids[i - 1]) {
      p3g::set_error("aggregate request contains duplicate report IDs");
      return PRIO3GPU_E_INVALID_MESSAGE;
    }
  }
  // A::AggregationParam::get_decoded (aggregator.rs:1605): Prio3's aggregation parameter is `()`,
  // whose decoding accepts only the empty byte string.
  if (agg_param_len != 0) {
    p3g::set_error("aggregation parameter must be empty for Prio3 (got %llu bytes)",
                   (unsigned long long)agg_param_len);
    return PRIO3GPU_E_INVALID_MESSAGE;
  }
  return 0;
}

int prio3gpu_gather_prepare_inits(const prio3gpu_sizes* sz, const uint8_t* msg,
                                  const prio3gpu_prepare_init_view* views, size_t n,
                                  uint8_t* nonces, uint8_t* public_shares,
                                  uint8_t* leader_prep_shares, uint8_t* faults) {
  if (!sz || (n && (!msg || !views || !nonces || !faults))) return PRIO3GPU_E_ARG;
  // Reports are independent: large batches (SumVec: 2.9 KB of leader prep share each) are copied
  // on up to 8 threads, each output row written once (zeroed only for a faulty report).
  auto run = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const prio3gpu_prepare_init_view& v = views[i];
      memcpy(nonces + 16 * i, msg + v.report_id_off, 16);
      uint8_t st = PRIO3GPU_OK;
      if (v.public_share_len != sz->public_share) st = PRIO3GPU_INVALID_MESSAGE;
      else if (v.message_type != 0 || v.prep_share_len != sz->prep_share)
        st = PRIO3GPU_VDAF_PREP_ERROR;
      const bool ok = st == PRIO3GPU_OK;
      if (public_shares && sz->public_share) {
        uint8_t* d = public_shares + i * sz->public_share;
        if (ok) memcpy(d, msg + v.public_share_off, sz->public_share);
        else memset(d, 0, sz->public_share);
      }
      if (leader_prep_shares) {
        uint8_t* d = leader_prep_shares + i * sz->prep_share;
        if (ok) memcpy(d, msg + v.prep_share_off, sz->prep_share);
        else memset(d, 0, sz->prep_share);
      }
      faults[i] = st;
    }
  };
  const size_t bytes = n * (size_t)(16 + sz->public_share + sz->prep_share);
  const size_t nt = bytes < (size_t(8) << 20) ? 1 : std::min<size_t>(8, (n + 4095) / 4096);
  if (nt <= 1) {
    run(0, n);
    return 0;
  }
  std::vector<std::thread> pool;
  const size_t per = (n + nt - 1) / nt;
  for (size_t t = 1; t < nt; ++t)
    pool.emplace_back(run, std::min(n, t * per), std::min(n, (t + 1) * per));
  run(0, std::min(n, per));
  for (auto& th : pool) th.join();
  return 0;
}

int prio3gpu_batch_aggregation_merge(uint32_t field_size, size_t output_len,
                                     prio3gpu_batch_aggregation* dst,
                                     const prio3gpu_batch_aggregation* src) {
  typedef unsigned __int128 u128;
  if (!dst || !src || (field_size != 8 && field_size != 16) ||
      (!dst->aggregate_share != !src->aggregate_share)) {
    p3g::set_error("batch_aggregation_merge: bad argument");
    return PRIO3GPU_E_ARG;
  }
  // Interval::merge (core/src/time.rs:289-302)
  uint64_t start = dst->interval_start, dur = dst->interval_duration;
  if (dur == 0) {
    start = src->interval_start;
    dur = src->interval_duration;
  } else if (src->interval_duration != 0) {
    u128 e0 = (u128)dst->interval_start + dst->interval_duration;
    u128 e1 = (u128)src->interval_start + src->interval_duration;
    const u128 end = e0 > e1 ? e0 : e1;
    start = std::min(dst->interval_start, src->interval_start);
    if (end - start > ~0ull) {
      p3g::set_error("batch_aggregation_merge: interval overflow");
      return PRIO3GPU_E_ARG;
    }
    dur = (uint64_t)(end - start);
  }
  // Aggregatable::merge: elementwise mod-p addition of canonical LE field elements
  if (dst->aggregate_share) {
    const u128 p = field_size == 16 ? (((u128)0xFFFFFFFFFFFFFFE4ull << 64) | 1u)
                                    : (u128)0xFFFFFFFF00000001ull;
    for (size_t e = 0; e < output_len; ++e) {
      uint8_t* d = dst->aggregate_share + e * field_size;
      const uint8_t* s = src->aggregate_share + e * field_size;
      u128 a = 0, b = 0;
      for (int i = (int)field_size - 1; i >= 0; --i) {
        a = (a << 8) | d[i];
        b = (b << 8) | s[i];
      }
      if (a >= p || b >= p) {
        p3g::set_error("batch_aggregation_merge: aggregate share element out of range");
        return PRIO3GPU_E_ARG;
      }
      u128 r = a + b;
      if (r < a || r >= p) r -= p;  // a, b < p < 2^128: one subtraction, wrap-around included
      for (uint32_t i = 0; i < field_size; ++i) d[i] = (uint8_t)(r >> (8 * i));
    }
  }
  dst->report_count += src->report_count;
  for (int i = 0; i < 32; ++i) dst->checksum[i] ^= src->checksum[i];
  dst->interval_start = start;
  dst->interval_duration = dur;
  return 0;
}

int prio3gpu_apply_faults(size_t n, const uint8_t* faults, uint8_t* status) {
  if (n && (!faults || !status)) return PRIO3GPU_E_ARG;
  for (size_t i = 0; i < n; ++i)
    if (status[i] == PRIO3GPU_OK) status[i] = faults[i];
  return 0;
}

int prio3gpu_decode_plaintext_input_shares(const prio3gpu_sizes* sz, const uint8_t* plaintexts,
                                           const uint64_t* offsets, size_t n, int agg_id,
                                           uint8_t* out_input_shares, uint8_t* status) {
  if (!sz || (n && (!plaintexts || !offsets || !out_input_shares || !status)))
    return PRIO3GPU_E_ARG;
  const uint32_t want = agg_id == 0 ? sz->leader_input_share : sz->helper_input_share;
  for (size_t i = 0; i < n; ++i) {
    uint8_t* dst = out_input_shares + i * (size_t)want;
    memset(dst, 0, want);
    if (status[i] != PRIO3GPU_OK) continue;
    Reader r(plaintexts + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
    const uint64_t ext_len = r.be(2);
    bool ok = r.need((size_t)ext_len);
    const size_t ext_end = r.off + (size_t)ext_len;
    std::vector<uint16_t> types;
    while (ok && r.off < ext_end) {
      const uint16_t t = (uint16_t)r.be(2);
      uint32_t dl = 0;
      r.opaque(2, &dl);
      ok = r.ok && r.off <= ext_end;
      for (uint16_t u : types) ok &= (u != t);  // duplicate extensions -> InvalidMessage
      types.push_back(t);
    }
    uint32_t pl = 0;
    const size_t po = ok ? r.opaque(4, &pl) : 0;
    ok = ok && r.ok && r.off == r.len && pl == want;
    if (!ok) {
      status[i] = PRIO3GPU_INVALID_MESSAGE;
      continue;
    }
    memcpy(dst, plaintexts + offsets[i] + po, want);
  }
  return 0;
}

int prio3gpu_encode_agg_job_resp(const uint8_t* nonces, const uint8_t* prep_msgs,
                                 uint32_t prep_msg_len, const uint8_t* status, size_t n,
                                 uint8_t* out, size_t cap, size_t* out_len) {
  if (!out_len || (n && (!nonces || !status))) return PRIO3GPU_E_ARG;
  Writer w(out, cap);
  size_t items = 0;
  for (size_t i = 0; i < n; ++i) items += 16 + 1 + (status[i] == 0 ? 1 + 4 + prep_msg_len : 1);
  w.be(items, 4);
  for (size_t i = 0; i < n; ++i) {
    w.bytes(nonces + 16 * i, 16);
    if (status[i] == 0) {  // Continue { Finish { prep_msg } }
      w.be(0, 1);
      w.be(2, 1);
      w.be(prep_msg_len, 4);
      w.bytes(prep_msgs ? prep_msgs + (size_t)prep_msg_len * i : nullptr, prep_msg_len);
    } else {  // Reject(PrepareError)
      w.be(2, 1);
      w.be(status[i], 1);
    }
  }
  *out_len = w.off;
  return (out && w.off > cap) ? PRIO3GPU_E_CAPACITY : 0;
}

int prio3gpu_encode_agg_init_req(int query_type, const uint8_t* batch_id, const uint8_t* agg_param,
                                 uint32_t agg_param_len, size_t n, const uint8_t* nonces,
                                 const uint64_t* times, const uint8_t* public_shares,
                                 uint32_t public_share_len, const uint8_t* hpke_config_ids,
                                 const uint8_t* encs, const uint64_t* enc_offsets,
                                 const uint8_t* payloads, const uint64_t* payload_offsets,
                                 const uint8_t* prep_shares, uint32_t prep_share_len,
                                 const uint8_t* status, uint8_t* out, size_t cap,
                                 size_t* out_len) {
  if (!out_len || (query_type != 1 && query_type != 2) || (query_type == 2 && !batch_id))
    return PRIO3GPU_E_ARG;
  if (n && (!nonces || !times || !hpke_config_ids || !enc_offsets || !payload_offsets ||
            !prep_shares))
    return PRIO3GPU_E_ARG;
  Writer w(out, cap);
  w.be(agg_param_len, 4);
  w.bytes(agg_param, agg_param_len);
  w.be((uint64_t)query_type, 1);
  if (query_type == 2) w.bytes(batch_id, 32);
  auto item_len = [&](size_t i) -> size_t {
    return 16 + 8 + 4 + public_share_len + 1 + 2 + (size_t)(enc_offsets[i + 1] - enc_offsets[i]) +
           4 + (size_t)(payload_offsets[i + 1] - payload_offsets[i]) + 1 + 4 + prep_share_len;
  };
  size_t items = 0;
  for (size_t i = 0; i < n; ++i)
    if (!(status && status[i])) items += item_len(i);  // failed leader prepare_init: not sent
  w.be(items, 4);
  const size_t body = w.off;
  *out_len = body + items;
  if (!out) return 0;
  if (*out_len > cap) return PRIO3GPU_E_CAPACITY;
  // PrepareInit i is written at its own offset: large jobs (SumVec: ~3 KB per report) are
  // encoded on up to 8 threads over report ranges, each range starting at its prefix offset.
  auto run = [&](size_t lo, size_t hi, size_t at) {
    Writer x(out + at, cap - at);
    for (size_t i = lo; i < hi; ++i) {
      if (status && status[i]) continue;
      x.bytes(nonces + 16 * i, 16);
      x.be(times[i], 8);
      x.be(public_share_len, 4);
      x.bytes(public_shares ? public_shares + (size_t)public_share_len * i : nullptr,
              public_share_len);
      x.be(hpke_config_ids[i], 1);
      const size_t el = (size_t)(enc_offsets[i + 1] - enc_offsets[i]);
      x.be(el, 2);
      x.bytes(encs + enc_offsets[i], el);
      const size_t pl = (size_t)(payload_offsets[i + 1] - payload_offsets[i]);
      x.be(pl, 4);
      x.bytes(payloads + payload_offsets[i], pl);
      x.be(0, 1);  // PingPongMessage::Initialize { prep_share }
      x.be(prep_share_len, 4);
      x.bytes(prep_shares + (size_t)prep_share_len * i, prep_share_len);
    }
  };
  const size_t nt = items < (size_t(8) << 20) ? 1 : std::min<size_t>(8, (n + 4095) / 4096);
  if (nt <= 1) {
    run(0, n, body);
    return 0;
  }
  const size_t per = (n + nt - 1) / nt;
  std::vector<size_t> start(nt, body);
  for (size_t t = 1; t < nt; ++t) {
    size_t acc = start[t - 1];
    for (size_t i = (t - 1) * per; i < std::min(n, t * per); ++i)
      if (!(status && status[i])) acc += item_len(i);
    start[t] = acc;
  }
  std::vector<std::thread> pool;
  for (size_t t = 1; t < nt; ++t)
    pool.emplace_back(run, std::min(n, t * per), std::min(n, (t + 1) * per), start[t]);
  run(0, std::min(n, per), body);
  for (auto& th : pool) th.join();
  return 0;
}

int prio3gpu_decode_agg_job_resp(const uint8_t* msg, size_t len,
                                 prio3gpu_prepare_resp_view* views, size_t max_views,
                                 size_t* out_n) {
  if (!msg || !out_n) return PRIO3GPU_E_ARG;
  Reader r(msg, len);
  const uint64_t list_len = r.be(4);
  if (!r.need((size_t)list_len) || r.off + list_len != len) return PRIO3GPU_E_ARG;
  size_t n = 0;
  while (r.ok && r.off < len) {
    prio3gpu_prepare_resp_view v{};
    v.report_id_off = r.fixed(16);
    v.result = (uint8_t)r.be(1);
    if (v.result == 0) {
      if (!parse_ping_pong(r, &v.message_type, &v.prep_share_off, &v.prep_share_len,
                           &v.prep_msg_off, &v.prep_msg_len))
        return PRIO3GPU_E_ARG;
    } else if (v.result == 2) {
      v.error = (uint8_t)r.be(1);
    } else if (v.result != 1) {
      return PRIO3GPU_E_ARG;
    }
    if (views) {
      if (n >= max_views) return PRIO3GPU_E_CAPACITY;
      views[n] = v;
    }
    ++n;
  }
  if (!r.ok) return PRIO3GPU_E_ARG;
  *out_n = n;
  return 0;
}

int prio3gpu_gather_helper_resps(const prio3gpu_sizes* sz, const uint8_t* msg,
                                 const prio3gpu_prepare_resp_view* views, size_t n_views,
                                 const uint8_t* nonces, size_t n, uint8_t* prep_msgs,
                                 uint8_t* status) {
  if (!sz || (n && (!nonces || !status)) || (n_views && (!msg || !views))) return PRIO3GPU_E_ARG;
  // the helper answers the reports the leader sent, in order (aggregation_job_driver.rs:530-600)
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    uint8_t* pm = prep_msgs ? prep_msgs + (size_t)sz->prep_msg * i : nullptr;
    if (pm && sz->prep_msg) memset(pm, 0, sz->prep_msg);
    if (status[i] != PRIO3GPU_OK) continue;
    if (k >= n_views || memcmp(msg + views[k].report_id_off, nonces + 16 * i, 16) != 0)
      return PRIO3GPU_E_ARG;  // unexpected report ID: the whole job fails
    const prio3gpu_prepare_resp_view& v = views[k++];
    if (v.result == 2) {
      status[i] = v.error;
    } else if (v.result == 0 && v.message_type == 2 && v.prep_msg_len == sz->prep_msg) {
      if (pm && sz->prep_msg) memcpy(pm, msg + v.prep_msg_off, sz->prep_msg);
    } else {
      status[i] = PRIO3GPU_VDAF_PREP_ERROR;  // not Finish{prep msg}: ping-pong mismatch
    }
  }
  return k == n_views ? 0 : PRIO3GPU_E_ARG;
}

}  // extern "C"

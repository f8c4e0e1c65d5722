/* prio3gpu_test.h -- test and benchmark hooks of libprio3gpu.so, kept out of the product ABI
 * (include/prio3gpu.h).  A Janus build binds only prio3gpu.h (rust/aggregator/src/gpu/ffi.rs);
 * these entry points exist for the parity tests (tests/test_gpu_squeeze.py,
 * tests/test_gpu_flp_branches.py) and the host benchmarks (tools/hpke_bench.py). */
#ifndef PRIO3GPU_TEST_H
#define PRIO3GPU_TEST_H

#include "prio3gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* TEST ONLY.  The XOF squeeze every kernel runs (prio `into_field_vec`, reached through
 * XofShake128::next_vec: ES-byte LE chunks, reject >= p) over caller-crafted rate blocks instead
 * of Keccak output: blocks[25 i .. 25 i + 25) is the state after the i-th permutation (words
 * 0..20 are the 168-byte rate block).  field_size 8 or 16; exact != 0 forces the per-element path
 * (as PRIO3GPU_EXACT_SQUEEZE=1 does in the real kernels).  Runs on the current HIP device. */
int prio3gpu_test_squeeze(int field_size, const uint64_t* blocks, size_t nblocks, uint32_t n,
                          uint8_t* out, int exact);
/* TEST ONLY.  The FLP-query phase of prepare_init (agg_id 0) over caller-supplied randomness
 * instead of the XOF's: leader_input_shares n x leader_input_share, query_rand n x qr_len x
 * field_size (qr_len = 1, 2 for FixedPoint), joint_rand n x joint_rand_len x field_size, own_parts
 * n x 16 (the prep share's joint-rand part).  Writes the prep shares; a query point that is a root
 * of unity sets status 5 (VdafPrepError), as prio does.  Lets tests reach the branches that
 * SHAKE128 output reaches with negligible probability (t^m == 1, r^m == 1). */
int prio3gpu_test_flp_query(prio3gpu_ctx* ctx, size_t n, const uint8_t* leader_input_shares,
                            const uint8_t* query_rand, const uint8_t* joint_rand,
                            const uint8_t* own_parts, uint8_t* out_prep_shares, uint8_t* status);

/* Device memory helpers (bench / tests that stage inputs in HBM without torch). */
int prio3gpu_dev_alloc(prio3gpu_ctx* ctx, size_t bytes, void** out);
int prio3gpu_dev_free(prio3gpu_ctx* ctx, void* p);
int prio3gpu_memcpy(prio3gpu_ctx* ctx, void* dst, const void* src, size_t bytes);

/* The batched HPKE open's X25519 ladder: on != 0 (default where the CPU has AVX-512 IFMA) runs
 * 8 reports per AVX-512 IFMA ladder, 0 the scalar radix-2^51 ladder for every report (A/B of the
 * two ladders in tools/hpke_bench.py; both are checked against each other in tests/test_hpke.py).
 * Process-wide; returns the previous setting, or PRIO3GPU_E_UNSUPPORTED for on != 0 on a CPU
 * without IFMA. */
int prio3gpu_test_hpke_set_ifma(int on);

#ifdef __cplusplus
}
#endif

#endif /* PRIO3GPU_TEST_H */

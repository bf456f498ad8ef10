/* syncfast_amd_test.h -- test hooks of libsyncfast_amd (not part of the
 * drop-in surface; no reference interface corresponds).
 *
 * The library reads its environment knobs once, when it is loaded
 * (syncfast_amd/csrc/sf_knobs.cpp); nothing on a launch or copy path reads
 * the environment.  A test that needs another value inside the same process
 * sets it here.  Names are the environment variables' (INTEGRATION.md,
 * "Environment knobs"): SF_* performance knobs and SF_TEST_* hooks.
 */
#ifndef SYNCFAST_AMD_TEST_H
#define SYNCFAST_AMD_TEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Set knob `name` to `value`; the previous value goes to *old_value (may be
 * NULL).  SF_EINVAL for an unknown name.  Not synchronised with calls in
 * flight on other threads: set knobs between calls. */
int sf_test_set_knob(const char* name, int64_t value, int64_t* old_value);

/* Current value of knob `name`. */
int sf_test_get_knob(const char* name, int64_t* value);

/* Process-wide counters of the routes the host entry points took:
 *   "pages_locked"      caller ranges the library page-locked (hipHostRegister)
 *   "not_anon_refused"  caller ranges it did not page-lock because they are not
 *                       private anonymous memory (a file mapping, shared
 *                       memory): those are copied through the pinned stages. */
int sf_test_get_stat(const char* name, int64_t* value);

/* The processing order sha1_table_kernel gets for a sorted explicit list:
 * d_order[0, n) (device uint32) receives the block indices ordered by
 * length class (4 mantissa bits, 8-bit key), descending, list order within
 * a class -- the counting sort of sf_sort.hip.  d_sizes: n device uint32.
 * Asynchronous on `stream`; SF_EINVAL for n >= 2^32. */
int sf_test_table_order(const uint32_t* d_sizes, uint64_t n, uint32_t* d_order, void* stream);

/* The same with `mbits` mantissa bits (1..6) of the length class: the key
 * is clamped at (16 << max(mbits, 4)) - 1 (8, 9 or 10 bits), as the
 * SF_TABLE_CLASS_BITS knob sorts.  SF_EINVAL for mbits outside 1..6. */
int sf_test_table_order_bits(const uint32_t* d_sizes, uint64_t n, uint32_t mbits, uint32_t* d_order, void* stream);

/* Called by the descriptor and path routes that pread a regular file
 * (sf_index_fd_blocks, sf_index_fd_fixed, sf_index_file_blocks,
 * sf_index_file) after each window has been read, on the calling thread,
 * with the window's index: a test changes the file at a known point of a
 * call.  NULL removes it.  Not synchronised with calls in flight. */
typedef void (*sf_test_read_hook_fn)(void* arg, uint64_t window);
int sf_test_set_read_hook(sf_test_read_hook_fn fn, void* arg);

/* The gather plan of sf_index_device_multi / _ex for n_devices shards of a
 * file_len-byte file at block_size, gathered to `root` (self_gather: the
 * one-device self send/recv of SF_TEST_MULTI_SELF_GATHER, n_devices == 1
 * only).  Per device r (n_devices entries each): table_offset[r] = where its
 * rows start in d_table (bytes), bytes[r] = its digest bytes, route[r] = 0
 * (empty shard: nothing hashed or sent), 1 (the root's rows, hashed in place
 * into d_table) or 2 (hashed into d_digests[r] and sent to the root, which
 * receives them at table_offset[r]).  Host only. */
int sf_test_multi_plan(uint64_t file_len, uint32_t block_size, uint32_t n_devices, uint32_t root, int self_gather,
                       uint64_t *table_offset, uint64_t *bytes, int *route);

/* Cross-XCD counter litmus (sf_litmus.hip): does a read of a counter see
 * adds made on other XCDs after the reading XCD's L2 holds its line?
 * mode 0 reads with a relaxed agent-scope atomic load (round 5's fused
 * launch polled that way), mode 1 with an agent-scope atomic add of an
 * opaque zero.  One launch on the current device,
 * synchronous.  out[8]: status (0 ok, 1 a hand-shake wait ran out), the
 * reader's XCD id, adds made from other XCDs, first read, read after every
 * add returned, a read-modify-write read after that, mode, 0.  A stale form
 * gives out[4] == out[3] < out[2] == out[5]. */
int sf_test_xcd_litmus(int mode, uint32_t out[8]);

#ifdef __cplusplus
}
#endif

#endif /* SYNCFAST_AMD_TEST_H */

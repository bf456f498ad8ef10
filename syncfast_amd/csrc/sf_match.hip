// sf_match.hip -- block lookup of a sync destination on the device
// (include/syncfast_amd.h, sf_block_set_*).
//
// The consumer of the signature table on the receiving side: for every
// FILE_BLOCK message of an incoming file, FsDestinationInner::sink asks its
// index whether it already holds that block (Index::get_block,
// /root/reference/src/index.rs:77-103, called at src/sync/fs.rs:461-476):
//   SELECT files.name, blocks.offset, blocks.size FROM blocks
//   INNER JOIN files ON ... WHERE blocks.hash = ? AND blocks.present = 1;
// and copies the first row's block, or records the block as missing.  SQLite
// answers from idx_blocks_hash, i.e. in (hash, rowid) order, so "first" is
// the present row with that digest and the smallest rowid.  Here the
// destination's rows (digest table in rowid order + present flags) become an
// open-addressing hash table in HBM, built once, and a whole file's block
// list is answered in one launch: row index of that first present row, or -1.
//
// Table: capacity = power of two >= 2 x rows (load <= 1/2), 8 B per slot:
// bits 0-39 = row + 1 (0 = empty), bits 40-63 = a 24-bit fingerprint of the
// digest (bytes 8-10), so a probe rejects a slot holding another digest
// without reading that row.  The slot index comes from digest bytes 0-7
// (SHA-1 output is uniform).  Insert: CAS into an empty slot; a slot already
// holding the same digest keeps the smaller row (atomicMin on the whole word:
// same fingerprint, so the row bits decide) -- the result does not depend on
// the order threads arrive in.  Linear probing; a probe stops at the first
// empty slot or matching digest.  Every lane's loop is bounded by the
// capacity, and the table is never full, so every wave exits.
// Random-access, HBM-latency-bound integer work: no MFMA, no LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sf_internal.hpp"

namespace sfm {

constexpr uint64_t kRowBits = 40;
constexpr uint64_t kRowMask = (1ull << kRowBits) - 1;

struct Key {
  uint32_t w[5];
};

__device__ __forceinline__ Key load_key(const uint8_t* __restrict__ table, uint64_t row) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(table + row * 20);  // rows are 4-B aligned
  Key k;
#pragma unroll
  for (int i = 0; i < 5; ++i) k.w[i] = p[i];
  return k;
}

__device__ __forceinline__ bool same_key(const uint8_t* __restrict__ table, uint64_t row, const Key& k) {
  const Key o = load_key(table, row);
  return o.w[0] == k.w[0] && o.w[1] == k.w[1] && o.w[2] == k.w[2] && o.w[3] == k.w[3] && o.w[4] == k.w[4];
}

__device__ __forceinline__ uint64_t slot_of(const Key& k, uint64_t mask) {
  return (((uint64_t)k.w[1] << 32) | k.w[0]) & mask;
}

__device__ __forceinline__ uint64_t tag_of(const Key& k) { return (uint64_t)(k.w[2] & 0xFFFFFFu) << kRowBits; }

__global__ void __launch_bounds__(256)
block_set_insert_kernel(const uint8_t* __restrict__ table, const uint8_t* __restrict__ present, uint64_t n,
                        unsigned long long* slots, uint64_t mask) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || (present && !present[r])) return;
  const Key k = load_key(table, r);
  const uint64_t tag = tag_of(k);
  const unsigned long long mine = tag | (r + 1);
  uint64_t i = slot_of(k, mask);
  for (uint64_t probes = 0; probes <= mask; ++probes, i = (i + 1) & mask) {
    unsigned long long cur = slots[i];
    if (cur == 0) {
      cur = atomicCAS(&slots[i], 0ull, mine);
      if (cur == 0) return;  // claimed an empty slot
    }
    // The slot holds another row: the same digest keeps the smaller row.
    if ((cur & ~kRowMask) == tag && same_key(table, (cur & kRowMask) - 1, k)) {
      atomicMin(&slots[i], mine);
      return;
    }
  }
}

__global__ void __launch_bounds__(256)
block_set_lookup_kernel(const uint8_t* __restrict__ table, const unsigned long long* __restrict__ slots,
                        uint64_t mask, const uint8_t* __restrict__ query, uint64_t nq, int64_t* __restrict__ rows) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const Key k = load_key(query, q);
  const uint64_t tag = tag_of(k);
  uint64_t i = slot_of(k, mask);
  int64_t found = -1;
  for (uint64_t probes = 0; probes <= mask; ++probes, i = (i + 1) & mask) {
    const unsigned long long cur = slots[i];
    if (cur == 0) break;
    if ((cur & ~kRowMask) == tag && same_key(table, (cur & kRowMask) - 1, k)) {
      found = (int64_t)(cur & kRowMask) - 1;
      break;
    }
  }
  rows[q] = found;
}

}  // namespace sfm

using namespace sfi;

// The opaque handle of include/syncfast_amd.h.
struct sf_block_set {
  const uint8_t* table;       // caller's digest table (kept alive by the caller)
  uint64_t rows;
  unsigned long long* slots;  // device, 8 B per slot
  uint64_t mask;              // capacity - 1
};

namespace {

int block_set_build(const void* d_table, const uint8_t* d_present, uint64_t n_rows, sf_block_set** out,
                    hipStream_t s) {
  if (!out) return SF_EINVAL;
  *out = nullptr;
  if ((n_rows && !d_table) || n_rows >= sfm::kRowMask) return SF_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_table) & 3u) return SF_EINVAL;  // 20-B rows read as dwords
  uint64_t cap = 1024;
  while (cap < 2 * n_rows) cap <<= 1;
  sf_block_set* bs = new sf_block_set{static_cast<const uint8_t*>(d_table), n_rows, nullptr, cap - 1};
  int rc = stream_alloc(reinterpret_cast<void**>(&bs->slots), cap * sizeof(unsigned long long), s);
  if (rc == SF_OK) rc = hip_err(hipMemsetAsync(bs->slots, 0, cap * sizeof(unsigned long long), s));
  if (rc == SF_OK && n_rows) {
    sfi::clear_stale_error();
    hipLaunchKernelGGL(sfm::block_set_insert_kernel, dim3((unsigned)ceil_div(n_rows, 256)), dim3(256), 0, s,
                       bs->table, d_present, n_rows, bs->slots, bs->mask);
    rc = hip_err(hipGetLastError());
  }
  if (rc != SF_OK) {
    stream_free(bs->slots, s);
    delete bs;
    return rc;
  }
  *out = bs;
  return SF_OK;
}

}  // namespace

extern "C" {

int sf_block_set_build(const void* d_table, const uint8_t* d_present, uint64_t n_rows, sf_block_set** out,
                       void* stream) {
  // rows per launch: the insert kernel takes one lane per row, so one launch
  // holds < 2^32 work-items (2^40 rows would not fit in HBM anyway at 20 B)
  if (n_rows > (1ull << 31)) return SF_EINVAL;
  return guarded([&] { return block_set_build(d_table, d_present, n_rows, out, as_stream(stream)); });
}

int sf_block_set_lookup(const sf_block_set* set, const void* d_query, uint64_t n_query, int64_t* d_rows,
                        void* stream) {
  if (!set || (n_query && (!d_query || !d_rows))) return SF_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_query) & 3u) return SF_EINVAL;
  const uint64_t per = 1ull << 31;  // queries per launch (< 2^32 work-items)
  for (uint64_t q0 = 0; q0 < n_query; q0 += per) {
    const uint64_t nq = std::min(per, n_query - q0);
    sfi::clear_stale_error();
    hipLaunchKernelGGL(sfm::block_set_lookup_kernel, dim3((unsigned)ceil_div(nq, 256)), dim3(256), 0,
                       as_stream(stream), set->table, set->slots, set->mask,
                       static_cast<const uint8_t*>(d_query) + q0 * 20, nq, d_rows + q0);
    const int rc = hip_err(hipGetLastError());
    if (rc) return rc;
  }
  return SF_OK;
}

int sf_block_set_free(sf_block_set* set, void* stream) {
  if (!set) return SF_OK;
  const int rc = set->slots ? hip_err(hipFreeAsync(set->slots, as_stream(stream))) : SF_OK;  // stream_free, with its error
  delete set;
  return rc;
}

}  // extern "C"

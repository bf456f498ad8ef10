// sf_capi.hip -- the C-ABI (include/syncfast_amd.h): the gfx950 kernels'
// launchers and the device-resident entry points.
//
// The only translation unit compiled for the GPU.  The host-memory entry
// points (buffer, file, fd, range, many files, wire stream) are in
// sf_host.cpp / sf_files.cpp and call the launchers below.  There is no CPU
// implementation of the block hashing in this library: without a HIP device
// the entry points return SF_ENODEV.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "sf_internal.hpp"
#include "sf_kernels.hpp"

namespace sfi __attribute__((visibility("hidden"))) {


constexpr int kTile = 128;  // bytes of each block staged per LDS step

// Most blocks one launch takes.  HIP caps a launch at 2^32 - 1 work-items
// (gridDim.x * blockDim.x), i.e. about 2^32 blocks at one lane per block;
// larger tables -- reachable only with tiny blocks, e.g. 16-B blocks over
// 64 GiB -- are hashed as several launches over consecutive block ranges
// (blocks are independent).  A multiple of 16, so every piece of a 16-B
// aligned fixed tiling stays 16-B aligned.  SF_TEST_LAUNCH_MAX_BLOCKS lowers
// it (test hook: exercises the split at small sizes).
inline uint64_t launch_max_blocks() {
  const int64_t v = knob(K_TEST_LAUNCH_MAX_BLOCKS);
  return v > 0 ? std::max<uint64_t>(16, (uint64_t)v & ~15ull) : (1ull << 31);
}

inline unsigned grid_for_blocks(uint64_t nblocks) {
  const uint64_t waves = ceil_div(nblocks, 64);
  return (unsigned)ceil_div(waves, sf::kWavesPerWG);
}

// K_t + W_t for the padding-only chunk of a `bytes`-long message (bytes a
// multiple of 64): W = {0x80000000, 0 x 13, bit length hi, lo}.
sf::PadSchedule pad_schedule(uint32_t bytes) {
  sf::PadSchedule p{};
  if (bytes == 0 || (bytes & 63u)) return p;
  uint32_t w[80] = {0};
  w[0] = 0x80000000u;
  w[14] = bytes >> 29;
  w[15] = bytes << 3;
  for (int t = 16; t < 80; t++) {
    const uint32_t x = w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16];
    w[t] = (x << 1) | (x >> 31);
  }
  for (int t = 0; t < 80; t++) {
    const uint32_t k = t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
    p.kw[t] = k + w[t];
  }
  p.bytes = bytes;
  return p;
}

int launch_fixed(const void* d_data, uint64_t len, uint32_t bs, uint64_t nblocks, void* d_digests,
                 hipStream_t stream, uint32_t* weak) {
  if (nblocks == 0) return SF_OK;
  const uint64_t maxb = launch_max_blocks();
  if (nblocks > maxb) {  // consecutive pieces of the tiling, one launch each
    for (uint64_t first = 0; first < nblocks; first += maxb) {
      const uint64_t cnt = std::min(maxb, nblocks - first), off = first * (uint64_t)bs;
      const int rc = launch_fixed(static_cast<const uint8_t*>(d_data) + off, std::min(len - off, cnt * (uint64_t)bs),
                                  bs, cnt, static_cast<uint8_t*>(d_digests) + first * 20, stream,
                                  weak ? weak + first : nullptr);
      if (rc) return rc;
    }
    return SF_OK;
  }
  const unsigned grid = grid_for_blocks(nblocks);
  const sf::PadSchedule pad = pad_schedule(bs);
  const uint8_t* d = static_cast<const uint8_t*>(d_data);
  uint8_t* o = static_cast<uint8_t*>(d_digests);
  if (weak) {  // opt-in fused Adler-32 (a separate instantiation; the default kernel is unchanged)
    sfi::clear_stale_error();
    hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, 1, true>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs,
                       nblocks, o, pad, weak);
    return hip_err(hipGetLastError());
  }
  sfi::clear_stale_error();
  hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, 1>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr);
  return hip_err(hipGetLastError());
}

// CUs of the current device (cached per device: a process may drive GPUs or
// partitions with different CU counts).
inline unsigned device_cus() {
  static std::atomic<int> cached[kMaxDevices];
  int d = 0, v = 0;
  if (hipGetDevice(&d) != hipSuccess) {
    (void)hipGetLastError();
    return 64;  // conservative (a quarter of MI355X's CUs)
  }
  if (d >= 0 && d < kMaxDevices && (v = cached[d].load(std::memory_order_relaxed)) > 0) return (unsigned)v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0) {
    (void)hipGetLastError();
    return 64;
  }
  if (d >= 0 && d < kMaxDevices) cached[d].store(v, std::memory_order_relaxed);
  return (unsigned)v;
}

// Explicit block lists of more than one wave's blocks are hashed in order of
// length (sha1_table_kernel's `order`): a wave runs as long as its longest
// block, so 64 blocks of mixed sizes side by side waste most lanes -- a list
// of content-defined sizes (mean 8 KiB, up to 32 KiB) hashed at 312 GiB/s in
// list order against 1834 GiB/s sorted (scripts/ragged_probe.py).  Small
// lists too (round 6; until then only from 2^17 blocks, on the reasoning that
// with every wave resident at once the longest block sets the time either
// way): a mixed wave also runs every step in the slot path's per-lane tail
// loop, its shortest block ending the branch-free steps, one compression at a
// time; sorted, the wave holding the longest blocks runs them two at a time.
// configs[0]'s one-window list (8,415 blocks): the kernel 1.28 -> 0.69 ms,
// the sort's three kernels 19 us (profiles/r06/sort_small/).  One wave has
// nothing to reorder.  SF_TEST_TABLE_SORT=0 / 1 never / always sorts (test hook).
constexpr uint64_t kTableSortMinBlocks = 65;
inline uint64_t table_sort_min() {
  const int64_t v = knob(K_TEST_TABLE_SORT);
  if (v >= 0) return v ? 1 : ~0ull;
  return kTableSortMinBlocks;
}
constexpr uint64_t kSortMaxBlocks = 1ull << 27;  // blocks per sorted piece (~1.2 GiB of workspace at most)

// Stream-ordered workspace holding the processing order of blocks [0, n) of
// a list: stable sort of the blocks by length class, descending, on `s`
// (list order within a class).  Stability matters: a wave's 64 blocks are
// then alike in length AND close together in memory; a class-bucketing by
// atomics scattered each class's blocks across the buffer and the list ran
// at half the rate (1410 vs 2609 GiB/s on one box, profiles/r03/bucket_sort_rejected/).
// The key takes the counting sort of sf_sort.hip (three kernels, ~21 us for
// 0.5 M blocks with the default 8-bit key, against ~56 us of GPU time for
// rocprim's radix sort with its key kernel; profiles/r03/sort/), the 9- and
// 10-bit keys of the SF_TABLE_CLASS_BITS knob too (512 / 1024 bins).
// Returns nullptr (unsorted launch) if anything fails.
uint32_t* table_order(const uint32_t* d_sizes, uint64_t n, hipStream_t s, void** ws_out) {
  *ws_out = nullptr;
  // mantissa bits of the length class, 1..6 (SF_TABLE_CLASS_BITS, A/B knob)
  const uint32_t mbits = (uint32_t)std::min<int64_t>(6, std::max<int64_t>(1, knob(K_TABLE_CLASS_BITS)));

  // classes < 32 << mbits; the key is clamped at (16 << mbits) - 1, so every
  // block of 2^16+ compressions (>= 4 MiB) shares the top class: 8 bits with
  // 4 mantissa bits (the default; class width 6.25 %), 9 with 5, 10 with 6
  // (1.6 %), all one counting pass of sf_sort.hip.
  const unsigned kbits = mbits <= 4 ? 8u : 4u + mbits;
  const uint32_t kmax = (1u << kbits) - 1u;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  // one counting pass over 256 / 512 / 1024 classes (sf_sort.hip)
  const size_t ob = up(n * 4), total = ob + up(sfi::class_order_workspace(n, kmax));
  uint8_t* ws = nullptr;
  if (sfi::stream_alloc(reinterpret_cast<void**>(&ws), total, s) != SF_OK) {
    (void)hipGetLastError();
    return nullptr;
  }
  uint32_t* order = reinterpret_cast<uint32_t*>(ws);
  if (sfi::class_order(d_sizes, n, mbits, kmax, ws + ob, order, s) != SF_OK) {
    (void)hipGetLastError();
    sfi::stream_free(ws, s);
    return nullptr;
  }
  *ws_out = ws;
  return order;
}

int launch_table(const void* d_data, uint64_t len, const uint64_t* d_offsets, const uint32_t* d_sizes,
                 uint64_t nblocks, void* d_digests, int* d_status, hipStream_t stream, uint32_t* weak) {
  if (nblocks == 0) return SF_OK;
  const bool sorted = nblocks >= table_sort_min();
  const uint64_t maxb = sorted ? std::min(launch_max_blocks(), kSortMaxBlocks) : launch_max_blocks();
  if (nblocks > maxb) {  // consecutive pieces of the table, one launch each
    for (uint64_t first = 0; first < nblocks; first += maxb) {
      const int rc = launch_table(d_data, len, d_offsets + first, d_sizes + first, std::min(maxb, nblocks - first),
                                  static_cast<uint8_t*>(d_digests) + first * 20, d_status, stream,
                                  weak ? weak + first : nullptr);
      if (rc) return rc;
    }
    return SF_OK;
  }
  void* ws = nullptr;
  const uint32_t* order = sorted ? table_order(d_sizes, nblocks, stream, &ws) : nullptr;
  const int rc = launch_table_kernel(weak != nullptr, static_cast<const uint8_t*>(d_data), len, d_offsets, d_sizes,
                                     nblocks, static_cast<uint8_t*>(d_digests), d_status, weak, order, stream);
  sfi::stream_free(ws, stream);
  return rc;
}

// Many equal-size, block-aligned files back to back, with their per-file
// blocks_hash (src/index.rs:661-682), and no wave waiting for another
// (round 6).  A file's blocks_hash is one sequential SHA-1 over its digest
// run, which exists only once its blocks are hashed; the batch is therefore
// hashed as the batch stream hashes its last batch, from
// this stream's pieces (sf_stream.hip, sf_chain.hip):
//   1. block columns [0, cut) of every file (sha1_fixed_chained_kernel, no jobs);
//   2. columns [cut, nbf) beside the FIRST half of every file's chain (its
//      digests [0, cut) exist: launch 1 finished them), the SHA-1 state kept
//      in HBM;
//   3. the second half of every chain alone, with schedule-building helper
//      waves (sha1_chain_helper_kernel).
// Round 5's single fused launch (sha1_staged_kernel: chain lanes polling
// per-stage counters, bounded) gave up once in five rounds for a reason no
// probe reproduced; this form runs config 3's shape at 2.76
// ms per 8 GiB against that launch's 2.71 and 2.97 for blocks-then-chains
// (profiles/r06/batch/).  Other shapes (runs not 16-B aligned, fewer than 128
// blocks per file, not a multiple of 64 or more than 16,384, SF_BATCH_FUSED=0):
// the block kernel, then the chain kernel.  d_status is not written.
int batch_with_hashes(const uint8_t* base, uint64_t flen, uint32_t bs, uint32_t nfiles, uint64_t nbf, uint8_t* dig,
                      uint8_t* fh, bool halves, hipStream_t s) {
  uint64_t cut = 0;
  // Files of more than 16,384 blocks (64 MiB at 4 KiB): chains of over 5,120
  // compressions run faster whole and alone with their helper waves than half
  // beside the blocks (64 x 128 MiB: 11.5 ms that way, 12.4 in halves; 16 x
  // 512 MiB 37.2 against 44.0; 256 x 32 MiB the other way, 4.89 against 4.28).
  if (halves && nbf % 64 == 0 && nbf >= 128 && nbf <= 16384 && (reinterpret_cast<uintptr_t>(dig) & 15) == 0 &&
      nbf * nfiles <= launch_max_blocks()) {
    const uint64_t half = (nbf * 20 / 64) / 2;  // data chunks of part 1 (as the chained launcher cuts them)
    const uint64_t need = ceil_div(half * 64, 20);  // digests part 1 reads
    cut = ceil_div(need, 64) * 64;                  // in whole block waves
    if (cut >= nbf) cut = 0;
  }
  if (!cut) {
    int rc = launch_fixed(base, nbf * nfiles * (uint64_t)bs, bs, nbf * nfiles, dig, s);
    if (rc) return rc;
    if (nbf % 4 == 0 && nbf * 20 <= 0xFFFFFFF0ull && (reinterpret_cast<uintptr_t>(dig) & 15) == 0) {
      // 16-B aligned runs: chains with schedule-building helper waves
      sf::ChainJob j = {}, none = {};
      j.runs = dig;
      j.hashes = fh;
      j.files = nfiles;
      j.run_len = (uint32_t)(nbf * 20);
      j.lo = 0;
      j.hi = j.run_len / 64;
      j.part = 0;
      j.waves = (uint32_t)ceil_div(nfiles, 64);
      return launch_chain_helper(j, none, s);
    }
    sfi::clear_stale_error();
    hipLaunchKernelGGL(sf::sha1_chain_kernel, dim3((unsigned)ceil_div(nfiles, 64)), dim3(64), 0, s, dig, nbf * 20,
                       nfiles, (uint32_t)(nbf * 20), fh);
    return hip_err(hipGetLastError());
  }
  void* state = nullptr;  // every file's SHA-1 state between the two halves of its chain
  {
    const int arc = sfi::stream_alloc(&state, (size_t)nfiles * 20, s);
    if (arc != SF_OK) return arc;
  }
  const sf_chain_job first = {dig, nfiles, 1, nbf, state, nullptr};
  const sf_chain_job second = {dig, nfiles, 2, nbf, state, fh};
  int rc = sf_index_device_batch_chained_cols(base, nfiles, flen, bs, 0, cut, dig, nullptr, 0, s);
  if (rc == SF_OK) rc = sf_index_device_batch_chained_cols(base, nfiles, flen, bs, cut, nbf, dig, &first, 1, s);
  if (rc == SF_OK) rc = sf_index_device_batch_chained_cols(nullptr, 0, flen, bs, 0, nbf, nullptr, &second, 1, s);
  sfi::stream_free(state, s);
  return rc;
}

// The FILE_BLOCK messages of digests [0, n): every message is 33 + digits(bs)
// bytes but the last, whose size field is `last`.
int launch_wire(const uint8_t* d_digests, uint64_t n, uint32_t bs, uint32_t last, uint8_t* d_out,
                hipStream_t stream) {
  if (n == 0) return SF_OK;
  const uint64_t maxb = launch_max_blocks();
  if (n > maxb) {  // consecutive runs of messages, one launch each
    uint64_t db = 1;
    for (uint64_t v = bs; v >= 10; v /= 10) db++;
    for (uint64_t first = 0; first < n; first += maxb) {
      const uint64_t cnt = std::min(maxb, n - first);
      const int rc = launch_wire(d_digests + first * 20, cnt, bs, first + cnt == n ? last : bs,
                                 d_out + first * (33 + db), stream);
      if (rc) return rc;
    }
    return SF_OK;
  }
  sfi::clear_stale_error();
  hipLaunchKernelGGL(sf::wire_file_blocks_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, stream, d_digests,
                     n, bs, last, d_out);
  return hip_err(hipGetLastError());
}

}  // namespace sfi

using namespace sfi;

extern "C" {

const char* sf_version(void) { return "syncfast_amd 0.1.0 (gfx950)"; }

const char* sf_strerror(int code) {
  switch (code) {
    case SF_OK: return "ok";
    case SF_EIO: return "I/O error";
    case SF_EAGAIN: return "the file changed while it was indexed (cut it again and retry)";
    case SF_ENOMEM: return "out of memory";
    case SF_ENODEV: return "no HIP device or HIP runtime error";
    case SF_EINVAL: return "invalid argument";
    case SF_ENOSPC: return "output capacity too small";
    case SF_ERANGE: return "block outside the input";
    case SF_ETIMEDOUT: return "device-side wait timed out (no longer returned)";
    default: return "unknown error";
  }
}

int sf_device_count(int* n) {
  if (!n) return SF_EINVAL;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return SF_OK;
}

int sf_set_device(int device) { return hip_err(hipSetDevice(device)); }

int sf_index_device_fixed(const void* d_data, uint64_t len, uint32_t block_size, void* d_digests,
                          uint64_t cap_blocks, uint64_t* n_blocks, void* stream) {
  int rc = check_fixed_args(len, block_size);
  if (rc) return rc;
  const uint64_t nb = len ? ceil_div(len, block_size) : 0;
  if (n_blocks) *n_blocks = nb;
  if (nb > cap_blocks) return SF_ENOSPC;
  if (nb && (!d_data || !d_digests)) return SF_EINVAL;
  return launch_fixed(d_data, len, block_size, nb, d_digests, as_stream(stream));
}

int sf_index_device_blocks(const void* d_data, uint64_t len, const uint64_t* d_offsets, const uint32_t* d_sizes,
                           uint64_t n_blocks, void* d_digests, int* d_status, void* stream) {
  if (n_blocks == 0) return SF_OK;
  // d_data may be NULL only when len == 0 (then every in-range block is
  // empty and the kernel dereferences nothing).
  if (!d_offsets || !d_sizes || !d_digests || (!d_data && len)) return SF_EINVAL;
  return launch_table(d_data, len, d_offsets, d_sizes, n_blocks, d_digests, d_status, as_stream(stream));
}

int sf_index_device_fixed_weak(const void* d_data, uint64_t len, uint32_t block_size, void* d_digests,
                               uint32_t* d_weak, uint64_t cap_blocks, uint64_t* n_blocks, void* stream) {
  int rc = check_fixed_args(len, block_size);
  if (rc) return rc;
  const uint64_t nb = len ? ceil_div(len, block_size) : 0;
  if (n_blocks) *n_blocks = nb;
  if (nb > cap_blocks) return SF_ENOSPC;
  if (nb && (!d_data || !d_digests || !d_weak)) return SF_EINVAL;
  return launch_fixed(d_data, len, block_size, nb, d_digests, as_stream(stream), d_weak);
}

int sf_index_device_blocks_weak(const void* d_data, uint64_t len, const uint64_t* d_offsets, const uint32_t* d_sizes,
                                uint64_t n_blocks, void* d_digests, uint32_t* d_weak, int* d_status, void* stream) {
  if (n_blocks == 0) return SF_OK;
  if (!d_offsets || !d_sizes || !d_digests || !d_weak || (!d_data && len)) return SF_EINVAL;
  return launch_table(d_data, len, d_offsets, d_sizes, n_blocks, d_digests, d_status, as_stream(stream), d_weak);
}

static int sf_index_device_batch_body(const void* d_data, uint64_t len, const sf_file_desc* files, uint32_t n_files,
                          uint32_t block_size, void* d_digests, uint64_t cap_blocks, void* d_file_hashes,
                          uint64_t* first_block, uint64_t* n_blocks, int* d_status, void* stream) {
  int rc = check_fixed_args(len, block_size);
  if (rc) return rc;
  if (n_files && !files) return SF_EINVAL;
  hipStream_t s = as_stream(stream);
  // Plan: per-file block ranges (host, O(n_files)).
  std::vector<uint64_t> fb(n_files + 1);
  uint64_t total = 0;
  bool contiguous_aligned = true;  // files back to back, every file a whole number of blocks
  uint64_t expect = files && n_files ? files[0].offset : 0;
  for (uint32_t f = 0; f < n_files; f++) {
    if (files[f].offset > len || files[f].len > len - files[f].offset) return SF_ERANGE;
    fb[f] = total;
    total += files[f].len ? ceil_div(files[f].len, block_size) : 0;
    if (files[f].offset != expect || files[f].len % block_size) contiguous_aligned = false;
    expect = files[f].offset + files[f].len;
  }
  fb[n_files] = total;
  if (first_block) memcpy(first_block, fb.data(), sizeof(uint64_t) * (n_files + 1));
  if (n_blocks) *n_blocks = total;
  if (total > cap_blocks) return SF_ENOSPC;
  if (n_files == 0) return SF_OK;
  if ((!d_data && len) || (total && !d_digests)) return SF_EINVAL;  // all-empty files need no data

  // Equal-size, block-aligned, back-to-back files: the block table is a fixed
  // tiling of the batch, and each file's digest run is a fixed tiling of the
  // digest table (block = nbf*20 bytes), so nothing needs uploading.
  bool equal_files = contiguous_aligned && total > 0;
  for (uint32_t f = 1; f < n_files && equal_files; f++)
    if (files[f].len != files[0].len) equal_files = false;
  if (equal_files && total / n_files * 20 <= 0xFFFFFFFFull) {
    const uint64_t nbf = total / n_files;
    const uint8_t* base = static_cast<const uint8_t*>(d_data) + files[0].offset;
    if (!d_file_hashes)
      return launch_fixed(base, total * (uint64_t)block_size, block_size, total, d_digests, s);
    return batch_with_hashes(base, files[0].len, block_size, n_files, nbf, static_cast<uint8_t*>(d_digests),
                             static_cast<uint8_t*>(d_file_hashes), knob(K_BATCH_FUSED) != 0, s);
  }

  // Block table for the ragged case, file table for blocks_hash; one device
  // workspace, uploaded once.
  const bool need_table = !contiguous_aligned && total > 0;
  const bool need_fh = d_file_hashes != nullptr;
  // block table: offsets (u64) then sizes (u32), padded to 16 B so the file
  // table's u64 offsets that follow stay 8-B aligned (host and device)
  const size_t tbl_bytes = need_table ? (total * (sizeof(uint64_t) + sizeof(uint32_t)) + 15) & ~(size_t)15 : 0;
  const size_t fh_bytes = need_fh ? (size_t)n_files * (sizeof(uint64_t) + sizeof(uint32_t)) : 0;
  std::vector<uint8_t> host_ws(tbl_bytes + fh_bytes + 16);
  uint64_t* h_off = reinterpret_cast<uint64_t*>(host_ws.data());
  uint32_t* h_sz = reinterpret_cast<uint32_t*>(host_ws.data() + total * sizeof(uint64_t) * (need_table ? 1 : 0));
  if (need_table) {
    uint64_t i = 0;
    for (uint32_t f = 0; f < n_files; f++)
      for (uint64_t o = 0; o < files[f].len; o += block_size, i++) {
        h_off[i] = files[f].offset + o;
        h_sz[i] = (uint32_t)std::min<uint64_t>(block_size, files[f].len - o);
      }
  }
  uint64_t* h_foff = reinterpret_cast<uint64_t*>(host_ws.data() + tbl_bytes);
  uint32_t* h_fsz = reinterpret_cast<uint32_t*>(host_ws.data() + tbl_bytes + (need_fh ? n_files * sizeof(uint64_t) : 0));
  if (need_fh) {
    for (uint32_t f = 0; f < n_files; f++) {
      const uint64_t nbf = fb[f + 1] - fb[f];
      if (nbf * 20 > 0xFFFFFFFFull) return SF_EINVAL;
      h_foff[f] = fb[f] * 20;
      h_fsz[f] = (uint32_t)(nbf * 20);
    }
  }
  // Stream-ordered workspace: allocated, filled, used and freed on `s`, so
  // the call stays asynchronous.  (hipMemcpyAsync from pageable memory
  // returns once the bytes are staged, so host_ws may go out of scope.)
  uint8_t* dws = nullptr;
  const size_t ws_bytes = tbl_bytes + fh_bytes;
  if (ws_bytes) {
    if ((rc = sfi::stream_alloc(reinterpret_cast<void**>(&dws), ws_bytes, s)) != SF_OK) return rc;
    SF_HIP(hipMemcpyAsync(dws, host_ws.data(), ws_bytes, hipMemcpyHostToDevice, s));
  }
  do {
    if (total) {
      if (contiguous_aligned) {
        const uint8_t* base = static_cast<const uint8_t*>(d_data) + files[0].offset;
        rc = launch_fixed(base, fb[n_files] * (uint64_t)block_size, block_size, total, d_digests, s);
      } else {
        rc = launch_table(d_data, len, reinterpret_cast<const uint64_t*>(dws),
                          reinterpret_cast<const uint32_t*>(dws + total * sizeof(uint64_t)), total, d_digests,
                          nullptr, s);
      }
      if (rc) break;
    }
    if (need_fh) {
      // blocks_hash of every file at once: one lane per file hashes its own
      // run of 20-byte digests (a file with no blocks hashes the empty string).
      const uint8_t* dg =
          total ? static_cast<const uint8_t*>(d_digests) : static_cast<const uint8_t*>(d_file_hashes);
      rc = launch_table(dg, total * 20, reinterpret_cast<const uint64_t*>(dws + tbl_bytes),
                        reinterpret_cast<const uint32_t*>(dws + tbl_bytes + n_files * sizeof(uint64_t)), n_files,
                        d_file_hashes, nullptr, s);
    }
  } while (0);
  sfi::stream_free(dws, s);
  return rc;
}

int sf_index_device_batch_chained(const void* d_data, uint32_t n_files, uint64_t file_len, uint32_t block_size,
                                  void* d_digests, const sf_chain_job* jobs, uint32_t n_jobs, void* stream) {
  const uint64_t nbf = block_size ? file_len / block_size : 0;
  return sf_index_device_batch_chained_cols(d_data, n_files, file_len, block_size, 0, nbf, d_digests, jobs, n_jobs,
                                            stream);
}

int sf_index_device_batch_chained_cols(const void* d_data, uint32_t n_files, uint64_t file_len, uint32_t block_size,
                                       uint64_t col_lo, uint64_t col_hi, void* d_digests, const sf_chain_job* jobs,
                                       uint32_t n_jobs, void* stream) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (n_files && (file_len == 0 || file_len % block_size)) return SF_EINVAL;
  if (n_jobs > 2 || (n_jobs && !jobs)) return SF_EINVAL;
  const uint64_t nbf = file_len / block_size;
  // the whole files, or a column range in whole block waves of whole-wave files
  const bool whole = col_lo == 0 && col_hi == nbf;
  if (n_files && !whole && (col_lo >= col_hi || col_hi > nbf || nbf % 64 || col_lo % 64 || col_hi % 64))
    return SF_EINVAL;
  const uint64_t total = n_files ? nbf * n_files : 0;
  if (total && (!d_data || !d_digests)) return SF_EINVAL;
  if (total > launch_max_blocks()) return SF_EINVAL;  // one launch per batch: split the batch
  sf::ChainJob cj[2] = {};
  for (uint32_t k = 0; k < n_jobs; k++) {
    const sf_chain_job& j = jobs[k];
    if (!j.n_files) continue;
    // each file's digest run must start 16-B aligned (20 * blocks % 16 == 0)
    if (!j.d_digests || j.blocks == 0 || j.blocks % 4 || j.blocks * 20 > 0xFFFFFFF0ull || j.part > 2 ||
        (j.part != 0 && !j.d_state) || (j.part != 1 && !j.d_hashes))
      return SF_EINVAL;
    const uint32_t run_len = (uint32_t)(j.blocks * 20), data_ch = run_len / 64, half = data_ch / 2;
    cj[k].runs = static_cast<const uint8_t*>(j.d_digests);
    cj[k].state = static_cast<uint8_t*>(j.d_state);
    cj[k].hashes = static_cast<uint8_t*>(j.d_hashes);
    cj[k].files = j.n_files;
    cj[k].run_len = run_len;
    cj[k].lo = j.part == 2 ? half : 0;
    cj[k].hi = j.part == 1 ? half : data_ch;
    cj[k].part = j.part;
    cj[k].waves = (uint32_t)ceil_div(j.n_files, 64);  // chain waves, one per workgroup
  }
  const uint32_t wpf = whole ? 1u : (uint32_t)(nbf / 64), wpp = whole ? 1u : (uint32_t)((col_hi - col_lo) / 64);
  const uint64_t bwaves = whole ? ceil_div(total, 64) : (uint64_t)n_files * wpp;
  if (total == 0) return launch_chain_helper(cj[0], cj[1], as_stream(stream));  // chains alone: helper waves
  // A chain wave of the block launch stages 64 files' runs through one
  // buffer resource with 32-bit offsets (file b of the wave at b * run_len):
  // runs of 62.9 MB or more (3.1 M blocks per file) could pass 4 GiB within
  // one wave and wrap.  Such a job runs first, alone, on the helper-wave
  // chain kernel (64-bit addressing), stream-ordered before this launch:
  // its digests and states were completed by earlier launches.
  for (int k = 0; k < 2; k++) {
    if (!cj[k].waves || 64ull * cj[k].run_len + 128 <= 0xF0000000ull) continue;
    const sf::ChainJob none = {};
    if ((rc = launch_chain_helper(cj[k], none, as_stream(stream))) != SF_OK) return rc;
    cj[k] = none;
  }
  return launch_chained(static_cast<const uint8_t*>(d_data), total * (uint64_t)block_size, block_size, total,
                        static_cast<uint8_t*>(d_digests), pad_schedule(block_size), cj[0], cj[1], bwaves, wpf, wpp,
                        whole ? 0u : (uint32_t)(col_lo / 64), as_stream(stream));
}

int sf_wire_file_blocks_device(const void* d_digests, uint64_t n_blocks, uint32_t block_size, uint64_t file_len,
                               void* d_out, uint64_t cap, uint64_t* n_out, void* stream) {
  if (block_size == 0 || block_size > SF_MAX_BLOCK_SIZE) return SF_EINVAL;
  const uint64_t nb = file_len ? ceil_div(file_len, block_size) : 0;
  if (nb != n_blocks) return SF_EINVAL;
  uint64_t db = 1;
  for (uint64_t v = block_size; v >= 10; v /= 10) db++;
  const uint32_t last = nb ? (uint32_t)(file_len - (nb - 1) * block_size) : 0;
  uint64_t dl = 1;
  for (uint64_t v = last; v >= 10; v /= 10) dl++;
  const uint64_t bytes = nb ? (nb - 1) * (33 + db) + (33 + dl) : 0;
  if (n_out) *n_out = bytes;
  if (bytes > cap) return SF_ENOSPC;
  if (!nb) return SF_OK;
  if (!d_digests || !d_out) return SF_EINVAL;
  return launch_wire(static_cast<const uint8_t*>(d_digests), nb, block_size, last, static_cast<uint8_t*>(d_out),
                     as_stream(stream));
}

int sf_fill_splitmix_device(void* d_out, uint64_t len, uint64_t seed, uint64_t start, void* stream) {
  if (len == 0) return SF_OK;
  if (!d_out) return SF_EINVAL;
  const uint64_t nvec = len / 16 + 1;
  const unsigned grid = (unsigned)std::min<uint64_t>(ceil_div(nvec, 256), 65536);
  sfi::clear_stale_error();
  hipLaunchKernelGGL(sf::fill_splitmix_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     static_cast<uint8_t*>(d_out), len, seed, start);
  return hip_err(hipGetLastError());
}

}  // extern "C"

// C-ABI entry points: the bodies above, exceptions turned into error codes.
extern "C" {

int sf_index_device_batch(const void* d_data, uint64_t len, const sf_file_desc* files, uint32_t n_files,
                          uint32_t block_size, void* d_digests, uint64_t cap_blocks, void* d_file_hashes,
                          uint64_t* first_block, uint64_t* n_blocks, int* d_status, void* stream) {
  return guarded([&] { return sf_index_device_batch_body(d_data, len, files, n_files, block_size, d_digests, cap_blocks, d_file_hashes, first_block, n_blocks, d_status, stream); });
}

}  // extern "C"

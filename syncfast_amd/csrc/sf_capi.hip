// sf_capi.hip -- the C-ABI (include/syncfast_amd.h) over the gfx950 kernels.
//
// Every entry point here is a host function with plain pointers/sizes; the
// compute happens in the kernels of sf_kernels.hpp.  There is no CPU
// implementation of the block hashing in this library: without a HIP device
// the device entry points return SF_ENODEV.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/syncfast_amd.h"
#include "sf_kernels.hpp"

#include "host_sha1.h"

// Internal status of the in-place route (never returned through the C-ABI):
// the caller's pages could not be page-locked, take the staged route.
#define SF_ENOTSUP (-95)

namespace {

constexpr int kTile = 128;  // bytes of each block staged per LDS step
#ifndef SF_FIXED_WPE
#define SF_FIXED_WPE 1  // min waves/SIMD of the shipped fixed kernel (A/B: make variant EXTRA=-DSF_FIXED_WPE=4)
#endif

#ifdef SF_TUNING
inline int variant_choice() {
  const char* e = getenv("SF_VARIANT");
  return e ? atoi(e) : 0;
}
#endif

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int hip_err(hipError_t e) {
  if (e == hipSuccess) return SF_OK;
  if (e == hipErrorOutOfMemory) return SF_ENOMEM;
  return SF_ENODEV;
}

#define SF_HIP(call)                       \
  do {                                     \
    hipError_t _e = (call);                \
    if (_e != hipSuccess) return hip_err(_e); \
  } while (0)

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

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
                 hipStream_t stream, uint32_t* weak = nullptr) {
  if (nblocks == 0) return SF_OK;
  const unsigned grid = grid_for_blocks(nblocks);
  const sf::PadSchedule pad = pad_schedule(bs);
  const uint8_t* d = static_cast<const uint8_t*>(d_data);
  uint8_t* o = static_cast<uint8_t*>(d_digests);
  if (weak) {  // opt-in fused Adler-32 (a separate instantiation; the default kernel is unchanged)
    hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, 1, true>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs,
                       nblocks, o, pad, weak);
    return hip_err(hipGetLastError());
  }
#ifdef SF_TUNING
  // Tuning builds only (make variant EXTRA=-DSF_TUNING): SF_VARIANT selects a
  // (tile, waves-per-SIMD) instantiation for interleaved A/B in one process.
  switch (variant_choice()) {
    case 1: hipLaunchKernelGGL((sf::sha1_fixed_kernel<128, 5>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 2: hipLaunchKernelGGL((sf::sha1_fixed_kernel<64, 6>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 3: hipLaunchKernelGGL((sf::sha1_fixed_kernel<64, 8>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 4: hipLaunchKernelGGL((sf::sha1_fixed_kernel<64, 1>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 5: hipLaunchKernelGGL((sf::sha1_fixed_kernel<128, 4>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 6: hipLaunchKernelGGL((sf::sha1_fixed_kernel<128, 2>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 7: hipLaunchKernelGGL((sf::sha1_fixed_kernel<128, 3>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
    case 8:
      if (bs % 64 == 0 && (reinterpret_cast<uintptr_t>(d) & 15u) == 0) {
        hipLaunchKernelGGL(sf::sha1_fixed2_kernel, dim3((unsigned)ceil_div(ceil_div(nblocks, 128), sf::kWavesPerWG)),
                           dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad);
        break;
      }
      hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, 1>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr);
      break;
    default: hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, 1>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr); break;
  }
#else
  hipLaunchKernelGGL((sf::sha1_fixed_kernel<kTile, SF_FIXED_WPE>), dim3(grid), dim3(sf::kThreads), 0, stream, d, len, bs, nblocks, o, pad, nullptr);
#endif
  return hip_err(hipGetLastError());
}

int launch_table(const void* d_data, uint64_t len, const uint64_t* d_offsets, const uint32_t* d_sizes,
                 uint64_t nblocks, void* d_digests, int* d_status, hipStream_t stream, uint32_t* weak = nullptr) {
  if (nblocks == 0) return SF_OK;
  const unsigned grid = grid_for_blocks(nblocks);
  if (weak)
    hipLaunchKernelGGL((sf::sha1_table_kernel<kTile, true>), dim3(grid), dim3(sf::kThreads), 0, stream,
                       static_cast<const uint8_t*>(d_data), len, d_offsets, d_sizes, nblocks,
                       static_cast<uint8_t*>(d_digests), d_status, weak);
  else
    hipLaunchKernelGGL((sf::sha1_table_kernel<kTile, false>), dim3(grid), dim3(sf::kThreads), 0, stream,
                       static_cast<const uint8_t*>(d_data), len, d_offsets, d_sizes, nblocks,
                       static_cast<uint8_t*>(d_digests), d_status, nullptr);
  return hip_err(hipGetLastError());
}

// Many equal-size, block-aligned files back to back, with their per-file
// blocks_hash.  Staged (S > 1): ONE launch of sha1_staged_kernel whose first
// workgroups run the per-file chains while the others hash the blocks in S
// column stages; only the last stage's chain work follows the last block.
// Unstaged: the block kernel, then the stand-alone chain kernel.
//
// The chain waves wait on block waves, so the staged launch needs (a) block
// workgroups to find free slots while every chain workgroup is resident and
// (b) somewhere to report a chain that gave up.  (a): the chain workgroups
// are kept to at most one per CU (a quarter of the staged kernel's 4
// workgroups per CU); larger batches (> 256 x 256 files) take the unstaged
// path, which never waits.  (b): d_status (device int32) receives
// SF_ETIMEDOUT; with d_status == NULL the unstaged path is taken.
// SF_CHAIN_SPIN_LIMIT (test knob) bounds the polls of each wait (default
// 2^24, several seconds).
inline unsigned device_cus() {
  static std::atomic<int> cached{0};
  int v = cached.load();
  if (v > 0) return (unsigned)v;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess ||
      hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0) {
    (void)hipGetLastError();
    return 64;  // conservative (a quarter of MI355X's CUs)
  }
  cached.store(v);
  return (unsigned)v;
}

inline uint32_t chain_spin_limit() {
  const char* e = getenv("SF_CHAIN_SPIN_LIMIT");
  return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 24);
}

int batch_staged(const uint8_t* base, uint64_t flen, uint32_t bs, uint32_t nfiles, uint64_t nbf, uint8_t* dig,
                 uint8_t* fh, int* d_status, hipStream_t s) {
  int S = 1;
  const char* se = getenv("SF_STAGES");  // A/B knob; default up to 16 stages
  const int smax = se ? std::max(1, atoi(se)) : 16;
  for (int cand : {32, 16, 8, 4, 2})
    if (cand <= smax && nbf % (64ull * cand) == 0 && ((uint64_t)nfiles * (nbf / cand)) % 64 == 0) {
      S = cand;
      break;
    }
  if (!d_status || ceil_div(nfiles, 64 * sf::kWavesPerWG) > device_cus()) S = 1;
  if (S == 1) {
    int rc = launch_fixed(base, nbf * nfiles * (uint64_t)bs, bs, nbf * nfiles, dig, s);
    if (rc) return rc;
    hipLaunchKernelGGL(sf::sha1_chain_kernel, dim3((unsigned)ceil_div(nfiles, 64)), dim3(64), 0, s, dig, nbf * 20,
                       nfiles, (uint32_t)(nbf * 20), fh);
    return hip_err(hipGetLastError());
  }
  const uint64_t m = nbf / S;
  const sf::PadSchedule pad = pad_schedule(bs);
  uint32_t* words = nullptr;  // [0, 32): stage counters
  const size_t wbytes = 32 * sizeof(uint32_t);
  SF_HIP(hipMallocAsync(reinterpret_cast<void**>(&words), wbytes, s));
  SF_HIP(hipMemsetAsync(words, 0, wbytes, s));
#ifdef SF_TUNING
  // SF_STAGED_EXP: 1 = no chain workgroups (publish only), 2 = no chains and
  // no publish (block hashing in stage order only) -- cost breakdown only.
  const char* xe = getenv("SF_STAGED_EXP");
  const int exp = xe ? atoi(xe) : 0;
#else
  const int exp = 0;
#endif
  const unsigned chain_wgs = exp ? 0u : (unsigned)ceil_div(nfiles, 64 * sf::kWavesPerWG);
  const unsigned grid = chain_wgs + grid_for_blocks((uint64_t)nfiles * nbf);
  hipLaunchKernelGGL(sf::sha1_staged_kernel<kTile>, dim3(grid), dim3(sf::kThreads), 0, s, base, bs, (uint64_t)nfiles,
                     nbf, m, flen, dig, nbf, pad, words, chain_wgs, exp == 2 ? nullptr : fh, d_status,
                     chain_spin_limit());
  int rc = hip_err(hipGetLastError());
  (void)hipFreeAsync(words, s);
  return rc;
}

int check_fixed_args(uint64_t len, uint32_t bs) {
  if (bs == 0 || bs > SF_MAX_BLOCK_SIZE) return SF_EINVAL;
  (void)len;
  return SF_OK;
}

// RAII pinned allocation (the in-place route's bounce buffer).
struct PinBuf {
  void* p = nullptr;
  ~PinBuf() { if (p) (void)hipHostFree(p); }
};

// Per-device resources of the host-memory entry points (streams, events,
// device stage buffers, digest table, pinned stages), kept between calls:
// setting them up cost ~8 ms per call (hipMalloc / hipHostMalloc of the
// stages), ten times the PCIe time of a 64 MiB file.  One call at a time uses
// a device's set; a concurrent call gets a private set.  Capacities only
// grow, up to kCacheMax per buffer; a larger buffer is allocated for the call
// alone.  sf_release_host_cache() frees the sets.  They are never freed from
// a static destructor: the HIP runtime may already be gone at exit.
constexpr uint64_t kCacheMax = 512ull << 20;
constexpr int kMaxDevices = 64;

struct HostRes {
  hipStream_t s[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  // Slots (device and pinned alike): 0, 1 = the two stages; 2 = the digest
  // table of one file; 3, 4 = the digest tables of sf_index_files' two
  // stages; 5, 6 = their blocks_hash arrays; 7 = their status words.
  static constexpr int kSlots = 8;
  void* dev[kSlots] = {};
  uint64_t dev_cap[kSlots] = {};
  void* pin[kSlots] = {};
  uint64_t pin_cap[kSlots] = {};
  void free_all() {
    for (int i = 0; i < kSlots; i++) {
      if (dev[i]) (void)hipFree(dev[i]);
      if (pin[i]) (void)hipHostFree(pin[i]);
      dev[i] = pin[i] = nullptr;
      dev_cap[i] = pin_cap[i] = 0;
    }
    for (int i = 0; i < 2; i++) {
      if (s[i]) (void)hipStreamDestroy(s[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      s[i] = nullptr;
      ev[i] = nullptr;
    }
  }
};

std::mutex g_res_mu[kMaxDevices];
HostRes* g_res[kMaxDevices];

class HostLease {
 public:
  HostLease() {
    int d = 0;
    if (hipGetDevice(&d) == hipSuccess && d >= 0 && d < kMaxDevices) {
      lk_ = std::unique_lock<std::mutex>(g_res_mu[d], std::try_to_lock);
      if (lk_.owns_lock()) {
        if (!g_res[d]) g_res[d] = new HostRes;
        r_ = g_res[d];
        return;
      }
    } else {
      (void)hipGetLastError();
    }
    own_ = new HostRes;
    r_ = own_;
  }
  ~HostLease() {
    for (int i = 0; i < 2; i++)  // an early error return may leave copies in flight
      if (r_->s[i]) (void)hipStreamSynchronize(r_->s[i]);
    for (void* p : tmp_dev_) (void)hipFree(p);
    for (void* p : tmp_pin_) (void)hipHostFree(p);
    if (own_) {
      own_->free_all();
      delete own_;
    }
  }
  HostLease(const HostLease&) = delete;
  HostLease& operator=(const HostLease&) = delete;
  int streams(hipStream_t*& s, hipEvent_t*& ev) {
    for (int i = 0; i < 2; i++) {
      if (!r_->s[i]) SF_HIP(hipStreamCreateWithFlags(&r_->s[i], hipStreamNonBlocking));
      if (!r_->ev[i]) SF_HIP(hipEventCreateWithFlags(&r_->ev[i], hipEventDisableTiming));
    }
    s = r_->s;
    ev = r_->ev;
    return SF_OK;
  }
  int dev(int i, uint64_t need, void** out) { return get(r_->dev[i], r_->dev_cap[i], need, false, out); }
  int pin(int i, uint64_t need, void** out) { return get(r_->pin[i], r_->pin_cap[i], need, true, out); }

 private:
  int get(void*& slot, uint64_t& cap, uint64_t need, bool pinned, void** out) {
    need = std::max<uint64_t>(need, 1);
    if (need <= cap) {
      *out = slot;
      return SF_OK;
    }
    void* p = nullptr;
    if (pinned) SF_HIP(hipHostMalloc(&p, need, hipHostMallocDefault));
    else SF_HIP(hipMalloc(&p, need));
    if (need > kCacheMax) {
      (pinned ? tmp_pin_ : tmp_dev_).push_back(p);
    } else {
      if (slot) (void)(pinned ? hipHostFree(slot) : hipFree(slot));
      slot = p;
      cap = need;
    }
    *out = p;
    return SF_OK;
  }
  std::unique_lock<std::mutex> lk_;
  HostRes* r_ = nullptr;
  HostRes* own_ = nullptr;
  std::vector<void*> tmp_dev_, tmp_pin_;
};

// Reader threads of the pread routes (sf_index_file, sf_index_files).
// SF_IO_THREADS overrides the default of 16 (A/B knob).  With the stat phase
// parallel too, 16 readers beat 8 on many small files (10,537 files of
// 0-200 KiB: 29.3 vs 24.1 GB/s, 12 and 24 no better; 8 MiB files flat at
// 33-34 GB/s; profiles/r02/e2e/io_threads_8_12_16_24.log).
inline unsigned io_threads() {
  const char* e = getenv("SF_IO_THREADS");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? (unsigned)std::min(v, 64) : 16u;
}

// Smallest host buffer / page-cache-resident file that sf_index_buffer /
// sf_index_file copy in place (page-locked) instead of staging through the
// pinned stages.  Per call, with the per-device set cached
// (scripts/inplace_min_probe.py): a buffer gains in place from 1 MiB up
// (7.6 vs 6.1 GB/s; 32 MiB: 45 vs 21); a file only from ~16 MiB (mapping and
// locking page-cache pages loses to the 8-thread pread below 8 MiB: 4 MiB
// 8.7 vs 10.3 GB/s; 32 MiB 24.3 vs 23.6).  SF_INPLACE_MIN_MIB overrides both
// (A/B knob).
inline uint64_t inplace_min_bytes(bool file) {
  const char* e = getenv("SF_INPLACE_MIN_MIB");
  const long v = e ? atol(e) : -1;
  if (v >= 0) return (uint64_t)v << 20;
  return file ? 16ull << 20 : 1ull << 20;
}

// Chunk of input handled per pipeline stage: a whole number of blocks, about
// 256 MiB.
inline uint64_t stage_bytes(uint32_t bs) {
  const uint64_t target = 256ull << 20;
  const uint64_t nb = std::max<uint64_t>(1, target / bs);
  return nb * bs;
}

// Shared driver of sf_index_buffer / sf_index_file: `read(dst, off, n)`
// fills a pinned staging buffer with input bytes [off, off+n).
template <typename ReadFn>
int index_pipelined(uint64_t len, uint32_t bs, sf_block_sig* out, uint64_t cap, uint64_t* n_out, ReadFn read) {
  const uint64_t nblocks = len ? ceil_div(len, bs) : 0;
  if (n_out) *n_out = nblocks;
  if (nblocks > cap) return SF_ENOSPC;
  if (nblocks == 0) return SF_OK;
  const uint64_t stage = std::min<uint64_t>(stage_bytes(bs), len);
  const uint64_t nstages = ceil_div(len, stage);
  HostLease res;
  hipStream_t* st;
  hipEvent_t* done;
  void *ddata[2], *pin[2], *ddig, *pdig;
  int rc = res.streams(st, done);
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, stage, &ddata[i]);
    if (rc == SF_OK) rc = res.pin(i, stage, &pin[i]);
  }
  if (rc == SF_OK) rc = res.dev(2, nblocks * 20, &ddig);
  if (rc == SF_OK) rc = res.pin(2, nblocks * 20, &pdig);
  if (rc != SF_OK) return rc;
  for (uint64_t k = 0; k < nstages && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    const uint64_t off = k * stage;
    const uint64_t n = std::min(stage, len - off);
    if (k >= 2) {
      if (hipEventSynchronize(done[b]) != hipSuccess) { rc = SF_ENODEV; break; }
    }
    rc = read(static_cast<uint8_t*>(pin[b]), off, n);
    if (rc != SF_OK) break;
    if (hipMemcpyAsync(ddata[b], pin[b], n, hipMemcpyHostToDevice, st[b]) != hipSuccess) { rc = SF_ENODEV; break; }
    const uint64_t first_blk = off / bs;
    const uint64_t nb = ceil_div(n, bs);
    rc = launch_fixed(ddata[b], n, bs, nb, static_cast<uint8_t*>(ddig) + first_blk * 20, st[b]);
    if (rc != SF_OK) break;
    if (hipEventRecord(done[b], st[b]) != hipSuccess) { rc = SF_ENODEV; break; }
  }
  for (int i = 0; i < 2; i++)
    if (hipStreamSynchronize(st[i]) != hipSuccess && rc == SF_OK) rc = SF_ENODEV;
  if (rc != SF_OK) return rc;
  SF_HIP(hipMemcpyAsync(pdig, ddig, nblocks * 20, hipMemcpyDeviceToHost, st[0]));
  SF_HIP(hipStreamSynchronize(st[0]));
  const uint8_t* dg = static_cast<const uint8_t*>(pdig);
  for (uint64_t i = 0; i < nblocks; i++) {
    out[i].offset = i * bs;
    out[i].size = (uint32_t)std::min<uint64_t>(bs, len - i * bs);
    memcpy(out[i].sha1, dg + 20 * i, 20);
  }
  return SF_OK;
}

}  // namespace

extern "C" {

const char* sf_version(void) { return "syncfast_amd 0.1.0 (gfx950)"; }

const char* sf_strerror(int code) {
  switch (code) {
    case SF_OK: return "ok";
    case SF_EIO: return "I/O error";
    case SF_ENOMEM: return "out of memory";
    case SF_ENODEV: return "no HIP device or HIP runtime error";
    case SF_EINVAL: return "invalid argument";
    case SF_ENOSPC: return "output capacity too small";
    case SF_ERANGE: return "block outside the input";
    case SF_ETIMEDOUT: return "device-side wait timed out (blocks_hash not computed)";
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

int sf_release_host_cache(void) {
  for (int d = 0; d < kMaxDevices; d++) {
    std::lock_guard<std::mutex> lk(g_res_mu[d]);  // waits for a call using the set
    if (g_res[d]) {
      g_res[d]->free_all();
      delete g_res[d];
      g_res[d] = nullptr;
    }
  }
  return SF_OK;
}

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

int sf_index_device_batch(const void* d_data, uint64_t len, const sf_file_desc* files, uint32_t n_files,
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
    return batch_staged(base, files[0].len, block_size, n_files, nbf, static_cast<uint8_t*>(d_digests),
                        static_cast<uint8_t*>(d_file_hashes), d_status, s);
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
    SF_HIP(hipMallocAsync(reinterpret_cast<void**>(&dws), ws_bytes, s));
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
  if (dws) (void)hipFreeAsync(dws, s);
  return rc;
}

int sf_index_device_batch_chained(const void* d_data, uint32_t n_files, uint64_t file_len, uint32_t block_size,
                                  void* d_digests, const sf_chain_job* jobs, uint32_t n_jobs, void* stream) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (n_files && (file_len == 0 || file_len % block_size)) return SF_EINVAL;
  if (n_jobs > 2 || (n_jobs && !jobs)) return SF_EINVAL;
  const uint64_t total = n_files ? (file_len / block_size) * n_files : 0;
  if (total && (!d_data || !d_digests)) return SF_EINVAL;
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
  // grid: C mixed workgroups (1 chain wave + 3 block waves), then 4 block
  // waves per workgroup for the rest
  const uint64_t C_ = cj[0].waves + cj[1].waves;
  const uint64_t bwaves = ceil_div(total, 64);
  const uint64_t rest = bwaves > 3 * C_ ? bwaves - 3 * C_ : 0;
  const unsigned grid = (unsigned)(C_ + ceil_div(rest, sf::kWavesPerWG));
  if (grid == 0) return SF_OK;
  hipLaunchKernelGGL(sf::sha1_fixed_chained_kernel<kTile>, dim3(grid), dim3(sf::kThreads), 0, as_stream(stream),
                     static_cast<const uint8_t*>(d_data), total * (uint64_t)block_size, block_size, total,
                     static_cast<uint8_t*>(d_digests), pad_schedule(block_size), cj[0], cj[1]);
  return hip_err(hipGetLastError());
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
  hipLaunchKernelGGL(sf::wire_file_blocks_kernel, dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const uint8_t*>(d_digests), nb, block_size, last, static_cast<uint8_t*>(d_out));
  return hip_err(hipGetLastError());
}

#ifndef SF_WIRE_CHUNK_DEFAULT
#define SF_WIRE_CHUNK_DEFAULT (1ull << 18)
#endif
static constexpr uint64_t kWireChunk = SF_WIRE_CHUNK_DEFAULT;  // messages per chunk (~9.4 MB at 4 KiB blocks)

int sf_wire_file_blocks_fd(const void* d_digests, uint64_t n_blocks, uint32_t block_size, uint64_t file_len, int fd,
                           uint64_t* n_written, void* stream) {
  if (n_written) *n_written = 0;
  if (block_size == 0 || block_size > SF_MAX_BLOCK_SIZE) return SF_EINVAL;
  const uint64_t nb = file_len ? ceil_div(file_len, block_size) : 0;
  if (nb != n_blocks) return SF_EINVAL;
  if (!nb) return SF_OK;
  if (!d_digests || fd < 0) return SF_EINVAL;
  uint64_t db = 1;
  for (uint64_t v = block_size; v >= 10; v /= 10) db++;
  const uint32_t last = (uint32_t)(file_len - (nb - 1) * block_size);
  uint64_t dl = 1;
  for (uint64_t v = last; v >= 10; v /= 10) dl++;
  const uint64_t msg = 33 + db;  // every message but the last
  const char* ce = getenv("SF_WIRE_CHUNK");  // messages per chunk (test knob)
  const uint64_t per = std::max<uint64_t>(1, ce ? strtoull(ce, nullptr, 10) : kWireChunk);
  const uint64_t nchunks = ceil_div(nb, per);
  const uint64_t cap = std::min(per, nb) * msg + (33 + dl);
  // Streams, events and the two chunk buffers (device + pinned) come from the
  // per-device set the other host entry points keep between calls: pinning
  // two chunk buffers per call cost more than the call's copies.
  HostLease res;
  hipStream_t* st;
  hipEvent_t* ev;
  void *dout[2], *pin[2];
  hipEvent_t ready = nullptr;
  uint64_t bytes_of[2] = {0, 0};
  int rc = res.streams(st, ev);
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, cap, &dout[i]);
    if (rc == SF_OK) rc = res.pin(i, cap, &pin[i]);
  }
  if (rc != SF_OK) return rc;
  SF_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  if (hipEventRecord(ready, as_stream(stream)) != hipSuccess ||  // the digests are produced on the caller's stream
      hipStreamWaitEvent(st[0], ready, 0) != hipSuccess || hipStreamWaitEvent(st[1], ready, 0) != hipSuccess)
    rc = SF_ENODEV;
  uint64_t written = 0;
  auto flush = [&](int b) {  // write chunk buffer b to fd, in order
    if (hipEventSynchronize(ev[b]) != hipSuccess) return SF_ENODEV;
    const uint8_t* p = static_cast<const uint8_t*>(pin[b]);
    for (uint64_t done = 0; done < bytes_of[b];) {
      const ssize_t w = write(fd, p + done, bytes_of[b] - done);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return SF_EIO;
      done += (uint64_t)w;
      written += (uint64_t)w;
    }
    return SF_OK;
  };
  // chunk k: device builds its messages, D2H into pin[k&1]; the host writes
  // chunk k-2 while the device works on chunk k.
  for (uint64_t k = 0; k < nchunks && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    if (k >= 2 && (rc = flush(b)) != SF_OK) break;
    const uint64_t i0 = k * per, n = std::min(per, nb - i0);
    const bool final_chunk = i0 + n == nb;
    const uint32_t lsz = final_chunk ? last : block_size;
    bytes_of[b] = (n - 1) * msg + (final_chunk ? 33 + dl : msg);
    hipLaunchKernelGGL(sf::wire_file_blocks_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st[b],
                       static_cast<const uint8_t*>(d_digests) + i0 * 20, n, block_size, lsz,
                       static_cast<uint8_t*>(dout[b]));
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(pin[b], dout[b], bytes_of[b], hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
        hipEventRecord(ev[b], st[b]) != hipSuccess)
      rc = SF_ENODEV;
  }
  for (uint64_t k = nchunks >= 2 ? nchunks - 2 : 0; k < nchunks && rc == SF_OK; k++) rc = flush((int)(k & 1));
  for (int i = 0; i < 2; i++) (void)hipStreamSynchronize(st[i]);
  (void)hipEventDestroy(ready);
  if (n_written) *n_written = written;
  return rc;
}

int sf_fill_splitmix_device(void* d_out, uint64_t len, uint64_t seed, uint64_t start, void* stream) {
  if (len == 0) return SF_OK;
  if (!d_out) return SF_EINVAL;
  const uint64_t nvec = len / 16 + 1;
  const unsigned grid = (unsigned)std::min<uint64_t>(ceil_div(nvec, 256), 65536);
  hipLaunchKernelGGL(sf::fill_splitmix_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     static_cast<uint8_t*>(d_out), len, seed, start);
  return hip_err(hipGetLastError());
}

// In-place route of sf_index_buffer / sf_index_file: the DMA engine reads the
// caller's pages (or the page-cache pages of a mapped file) directly, no
// staging memcpy.  Per ~256 MiB stage, on alternating streams: H2D, the
// block kernel, D2H of the stage's digests.  The host overlaps the rest with
// the PCIe link:
//   - the pages are page-locked (hipHostRegister) one region ahead of the
//     copy that reads them, instead of all before the first copy;
//   - stage k-1's rows are written and its digests folded into the file's
//     blocks_hash (src/index.rs:661-682) while stage k is on the link.
// Region k = [page_up(data + k*stage), page_up(data + (k+1)*stage)), so a
// stage's bytes lie in regions k-1 (its head, up to the first page edge) and
// k, and no page is registered twice.  A
// region that cannot be registered after the first one switches the rest of
// the stages to a pinned bounce buffer (memcpy, one stage at a time): slower,
// same result.  For a mapped file (fd >= 0) the bounce buffer is filled
// with pread from the fd, never by touching the mapping: a region that cannot
// be page-locked is typically one past a concurrent truncation, and reading
// the mapping there would raise SIGBUS; pread returns short instead, and the
// call fails with SF_EIO (the reference's read() would see the short file).
// Returns SF_ENOTSUP (nothing done) when the first region cannot be
// registered, so the caller can take its staged route.
// SF_INPLACE_SERIAL=1 registers the whole range first and writes rows and
// blocks_hash after the last stage (the previous form; A/B knob).
static int index_inplace(const uint8_t* data, uint64_t len, uint32_t bs, sf_block_sig* out, uint64_t cap,
                         uint64_t* n_out, uint8_t* blocks_hash, int fd = -1) {
  const uint64_t nblocks = ceil_div(len, bs);
  if (n_out) *n_out = nblocks;
  if (nblocks > cap) return SF_ENOSPC;
  const char* ser = getenv("SF_INPLACE_SERIAL");
  const bool serial = ser && atoi(ser);
  const uint64_t stage = std::min<uint64_t>(stage_bytes(bs), len);
  const uint64_t nstages = ceil_div(len, stage);
  const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
  const uintptr_t lo = (uintptr_t)data & ~(uintptr_t)(pg - 1);
  const uintptr_t hi = ((uintptr_t)data + len + pg - 1) & ~(uintptr_t)(pg - 1);
  auto edge = [&](uint64_t k) -> uintptr_t {  // start of region k (k = nstages: end of the range)
    if (k == 0) return lo;
    if (k >= nstages) return hi;
    return std::min<uintptr_t>(hi, ((uintptr_t)data + k * stage + pg - 1) & ~(uintptr_t)(pg - 1));
  };
  enum { kEmpty, kLocked, kPageable, kPinned };  // kPinned: the caller's pages are already page-locked
  std::vector<std::pair<void*, int>> regs;  // (region start, state)
  struct Unreg {
    std::vector<std::pair<void*, int>>* r;
    ~Unreg() {
      for (auto& x : *r)
        if (x.second == kLocked) (void)hipHostUnregister(x.first);
    }
  } unreg{&regs};
  // A buffer that is already page-locked (hipHostMalloc, or registered by the
  // caller) is copied from as it is: hipHostRegister would refuse it.
  auto pinned_at = [](const void* p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return at.type == hipMemoryTypeHost;
  };
  const bool prepinned = pinned_at(data) && pinned_at(data + len - 1);
  const char* fail_at = getenv("SF_INPLACE_FAIL_AT");  // test hook: region k "fails" to register
  const long fail_k = fail_at ? atol(fail_at) : -1;
  auto reg = [&](uint64_t k) {
    const uintptr_t a = serial ? lo : edge(k), e = serial ? hi : edge(k + 1);
    // after one failure every later region stays pageable (a stage straddles
    // the page it shares with the previous region)
    if (e <= a) { regs.push_back({(void*)a, kEmpty}); return; }
    if (prepinned) { regs.push_back({(void*)a, kPinned}); return; }
    if ((!regs.empty() && regs.back().second == kPageable) || (long)k == fail_k) {
      regs.push_back({(void*)a, kPageable});
      return;
    }
    const hipError_t err = hipHostRegister((void*)a, e - a, hipHostRegisterReadOnly);
    if (err != hipSuccess) (void)hipGetLastError();
    regs.push_back({(void*)a, err == hipSuccess                               ? kLocked
                              : err == hipErrorHostMemoryAlreadyRegistered ? kPinned
                                                                           : kPageable});
  };
  reg(0);
  if (regs[0].second != kLocked && regs[0].second != kPinned) return SF_ENOTSUP;
  PinBuf bounce;  // only if a region after the first cannot be registered
  HostLease res;  // declared after unreg and bounce: its release waits for the streams first
  hipStream_t* st;
  hipEvent_t* done;
  void *ddata[2], *ddig, *pdig;
  int rc = res.streams(st, done);
  for (int i = 0; i < 2 && rc == SF_OK; i++) rc = res.dev(i, stage, &ddata[i]);
  if (rc == SF_OK) rc = res.dev(2, nblocks * 20, &ddig);
  if (rc == SF_OK) rc = res.pin(2, nblocks * 20, &pdig);
  if (rc != SF_OK) return rc;
  sf_host_sha1_stream bh;
  sf_host_sha1_begin(&bh);
  const uint8_t* dg = static_cast<const uint8_t*>(pdig);
  auto rows = [&](uint64_t k) {  // rows + blocks_hash of stage k (its digests are on the host)
    const uint64_t b0 = k * stage / bs, b1 = std::min(nblocks, ceil_div((k + 1) * stage, bs));
    for (uint64_t i = b0; i < b1; i++) {
      out[i].offset = i * bs;
      out[i].size = (uint32_t)std::min<uint64_t>(bs, len - i * bs);
      memcpy(out[i].sha1, dg + 20 * i, 20);
    }
    if (blocks_hash) sf_host_sha1_update(&bh, dg + 20 * b0, (b1 - b0) * 20);
  };
  for (uint64_t k = 0; k < nstages && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    const uint64_t off = k * stage;
    const uint64_t n = std::min(stage, len - off);
    const uint64_t b0 = off / bs, nb = ceil_div(n, bs);
    uint8_t* dd = static_cast<uint8_t*>(ddig) + b0 * 20;
    const uint8_t* src = data + off;
    if (!serial && regs.back().second == kPageable) {  // region k is not page-locked: bounce
      for (int i = 0; i < 2; i++)
        if (hipStreamSynchronize(st[i]) != hipSuccess) rc = SF_ENODEV;
      if (rc != SF_OK) break;
      if (!bounce.p) SF_HIP(hipHostMalloc(&bounce.p, stage, hipHostMallocDefault));
      if (fd >= 0) {
        uint8_t* d = static_cast<uint8_t*>(bounce.p);
        for (uint64_t got = 0; got < n && rc == SF_OK;) {
          const ssize_t r = pread(fd, d + got, n - got, (off_t)(off + got));
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) rc = SF_EIO;  // error, or the file shrank under us
          else got += (uint64_t)r;
        }
        if (rc != SF_OK) break;
      } else {
        memcpy(bounce.p, src, n);
      }
      src = static_cast<const uint8_t*>(bounce.p);
    }
    // A copy must lie inside ONE registration: a stage that starts mid-page
    // copies its head (up to the page edge, in region k-1) separately from
    // the rest (region k).
    const uint64_t head = (serial || src != data + off || k == 0) ? 0 : std::min<uint64_t>(n, edge(k) - (uintptr_t)src);
    // stream b is in order: the copy into ddata[b] waits for the kernel of
    // stage k-2 that read it.
    if ((head && hipMemcpyAsync(ddata[b], src, head, hipMemcpyHostToDevice, st[b]) != hipSuccess) ||
        (n > head && hipMemcpyAsync(static_cast<uint8_t*>(ddata[b]) + head, src + head, n - head,
                                    hipMemcpyHostToDevice, st[b]) != hipSuccess)) {
      rc = SF_ENODEV;
      break;
    }
    rc = launch_fixed(ddata[b], n, bs, nb, dd, st[b]);
    if (rc != SF_OK) break;
    if (!serial) {
      if (hipMemcpyAsync(static_cast<uint8_t*>(pdig) + b0 * 20, dd, nb * 20, hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
          hipEventRecord(done[b], st[b]) != hipSuccess) { rc = SF_ENODEV; break; }
      if (k + 1 < nstages) reg(k + 1);
      if (k >= 1) {
        if (hipEventSynchronize(done[b ^ 1]) != hipSuccess) { rc = SF_ENODEV; break; }
        rows(k - 1);
      }
    }
  }
  for (int i = 0; i < 2; i++)
    if (hipStreamSynchronize(st[i]) != hipSuccess && rc == SF_OK) rc = SF_ENODEV;
  if (rc != SF_OK) return rc;
  if (serial) {
    SF_HIP(hipMemcpyAsync(pdig, ddig, nblocks * 20, hipMemcpyDeviceToHost, st[0]));
    SF_HIP(hipStreamSynchronize(st[0]));
    for (uint64_t k = 0; k < nstages; k++) rows(k);
  } else {
    rows(nstages - 1);
  }
  if (blocks_hash) sf_host_sha1_final(&bh, blocks_hash);
  return SF_OK;
}

}  // extern "C"

namespace {

// Staged file pipeline (sf_index_file's pread route and the sequential
// route of sf_index_fd): two pinned stages of whole blocks (the last one
// short).  `fill(dst, off, cap, &n, &eof)` puts the next input bytes into a
// pinned stage; per stage, on alternating streams, H2D + block kernel + D2H of
// the stage's digests.  While stage k is being filled, stage k-1 is on the
// device and stage k-2's rows are emitted (`emit(first_block, n_blocks,
// digests, stage_bytes)`) and its digests folded into the streaming
// blocks_hash (src/index.rs:661-682), in order.  No device memory maps or
// registers the caller's file: the host only ever reads it with read/pread.
inline uint64_t file_stage_bytes(uint32_t bs) {
  const char* se = getenv("SF_STREAM_STAGE_MIB");  // test knob: small stages exercise the pipeline
  const uint64_t want = se ? std::max<uint64_t>(1, strtoull(se, nullptr, 10)) << 20 : (256ull << 20);
  return std::max<uint64_t>(1, want / bs) * bs;
}

template <typename FillFn, typename EmitFn>
int staged_pipeline(uint32_t bs, uint64_t stage, FillFn fill, EmitFn emit, uint8_t* blocks_hash) {
  const uint64_t sblocks = stage / bs;
  HostLease res;
  hipStream_t* st;
  hipEvent_t* done;
  void *ddata[2], *pin[2], *ddig[2], *pdig[2];
  int rc = res.streams(st, done);
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, stage, &ddata[i]);
    if (rc == SF_OK) rc = res.pin(i, stage, &pin[i]);
    if (rc == SF_OK) rc = res.dev(3 + i, sblocks * 20, &ddig[i]);
    if (rc == SF_OK) rc = res.pin(3 + i, sblocks * 20, &pdig[i]);
  }
  if (rc != SF_OK) return rc;
  sf_host_sha1_stream bh;
  sf_host_sha1_begin(&bh);
  uint64_t bytes_of[2] = {0, 0}, first_of[2] = {0, 0};
  bool busy[2] = {false, false};
  auto harvest = [&](int b) {
    if (hipEventSynchronize(done[b]) != hipSuccess) return SF_ENODEV;
    busy[b] = false;
    const uint64_t nb = ceil_div(bytes_of[b], bs);
    const uint8_t* dg = static_cast<const uint8_t*>(pdig[b]);
    const int r = emit(first_of[b], nb, dg, bytes_of[b]);
    if (r != SF_OK) return r;
    if (blocks_hash) sf_host_sha1_update(&bh, dg, nb * 20);
    return SF_OK;
  };
  uint64_t total = 0;
  bool eof = false;
  for (uint64_t k = 0; !eof && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    if (busy[b] && (rc = harvest(b)) != SF_OK) break;  // stage k-2 (stage k-1 is later in file order)
    uint8_t* dst = static_cast<uint8_t*>(pin[b]);
    uint64_t n = 0;
    if ((rc = fill(dst, total, stage, &n, &eof)) != SF_OK || n == 0) break;
    const uint64_t nb = ceil_div(n, bs);
    bytes_of[b] = n;
    first_of[b] = total / bs;  // every earlier stage was whole blocks
    total += n;
    if (hipMemcpyAsync(ddata[b], dst, n, hipMemcpyHostToDevice, st[b]) != hipSuccess) { rc = SF_ENODEV; break; }
    if ((rc = launch_fixed(ddata[b], n, bs, nb, ddig[b], st[b])) != SF_OK) break;
    if (hipMemcpyAsync(pdig[b], ddig[b], nb * 20, hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
        hipEventRecord(done[b], st[b]) != hipSuccess) { rc = SF_ENODEV; break; }
    busy[b] = true;
  }
  // the (at most two) stages still in flight, in file order
  int order[2] = {0, 1};
  if (busy[0] && busy[1] && first_of[1] < first_of[0]) std::swap(order[0], order[1]);
  for (int b : order)
    if (busy[b]) {
      const int r = harvest(b);
      if (rc == SF_OK) rc = r;
    }
  if (rc == SF_OK && blocks_hash) sf_host_sha1_final(&bh, blocks_hash);
  return rc;
}

// Rows in a growing malloc'd buffer (sf_index_fd; the sequential route of
// sf_index_file).
struct RowBuf {
  sf_block_sig* p = nullptr;
  uint64_t n = 0, cap = 0;
  ~RowBuf() { free(p); }
  bool grow(uint64_t need) {
    if (need <= cap) return true;
    uint64_t c = std::max<uint64_t>({need, 2 * cap, 1024});
    void* q = realloc(p, c * sizeof(sf_block_sig));
    if (!q) return false;
    p = static_cast<sf_block_sig*>(q);
    cap = c;
    return true;
  }
  sf_block_sig* release() {
    sf_block_sig* q = p;
    p = nullptr;
    n = cap = 0;
    return q;
  }
};

inline void write_rows(sf_block_sig* o, uint64_t first, uint64_t nb, const uint8_t* dg, uint64_t bytes, uint32_t bs) {
  for (uint64_t i = 0; i < nb; i++) {
    o[i].offset = (first + i) * bs;
    o[i].size = (uint32_t)std::min<uint64_t>(bs, bytes - i * bs);
    memcpy(o[i].sha1, dg + 20 * i, 20);
  }
}

// Sequential route (input that cannot seek: a pipe, FIFO, socket or
// character device -- what index_file's File::open + read accepts,
// src/index.rs:615,625): read() to EOF.
static int index_stream(int fd, uint32_t bs, RowBuf& rows, uint8_t* blocks_hash) {
  auto fill = [&](uint8_t* dst, uint64_t, uint64_t cap, uint64_t* n, bool* eof) {
    *n = 0;
    while (*n < cap) {
      const ssize_t r = read(fd, dst + *n, cap - *n);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) return SF_EIO;
      if (r == 0) { *eof = true; break; }
      *n += (uint64_t)r;
    }
    return SF_OK;
  };
  auto emit = [&](uint64_t first, uint64_t nb, const uint8_t* dg, uint64_t bytes) {
    if (!rows.grow(rows.n + nb)) return SF_ENOMEM;
    write_rows(rows.p + rows.n, first, nb, dg, bytes, bs);
    rows.n += nb;
    return SF_OK;
  };
  return staged_pipeline(bs, file_stage_bytes(bs), fill, emit, blocks_hash);
}

// Regular file of known length: each stage is read by several threads in
// parallel (one pread stream per slice; one thread copies from the page
// cache at ~16 GB/s, below PCIe).  A short read (the file shrank) is SF_EIO.
// Read-ahead (SF_FADVISE, default on): the file is declared sequential and,
// before stage k is read, the kernel is asked to start fetching stage k+1
// (POSIX_FADV_WILLNEED), so a file that is not in the page cache streams from
// the disk while stage k is copied; for a resident file both are no-ops.
inline bool fadvise_on() {
  const char* e = getenv("SF_FADVISE");
  return !e || atoi(e) != 0;
}

// Bytes [base, base + len) of the file (base a multiple of bs: a shard of
// one logical file); row offsets are file offsets.
static int index_file_pread(int fd, uint64_t base, uint64_t len, uint32_t bs, sf_block_sig* out,
                            uint8_t* blocks_hash) {
  const unsigned nthreads = std::max(1u, std::min(io_threads(), std::thread::hardware_concurrency()));
  const bool adv = fadvise_on();
  if (adv) (void)posix_fadvise(fd, (off_t)base, (off_t)len, POSIX_FADV_SEQUENTIAL);
  auto fill = [&](uint8_t* dst, uint64_t off, uint64_t cap, uint64_t* nout, bool* eof) {
    const uint64_t n = std::min(cap, len - off);
    *nout = n;
    *eof = off + n >= len;
    if (adv && !*eof)
      (void)posix_fadvise(fd, (off_t)(base + off + n), (off_t)std::min(cap, len - off - n), POSIX_FADV_WILLNEED);
    auto read_slice = [&](uint64_t a, uint64_t b) {
      for (uint64_t got = a; got < b;) {
        const ssize_t r = pread(fd, dst + got, b - got, (off_t)(base + off + got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return SF_EIO;
        got += (uint64_t)r;
      }
      return SF_OK;
    };
    const uint64_t slice = std::max<uint64_t>(4ull << 20, ceil_div(n, nthreads));
    std::vector<std::thread> pool;
    std::vector<int> rcs(nthreads, SF_OK);
    for (unsigned t = 1; t < nthreads && t * slice < n; t++)
      pool.emplace_back([&, t] { rcs[t] = read_slice(t * slice, std::min(n, (t + 1) * slice)); });
    rcs[0] = read_slice(0, std::min(n, slice));
    for (auto& th : pool) th.join();
    for (int r : rcs)
      if (r) return r;
    return SF_OK;
  };
  auto emit = [&](uint64_t first, uint64_t nb, const uint8_t* dg, uint64_t bytes) {
    write_rows(out + first, base / bs + first, nb, dg, bytes, bs);
    return SF_OK;
  };
  return staged_pipeline(bs, file_stage_bytes(bs), fill, emit, blocks_hash);
}

}  // namespace

extern "C" {

int sf_index_buffer(const uint8_t* data, uint64_t len, uint32_t block_size, sf_block_sig* out, uint64_t cap,
                    uint64_t* n_out) {
  int rc = check_fixed_args(len, block_size);
  if (rc) return rc;
  if (len && (!data || !out)) return SF_EINVAL;
  // Large buffers: page-lock in place (no staging memcpy); SF_NO_HOSTREG=1
  // forces the staged path (A/B knob).
  const char* noreg = getenv("SF_NO_HOSTREG");
  if (len && len >= inplace_min_bytes(false) && !(noreg && atoi(noreg))) {
    rc = index_inplace(data, len, block_size, out, cap, n_out, nullptr);
    if (rc != SF_ENOTSUP) return rc;
  }
  return index_pipelined(len, block_size, out, cap, n_out, [&](uint8_t* dst, uint64_t off, uint64_t n) {
    memcpy(dst, data + off, n);
    return SF_OK;
  });
}

int sf_index_file(const char* path, uint32_t block_size, sf_block_sig* out, uint64_t cap, uint64_t* n_out,
                  uint8_t blocks_hash[20]) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (!path) return SF_EINVAL;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return SF_EIO;
  struct stat sb;
  if (fstat(fd, &sb) != 0 || S_ISDIR(sb.st_mode)) { close(fd); return SF_EIO; }
  if (!S_ISREG(sb.st_mode)) {
    // Not seekable (FIFO, socket, character device): the sequential route.
    // The input is consumed, so with too small a cap the rows are lost and
    // SF_ENOSPC reports the need (sf_index_fd has no cap to miss).
    RowBuf rows;
    uint8_t bh[20];
    rc = index_stream(fd, block_size, rows, bh);
    close(fd);
    if (rc != SF_OK) return rc;
    if (n_out) *n_out = rows.n;
    if (rows.n > cap) return SF_ENOSPC;
    if (rows.n && !out) return SF_EINVAL;
    if (rows.n) memcpy(out, rows.p, rows.n * sizeof(sf_block_sig));
    if (blocks_hash) memcpy(blocks_hash, bh, 20);
    return SF_OK;
  }
  const off_t end = lseek(fd, 0, SEEK_END);
  if (end < 0) { close(fd); return SF_EIO; }
  const uint64_t len = (uint64_t)end;
  const uint64_t nb = len ? ceil_div(len, block_size) : 0;
  if (n_out) *n_out = nb;
  if (nb > cap) { close(fd); return SF_ENOSPC; }
  if (nb && !out) { close(fd); return SF_EINVAL; }
  // Opt-in (SF_FILE_INPLACE=1): a large file already in the page cache is
  // mapped and the mapping page-locked in place (hipHostRegister), so the DMA
  // engine reads the page-cache pages directly -- no pread copy (the in-place
  // path of sf_index_buffer).  Not the default: a registered file mapping is
  // a GPU userptr, and a concurrent truncation of the file invalidates it
  // under the in-flight copies -- measured on MI355X, the process's queues
  // then never resume and the call hangs (tests/test_gpu_robustness.py).  The
  // default pread pipeline only ever reads the file, so a file that shrinks
  // mid-call gives SF_EIO, like the short read the reference would see.
  const char* inpl = getenv("SF_FILE_INPLACE");
  if (len && len >= inplace_min_bytes(true) && inpl && atoi(inpl)) {
    void* m = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd, 0);
    if (m != MAP_FAILED) {
      const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
      std::vector<unsigned char> res(ceil_div(len, pg));
      uint64_t resident = 0;
      if (mincore(m, len, res.data()) == 0)
        for (unsigned char r : res) resident += r & 1u;
      if (resident * 10 >= res.size() * 9) {
        rc = index_inplace(static_cast<const uint8_t*>(m), len, block_size, out, cap, n_out, blocks_hash, fd);
        if (rc != SF_ENOTSUP) {
          munmap(m, len);
          close(fd);
          return rc;
        }
      }
      munmap(m, len);
    }
  }
  if (nb == 0) {
    close(fd);
    static const uint8_t none = 0;
    if (blocks_hash) sf_host_sha1_impl(&none, 0, blocks_hash, 0);
    return SF_OK;
  }
  rc = index_file_pread(fd, 0, len, block_size, out, blocks_hash);
  close(fd);
  return rc;
}

int sf_index_file_range(const char* path, uint64_t start, uint64_t len, uint32_t block_size, sf_block_sig* out,
                        uint64_t cap, uint64_t* n_out) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (!path || (len && start % block_size)) return SF_EINVAL;  // an empty shard may start anywhere up to EOF
  const uint64_t nb = len ? ceil_div(len, block_size) : 0;
  if (n_out) *n_out = nb;
  if (nb > cap) return SF_ENOSPC;
  if (nb && !out) return SF_EINVAL;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return SF_EIO;
  struct stat sb;
  if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) { close(fd); return SF_EIO; }
  if (start > (uint64_t)sb.st_size || len > (uint64_t)sb.st_size - start) { close(fd); return SF_ERANGE; }
  rc = nb ? index_file_pread(fd, start, len, block_size, out, nullptr) : SF_OK;
  close(fd);
  return rc;
}

int sf_index_fd(int fd, uint32_t block_size, sf_block_sig** rows, uint64_t* n_out, uint8_t blocks_hash[20]) {
  if (rows) *rows = nullptr;
  if (n_out) *n_out = 0;
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (fd < 0 || !rows || !n_out) return SF_EINVAL;
  RowBuf rb;
  rc = index_stream(fd, block_size, rb, blocks_hash);
  if (rc != SF_OK) return rc;
  *n_out = rb.n;
  *rows = rb.release();
  return SF_OK;
}

void sf_free_rows(sf_block_sig* rows) { free(rows); }

// ---- sf_index_files: many files, one pipeline ----------------------------

namespace {

struct FileStage {
  std::vector<uint32_t> files;    // file indices, in order
  std::vector<sf_file_desc> desc;  // where each file sits in the stage buffer
  uint64_t bytes = 0;              // stage buffer bytes (16-B aligned slots)
  uint64_t rows = 0;
};

// Page-cache-resident large files of a stage, mapped and page-locked in place
// so their bytes go to the device by DMA straight from the page cache (no
// pread copy into the pinned stage).  Released once the stage's copies are
// done (its event has completed, or the streams are synchronised).
struct StageMaps {
  std::vector<std::pair<void*, uint64_t>> m;
  void release() {
    for (auto& x : m) {
      (void)hipHostUnregister(x.first);
      munmap(x.first, x.second);
    }
    m.clear();
  }
  ~StageMaps() { release(); }
};

// Files of a stage that are DMA'd from their page-locked mappings instead of
// being read (opt-in; like SF_FILE_INPLACE, a file truncated while its
// registered mapping is being copied hangs the queues, so it is off unless
// asked for).
// being read into the pinned stage: none by default.  With the per-device
// cache, the 8-thread pread stage beats per-file registration at every size
// measured (scripts/map_min_probe.py: 16 MiB files 40 vs 23 GB/s, 64 MiB 46
// vs 33, 128 MiB 45 vs 34).  SF_MAP_MIN_MIB=n maps files >= n MiB (A/B knob).
// Files larger than a stage still take sf_index_file's in-place route.
inline uint64_t map_min_bytes() {
  const char* e = getenv("SF_MAP_MIN_MIB");
  const long v = e ? atol(e) : -1;
  return v >= 0 ? (uint64_t)v << 20 : ~0ull;
}

// mapped[k] = the k-th file of the stage is mapped + registered (at ptrs[k]).
void map_stage(const char* const* paths, const FileStage& st, const std::vector<uint64_t>& size, StageMaps& maps,
               std::vector<const uint8_t*>& ptrs) {
  ptrs.assign(st.files.size(), nullptr);
  const uint64_t map_min = map_min_bytes();
  const char* nomm = getenv("SF_NO_MMAP");
  if (nomm && atoi(nomm)) return;
  const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
  std::vector<unsigned char> res;
  for (size_t k = 0; k < st.files.size(); k++) {
    const uint64_t n = size[st.files[k]];
    if (n < map_min) continue;
    const int fd = open(paths[st.files[k]], O_RDONLY);
    if (fd < 0) continue;  // the pread route reports the error
    struct stat sb;
    void* m = (fstat(fd, &sb) == 0 && (uint64_t)sb.st_size == n) ? mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0)
                                                                  : MAP_FAILED;
    close(fd);
    if (m == MAP_FAILED) continue;
    res.resize(ceil_div(n, pg));
    uint64_t resident = 0;
    if (mincore(m, n, res.data()) == 0)
      for (unsigned char r : res) resident += r & 1u;
    if (resident * 10 >= res.size() * 9 && hipHostRegister(m, n, hipHostRegisterReadOnly) == hipSuccess) {
      maps.m.push_back({m, n});
      ptrs[k] = static_cast<const uint8_t*>(m);
    } else {
      (void)hipGetLastError();
      munmap(m, n);
    }
  }
}

// Fill `dst` with the stage's files: (file, <=16 MiB slice) work items taken
// by up to 8 threads from an atomic counter.
int read_stage(const char* const* paths, const FileStage& st, const std::vector<uint64_t>& size, uint8_t* dst,
               std::atomic<int64_t>& bad, const std::vector<const uint8_t*>& mapped) {
  constexpr uint64_t kSlice = 16ull << 20;
  struct Item { uint32_t k; uint64_t a, b; };
  std::vector<Item> items;
  for (uint32_t k = 0; k < st.files.size(); k++) {
    if (mapped[k]) continue;  // goes to the device straight from its mapping
    const uint64_t n = size[st.files[k]];
    for (uint64_t a = 0; a < n; a += kSlice) items.push_back({k, a, std::min(n, a + kSlice)});
  }
  std::atomic<size_t> next{0};
  std::atomic<int> rc{SF_OK};
  auto worker = [&] {
    for (size_t i; (i = next.fetch_add(1)) < items.size() && rc.load() == SF_OK;) {
      const Item& it = items[i];
      const uint32_t f = st.files[it.k];
      const int fd = open(paths[f], O_RDONLY);
      bool ok = fd >= 0;
      uint8_t* d = dst + st.desc[it.k].offset;
      for (uint64_t got = it.a; ok && got < it.b;) {
        const ssize_t r = pread(fd, d + got, it.b - got, (off_t)got);
        if (r <= 0) ok = false;  // error, or EOF before the size stat() gave
        else got += (uint64_t)r;
      }
      if (fd >= 0) close(fd);
      if (!ok) {
        int64_t want = -1;
        bad.compare_exchange_strong(want, (int64_t)f);
        rc.store(SF_EIO);
      }
    }
  };
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned nthreads = (unsigned)std::min<size_t>(std::min(io_threads(), hw), std::max<size_t>(1, items.size()));
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < nthreads; t++) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  return rc.load();
}

}  // namespace

int sf_index_files(const char* const* paths, uint32_t n_files, uint32_t block_size, uint64_t stage_bytes_hint,
                   sf_block_sig* out, uint64_t cap, uint64_t* first_row, uint8_t* blocks_hashes, uint64_t* n_out,
                   uint32_t* bad_file) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (n_files && (!paths || !first_row || !blocks_hashes)) return SF_EINVAL;
  const uint32_t bs = block_size;
  auto fail = [&](uint32_t f, int code) {
    if (bad_file) *bad_file = f;
    return code;
  };
  // 1. Sizes and the row plan (ENOSPC before any file is read).  The stat
  // calls run on the reader threads, 1024 files per work item: one stat is
  // a few us, so a walk of tens of thousands of small files paid ~1/3 of its
  // time here on one thread.  The first failing file (lowest index) is
  // reported, as the sequential loop did.
  std::vector<uint64_t> size(n_files);
  std::vector<int> st_rc(n_files, SF_OK);
  {
    constexpr uint32_t kStatChunk = 1024;
    const uint32_t nchunks = (uint32_t)ceil_div(n_files, kStatChunk);
    std::atomic<uint32_t> next{0};
    auto worker = [&] {
      for (uint32_t c; (c = next.fetch_add(1)) < nchunks;) {
        const uint32_t f1 = std::min<uint32_t>(n_files, (c + 1) * kStatChunk);
        for (uint32_t f = c * kStatChunk; f < f1; f++) {
          struct stat sb;
          if (!paths[f]) st_rc[f] = SF_EINVAL;
          else if (stat(paths[f], &sb) != 0 || !S_ISREG(sb.st_mode)) st_rc[f] = SF_EIO;
          else size[f] = (uint64_t)sb.st_size;
        }
      }
    };
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned nthreads = (unsigned)std::min<uint64_t>(std::min(io_threads(), hw), nchunks);
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < nthreads; t++) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
  }
  uint64_t total = 0;
  for (uint32_t f = 0; f < n_files; f++) {
    if (st_rc[f] != SF_OK) return fail(f, st_rc[f]);
    first_row[f] = total;
    total += size[f] ? ceil_div(size[f], bs) : 0;
  }
  if (n_files) first_row[n_files] = total;
  if (n_out) *n_out = total;
  if (total > cap) return SF_ENOSPC;
  if (total && !out) return SF_EINVAL;
  if (n_files == 0) return SF_OK;

  // 2. Stages: consecutive files packed at 16-B aligned offsets (the LDS
  // path) up to the stage size; larger files go through sf_index_file.
  const uint64_t stage = stage_bytes_hint ? ((stage_bytes_hint + 15) & ~15ull) : (256ull << 20);
  std::vector<FileStage> stages;
  std::vector<uint32_t> big;
  for (uint32_t f = 0; f < n_files; f++) {
    const uint64_t slot = (size[f] + 15) & ~15ull;
    if (size[f] > stage) {
      big.push_back(f);
      continue;
    }
    if (stages.empty() || stages.back().bytes + slot > stage) stages.emplace_back();
    FileStage& st = stages.back();
    st.files.push_back(f);
    st.desc.push_back({st.bytes, size[f]});
    st.bytes += slot;
    st.rows += size[f] ? ceil_div(size[f], bs) : 0;
  }
  for (uint32_t f : big) {
    const uint64_t want = first_row[f + 1] - first_row[f];
    uint64_t got = 0;
    rc = sf_index_file(paths[f], bs, out + first_row[f], want, &got, blocks_hashes + 20ull * f);
    if (rc == SF_ENOSPC || (rc == SF_OK && got != want)) return fail(f, SF_EIO);  // changed meanwhile
    if (rc) return rc == SF_EIO ? fail(f, rc) : rc;
  }
  if (stages.empty()) return SF_OK;

  // 3. Pipeline: read stage k (host threads) while stage k-1 copies and
  // hashes on its own stream; harvest a stage's rows when its buffer is
  // reused or at the end.
  uint64_t max_bytes = 16, max_rows = 1, max_files = 1;
  for (const FileStage& st : stages) {
    max_bytes = std::max(max_bytes, st.bytes);
    max_rows = std::max(max_rows, st.rows);
    max_files = std::max<uint64_t>(max_files, st.files.size());
  }
  HostLease res;
  hipStream_t* streams;
  hipEvent_t* done;
  rc = res.streams(streams, done);
  struct Buf {
    void* p;
  } ddata[2], ddig[2], dfh[2], pin[2], pdig[2], pfh[2], dstat, pstat;
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, max_bytes, &ddata[i].p);
    if (rc == SF_OK) rc = res.dev(3 + i, max_rows * 20, &ddig[i].p);
    if (rc == SF_OK) rc = res.dev(5 + i, max_files * 20, &dfh[i].p);
    if (rc == SF_OK) rc = res.pin(i, std::min<uint64_t>(max_bytes, stage), &pin[i].p);
    if (rc == SF_OK) rc = res.pin(3 + i, max_rows * 20, &pdig[i].p);
    if (rc == SF_OK) rc = res.pin(5 + i, max_files * 20, &pfh[i].p);
  }
  if (rc == SF_OK) rc = res.dev(7, 2 * 16, &dstat.p);  // one int32 status per stage buffer, 16 B apart
  if (rc == SF_OK) rc = res.pin(7, 2 * 16, &pstat.p);
  if (rc != SF_OK) return rc;
  auto stat_dev = [&](int b) { return reinterpret_cast<int*>(static_cast<uint8_t*>(dstat.p) + 16 * b); };
  auto stat_host = [&](int b) { return *reinterpret_cast<volatile int*>(static_cast<uint8_t*>(pstat.p) + 16 * b); };
  // Per stage: each file's blocks_hash from a device chain (one lane per
  // file, in the batch launch) while the runs are short; on the host (SHA-NI
  // over the digests, in harvest) once the longest run would keep a lone
  // chain lane busy past the stage's copy.  A chain costs ~1.1 us per 64 B of
  // digests: 128 MiB files (640 KiB runs) took 11.6 ms per 256 MiB stage,
  // against 4.7 ms of PCIe (scripts/map_min_probe.py).
  constexpr uint64_t kDevChainMaxRun = 192u << 10;
  std::vector<char> dev_bh(stages.size(), 1);
  for (size_t k = 0; k < stages.size(); k++)
    for (uint32_t f : stages[k].files)
      if ((first_row[f + 1] - first_row[f]) * 20 > kDevChainMaxRun) dev_bh[k] = 0;
  auto harvest = [&](size_t k) {  // SF_OK, or the stage's device status (SF_ETIMEDOUT)
    const FileStage& st = stages[k];
    const int b = (int)(k & 1);
    if (dev_bh[k] && stat_host(b) != SF_OK) return stat_host(b);
    const uint8_t* dg = static_cast<const uint8_t*>(pdig[b].p);
    const uint8_t* fh = static_cast<const uint8_t*>(pfh[b].p);
    uint64_t r = 0;
    for (size_t j = 0; j < st.files.size(); j++) {
      const uint32_t f = st.files[j];
      sf_block_sig* o = out + first_row[f];
      const uint64_t nb = first_row[f + 1] - first_row[f];
      for (uint64_t i = 0; i < nb; i++, r++) {
        o[i].offset = i * bs;
        o[i].size = (uint32_t)std::min<uint64_t>(bs, size[f] - i * bs);
        memcpy(o[i].sha1, dg + 20 * r, 20);
      }
      if (dev_bh[k]) memcpy(blocks_hashes + 20ull * f, fh + 20 * j, 20);
      else sf_host_sha1_impl(dg + 20 * (r - nb), nb * 20, blocks_hashes + 20ull * f, 0);
    }
    return SF_OK;
  };
  std::atomic<int64_t> bad{-1};
  StageMaps maps[2];
  std::vector<const uint8_t*> mptr;
  for (size_t k = 0; k < stages.size() && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    const FileStage& st = stages[k];
    if (k >= 2) {
      if (hipEventSynchronize(done[b]) != hipSuccess) { rc = SF_ENODEV; break; }
      if ((rc = harvest(k - 2)) != SF_OK) break;
    }
    maps[b].release();  // stage k-2's copies are done (its event was waited for above)
    map_stage(paths, st, size, maps[b], mptr);
    rc = read_stage(paths, st, size, static_cast<uint8_t*>(pin[b].p), bad, mptr);
    if (rc) break;
    hipStream_t s = streams[b];
    // H2D: each mapped file from its mapping, every run of consecutive
    // pread files from the pinned stage in one copy.
    uint8_t* dd = static_cast<uint8_t*>(ddata[b].p);
    const uint8_t* pp = static_cast<const uint8_t*>(pin[b].p);
    for (size_t j = 0; j < st.files.size() && rc == SF_OK;) {
      const uint64_t o = st.desc[j].offset;
      if (mptr[j]) {
        if (st.desc[j].len && hipMemcpyAsync(dd + o, mptr[j], st.desc[j].len, hipMemcpyHostToDevice, s) != hipSuccess)
          rc = SF_ENODEV;
        j++;
        continue;
      }
      size_t e = j;
      while (e < st.files.size() && !mptr[e]) e++;
      const uint64_t end = e < st.files.size() ? st.desc[e].offset : st.bytes;
      if (end > o && hipMemcpyAsync(dd + o, pp + o, end - o, hipMemcpyHostToDevice, s) != hipSuccess) rc = SF_ENODEV;
      j = e;
    }
    if (rc) break;
    uint64_t nb = 0;
    if (dev_bh[k] && hipMemsetAsync(stat_dev(b), 0, sizeof(int), s) != hipSuccess) { rc = SF_ENODEV; break; }
    rc = sf_index_device_batch(ddata[b].p, st.bytes, st.desc.data(), (uint32_t)st.files.size(), bs, ddig[b].p,
                               max_rows, dev_bh[k] ? dfh[b].p : nullptr, nullptr, &nb,
                               dev_bh[k] ? stat_dev(b) : nullptr, s);
    if (rc) break;
    if ((nb && hipMemcpyAsync(pdig[b].p, ddig[b].p, nb * 20, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (dev_bh[k] && hipMemcpyAsync(pfh[b].p, dfh[b].p, st.files.size() * 20, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (dev_bh[k] && hipMemcpyAsync(static_cast<uint8_t*>(pstat.p) + 16 * b, stat_dev(b), sizeof(int),
                                     hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipEventRecord(done[b], s) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
  }
  for (int i = 0; i < 2; i++)
    if (hipStreamSynchronize(streams[i]) != hipSuccess && rc == SF_OK) rc = SF_ENODEV;
  for (int i = 0; i < 2; i++) maps[i].release();  // every copy has completed
  if (rc == SF_OK)
    for (size_t k = stages.size() >= 2 ? stages.size() - 2 : 0; k < stages.size() && rc == SF_OK; k++)
      rc = harvest(k);
  if (rc == SF_EIO && bad.load() >= 0) return fail((uint32_t)bad.load(), rc);
  return rc;
}

int sf_sha1_host(const uint8_t* data, uint64_t len, uint8_t out[20]) {
  if (!out || (len && !data)) return SF_EINVAL;
  sf_host_sha1_impl(data, len, out, 0);
  return SF_OK;
}

int sf_blocks_hash(const uint8_t* digests, uint64_t n, uint8_t out[20]) {
  if (!out || (n && !digests)) return SF_EINVAL;
  sf_host_sha1_impl(digests, n * 20, out, 0);
  return SF_OK;
}

int sf_blocks_hash_sigs(const sf_block_sig* sigs, uint64_t n, uint8_t out[20]) {
  if (!out || (n && !sigs)) return SF_EINVAL;
  // Gather the digests into one contiguous run (AoS rows are 32 B apart).
  std::vector<uint8_t> buf(n * 20);
  for (uint64_t i = 0; i < n; i++) memcpy(buf.data() + 20 * i, sigs[i].sha1, 20);
  sf_host_sha1_impl(buf.data(), n * 20, out, 0);
  return SF_OK;
}

}  // extern "C"

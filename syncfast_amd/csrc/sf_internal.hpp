// sf_internal.hpp -- library-internal declarations shared by the C-ABI's
// translation units (not part of include/syncfast_amd.h):
//   sf_capi.hip   the gfx950 kernels' launchers and the device-resident entry
//                 points (the only TU compiled for the GPU);
//   sf_host.cpp   the host-memory entry points: per-device cache of streams
//                 and staging buffers, the buffer / file / fd / range
//                 pipelines, the wire stream, host SHA-1 helpers;
//   sf_files.cpp  sf_index_files, the many-file pipeline;
//   sf_fds.cpp    sf_index_fds_blocks, the default mode over many files;
//   sf_multi.cpp  one process, N devices;
//   sf_pool.cpp   the host worker threads of every pipeline (run_pool).
// The .cpp files use only the HIP runtime API (no kernels), so they build
// with the host compiler.
#pragma once
#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__ 1
#endif
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <sys/types.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/syncfast_amd.h"

// Internal status of the in-place route (never returned through the C-ABI):
// the caller's pages could not be page-locked, take the staged route.
#define SF_ENOTSUP (-95)

#define SF_HIP(call)                       \
  do {                                     \
    hipError_t _e = (call);                \
    if (_e != hipSuccess) return sfi::hip_err(_e); \
  } while (0)

namespace sfi __attribute__((visibility("hidden"))) {

// Environment knobs, read once when the library is loaded (sf_knobs.cpp);
// the launch and copy paths read these slots, never the environment.
// Order = kKnobDefs[] (names, defaults).
enum Knob {
  K_IO_THREADS, K_INPLACE_MIN_MIB, K_INPLACE_SERIAL, K_FADVISE, K_NO_HOSTREG, K_TABLE_CLASS_BITS, K_TRACE,
  K_BATCH_FUSED,
  K_TEST_INPLACE_FAIL_AT, K_TEST_WIRE_CHUNK, K_TEST_STREAM_STAGE_MIB, K_TEST_LAUNCH_MAX_BLOCKS, K_TEST_TABLE_SORT,
  K_TEST_MULTI_SELF_GATHER, K_TEST_CUT_WINDOW_MIB, K_TEST_STREAM_POOL, K_COUNT
};
struct KnobDef {
  const char* env;
  int64_t dflt;
};
extern const KnobDef kKnobDefs[K_COUNT];
extern std::atomic<int64_t> g_knob[K_COUNT];
inline int64_t knob(Knob k) { return g_knob[k].load(std::memory_order_relaxed); }

// Counters of the routes the host entry points took (read by the tests
// through sf_test_get_stat): pages the library page-locked, and ranges it
// refused to page-lock because they are not private anonymous memory.
enum Stat { S_PAGES_LOCKED, S_NOT_ANON_REFUSED, S_COUNT };
extern std::atomic<int64_t> g_stat[S_COUNT];
inline void stat_add(Stat s, int64_t v = 1) { g_stat[s].fetch_add(v, std::memory_order_relaxed); }

// Test hook (sf_test_set_read_hook, sf_knobs.cpp): the pread routes call it
// after each window of a regular file has been read.
void read_hook(uint64_t window);

// A C++ exception must not cross the extern "C" boundary: a C or Rust caller
// would get std::terminate.  Every entry point that allocates, starts threads
// or takes locks on the host runs its body through guarded(): host allocation
// failure -> SF_ENOMEM, a thread or lock the system refuses (EAGAIN and the
// like) -> SF_ENOMEM, anything else -> SF_EIO.
template <typename F>
inline int guarded(F&& body) noexcept {
  try {
    return body();
  } catch (const std::bad_alloc&) {
    return SF_ENOMEM;
  } catch (const std::system_error&) {
    return SF_ENOMEM;
  } catch (...) {
    return SF_EIO;
  }
}

// Runs `worker` on the calling thread and on up to nthreads-1 of the
// library's kept helper threads (sf_pool.cpp).  The workers share an atomic
// work counter, so helpers busy elsewhere or a thread the system refuses only
// lower the parallelism.  Returns when every helper that started the worker
// has finished it; an exception from any of them is rethrown here.
void run_pool_fn(unsigned nthreads, const std::function<void()>& worker);
template <typename F>
inline void run_pool(unsigned nthreads, F&& worker) {
  if (nthreads <= 1) {
    worker();
    return;
  }
  run_pool_fn(nthreads, std::function<void()>(std::ref(worker)));
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int hip_err(hipError_t e) {
  if (e == hipSuccess) return SF_OK;
  if (e == hipErrorOutOfMemory) return SF_ENOMEM;
  return SF_ENODEV;
}

// hipGetLastError() answers the last failing HIP call of this thread, whatever
// it was, until it is read.  A launcher reads it after its launch, so it first
// clears what an earlier call left there -- one of ours whose status is
// ignored on purpose (hipHostUnregister in cleanup, an attribute probe), or
// the caller's, or another library's on the same thread -- which would
// otherwise be reported as the launch's failure (SF_ENODEV from a good launch).
inline void clear_stale_error() { (void)hipGetLastError(); }

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

inline int check_fixed_args(uint64_t len, uint32_t bs) {
  if (bs == 0 || bs > SF_MAX_BLOCK_SIZE) return SF_EINVAL;
  (void)len;
  return SF_OK;
}

// Launchers of the gfx950 kernels (sf_capi.hip).
int launch_fixed(const void* d_data, uint64_t len, uint32_t bs, uint64_t nblocks, void* d_digests,
                 hipStream_t stream, uint32_t* weak = nullptr);
// Explicit block list (sha1_table_kernel; sorted by length class from 65
// blocks).  d_status may be NULL.
int launch_table(const void* d_data, uint64_t len, const uint64_t* d_offsets, const uint32_t* d_sizes,
                 uint64_t nblocks, void* d_digests, int* d_status, hipStream_t stream, uint32_t* weak = nullptr);
// Stream-ordered scratch (sf_alloc.cpp): allocated, used and freed on one
// stream, from the library's pool of the stream's device, whose blocks are
// reused on the freeing stream only.  stream_alloc returns an SF_ code.
int stream_alloc(void** p, size_t bytes, hipStream_t s);
void stream_free(void* p, hipStream_t s);
int launch_wire(const uint8_t* d_digests, uint64_t n, uint32_t bs, uint32_t last, uint8_t* d_out,
                hipStream_t stream);
// FILE_BLOCK runs of explicit lists (sf_wire.hip): end offsets of every
// message (stream-ordered allocation, hipFreeAsync on s), the end offset of
// every chunk of `per` messages, and messages [first, first + cnt) written
// from the start of d_out (base = end offset of message first - 1).
int wire_plan(const uint32_t* d_sizes, uint64_t n, uint64_t** d_ends, hipStream_t s);
int wire_chunk_ends(const uint64_t* d_ends, uint64_t n, uint64_t per, uint64_t* d_chunk_ends, hipStream_t s);
int wire_build(const uint8_t* d_digests, const uint32_t* d_sizes, const uint64_t* d_ends, uint64_t first,
               uint64_t cnt, uint64_t base, uint8_t* d_out, hipStream_t s);

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
  // stages; 5, 6 = their blocks_hash arrays; 7 = unused.
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

// Defined in sf_host.cpp.
extern std::mutex g_res_mu[kMaxDevices];
extern HostRes* g_res[kMaxDevices];

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
    // Cached buffers grow in steps (powers of two to 16 MiB, then 16 MiB
    // multiples): a stage of packed small files (just under 256 MiB) and then
    // a stage of 8 MiB files (exactly 256 MiB) share one allocation instead of
    // paying a free + reallocation of every stage buffer (~0.13 ms per MiB,
    // pinned and device: scripts/files_trace.py, scripts/pin_alloc_probe.py).
    if (need <= kCacheMax) {
      uint64_t r = need <= (16ull << 20) ? 4096 : need;
      if (need <= (16ull << 20))
        while (r < need) r <<= 1;
      else
        r = (need + (16ull << 20) - 1) & ~((16ull << 20) - 1);
      need = std::min(r, kCacheMax);
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

// fstat(fd) as a stamp (and the file's mode); false if fstat fails.  Two
// stamps match when dev, ino, size and mtime are equal and, unless the link
// count changed, ctime too (include/syncfast_amd.h, sf_file_stamp).
bool stamp_of(int fd, sf_file_stamp* s, mode_t* mode);
bool same_stamp(const sf_file_stamp& a, const sf_file_stamp& b);

// Fixed tiling of bytes [base, base + len) of the regular file open on fd
// (base a multiple of bs) through the staged pread pipeline (sf_host.cpp) on
// the calling thread's current device: rows (file offsets) into out[0, ...),
// blocks_hash (may be NULL) over this range's digests.  A short read is SF_EIO.
int index_file_pread(int fd, uint64_t base, uint64_t len, uint32_t bs, sf_block_sig* out, uint8_t* blocks_hash);

// Reader threads of the pread routes (sf_index_file, sf_index_files).
// SF_IO_THREADS overrides the default of 16 (A/B knob, latched at load).  With the stat phase
// parallel too, 16 readers beat 8 on many small files (10,537 files of
// 0-200 KiB: 29.3 vs 24.1 GB/s, 12 and 24 no better; 8 MiB files flat at
// 33-34 GB/s; profiles/r02/e2e/io_threads_8_12_16_24.log).
inline unsigned io_threads() {
  const int64_t v = knob(K_IO_THREADS);
  return v > 0 ? (unsigned)std::min<int64_t>(v, 64) : 16u;
}

// Processing order of an explicit block list (sf_sort.hip): d_order[0, n)
// receives the block indices sorted by length class (kmax < 1024: one
// counting pass over 256, 512 or 1024 bins), descending, list order within a
// class.  d_ws: class_order_workspace(n, kmax) bytes of device memory.
// Stream-ordered on s.
size_t class_order_workspace(uint64_t n, uint32_t kmax);
int class_order(const uint32_t* d_sizes, uint64_t n, uint32_t mbits, uint32_t kmax, void* d_ws, uint32_t* d_order,
                hipStream_t s);
// sha1_table_kernel<128, weak_form> on `stream` (sf_table.hip, its own
// translation unit), one group of 64 blocks per wave; SF_OK or the launch
// error.
int launch_table_kernel(bool weak_form, const uint8_t* d_data, uint64_t len, const uint64_t* d_offsets,
                        const uint32_t* d_sizes, uint64_t nblocks, uint8_t* d_digests, int* d_status, uint32_t* weak,
                        const uint32_t* order, hipStream_t stream);

}  // namespace sfi

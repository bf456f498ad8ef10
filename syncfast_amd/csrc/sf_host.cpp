// sf_host.cpp -- the C-ABI's host-memory entry points (include/syncfast_amd.h):
// bytes in host memory, in a file or behind a descriptor -> pinned stages ->
// H2D -> the gfx950 kernels (launched through sf_capi.hip) -> D2H of the rows,
// plus the per-device cache of streams and buffers these calls share, the
// streamed FILE_BLOCK run and the host SHA-1 helpers.  HIP runtime API only:
// built with the host compiler.
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>

#include <algorithm>
#include <atomic>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "host_sha1.h"
#include "sf_internal.hpp"

namespace sfi __attribute__((visibility("hidden"))) {
std::mutex g_res_mu[kMaxDevices];
HostRes* g_res[kMaxDevices];
}  // namespace sfi

using namespace sfi;

namespace {

// Host ranges page-locked by this library's in-place routes, process-wide.
// hipHostRegister refuses a range that overlaps a registered one
// (AlreadyRegistered).  If that registration is one of ours, the concurrent
// call that made it will unregister it while our copies may still read it,
// so such a range is bounced through pinned stages instead; a registration
// the caller made stays for the length of the call and is copied from.
enum PageLock { kLockedByUs, kPinnedByCaller, kNotLocked };
std::mutex g_lock_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_locked;

bool locked_by_us(uintptr_t a, uintptr_t e) {  // caller holds g_lock_mu
  for (const auto& r : g_locked)
    if (r.first < e && a < r.second) return true;
  return false;
}

// PROCMAP_QUERY (Linux 6.11+, include/uapi/linux/fs.h): one ioctl on
// /proc/self/maps answers "the first VMA at or after addr with these
// properties".  Declared here: the image's kernel headers predate it.
struct ProcmapQuery {
  uint64_t size, query_flags, query_addr;
  uint64_t vma_start, vma_end, vma_flags, vma_page_size, vma_offset, inode;
  uint32_t dev_major, dev_minor, vma_name_size, build_id_size;
  uint64_t vma_name_addr, build_id_addr;
};
constexpr uint64_t kQueryCoveringOrNext = 0x10, kQueryFileBacked = 0x20;
constexpr unsigned long kProcmapQuery = _IOWR('f', 17, ProcmapQuery);

// Is [a, e) private anonymous memory only (heap, anonymous mmap, stack)?
// The in-place routes page-lock the caller's pages (hipHostRegister makes
// them a GPU userptr).  For a file mapping -- and shared memory, which has a
// file behind it too -- a concurrent truncation invalidates that userptr under
// the copies in flight, and on MI355X the process's queues then never resumed
// (tests/test_gpu_robustness.py).  Such ranges are never
// page-locked: they go through the pinned stages.  The ioctl where the kernel
// has it, else /proc/self/maps parsed.
bool private_anonymous(uintptr_t a, uintptr_t e) {
  const int fd = open("/proc/self/maps", O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  ProcmapQuery q{};
  q.size = sizeof(q);
  q.query_flags = kQueryCoveringOrNext | kQueryFileBacked;
  q.query_addr = a;
  if (ioctl(fd, kProcmapQuery, &q) == 0) {
    close(fd);
    return q.vma_start >= e;  // the first file-backed VMA at or after a starts past the range
  }
  if (errno == ENOENT) {  // no file-backed VMA at or after a
    close(fd);
    return true;
  }
  // Older kernel: scan the text.  A VMA overlapping [a, e) must be anonymous
  // (inode 0, device 00:00) and private ('p').
  std::string txt;
  char buf[1 << 16];
  for (ssize_t r; (r = read(fd, buf, sizeof(buf))) != 0;) {
    if (r < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    txt.append(buf, (size_t)r);
  }
  close(fd);
  bool covered = true;
  for (size_t pos = 0; pos < txt.size();) {
    size_t nl = txt.find('\n', pos);
    if (nl == std::string::npos) nl = txt.size();
    unsigned long lo = 0, hi = 0, off = 0, ino = 0;
    unsigned maj = 0, mnr = 0;
    char perms[8] = {0};
    if (sscanf(txt.c_str() + pos, "%lx-%lx %7s %lx %x:%x %lu", &lo, &hi, perms, &off, &maj, &mnr, &ino) == 7 &&
        lo < e && a < hi && (ino != 0 || maj != 0 || mnr != 0 || perms[3] != 'p'))
      covered = false;
    pos = nl + 1;
  }
  return covered;
}

// Memory the caller page-locked itself (hipHostMalloc, hipHostRegister):
// copied from as it is.
bool pinned_by_hip(uintptr_t a, uintptr_t e) {
  for (uintptr_t p : {a, e - 1}) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, (const void*)p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
  }
  return true;
}

PageLock lock_pages(uintptr_t a, uintptr_t e) {
  std::lock_guard<std::mutex> lk(g_lock_mu);
  if (locked_by_us(a, e)) return kNotLocked;
  if (!private_anonymous(a, e)) {
    if (pinned_by_hip(a, e)) return kPinnedByCaller;
    stat_add(S_NOT_ANON_REFUSED);
    return kNotLocked;
  }
  const hipError_t err = hipHostRegister((void*)a, e - a, hipHostRegisterReadOnly);
  if (err == hipSuccess) {
    g_locked.push_back({a, e});
    stat_add(S_PAGES_LOCKED);
    return kLockedByUs;
  }
  (void)hipGetLastError();
  return err == hipErrorHostMemoryAlreadyRegistered ? kPinnedByCaller : kNotLocked;
}

void unlock_pages(uintptr_t a) {
  std::lock_guard<std::mutex> lk(g_lock_mu);
  (void)hipHostUnregister((void*)a);
  for (size_t i = 0; i < g_locked.size(); i++)
    if (g_locked[i].first == a) {
      g_locked.erase(g_locked.begin() + (long)i);
      break;
    }
}

bool range_locked_by_us(uintptr_t a, uintptr_t e) {
  std::lock_guard<std::mutex> lk(g_lock_mu);
  return locked_by_us(a, e);
}

// RAII pinned allocation (the in-place route's bounce buffer).
struct PinBuf {
  void* p = nullptr;
  ~PinBuf() { if (p) (void)hipHostFree(p); }
};

// Smallest host buffer that sf_index_buffer / sf_index_buffer_blocks copy in
// place (page-locked) instead of staging through the pinned stages.  Per call,
// with the per-device set cached (scripts/inplace_min_probe.py): a buffer
// gains in place from 1 MiB up (7.6 vs 6.1 GB/s; 32 MiB: 45 vs 21).
// SF_INPLACE_MIN_MIB overrides it (A/B knob).
inline uint64_t inplace_min_bytes() {
  const int64_t v = knob(K_INPLACE_MIN_MIB);
  return v >= 0 ? (uint64_t)v << 20 : 1ull << 20;
}

// Chunk of input handled per pipeline stage: a whole number of blocks, about
// 256 MiB.
inline uint64_t stage_bytes(uint32_t bs) {
  const uint64_t target = 256ull << 20;
  const uint64_t nb = std::max<uint64_t>(1, target / bs);
  return nb * bs;
}

// In-place route of sf_index_buffer: the DMA engine reads the caller's pages
// directly, no staging memcpy.  Only private anonymous memory is page-locked
// (lock_pages); a file mapping passed as a buffer takes the staged route.  Per ~256 MiB stage, on alternating streams: H2D, the
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
// same result.  Returns SF_ENOTSUP (nothing done) when the first region cannot
// be registered, so the caller can take its staged route.
// SF_INPLACE_SERIAL=1 registers the whole range first and writes rows and
// blocks_hash after the last stage (the previous form; A/B knob).
int index_inplace(const uint8_t* data, uint64_t len, uint32_t bs, sf_block_sig* out, uint64_t cap,
                  uint64_t* n_out, uint8_t* blocks_hash) {
  const uint64_t nblocks = ceil_div(len, bs);
  if (n_out) *n_out = nblocks;
  if (nblocks > cap) return SF_ENOSPC;
  const bool serial = knob(K_INPLACE_SERIAL) != 0;
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
        if (x.second == kLocked) unlock_pages((uintptr_t)x.first);
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
  // (pages a concurrent call of ours locked are not the caller's pinning)
  const bool prepinned = pinned_at(data) && pinned_at(data + len - 1) && !range_locked_by_us(lo, hi);
  const int64_t fail_k = knob(K_TEST_INPLACE_FAIL_AT);  // test hook: region k "fails" to register
  auto reg = [&](uint64_t k) {
    const uintptr_t a = serial ? lo : edge(k), e = serial ? hi : edge(k + 1);
    // after one failure every later region stays pageable (a stage straddles
    // the page it shares with the previous region)
    if (e <= a) { regs.push_back({(void*)a, kEmpty}); return; }
    if (prepinned) { regs.push_back({(void*)a, kPinned}); return; }
    if ((!regs.empty() && regs.back().second == kPageable) || (int64_t)k == fail_k) {
      regs.push_back({(void*)a, kPageable});
      return;
    }
    const PageLock pl = lock_pages(a, e);
    regs.push_back({(void*)a, pl == kLockedByUs ? kLocked : pl == kPinnedByCaller ? kPinned : kPageable});
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
      memcpy(bounce.p, src, n);
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

}  // namespace

extern "C" {

static int sf_release_host_cache_body(void) {
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

#ifndef SF_WIRE_CHUNK_DEFAULT
#define SF_WIRE_CHUNK_DEFAULT (1ull << 18)
#endif
static constexpr uint64_t kWireChunk = SF_WIRE_CHUNK_DEFAULT;  // messages per chunk (~9.4 MB at 4 KiB blocks)

static int sf_wire_file_blocks_fd_body(const void* d_digests, uint64_t n_blocks, uint32_t block_size, uint64_t file_len, int fd,
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
  const int64_t wc = knob(K_TEST_WIRE_CHUNK);  // messages per chunk (SF_TEST_WIRE_CHUNK test hook)
  const uint64_t per = wc > 0 ? (uint64_t)wc : kWireChunk;
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
    if (launch_wire(static_cast<const uint8_t*>(d_digests) + i0 * 20, n, block_size, lsz,
                    static_cast<uint8_t*>(dout[b]), st[b]) != SF_OK ||
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

// The FILE_BLOCK run of an explicit list streamed to fd: chunks of
// SF_TEST_WIRE_CHUNK messages (default 2^18).  The whole run is planned once
// (message lengths, one scan, every chunk's end offset read back in one copy:
// the only wait before the chunks), then chunk k is built on the device and
// copied back while the host writes chunk k-2 -- no per-chunk host stall.
static int sf_wire_blocks_fd_body(const void* d_digests, const uint32_t* d_sizes, uint64_t n_blocks, int fd,
                                  uint64_t* n_written, void* stream) {
  if (n_written) *n_written = 0;
  if (n_blocks == 0) return SF_OK;
  if (!d_digests || !d_sizes || fd < 0) return SF_EINVAL;
  const int64_t wc = knob(K_TEST_WIRE_CHUNK);  // messages per chunk (SF_TEST_WIRE_CHUNK test hook)
  const uint64_t per = wc > 0 ? (uint64_t)wc : kWireChunk;
  const uint64_t nchunks = ceil_div(n_blocks, per);
  hipStream_t cs = as_stream(stream);  // digests and sizes are produced on the caller's stream
  uint64_t* ends = nullptr;
  int rc = wire_plan(d_sizes, n_blocks, &ends, cs);
  if (rc != SF_OK) return rc;
  struct FreeEnds {
    uint64_t* p;
    hipStream_t s;
    ~FreeEnds() { stream_free(p, s); }
  } free_ends{ends, cs};
  std::vector<uint64_t> cend(nchunks);
  uint64_t* d_cend = nullptr;
  if ((rc = stream_alloc(reinterpret_cast<void**>(&d_cend), nchunks * 8, cs)) != SF_OK) return rc;
  if ((rc = wire_chunk_ends(ends, n_blocks, per, d_cend, cs)) == SF_OK &&
      (hipMemcpyAsync(cend.data(), d_cend, nchunks * 8, hipMemcpyDeviceToHost, cs) != hipSuccess ||
       hipStreamSynchronize(cs) != hipSuccess))
    rc = SF_ENODEV;
  stream_free(d_cend, cs);
  if (rc != SF_OK) return rc;
  uint64_t cap = 1;
  for (uint64_t k = 0; k < nchunks; k++) cap = std::max(cap, cend[k] - (k ? cend[k - 1] : 0));
  HostLease res;
  hipStream_t* st;
  hipEvent_t* ev;
  void *dout[2], *pin[2];
  uint64_t bytes_of[2] = {0, 0};
  rc = res.streams(st, ev);
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, cap, &dout[i]);
    if (rc == SF_OK) rc = res.pin(i, cap, &pin[i]);
  }
  if (rc != SF_OK) return rc;  // (the plan is complete: cs was synchronised above)
  uint64_t written = 0;
  auto flush = [&](int b) {
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
  for (uint64_t k = 0; k < nchunks && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    if (k >= 2 && (rc = flush(b)) != SF_OK) break;
    const uint64_t i0 = k * per, cnt = std::min(per, n_blocks - i0), base = k ? cend[k - 1] : 0;
    bytes_of[b] = cend[k] - base;
    if ((rc = wire_build(static_cast<const uint8_t*>(d_digests), d_sizes, ends, i0, cnt, base,
                         static_cast<uint8_t*>(dout[b]), st[b])) != SF_OK)
      break;
    if (hipMemcpyAsync(pin[b], dout[b], bytes_of[b], hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
        hipEventRecord(ev[b], st[b]) != hipSuccess)
      rc = SF_ENODEV;
  }
  for (uint64_t k = nchunks >= 2 ? nchunks - 2 : 0; k < nchunks && rc == SF_OK; k++) rc = flush((int)(k & 1));
  for (int i = 0; i < 2; i++) (void)hipStreamSynchronize(st[i]);  // before the plan is freed on cs
  if (n_written) *n_written = written;
  return rc;
}

}  // extern "C"

namespace {

// Staged pipeline (sf_index_file's pread route, the sequential route of
// sf_index_fd, sf_index_buffer below its in-place size): two pinned stages of whole blocks (the last one
// short).  `fill(dst, off, cap, &n, &eof)` puts the next input bytes into a
// pinned stage; per stage, on alternating streams, H2D + block kernel + D2H of
// the stage's digests.  While stage k is being filled, stage k-1 is on the
// device and stage k-2's rows are emitted (`emit(first_block, n_blocks,
// digests, stage_bytes)`) and its digests folded into the streaming
// blocks_hash (src/index.rs:661-682), in order.  No device memory maps or
// registers the caller's file: the host only ever reads it with read/pread.
inline uint64_t file_stage_bytes(uint32_t bs) {
  const int64_t sm = knob(K_TEST_STREAM_STAGE_MIB);  // test hook: small stages exercise the pipeline
  const uint64_t want = sm > 0 ? (uint64_t)sm << 20 : (256ull << 20);
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
inline bool fadvise_on() { return knob(K_FADVISE) != 0; }

}  // namespace

namespace sfi {

// Bytes [base, base + len) of the file (base a multiple of bs: a shard of
// one logical file); row offsets are file offsets.
int index_file_pread(int fd, uint64_t base, uint64_t len, uint32_t bs, sf_block_sig* out, uint8_t* blocks_hash) {
  const unsigned nthreads = std::max(1u, std::min(io_threads(), std::thread::hardware_concurrency()));
  const bool adv = fadvise_on();
  if (adv) (void)posix_fadvise(fd, (off_t)base, (off_t)len, POSIX_FADV_SEQUENTIAL);
  uint64_t window = 0;
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
    const uint64_t nslices = ceil_div(n, slice);
    std::atomic<uint64_t> next{0};
    std::atomic<int> rc{SF_OK};
    run_pool((unsigned)std::min<uint64_t>(nthreads, nslices), [&] {
      for (uint64_t i; (i = next.fetch_add(1)) < nslices && rc.load() == SF_OK;) {
        const int r = read_slice(i * slice, std::min(n, (i + 1) * slice));
        if (r != SF_OK) rc.store(r);
      }
    });
    read_hook(window++);
    return rc.load();
  };
  auto emit = [&](uint64_t first, uint64_t nb, const uint8_t* dg, uint64_t bytes) {
    write_rows(out + first, base / bs + first, nb, dg, bytes, bs);
    return SF_OK;
  };
  return staged_pipeline(bs, file_stage_bytes(bs), fill, emit, blocks_hash);
}

}  // namespace sfi

namespace {

// Copy n bytes into a pinned stage with several threads (one thread moves
// ~10-16 GB/s, below the PCIe link the stage is waiting for).
inline void par_memcpy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  const unsigned nthreads = std::max(1u, std::min(io_threads(), std::thread::hardware_concurrency()));
  const uint64_t slice = std::max<uint64_t>(4ull << 20, ceil_div(n, nthreads));
  const uint64_t nslices = ceil_div(n, slice);
  if (nslices <= 1) {
    if (n) memcpy(dst, src, n);
    return;
  }
  std::atomic<uint64_t> next{0};
  run_pool((unsigned)std::min<uint64_t>(nthreads, nslices), [&] {
    for (uint64_t i; (i = next.fetch_add(1)) < nslices;) {
      const uint64_t a = i * slice, b = std::min(n, a + slice);
      memcpy(dst + a, src + a, b - a);
    }
  });
}

// One stage of an explicit block list: blocks [b0, b1), whose bytes all lie
// in the window [w0, w1) of the caller's buffer.
struct ListStage {
  uint64_t b0, b1, w0, w1;
};
constexpr uint64_t kListStageMaxBlocks = 1ull << 22;  // keeps a stage's list and digests (~135 MiB) bounded

// sf_index_buffer_blocks: the list is cut into stages of consecutive blocks
// whose window spans at most ~256 MiB (a larger block is a stage of its own);
// per stage, on alternating streams: the window and the stage's list
// (offsets relative to the window, sizes) are copied into pinned buffers and
// to HBM, sha1_table_kernel hashes the blocks, the digests come back.  While
// stage k is copied in, stage k-1 is on the device and stage k-2's rows are
// written and folded into blocks_hash, in list order.
// `fill(dst, w0, w1)` puts bytes [w0, w1) of the input into the pinned stage.
// `direct` (the buffer form): the caller's bytes, copied to HBM in place --
// page-locked region by region one stage ahead, as index_inplace does -- when
// the stage windows are disjoint and at least two pages each (a chunker's
// list); a region that cannot be page-locked sends it and every later stage
// through `fill`.
template <typename FillFn>
int index_list_pipeline(FillFn fill, const uint64_t* offsets, const uint32_t* sizes, uint64_t n, sf_block_sig* out,
                        uint8_t* blocks_hash, const uint8_t* direct = nullptr) {
  const uint64_t target = file_stage_bytes(1);  // ~256 MiB (SF_TEST_STREAM_STAGE_MIB test hook)
  std::vector<ListStage> stages;
  uint64_t max_win = 0, max_blocks = 0;
  for (uint64_t i = 0; i < n;) {
    ListStage s{i, i + 1, offsets[i], offsets[i] + sizes[i]};
    for (i++; i < n && i - s.b0 < kListStageMaxBlocks; i++) {
      const uint64_t e = std::max(s.w1, offsets[i] + sizes[i]);
      if (e - s.w0 > target) break;
      s.w1 = e;
    }
    s.b1 = i;
    max_win = std::max(max_win, s.w1 - s.w0);
    max_blocks = std::max(max_blocks, s.b1 - s.b0);
    stages.push_back(s);
  }
  // In-place regions: region k = [edge(k), edge(k+1)), edge(k) = the page
  // edge at or above stage k's window start (edge(0) below it), so stage k's
  // bytes lie in region k-1 (its head, up to edge(k)) and region k.
  const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
  const size_t nst = stages.size();
  bool inplace = direct != nullptr;
  if (inplace) {
    inplace = knob(K_NO_HOSTREG) == 0 && stages.back().w1 - stages[0].w0 >= inplace_min_bytes();
    for (size_t k = 0; k < nst && inplace; k++)
      inplace = stages[k].w1 - stages[k].w0 >= 2 * pg && (k == 0 || stages[k - 1].w1 <= stages[k].w0);
  }
  auto edge = [&](size_t k) -> uintptr_t {
    const uintptr_t up = ~(uintptr_t)(pg - 1);
    if (k == 0) return (uintptr_t)(direct + stages[0].w0) & up;
    if (k >= nst) return ((uintptr_t)(direct + stages[nst - 1].w1) + pg - 1) & up;
    return ((uintptr_t)(direct + stages[k].w0) + pg - 1) & up;
  };
  enum { kLocked, kPinned, kFailed };
  std::vector<int> region;  // state of region k
  struct Unreg {  // declared before the lease: the lease's release syncs the streams first
    std::vector<int>* r;
    std::function<uintptr_t(size_t)> e;
    ~Unreg() {
      for (size_t k = 0; k < r->size(); k++)
        if ((*r)[k] == kLocked) unlock_pages(e(k));
    }
  } unreg{&region, edge};
  const int64_t fail_k = knob(K_TEST_INPLACE_FAIL_AT);  // test hook: region k "fails" to page-lock
  auto lock_region = [&](size_t k) {
    if ((!region.empty() && region.back() == kFailed) || (int64_t)k == fail_k) { region.push_back(kFailed); return; }
    const PageLock pl = lock_pages(edge(k), edge(k + 1));
    region.push_back(pl == kLockedByUs ? kLocked : pl == kPinnedByCaller ? kPinned : kFailed);
  };
  if (inplace) lock_region(0);
  HostLease res;
  hipStream_t* st;
  hipEvent_t* done;
  void *ddata[2], *pin[2], *dlist[2], *plist[2], *ddig[2], *pdig[2];
  const uint64_t list_bytes = max_blocks * (sizeof(uint64_t) + sizeof(uint32_t));
  int rc = res.streams(st, done);
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, max_win, &ddata[i]);
    if (rc == SF_OK) rc = res.pin(i, max_win, &pin[i]);
    if (rc == SF_OK) rc = res.dev(3 + i, max_blocks * 20, &ddig[i]);
    if (rc == SF_OK) rc = res.pin(3 + i, max_blocks * 20, &pdig[i]);
    if (rc == SF_OK) rc = res.dev(5 + i, list_bytes, &dlist[i]);
    if (rc == SF_OK) rc = res.pin(5 + i, list_bytes, &plist[i]);
  }
  if (rc != SF_OK) return rc;
  sf_host_sha1_stream bh;
  sf_host_sha1_begin(&bh);
  int64_t stage_of[2] = {-1, -1};  // stage in flight on each buffer set
  auto harvest = [&](int b) {
    if (hipEventSynchronize(done[b]) != hipSuccess) return SF_ENODEV;
    const ListStage& s = stages[(size_t)stage_of[b]];
    stage_of[b] = -1;
    const uint8_t* dg = static_cast<const uint8_t*>(pdig[b]);
    for (uint64_t i = s.b0; i < s.b1; i++) {
      out[i].offset = offsets[i];
      out[i].size = sizes[i];
      memcpy(out[i].sha1, dg + 20 * (i - s.b0), 20);
    }
    if (blocks_hash) sf_host_sha1_update(&bh, dg, (s.b1 - s.b0) * 20);
    return SF_OK;
  };
  for (size_t k = 0; k < stages.size() && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    if (stage_of[b] >= 0 && (rc = harvest(b)) != SF_OK) break;  // stage k-2 (k-1 comes later in list order)
    const ListStage& s = stages[k];
    const uint64_t nb = s.b1 - s.b0, win = s.w1 - s.w0;
    const bool direct_k = inplace && region[k] != kFailed && (k == 0 || region[k - 1] != kFailed);
    if (!direct_k && (rc = fill(static_cast<uint8_t*>(pin[b]), s.w0, s.w1)) != SF_OK) break;
    uint64_t* lo = static_cast<uint64_t*>(plist[b]);
    uint32_t* lz = reinterpret_cast<uint32_t*>(lo + nb);
    for (uint64_t i = 0; i < nb; i++) {
      lo[i] = offsets[s.b0 + i] - s.w0;
      lz[i] = sizes[s.b0 + i];
    }
    const uint64_t* d_off = static_cast<const uint64_t*>(dlist[b]);
    const uint32_t* d_sz = reinterpret_cast<const uint32_t*>(d_off + nb);
    bool copy_ok = true;
    if (direct_k) {  // a copy lies inside ONE registration: the head (region k-1) apart from the rest
      const uint8_t* src = direct + s.w0;
      const uint64_t head = k == 0 ? 0 : std::min<uint64_t>(win, edge(k) - (uintptr_t)src);
      copy_ok = (!head || hipMemcpyAsync(ddata[b], src, head, hipMemcpyHostToDevice, st[b]) == hipSuccess) &&
                (win == head || hipMemcpyAsync(static_cast<uint8_t*>(ddata[b]) + head, src + head, win - head,
                                               hipMemcpyHostToDevice, st[b]) == hipSuccess);
    } else if (win) {
      copy_ok = hipMemcpyAsync(ddata[b], pin[b], win, hipMemcpyHostToDevice, st[b]) == hipSuccess;
    }
    if (!copy_ok || hipMemcpyAsync(dlist[b], plist[b], nb * (sizeof(uint64_t) + sizeof(uint32_t)),
                                   hipMemcpyHostToDevice, st[b]) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
    if (inplace && k + 1 < nst) lock_region(k + 1);  // one region ahead of the copies that read it
    // every block was checked to lie in [0, len), so in its window: no status word
    if ((rc = launch_table(ddata[b], win, d_off, d_sz, nb, ddig[b], nullptr, st[b])) != SF_OK) break;
    if (hipMemcpyAsync(pdig[b], ddig[b], nb * 20, hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
        hipEventRecord(done[b], st[b]) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
    stage_of[b] = (int64_t)k;
  }
  // the (at most two) stages still in flight, in list order
  int order[2] = {0, 1};
  if (stage_of[0] >= 0 && stage_of[1] >= 0 && stage_of[1] < stage_of[0]) std::swap(order[0], order[1]);
  for (int b : order)
    if (stage_of[b] >= 0) {
      const int r = harvest(b);
      if (rc == SF_OK) rc = r;
    }
  if (rc == SF_OK && blocks_hash) sf_host_sha1_final(&bh, blocks_hash);
  return rc;
}

// ------------------------------------------------ one open regular file
// index_file opens the file once and takes its mtime, its boundaries and its
// bytes from that one handle (src/index.rs:615-625).  The descriptor routes
// read the caller's open file with pread and compare its stamp (fstat) when
// the call starts -- against the caller's, taken before its chunker read the
// file -- and after the last window is read: a file changed in between gives
// SF_EAGAIN, never rows that mix one version's boundaries with another's bytes.
}  // namespace

namespace sfi {

bool stamp_of(int fd, sf_file_stamp* s, mode_t* mode) {
  struct stat sb;
  if (fstat(fd, &sb) != 0) return false;
  s->dev = (uint64_t)sb.st_dev;
  s->ino = (uint64_t)sb.st_ino;
  s->size = (uint64_t)sb.st_size;
  s->nlink = (uint64_t)sb.st_nlink;
  s->mtime_sec = (int64_t)sb.st_mtim.tv_sec;
  s->mtime_nsec = (int64_t)sb.st_mtim.tv_nsec;
  s->ctime_sec = (int64_t)sb.st_ctim.tv_sec;
  s->ctime_nsec = (int64_t)sb.st_ctim.tv_nsec;
  if (mode) *mode = sb.st_mode;
  return true;
}

// ctime also moves when a link is added or removed (a rename over the path
// unlinks the open file, whose bytes do not change): it is compared only
// while the link count stays the same (include/syncfast_amd.h).
bool same_stamp(const sf_file_stamp& a, const sf_file_stamp& b) {
  return a.dev == b.dev && a.ino == b.ino && a.size == b.size && a.mtime_sec == b.mtime_sec &&
         a.mtime_nsec == b.mtime_nsec &&
         (a.nlink != b.nlink || (a.ctime_sec == b.ctime_sec && a.ctime_nsec == b.ctime_nsec));
}

}  // namespace sfi

namespace {

// body(stamp, mode) between two stamps of fd.  A read that came up short (the
// file shrank: SF_EIO) or a complete one over a file whose stamp moved is
// SF_EAGAIN; other results (argument errors, SF_ENOSPC, device errors) pass.
template <typename Body>
int stamped(int fd, const sf_file_stamp* expect, Body body) {
  sf_file_stamp before{}, after{};
  mode_t mode = 0;
  if (!stamp_of(fd, &before, &mode)) return SF_EIO;
  if (expect && !same_stamp(before, *expect)) return SF_EAGAIN;
  const int rc = body(before, mode);
  if (rc != SF_OK && rc != SF_EIO) return rc;
  if (!stamp_of(fd, &after, nullptr)) return SF_EIO;
  return same_stamp(before, after) ? rc : SF_EAGAIN;
}

// Bytes [w0, w0 + m) of fd into dst: pread slices on the reader threads.  A
// short read (the file shrank after the list was made) is SF_EIO.
int pread_window(int fd, uint8_t* dst, uint64_t w0, uint64_t m) {
  const unsigned nthreads = std::max(1u, std::min(io_threads(), std::thread::hardware_concurrency()));
  const uint64_t slice = std::max<uint64_t>(4ull << 20, ceil_div(m, nthreads));
  const uint64_t nslices = ceil_div(m, slice);
  std::atomic<uint64_t> next{0};
  std::atomic<int> frc{SF_OK};
  run_pool((unsigned)std::min<uint64_t>(nthreads, std::max<uint64_t>(nslices, 1)), [&] {
    for (uint64_t k; (k = next.fetch_add(1)) < nslices && frc.load() == SF_OK;) {
      const uint64_t a = k * slice, e = std::min(m, a + slice);
      for (uint64_t got = a; got < e;) {
        const ssize_t r = pread(fd, dst + got, e - got, (off_t)(w0 + got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          frc.store(SF_EIO);
          break;
        }
        got += (uint64_t)r;
      }
    }
  });
  return frc.load();
}

void empty_blocks_hash(uint8_t* blocks_hash) {  // compute_blocks_hash of no blocks: SHA-1("")
  if (!blocks_hash) return;
  sf_host_sha1_stream bh;
  sf_host_sha1_begin(&bh);
  sf_host_sha1_final(&bh, blocks_hash);
}

// An explicit list over the regular file open on fd, len bytes long: checked
// against len, then windows pread into the pinned stages of the list pipeline.
int index_fd_list(int fd, uint64_t len, const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                  sf_block_sig* out, uint8_t* blocks_hash) {
  for (uint64_t i = 0; i < n; i++) {
    if (offsets[i] > len || sizes[i] > len - offsets[i]) return SF_ERANGE;
    if (i && offsets[i] < offsets[i - 1]) return SF_EINVAL;
  }
  if (n == 0) {
    empty_blocks_hash(blocks_hash);
    return SF_OK;
  }
  uint64_t window = 0;
  auto fill = [&](uint8_t* dst, uint64_t w0, uint64_t w1) {
    const int r = pread_window(fd, dst, w0, w1 - w0);
    read_hook(window++);
    return r;
  };
  return index_list_pipeline(fill, offsets, sizes, n, out, blocks_hash);
}

}  // namespace

extern "C" {

static int sf_index_buffer_blocks_body(const uint8_t* data, uint64_t len, const uint64_t* offsets,
                                       const uint32_t* sizes, uint64_t n, sf_block_sig* out, uint8_t* blocks_hash) {
  if (n && (!offsets || !sizes || !out)) return SF_EINVAL;
  if (len && !data) return SF_EINVAL;
  // The whole list is checked before any byte moves (the device form zeroes
  // an out-of-range block's digest instead; a host caller gets the error).
  for (uint64_t i = 0; i < n; i++) {
    if (offsets[i] > len || sizes[i] > len - offsets[i]) return SF_ERANGE;
    if (i && offsets[i] < offsets[i - 1]) return SF_EINVAL;
  }
  if (n == 0) {
    if (blocks_hash) {  // compute_blocks_hash of no blocks: SHA-1 of the empty string
      sf_host_sha1_stream bh;
      sf_host_sha1_begin(&bh);
      sf_host_sha1_final(&bh, blocks_hash);
    }
    return SF_OK;
  }
  auto fill = [&](uint8_t* dst, uint64_t w0, uint64_t w1) {
    par_memcpy(dst, data + w0, w1 - w0);
    return SF_OK;
  };
  return index_list_pipeline(fill, offsets, sizes, n, out, blocks_hash, data);
}

static int sf_index_file_blocks_body(const char* path, const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                                     sf_block_sig* out, uint8_t* blocks_hash) {
  if (!path || (n && (!offsets || !sizes || !out))) return SF_EINVAL;
  struct Fd {  // closed on every return, and if an exception unwinds to guarded()
    int fd;
    ~Fd() { if (fd >= 0) close(fd); }
  } f{open(path, O_RDONLY | O_NONBLOCK)};  // a FIFO is refused below, not waited on
  const int fd = f.fd;
  if (fd < 0) return SF_EIO;
  return stamped(fd, nullptr, [&](const sf_file_stamp& st, mode_t mode) {
    if (!S_ISREG(mode)) return SF_EIO;  // the list names file offsets: a seekable file
    return index_fd_list(fd, st.size, offsets, sizes, n, out, blocks_hash);
  });
}

static int sf_index_fd_blocks_body(int fd, const sf_file_stamp* expect, const uint64_t* offsets,
                                   const uint32_t* sizes, uint64_t n, sf_block_sig* out, uint8_t* blocks_hash) {
  if (fd < 0 || (n && (!offsets || !sizes || !out))) return SF_EINVAL;
  return stamped(fd, expect, [&](const sf_file_stamp& st, mode_t mode) {
    if (!S_ISREG(mode)) return SF_EINVAL;  // a pipe cannot be read twice: sf_index_buffer_blocks
    return index_fd_list(fd, st.size, offsets, sizes, n, out, blocks_hash);
  });
}

static int sf_index_fd_fixed_body(int fd, const sf_file_stamp* expect, uint32_t block_size, sf_block_sig* out,
                                  uint64_t cap, uint64_t* n_out, uint8_t* blocks_hash) {
  if (n_out) *n_out = 0;
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (fd < 0) return SF_EINVAL;
  return stamped(fd, expect, [&](const sf_file_stamp& st, mode_t mode) {
    if (!S_ISREG(mode)) return SF_EINVAL;  // a stream: sf_index_fd
    const uint64_t nb = st.size ? ceil_div(st.size, block_size) : 0;
    if (n_out) *n_out = nb;
    if (nb > cap) return SF_ENOSPC;
    if (nb && !out) return SF_EINVAL;
    if (nb == 0) {
      empty_blocks_hash(blocks_hash);
      return SF_OK;
    }
    return index_file_pread(fd, 0, st.size, block_size, out, blocks_hash);
  });
}

int sf_file_stamp_fd(int fd, sf_file_stamp* out) {
  if (fd < 0 || !out) return SF_EINVAL;
  return stamp_of(fd, out, nullptr) ? SF_OK : SF_EIO;
}

static int sf_index_buffer_body(const uint8_t* data, uint64_t len, uint32_t block_size, sf_block_sig* out, uint64_t cap,
                    uint64_t* n_out) {
  int rc = check_fixed_args(len, block_size);
  if (rc) return rc;
  if (len && (!data || !out)) return SF_EINVAL;
  // Large buffers of private anonymous memory: page-locked in place (no
  // staging memcpy); SF_NO_HOSTREG=1 forces the staged path (A/B knob).
  if (len && len >= inplace_min_bytes() && knob(K_NO_HOSTREG) == 0) {
    rc = index_inplace(data, len, block_size, out, cap, n_out, nullptr);
    if (rc != SF_ENOTSUP) return rc;
  }
  // Staged: memcpy into the pinned stages, the file route's pipeline.
  const uint64_t nb = len ? ceil_div(len, block_size) : 0;
  if (n_out) *n_out = nb;
  if (nb > cap) return SF_ENOSPC;
  if (nb == 0) return SF_OK;
  auto fill = [&](uint8_t* dst, uint64_t off, uint64_t scap, uint64_t* n, bool* eof) {
    *n = std::min(scap, len - off);
    *eof = off + *n >= len;
    memcpy(dst, data + off, *n);
    return SF_OK;
  };
  auto emit = [&](uint64_t first, uint64_t nbk, const uint8_t* dg, uint64_t bytes) {
    write_rows(out + first, first, nbk, dg, bytes, block_size);
    return SF_OK;
  };
  return staged_pipeline(block_size, std::min(file_stage_bytes(block_size), nb * block_size), fill, emit, nullptr);
}

static int sf_index_file_body(const char* path, uint32_t block_size, sf_block_sig* out, uint64_t cap, uint64_t* n_out,
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
  // The file is only ever read (pread into the pinned stages), never mapped
  // and page-locked: a registered file mapping is a GPU userptr, and a
  // concurrent truncation of the file invalidates it under the in-flight
  // copies -- measured on MI355X, the process's queues then never resumed
  // (DESIGN.md 6).  A file that shrinks mid-call gives SF_EIO, like the short
  // read the reference would see.
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

static int sf_index_file_range_body(const char* path, uint64_t start, uint64_t len, uint32_t block_size, sf_block_sig* out,
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

static int sf_index_fd_body(int fd, uint32_t block_size, sf_block_sig** rows, uint64_t* n_out, uint8_t blocks_hash[20]) {
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

static int sf_blocks_hash_sigs_body(const sf_block_sig* sigs, uint64_t n, uint8_t out[20]) {
  if (!out || (n && !sigs)) return SF_EINVAL;
  // The digests gathered into contiguous runs (AoS rows are 32 B apart), a
  // fixed buffer at a time, streamed through one SHA-1.
  uint8_t buf[20 * 3276];
  sf_host_sha1_stream h;
  sf_host_sha1_begin(&h);
  for (uint64_t i = 0; i < n;) {
    const uint64_t m = std::min<uint64_t>(n - i, sizeof(buf) / 20);
    for (uint64_t j = 0; j < m; j++) memcpy(buf + 20 * j, sigs[i + j].sha1, 20);
    sf_host_sha1_update(&h, buf, m * 20);
    i += m;
  }
  sf_host_sha1_final(&h, out);
  return SF_OK;
}

}  // extern "C"

// C-ABI entry points: the bodies above, exceptions turned into error codes.
extern "C" {

int sf_release_host_cache(void) {
  return guarded([&] { return sf_release_host_cache_body(); });
}

int sf_wire_blocks_fd(const void* d_digests, const uint32_t* d_sizes, uint64_t n_blocks, int fd, uint64_t* n_written,
                      void* stream) {
  return guarded([&] { return sf_wire_blocks_fd_body(d_digests, d_sizes, n_blocks, fd, n_written, stream); });
}

int sf_wire_file_blocks_fd(const void* d_digests, uint64_t n_blocks, uint32_t block_size, uint64_t file_len, int fd,
                           uint64_t* n_written, void* stream) {
  return guarded([&] { return sf_wire_file_blocks_fd_body(d_digests, n_blocks, block_size, file_len, fd, n_written, stream); });
}

int sf_index_buffer(const uint8_t* data, uint64_t len, uint32_t block_size, sf_block_sig* out, uint64_t cap,
                    uint64_t* n_out) {
  return guarded([&] { return sf_index_buffer_body(data, len, block_size, out, cap, n_out); });
}

int sf_index_buffer_blocks(const uint8_t* data, uint64_t len, const uint64_t* offsets, const uint32_t* sizes,
                           uint64_t n_blocks, sf_block_sig* out, uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_buffer_blocks_body(data, len, offsets, sizes, n_blocks, out, blocks_hash); });
}

int sf_index_file_blocks(const char* path, const uint64_t* offsets, const uint32_t* sizes, uint64_t n_blocks,
                         sf_block_sig* out, uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_file_blocks_body(path, offsets, sizes, n_blocks, out, blocks_hash); });
}

int sf_index_fd_blocks(int fd, const sf_file_stamp* expect, const uint64_t* offsets, const uint32_t* sizes,
                       uint64_t n_blocks, sf_block_sig* out, uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_fd_blocks_body(fd, expect, offsets, sizes, n_blocks, out, blocks_hash); });
}

int sf_index_fd_fixed(int fd, const sf_file_stamp* expect, uint32_t block_size, sf_block_sig* out, uint64_t cap,
                      uint64_t* n_out, uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_fd_fixed_body(fd, expect, block_size, out, cap, n_out, blocks_hash); });
}

int sf_index_file(const char* path, uint32_t block_size, sf_block_sig* out, uint64_t cap, uint64_t* n_out,
                  uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_file_body(path, block_size, out, cap, n_out, blocks_hash); });
}

int sf_index_file_range(const char* path, uint64_t start, uint64_t len, uint32_t block_size, sf_block_sig* out,
                        uint64_t cap, uint64_t* n_out) {
  return guarded([&] { return sf_index_file_range_body(path, start, len, block_size, out, cap, n_out); });
}

int sf_index_fd(int fd, uint32_t block_size, sf_block_sig** rows, uint64_t* n_out, uint8_t blocks_hash[20]) {
  return guarded([&] { return sf_index_fd_body(fd, block_size, rows, n_out, blocks_hash); });
}

int sf_blocks_hash_sigs(const sf_block_sig* sigs, uint64_t n, uint8_t out[20]) {
  return guarded([&] { return sf_blocks_hash_sigs_body(sigs, n, out); });
}

}  // extern "C"

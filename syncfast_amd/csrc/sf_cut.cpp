// sf_cut.cpp -- sf_cut_fd (include/syncfast_amd.h): the caller's
// content-defined chunker over one file, on several threads, with exactly the
// boundaries one chunker streaming the file would find.
//
// The reference cuts a file with one cdchunking stream (src/index.rs:622-647);
// in the drop-in's default mode that host loop is the whole cost of indexing
// one large file (the hashing runs on the GPU).  The
// chunker restarts at every boundary (read_block relies on it,
// src/sync/fs.rs:26-40), so the boundaries form a chain in which each one is
// a function of the previous: next(b) = where a fresh chunker started at b
// cuts first.  Cut speculatively from a few starting points, the chains meet
// the true one as soon as one of their boundaries coincides with a true
// boundary, and from there they are the true chain.  So: split the file into
// segments, cut each from its first byte with a fresh chunker (in parallel,
// each running just past its segment's end), then join left to right: the
// true chain is known up to some boundary L past the next segment's start;
// if one of its boundaries beyond that start is also one of the segment's,
// the segment's chain is true from there; otherwise the file is cut again
// from L on one thread until a boundary coincides with one of the segment's
// (or the segment is passed).  The join never trusts a boundary it has not
// matched, so the result is the sequential one for any thread count; the
// parallel part only saves time when the chains meet early, which for a
// chunker whose state is a hash of recent bytes happens within a few chunks.
// sf_index_fd_cut adds the hashing, window by window (up to 512 MiB): each
// thread reads its segment piece by piece into a pinned copy of the window,
// starts each piece's copy to HBM and cuts it while it is in cache; the
// joined list is hashed from HBM (sha1_table_kernel) -- no second read of the
// file.  A window keeps the chunks a boundary closes inside it, and the next
// window starts at the last such boundary.
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <vector>

#include "host_sha1.h"
#include "sf_internal.hpp"

using namespace sfi;

namespace {

constexpr uint64_t kPiece = 1ull << 20;   // bytes read and fed to a chunker at a time
constexpr uint64_t kMinSeg = 4ull << 20;  // a segment is at least this long

struct Chunker {
  const sf_chunker_ops* ops;
  void* ch;
  explicit Chunker(const sf_chunker_ops* o) : ops(o), ch(o->create(o->ctx)) {}
  ~Chunker() {
    if (ch) ops->destroy(ch);
  }
  Chunker(const Chunker&) = delete;
  Chunker& operator=(const Chunker&) = delete;
};

// Bytes [pos, pos + want) of the file: read into `buf` (pread), or a pointer
// into memory that already holds them.  nullptr: a read failed or came short.
using Fetch = std::function<const uint8_t*(uint64_t pos, uint64_t want, uint8_t* buf)>;

const uint8_t* pread_fetch(int fd, uint64_t pos, uint64_t want, uint8_t* buf) {
  for (uint64_t got = 0; got < want;) {
    const ssize_t r = pread(fd, buf + got, want - got, (off_t)(pos + got));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return nullptr;  // an error, or the file shrank below len
    got += (uint64_t)r;
  }
  return buf;
}

// Cuts bytes [start, len) with a fresh chunker (start is a chunk's first
// byte) and calls on_end(end) for each chunk's end until it returns false or
// the bytes run out; when len is the end of the file (eof), a last chunk that
// no boundary closes ends there too.  SF_OK, SF_EIO (a read failed or came
// short), SF_EINVAL (the chunker answered more bytes than it was given),
// SF_ENOMEM.
int cut_from(const Fetch& fetch, uint64_t len, bool eof, const sf_chunker_ops* ops, uint64_t start,
             std::vector<uint8_t>& buf, const std::function<bool(uint64_t)>& on_end) {
  Chunker c(ops);
  if (!c.ch) return SF_ENOMEM;
  uint64_t pos = start, last = start;
  while (pos < len) {
    const uint64_t want = std::min<uint64_t>(kPiece, len - pos);
    const uint8_t* p = fetch(pos, want, buf.data());
    if (!p) return SF_EIO;
    for (uint64_t q = 0; q < want;) {
      const size_t k = ops->next(c.ch, p + q, (size_t)(want - q));
      if (k == 0) break;
      if (k > want - q) return SF_EINVAL;
      q += k;
      last = pos + q;
      if (!on_end(last)) return SF_OK;
    }
    pos += want;
  }
  if (eof && last < len) on_end(len);  // the last chunk ends with the file
  return SF_OK;
}

// Segments of bytes [A, B): k of (B - A) / k bytes, the last one longer by
// the rest (the fused route plans its reads with the same rule).
inline uint64_t seg_count(uint64_t A, uint64_t B, uint32_t threads) {
  return std::max<uint64_t>(1, std::min<uint64_t>(threads ? threads : io_threads(), (B - A) / kMinSeg));
}

// The segments of bytes [A, B) and the join (the file comment); A is a true
// boundary, and B the end of the file if eof.  `fetch` supplies the bytes,
// `seg_begin(i, a, b)` / `seg_end` run on the thread that takes segment i =
// [a, b) before and after it is cut (the fused route claims the segment, then
// starts its copy to HBM once every byte of it has been read).  The true chain's ends in (A, B] go to `ends`; without eof, only
// the ends of chunks that a boundary closes inside [A, B).
using SegHook = std::function<int(uint64_t, uint64_t, uint64_t)>;

int cut_joined(const Fetch& fetch, uint64_t A, uint64_t B, bool eof, const sf_chunker_ops* ops, uint32_t threads,
               const SegHook& seg_begin, std::vector<uint64_t>& ends, const SegHook& seg_end = nullptr) {
  ends.clear();
  if (B <= A) return SF_OK;
  const uint64_t len = B;
  const uint64_t k = seg_count(A, B, threads);
  std::vector<uint64_t> P(k + 1);
  for (uint64_t i = 0; i <= k; i++) P[i] = A + (B - A) / k * i;
  P[k] = B;
  // 1. every segment's speculative chain, up to its first end at or past the
  // next segment's start (segment 0's is true: it starts at byte 0)
  std::vector<std::vector<uint64_t>> C(k);
  std::vector<int> rcs(k, SF_OK);
  std::atomic<uint64_t> next{0};
  run_pool((unsigned)k, [&] {
    std::vector<uint8_t> buf(kPiece);
    for (uint64_t i; (i = next.fetch_add(1)) < k;) {
      if ((rcs[i] = seg_begin(i, P[i], P[i + 1])) != SF_OK) continue;
      const uint64_t stop = P[i + 1];
      std::vector<uint64_t>& out = C[i];
      rcs[i] = cut_from(fetch, len, eof, ops, P[i], buf, [&](uint64_t e) {
        out.push_back(e);
        return e < stop;
      });
      if (rcs[i] == SF_OK && seg_end) rcs[i] = seg_end(i, P[i], P[i + 1]);
    }
  });
  for (int rc : rcs)
    if (rc != SF_OK) return rc;
  // 2. join left to right (the true chain so far ends at L: A before its
  // first end)
  ends = std::move(C[0]);
  std::vector<uint8_t> buf(kPiece);
  auto last_end = [&] { return ends.empty() ? A : ends.back(); };
  for (uint64_t i = 1; i < k && last_end() < len; i++) {
    const std::vector<uint64_t>& Ci = C[i];
    const uint64_t L = last_end();
    auto in_ci = [&](uint64_t e) { return std::binary_search(Ci.begin(), Ci.end(), e); };
    // a true end already known past P[i] that the segment's chain has too
    bool synced = false;
    for (auto it = std::upper_bound(ends.begin(), ends.end(), P[i]); it != ends.end(); ++it)
      if (in_ci(*it)) {
        synced = true;
        break;
      }
    if (synced) {
      ends.insert(ends.end(), std::upper_bound(Ci.begin(), Ci.end(), L), Ci.end());
      continue;
    }
    // otherwise cut again from L until an end is one of the segment's, or
    // the segment's chain is passed
    const uint64_t c_last = Ci.empty() ? P[i + 1] : Ci.back();  // an empty chain: re-cut through its segment
    uint64_t met = 0;
    const int rc = cut_from(fetch, len, eof, ops, L, buf, [&](uint64_t e) {
      ends.push_back(e);
      if (in_ci(e)) {
        met = e;
        return false;
      }
      return e < c_last;
    });
    if (rc != SF_OK) return rc;
    if (met) ends.insert(ends.end(), std::upper_bound(Ci.begin(), Ci.end(), met), Ci.end());
  }
  // the chain may stop short of B when the last segments were joined by
  // re-cutting: finish it
  if (last_end() < len)
    return cut_from(fetch, len, eof, ops, last_end(), buf, [&](uint64_t e) {
      ends.push_back(e);
      return true;
    });
  return SF_OK;
}

}  // namespace

extern "C" {

static int sf_cut_fd_body(int fd, const sf_file_stamp* expect, const sf_chunker_ops* ops, uint32_t threads,
                          uint64_t** offsets, uint32_t** sizes, uint64_t* n_blocks) {
  if (offsets) *offsets = nullptr;
  if (sizes) *sizes = nullptr;
  if (n_blocks) *n_blocks = 0;
  if (fd < 0 || !ops || !ops->create || !ops->next || !ops->destroy || !offsets || !sizes || !n_blocks)
    return SF_EINVAL;
  sf_file_stamp before{}, after{};
  mode_t mode = 0;
  if (!stamp_of(fd, &before, &mode)) return SF_EIO;
  if (!S_ISREG(mode)) return SF_EINVAL;  // segments need offsets: a regular file
  if (expect && !same_stamp(before, *expect)) return SF_EAGAIN;
  const uint64_t len = before.size;
  std::vector<uint64_t> ends;  // the true chain: every chunk's end, in order
  const Fetch fetch = [fd](uint64_t pos, uint64_t want, uint8_t* buf) { return pread_fetch(fd, pos, want, buf); };
  const int rc = cut_joined(fetch, 0, len, true, ops, threads, [](uint64_t, uint64_t, uint64_t) { return SF_OK; }, ends);
  if (rc != SF_OK) {
    if (rc == SF_EIO && stamp_of(fd, &after, nullptr) && !same_stamp(before, after)) return SF_EAGAIN;
    return rc;
  }
  if (!stamp_of(fd, &after, nullptr)) return SF_EIO;
  if (!same_stamp(before, after)) return SF_EAGAIN;  // written while cut: not one version's boundaries
  const uint64_t n = ends.size();
  uint64_t* o = static_cast<uint64_t*>(malloc((n ? n : 1) * sizeof(uint64_t)));
  uint32_t* z = static_cast<uint32_t*>(malloc((n ? n : 1) * sizeof(uint32_t)));
  if (!o || !z) {
    free(o);
    free(z);
    return SF_ENOMEM;
  }
  for (uint64_t j = 0, b = 0; j < n; b = ends[j], j++) {
    if (ends[j] - b > 0xFFFFFFFFull) {  // a chunk of 4 GiB or more: no sf_block_sig size holds it
      free(o);
      free(z);
      return SF_EINVAL;
    }
    o[j] = b;
    z[j] = (uint32_t)(ends[j] - b);
  }
  *offsets = o;
  *sizes = z;
  *n_blocks = n;
  return SF_OK;
}

int sf_cut_fd(int fd, const sf_file_stamp* expect, const sf_chunker_ops* ops, uint32_t threads, uint64_t** offsets,
              uint32_t** sizes, uint64_t* n_blocks) {
  return guarded([&] { return sf_cut_fd_body(fd, expect, ops, threads, offsets, sizes, n_blocks); });
}

void sf_free_cuts(void* p) { free(p); }

// The fused form's window: a pinned copy of up to this many bytes of the file
// (the host cache's largest buffer) and its copy in HBM.
static constexpr uint64_t kFusedMax = 512ull << 20;

static int sf_index_fd_cut_body(int fd, const sf_file_stamp* expect, const sf_chunker_ops* ops, uint32_t threads,
                                sf_block_sig** rows, uint64_t* n_out, uint8_t* blocks_hash) {
  if (rows) *rows = nullptr;
  if (n_out) *n_out = 0;
  if (fd < 0 || !ops || !ops->create || !ops->next || !ops->destroy || !rows || !n_out || !blocks_hash)
    return SF_EINVAL;
  sf_file_stamp before{}, after{};
  mode_t mode = 0;
  if (!stamp_of(fd, &before, &mode)) return SF_EIO;
  if (!S_ISREG(mode)) return SF_EINVAL;
  if (expect && !same_stamp(before, *expect)) return SF_EAGAIN;
  const uint64_t len = before.size;
  const auto ts = std::chrono::steady_clock::now();  // setup (lease, streams, windows): traced apart
  int dev = 0;
  SF_HIP(hipGetDevice(&dev));
  const int64_t wk = knob(K_TEST_CUT_WINDOW_MIB);  // test hook: small windows exercise the window seams
  const uint64_t W = wk > 0 ? (uint64_t)wk << 20 : kFusedMax;
  // held by pointer: released before the two-call fallback below, which
  // takes a lease of its own (a nested lease would try_lock the device's
  // cache mutex this thread already owns)
  auto res = std::make_unique<HostLease>();
  hipStream_t* st;  // st[0]: the window's copies to HBM; st[1]: list upload, kernel, digests back
  hipEvent_t* done_ev;  // done_ev[w & 1]: window w's digests are in host memory
  uint8_t *pin = nullptr, *dwin[2] = {nullptr, nullptr};
  const uint64_t wbytes = std::min(len, W);
  int rc = res->streams(st, done_ev);
  if (rc == SF_OK) rc = res->pin(0, wbytes, reinterpret_cast<void**>(&pin));
  // two device windows: window w + 1 is read and copied while window w's
  // chunks are hashed (its device work overlaps the next window's cutting)
  if (rc == SF_OK) rc = res->dev(0, wbytes, reinterpret_cast<void**>(&dwin[0]));
  if (rc == SF_OK && len > W) rc = res->dev(1, wbytes, reinterpret_cast<void**>(&dwin[1]));
  if (rc != SF_OK) return rc;
  struct Ev {  // window w's copies to HBM are done (the pinned window may be refilled)
    hipEvent_t e = nullptr;
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } copied;
  SF_HIP(hipEventCreateWithFlags(&copied.e, hipEventDisableTiming));
  const bool trace = knob(K_TRACE) != 0;  // SF_TRACE=1: phase times on stderr (probe only)
  const auto t0 = std::chrono::steady_clock::now();
  const double t_setup = std::chrono::duration<double, std::milli>(t0 - ts).count();
  auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  double t_cut = 0, t_dev = 0, t_issue = 0;  // issue: list, buffers and the launch, enqueued
  double t_ph[4] = {0, 0, 0, 0};  // issue's parts (trace): buffers, list upload, launch, digests back
  std::vector<sf_block_sig> rows_v;
  sf_host_sha1_stream bh;
  sf_host_sha1_begin(&bh);
  const uint64_t nseg_max = 4096;
  std::vector<std::atomic<int>> seg_in(nseg_max);
  std::vector<std::atomic<const void*>> seg_owner(nseg_max);  // the thread cutting segment i (its tl_me)
  std::atomic<bool> copy_failed{false};
  for (auto& o : seg_owner) o.store(nullptr, std::memory_order_relaxed);
  std::vector<uint64_t> ends;
  // A window whose chunks are on the device: where it starts, how many, and
  // the pinned list (offsets then sizes) and digests its rows come from.
  struct Pending {
    bool on = false;
    uint64_t A = 0, n = 0;
    const uint8_t* plist = nullptr;
    const uint8_t* pdig = nullptr;
  } pend[2];
  // rows + blocks_hash of window w, in window order, once its digests are back
  auto harvest = [&](uint64_t w) -> int {
    Pending& p = pend[w & 1];
    if (!p.on) return SF_OK;
    const double d0 = ms();
    SF_HIP(hipEventSynchronize(done_ev[w & 1]));
    t_dev += ms() - d0;
    const uint64_t* lo = reinterpret_cast<const uint64_t*>(p.plist);
    const uint32_t* lz = reinterpret_cast<const uint32_t*>(lo + p.n);
    const size_t r0 = rows_v.size();
    rows_v.resize(r0 + p.n);
    for (uint64_t j = 0; j < p.n; j++) {
      rows_v[r0 + j].offset = p.A + lo[j];
      rows_v[r0 + j].size = lz[j];
      memcpy(rows_v[r0 + j].sha1, p.pdig + 20 * j, 20);
    }
    sf_host_sha1_update(&bh, p.pdig, p.n * 20);  // compute_blocks_hash (src/index.rs:661-682), in order
    p.on = false;
    return SF_OK;
  };
  // Window by window: bytes [A, B) read once into the pinned window by the
  // threads that cut them (a segment each, its copy to HBM started at once),
  // cut and joined; the chunks a boundary closes inside the window are hashed
  // from HBM, and the next window starts at the last of those boundaries (the
  // chunk running over B is cut again from there).  Window w's list upload,
  // kernel and digests run on st[1] while window w + 1 is read and cut; its
  // rows are taken after that cut (harvest), so rows stay in file order.
  uint64_t w = 0;
  for (uint64_t A = 0; A < len || (len == 0 && A == 0); w++) {
    const uint64_t B = std::min(len, A + W);
    const bool eof = B == len;
    uint8_t* const dw = dwin[w & 1];
    const uint64_t k = seg_count(A, B, threads);
    if (k > nseg_max) return SF_EINVAL;
    const uint64_t seg_len = std::max<uint64_t>(1, (B - A) / k);
    for (uint64_t i = 0; i < k; i++) seg_in[i].store(0, std::memory_order_relaxed);
    auto seg_of = [&](uint64_t pos) { return std::min<uint64_t>((pos - A) / seg_len, k - 1); };
    auto seg_hi = [&](uint64_t j) { return j + 1 == k ? B : A + (j + 1) * seg_len; };
    // A thread reads the segment it cuts piece by piece into its place in the
    // pinned window, starts the piece's copy to HBM and cuts it while it is in
    // cache; bytes of a segment another thread owns come from pread into a
    // private buffer until that segment is complete, then from the window.
    static thread_local char tl_me;
    const Fetch fetch = [&](uint64_t pos, uint64_t want, uint8_t* buf) -> const uint8_t* {
      const uint64_t j = seg_of(pos);
      bool in = true;
      for (uint64_t q = j; in && q <= seg_of(pos + want - 1); q++)
        in = seg_in[q].load(std::memory_order_acquire) == 1;
      if (in) return pin + (pos - A);
      if (seg_owner[j].load(std::memory_order_relaxed) != &tl_me) return pread_fetch(fd, pos, want, buf);
      const uint64_t own = std::min(want, seg_hi(j) - pos);  // this thread's segment: into the window
      const uint8_t* p = own == want ? pread_fetch(fd, pos, want, pin + (pos - A))
                                     : pread_fetch(fd, pos, want, buf);  // a piece across the segment's end
      if (!p) return nullptr;
      if (own != want) memcpy(pin + (pos - A), p, own);
      // the piece's copy to HBM starts now, while the chunker cuts it
      if (hipMemcpyAsync(dw + (pos - A), pin + (pos - A), own, hipMemcpyHostToDevice, st[0]) != hipSuccess) {
        (void)hipGetLastError();
        copy_failed.store(true, std::memory_order_relaxed);
        return nullptr;
      }
      return p;
    };
    const auto seg_begin = [&](uint64_t i, uint64_t a, uint64_t b) -> int {
      if (i >= k || a != A + i * seg_len || b != seg_hi(i)) return SF_EINVAL;  // the plan must be cut_joined's
      if (hipSetDevice(dev) != hipSuccess) {  // this thread enqueues the segment's copies
        (void)hipGetLastError();
        return SF_ENODEV;
      }
      seg_owner[i].store(&tl_me, std::memory_order_relaxed);
      return SF_OK;
    };
    const auto seg_end = [&](uint64_t i, uint64_t, uint64_t) -> int {  // every byte of segment i is in
      seg_owner[i].store(nullptr, std::memory_order_relaxed);
      seg_in[i].store(1, std::memory_order_release);
      return SF_OK;
    };
    const double c0 = ms();
    rc = len ? cut_joined(fetch, A, B, eof, ops, threads, seg_begin, ends, seg_end) : SF_OK;
    if (copy_failed.load(std::memory_order_relaxed)) rc = SF_ENODEV;
    t_cut += ms() - c0;
    if (rc == SF_EIO && stamp_of(fd, &after, nullptr) && !same_stamp(before, after)) rc = SF_EAGAIN;
    if (rc != SF_OK) return rc;
    // the window's copies are queued on st[0]; the pinned window is refilled
    // only once they are done (below, before the next window's cut)
    SF_HIP(hipEventRecord(copied.e, st[0]));
    if (!eof && ends.empty()) {  // no boundary in a whole window (a chunk longer than W): two calls
      SF_HIP(hipStreamSynchronize(st[0]));
      SF_HIP(hipStreamSynchronize(st[1]));
      res.reset();  // the window's buffers and streams go back before sf_index_fd_blocks leases them
      uint64_t *o = nullptr, n = 0;
      uint32_t* z = nullptr;
      if ((rc = sf_cut_fd_body(fd, &before, ops, threads, &o, &z, &n)) != SF_OK) return rc;
      sf_block_sig* out = static_cast<sf_block_sig*>(malloc((n ? n : 1) * sizeof(sf_block_sig)));
      rc = out ? sf_index_fd_blocks(fd, &before, o, z, n, out, blocks_hash) : SF_ENOMEM;
      free(o);
      free(z);
      if (rc != SF_OK) {
        free(out);
        return rc;
      }
      *rows = out;
      *n_out = n;
      return SF_OK;
    }
    // the previous window's rows (its device work ran during this cut)
    if (w > 0 && (rc = harvest(w - 1)) != SF_OK) return rc;
    // hash the window's chunks: one launch over its bytes in HBM, on st[1]
    // after the window's copies
    const uint64_t n = ends.size();
    const double i0 = ms();
    if (n) {
      uint8_t *plist = nullptr, *dlist = nullptr, *pdig = nullptr, *ddig = nullptr;
      const uint64_t lbytes = n * (sizeof(uint64_t) + sizeof(uint32_t));
      const int b = (int)(w & 1);
      if ((rc = res->pin(5 + b, lbytes, reinterpret_cast<void**>(&plist))) != SF_OK ||
          (rc = res->dev(5 + b, lbytes, reinterpret_cast<void**>(&dlist))) != SF_OK ||
          (rc = res->pin(3 + b, n * 20, reinterpret_cast<void**>(&pdig))) != SF_OK ||
          (rc = res->dev(3 + b, n * 20, reinterpret_cast<void**>(&ddig))) != SF_OK)
        return rc;
      const double p1 = ms();
      t_ph[0] += p1 - i0;
      uint64_t* lo = reinterpret_cast<uint64_t*>(plist);
      uint32_t* lz = reinterpret_cast<uint32_t*>(lo + n);
      for (uint64_t j = 0, e = A; j < n; e = ends[j], j++) {
        if (ends[j] - e > 0xFFFFFFFFull) return SF_EINVAL;
        lo[j] = e - A;  // offsets in the window
        lz[j] = (uint32_t)(ends[j] - e);
      }
      SF_HIP(hipStreamWaitEvent(st[1], copied.e, 0));
      SF_HIP(hipMemcpyAsync(dlist, plist, lbytes, hipMemcpyHostToDevice, st[1]));
      const uint64_t* d_off = reinterpret_cast<const uint64_t*>(dlist);
      const double p2 = ms();
      t_ph[1] += p2 - p1;
      if ((rc = launch_table(dw, B - A, d_off, reinterpret_cast<const uint32_t*>(d_off + n), n, ddig, nullptr,
                             st[1])) != SF_OK)
        return rc;
      const double p3 = ms();
      t_ph[2] += p3 - p2;
      SF_HIP(hipMemcpyAsync(pdig, ddig, n * 20, hipMemcpyDeviceToHost, st[1]));
      SF_HIP(hipEventRecord(done_ev[b], st[1]));
      t_ph[3] += ms() - p3;
      pend[b].on = true;
      pend[b].A = A;
      pend[b].n = n;
      pend[b].plist = plist;
      pend[b].pdig = pdig;
    }
    t_issue += ms() - i0;
    if (eof) break;
    A = ends.back();
    // the next window is read into the pinned window: this window's copies
    // out of it must be done (they ran while it was cut; this waits for the tail)
    const double d0 = ms();
    SF_HIP(hipEventSynchronize(copied.e));
    t_dev += ms() - d0;
  }
  const double h0 = ms();
  if ((rc = harvest(w)) != SF_OK) return rc;  // the last window
  const double t_last = ms() - h0;
  if (!stamp_of(fd, &after, nullptr)) return SF_EIO;
  if (!same_stamp(before, after)) return SF_EAGAIN;  // written while read: not one version's rows
  if (trace)
    fprintf(stderr,
            "sf_index_fd_cut trace: %llu B, %zu blocks, %llu windows: setup %.3f, cut+join %.3f, issue %.3f "
            "(buffers %.3f, list %.3f, launch %.3f, back %.3f), waits %.3f (last harvest %.3f), total %.3f ms "
            "(setup not included)\n",
            (unsigned long long)len, rows_v.size(), (unsigned long long)(w + 1), t_setup, t_cut, t_issue, t_ph[0],
            t_ph[1], t_ph[2], t_ph[3], t_dev, t_last, ms());
  sf_block_sig* out = static_cast<sf_block_sig*>(malloc((rows_v.empty() ? 1 : rows_v.size()) * sizeof(sf_block_sig)));
  if (!out) return SF_ENOMEM;
  if (!rows_v.empty()) memcpy(out, rows_v.data(), rows_v.size() * sizeof(sf_block_sig));
  sf_host_sha1_final(&bh, blocks_hash);
  *rows = out;
  *n_out = rows_v.size();
  return SF_OK;
}

int sf_index_fd_cut(int fd, const sf_file_stamp* expect, const sf_chunker_ops* ops, uint32_t threads,
                    sf_block_sig** rows, uint64_t* n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]) {
  return guarded([&] { return sf_index_fd_cut_body(fd, expect, ops, threads, rows, n_out, blocks_hash); });
}

}  // extern "C"

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
// Host only: no HIP call.
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <vector>

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

// Cuts the file from `start` (a chunk's first byte) with a fresh chunker and
// calls on_end(end) for each chunk's end (the end of the file included, for a
// last chunk that no boundary closes) until it returns false or the file
// ends.  SF_OK, SF_EIO (a read failed or came short of len), SF_EINVAL (the
// chunker answered more bytes than it was given), SF_ENOMEM.
int cut_from(int fd, uint64_t len, const sf_chunker_ops* ops, uint64_t start, std::vector<uint8_t>& buf,
             const std::function<bool(uint64_t)>& on_end) {
  Chunker c(ops);
  if (!c.ch) return SF_ENOMEM;
  uint64_t pos = start, last = start;
  while (pos < len) {
    const uint64_t want = std::min<uint64_t>(kPiece, len - pos);
    uint64_t got = 0;
    while (got < want) {
      const ssize_t r = pread(fd, buf.data() + got, want - got, (off_t)(pos + got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return SF_EIO;  // an error, or the file shrank below len
      got += (uint64_t)r;
    }
    for (uint64_t q = 0; q < want;) {
      const size_t k = ops->next(c.ch, buf.data() + q, (size_t)(want - q));
      if (k == 0) break;
      if (k > want - q) return SF_EINVAL;
      q += k;
      last = pos + q;
      if (!on_end(last)) return SF_OK;
    }
    pos += want;
  }
  if (last < len) on_end(len);  // the last chunk ends with the file
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
  if (len) {
    const uint64_t want = threads ? threads : io_threads();
    const uint64_t k = std::max<uint64_t>(1, std::min<uint64_t>(want, len / kMinSeg));
    std::vector<uint64_t> P(k + 1);
    for (uint64_t i = 0; i <= k; i++) P[i] = len / k * i;
    P[k] = len;
    // 1. every segment's speculative chain, up to its first end at or past
    // the next segment's start (segment 0's is true: it starts at byte 0)
    std::vector<std::vector<uint64_t>> C(k);
    std::vector<int> rcs(k, SF_OK);
    std::atomic<uint64_t> next{0};
    run_pool((unsigned)k, [&] {
      std::vector<uint8_t> buf(kPiece);
      for (uint64_t i; (i = next.fetch_add(1)) < k;) {
        const uint64_t stop = P[i + 1];
        std::vector<uint64_t>& out = C[i];
        rcs[i] = cut_from(fd, len, ops, P[i], buf, [&](uint64_t e) {
          out.push_back(e);
          return e < stop;
        });
      }
    });
    for (int rc : rcs)
      if (rc != SF_OK) {
        if (rc == SF_EIO && stamp_of(fd, &after, nullptr) && !same_stamp(before, after)) return SF_EAGAIN;
        return rc;
      }
    // 2. join left to right
    ends = std::move(C[0]);
    std::vector<uint8_t> buf(kPiece);
    for (uint64_t i = 1; i < k && ends.back() < len; i++) {
      const std::vector<uint64_t>& Ci = C[i];
      const uint64_t L = ends.back();
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
      const uint64_t c_last = Ci.empty() ? 0 : Ci.back();
      uint64_t met = 0;
      const int rc = cut_from(fd, len, ops, L, buf, [&](uint64_t e) {
        ends.push_back(e);
        if (in_ci(e)) {
          met = e;
          return false;
        }
        return e < c_last;
      });
      if (rc != SF_OK) {
        if (rc == SF_EIO && stamp_of(fd, &after, nullptr) && !same_stamp(before, after)) return SF_EAGAIN;
        return rc;
      }
      if (met) ends.insert(ends.end(), std::upper_bound(Ci.begin(), Ci.end(), met), Ci.end());
    }
    // the last segment's chain may stop short of the file's end only if
    // every segment was joined by re-cutting: finish the chain
    if (ends.back() < len) {
      const int rc = cut_from(fd, len, ops, ends.back(), buf, [&](uint64_t e) {
        ends.push_back(e);
        return true;
      });
      if (rc != SF_OK) return rc;
    }
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

}  // extern "C"

// sf_fds.cpp -- sf_index_fds_blocks (include/syncfast_amd.h): the reference's
// default, content-defined mode over many files as ONE pipeline.
//
// The reference's index_path (src/index.rs:685-715) calls index_file
// (src/index.rs:610-659) once per file, and index_file cuts each file with the
// cdchunking crate and hashes every block.  Here the caller's chunker has cut
// every file on its own open descriptor (stamp first, then the chunker, as
// sf_index_fd_blocks expects); this call reads the files again with pread by
// windows packed into pinned stages (a pool of reader threads), and per stage
// does one H2D copy of the bytes and of the stage's block list, one
// length-class sort + one sha1_table_kernel launch over every block of every
// file in it, one D2H of the digests.  Stage k is read while stage k-1 is on
// the device and stage k-2's rows and blocks_hash values are written (host
// threads; each file's blocks_hash is SHA-1 over its digests in list order,
// src/index.rs:661-682).  A file whose stamp moved between the caller's stamp
// and its last window read is SF_EAGAIN for that file alone: its rows are not
// valid, every other file's are.  HIP runtime API only: built with the host
// compiler.
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "host_sha1.h"
#include "sf_internal.hpp"

using namespace sfi;

namespace {

// Blocks of file f, [b0, b1), whose bytes lie in its window [w0, w1); the
// window lands at byte `dst` of its stage buffer, dst = w0 (mod 16), so every
// block keeps its file alignment (16-B aligned waves take the aligned LDS path).
struct Piece {
  uint32_t f;
  uint64_t b0, b1, w0, w1, dst;
  bool first, last;  // the file's first / last piece
  int32_t stream;    // multi-piece files: their blocks_hash stream, else -1
};

struct Stage {
  std::vector<Piece> pieces;
  uint64_t bytes = 0, blocks = 0;
};

// Blocks per stage at most: a stage's list and digests stay ~135 MiB.
constexpr uint64_t kMaxStageBlocks = 1ull << 22;

// SF_TRACE=1: phase times of each call on stderr (probe only).
struct Trace {
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  double check_ms = 0, read_ms = 0, issue_ms = 0, wait_ms = 0, harvest_ms = 0;
  Trace() : on(knob(K_TRACE) != 0) { t0 = last = std::chrono::steady_clock::now(); }
  void lap(double& acc) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    acc += std::chrono::duration<double, std::milli>(now - last).count();
    last = now;
  }
  void report(uint32_t files, uint64_t blocks, size_t stages) {
    if (!on) return;
    const double tot = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr,
            "sf_index_fds_blocks trace: %u files, %llu blocks, %zu stages: check %.2f read %.2f issue %.2f "
            "wait %.2f harvest %.2f total %.2f ms\n",
            files, (unsigned long long)blocks, stages, check_ms, read_ms, issue_ms, wait_ms, harvest_ms, tot);
  }
};

inline unsigned pool_threads(uint64_t items) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  return (unsigned)std::min<uint64_t>(std::min(io_threads(), hw), std::max<uint64_t>(1, items));
}

}  // namespace

extern "C" {

static int sf_index_fds_blocks_body(const int* fds, const sf_file_stamp* stamps, uint32_t n_files,
                                    const uint64_t* const* offsets, const uint32_t* const* sizes,
                                    const uint64_t* n_blocks, uint64_t stage_bytes, sf_block_sig* out, uint64_t cap,
                                    uint64_t* first_row, uint8_t* blocks_hashes, int* file_status,
                                    uint32_t* bad_file) {
  if (n_files && (!fds || !offsets || !sizes || !n_blocks || !first_row || !blocks_hashes)) return SF_EINVAL;
  uint64_t total = 0;
  for (uint32_t f = 0; f < n_files; f++) {
    if (n_blocks[f] && (!offsets[f] || !sizes[f])) return SF_EINVAL;
    first_row[f] = total;
    total += n_blocks[f];
  }
  if (n_files) first_row[n_files] = total;
  if (total > cap) return SF_ENOSPC;
  if (total && !out) return SF_EINVAL;
  if (n_files == 0) return SF_OK;
  Trace tr;

  // 1. Each file's stamp (against the caller's, taken before its chunker
  // read the file) and its list (against the size in that stamp), on the
  // reader threads, 256 files per work item.  A file that fails here is not
  // read; the others go on.
  std::unique_ptr<std::atomic<int>[]> status(new std::atomic<int>[n_files]);
  std::vector<sf_file_stamp> before(n_files);
  {
    constexpr uint32_t kChunk = 256;
    const uint32_t nchunks = (uint32_t)ceil_div(n_files, kChunk);
    std::atomic<uint32_t> next{0};
    run_pool(pool_threads(nchunks), [&] {
      for (uint32_t c; (c = next.fetch_add(1)) < nchunks;) {
        for (uint32_t f = c * kChunk; f < std::min<uint32_t>(n_files, (c + 1) * kChunk); f++) {
          int rc = SF_OK;
          mode_t mode = 0;
          if (fds[f] < 0) rc = SF_EINVAL;
          else if (!stamp_of(fds[f], &before[f], &mode)) rc = SF_EIO;
          else if (!S_ISREG(mode)) rc = SF_EINVAL;  // a pipe cannot be read twice: sf_index_buffer_blocks
          else if (stamps && !same_stamp(before[f], stamps[f])) rc = SF_EAGAIN;
          const uint64_t len = before[f].size;
          for (uint64_t i = 0; rc == SF_OK && i < n_blocks[f]; i++) {
            if (offsets[f][i] > len || sizes[f][i] > len - offsets[f][i]) rc = SF_ERANGE;
            else if (i && offsets[f][i] < offsets[f][i - 1]) rc = SF_EINVAL;
          }
          status[f].store(rc, std::memory_order_relaxed);
        }
      }
    });
  }
  tr.lap(tr.check_ms);

  // 2. Stages: every good file's blocks in windows of at most a stage
  // (consecutive blocks; a larger block is a window of its own), windows
  // packed in file order into stages of about stage_bytes.
  const uint64_t target = stage_bytes ? ((stage_bytes + 15) & ~15ull) : (256ull << 20);
  std::vector<Stage> stages(1);
  int32_t nstreams = 0;
  for (uint32_t f = 0; f < n_files; f++) {
    if (status[f].load(std::memory_order_relaxed) != SF_OK || n_blocks[f] == 0) continue;
    const uint64_t* off = offsets[f];
    const uint32_t* sz = sizes[f];
    const size_t s0 = stages.size();
    uint64_t npieces = 0;
    for (uint64_t i = 0; i < n_blocks[f]; npieces++) {
      Piece p{f, i, i + 1, off[i], off[i] + sz[i], 0, i == 0, false, -1};
      for (i++; i < n_blocks[f] && i - p.b0 < kMaxStageBlocks; i++) {
        const uint64_t e = std::max(p.w1, off[i] + sz[i]);
        if (e - p.w0 > target) break;
        p.w1 = e;
      }
      p.b1 = i;
      p.last = i == n_blocks[f];
      Stage* st = &stages.back();
      const uint64_t nb = p.b1 - p.b0, win = p.w1 - p.w0;
      p.dst = ((st->bytes + 15) & ~15ull) + (p.w0 & 15);
      if (!st->pieces.empty() && (p.dst + win > target || st->blocks + nb > kMaxStageBlocks)) {
        stages.emplace_back();
        st = &stages.back();
        p.dst = p.w0 & 15;
      }
      st->bytes = p.dst + win;
      st->blocks += nb;
      st->pieces.push_back(p);
    }
    if (npieces > 1) {  // the file's blocks_hash is streamed over its pieces
      const int32_t id = nstreams++;
      for (size_t k = s0 - 1; k < stages.size(); k++)
        for (Piece& q : stages[k].pieces)
          if (q.f == f) q.stream = id;
    }
  }
  if (stages.back().pieces.empty()) stages.pop_back();
  std::vector<sf_host_sha1_stream> streams_bh((size_t)nstreams);

  uint64_t max_bytes = 16, max_blocks = 1;
  for (const Stage& st : stages) {
    max_bytes = std::max(max_bytes, st.bytes);
    max_blocks = std::max(max_blocks, st.blocks);
  }
  int rc = SF_OK;
  if (!stages.empty()) {
    HostLease res;
    hipStream_t* st;
    hipEvent_t* done;
    void *ddata[2], *pin[2], *dlist[2], *plist[2], *ddig[2], *pdig[2];
    const uint64_t list_bytes = max_blocks * (sizeof(uint64_t) + sizeof(uint32_t));
    rc = res.streams(st, done);
    for (int i = 0; i < 2 && rc == SF_OK; i++) {
      rc = res.dev(i, max_bytes, &ddata[i]);
      if (rc == SF_OK) rc = res.pin(i, max_bytes, &pin[i]);
      if (rc == SF_OK) rc = res.dev(3 + i, max_blocks * 20, &ddig[i]);
      if (rc == SF_OK) rc = res.pin(3 + i, max_blocks * 20, &pdig[i]);
      if (rc == SF_OK) rc = res.dev(5 + i, list_bytes, &dlist[i]);
      if (rc == SF_OK) rc = res.pin(5 + i, list_bytes, &plist[i]);
    }
    if (rc != SF_OK) return rc;

    // Rows and blocks_hash of the stage on buffer set b: the pieces on the
    // reader threads (rows; one-piece files' blocks_hash in one SHA-1), then
    // the multi-piece files' streams folded in piece order.
    int64_t stage_of[2] = {-1, -1};
    auto harvest = [&](int b) {
      if (hipEventSynchronize(done[b]) != hipSuccess) return SF_ENODEV;
      const Stage& s = stages[(size_t)stage_of[b]];
      stage_of[b] = -1;
      const uint8_t* dg = static_cast<const uint8_t*>(pdig[b]);
      std::vector<uint64_t> row0(s.pieces.size());
      for (size_t j = 0, r = 0; j < s.pieces.size(); j++) {
        row0[j] = r;
        r += s.pieces[j].b1 - s.pieces[j].b0;
      }
      const size_t per = 64;  // pieces per work item
      const size_t nitems = ceil_div(s.pieces.size(), per);
      std::atomic<size_t> next{0};
      run_pool(pool_threads(s.blocks >= 4096 ? nitems : 1), [&] {
        for (size_t it; (it = next.fetch_add(1)) < nitems;) {
          for (size_t j = it * per; j < std::min(s.pieces.size(), (it + 1) * per); j++) {
            const Piece& p = s.pieces[j];
            const uint64_t* off = offsets[p.f];
            const uint32_t* sz = sizes[p.f];
            sf_block_sig* o = out + first_row[p.f];
            const uint8_t* d = dg + 20 * row0[j];
            for (uint64_t i = p.b0; i < p.b1; i++, d += 20) {
              o[i].offset = off[i];
              o[i].size = sz[i];
              memcpy(o[i].sha1, d, 20);
            }
            if (p.stream < 0) sf_host_sha1_impl(dg + 20 * row0[j], (p.b1 - p.b0) * 20, blocks_hashes + 20ull * p.f, 0);
          }
        }
      });
      for (size_t j = 0; j < s.pieces.size(); j++) {
        const Piece& p = s.pieces[j];
        if (p.stream < 0) continue;
        sf_host_sha1_stream& h = streams_bh[(size_t)p.stream];
        if (p.first) sf_host_sha1_begin(&h);
        sf_host_sha1_update(&h, dg + 20 * row0[j], (p.b1 - p.b0) * 20);
        if (p.last) sf_host_sha1_final(&h, blocks_hashes + 20ull * p.f);
      }
      return SF_OK;
    };

    for (size_t k = 0; k < stages.size() && rc == SF_OK; k++) {
      const int b = (int)(k & 1);
      if (stage_of[b] >= 0) {  // stage k-2 (stage k-1 is later in file order)
        tr.lap(tr.issue_ms);
        if (hipEventSynchronize(done[b]) != hipSuccess) { rc = SF_ENODEV; break; }
        tr.lap(tr.wait_ms);
        if ((rc = harvest(b)) != SF_OK) break;
        tr.lap(tr.harvest_ms);
      }
      const Stage& s = stages[k];
      // read: (piece, <= 16 MiB slice) work items; a short read marks the
      // piece's file SF_EIO, the stage goes on
      constexpr uint64_t kSlice = 16ull << 20;
      struct Item { uint32_t j; uint64_t a, e; };
      std::vector<Item> items;
      for (uint32_t j = 0; j < s.pieces.size(); j++) {
        const uint64_t win = s.pieces[j].w1 - s.pieces[j].w0;
        for (uint64_t a = 0; a < win; a += kSlice) items.push_back({j, a, std::min(win, a + kSlice)});
      }
      uint8_t* dst = static_cast<uint8_t*>(pin[b]);
      std::atomic<size_t> next{0};
      run_pool(pool_threads(items.size()), [&] {
        for (size_t i; (i = next.fetch_add(1)) < items.size();) {
          const Item& it = items[i];
          const Piece& p = s.pieces[it.j];
          for (uint64_t got = it.a; got < it.e;) {
            const ssize_t r = pread(fds[p.f], dst + p.dst + got, it.e - got, (off_t)(p.w0 + got));
            if (r < 0 && errno == EINTR) continue;  // a signal (profiler, Python handler) is not a bad file
            if (r <= 0) {  // error, or EOF before the size in the stamp: the file shrank
              int ok = SF_OK;
              status[p.f].compare_exchange_strong(ok, SF_EIO);
              break;
            }
            got += (uint64_t)r;
          }
        }
      });
      read_hook(k);
      // a file whose last window is in: its stamp again (as stamped() does for
      // one file: a short read, or a full one over a file that moved, of a
      // file whose stamp moved is SF_EAGAIN)
      for (const Piece& p : s.pieces) {
        if (!p.last) continue;
        const int cur = status[p.f].load(std::memory_order_relaxed);
        if (cur != SF_OK && cur != SF_EIO) continue;
        sf_file_stamp after{};
        if (!stamp_of(fds[p.f], &after, nullptr)) status[p.f].store(SF_EIO);
        else if (!same_stamp(before[p.f], after)) status[p.f].store(SF_EAGAIN);
      }
      tr.lap(tr.read_ms);
      // the stage's list: offsets in the stage buffer, sizes
      uint64_t* lo = static_cast<uint64_t*>(plist[b]);
      uint32_t* lz = reinterpret_cast<uint32_t*>(lo + s.blocks);
      uint64_t r = 0;
      for (const Piece& p : s.pieces) {
        const uint64_t* off = offsets[p.f];
        const uint32_t* sz = sizes[p.f];
        for (uint64_t i = p.b0; i < p.b1; i++, r++) {
          lo[r] = p.dst + (off[i] - p.w0);
          lz[r] = sz[i];
        }
      }
      const uint64_t* d_off = static_cast<const uint64_t*>(dlist[b]);
      const uint32_t* d_sz = reinterpret_cast<const uint32_t*>(d_off + s.blocks);
      if ((s.bytes && hipMemcpyAsync(ddata[b], pin[b], s.bytes, hipMemcpyHostToDevice, st[b]) != hipSuccess) ||
          hipMemcpyAsync(dlist[b], plist[b], s.blocks * (sizeof(uint64_t) + sizeof(uint32_t)), hipMemcpyHostToDevice,
                         st[b]) != hipSuccess) {
        rc = SF_ENODEV;
        break;
      }
      // every block was checked to lie in its file, so in its window: no status word
      if ((rc = launch_table(ddata[b], s.bytes, d_off, d_sz, s.blocks, ddig[b], nullptr, st[b])) != SF_OK) break;
      if (hipMemcpyAsync(pdig[b], ddig[b], s.blocks * 20, hipMemcpyDeviceToHost, st[b]) != hipSuccess ||
          hipEventRecord(done[b], st[b]) != hipSuccess) {
        rc = SF_ENODEV;
        break;
      }
      stage_of[b] = (int64_t)k;
    }
    tr.lap(tr.issue_ms);
    // the (at most two) stages still in flight, in file order
    int order[2] = {0, 1};
    if (stage_of[0] >= 0 && stage_of[1] >= 0 && stage_of[1] < stage_of[0]) std::swap(order[0], order[1]);
    for (int b : order)
      if (stage_of[b] >= 0) {
        const int r2 = harvest(b);
        if (rc == SF_OK) rc = r2;
      }
    tr.lap(tr.harvest_ms);
  }
  if (rc != SF_OK) return rc;  // a device error: no file's rows are valid

  // Files with no blocks: compute_blocks_hash of nothing, SHA-1("").  A file
  // that failed: its blocks_hash zeroed, its rows not valid.  The call's
  // result is the first failing file's, named by *bad_file.
  int first_bad = -1;
  for (uint32_t f = 0; f < n_files; f++) {
    const int s = status[f].load(std::memory_order_relaxed);
    if (file_status) file_status[f] = s;
    if (s != SF_OK) {
      memset(blocks_hashes + 20ull * f, 0, 20);
      if (first_bad < 0) first_bad = (int)f;
    } else if (n_blocks[f] == 0) {
      sf_host_sha1_impl(reinterpret_cast<const uint8_t*>(""), 0, blocks_hashes + 20ull * f, 0);
    }
  }
  tr.report(n_files, total, stages.size());
  if (first_bad >= 0) {
    if (bad_file) *bad_file = (uint32_t)first_bad;
    return status[first_bad].load();
  }
  return SF_OK;
}

int sf_index_fds_blocks(const int* fds, const sf_file_stamp* stamps, uint32_t n_files, const uint64_t* const* offsets,
                        const uint32_t* const* sizes, const uint64_t* n_blocks, uint64_t stage_bytes,
                        sf_block_sig* out, uint64_t cap, uint64_t* first_row, uint8_t* blocks_hashes, int* file_status,
                        uint32_t* bad_file) {
  return guarded([&] {
    return sf_index_fds_blocks_body(fds, stamps, n_files, offsets, sizes, n_blocks, stage_bytes, out, cap, first_row,
                                    blocks_hashes, file_status, bad_file);
  });
}

}  // extern "C"

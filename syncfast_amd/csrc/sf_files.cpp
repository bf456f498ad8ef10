// sf_files.cpp -- sf_index_files (include/syncfast_amd.h): many files from
// disk through one pipeline, what index_path (src/index.rs:685-715) does with
// one index_file per file.  HIP runtime API only: built with the host compiler.
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "host_sha1.h"
#include "sf_internal.hpp"

using namespace sfi;

namespace {

// SF_TRACE=1: phase times of each sf_index_files call on stderr (probe only).
struct Trace {
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  double stat_ms = 0, big_ms = 0, wait_ms = 0, harvest_ms = 0, read_ms = 0, issue_ms = 0;
  Trace() {
    on = knob(K_TRACE) != 0;
    t0 = last = std::chrono::steady_clock::now();
  }
  void lap(double& acc) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    acc += std::chrono::duration<double, std::milli>(now - last).count();
    last = now;
  }
  void report(uint32_t files, size_t stages) {
    if (!on) return;
    const double tot = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr,
            "sf_index_files trace: %u files, %zu stages: stat %.2f big %.2f read %.2f issue %.2f wait %.2f "
            "harvest %.2f total %.2f ms\n",
            files, stages, stat_ms, big_ms, read_ms, issue_ms, wait_ms, harvest_ms, tot);
  }
};

struct FileStage {
  std::vector<uint32_t> files;    // file indices, in order
  std::vector<sf_file_desc> desc;  // where each file sits in the stage buffer
  uint64_t bytes = 0;              // stage buffer bytes (16-B aligned slots)
  uint64_t rows = 0;
};

// Fill `dst` with the stage's files: (file, <=16 MiB slice) work items taken
// by up to io_threads() threads from an atomic counter.  Files are only read
// (pread), never mapped and page-locked: a truncation under a registered
// mapping hangs the GPU queues.
int read_stage(const char* const* paths, const FileStage& st, const std::vector<uint64_t>& size, uint8_t* dst,
               std::atomic<int64_t>& bad) {
  constexpr uint64_t kSlice = 16ull << 20;
  struct Item { uint32_t k; uint64_t a, b; };
  std::vector<Item> items;
  for (uint32_t k = 0; k < st.files.size(); k++) {
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
        if (r < 0 && errno == EINTR) continue;  // a signal (profiler, Python handler) is not a bad file
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
  run_pool(nthreads, worker);
  return rc.load();
}

}  // namespace

extern "C" {

static int sf_index_files_body(const char* const* paths, uint32_t n_files, uint32_t block_size, uint64_t stage_bytes_hint,
                   sf_block_sig* out, uint64_t cap, uint64_t* first_row, uint8_t* blocks_hashes, uint64_t* n_out,
                   uint32_t* bad_file) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (n_files && (!paths || !first_row || !blocks_hashes)) return SF_EINVAL;
  const uint32_t bs = block_size;
  Trace tr;
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
    run_pool(nthreads, worker);
  }
  tr.lap(tr.stat_ms);
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
  tr.lap(tr.big_ms);
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
  } ddata[2], ddig[2], dfh[2], pin[2], pdig[2], pfh[2];
  for (int i = 0; i < 2 && rc == SF_OK; i++) {
    rc = res.dev(i, max_bytes, &ddata[i].p);
    if (rc == SF_OK) rc = res.dev(3 + i, max_rows * 20, &ddig[i].p);
    if (rc == SF_OK) rc = res.dev(5 + i, max_files * 20, &dfh[i].p);
    if (rc == SF_OK) rc = res.pin(i, std::min<uint64_t>(max_bytes, stage), &pin[i].p);
    if (rc == SF_OK) rc = res.pin(3 + i, max_rows * 20, &pdig[i].p);
    if (rc == SF_OK) rc = res.pin(5 + i, max_files * 20, &pfh[i].p);
  }
  if (rc != SF_OK) return rc;
  // Per stage: each file's blocks_hash from a device chain (one lane per
  // file, after the stage's blocks) while the runs are short; on the host
  // (SHA-NI over the digests, in harvest) once the longest run would keep a
  // lone chain lane busy past the stage's copy.  A chain costs ~1.1 us per
  // 64 B of digests: 128 MiB files (640 KiB runs) took 11.6 ms per 256 MiB
  // stage, against 4.7 ms of PCIe (scripts/map_min_probe.py).
  // The batch call gets no status word, so it takes the path that never
  // waits (block kernel, then chain kernel; sf_index_device_batch): the
  // chains are hidden behind the next stage's copy either way, and the fused
  // launch's bounded wait -- which gave up once in round 5 -- is not on this
  // route at all.
  constexpr uint64_t kDevChainMaxRun = 192u << 10;
  std::vector<char> dev_bh(stages.size(), 1);
  for (size_t k = 0; k < stages.size(); k++)
    for (uint32_t f : stages[k].files)
      if ((first_row[f + 1] - first_row[f]) * 20 > kDevChainMaxRun) dev_bh[k] = 0;
  auto harvest = [&](size_t k) {
    const FileStage& st = stages[k];
    const int b = (int)(k & 1);
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
  for (size_t k = 0; k < stages.size() && rc == SF_OK; k++) {
    const int b = (int)(k & 1);
    const FileStage& st = stages[k];
    tr.lap(tr.issue_ms);
    if (k >= 2) {
      if (hipEventSynchronize(done[b]) != hipSuccess) { rc = SF_ENODEV; break; }
      tr.lap(tr.wait_ms);
      if ((rc = harvest(k - 2)) != SF_OK) break;
      tr.lap(tr.harvest_ms);
    }
    rc = read_stage(paths, st, size, static_cast<uint8_t*>(pin[b].p), bad);
    tr.lap(tr.read_ms);
    if (rc) break;
    hipStream_t s = streams[b];
    // H2D: the whole stage in one copy
    if (st.bytes && hipMemcpyAsync(ddata[b].p, pin[b].p, st.bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
    uint64_t nb = 0;
    rc = sf_index_device_batch(ddata[b].p, st.bytes, st.desc.data(), (uint32_t)st.files.size(), bs, ddig[b].p,
                               max_rows, dev_bh[k] ? dfh[b].p : nullptr, nullptr, &nb, nullptr, s);
    if (rc) break;
    if ((nb && hipMemcpyAsync(pdig[b].p, ddig[b].p, nb * 20, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (dev_bh[k] && hipMemcpyAsync(pfh[b].p, dfh[b].p, st.files.size() * 20, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipEventRecord(done[b], s) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
  }
  tr.lap(tr.issue_ms);
  for (int i = 0; i < 2; i++)
    if (hipStreamSynchronize(streams[i]) != hipSuccess && rc == SF_OK) rc = SF_ENODEV;
  tr.lap(tr.wait_ms);
  if (rc == SF_OK)
    for (size_t k = stages.size() >= 2 ? stages.size() - 2 : 0; k < stages.size() && rc == SF_OK; k++)
      rc = harvest(k);
  tr.lap(tr.harvest_ms);
  tr.report(n_files, stages.size());
  if (rc == SF_EIO && bad.load() >= 0) return fail((uint32_t)bad.load(), rc);
  return rc;
}

}  // extern "C"

// C-ABI entry points: the bodies above, exceptions turned into error codes.
extern "C" {

int sf_index_files(const char* const* paths, uint32_t n_files, uint32_t block_size, uint64_t stage_bytes_hint,
                   sf_block_sig* out, uint64_t cap, uint64_t* first_row, uint8_t* blocks_hashes, uint64_t* n_out,
                   uint32_t* bad_file) {
  return guarded([&] { return sf_index_files_body(paths, n_files, block_size, stage_bytes_hint, out, cap, first_row, blocks_hashes, n_out, bad_file); });
}

}  // extern "C"

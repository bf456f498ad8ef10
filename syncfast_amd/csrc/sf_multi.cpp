// sf_multi.cpp -- one process, N devices (include/syncfast_amd.h):
// sf_shard_range, sf_index_file_multi (one file on disk, its shards read and
// hashed on N GPUs in parallel, rows straight into the caller's table) and
// sf_index_device_multi (device-resident shards hashed on N GPUs, every
// shard's digest table gathered to one device over xGMI with RCCL).
//
// The reference indexes one file on one thread (src/index.rs:610-659).
// Blocks are independent, so a file splits into contiguous block-aligned
// shards, one per device; the only exchange is the one the file's
// blocks_hash needs (src/index.rs:661-682 hashes ALL of a file's digests, in
// order): the shards' tables meet on one device (the device-resident form)
// or in the caller's host array (the file form).
//
// RCCL is loaded on first use (dlopen of librccl.so.1), so a caller that
// never asks for a gather does not pay for loading it; communicators are made
// once per device list with ncclCommInitAll and kept.  HIP runtime API only:
// built with the host compiler.
#include <dlfcn.h>
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "host_sha1.h"
#include "sf_internal.hpp"
#include "../../include/syncfast_amd_test.h"

using namespace sfi;

namespace {

// Blocks dealt as evenly as possible over n shards (the first nblocks % n get
// one more): shard r = bytes [start, start + len), the block-aligned range
// syncfast_amd.shard.shard_range gives rank r of an n-rank group.
void shard_of(uint64_t total, uint32_t bs, uint32_t n, uint32_t r, uint64_t* start, uint64_t* len,
              uint64_t* first_block = nullptr) {
  const uint64_t nblocks = total ? (total + bs - 1) / bs : 0;
  const uint64_t per = nblocks / n, extra = nblocks % n;
  const uint64_t first = (uint64_t)r * per + std::min<uint64_t>(r, extra);
  const uint64_t count = per + (r < extra ? 1 : 0);
  const uint64_t s = std::min(total, first * bs), e = std::min(total, (first + count) * bs);
  *start = s;
  *len = e - s;
  if (first_block) *first_block = first;
}

// ---------------------------------------------------------------- RCCL
struct Rccl {
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  bool ok = false;
};

std::mutex g_rccl_mu;
Rccl g_rccl;
bool g_rccl_tried = false;
// communicators per device list (one ncclCommInitAll each; never destroyed
// from a static destructor: the runtime may be gone at exit)
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

const Rccl* rccl() {  // caller holds g_rccl_mu
  if (!g_rccl_tried) {
    g_rccl_tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      Rccl r;
      r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
      r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
      r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
      r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
      r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
      r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
      r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv;
      if (r.ok) g_rccl = r;
    }
  }
  return g_rccl.ok ? &g_rccl : nullptr;
}

int comms_for(const std::vector<int>& devs, std::vector<ncclComm_t>** out) {  // caller holds g_rccl_mu
  auto it = g_comms.find(devs);
  if (it == g_comms.end()) {
    const Rccl* R = rccl();
    if (!R) return SF_ENODEV;
    std::vector<ncclComm_t> c(devs.size());
    if (R->comm_init_all(c.data(), (int)devs.size(), devs.data()) != ncclSuccess) return SF_ENODEV;
    it = g_comms.emplace(devs, std::move(c)).first;
  }
  *out = &it->second;
  return SF_OK;
}

// Restores the calling thread's current device on every return.
struct DeviceGuard {
  int d = -1;
  DeviceGuard() {
    if (hipGetDevice(&d) != hipSuccess) {
      (void)hipGetLastError();
      d = -1;
    }
  }
  ~DeviceGuard() {
    if (d >= 0) (void)hipSetDevice(d);
  }
};

}  // namespace

extern "C" {

int sf_shard_range(uint64_t file_len, uint32_t block_size, uint32_t n_shards, uint32_t shard, uint64_t* start,
                   uint64_t* len) {
  if (block_size == 0 || n_shards == 0 || shard >= n_shards || !start || !len) return SF_EINVAL;
  shard_of(file_len, block_size, n_shards, shard, start, len);
  return SF_OK;
}

static int sf_index_file_multi_body(const char* path, uint32_t block_size, uint32_t n_devices, sf_block_sig* out,
                                    uint64_t cap, uint64_t* n_out, uint8_t* blocks_hash) {
  if (n_out) *n_out = 0;
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (!path || !blocks_hash) return SF_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) {
    (void)hipGetLastError();
    ndev = 0;
  }
  if (n_devices == 0) n_devices = (uint32_t)ndev;  // every visible device
  if (ndev == 0) return SF_ENODEV;
  if (n_devices > (uint32_t)ndev || n_devices > (uint32_t)kMaxDevices) return SF_EINVAL;
  struct Fd {
    int fd;
    ~Fd() { if (fd >= 0) close(fd); }
  } f{open(path, O_RDONLY | O_NONBLOCK)};
  if (f.fd < 0) return SF_EIO;
  sf_file_stamp before{}, after{};
  mode_t mode = 0;
  if (!stamp_of(f.fd, &before, &mode)) return SF_EIO;
  if (!S_ISREG(mode)) return SF_EINVAL;  // shards need offsets: a regular file (a stream: sf_index_fd)
  const uint64_t len = before.size, nb = len ? ceil_div(len, block_size) : 0;
  if (n_out) *n_out = nb;
  if (nb > cap) return SF_ENOSPC;
  if (nb && !out) return SF_EINVAL;
  // One host thread per device: shard r of the file through the staged pread
  // pipeline on device r (its own PCIe link, its own cached stages), rows
  // straight into out at the shard's first row.
  std::vector<int> rcs(n_devices, SF_OK);
  {
    std::vector<std::thread> th;
    th.reserve(n_devices);
    auto work = [&](uint32_t r) {
      uint64_t start, slen, first;
      shard_of(len, block_size, n_devices, r, &start, &slen, &first);
      if (slen == 0) return;
      if (hipSetDevice((int)r) != hipSuccess) {
        (void)hipGetLastError();
        rcs[r] = SF_ENODEV;
        return;
      }
      rcs[r] = guarded([&] { return index_file_pread(f.fd, start, slen, block_size, out + first, nullptr); });
    };
    try {
      for (uint32_t r = 1; r < n_devices; r++) th.emplace_back(work, r);
    } catch (...) {
      for (auto& t : th) t.join();
      throw;
    }
    {
      DeviceGuard g;  // the calling thread takes shard 0 and gets its device back
      work(0);
    }
    for (auto& t : th) t.join();
  }
  for (int r : rcs)
    if (r != SF_OK && r != SF_EIO) return r;
  if (!stamp_of(f.fd, &after, nullptr)) return SF_EIO;
  if (!same_stamp(before, after)) return SF_EAGAIN;  // written while read: not one version's rows
  for (int r : rcs)
    if (r != SF_OK) return r;
  // blocks_hash over every digest in file order (src/index.rs:661-682)
  sf_host_sha1_stream h;
  sf_host_sha1_begin(&h);
  uint8_t buf[20 * 3276];
  for (uint64_t i = 0; i < nb;) {
    const uint64_t k = std::min<uint64_t>(nb - i, 3276);
    for (uint64_t j = 0; j < k; j++) memcpy(buf + 20 * j, out[i + j].sha1, 20);
    sf_host_sha1_update(&h, buf, 20 * k);
    i += k;
  }
  sf_host_sha1_final(&h, blocks_hash);
  return SF_OK;
}

}  // extern "C"

namespace {

// Where each device's digests go in one sf_index_device_multi call (the
// gather plan, exposed to the tests as sf_test_multi_plan): shard r of the
// file (sf_shard_range) has first_row = its first block and bytes = 20 B per
// block; the root's rows are hashed straight into the table (kInPlace),
// every other non-empty shard's into its device's scratch and received by
// the root at table offset first_row * 20 (kSent); an empty shard takes
// neither (kNone).  With self_gather (one device, test hook) the only shard
// is sent too: a self send/recv through RCCL.  The kInPlace and kSent ranges
// tile [0, nblocks * 20) exactly once.
enum Route { kNone = 0, kInPlace = 1, kSent = 2 };
struct ShardPlan {
  uint64_t start = 0, len = 0, first_row = 0, bytes = 0;
  Route route = kNone;
};

void multi_plan(uint64_t file_len, uint32_t bs, uint32_t n, uint32_t root, bool self_gather, ShardPlan* p) {
  for (uint32_t r = 0; r < n; r++) {
    shard_of(file_len, bs, n, r, &p[r].start, &p[r].len, &p[r].first_row);
    p[r].bytes = p[r].len ? ceil_div(p[r].len, bs) * 20 : 0;
    p[r].route = !p[r].len ? kNone : (r == root && !self_gather) ? kInPlace : kSent;
  }
}

// One event per device, recorded on a hash stream for a gather stream to wait
// on (created on first use, kept; only touched under g_rccl_mu).
hipEvent_t g_multi_ev[kMaxDevices] = {};

}  // namespace

extern "C" {

int sf_test_multi_plan(uint64_t file_len, uint32_t block_size, uint32_t n_devices, uint32_t root, int self_gather,
                       uint64_t* table_offset, uint64_t* bytes, int* route) {
  if (block_size == 0 || n_devices == 0 || n_devices > (uint32_t)kMaxDevices || root >= n_devices || !table_offset ||
      !bytes || !route)
    return SF_EINVAL;
  std::vector<ShardPlan> p(n_devices);
  multi_plan(file_len, block_size, n_devices, root, self_gather != 0 && n_devices == 1, p.data());
  for (uint32_t r = 0; r < n_devices; r++) {
    table_offset[r] = p[r].first_row * 20;
    bytes[r] = p[r].bytes;
    route[r] = (int)p[r].route;
  }
  return SF_OK;
}

static int sf_index_device_multi_body(uint32_t n_devices, const void* const* d_shards, uint64_t file_len,
                                      uint32_t block_size, void* const* d_digests, uint32_t root, void* d_table,
                                      void* const* streams, void* const* gather_streams) {
  int rc = check_fixed_args(0, block_size);
  if (rc) return rc;
  if (n_devices == 0 || n_devices > (uint32_t)kMaxDevices || root >= n_devices || !d_shards || !d_digests ||
      !d_table)
    return SF_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) {
    (void)hipGetLastError();
    ndev = 0;
  }
  if (ndev == 0) return SF_ENODEV;
  if (n_devices > (uint32_t)ndev) return SF_EINVAL;
  // SF_TEST_MULTI_SELF_GATHER (test hook): on one device, the shard goes to
  // d_digests[0] and reaches the table through RCCL (a self send/recv), so a
  // one-GPU box exercises the communicator and the grouped exchange.
  const bool self_gather = n_devices == 1 && knob(K_TEST_MULTI_SELF_GATHER) != 0 && d_digests[0];
  std::vector<ShardPlan> plan(n_devices);
  multi_plan(file_len, block_size, n_devices, root, self_gather, plan.data());
  for (uint32_t r = 0; r < n_devices; r++)
    if (plan[r].route != kNone && (!d_shards[r] || (plan[r].route == kSent && !d_digests[r]))) return SF_EINVAL;
  auto hs = [&](uint32_t r) { return streams ? as_stream(streams[r]) : nullptr; };
  auto gs = [&](uint32_t r) { return gather_streams ? as_stream(gather_streams[r]) : hs(r); };
  const bool exchange = n_devices > 1 || self_gather;
  DeviceGuard g;
  // The whole call under g_rccl_mu when there is an exchange: the per-device
  // events and the communicators are shared by every call.
  std::unique_lock<std::mutex> lk(g_rccl_mu, std::defer_lock);
  if (exchange) lk.lock();
  // 1. every shard hashed on its own device, on its hash stream; the root's
  // straight into its place in the table; then the device's gather stream
  // (when it is another stream) waits for that hashing -- the root's too, so
  // d_table is complete once gather_streams[root] has run past the call
  for (uint32_t r = 0; r < n_devices; r++) {
    if (plan[r].route == kNone) continue;
    SF_HIP(hipSetDevice((int)r));
    uint8_t* dst = plan[r].route == kInPlace ? static_cast<uint8_t*>(d_table) + plan[r].first_row * 20
                                             : static_cast<uint8_t*>(d_digests[r]);
    if ((rc = launch_fixed(d_shards[r], plan[r].len, block_size, plan[r].bytes / 20, dst, hs(r))) != SF_OK) return rc;
    if (exchange && gs(r) != hs(r)) {
      if (!g_multi_ev[r]) SF_HIP(hipEventCreateWithFlags(&g_multi_ev[r], hipEventDisableTiming));
      SF_HIP(hipEventRecord(g_multi_ev[r], hs(r)));
      SF_HIP(hipStreamWaitEvent(gs(r), g_multi_ev[r], 0));
    }
  }
  if (!exchange) return SF_OK;
  // 2. the gather: every other device sends its table to the root, which
  // receives each at its rows (uneven counts: grouped point-to-point, not
  // ncclGather), all in one group, on the gather streams
  std::vector<int> devs(n_devices);
  for (uint32_t r = 0; r < n_devices; r++) devs[r] = (int)r;
  std::vector<ncclComm_t>* comms = nullptr;
  if ((rc = comms_for(devs, &comms)) != SF_OK) return rc;
  const Rccl* R = rccl();
  if (R->group_start() != ncclSuccess) return SF_ENODEV;
  bool ok = true;
  for (uint32_t r = 0; r < n_devices && ok; r++) {
    if (plan[r].route != kSent) continue;
    ok = R->send(d_digests[r], plan[r].bytes, ncclUint8, (int)root, (*comms)[r], gs(r)) == ncclSuccess &&
         R->recv(static_cast<uint8_t*>(d_table) + plan[r].first_row * 20, plan[r].bytes, ncclUint8, (int)r,
                 (*comms)[root], gs(root)) == ncclSuccess;
  }
  if (R->group_end() != ncclSuccess) ok = false;
  return ok ? SF_OK : SF_ENODEV;
}

int sf_index_file_multi(const char* path, uint32_t block_size, uint32_t n_devices, sf_block_sig* out, uint64_t cap,
                        uint64_t* n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]) {
  return guarded([&] { return sf_index_file_multi_body(path, block_size, n_devices, out, cap, n_out, blocks_hash); });
}

int sf_index_device_multi(uint32_t n_devices, const void* const* d_shards, uint64_t file_len, uint32_t block_size,
                          void* const* d_digests, uint32_t root, void* d_table, void* const* streams) {
  return guarded([&] {
    return sf_index_device_multi_body(n_devices, d_shards, file_len, block_size, d_digests, root, d_table, streams,
                                      nullptr);
  });
}

int sf_index_device_multi_ex(uint32_t n_devices, const void* const* d_shards, uint64_t file_len, uint32_t block_size,
                             void* const* d_digests, uint32_t root, void* d_table, void* const* hash_streams,
                             void* const* gather_streams) {
  return guarded([&] {
    return sf_index_device_multi_body(n_devices, d_shards, file_len, block_size, d_digests, root, d_table,
                                      hash_streams, gather_streams);
  });
}

}  // extern "C"

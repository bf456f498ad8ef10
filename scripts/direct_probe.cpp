// Cold-file read rate on the box: a 4 GiB file written, fsync'ed and dropped
// from the page cache (posix_fadvise DONTNEED, no root needed), then read
// by 16 threads in 16 MiB slices into pinned memory, buffered (the pread
// route of sf_index_file today) or with O_DIRECT (no page cache, DMA from
// the device into the pinned stage).  Alternating, 3 rounds; residency is
// checked with mincore before each cold read.
// hipcc -O2 -std=c++17 scripts/direct_probe.cpp -o /tmp/direct_probe -lpthread
#include <hip/hip_runtime_api.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double resident(const char* path, size_t n) {
  const int fd = open(path, O_RDONLY);
  void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
  const size_t pg = 4096, np = (n + pg - 1) / pg;
  std::vector<unsigned char> v(np);
  mincore(m, n, v.data());
  size_t r = 0;
  for (unsigned char c : v) r += c & 1;
  munmap(m, n);
  close(fd);
  return (double)r / np;
}

static void drop(const char* path) {
  const int fd = open(path, O_RDONLY);
  fdatasync(fd);
  posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
  close(fd);
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/sf_direct.bin";
  const size_t n = 4ull << 30, slice = 16u << 20;
  const int threads = 16;
  uint8_t* pin = nullptr;
  if (hipHostMalloc((void**)&pin, n, hipHostMallocDefault) != hipSuccess) return 1;
  {
    const int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    std::vector<uint8_t> buf(slice);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t off = 0; off < n; off += slice) {
      for (size_t i = 0; i < slice; i += 8) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        memcpy(&buf[i], &x, 8);
      }
      if (write(fd, buf.data(), slice) != (ssize_t)slice) return 2;
    }
    fsync(fd);
    close(fd);
  }
  for (int rep = 0; rep < 3; rep++)
    for (int direct = 0; direct < 2; direct++) {
      drop(path);
      const double res = resident(path, n);
      const int fd = open(path, O_RDONLY | (direct ? O_DIRECT : 0));
      if (fd < 0) {
        std::printf("open %s failed\n", direct ? "O_DIRECT" : "buffered");
        continue;
      }
      std::atomic<size_t> next{0};
      std::atomic<int> bad{0};
      const double t0 = now();
      std::vector<std::thread> th;
      for (int t = 0; t < threads; t++)
        th.emplace_back([&] {
          for (size_t k; (k = next.fetch_add(1)) < n / slice;)
            for (size_t got = 0; got < slice;) {
              const ssize_t r = pread(fd, pin + k * slice + got, slice - got, (off_t)(k * slice + got));
              if (r <= 0) { bad++; break; }
              got += (size_t)r;
            }
        });
      for (auto& t : th) t.join();
      const double dt = now() - t0;
      close(fd);
      std::printf("rep %d %-8s resident %.3f  %.3f s  %.2f GB/s  errors %d\n", rep, direct ? "O_DIRECT" : "buffered",
                  res, dt, n / dt / 1e9, bad.load());
      std::fflush(stdout);
    }
  // warm (page cache) buffered read, for scale
  {
    const int fd = open(path, O_RDONLY);
    for (size_t off = 0; off < n; off += slice) (void)pread(fd, pin + off, slice, (off_t)off);
    std::atomic<size_t> next{0};
    const double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
      th.emplace_back([&] {
        for (size_t k; (k = next.fetch_add(1)) < n / slice;) (void)pread(fd, pin + k * slice, slice, (off_t)(k * slice));
      });
    for (auto& t : th) t.join();
    const double dt = now() - t0;
    std::printf("warm     buffered resident %.3f  %.3f s  %.2f GB/s\n", resident(path, n), dt, n / dt / 1e9);
    close(fd);
  }
  unlink(path);
  return 0;
}

// write_probe.cpp -- how fast one ark file can be filled on the box's filesystem (the ark writer of the
// native JOB runner, fdlp_job.cpp): one thread writing 4 MiB pieces, T threads pwrite-ing disjoint
// ranges of the same file, and T threads copying into a shared mapping of it (ftruncate + mmap).
//   g++ -O2 -pthread benchmarks/write_probe.cpp -o /tmp/write_probe && /tmp/write_probe <dir> [MiB]
#include <fcntl.h>
#include <linux/falloc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const size_t mib = argc > 2 ? (size_t)atol(argv[2]) : 1100;
  const size_t n = mib << 20;
  std::vector<char> buf(n);
  for (size_t i = 0; i < n; i += 64) buf[i] = (char)i;
  const std::string path = dir + "/write_probe.bin";
  auto report = [&](const char* what, int th, double t) {
    printf("{\"mode\": \"%s\", \"threads\": %d, \"MiB\": %zu, \"seconds\": %.4f, \"GBps\": %.2f}\n", what, th, mib, t,
           n / t / 1e9);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    {  // one thread, write() in 4 MiB pieces
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
      for (size_t o = 0; o < n; o += 4 << 20) {
        const size_t k = std::min<size_t>(4 << 20, n - o);
        if (write(fd, buf.data() + o, k) != (ssize_t)k) return 1;
      }
      close(fd);
      report("write", 1, now_s() - t0);
    }
    for (size_t piece : {(size_t)1 << 20, (size_t)64 << 20}) {  // one thread, other piece sizes
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
      for (size_t o = 0; o < n; o += piece) {
        const size_t k = std::min(piece, n - o);
        if (write(fd, buf.data() + o, k) != (ssize_t)k) return 1;
      }
      close(fd);
      report(piece == ((size_t)1 << 20) ? "write_1MiB" : "write_64MiB", 1, now_s() - t0);
    }
    {  // fallocate the whole size first, then one thread writes 4 MiB pieces
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
      const int fa = posix_fallocate(fd, 0, (off_t)n);
      for (size_t o = 0; o < n; o += 4 << 20) {
        const size_t k = std::min<size_t>(4 << 20, n - o);
        if (pwrite(fd, buf.data() + o, k, (off_t)o) != (ssize_t)k) return 1;
      }
      close(fd);
      report(fa == 0 ? "fallocate_write" : "fallocate_failed_write", 1, now_s() - t0);
    }
    for (int keep : {1, 0}) {  // fallocate each 21 MiB piece just before writing it (KEEP_SIZE or extending)
      const size_t piece = (size_t)21 << 20;
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
      bool ok = true;
      for (size_t o = 0; o < n; o += piece) {
        const size_t k = std::min(piece, n - o);
        ok = ok && fallocate(fd, keep ? FALLOC_FL_KEEP_SIZE : 0, (off_t)o, (off_t)k) == 0;
        if (write(fd, buf.data() + o, k) != (ssize_t)k) return 1;
      }
      close(fd);
      report(!ok ? "piece_fallocate_failed" : keep ? "piece_fallocate_keep_size" : "piece_fallocate_extend", 1, now_s() - t0);
    }
    for (int th : {2, 4, 8}) {  // T threads, pwrite of disjoint contiguous ranges
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
      std::vector<std::thread> ts;
      for (int t = 0; t < th; ++t)
        ts.emplace_back([&, t] {
          const size_t a = n * t / th, b = n * (t + 1) / th;
          for (size_t o = a; o < b; o += 4 << 20) {
            const size_t k = std::min<size_t>(4 << 20, b - o);
            if (pwrite(fd, buf.data() + o, k, (off_t)o) != (ssize_t)k) abort();
          }
        });
      for (auto& x : ts) x.join();
      close(fd);
      report("pwrite", th, now_s() - t0);
    }
    for (int th : {1, 4, 8}) {  // ftruncate + shared mapping, T threads memcpy
      unlink(path.c_str());
      const double t0 = now_s();
      int fd = open(path.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0644);
      if (ftruncate(fd, (off_t)n) != 0) return 1;
      char* m = (char*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (m == MAP_FAILED) return 1;
      std::vector<std::thread> ts;
      for (int t = 0; t < th; ++t)
        ts.emplace_back([&, t] {
          const size_t a = n * t / th, b = n * (t + 1) / th;
          memcpy(m + a, buf.data() + a, b - a);
        });
      for (auto& x : ts) x.join();
      munmap(m, n);
      close(fd);
      report("mmap", th, now_s() - t0);
    }
  }
  unlink(path.c_str());
  return 0;
}

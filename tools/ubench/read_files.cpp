// Diagnostics: file-read scaling on tmpfs (config-5-like sizes, 4 KiB-1 MiB) with N threads,
// with and without a private fd table per thread.  g++ -O2 -std=c++17 read_files.cpp -lpthread
// usage: read_files make; read_files  (hipcc -O2 read_files.cpp -o read_files)
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sched.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <string>
#include <thread>
#include <cstring>
#include <vector>
int main(int argc, char** argv) {
  // "big": config-5 shape (100 k files, 4 KiB-4 MiB); default 20 k files of 4 KiB-1 MiB
  const bool big = std::getenv("RD_BIG") != nullptr;
  int n = big ? 100000 : 20000; const bool make = argc > 1 && std::string(argv[1]) == "make";
  const double hi = big ? 4194304.0 : 1048576.0;
  std::mt19937_64 g(1); std::vector<size_t> sz(n); std::vector<std::string> paths(n);
  size_t total = 0;
  for (int i = 0; i < n; i++) { double u = std::uniform_real_distribution<double>(std::log(4096.0), std::log(hi))(g); sz[i] = (size_t)std::exp(u); paths[i] = "/dev/shm/rdtest/f" + std::to_string(i); total += sz[i]; }
  // RD_DIR=d: read the files d/* instead (e.g. bench_config5.py --keep's directory)
  if (const char* dir = std::getenv("RD_DIR")) {
    paths.clear(); sz.clear(); total = 0;
    if (DIR* dp = opendir(dir)) {
      while (dirent* e = readdir(dp)) {
        if (e->d_name[0] == '.') continue;
        std::string p = std::string(dir) + "/" + e->d_name;
        struct stat st;
        if (stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode)) { paths.push_back(p); sz.push_back(st.st_size); total += st.st_size; }
      }
      closedir(dp);
    }
    std::sort(paths.begin(), paths.end());
    for (size_t i = 0; i < paths.size(); i++) { struct stat st; stat(paths[i].c_str(), &st); sz[i] = st.st_size; }
    n = (int)paths.size();
    printf("RD_DIR %s: %d files %.2f GB\n", dir, n, total / 1e9);
  }
  if (make) { system("mkdir -p /dev/shm/rdtest"); std::vector<char> buf(4 << 20, 7); for (int i = 0; i < n; i++) { FILE* f = fopen(paths[i].c_str(), "wb"); fwrite(buf.data(), 1, sz[i], f); fclose(f);} return 0; }
  std::vector<char> pageable(total); std::vector<size_t> off(n); size_t o = 0; for (int i = 0; i < n; i++) { off[i] = o; o += sz[i]; }
  char* pinned = nullptr;
  if (hipHostMalloc((void**)&pinned, total, hipHostMallocDefault) != hipSuccess) return 1;
  memset(pinned, 1, total);
  // RD_H2D=1: a background thread copies a pinned 1 GiB buffer to the device in a loop meanwhile
  std::atomic<bool> stop{false};
  std::thread h2d;
  if (std::getenv("RD_H2D")) {
    h2d = std::thread([&] {
      void *hs = nullptr, *ds = nullptr;
      hipHostMalloc(&hs, 1ull << 30, hipHostMallocDefault);
      hipMalloc(&ds, 1ull << 30);
      size_t k = 0;
      auto t0 = std::chrono::steady_clock::now();
      while (!stop) { hipMemcpy(ds, hs, 1ull << 30, hipMemcpyHostToDevice); k++; }
      double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      printf("background H2D: %.1f GB/s\n", k * 1.073741824 / dt);
    });
  }
  for (int pin : {0, 1}) for (int threads : {1, 4, 16}) for (int un : {0}) {
    char* dstp = pin ? pinned : pageable.data();
    std::atomic<int> next{0};
    auto w = [&](bool own) { if (own && un) unshare(CLONE_FILES); for (;;) { int i = next++; if (i >= n) return; int fd = open(paths[i].c_str(), O_RDONLY | O_CLOEXEC); size_t got = 0; while (got < sz[i]) { ssize_t r = pread(fd, dstp + off[i] + got, sz[i] - got, got); if (r <= 0) break; got += r; } close(fd);} };
    auto t0 = std::chrono::steady_clock::now();
    // RD_BATCH=k: files in batches of k, fresh threads per batch (the engine's read_files structure)
    const int bsz = std::getenv("RD_BATCH") ? std::atoi(std::getenv("RD_BATCH")) : n;
    for (int b0 = 0; b0 < n; b0 += bsz) {
      std::atomic<int> nx{b0};
      const int b1 = std::min(n, b0 + bsz);
      auto wb = [&](bool own) { if (own && un) unshare(CLONE_FILES); for (;;) { int i = nx++; if (i >= b1) return; int fd = open(paths[i].c_str(), O_RDONLY | O_CLOEXEC); size_t got = 0; while (got < sz[i]) { ssize_t r = pread(fd, dstp + off[i] + got, sz[i] - got, got); if (r <= 0) break; got += r; } close(fd);} };
      std::vector<std::thread> ts; for (int t = 1; t < threads; t++) ts.emplace_back(wb, true); wb(false); for (auto& t : ts) t.join();
    }
    (void)next; (void)w;
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%s threads=%d: %.0f files/s %.2f GB/s\n", pin ? "pinned" : "pageable", threads, n / dt, total / dt / 1e9);
  }
  stop = true;
  if (h2d.joinable()) h2d.join();
}

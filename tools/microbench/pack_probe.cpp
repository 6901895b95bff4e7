// Host-side cost of packing a 1K-signature batch (~336 KB: key indices, signatures, offsets,
// lengths, 256-B messages) from pageable memory into pinned memory, as submit_host does for the
// p50 @ 1K path: one thread vs T threads (persistent workers woken per batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main() {
  const size_t bytes = 1024 * (4 + 64 + 8 + 4 + 256);
  std::vector<uint8_t> src(bytes, 7);
  void* dst = nullptr;
  if (hipHostMalloc(&dst, bytes, 0) != hipSuccess) return 1;
  auto now = [] { return std::chrono::steady_clock::now(); };
  for (int threads : {1, 2, 4, 8}) {
    std::atomic<int> go{0}, done{0};
    std::atomic<bool> stop{false};
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++)
      pool.emplace_back([&, t] {
        int seen = 0;
        while (!stop.load()) {
          const int g = go.load(std::memory_order_acquire);
          if (g == seen) continue;
          seen = g;
          const size_t lo = bytes * t / threads, hi = bytes * (t + 1) / threads;
          std::memcpy(static_cast<uint8_t*>(dst) + lo, src.data() + lo, hi - lo);
          done.fetch_add(1, std::memory_order_acq_rel);
        }
      });
    std::vector<double> us;
    for (int it = 0; it < 2000; it++) {
      const auto t0 = now();
      done.store(0);
      go.fetch_add(1, std::memory_order_acq_rel);
      std::memcpy(dst, src.data(), bytes / threads);
      while (done.load(std::memory_order_acquire) != threads - 1) {
      }
      us.push_back(std::chrono::duration<double, std::micro>(now() - t0).count());
    }
    stop = true;
    for (auto& th : pool) th.join();
    std::sort(us.begin(), us.end());
    std::printf("pack %zu B with %d thread(s): p50 %.1f us, p90 %.1f us\n", bytes, threads, us[us.size() / 2],
                us[us.size() * 9 / 10]);
  }
  (void)hipHostFree(dst);
  return 0;
}

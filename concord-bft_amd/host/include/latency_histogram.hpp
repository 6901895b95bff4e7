// HDR-style latency histograms around the signature-verification calls, the idiom of the
// reference's diagnostics TimeRecorder / DEFINE_SHARED_RECORDER (diagnostics/include/
// performance_handler.h:48-94, used around verify sites at PreProcessReplyMsg.cpp:84 and
// PreProcessorRecorder.hpp:60), without the hdr_histogram dependency: values in nanoseconds,
// log2 magnitude buckets with 64 linear sub-buckets each (relative error < 1.6 %), lock-free
// atomic counts, percentiles on demand.  Header-only.
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <string>

namespace concord::hip {

class LatencyHistogram {
 public:
  static constexpr int kSub = 64;  // linear sub-buckets per power of two
  static constexpr int kMag = 48;  // magnitudes: values up to 2^48 ns (~3 days)

  void record(uint64_t ns) {
    counts_[index(ns)].fetch_add(1, std::memory_order_relaxed);
    total_.fetch_add(1, std::memory_order_relaxed);
    sum_.fetch_add(ns, std::memory_order_relaxed);
    uint64_t m = max_.load(std::memory_order_relaxed);
    while (ns > m && !max_.compare_exchange_weak(m, ns, std::memory_order_relaxed)) {
    }
  }
  uint64_t count() const { return total_.load(std::memory_order_relaxed); }
  uint64_t max() const { return max_.load(std::memory_order_relaxed); }
  double mean() const { return count() ? (double)sum_.load(std::memory_order_relaxed) / (double)count() : 0.0; }
  // Smallest bucket upper bound below which at least q (0..1) of the recorded values fall.
  uint64_t percentile(double q) const {
    const uint64_t n = count();
    if (!n) return 0;
    const uint64_t want = q <= 0 ? 1 : (uint64_t)(q * (double)n + 0.999999);
    uint64_t seen = 0;
    for (size_t i = 0; i < counts_.size(); i++) {
      seen += counts_[i].load(std::memory_order_relaxed);
      if (seen >= want) return upper(i);
    }
    return max();
  }
  void reset() {
    for (auto& c : counts_) c.store(0, std::memory_order_relaxed);
    total_ = 0;
    sum_ = 0;
    max_ = 0;
  }

  // RAII timer: records the elapsed time of its scope (TimeRecorder's scoped form)
  class Scope {
   public:
    explicit Scope(LatencyHistogram& h) : h_(h), t0_(std::chrono::steady_clock::now()) {}
    ~Scope() {
      h_.record((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_)
                    .count());
    }

   private:
    LatencyHistogram& h_;
    std::chrono::steady_clock::time_point t0_;
  };

 private:
  static size_t index(uint64_t v) {
    if (v < (uint64_t)kSub) return (size_t)v;  // magnitude 0: exact
    const int msb = 63 - __builtin_clzll(v);    // >= 6
    const int mag = msb - 5;                    // 1..
    if (mag >= kMag) return (size_t)kMag * kSub - 1;
    return (size_t)mag * kSub + (size_t)((v >> (msb - 6)) & (kSub - 1));
  }
  static uint64_t upper(size_t i) {
    const size_t mag = i / kSub, sub = i % kSub;
    if (mag == 0) return sub;
    return ((uint64_t)(kSub + sub + 1) << (mag - 1)) - 1;
  }

  std::array<std::atomic<uint64_t>, (size_t)kMag * kSub> counts_{};
  std::atomic<uint64_t> total_{0}, sum_{0}, max_{0};
};

// The process-wide recorders of the signature path (DEFINE_SHARED_RECORDER's role).
struct VerifyRecorders {
  LatencyHistogram ed25519_verify;           // HipEdDSAVerifier::verify(), call to verdict (coalesced)
  LatencyHistogram rsa_verify;               // HipRSAVerifier::verify()
  LatencyHistogram verify_batch;             // concord::hip::verifyBatch(), one mixed batch
  LatencyHistogram sig_manager_batch;        // HipSigManager::verifySigBatch()
};
inline VerifyRecorders& recorders() {
  static VerifyRecorders r;
  return r;
}

}  // namespace concord::hip

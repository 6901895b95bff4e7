// Per-request path benchmark (VERDICT r2 "measure the per-request path"): what the reference's
// pool threads do — each request validated on its own thread, one IVerifier::verify /
// SigManager::verifySig per signature (ClientRequestMsg.cpp:197-213 from RequestThreadPool,
// ReplicaImp.cpp:290-316; 40 + 24 threads, ReplicaConfig.hpp:202-212).  The GPU engine coalesces
// the concurrent single calls into batches (hip_ed25519.cpp, Ed25519Engine::verifyOne).
//
//   host_bench [threads=64] [calls_per_thread=2000] [nkeys=1024] [cpu_threads=16]
//
// Legs (every verdict checked; exit 1 on any mismatch):
//   verify_mt      T threads x HipEdDSAVerifier::verify
//   verifysig_mt   T threads x HipSigManager::verifySig (the reference's own method, inherited)
//   single         one thread, one call at a time: the unloaded single-verify latency
//   openssl_mt     the same signatures, OpenSSL 3 EVP_DigestVerify on cpu_threads threads (the
//                  reference-style CPU verifier, EVP_PKEY cached per key)
// Prints one JSON object.
#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <sys/resource.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "ReplicaConfig.hpp"
#include "hip_crypto.hpp"
#include "hip_sig_manager.hpp"

using namespace concord::hip;
using bftEngine::impl::PrincipalId;
using bftEngine::impl::ReplicaIdsConfig;
using bftEngine::impl::ReplicasInfo;
using Clock = std::chrono::steady_clock;

namespace {
std::string seedHex(int i) {
  std::mt19937 g(777 + i);
  uint8_t b[32];
  for (auto& x : b) x = (uint8_t)g();
  return toHex(b, 32);
}

struct Work {
  std::vector<uint32_t> key;
  std::vector<std::string> msg, sig;
  std::vector<char> expect;
};

double pct(std::vector<double>& v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
}

struct LegResult {
  double per_s, p50_us, p99_us;
  uint64_t batches, calls, mismatches;
  double cores_busy;  // process CPU time (user + system) / wall time over the leg
};

double cpuSeconds() {
  rusage u{};
  getrusage(RUSAGE_SELF, &u);
  return (double)u.ru_utime.tv_sec + 1e-6 * (double)u.ru_utime.tv_usec + (double)u.ru_stime.tv_sec +
         1e-6 * (double)u.ru_stime.tv_usec;
}

template <class Fn>
LegResult runThreads(int T, int calls, const std::vector<Work>& w, Fn fn) {
  std::vector<std::vector<double>> lat(T);
  std::atomic<uint64_t> bad{0};
  const uint64_t b0 = ed25519EngineStats().batches;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      lat[t].reserve(calls);
      ready++;
      while (!go.load()) std::this_thread::yield();
      const Work& x = w[t];
      for (int k = 0; k < calls; k++) {
        const auto c0 = Clock::now();
        const bool v = fn(x, k);
        lat[t].push_back(std::chrono::duration<double, std::micro>(Clock::now() - c0).count());
        if (v != (bool)x.expect[k]) bad++;
      }
    });
  while (ready.load() < T) std::this_thread::yield();
  const double cpu0 = cpuSeconds();
  const auto t0 = Clock::now();
  go = true;
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  const double cpu = cpuSeconds() - cpu0;
  std::vector<double> all;
  for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
  LegResult r{(double)T * calls / secs, pct(all, 0.5), pct(all, 0.99), ed25519EngineStats().batches - b0,
              (uint64_t)T * calls, bad.load(), cpu / secs};
  return r;
}

void printLeg(const char* name, const LegResult& r, int threads, bool last = false) {
  std::printf("\"%s\": {\"threads\": %d, \"calls\": %llu, \"verifies_per_s\": %.1f, \"p50_us\": %.1f, "
              "\"p99_us\": %.1f, \"gpu_batches\": %llu, \"calls_per_batch\": %.2f, \"mismatches\": %llu, "
              "\"cores_busy\": %.2f, \"cpu_us_per_call\": %.2f}%s",
              name, threads, (unsigned long long)r.calls, r.per_s, r.p50_us, r.p99_us, (unsigned long long)r.batches,
              r.batches ? (double)r.calls / (double)r.batches : 0.0, (unsigned long long)r.mismatches, r.cores_busy,
              r.per_s > 0 ? 1e6 * r.cores_busy / r.per_s : 0.0, last ? "" : ", ");
}
}  // namespace

int main(int argc, char** argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 64;
  const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
  const int nkeys = argc > 3 ? std::atoi(argv[3]) : 1024;
  const int cpuT = argc > 4 ? std::atoi(argv[4]) : 16;
  bftEngine::ReplicaConfig::instance().clientTransactionSigningEnabled = true;

  // principals: 4 replicas (0..3), nkeys external clients (4 ..)
  std::vector<std::unique_ptr<EdDSASigner>> signers;
  std::vector<std::string> pubs;
  for (int k = 0; k < nkeys; k++) {
    signers.emplace_back(new EdDSASigner(seedHex(k), KeyFormat::HexaDecimalStrippedFormat));
    pubs.push_back(signers.back()->getPubKeyHex());
  }
  ReplicaIdsConfig cfg;
  cfg.replicaId = 0;
  cfg.numOfExternalClients = (uint16_t)nkeys;
  ReplicasInfo ri(cfg);
  HipSigManager::ReplicaKeys replicaKeys;
  EdDSASigner rs(seedHex(100000), KeyFormat::HexaDecimalStrippedFormat);
  for (PrincipalId r = 0; r < 4; r++) replicaKeys.insert({r, rs.getPubKeyHex()});
  HipSigManager::ClientKeys clientKeys;
  for (int k = 0; k < nkeys; k++) clientKeys.insert({pubs[k], {(uint16_t)(4 + k)}});
  std::unique_ptr<HipSigManager> sm(HipSigManager::initInTesting(0, seedHex(100000), replicaKeys,
                                                                 KeyFormat::HexaDecimalStrippedFormat, &clientKeys,
                                                                 KeyFormat::HexaDecimalStrippedFormat, ri));
  std::vector<std::unique_ptr<HipEdDSAVerifier>> verifiers;
  for (int k = 0; k < nkeys; k++)
    verifiers.emplace_back(new HipEdDSAVerifier(pubs[k], KeyFormat::HexaDecimalStrippedFormat));

  // T threads x calls requests, 256-byte payloads, every 10th signature corrupted
  std::vector<Work> w(T);
  for (int t = 0; t < T; t++) {
    std::mt19937 g(31 * t + 7);
    for (int k = 0; k < calls; k++) {
      const uint32_t key = g() % nkeys;
      std::string m(256, '\0');
      for (auto& ch : m) ch = (char)g();
      std::string s = signers[key]->sign(m);
      const bool ok = (t * calls + k) % 10 != 3;
      if (!ok) s[5 + g() % 50] ^= 0x10;
      w[t].key.push_back(key);
      w[t].msg.push_back(std::move(m));
      w[t].sig.push_back(std::move(s));
      w[t].expect.push_back(ok);
    }
  }
  // warm-up: every key loaded on the device, the engine's buffers sized
  runThreads(T, std::min(calls, 50), w, [&](const Work& x, int k) { return verifiers[x.key[k]]->verify(x.msg[k], x.sig[k]); });

  const LegResult a =
      runThreads(T, calls, w, [&](const Work& x, int k) { return verifiers[x.key[k]]->verify(x.msg[k], x.sig[k]); });
  const LegResult b = runThreads(T, calls, w, [&](const Work& x, int k) {
    return sm->verifySig((PrincipalId)(4 + x.key[k]), x.msg[k].data(), x.msg[k].size(), x.sig[k].data(),
                         (uint16_t)x.sig[k].size());
  });
  const int singles = std::min(calls, 500);
  const LegResult c =
      runThreads(1, singles, w, [&](const Work& x, int k) { return verifiers[x.key[k]]->verify(x.msg[k], x.sig[k]); });

  // OpenSSL on the host: EVP_PKEY cached per key (SigManager keeps one verifier per key)
  std::vector<EVP_PKEY*> pk(nkeys);
  for (int k = 0; k < nkeys; k++) {
    std::vector<uint8_t> raw;
    fromHex(pubs[k], raw);
    pk[k] = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, raw.data(), 32);
  }
  const int cpuCalls = std::max(1, std::min(calls, 4000 * cpuT / std::max(1, T)));
  std::vector<Work> wc(w.begin(), w.begin() + std::min(T, cpuT));
  const LegResult d = runThreads((int)wc.size(), cpuCalls, wc, [&](const Work& x, int k) {
    EVP_MD_CTX* ctx = EVP_MD_CTX_new();
    const bool ok = EVP_DigestVerifyInit(ctx, nullptr, nullptr, nullptr, pk[x.key[k]]) == 1 &&
                    EVP_DigestVerify(ctx, reinterpret_cast<const unsigned char*>(x.sig[k].data()), x.sig[k].size(),
                                     reinterpret_cast<const unsigned char*>(x.msg[k].data()), x.msg[k].size()) == 1;
    EVP_MD_CTX_free(ctx);
    return ok;
  });
  for (auto* p : pk) EVP_PKEY_free(p);

  const auto hv = recorders().ed25519_verify.percentile(0.5);
  std::printf("{");
  printLeg("verify_mt", a, T);
  printLeg("verifysig_mt", b, T);
  printLeg("single", c, 1);
  printLeg("openssl_mt", d, (int)wc.size());
  const auto st = ed25519EngineStats();
  std::printf("\"gpu_vs_openssl_mt\": %.2f, \"engine\": {\"batches\": %llu, \"items\": %llu, \"gpu_errors\": %llu}, "
              "\"verify_histogram_p50_us\": %.1f, \"nkeys\": %d, \"msg_len\": 256, \"invalid_every\": 10}\n",
              a.per_s / d.per_s, (unsigned long long)st.batches, (unsigned long long)st.items,
              (unsigned long long)st.gpu_errors, hv / 1e3, nkeys);
  const bool exact = !a.mismatches && !b.mismatches && !c.mismatches && !d.mismatches && !st.gpu_errors;
  return exact ? 0 : 1;
}

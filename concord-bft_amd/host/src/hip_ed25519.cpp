// HipEdDSAVerifier / EdDSASigner over libcbft_hipcrypto, and the process-wide Ed25519 engine that
// owns the device key table (see hip_crypto.hpp).
#include "hip_crypto.hpp"

#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "cbft_hipcrypto.h"

namespace concord::hip {

// ---------------------------------------------------------------------------------- encoding
std::string toHex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool fromHex(const std::string& hex, std::vector<uint8_t>& out) {
  if (hex.size() % 2) return false;
  out.resize(hex.size() / 2);
  for (size_t i = 0; i < out.size(); i++) {
    int a = hexval(hex[2 * i]), b = hexval(hex[2 * i + 1]);
    if (a < 0 || b < 0) return false;
    out[i] = (uint8_t)(a * 16 + b);
  }
  return true;
}

static bool base64Decode(const std::string& in, std::vector<uint8_t>& out) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
  };
  out.clear();
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    int v = val(c);
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
    }
  }
  return true;
}

static std::string base64Encode(const uint8_t* p, size_t n) {
  static const char* t = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string s;
  for (size_t i = 0; i < n; i += 3) {
    uint32_t v = (uint32_t)p[i] << 16 | (i + 1 < n ? (uint32_t)p[i + 1] << 8 : 0) | (i + 2 < n ? p[i + 2] : 0);
    s += t[(v >> 18) & 63];
    s += t[(v >> 12) & 63];
    s += i + 1 < n ? t[(v >> 6) & 63] : '=';
    s += i + 2 < n ? t[v & 63] : '=';
  }
  return s;
}

// SubjectPublicKeyInfo of an Ed25519 key (RFC 8410 §4): 12-byte DER prefix + 32 key bytes
static const uint8_t kSpkiPrefix[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};

bool parseEd25519PublicKey(const std::string& s, KeyFormat fmt, uint8_t out[32]) {
  std::vector<uint8_t> b;
  if (fmt == KeyFormat::HexaDecimalStrippedFormat) {
    if (!fromHex(s, b)) return false;
    if (b.size() == 44 && std::memcmp(b.data(), kSpkiPrefix, 12) == 0) b.erase(b.begin(), b.begin() + 12);
  } else {
    const std::string begin = "-----BEGIN PUBLIC KEY-----", end = "-----END PUBLIC KEY-----";
    auto p = s.find(begin), q = s.find(end);
    if (p == std::string::npos || q == std::string::npos || q < p) return false;
    if (!base64Decode(s.substr(p + begin.size(), q - p - begin.size()), b)) return false;
    if (b.size() != 44 || std::memcmp(b.data(), kSpkiPrefix, 12) != 0) return false;
    b.erase(b.begin(), b.begin() + 12);
  }
  if (b.size() != 32) return false;
  std::memcpy(out, b.data(), 32);
  return true;
}

std::string ed25519PublicKeyToPem(const uint8_t raw[32]) {
  uint8_t der[44];
  std::memcpy(der, kSpkiPrefix, 12);
  std::memcpy(der + 12, raw, 32);
  return "-----BEGIN PUBLIC KEY-----\n" + base64Encode(der, 44) + "\n-----END PUBLIC KEY-----\n";
}

// ---------------------------------------------------------------------------------- engine
static int g_device = -1;
void setEd25519Device(int device) { g_device = device; }

// Comb radix the engine's key table starts with, for the expected number of keys
// ($CBFT_EXPECTED_KEYS, default 4,096) against the library's 64 GB budget: radix 13 (10.5 MB per
// key) up to ~6,100 keys, 11 (3.0 MB) up to ~21,000, then 8 (0.53 MB).  More keys than expected is
// safe: the library re-radixes the table once the budget would be exceeded
// (cbft_ed25519_append_keys).
static int engineRadix() {
  if (const char* e = std::getenv("CBFT_COMB_RADIX")) return std::atoi(e);
  double keys = 4096;
  if (const char* e = std::getenv("CBFT_EXPECTED_KEYS")) keys = std::atof(e);
  auto bytes_per_key = [](int w, int npos) { return (double)npos * ((1 << (w - 1)) + 1) * 128.0; };
  if (keys * bytes_per_key(13, 20) <= 64e9) return 13;
  if (keys * bytes_per_key(11, 23) <= 64e9) return 11;
  return 8;
}

// Per-process owner of the GPU context and of the device key table.
//
// Keys are registered when a verifier is constructed and reference-counted per slot (equal keys
// share a slot, as SigManager shares one verifier object between principals with the same key,
// SigManager.cpp:139-150).  A new key is appended to the device table (its comb table built
// alone; loaded keys untouched) before the first batch that needs it; a slot whose last verifier
// is gone is reused by the next new key (rebuilt in place, cbft_ed25519_replace_keys), so client
// key rotation (SigManager::setClientPublicKey) does not grow the table.
//
// verifyOne() coalesces concurrent single verifies (the reference calls IVerifier::verify from
// 40 + 24 pool threads, ReplicaConfig.hpp:202-212): callers queue their request; one of them
// leads a batch as soon as fewer than maxInflight_ batches are on the GPU, taking everything
// queued by then.  A lone caller goes straight to the GPU; under load, requests that arrive
// while batches run are verified together in the next one.
//
// Waiting.  Each request waits on its own 32-bit state word (futex), never on the queue's mutex:
// the leader of a batch publishes every verdict with one release store per request and wakes
// only the requests that went to sleep.  A woken request reads its verdict and returns without
// touching q_mu_ (with condition variables on the queue mutex, the ~20 requests of a batch woke
// into a convoy on that mutex: round 3's per-request profile).  A waiter first spins for a few
// microseconds with yields when $CBFT_ENGINE_SPIN_US is set (default 0: it sleeps at once, the fastest
// setting in profiles/r04_ab/spin0_*.json), then sleeps.
class Ed25519Engine {
 public:
  static constexpr int kMaxInflight = 4;  // profiles/r03_host_bench_sweep.txt (zero-copy, blocking-sync small batches)
  static constexpr size_t kMaxBatch = 65536;

  static std::shared_ptr<Ed25519Engine> get() {
    static std::mutex m;
    static std::weak_ptr<Ed25519Engine> inst;
    std::lock_guard<std::mutex> g(m);
    auto sp = inst.lock();
    if (!sp) {
      sp = std::shared_ptr<Ed25519Engine>(new Ed25519Engine());
      inst = sp;
    }
    return sp;
  }
  ~Ed25519Engine() {
    if (ctx_) cbft_close(ctx_);
  }

  uint32_t registerKey(const uint8_t raw[32]) {
    std::lock_guard<std::mutex> ag(append_mu_);  // a slot rebuild is a device-table write
    std::lock_guard<std::mutex> g(keys_mu_);
    std::string k(reinterpret_cast<const char*>(raw), 32);
    auto it = index_.find(k);
    if (it != index_.end()) {
      refs_[it->second]++;
      return it->second;
    }
    uint32_t idx;
    if (!free_.empty()) {
      idx = free_.back();
      free_.pop_back();
      std::memcpy(&keys_[(size_t)idx * 32], raw, 32);
      if (idx < loaded_.load()) {  // on the device already: rebuild the slot in place
        const int rc = cbft_ed25519_replace_keys(ctx_, table_, &idx, raw, 1);
        if (rc != CBFT_OK) {
          free_.push_back(idx);
          throw std::runtime_error(std::string("cbft_ed25519_replace_keys: ") + cbft_strerror(rc) + " " +
                                   cbft_last_error());
        }
      }
      refs_[idx] = 1;
    } else {
      idx = (uint32_t)(keys_.size() / 32);
      keys_.insert(keys_.end(), raw, raw + 32);
      refs_.push_back(1);
    }
    index_.emplace(std::move(k), idx);
    return idx;
  }

  void addRef(uint32_t idx) {
    std::lock_guard<std::mutex> g(keys_mu_);
    refs_[idx]++;
  }

  void releaseKey(uint32_t idx) {
    std::lock_guard<std::mutex> g(keys_mu_);
    if (--refs_[idx]) return;
    index_.erase(std::string(reinterpret_cast<const char*>(&keys_[(size_t)idx * 32]), 32));
    free_.push_back(idx);
  }

  // One GPU batch; out[i] = verdict of reqs[i] (false for non-Ed25519 verifiers).  Throws on a
  // GPU failure (callers turn it into false verdicts).
  void verify(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
    out.assign(reqs.size(), false);
    // wrong-length signatures (EVP returns 0) and messages the kernel's 32-bit SHA-512 length
    // cannot hold are rejected without a GPU round trip
    std::vector<size_t> pos;
    pos.reserve(reqs.size());
    size_t blob = 0;
    uint32_t maxKey = 0;
    std::vector<const HipEdDSAVerifier*> ver(reqs.size(), nullptr);
    for (size_t i = 0; i < reqs.size(); i++) {
      ver[i] = dynamic_cast<const HipEdDSAVerifier*>(reqs[i].verifier);
      if (reqs[i].sigLength == 64 && ver[i] && reqs[i].dataLength <= kMaxMsg) {
        pos.push_back(i);
        blob += reqs[i].dataLength;
        maxKey = std::max(maxKey, ver[i]->engineKeyIndex());
      }
    }
    if (pos.empty()) return;
    const size_t n = pos.size();
    std::vector<uint32_t> kidx(n), len(n);
    std::vector<uint64_t> off(n);
    std::vector<uint8_t> sig(n * 64), msg(blob ? blob : 1), bitmap((n + 7) / 8);
    size_t o = 0;
    for (size_t j = 0; j < n; j++) {
      const VerifyRequest& r = reqs[pos[j]];
      kidx[j] = ver[pos[j]]->engineKeyIndex();
      std::memcpy(&sig[64 * j], r.sig, 64);
      off[j] = o;
      len[j] = (uint32_t)r.dataLength;
      if (r.dataLength) std::memcpy(&msg[o], r.data, r.dataLength);
      o += r.dataLength;
    }
    ensureLoaded(maxKey);
    batches_++;
    items_ += n;
    int rc = cbft_ed25519_verify_batch(ctx_, table_, kidx.data(), sig.data(), msg.data(), off.data(), len.data(), n,
                                       bitmap.data());
    if (rc != CBFT_OK)
      throw std::runtime_error(std::string("cbft_ed25519_verify_batch: ") + cbft_strerror(rc) + " " +
                               cbft_last_error());
    for (size_t j = 0; j < n; j++) out[pos[j]] = (bitmap[j >> 3] >> (j & 7)) & 1;
  }

  // verify() for a batch API caller: a GPU failure gives false verdicts (IVerifier's contract:
  // verification never throws, openssl_crypto.cpp:247-253) and is counted.
  void verifyNoThrow(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
    try {
      verify(reqs, out);
    } catch (...) {
      gpu_errors_++;
      out.assign(reqs.size(), false);
    }
  }

  bool verifyOne(const HipEdDSAVerifier* v, const char* data, size_t len, const char* sig, size_t sigLen) {
    if (sigLen != 64 || len > kMaxMsg) return false;
    LatencyHistogram::Scope timer(recorders().ed25519_verify);
    Pending p{v, data, len, sig, sigLen};
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      queue_.push_back(&p);
      if (!leader_ && inflight_ < maxInflight_) {  // a GPU slot is free: go now, with whatever is queued
        p.state.store(kLead, std::memory_order_relaxed);
        leader_ = true;
      }
    }
    for (;;) {
      const int st = waitState(p);
      if (st == kDone) return p.verdict;
      // kLead: lead one batch, everything queued so far (up to kMaxBatch)
      p.state.store(kWaiting, std::memory_order_relaxed);
      std::vector<Pending*> batch;
      {
        std::lock_guard<std::mutex> lk(q_mu_);
        if (queue_.size() <= kMaxBatch) {
          batch.swap(queue_);
        } else {
          batch.assign(queue_.begin(), queue_.begin() + kMaxBatch);
          queue_.erase(queue_.begin(), queue_.begin() + kMaxBatch);
        }
        leader_ = false;
        inflight_++;
        appointLocked();  // requests that queued meanwhile may lead the next batch if a slot is free
      }
      runBatch(batch);
      {
        std::lock_guard<std::mutex> lk(q_mu_);
        inflight_--;
        appointLocked();
      }
      for (Pending* q : batch) post(*q, kDone);  // verdicts were written by runBatch
    }
  }

  EngineStats stats() {
    std::lock_guard<std::mutex> g(keys_mu_);
    return EngineStats{batches_.load(), items_.load(), gpu_errors_.load(),
                       (uint32_t)(keys_.size() / 32 - free_.size()), (uint32_t)(keys_.size() / 32)};
  }

 private:
  static constexpr size_t kMaxMsg = 0xFFFFFF00u;
  // request states; a waiter about to sleep marks its word kSleeping (the poster then wakes it)
  static constexpr int kWaiting = 0, kLead = 1, kDone = 2, kSleeping = 3;
  struct Pending {
    const HipEdDSAVerifier* v;
    const char* data;
    size_t len;
    const char* sig;
    size_t sigLen;
    bool verdict = false;
    std::atomic<int> state{kWaiting};
  };
  static long futex(std::atomic<int>* w, int op, int val) {
    return syscall(SYS_futex, reinterpret_cast<int*>(w), op | FUTEX_PRIVATE_FLAG, val, nullptr, nullptr, 0);
  }
  // this request's next state (kLead or kDone): spin briefly, then sleep on the futex word
  int waitState(Pending& p) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      int st = p.state.load(std::memory_order_acquire);
      if (st == kLead || st == kDone) return st;
      if (std::chrono::steady_clock::now() - t0 < spin_) {
        std::this_thread::yield();
        continue;
      }
      if (st == kWaiting && !p.state.compare_exchange_strong(st, kSleeping, std::memory_order_acq_rel)) continue;
      futex(&p.state, FUTEX_WAIT, kSleeping);  // returns when the word is no longer kSleeping
    }
  }
  // hand request q its next state; wake it only if it went to sleep
  static void post(Pending& q, int st) {
    if (q.state.exchange(st, std::memory_order_acq_rel) == kSleeping) futex(&q.state, FUTEX_WAKE, 1);
  }

  // With no leader and a free GPU slot, the oldest queued request leads the next batch (q_mu_
  // held).  Waking only that one request, and each finished request only once, keeps 64 pool
  // threads from stampeding at every batch boundary.
  void appointLocked() {
    if (leader_ || queue_.empty() || inflight_ >= maxInflight_) return;
    Pending* h = queue_.front();
    leader_ = true;
    post(*h, kLead);
  }

  void runBatch(std::vector<Pending*>& batch) {
    std::vector<VerifyRequest> reqs(batch.size());
    for (size_t i = 0; i < batch.size(); i++)
      reqs[i] = {batch[i]->v, batch[i]->data, batch[i]->len, batch[i]->sig, batch[i]->sigLen};
    std::vector<bool> out;
    verifyNoThrow(reqs, out);
    for (size_t i = 0; i < batch.size(); i++) batch[i]->verdict = out[i];
  }

  Ed25519Engine() {
    int dev = g_device;
    if (dev < 0) {
      const char* e = std::getenv("CBFT_DEVICE");
      dev = e ? std::atoi(e) : 0;
    }
    int rc = cbft_open(&ctx_, dev, 0);
    if (rc == CBFT_OK) rc = cbft_ed25519_load_keys_ex(ctx_, nullptr, 0, engineRadix(), &table_);
    if (rc != CBFT_OK)
      throw std::runtime_error(std::string("Ed25519 engine: ") + cbft_strerror(rc) + " " + cbft_last_error());
  }

  // Append every registered key not yet on the device, if key `need` is among them.
  void ensureLoaded(uint32_t need) {
    if (need < loaded_.load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> ag(append_mu_);
    const uint32_t have = loaded_.load();
    if (need < have) return;  // another thread appended it meanwhile
    std::vector<uint8_t> fresh;
    {
      std::lock_guard<std::mutex> g(keys_mu_);
      fresh.assign(keys_.begin() + (size_t)have * 32, keys_.end());
    }
    uint32_t first = 0;
    const uint32_t m = (uint32_t)(fresh.size() / 32);
    int rc = cbft_ed25519_append_keys(ctx_, table_, fresh.data(), m, &first);
    if (rc != CBFT_OK || first != have)
      throw std::runtime_error(std::string("cbft_ed25519_append_keys: ") + cbft_strerror(rc) + " " +
                               cbft_last_error());
    loaded_.store(have + m, std::memory_order_release);
  }

  cbft_ctx* ctx_ = nullptr;
  uint32_t table_ = CBFT_NO_KEY_TABLE;
  std::mutex keys_mu_;  // guards keys_, index_, refs_, free_
  std::vector<uint8_t> keys_;
  std::map<std::string, uint32_t> index_;
  std::vector<uint32_t> refs_;
  std::vector<uint32_t> free_;
  std::mutex append_mu_;  // one device-table write (append / slot rebuild) at a time
  std::atomic<uint32_t> loaded_{0};
  std::mutex q_mu_;  // coalescing queue
  std::vector<Pending*> queue_;
  int maxInflight_ = [] {  // GPU batches in flight ($CBFT_ENGINE_INFLIGHT, default kMaxInflight)
    const char* e = std::getenv("CBFT_ENGINE_INFLIGHT");
    const int v = e ? std::atoi(e) : kMaxInflight;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  bool leader_ = false;
  int inflight_ = 0;
  // $CBFT_ENGINE_SPIN_US: spin before sleeping (default 0: 64 pool threads yield-spinning on the
  // box's 16 cores cost more than the futex wake; 64-thread verify(): 508 K/s at 0, 455 K/s at 20 us)
  std::chrono::microseconds spin_{[] {
    const char* e = std::getenv("CBFT_ENGINE_SPIN_US");
    return e ? std::atoi(e) : 0;
  }()};
  std::atomic<uint64_t> batches_{0}, items_{0}, gpu_errors_{0};
};

EngineStats ed25519EngineStats() { return Ed25519Engine::get()->stats(); }

Ed25519KeyRef::Ed25519KeyRef(const Ed25519KeyRef& o) : engine_(o.engine_), index_(o.index_) { engine_->addRef(index_); }
Ed25519KeyRef::~Ed25519KeyRef() { engine_->releaseKey(index_); }

// ---------------------------------------------------------------------------------- verifier
static Ed25519KeyRef registerEd25519(const std::string& str_pub_key, KeyFormat fmt, uint8_t raw[32]) {
  if (!parseEd25519PublicKey(str_pub_key, fmt, raw)) throw std::invalid_argument("HipEdDSAVerifier: bad public key");
  auto engine = Ed25519Engine::get();
  const uint32_t idx = engine->registerKey(raw);
  return Ed25519KeyRef(std::move(engine), idx);
}

HipEdDSAVerifier::HipEdDSAVerifier(const std::string& str_pub_key, KeyFormat fmt)
    : key_str_(str_pub_key), raw_{}, key_(registerEd25519(str_pub_key, fmt, raw_)) {}

HipEdDSAVerifier::~HipEdDSAVerifier() = default;

bool HipEdDSAVerifier::verify(const std::string& data, const std::string& sig) const {
  return key_.engine().verifyOne(this, data.data(), data.size(), sig.data(), sig.size());
}

void HipEdDSAVerifier::verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
  out.assign(reqs.size(), false);
  if (reqs.empty()) return;
  const HipEdDSAVerifier* any = nullptr;
  for (auto& r : reqs)
    if ((any = dynamic_cast<const HipEdDSAVerifier*>(r.verifier))) break;
  if (!any) return;
  any->key_.engine().verifyNoThrow(reqs, out);
}

// ---------------------------------------------------------------------------------- signer
EdDSASigner::EdDSASigner(const std::string& str_priv_key, KeyFormat fmt) : key_str_(str_priv_key), pkey_(nullptr) {
  std::vector<uint8_t> seed;
  if (fmt == KeyFormat::HexaDecimalStrippedFormat) {
    if (!fromHex(str_priv_key, seed) || seed.size() != 32) throw std::invalid_argument("EdDSASigner: bad key");
    pkey_ = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, seed.data(), 32);
  } else {
    const std::string begin = "-----BEGIN PRIVATE KEY-----", end = "-----END PRIVATE KEY-----";
    auto p = str_priv_key.find(begin), q = str_priv_key.find(end);
    std::vector<uint8_t> der;
    if (p == std::string::npos || q == std::string::npos ||
        !base64Decode(str_priv_key.substr(p + begin.size(), q - p - begin.size()), der) || der.size() != 48)
      throw std::invalid_argument("EdDSASigner: bad PEM key");
    pkey_ = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, der.data() + 16, 32);  // RFC 8410 §7
  }
  if (!pkey_) throw std::invalid_argument("EdDSASigner: key rejected");
}

EdDSASigner::~EdDSASigner() {
  if (pkey_) EVP_PKEY_free(static_cast<EVP_PKEY*>(pkey_));
}

std::string EdDSASigner::sign(const std::string& data) {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  std::string sig(64, '\0');
  size_t sl = 64;
  bool ok = ctx && EVP_DigestSignInit(ctx, nullptr, nullptr, nullptr, static_cast<EVP_PKEY*>(pkey_)) == 1 &&
            EVP_DigestSign(ctx, reinterpret_cast<unsigned char*>(&sig[0]), &sl,
                           reinterpret_cast<const unsigned char*>(data.data()), data.size()) == 1;
  EVP_MD_CTX_free(ctx);
  if (!ok) throw std::runtime_error("EdDSASigner::sign failed");
  return sig;
}

std::string EdDSASigner::getPubKeyHex() const {
  uint8_t pk[32];
  size_t l = 32;
  EVP_PKEY_get_raw_public_key(static_cast<EVP_PKEY*>(pkey_), pk, &l);
  return toHex(pk, 32);
}

}  // namespace concord::hip

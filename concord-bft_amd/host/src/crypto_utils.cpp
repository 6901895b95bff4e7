// Ed25519 IVerifier / ISigner implementations over libcbft_hipcrypto (see crypto_utils.hpp).
#include "crypto_utils.hpp"

#include <openssl/evp.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>

#include "cbft_hipcrypto.h"

namespace concord::util::crypto {

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

// Per-process owner of the GPU context and of the device key table.  Keys are registered when a
// verifier is constructed (deduplicated: equal keys share an index, as SigManager shares one
// verifier object between principals with the same key, SigManager.cpp:139-150); the device
// table is rebuilt lazily before the first batch that needs a newly registered key.
class Ed25519Engine {
 public:
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
    std::lock_guard<std::mutex> g(mu_);
    std::string k(reinterpret_cast<const char*>(raw), 32);
    auto it = index_.find(k);
    if (it != index_.end()) return it->second;
    uint32_t idx = (uint32_t)keys_.size() / 32;
    keys_.insert(keys_.end(), raw, raw + 32);
    index_.emplace(std::move(k), idx);
    return idx;
  }

  void verify(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
    out.assign(reqs.size(), false);
    // signatures of the wrong length are rejected without a GPU round trip (EVP returns 0)
    std::vector<size_t> pos;
    pos.reserve(reqs.size());
    size_t blob = 0;
    std::vector<const EdDSAVerifier*> ver(reqs.size(), nullptr);
    for (size_t i = 0; i < reqs.size(); i++) {
      ver[i] = dynamic_cast<const EdDSAVerifier*>(reqs[i].verifier);
      if (reqs[i].sigLength == 64 && ver[i]) {
        pos.push_back(i);
        blob += reqs[i].dataLength;
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
    // the device table must cover every registered key; a rebuild (new key) takes the table
    // lock exclusively, verifies hold it shared for the duration of the GPU call
    std::shared_lock<std::shared_mutex> rd(tbl_mu_);
    while (true) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if (loaded_ == keys_.size() / 32 && table_ != CBFT_NO_KEY_TABLE) break;
      }
      rd.unlock();
      {
        std::unique_lock<std::shared_mutex> wr(tbl_mu_);
        std::lock_guard<std::mutex> g(mu_);
        ensureTableLocked();
      }
      rd.lock();
    }
    int rc = cbft_ed25519_verify_batch(ctx_, table_, kidx.data(), sig.data(), msg.data(), off.data(), len.data(), n,
                                       bitmap.data());
    if (rc != CBFT_OK)
      throw std::runtime_error(std::string("cbft_ed25519_verify_batch: ") + cbft_strerror(rc) + " " +
                               cbft_last_error());
    for (size_t j = 0; j < n; j++) out[pos[j]] = (bitmap[j >> 3] >> (j & 7)) & 1;
  }

 private:
  Ed25519Engine() {
    int dev = g_device;
    if (dev < 0) {
      const char* e = std::getenv("CBFT_DEVICE");
      dev = e ? std::atoi(e) : 0;
    }
    int rc = cbft_open(&ctx_, dev, 0);
    if (rc != CBFT_OK)
      throw std::runtime_error(std::string("cbft_open: ") + cbft_strerror(rc) + " " + cbft_last_error());
  }

  void ensureTableLocked() {
    const uint32_t nkeys = (uint32_t)keys_.size() / 32;
    if (nkeys == loaded_ && table_ != CBFT_NO_KEY_TABLE) return;
    uint32_t id;
    int rc = cbft_ed25519_load_keys(ctx_, keys_.data(), nkeys, &id);
    if (rc != CBFT_OK)
      throw std::runtime_error(std::string("cbft_ed25519_load_keys: ") + cbft_strerror(rc) + " " +
                               cbft_last_error());
    if (table_ != CBFT_NO_KEY_TABLE) cbft_ed25519_unload_keys(ctx_, table_);
    table_ = id;
    loaded_ = nkeys;
  }

  cbft_ctx* ctx_ = nullptr;
  std::mutex mu_;                // guards keys_, index_, table_, loaded_
  std::shared_mutex tbl_mu_;     // device table lifetime vs in-flight verifies
  std::vector<uint8_t> keys_;
  std::map<std::string, uint32_t> index_;
  uint32_t table_ = CBFT_NO_KEY_TABLE;
  uint32_t loaded_ = 0;
};

// ---------------------------------------------------------------------------------- verifier
EdDSAVerifier::EdDSAVerifier(const std::string& str_pub_key, KeyFormat fmt) : key_str_(str_pub_key) {
  if (!parseEd25519PublicKey(str_pub_key, fmt, raw_)) throw std::invalid_argument("EdDSAVerifier: bad public key");
  engine_ = Ed25519Engine::get();
  key_index_ = engine_->registerKey(raw_);
}

EdDSAVerifier::~EdDSAVerifier() = default;

bool EdDSAVerifier::verify(const std::string& data, const std::string& sig) const {
  std::vector<VerifyRequest> r{{this, data.data(), data.size(), sig.data(), sig.size()}};
  std::vector<bool> out;
  engine_->verify(r, out);
  return out[0];
}

void EdDSAVerifier::verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
  out.assign(reqs.size(), false);
  if (reqs.empty()) return;
  const EdDSAVerifier* any = nullptr;
  for (auto& r : reqs)
    if ((any = dynamic_cast<const EdDSAVerifier*>(r.verifier))) break;
  if (!any) return;
  any->engine_->verify(reqs, out);
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

}  // namespace concord::util::crypto

// HipRSAVerifier over libcbft_hipcrypto (see hip_crypto.hpp), the mixed-batch dispatcher and
// makeVerifier() / makeSigner().
//
// Reference: concord::util::crypto::RSAVerifier (util/src/crypto_utils.cpp:101-117,155-168):
// Crypto++ RSASS<PKCS1v15, SHA256> keyed from hex DER (X509PublicKey) or PEM.  Key parsing here
// uses the host OpenSSL (d2i_PUBKEY / PEM_read_bio_PUBKEY); every verification runs on the GPU.
#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/pem.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>

#include "cbft_hipcrypto.h"
#include "hip_crypto.hpp"

namespace concord::hip {

namespace {

EVP_PKEY* parsePublicKey(const std::string& s, KeyFormat fmt) {
  if (fmt == KeyFormat::HexaDecimalStrippedFormat) {
    std::vector<uint8_t> der;
    if (!fromHex(s, der) || der.empty()) return nullptr;
    const unsigned char* p = der.data();
    return d2i_PUBKEY(nullptr, &p, (long)der.size());
  }
  BIO* bio = BIO_new_mem_buf(s.data(), (int)s.size());
  if (!bio) return nullptr;
  EVP_PKEY* k = PEM_read_bio_PUBKEY(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  return k;
}

EVP_PKEY* parsePrivateKey(const std::string& s, KeyFormat fmt) {
  if (fmt == KeyFormat::HexaDecimalStrippedFormat) {
    std::vector<uint8_t> der;
    if (!fromHex(s, der) || der.empty()) return nullptr;
    const unsigned char* p = der.data();
    return d2i_AutoPrivateKey(nullptr, &p, (long)der.size());
  }
  BIO* bio = BIO_new_mem_buf(s.data(), (int)s.size());
  if (!bio) return nullptr;
  EVP_PKEY* k = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  return k;
}

// (modulus as 256 big-endian bytes, e) of a 2048-bit RSA key, or false
bool rsaPublicParts(EVP_PKEY* k, uint8_t mod[256], uint32_t* e) {
  if (!k || EVP_PKEY_get_base_id(k) != EVP_PKEY_RSA) return false;
  BIGNUM *bn = nullptr, *be = nullptr;
  bool ok = EVP_PKEY_get_bn_param(k, OSSL_PKEY_PARAM_RSA_N, &bn) == 1 &&
            EVP_PKEY_get_bn_param(k, OSSL_PKEY_PARAM_RSA_E, &be) == 1 && BN_num_bits(bn) == 2048 &&
            BN_num_bits(be) <= 32 && BN_bn2binpad(bn, mod, 256) == 256;
  if (ok) *e = (uint32_t)BN_get_word(be);
  BN_free(bn);
  BN_free(be);
  return ok;
}

[[noreturn]] void fail(const char* what, int rc) {
  throw std::runtime_error(std::string(what) + ": " + cbft_strerror(rc) + " " + cbft_last_error());
}

}  // namespace

// Per-process owner of the GPU context and the device RSA key table (keys deduplicated, the
// table rebuilt lazily before the first batch that needs a newly registered key) — the RSA twin
// of Ed25519Engine in crypto_utils.cpp.
class RsaEngine {
 public:
  static std::shared_ptr<RsaEngine> get() {
    static std::mutex m;
    static std::weak_ptr<RsaEngine> inst;
    std::lock_guard<std::mutex> g(m);
    auto sp = inst.lock();
    if (!sp) {
      sp = std::shared_ptr<RsaEngine>(new RsaEngine());
      inst = sp;
    }
    return sp;
  }
  ~RsaEngine() {
    if (ctx_) cbft_close(ctx_);
  }

  uint32_t registerKey(const uint8_t mod[256], uint32_t e) {
    std::lock_guard<std::mutex> g(mu_);
    std::string k(reinterpret_cast<const char*>(mod), 256);
    k.append(reinterpret_cast<const char*>(&e), 4);
    auto it = index_.find(k);
    if (it != index_.end()) return it->second;
    const uint32_t idx = (uint32_t)exps_.size();
    mods_.insert(mods_.end(), mod, mod + 256);
    exps_.push_back(e);
    index_.emplace(std::move(k), idx);
    return idx;
  }

  // GPU failures become false verdicts (IVerifier never throws for a signature) and are counted
  void verifyNoThrow(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
    try {
      verify(reqs, out);
    } catch (...) {
      gpu_errors_++;
      out.assign(reqs.size(), false);
    }
  }

  void verify(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
    out.assign(reqs.size(), false);
    std::vector<size_t> pos;
    std::vector<const HipRSAVerifier*> ver(reqs.size(), nullptr);
    std::vector<std::string> sigs;  // normalised to 256 bytes (Crypto++ reads any length)
    size_t blob = 0;
    for (size_t i = 0; i < reqs.size(); i++) {
      ver[i] = dynamic_cast<const HipRSAVerifier*>(reqs[i].verifier);
      if (!ver[i]) continue;
      size_t lead = 0;
      while (lead < reqs[i].sigLength && reqs[i].sig[lead] == 0) lead++;
      const size_t sig_len = reqs[i].sigLength - lead;
      if (sig_len > 256) continue;  // see RSAVerifier::verify
      std::string s(256 - sig_len, '\0');
      s.append(reqs[i].sig + lead, sig_len);
      sigs.push_back(std::move(s));
      pos.push_back(i);
      blob += reqs[i].dataLength;
    }
    if (pos.empty()) return;
    const size_t n = pos.size();
    std::vector<uint32_t> kidx(n), len(n);
    std::vector<uint64_t> off(n);
    std::vector<uint8_t> sig(n * 256), msg(blob ? blob : 1), bitmap((n + 7) / 8);
    size_t o = 0;
    for (size_t j = 0; j < n; j++) {
      const VerifyRequest& r = reqs[pos[j]];
      kidx[j] = ver[pos[j]]->engineKeyIndex();
      std::memcpy(&sig[256 * j], sigs[j].data(), 256);
      off[j] = o;
      len[j] = (uint32_t)r.dataLength;
      if (r.dataLength) std::memcpy(&msg[o], r.data, r.dataLength);
      o += r.dataLength;
    }
    std::shared_lock<std::shared_mutex> rd(tbl_mu_);
    while (true) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if (loaded_ == exps_.size() && table_ != kNoTable) break;
      }
      rd.unlock();
      refreshTable();  // builds beside the old table; verifies keep using it meanwhile
      rd.lock();
    }
    const int rc = cbft_rsa_verify_batch(ctx_, table_, kidx.data(), sig.data(), msg.data(), off.data(), len.data(),
                                         n, bitmap.data());
    if (rc != CBFT_OK) fail("cbft_rsa_verify_batch", rc);
    for (size_t j = 0; j < n; j++) out[pos[j]] = (bitmap[j >> 3] >> (j & 7)) & 1;
  }

 private:
  static constexpr uint32_t kNoTable = 0;  // table ids start at 1
  RsaEngine() {
    const char* e = std::getenv("CBFT_DEVICE");
    const int rc = cbft_open(&ctx_, e ? std::atoi(e) : 0, 0);
    if (rc != CBFT_OK) fail("cbft_open", rc);
  }

  // Rebuild the device key table for the keys registered so far WITHOUT blocking verifies: the
  // new table is built while readers keep the old one (tbl_mu_ shared), then swapped in under a
  // short exclusive lock; the old one is unloaded once no reader can hold it.  RSA key records are
  // 1.5 KB each, so a rebuild is cheap (one rsa_keys_kernel launch) and the two tables together
  // stay small; builds are serialised by build_mu_.
  void refreshTable() {
    std::lock_guard<std::mutex> b(build_mu_);
    std::vector<uint8_t> mods;
    std::vector<uint32_t> exps;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (loaded_ == exps_.size() && table_ != kNoTable) return;
      mods = mods_;
      exps = exps_;
    }
    uint32_t id;
    const int rc = cbft_rsa_load_keys(ctx_, mods.data(), exps.data(), (uint32_t)exps.size(), &id);
    if (rc != CBFT_OK) fail("cbft_rsa_load_keys", rc);
    uint32_t old;
    {
      std::unique_lock<std::shared_mutex> wr(tbl_mu_);
      std::lock_guard<std::mutex> g(mu_);
      old = table_;
      table_ = id;
      loaded_ = (uint32_t)exps.size();
    }
    if (old != kNoTable) cbft_rsa_unload_keys(ctx_, old);  // readers now see table_ = id
  }

  cbft_ctx* ctx_ = nullptr;
  std::mutex mu_;             // guards mods_, exps_, index_, table_, loaded_
  std::shared_mutex tbl_mu_;  // device table lifetime vs in-flight verifies
  std::mutex build_mu_;       // one table rebuild at a time
  std::vector<uint8_t> mods_;
  std::vector<uint32_t> exps_;
  std::map<std::string, uint32_t> index_;
  uint32_t table_ = kNoTable;
  uint32_t loaded_ = 0;
  std::atomic<uint64_t> gpu_errors_{0};
};

// ---------------------------------------------------------------------------------- verifier
HipRSAVerifier::HipRSAVerifier(const std::string& str_pub_key, KeyFormat fmt) : key_str_(str_pub_key) {
  EVP_PKEY* k = parsePublicKey(str_pub_key, fmt);
  uint8_t mod[256];
  uint32_t e = 0;
  const bool ok = rsaPublicParts(k, mod, &e);
  EVP_PKEY_free(k);
  if (!ok) throw std::invalid_argument("HipRSAVerifier: not a 2048-bit RSA public key with a 32-bit exponent");
  engine_ = RsaEngine::get();
  key_index_ = engine_->registerKey(mod, e);
}

HipRSAVerifier::~HipRSAVerifier() = default;

bool HipRSAVerifier::verify(const std::string& data, const std::string& sig) const {
  LatencyHistogram::Scope timer(recorders().rsa_verify);
  std::vector<VerifyRequest> r{{this, data.data(), data.size(), sig.data(), sig.size()}};
  std::vector<bool> out;
  engine_->verifyNoThrow(r, out);
  return out[0];
}

void HipRSAVerifier::verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
  out.assign(reqs.size(), false);
  for (auto& r : reqs)
    if (auto v = dynamic_cast<const HipRSAVerifier*>(r.verifier)) {
      v->engine_->verifyNoThrow(reqs, out);
      return;
    }
}

// ---------------------------------------------------------------------------------- dispatch
KeyKind publicKeyKind(const std::string& str_pub_key, KeyFormat fmt) {
  uint8_t raw[32];
  if (parseEd25519PublicKey(str_pub_key, fmt, raw)) return KeyKind::Ed25519;
  EVP_PKEY* k = parsePublicKey(str_pub_key, fmt);
  const KeyKind kind = (k && EVP_PKEY_get_base_id(k) == EVP_PKEY_RSA) ? KeyKind::RSA : KeyKind::Unknown;
  EVP_PKEY_free(k);
  return kind;
}

KeyKind privateKeyKind(const std::string& str_priv_key, KeyFormat fmt) {
  std::vector<uint8_t> seed;
  if (fmt == KeyFormat::HexaDecimalStrippedFormat && fromHex(str_priv_key, seed) && seed.size() == 32)
    return KeyKind::Ed25519;  // an RFC 8032 seed
  EVP_PKEY* k = parsePrivateKey(str_priv_key, fmt);
  const int id = k ? EVP_PKEY_get_base_id(k) : 0;
  EVP_PKEY_free(k);
  return id == EVP_PKEY_ED25519 ? KeyKind::Ed25519 : id == EVP_PKEY_RSA ? KeyKind::RSA : KeyKind::Unknown;
}

std::shared_ptr<IVerifier> makeVerifier(const std::string& str_pub_key, KeyFormat fmt) {
  switch (publicKeyKind(str_pub_key, fmt)) {
    case KeyKind::Ed25519:
      return std::make_shared<HipEdDSAVerifier>(str_pub_key, fmt);
    case KeyKind::RSA:
      return std::make_shared<HipRSAVerifier>(str_pub_key, fmt);
    default:
      throw std::invalid_argument("makeVerifier: neither an Ed25519 nor an RSA public key");
  }
}

std::unique_ptr<ISigner> makeSigner(const std::string& str_priv_key, KeyFormat fmt) {
  switch (privateKeyKind(str_priv_key, fmt)) {
    case KeyKind::Ed25519:
      return std::make_unique<EdDSASigner>(str_priv_key, fmt);
    case KeyKind::RSA:
      return std::make_unique<concord::util::crypto::RSASigner>(str_priv_key, fmt);
    default:
      throw std::invalid_argument("makeSigner: neither an Ed25519 nor an RSA private key");
  }
}

void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out) {
  LatencyHistogram::Scope timer(recorders().verify_batch);
  out.assign(reqs.size(), false);
  bool any_ed = false, any_rsa = false;
  for (size_t i = 0; i < reqs.size(); i++) {
    const IVerifier* v = reqs[i].verifier;
    if (!v) continue;
    if (dynamic_cast<const HipEdDSAVerifier*>(v)) {
      any_ed = true;
    } else if (dynamic_cast<const HipRSAVerifier*>(v)) {
      any_rsa = true;
    } else {
      out[i] = v->verify(std::string(reqs[i].data, reqs[i].dataLength), std::string(reqs[i].sig, reqs[i].sigLength));
    }
  }
  std::vector<bool> part;
  if (any_ed) {
    HipEdDSAVerifier::verifyBatch(reqs, part);
    for (size_t i = 0; i < reqs.size(); i++)
      if (dynamic_cast<const HipEdDSAVerifier*>(reqs[i].verifier)) out[i] = part[i];
  }
  if (any_rsa) {
    HipRSAVerifier::verifyBatch(reqs, part);
    for (size_t i = 0; i < reqs.size(); i++)
      if (dynamic_cast<const HipRSAVerifier*>(reqs[i].verifier)) out[i] = part[i];
  }
}

}  // namespace concord::hip

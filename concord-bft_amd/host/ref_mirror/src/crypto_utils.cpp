// Standalone-build restatement of the reference's RSAVerifier / RSASigner
// (util/src/crypto_utils.cpp:101-168: Crypto++ RSASS<PKCS1v15, SHA256>, keys as hex DER
// X509PublicKey / PKCS8PrivateKey or PEM) on the host CPU, over the host OpenSSL.  Only the
// reference's SigManager base class constructs these (SigManager.cpp:138,146); the product's
// HipSigManager replaces every verifier with a GPU one.  See ../README.md.
#include "crypto_utils.hpp"

#include <openssl/bio.h>
#include <openssl/evp.h>
#include <openssl/pem.h>

#include <stdexcept>
#include <vector>

namespace concord::util::crypto {

namespace {
bool unhex(const std::string& hex, std::vector<uint8_t>& out) {
  auto v = [](char c) {
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
  };
  if (hex.size() % 2) return false;
  out.resize(hex.size() / 2);
  for (size_t i = 0; i < out.size(); i++) {
    const int a = v(hex[2 * i]), b = v(hex[2 * i + 1]);
    if (a < 0 || b < 0) return false;
    out[i] = (uint8_t)(a * 16 + b);
  }
  return true;
}

EVP_PKEY* readKey(const std::string& s, KeyFormat fmt, bool priv) {
  if (fmt == KeyFormat::HexaDecimalStrippedFormat) {
    std::vector<uint8_t> der;
    if (!unhex(s, der) || der.empty()) return nullptr;
    const unsigned char* p = der.data();
    return priv ? d2i_AutoPrivateKey(nullptr, &p, (long)der.size()) : d2i_PUBKEY(nullptr, &p, (long)der.size());
  }
  BIO* bio = BIO_new_mem_buf(s.data(), (int)s.size());
  if (!bio) return nullptr;
  EVP_PKEY* k = priv ? PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr)
                     : PEM_read_bio_PUBKEY(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  return k;
}
}  // namespace

class RSAVerifier::Impl {
 public:
  EVP_PKEY* key = nullptr;
  ~Impl() { EVP_PKEY_free(key); }
};

RSAVerifier::RSAVerifier(const std::string& str_pub_key, KeyFormat fmt)
    : impl_(new Impl), key_str_(str_pub_key) {
  impl_->key = readKey(str_pub_key, fmt, false);
  if (!impl_->key || EVP_PKEY_get_base_id(impl_->key) != EVP_PKEY_RSA)
    throw std::invalid_argument("RSAVerifier: not an RSA public key");
}
RSAVerifier::~RSAVerifier() = default;

bool RSAVerifier::verify(const std::string& data, const std::string& sig) const {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  const bool ok = ctx && EVP_DigestVerifyInit(ctx, nullptr, EVP_sha256(), nullptr, impl_->key) == 1 &&
                  EVP_DigestVerify(ctx, reinterpret_cast<const unsigned char*>(sig.data()), sig.size(),
                                   reinterpret_cast<const unsigned char*>(data.data()), data.size()) == 1;
  EVP_MD_CTX_free(ctx);
  return ok;
}
uint32_t RSAVerifier::signatureLength() const { return (uint32_t)EVP_PKEY_get_size(impl_->key); }

class RSASigner::Impl {
 public:
  EVP_PKEY* key = nullptr;
  ~Impl() { EVP_PKEY_free(key); }
};

RSASigner::RSASigner(const std::string& str_priv_key, KeyFormat fmt) : impl_(new Impl), key_str_(str_priv_key) {
  impl_->key = readKey(str_priv_key, fmt, true);
  if (!impl_->key || EVP_PKEY_get_base_id(impl_->key) != EVP_PKEY_RSA)
    throw std::invalid_argument("RSASigner: not an RSA private key");
}
RSASigner::~RSASigner() = default;

std::string RSASigner::sign(const std::string& data) {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  std::string sig((size_t)EVP_PKEY_get_size(impl_->key), '\0');
  size_t sl = sig.size();
  const bool ok = ctx && EVP_DigestSignInit(ctx, nullptr, EVP_sha256(), nullptr, impl_->key) == 1 &&
                  EVP_DigestSign(ctx, reinterpret_cast<unsigned char*>(&sig[0]), &sl,
                                 reinterpret_cast<const unsigned char*>(data.data()), data.size()) == 1;
  EVP_MD_CTX_free(ctx);
  if (!ok) throw std::runtime_error("RSASigner::sign failed");
  sig.resize(sl);
  return sig;
}
uint32_t RSASigner::signatureLength() const { return (uint32_t)EVP_PKEY_get_size(impl_->key); }

}  // namespace concord::util::crypto

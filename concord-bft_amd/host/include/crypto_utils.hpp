// concord::util::crypto plugin interface (mirror of the reference's
// util/include/crypto_utils.hpp:25-55, same names, argument meaning and error behaviour) plus
// the Ed25519 implementations backed by libcbft_hipcrypto.
//
//   IVerifier / ISigner            crypto_utils.hpp:41-55 (byte-for-byte the same virtual API)
//   KeyFormat                      crypto_utils.hpp:26
//   EdDSAVerifier : IVerifier      new (the "existing EdDSAVerifier" of
//                                  BASELINE.json does not exist in the reference; semantics are
//                                  OpenSSL 3.0.2 Ed25519, util/src/openssl_crypto.cpp:229-253)
//   EdDSASigner : ISigner          new; RFC 8032 signing through the host OpenSSL (not on the
//                                  verify path; the reference signs on the host too)
//
// Batch side-API (the point of the engine): EdDSAVerifier::verifyBatch() verifies many
// (verifier, data, sig) triples in one GPU launch; verdicts are identical to calling verify()
// on each triple.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace concord::util::crypto {

enum class KeyFormat : std::uint16_t { HexaDecimalStrippedFormat, PemFormat };

class IVerifier {
 public:
  virtual bool verify(const std::string& data, const std::string& sig) const = 0;
  virtual uint32_t signatureLength() const = 0;
  virtual ~IVerifier() = default;
  virtual std::string getPubKey() const = 0;
};

class ISigner {
 public:
  virtual std::string sign(const std::string& data) = 0;
  virtual uint32_t signatureLength() const = 0;
  virtual ~ISigner() = default;
  virtual std::string getPrivKey() const = 0;
};

class Ed25519Engine;  // per-GPU owner of the cbft_ctx and of the device key table

// One (verifier, message, signature) triple of a batch.  Pointers are borrowed.
struct VerifyRequest {
  const class EdDSAVerifier* verifier;
  const char* data;
  size_t dataLength;
  const char* sig;
  size_t sigLength;
};

class EdDSAVerifier : public IVerifier {
 public:
  // Throws std::invalid_argument on a malformed key string (the reference's verifiers throw on
  // key parsing, SigManager.cpp:253-259); a well-formed 32-byte key that is not a curve point is
  // accepted here and every signature under it verifies false (OpenSSL does the same).
  EdDSAVerifier(const std::string& str_pub_key, KeyFormat fmt);
  ~EdDSAVerifier() override;
  EdDSAVerifier(const EdDSAVerifier&) = default;

  bool verify(const std::string& data, const std::string& sig) const override;
  uint32_t signatureLength() const override { return 64; }
  std::string getPubKey() const override { return key_str_; }

  const uint8_t* rawKey() const { return raw_; }
  uint32_t engineKeyIndex() const { return key_index_; }

  // Verifies every request in one batch on the GPU; out[i] = verdict of reqs[i].
  static void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

 private:
  std::string key_str_;
  uint8_t raw_[32];
  uint32_t key_index_;
  std::shared_ptr<Ed25519Engine> engine_;
};

class EdDSASigner : public ISigner {
 public:
  // str_priv_key: 32-byte RFC 8032 seed, hex (HexaDecimalStrippedFormat) or PKCS#8 PEM.
  EdDSASigner(const std::string& str_priv_key, KeyFormat fmt);
  ~EdDSASigner() override;
  EdDSASigner(const EdDSASigner&) = delete;  // owns an EVP_PKEY
  EdDSASigner& operator=(const EdDSASigner&) = delete;
  EdDSASigner(EdDSASigner&& o) noexcept : key_str_(std::move(o.key_str_)), pkey_(o.pkey_) { o.pkey_ = nullptr; }
  std::string sign(const std::string& data) override;
  uint32_t signatureLength() const override { return 64; }
  std::string getPrivKey() const override { return key_str_; }
  std::string getPubKeyHex() const;

 private:
  std::string key_str_;
  void* pkey_;  // EVP_PKEY*
};

// Helpers shared by the key parsers (hex <-> bytes, PEM SubjectPublicKeyInfo for Ed25519).
std::string toHex(const uint8_t* p, size_t n);
bool fromHex(const std::string& hex, std::vector<uint8_t>& out);
bool parseEd25519PublicKey(const std::string& s, KeyFormat fmt, uint8_t out[32]);
std::string ed25519PublicKeyToPem(const uint8_t raw[32]);

// Selects the GPU the engine opens (default 0; CBFT_DEVICE env var overrides).  Must be called
// before the first verifier is constructed.
void setEd25519Device(int device);

}  // namespace concord::util::crypto

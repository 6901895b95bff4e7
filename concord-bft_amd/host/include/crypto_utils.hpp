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
//   RSAVerifier : IVerifier        crypto_utils.hpp:84-96 / crypto_utils.cpp:101-117,155-168:
//                                  RSASS<PKCS1v15, SHA256> (Crypto++ 8.2.0 semantics, restated in
//                                  oracle/rsa_ref.py) verified on the GPU (cbft_rsa_*); 2048-bit
//                                  moduli, 32-bit public exponents
//   RSASigner : ISigner            crypto_utils.hpp:98-110; host OpenSSL (not on the verify path)
//
// Batch side-API (the point of the engine): verifyBatch() verifies many (verifier, data, sig)
// triples with one GPU launch per algorithm; verdicts are identical to calling verify() on each
// triple.
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
class RsaEngine;      // same for RSA keys

// One (verifier, message, signature) triple of a batch.  Pointers are borrowed.
struct VerifyRequest {
  const IVerifier* verifier;
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

  // Verifies every request whose verifier is an EdDSAVerifier in one GPU batch; out[i] = verdict
  // of reqs[i] (false for other verifier types).
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

class RSAVerifier : public IVerifier {
 public:
  // str_pub_key: X.509 SubjectPublicKeyInfo, hex DER (HexaDecimalStrippedFormat, what
  // Crypto++'s RSA::PublicKey::Save writes) or PEM.  Throws std::invalid_argument on a key that
  // does not parse, is not RSA, or is not a 2048-bit modulus with a public exponent < 2^32.
  RSAVerifier(const std::string& str_pub_key, KeyFormat fmt);
  ~RSAVerifier() override;
  RSAVerifier(const RSAVerifier&) = default;

  // Crypto++ VerifyMessage semantics: the signature is read as a big-endian integer of any
  // length (leading zero bytes are insignificant).  A signature with more than 256 significant
  // bytes is rejected here (Crypto++ would reduce it mod n; such inputs are never produced by a
  // signer and the reference's callers check signatureLength() first, ClientRequestMsg.cpp:156).
  bool verify(const std::string& data, const std::string& sig) const override;
  uint32_t signatureLength() const override { return 256; }
  std::string getPubKey() const override { return key_str_; }

  uint32_t engineKeyIndex() const { return key_index_; }
  // Verifies every request whose verifier is an RSAVerifier in one GPU batch.
  static void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

 private:
  std::string key_str_;
  uint32_t key_index_;
  std::shared_ptr<RsaEngine> engine_;
};

class RSASigner : public ISigner {
 public:
  // str_priv_key: PKCS#8 / PKCS#1 private key, hex DER or PEM (crypto_utils.cpp:141-152).
  RSASigner(const std::string& str_priv_key, KeyFormat fmt);
  ~RSASigner() override;
  RSASigner(const RSASigner&) = delete;
  RSASigner& operator=(const RSASigner&) = delete;
  std::string sign(const std::string& data) override;
  uint32_t signatureLength() const override { return 256; }
  std::string getPrivKey() const override { return key_str_; }

 private:
  std::string key_str_;
  void* pkey_;  // EVP_PKEY*
};

// Builds the verifier a key string calls for: an Ed25519 key (raw 32 bytes or its
// SubjectPublicKeyInfo) -> EdDSAVerifier, an RSA SubjectPublicKeyInfo -> RSAVerifier; throws
// std::invalid_argument otherwise (SigManager.cpp:138,146,255 construct verifiers per key).
std::shared_ptr<IVerifier> makeVerifier(const std::string& str_pub_key, KeyFormat fmt);

// Verifies a mixed batch: one GPU launch per algorithm; other IVerifier types run verify().
void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

// Helpers shared by the key parsers (hex <-> bytes, PEM SubjectPublicKeyInfo for Ed25519).
std::string toHex(const uint8_t* p, size_t n);
bool fromHex(const std::string& hex, std::vector<uint8_t>& out);
bool parseEd25519PublicKey(const std::string& s, KeyFormat fmt, uint8_t out[32]);
std::string ed25519PublicKeyToPem(const uint8_t raw[32]);

// Number of GPU batches the Ed25519 engine has run for coalesced single verify() calls
// (instrumentation: N concurrent verify() calls complete in fewer than N batches).
uint64_t ed25519EngineBatches();

// Selects the GPU the engine opens (default 0; CBFT_DEVICE env var overrides).  Must be called
// before the first verifier is constructed.
void setEd25519Device(int device);

}  // namespace concord::util::crypto

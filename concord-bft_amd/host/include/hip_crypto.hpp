// GPU-backed implementations of the reference's signature plugin interface
// (concord::util::crypto::IVerifier / ISigner, util/include/crypto_utils.hpp:41-55) over
// libcbft_hipcrypto, in namespace concord::hip so that nothing here redefines a reference symbol:
// this header and hip_verifiers.cpp / hip_rsa.cpp compile against the reference's own
// crypto_utils.hpp (tests/test_reference_boundary.py) or, where the reference cannot be built,
// against the restatement in ref_mirror/include/crypto_utils.hpp.
//
//   HipEdDSAVerifier : IVerifier   Ed25519 (RFC 8032 as OpenSSL 3.0.2 EVP_DigestVerify accepts it,
//                                  util/src/openssl_crypto.cpp:229-253 idiom); the reference has no
//                                  Ed25519, so semantics are pinned by the
//                                  golden vectors
//   HipRSAVerifier : IVerifier     RSASS<PKCS1v15, SHA256> with Crypto++ 8.2.0 semantics
//                                  (util/src/crypto_utils.cpp:101-117), 2048-bit moduli
//   EdDSASigner : ISigner          Ed25519 signing on the host OpenSSL (signing is not the hot path)
//   makeVerifier / makeSigner      the branch SigManager needs where it hard-codes RSAVerifier /
//                                  RSASigner (SigManager.cpp:138,146,255)
//   verifyBatch                    the batch side-API: many (verifier, data, sig) triples, one GPU
//                                  launch per algorithm, verdicts identical to verify() on each
//
// Contract kept from the reference: verify() returns false for any bad signature and never throws
// (openssl_crypto.cpp:247-253); a GPU failure is reported as false and counted
// (engineStats().gpu_errors), never thrown into the pool threads that call verify().  Key parsing
// throws std::invalid_argument.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "crypto_utils.hpp"
#include "latency_histogram.hpp"

namespace concord::hip {

using concord::util::crypto::ISigner;
using concord::util::crypto::IVerifier;
using concord::util::crypto::KeyFormat;

class Ed25519Engine;  // per-process owner of the cbft_ctx and of the device key table
class RsaEngine;      // the same for RSA keys

// One (verifier, message, signature) triple of a batch.  Pointers are borrowed.
struct VerifyRequest {
  const IVerifier* verifier;
  const char* data;
  size_t dataLength;
  const char* sig;
  size_t sigLength;
};

// A registered Ed25519 key slot: copies share the slot, the last copy releases it (a released
// slot is reused by the next new key: rotated client keys do not grow the device table).
class Ed25519KeyRef {
 public:
  Ed25519KeyRef(std::shared_ptr<Ed25519Engine> engine, uint32_t index) : engine_(std::move(engine)), index_(index) {}
  Ed25519KeyRef(const Ed25519KeyRef& o);
  Ed25519KeyRef& operator=(const Ed25519KeyRef&) = delete;
  ~Ed25519KeyRef();
  uint32_t index() const { return index_; }
  Ed25519Engine& engine() const { return *engine_; }

 private:
  std::shared_ptr<Ed25519Engine> engine_;
  uint32_t index_;
};

class HipEdDSAVerifier : public IVerifier {
 public:
  // Raw 32-byte key or its SubjectPublicKeyInfo (RFC 8410), hex or PEM.  Throws
  // std::invalid_argument on a malformed key; a well-formed 32-byte string that is not a curve
  // point is accepted and every signature under it verifies false (as OpenSSL does).
  HipEdDSAVerifier(const std::string& str_pub_key, KeyFormat fmt);
  ~HipEdDSAVerifier() override;
  HipEdDSAVerifier(const HipEdDSAVerifier&) = default;

  bool verify(const std::string& data, const std::string& sig) const override;
  uint32_t signatureLength() const override { return 64; }
  std::string getPubKey() const override { return key_str_; }

  const uint8_t* rawKey() const { return raw_; }
  uint32_t engineKeyIndex() const { return key_.index(); }
  // Verifies every request whose verifier is a HipEdDSAVerifier in one GPU batch; out[i] =
  // verdict of reqs[i] (false for other verifier types).
  static void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

 private:
  std::string key_str_;
  uint8_t raw_[32];
  Ed25519KeyRef key_;
};

class HipRSAVerifier : public IVerifier {
 public:
  // X.509 SubjectPublicKeyInfo, hex DER (HexaDecimalStrippedFormat, as Crypto++'s
  // RSA::PublicKey::Save writes it) or PEM.  Throws std::invalid_argument unless it is a 2048-bit
  // RSA key with a public exponent < 2^32.
  HipRSAVerifier(const std::string& str_pub_key, KeyFormat fmt);
  ~HipRSAVerifier() override;
  HipRSAVerifier(const HipRSAVerifier&) = default;

  // Crypto++ VerifyMessage semantics: the signature is a big-endian integer of any length
  // (leading zero bytes are insignificant); more than 256 significant bytes is rejected (the
  // reference's callers check signatureLength() first, ClientRequestMsg.cpp:156).
  bool verify(const std::string& data, const std::string& sig) const override;
  uint32_t signatureLength() const override { return 256; }
  std::string getPubKey() const override { return key_str_; }

  uint32_t engineKeyIndex() const { return key_index_; }
  static void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

 private:
  std::string key_str_;
  uint32_t key_index_;
  std::shared_ptr<RsaEngine> engine_;
};

class EdDSASigner : public ISigner {
 public:
  // 32-byte RFC 8032 seed in hex, or a PKCS#8 PEM private key
  EdDSASigner(const std::string& str_priv_key, KeyFormat fmt);
  ~EdDSASigner() override;
  EdDSASigner(const EdDSASigner&) = delete;
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

enum class KeyKind { Ed25519, RSA, Unknown };
// What a public-key string holds (Ed25519: raw 32 bytes or its SubjectPublicKeyInfo; RSA: an
// RSA SubjectPublicKeyInfo), without registering it anywhere.
KeyKind publicKeyKind(const std::string& str_pub_key, KeyFormat fmt);
KeyKind privateKeyKind(const std::string& str_priv_key, KeyFormat fmt);

// The verifier a key calls for: Ed25519 -> HipEdDSAVerifier, RSA -> HipRSAVerifier; throws
// std::invalid_argument otherwise.
std::shared_ptr<IVerifier> makeVerifier(const std::string& str_pub_key, KeyFormat fmt);
// Ed25519 seed -> EdDSASigner; an RSA private key -> concord::util::crypto::RSASigner (the
// reference's own class); throws std::invalid_argument otherwise.
std::unique_ptr<ISigner> makeSigner(const std::string& str_priv_key, KeyFormat fmt);

// A mixed batch: one GPU launch per algorithm; any other IVerifier runs its own verify().
void verifyBatch(const std::vector<VerifyRequest>& reqs, std::vector<bool>& out);

// Key-string helpers shared by the parsers.
std::string toHex(const uint8_t* p, size_t n);
bool fromHex(const std::string& hex, std::vector<uint8_t>& out);
bool parseEd25519PublicKey(const std::string& s, KeyFormat fmt, uint8_t out[32]);
std::string ed25519PublicKeyToPem(const uint8_t raw[32]);

// Engine instrumentation.
struct EngineStats {
  uint64_t batches;      // GPU batches run for verify() / verifyBatch()
  uint64_t items;        // signatures in them
  uint64_t gpu_errors;   // batches whose GPU call failed (their signatures verified false)
  uint32_t live_keys;    // Ed25519 key slots in use
  uint32_t table_keys;   // Ed25519 key slots on the device (live + free for reuse)
};
EngineStats ed25519EngineStats();

// Selects the GPU the engines open (default 0; $CBFT_DEVICE overrides).  Call before the first
// verifier is constructed.
void setEd25519Device(int device);

}  // namespace concord::hip

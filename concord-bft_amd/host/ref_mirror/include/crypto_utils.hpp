// Standalone-build restatement of the reference's plugin-interface header
// util/include/crypto_utils.hpp:25-110: KeyFormat, IVerifier, ISigner (byte-for-byte the same
// virtual API) and the RSAVerifier / RSASigner the reference's SigManager constructs
// (SigManager.cpp:138,146,255).  The product code (hip_crypto.hpp, hip_sig_manager.hpp) includes
// "crypto_utils.hpp" and compiles unchanged against this file or against the reference's own
// (tests/test_reference_boundary.py compiles it against /root/reference); see ../README.md.
#pragma once

#include <cstdint>
#include <memory>
#include <string>

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

// RSASS<PKCS1v15, SHA256> on the host CPU (crypto_utils.cpp:101-168 of the reference; here over
// the host OpenSSL): X.509 SubjectPublicKeyInfo / PKCS#8 keys, hex DER or PEM.
class RSAVerifier : public IVerifier {
 public:
  RSAVerifier(const std::string& str_pub_key, KeyFormat fmt);
  bool verify(const std::string& data, const std::string& sig) const override;
  uint32_t signatureLength() const override;
  std::string getPubKey() const override { return key_str_; }
  ~RSAVerifier();

 private:
  class Impl;
  std::unique_ptr<Impl> impl_;
  std::string key_str_;
};

class RSASigner : public ISigner {
 public:
  RSASigner(const std::string& str_priv_key, KeyFormat fmt);
  std::string sign(const std::string& data) override;
  uint32_t signatureLength() const override;
  std::string getPrivKey() const override { return key_str_; }
  ~RSASigner();

 private:
  class Impl;
  std::unique_ptr<Impl> impl_;
  std::string key_str_;
};
}  // namespace concord::util::crypto

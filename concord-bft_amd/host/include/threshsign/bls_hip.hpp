// BLS BN-P254 threshold signatures over libcbft_hipcrypto: the objects a Cryptosystem subclass
// returns from createThresholdVerifier / createThresholdSigner (ThresholdSignaturesTypes.h:280,294
// of the reference), with the reference's class names and behaviour:
//
//   BlsThresholdVerifier   threshsign/src/bls/relic/BlsThresholdVerifier.cpp:26-96
//   BlsMultisigVerifier    threshsign/src/bls/relic/BlsMultisigVerifier.cpp:27-105
//   BlsThresholdAccumulator, BlsMultisigAccumulator, and the k = n - 1 "almost multisig" case
//                          ThresholdAccumulatorBase.cpp:14-147, BlsAccumulatorBase.cpp:33-84,
//                          BlsThresholdAccumulator.cpp:29-55, BlsMultisigAccumulator.cpp:30-65,
//                          BlsAlmostMultisigAccumulator.cpp:28-46
//   BlsThresholdSigner     threshsign/src/bls/relic/BlsThresholdSigner.cpp:25-47
//
// Difference by design: where the reference verifies pending shares one pairing pair at a time
// (ThresholdAccumulatorBase::verifyPendingShares), this accumulator verifies all pending shares
// in one GPU launch and then applies the reference's walk (id order, stop at reqSigners, the
// rest of the invalid ones reported), so valid/invalid sets are identical.
//
// Key encodings: PK and vk_i are 65-byte compressed G2 points as hex strings (130 characters,
// ThresholdSignaturesTypes.cpp:220-228); share secret keys are decimal strings
// (BlsSecretKey.h:37, BNT::toString base 10).  The G2/G1 encodings are RELIC's (Montgomery-form
// y parity), pinned by the reference's own key files (tests/golden/relic_bls_keys.json).
#pragma once

#include <array>
#include <memory>
#include <string>
#include <vector>

#include "threshsign/IThresholdAccumulator.h"
#include "threshsign/IThresholdSigner.h"
#include "threshsign/IThresholdVerifier.h"
#include "threshsign/VectorOfShares.h"

namespace BLS {
namespace Hip {

class BlsEngine;  // per-process owner of a cbft_ctx (device from CBFT_DEVICE, default 0)

class BlsPublicKey : public IShareVerificationKey {
 public:
  BlsPublicKey() = default;
  explicit BlsPublicKey(const std::string& hex);  // throws std::invalid_argument if not 130 hex
  std::string toString() const override { return hex_; }
  const std::array<uint8_t, 65>& bytes() const { return raw_; }
  bool operator==(const BlsPublicKey& o) const { return raw_ == o.raw_; }

 private:
  std::string hex_;
  std::array<uint8_t, 65> raw_{};
};

class BlsSecretKey : public IShareSecretKey {
 public:
  explicit BlsSecretKey(const std::string& decimal);  // throws std::invalid_argument
  std::string toString() const override { return dec_; }
  const std::array<uint8_t, 32>& bytes() const { return be_; }  // big-endian

 private:
  std::string dec_;
  std::array<uint8_t, 32> be_{};
};

class BlsThresholdVerifier : public IThresholdVerifier {
 public:
  // vkHex: numSigners share verification keys vk_1..vk_n (the reference's vector has a dummy
  // entry 0; here index 0 is vk_1).
  BlsThresholdVerifier(const std::string& pkHex, NumSharesType reqSigners, NumSharesType numSigners,
                       const std::vector<std::string>& vkHex);
  ~BlsThresholdVerifier() override;

  IThresholdAccumulator* newAccumulator(bool withShareVerification) const override;
  bool verify(const char* msg, int msgLen, const char* sig, int sigLen) const override;
  int requiredLengthForSignedData() const override { return 33; }
  const IPublicKey& getPublicKey() const override { return pk_; }
  const IShareVerificationKey& getShareVerificationKey(ShareID signer) const override;

  NumSharesType getNumRequiredShares() const { return req_; }
  NumSharesType getNumTotalShares() const { return num_; }
  uint32_t keysetId() const { return keyset_; }
  const std::shared_ptr<BlsEngine>& engine() const { return engine_; }

 protected:
  BlsPublicKey pk_;
  std::vector<BlsPublicKey> vks_;
  NumSharesType req_, num_;
  std::shared_ptr<BlsEngine> engine_;
  uint32_t keyset_ = 0;
};

class BlsMultisigVerifier : public BlsThresholdVerifier {
 public:
  // PK is the sum of the vk_i (BlsMultisigVerifier.cpp:33-38); pkHex is not needed.
  BlsMultisigVerifier(NumSharesType reqSigners, NumSharesType numSigners, const std::vector<std::string>& vkHex);
  IThresholdAccumulator* newAccumulator(bool withShareVerification) const override;
  // n-of-n: 33 bytes; otherwise 33 + 256 (signer bitmap) (BlsMultisigVerifier.cpp:67-73)
  int requiredLengthForSignedData() const override;
  // throws std::runtime_error on a wrong-size k-of-n signature (BlsMultisigVerifier.cpp:77)
  bool verify(const char* msg, int msgLen, const char* sig, int sigLen) const override;
};

// Accumulator state machine of ThresholdAccumulatorBase (pending / valid / invalid shares).
class BlsAccumulatorBase : public IThresholdAccumulator {
 public:
  BlsAccumulatorBase(const BlsThresholdVerifier& v, NumSharesType reqSigners, bool withShareVerification);
  int add(const char* sigShareWithId, int len) override;
  void setExpectedDigest(const unsigned char* msg, int len) override;
  bool hasShareVerificationEnabled() const override { return verify_; }
  int getNumValidShares() const override;
  std::set<ShareID> getInvalidShareIds() const override { return invalid_; }
  int addNumById(ShareID signer, const uint8_t* share33);

 protected:
  using Share = std::array<uint8_t, 33>;
  bool hasExpectedDigest() const { return !digest_.empty(); }
  void verifyPendingShares();
  // valid shares as 37-byte (id || point) records in id order
  std::vector<uint8_t> validRecords() const;

  const BlsThresholdVerifier& v_;
  NumSharesType req_, num_;
  bool verify_;
  std::vector<uint8_t> digest_;
  std::vector<Share> pending_, valid_;
  VectorOfShares pendingBits_, validBits_;
  std::set<ShareID> invalid_;
};

class BlsThresholdAccumulator : public BlsAccumulatorBase {
 public:
  using BlsAccumulatorBase::BlsAccumulatorBase;
  // sum lambda_i sigma_i over the valid shares -> 33 bytes (throws std::runtime_error if
  // threshSigLen < 33 or a share does not decode)
  void getFullSignedData(char* outThreshSig, int threshSigLen) override;
};

class BlsMultisigAccumulator : public BlsAccumulatorBase {
 public:
  using BlsAccumulatorBase::BlsAccumulatorBase;
  // sum sigma_i -> 33 bytes, || 256-byte signer bitmap when reqSigners != numSigners
  void getFullSignedData(char* outThreshSig, int threshSigLen) override;
};

class BlsThresholdSigner : public IThresholdSigner {
 public:
  // vkHex empty: the verification key is derived from the secret key on the GPU (sk * g2), as
  // the reference's constructor does (BlsThresholdSigner.cpp:25)
  BlsThresholdSigner(ShareID id, const std::string& secretKeyDecimal, const std::string& vkHex = "");
  int requiredLengthForSignedData() const override { return 37; }
  // outSig = 4-byte big-endian id || sk * H(hash); throws std::runtime_error if outSigLen < 37
  void signData(const char* hash, int hashLen, char* outSig, int outSigLen) override;
  const IShareSecretKey& getShareSecretKey() const override { return sk_; }
  const IShareVerificationKey& getShareVerificationKey() const override { return vk_; }

 private:
  ShareID id_;
  BlsSecretKey sk_;
  BlsPublicKey vk_;
  std::shared_ptr<BlsEngine> engine_;
};

}  // namespace Hip
}  // namespace BLS

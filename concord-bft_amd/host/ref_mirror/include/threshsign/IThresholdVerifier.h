// Mirror of threshsign/include/threshsign/IThresholdVerifier.h:23-38 (same virtual API).
#pragma once

#include <cstdint>

#include "IPublicKey.h"
#include "IThresholdAccumulator.h"
#include "ThresholdSignaturesTypes.h"

class IThresholdVerifier {
 public:
  virtual ~IThresholdVerifier() = default;

  // Caller owns the returned accumulator (CollectorOfThresholdSignatures.hpp:377 wraps it).
  virtual IThresholdAccumulator* newAccumulator(bool withShareVerification) const = 0;
  virtual bool verify(const char* msg, int msgLen, const char* sig, int sigLen) const = 0;
  virtual int requiredLengthForSignedData() const = 0;
  virtual const IPublicKey& getPublicKey() const = 0;
  virtual const IShareVerificationKey& getShareVerificationKey(ShareID signer) const = 0;

  static const uint32_t maxSize_ = 2048;
  static uint32_t maxSize() { return maxSize_; }
};

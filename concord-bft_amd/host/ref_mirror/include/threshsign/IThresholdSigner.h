// Mirror of threshsign/include/threshsign/IThresholdSigner.h:19-30 (same virtual API).
#pragma once

#include <cstdint>

#include "IPublicKey.h"

class IThresholdSigner {
 public:
  virtual ~IThresholdSigner() = default;
  virtual int requiredLengthForSignedData() const = 0;
  virtual void signData(const char* hash, int hashLen, char* outSig, int outSigLen) = 0;
  virtual const IShareSecretKey& getShareSecretKey() const = 0;
  virtual const IShareVerificationKey& getShareVerificationKey() const = 0;

  static const uint32_t maxSize_ = 2048;
  static uint32_t maxSize() { return maxSize_; }
};

// Mirror of threshsign/include/threshsign/IThresholdAccumulator.h:22-72 (same virtual API).
#pragma once

#include <set>

#include "ThresholdSignaturesTypes.h"

class IThresholdAccumulator {
 public:
  virtual ~IThresholdAccumulator() {}

  // Adds a share (4-byte big-endian signer id || signature share); returns the number of valid
  // shares (or of pending shares while verification waits for the digest).
  virtual int add(const char* sigShareWithId, int len) = 0;
  // Sets the message the shares sign; throws std::runtime_error if called again with another one.
  virtual void setExpectedDigest(const unsigned char* msg, int len) = 0;
  virtual bool hasShareVerificationEnabled() const = 0;
  virtual int getNumValidShares() const = 0;
  virtual std::set<ShareID> getInvalidShareIds() const = 0;
  // Computes the combined signature into outThreshSig (threshSigLen bytes of capacity).
  virtual void getFullSignedData(char* outThreshSig, int threshSigLen) = 0;
};

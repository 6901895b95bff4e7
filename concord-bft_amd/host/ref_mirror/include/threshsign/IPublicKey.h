// Mirror of threshsign/include/threshsign/IPublicKey.h:18-35 and ISecretKey.h:17-32.
#pragma once

#include <string>

class IPublicKey {
 public:
  virtual ~IPublicKey() {}
  virtual std::string toString() const = 0;
};

class IShareVerificationKey : public IPublicKey {
 public:
  virtual ~IShareVerificationKey() {}
};

class ISecretKey {
 public:
  virtual ~ISecretKey() {}
  virtual std::string toString() const = 0;
};

class IShareSecretKey : public ISecretKey {
 public:
  virtual ~IShareSecretKey() {}
};

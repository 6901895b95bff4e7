// Signer-id set, ids 1..MAX_NUM_OF_SHARES (mirror of threshsign/include/threshsign/
// VectorOfShares.h:28-102; serialization VectorOfShares.cpp:136-188: 256 bytes, bit (id - 1)
// LSB-first).
#pragma once

#include <bitset>

#include "ThresholdSignaturesTypes.h"

class VectorOfShares {
 public:
  void add(ShareID e);
  void remove(ShareID e);
  bool contains(ShareID e) const;
  int count() const { return size_; }
  void clear() {
    data_.reset();
    size_ = 0;
  }
  // iteration: for (id = first(); !isEnd(id); id = next(id))
  ShareID first() const { return next(0); }
  ShareID next(ShareID cur) const;
  bool isEnd(ShareID e) const { return e > MAX_NUM_OF_SHARES; }
  ShareID findFirstGap() const;  // smallest id not in the set (MAX_NUM_OF_SHARES + 1 if full)
  bool operator==(const VectorOfShares& v) const { return data_ == v.data_; }
  bool operator!=(const VectorOfShares& v) const { return data_ != v.data_; }

  // throws std::runtime_error if capacity < getByteCount()
  void toBytes(unsigned char* buf, int capacity) const;
  void fromBytes(const unsigned char* buf, int len);
  static int getByteCount() { return (MAX_NUM_OF_SHARES + 7) / 8; }

 private:
  std::bitset<MAX_NUM_OF_SHARES> data_;  // bit id-1
  int size_ = 0;
};

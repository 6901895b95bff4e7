// Standalone-build restatement of the reference's VectorOfShares (threshsign/src/
// VectorOfShares.cpp:25-188; serialization :136-188: 256 bytes, bit (id - 1) LSB-first).  Only
// for builds without the reference's threshsign library; see ref_mirror/README.md.
#include "threshsign/VectorOfShares.h"

#include <cstring>
#include <stdexcept>

void VectorOfShares::add(ShareID e) {
  if (e < 1 || e > MAX_NUM_OF_SHARES) throw std::out_of_range("VectorOfShares: id out of range");
  if (!data_[(size_t)e - 1]) {
    data_[(size_t)e - 1] = true;
    size_++;
  }
}
void VectorOfShares::remove(ShareID e) {
  if (e < 1 || e > MAX_NUM_OF_SHARES) throw std::out_of_range("VectorOfShares: id out of range");
  if (data_[(size_t)e - 1]) {
    data_[(size_t)e - 1] = false;
    size_--;
  }
}
bool VectorOfShares::contains(ShareID e) const {
  return e >= 1 && e <= MAX_NUM_OF_SHARES && data_[(size_t)e - 1];
}
ShareID VectorOfShares::next(ShareID cur) const {
  for (size_t i = (size_t)(cur < 0 ? 0 : cur); i < data_.size(); i++)
    if (data_[i]) return (ShareID)(i + 1);
  return MAX_NUM_OF_SHARES + 1;
}
ShareID VectorOfShares::findFirstGap() const {
  for (size_t i = 0; i < data_.size(); i++)
    if (!data_[i]) return (ShareID)(i + 1);
  return MAX_NUM_OF_SHARES + 1;
}
void VectorOfShares::toBytes(unsigned char* buf, int capacity) const {
  const int n = getByteCount();
  if (n > capacity) throw std::runtime_error("Need more buffer space to serialize VectorOfShares");
  std::memset(buf, 0, (size_t)n);
  for (size_t i = 0; i < data_.size(); i++)
    if (data_[i]) buf[i / 8] = (unsigned char)(buf[i / 8] | (1u << (i % 8)));
}
void VectorOfShares::fromBytes(const unsigned char* buf, int len) {
  clear();
  for (int b = 0; b < len && b < getByteCount(); b++)
    for (int c = 0; c < 8; c++)
      if ((buf[b] >> c) & 1) add(b * 8 + c + 1);
}

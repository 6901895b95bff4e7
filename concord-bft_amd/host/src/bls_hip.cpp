// BLS::Hip threshold verifier / accumulator / signer over libcbft_hipcrypto (see bls_hip.hpp).
#include "threshsign/bls_hip.hpp"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>

#include "cbft_hipcrypto.h"

namespace BLS {
namespace Hip {

// ------------------------------------------------------------------------------ engine
class BlsEngine {
 public:
  static std::shared_ptr<BlsEngine> get() {
    static std::mutex m;
    static std::weak_ptr<BlsEngine> inst;
    std::lock_guard<std::mutex> g(m);
    auto sp = inst.lock();
    if (!sp) {
      sp = std::shared_ptr<BlsEngine>(new BlsEngine());
      inst = sp;
    }
    return sp;
  }
  ~BlsEngine() {
    if (ctx_) cbft_close(ctx_);
  }
  cbft_ctx* ctx() const { return ctx_; }

 private:
  BlsEngine() {
    const char* d = std::getenv("CBFT_DEVICE");
    int rc = cbft_open(&ctx_, d ? std::atoi(d) : 0, 0);
    if (rc) throw std::runtime_error(std::string("cbft_open: ") + cbft_strerror(rc) + " " + cbft_last_error());
  }
  cbft_ctx* ctx_ = nullptr;
};

static void check(int rc, const char* what) {
  if (rc) throw std::runtime_error(std::string(what) + ": " + cbft_strerror(rc) + " " + cbft_last_error());
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// ------------------------------------------------------------------------------ keys
BlsPublicKey::BlsPublicKey(const std::string& hex) : hex_(hex) {
  if (hex.size() != 130) throw std::invalid_argument("BLS G2 key: expected 130 hex characters");
  for (size_t i = 0; i < 65; i++) {
    int a = hexval(hex[2 * i]), b = hexval(hex[2 * i + 1]);
    if (a < 0 || b < 0) throw std::invalid_argument("BLS G2 key: not hex");
    raw_[i] = (uint8_t)(a * 16 + b);
  }
}

static std::string toHex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

BlsSecretKey::BlsSecretKey(const std::string& decimal) : dec_(decimal) {
  if (decimal.empty()) throw std::invalid_argument("BLS secret key: empty");
  for (char ch : decimal) {  // be_ = be_ * 10 + digit, big-endian bytes
    if (ch < '0' || ch > '9') throw std::invalid_argument("BLS secret key: not a decimal number");
    unsigned carry = (unsigned)(ch - '0');
    for (int i = 31; i >= 0; i--) {
      unsigned v = be_[i] * 10u + carry;
      be_[i] = (uint8_t)v;
      carry = v >> 8;
    }
    if (carry) throw std::invalid_argument("BLS secret key: exceeds 256 bits");
  }
}

// ------------------------------------------------------------------------------ verifiers
BlsThresholdVerifier::BlsThresholdVerifier(const std::string& pkHex, NumSharesType reqSigners,
                                           NumSharesType numSigners, const std::vector<std::string>& vkHex)
    : req_(reqSigners), num_(numSigners) {
  if (numSigners < 1 || numSigners > MAX_NUM_OF_SHARES || reqSigners < 1 || reqSigners > numSigners)
    throw std::invalid_argument("BLS verifier: need 1 <= reqSigners <= numSigners <= 2048");
  if (vkHex.size() != (size_t)numSigners) throw std::invalid_argument("BLS verifier: need numSigners keys");
  if (!pkHex.empty()) pk_ = BlsPublicKey(pkHex);
  vks_.reserve(vkHex.size());
  std::vector<uint8_t> vk65(65 * vkHex.size());
  for (size_t i = 0; i < vkHex.size(); i++) {
    vks_.emplace_back(vkHex[i]);
    std::memcpy(&vk65[65 * i], vks_.back().bytes().data(), 65);
  }
  engine_ = BlsEngine::get();
  check(cbft_bls_load_keys(engine_->ctx(), pk_.bytes().data(), vk65.data(), (uint32_t)numSigners, &keyset_),
        "cbft_bls_load_keys");
}

BlsThresholdVerifier::~BlsThresholdVerifier() {
  if (engine_) (void)cbft_bls_unload_keys(engine_->ctx(), keyset_);
}

const IShareVerificationKey& BlsThresholdVerifier::getShareVerificationKey(ShareID signer) const {
  if (signer < 1 || signer > num_) throw std::out_of_range("BLS verifier: signer id out of range");
  return vks_[(size_t)signer - 1];
}

IThresholdAccumulator* BlsThresholdVerifier::newAccumulator(bool withShareVerification) const {
  // k = n - 1 takes the reference's "almost multisig" accumulator, which never verifies shares
  // (BlsThresholdVerifier.cpp:61-67); its precomputed coefficients equal the Lagrange ones.
  if (req_ == num_ - 1) return new BlsThresholdAccumulator(*this, req_, false);
  return new BlsThresholdAccumulator(*this, req_, withShareVerification);
}

bool BlsThresholdVerifier::verify(const char* msg, int msgLen, const char* sig, int sigLen) const {
  if (!msg || msgLen < 0 || !sig || sigLen != 33) return false;
  int ok = 0;
  check(cbft_bls_verify(engine_->ctx(), keyset_, reinterpret_cast<const uint8_t*>(msg), (uint32_t)msgLen,
                        reinterpret_cast<const uint8_t*>(sig), &ok),
        "cbft_bls_verify");
  return ok != 0;
}

static std::vector<uint8_t> allSigners(NumSharesType n) {
  VectorOfShares v;
  for (ShareID i = 1; i <= n; i++) v.add(i);
  std::vector<uint8_t> b((size_t)VectorOfShares::getByteCount());
  v.toBytes(b.data(), (int)b.size());
  return b;
}

BlsMultisigVerifier::BlsMultisigVerifier(NumSharesType reqSigners, NumSharesType numSigners,
                                         const std::vector<std::string>& vkHex)
    : BlsThresholdVerifier("", reqSigners, numSigners, vkHex) {
  if (req_ == num_) {  // PK = sum of all vk_i; reload the key set with it in slot 0
    uint8_t pk65[65];
    std::vector<uint8_t> all = allSigners(num_);
    check(cbft_bls_sum_keys(engine_->ctx(), keyset_, all.data(), pk65), "cbft_bls_sum_keys");
    pk_ = BlsPublicKey(toHex(pk65, 65));
    std::vector<uint8_t> vk65(65 * vks_.size());
    for (size_t i = 0; i < vks_.size(); i++) std::memcpy(&vk65[65 * i], vks_[i].bytes().data(), 65);
    uint32_t id = 0;
    check(cbft_bls_load_keys(engine_->ctx(), pk65, vk65.data(), (uint32_t)num_, &id), "cbft_bls_load_keys");
    (void)cbft_bls_unload_keys(engine_->ctx(), keyset_);
    keyset_ = id;
  }
}

IThresholdAccumulator* BlsMultisigVerifier::newAccumulator(bool withShareVerification) const {
  return new BlsMultisigAccumulator(*this, req_, withShareVerification);
}

int BlsMultisigVerifier::requiredLengthForSignedData() const {
  return 33 + (req_ != num_ ? VectorOfShares::getByteCount() : 0);
}

bool BlsMultisigVerifier::verify(const char* msg, int msgLen, const char* sig, int sigLen) const {
  if (req_ == num_) return BlsThresholdVerifier::verify(msg, msgLen, sig, 33);
  if (sigLen != requiredLengthForSignedData()) throw std::runtime_error("Signature does not have the right size");
  if (!msg || msgLen < 0 || !sig) return false;
  VectorOfShares signers;
  signers.fromBytes(reinterpret_cast<const unsigned char*>(sig) + 33, VectorOfShares::getByteCount());
  if (signers.count() < req_) return false;
  for (ShareID id = signers.first(); !signers.isEnd(id); id = signers.next(id))
    if (id > num_) return false;  // no such signer (the reference would index past its key vector)
  int ok = 0;
  check(cbft_bls_verify_multisig(engine_->ctx(), keyset_, reinterpret_cast<const uint8_t*>(msg), (uint32_t)msgLen,
                                 reinterpret_cast<const uint8_t*>(sig),
                                 reinterpret_cast<const uint8_t*>(sig) + 33, &ok),
        "cbft_bls_verify_multisig");
  return ok != 0;
}

// ------------------------------------------------------------------------------ accumulators
BlsAccumulatorBase::BlsAccumulatorBase(const BlsThresholdVerifier& v, NumSharesType reqSigners,
                                       bool withShareVerification)
    : v_(v),
      req_(reqSigners),
      num_(v.getNumTotalShares()),
      verify_(withShareVerification),
      pending_((size_t)num_ + 1),
      valid_((size_t)num_ + 1) {}

int BlsAccumulatorBase::getNumValidShares() const {
  return (!verify_ || hasExpectedDigest()) ? validBits_.count() : 0;
}

// BlsSigshareParser (BlsAccumulatorBase.cpp:33-43): 4-byte big-endian id, then the G1 point.
int BlsAccumulatorBase::add(const char* sigShare, int len) {
  if (!sigShare || len < 4) throw std::invalid_argument("BLS share: shorter than its id");
  const uint8_t* b = reinterpret_cast<const uint8_t*>(sigShare);
  const ShareID id = (ShareID)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
  uint8_t s[33];
  if (len - 4 == 33) {
    std::memcpy(s, b + 4, 33);
  } else {
    std::memset(s, 0xff, 33);  // wrong length: a point that never decodes (RELIC would error)
  }
  return addNumById(id, s);
}

static void putRecord(std::vector<uint8_t>& out, ShareID id, const uint8_t* s33) {
  out.push_back((uint8_t)(id >> 24));
  out.push_back((uint8_t)(id >> 16));
  out.push_back((uint8_t)(id >> 8));
  out.push_back((uint8_t)id);
  out.insert(out.end(), s33, s33 + 33);
}

// ThresholdAccumulatorBase::addNumById (ThresholdAccumulatorBase.cpp:87-147)
int BlsAccumulatorBase::addNumById(ShareID signer, const uint8_t* share33) {
  if (signer < 1 || signer > num_) {  // reference: debug assert; here the share is refused
    invalid_.insert(signer);
    return (verify_ && !hasExpectedDigest()) ? pendingBits_.count() : validBits_.count();
  }
  const size_t idx = (size_t)signer;
  if (verify_ && !hasExpectedDigest()) {
    if (!pendingBits_.contains(signer)) {
      std::memcpy(pending_[idx].data(), share33, 33);
      pendingBits_.add(signer);
    }
    return pendingBits_.count();
  }
  if (validBits_.count() == req_) return validBits_.count();
  if (!validBits_.contains(signer)) {
    bool ok = true;
    if (verify_) {
      std::vector<uint8_t> rec;
      putRecord(rec, signer, share33);
      uint8_t bit = 0;
      check(cbft_bls_verify_shares(v_.engine()->ctx(), v_.keysetId(), digest_.data(), (uint32_t)digest_.size(),
                                   rec.data(), 1, &bit),
            "cbft_bls_verify_shares");
      ok = (bit & 1) != 0;
    }
    if (ok) {
      std::memcpy(valid_[idx].data(), share33, 33);
      validBits_.add(signer);
    }
  }
  return validBits_.count();
}

// ThresholdAccumulatorBase::setExpectedDigest (ThresholdAccumulatorBase.cpp:19-57)
void BlsAccumulatorBase::setExpectedDigest(const unsigned char* msg, int len) {
  if (!msg || len <= 0) throw std::invalid_argument("setExpectedDigest: empty digest");
  if (!hasExpectedDigest()) {
    digest_.assign(msg, msg + len);
    if (verify_) verifyPendingShares();
    return;
  }
  if ((int)digest_.size() != len) throw std::runtime_error("Cannot reset expected digest with different length");
  if (std::memcmp(digest_.data(), msg, (size_t)len) != 0)
    throw std::runtime_error("Cannot reset expected digest to a different one");
}

// All pending shares in one launch, then the reference's walk (ThresholdAccumulatorBase.cpp:59-85):
// id order, stop once reqSigners are valid, failed ones before that point reported invalid.
void BlsAccumulatorBase::verifyPendingShares() {
  std::vector<ShareID> ids;
  std::vector<uint8_t> recs;
  for (ShareID id = pendingBits_.first(); !pendingBits_.isEnd(id); id = pendingBits_.next(id)) {
    ids.push_back(id);
    putRecord(recs, id, pending_[(size_t)id].data());
  }
  if (!ids.empty()) {
    std::vector<uint8_t> bits((ids.size() + 7) / 8);
    check(cbft_bls_verify_shares(v_.engine()->ctx(), v_.keysetId(), digest_.data(), (uint32_t)digest_.size(),
                                 recs.data(), (uint32_t)ids.size(), bits.data()),
          "cbft_bls_verify_shares");
    for (size_t j = 0; j < ids.size(); j++) {
      if (validBits_.count() == req_) break;
      const ShareID id = ids[j];
      if ((bits[j >> 3] >> (j & 7)) & 1) {
        valid_[(size_t)id] = pending_[(size_t)id];
        validBits_.add(id);
      } else {
        invalid_.insert(id);
      }
    }
  }
  pending_.clear();
}

std::vector<uint8_t> BlsAccumulatorBase::validRecords() const {
  std::vector<uint8_t> recs;
  for (ShareID id = validBits_.first(); !validBits_.isEnd(id); id = validBits_.next(id))
    putRecord(recs, id, valid_[(size_t)id].data());
  return recs;
}

static void combineInto(const BlsThresholdVerifier& v, const std::vector<uint8_t>& recs, int multisig,
                        uint8_t* out33) {
  const uint32_t k = (uint32_t)(recs.size() / 37);
  if (k == 0) {  // identity (G1T::Identity(), BlsThresholdAccumulator.cpp:34)
    std::memset(out33, 0, 33);
    return;
  }
  check(cbft_bls_combine(v.engine()->ctx(), recs.data(), k, multisig, out33), "cbft_bls_combine");
}

void BlsThresholdAccumulator::getFullSignedData(char* out, int len) {
  if (!out || len < 33) throw std::runtime_error("Not enough capacity to store threshold signature");
  combineInto(v_, validRecords(), 0, reinterpret_cast<uint8_t*>(out));
}

void BlsMultisigAccumulator::getFullSignedData(char* out, int len) {
  const int vec = (req_ != num_) ? VectorOfShares::getByteCount() : 0;
  if (!out || len < 33 + vec) throw std::runtime_error("Not enough capacity to store multisignature");
  combineInto(v_, validRecords(), 1, reinterpret_cast<uint8_t*>(out));
  if (vec) validBits_.toBytes(reinterpret_cast<unsigned char*>(out) + 33, vec);
}

// ------------------------------------------------------------------------------ signer
BlsThresholdSigner::BlsThresholdSigner(ShareID id, const std::string& secretKeyDecimal, const std::string& vkHex)
    : id_(id), sk_(secretKeyDecimal), vk_(vkHex.empty() ? BlsPublicKey() : BlsPublicKey(vkHex)) {
  if (id < 1 || id > MAX_NUM_OF_SHARES) throw std::invalid_argument("BLS signer: id out of range");
  engine_ = BlsEngine::get();
  if (vkHex.empty()) {  // the reference derives it: publicKey_(secretKey) = sk * g2 (BlsThresholdSigner.cpp:25)
    uint8_t vk65[65];
    check(cbft_bls_public_key(engine_->ctx(), sk_.bytes().data(), vk65), "cbft_bls_public_key");
    vk_ = BlsPublicKey(toHex(vk65, 65));
  }
}

void BlsThresholdSigner::signData(const char* hash, int hashLen, char* outSig, int outSigLen) {
  if (!outSig || outSigLen < 37) throw std::runtime_error("BLS signer: output buffer shorter than 37 bytes");
  if (!hash || hashLen < 0) throw std::invalid_argument("BLS signer: no message");
  check(cbft_bls_sign(engine_->ctx(), sk_.bytes().data(), (uint32_t)id_, reinterpret_cast<const uint8_t*>(hash),
                      (uint32_t)hashLen, reinterpret_cast<uint8_t*>(outSig)),
        "cbft_bls_sign");
}

}  // namespace Hip
}  // namespace BLS

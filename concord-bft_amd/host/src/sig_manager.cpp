// SigManager with verifySigBatch over libcbft_hipcrypto (see sig_manager.hpp).
#include "sig_manager.hpp"

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace bftEngine::impl {

using concord::util::crypto::EdDSASigner;
using concord::util::crypto::EdDSAVerifier;
using concord::util::crypto::IVerifier;
using concord::util::crypto::RSASigner;
using concord::util::crypto::KeyFormat;
using concord::util::crypto::VerifyRequest;

SigManager::SigManager(PrincipalId myId, const std::pair<Key, KeyFormat>& mySigPrivateKey,
                       const std::vector<std::pair<std::set<PrincipalId>, Key>>& publicKeys, KeyFormat keysFormat,
                       const ReplicasInfo& replicasInfo)
    : myId_(myId), replicasInfo_(replicasInfo) {
  if (!mySigPrivateKey.first.empty()) {
    // an Ed25519 seed (hex) or an RSA private key (the reference's replicas sign with RSA)
    try {
      mySigner_ = std::make_unique<EdDSASigner>(mySigPrivateKey.first, mySigPrivateKey.second);
    } catch (const std::invalid_argument&) {
      mySigner_ = std::make_unique<RSASigner>(mySigPrivateKey.first, mySigPrivateKey.second);
    }
  }
  // one verifier object per distinct key, shared by every principal mapped to it
  // (SigManager.cpp:139-150); Ed25519 or RSA by key type
  for (const auto& [ids, key] : publicKeys) {
    auto v = concord::util::crypto::makeVerifier(key, keysFormat);
    for (PrincipalId id : ids) verifiers_[id] = v;
  }
}

uint16_t SigManager::getSigLength(PrincipalId pid) const {
  std::shared_lock lock(mutex_);
  auto it = verifiers_.find(pid);
  return it == verifiers_.end() ? 0 : (uint16_t)it->second->signatureLength();
}

void SigManager::account(PrincipalId pid, bool result) const {
  const bool client = replicasInfo_.isIdOfExternalClient(pid);
  if (result) {
    if (client)
      metrics_.external_client_request_signatures_verified++;
    else
      metrics_.peer_replicas_signatures_verified++;
  } else {
    if (client)
      metrics_.external_client_request_signature_verification_failed++;
    else
      metrics_.peer_replicas_signature_verification_failed++;
  }
}

bool SigManager::verifySig(PrincipalId pid, const char* data, size_t dataLength, const char* sig,
                           uint16_t sigLength) const {
  std::vector<SigBatchItem> one{{pid, data, dataLength, sig, sigLength}};
  std::vector<bool> out;
  verifySigBatch(one, out);
  return out[0];
}

void SigManager::verifySigBatch(const std::vector<SigBatchItem>& items, std::vector<bool>& out) const {
  out.assign(items.size(), false);
  std::vector<VerifyRequest> reqs(items.size());
  std::vector<char> known(items.size(), 0);
  {
    std::shared_lock lock(mutex_);
    for (size_t i = 0; i < items.size(); i++) {
      auto it = verifiers_.find(items[i].pid);
      if (it == verifiers_.end()) {
        reqs[i] = {nullptr, nullptr, 0, nullptr, 0};
        continue;
      }
      known[i] = 1;
      reqs[i] = {it->second.get(), items[i].data, items[i].dataLength, items[i].sig, items[i].sigLength};
    }
    concord::util::crypto::verifyBatch(reqs, out);  // verifiers stay alive under the shared lock
  }
  for (size_t i = 0; i < items.size(); i++) {
    if (!known[i]) {
      metrics_.signature_verification_failed_on_unrecognized_participant_id++;
      out[i] = false;
      continue;
    }
    account(items[i].pid, out[i]);
  }
}

void SigManager::sign(const char* data, size_t dataLength, char* outSig, uint16_t outSigLength) const {
  if (!mySigner_) throw std::runtime_error("SigManager::sign: no private key");
  std::string s = mySigner_->sign(std::string(data, dataLength));
  std::memcpy(outSig, s.data(), std::min<size_t>(s.size(), outSigLength));
}

uint16_t SigManager::getMySigLength() const { return mySigner_ ? (uint16_t)mySigner_->signatureLength() : 0; }

void SigManager::setClientPublicKey(const std::string& key, PrincipalId id, KeyFormat fmt) {
  auto v = concord::util::crypto::makeVerifier(key, fmt);  // throws on a bad key, like the reference
  std::unique_lock lock(mutex_);
  verifiers_.insert_or_assign(id, std::move(v));
}

bool SigManager::hasVerifier(PrincipalId pid) const {
  std::shared_lock lock(mutex_);
  return verifiers_.count(pid) != 0;
}

}  // namespace bftEngine::impl

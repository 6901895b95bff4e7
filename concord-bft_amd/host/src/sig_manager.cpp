// SigManager / ReplicasInfo over libcbft_hipcrypto (see sig_manager.hpp).
#include "sig_manager.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace bftEngine::impl {

using concord::util::crypto::EdDSASigner;
using concord::util::crypto::IVerifier;
using concord::util::crypto::KeyFormat;
using concord::util::crypto::RSASigner;
using concord::util::crypto::VerifyRequest;

// ------------------------------------------------------------------------------ ReplicasInfo
ReplicasInfo::ReplicasInfo(const ReplicaIdsConfig& c) : cfg_(c), myId_(c.replicaId) {
  if (c.numReplicas != 3 * c.fVal + 2 * c.cVal + 1)
    throw std::invalid_argument("ReplicasInfo: numReplicas != 3f + 2c + 1");  // ReplicasInfo.cpp:143
  const uint32_t n = c.numReplicas, ro = c.numRoReplicas, px = c.numOfClientProxies, ext = c.numOfExternalClients,
                 svc = c.numOfClientServices, op = c.operatorEnabled ? 1u : 0u;
  maxValidPrincipalId_ = n + ro + px + ext + n + svc - 1;  // internal clients: one per replica
  for (uint32_t i = n; i < n + ro; i++) roReplicas_.insert(i);
  for (uint32_t i = n + ro; i < n + ro + px; i++) clientProxies_.insert(i);
  const uint32_t es = n + ro + px, ee = es + ext;
  for (uint32_t i = es; i < ee - op; i++) externalClients_.insert(i);
  externalClients_.insert(ee + svc - 1);  // ReplicasInfo.cpp:115 (the operator's id when enabled)
  for (uint32_t i = ee - op; i < ee - op + svc; i++) clientServices_.insert(i);
  for (uint32_t i = ee + svc; i < ee + svc + n; i++) internalClients_.insert(i);
}

// ------------------------------------------------------------------------------ SigManager
SigManager* SigManager::instance(SigManager* sm) {
  static SigManager* instance_ = nullptr;
  if (sm) instance_ = sm;
  return instance_;
}

SigManager* SigManager::initInTesting(ReplicaId myId, const Key& mySigPrivateKey,
                                      const std::set<std::pair<PrincipalId, const std::string>>& publicKeysOfReplicas,
                                      KeyFormat replicasKeysFormat,
                                      const std::set<std::pair<const std::string, std::set<uint16_t>>>* publicKeysOfClients,
                                      KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo) {
  // SigManager.cpp:34-94: replica keys first (one key per replica), then the client keys (one
  // key per set of principal ids)
  std::vector<std::pair<Key, KeyFormat>> publickeys;
  std::map<PrincipalId, KeyIndex> mapping;
  KeyIndex i = 0;
  const PrincipalId replicaHigh = replicasInfo.getNumberOfReplicas() + replicasInfo.getNumberOfRoReplicas() - 1;
  for (const auto& [id, key] : publicKeysOfReplicas) {
    if (id > replicaHigh) throw std::invalid_argument("SigManager: replica key for id " + std::to_string(id));
    publickeys.emplace_back(key, replicasKeysFormat);
    mapping.emplace(id, i++);
  }
  if (publicKeysOfClients) {
    const PrincipalId low = replicasInfo.getNumberOfRoReplicas() + replicasInfo.getNumberOfReplicas() +
                            replicasInfo.getNumOfClientProxies();
    const PrincipalId high = low + replicasInfo.getNumberOfExternalClients() +
                             replicasInfo.getNumberOfInternalClients() + replicasInfo.getNumberOfClientServices() - 1;
    for (const auto& [key, ids] : *publicKeysOfClients) {
      if (key.empty()) throw std::invalid_argument("SigManager: empty client key");
      publickeys.emplace_back(key, clientsKeysFormat);
      for (uint16_t e : ids) {
        if (e < low || e > high) throw std::invalid_argument("SigManager: invalid participant id " + std::to_string(e));
        mapping.emplace(e, i);
      }
      ++i;
    }
  }
  return new SigManager(myId, replicasInfo.getNumberOfReplicas(), {mySigPrivateKey, replicasKeysFormat}, publickeys,
                        mapping, replicasInfo.clientTransactionSigningEnabled() && publicKeysOfClients != nullptr,
                        replicasInfo);
}

SigManager* SigManager::init(ReplicaId myId, const Key& mySigPrivateKey,
                             const std::set<std::pair<PrincipalId, const std::string>>& publicKeysOfReplicas,
                             KeyFormat replicasKeysFormat,
                             const std::set<std::pair<const std::string, std::set<uint16_t>>>* publicKeysOfClients,
                             KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo) {
  return instance(initInTesting(myId, mySigPrivateKey, publicKeysOfReplicas, replicasKeysFormat, publicKeysOfClients,
                                clientsKeysFormat, replicasInfo));
}

SigManager::SigManager(PrincipalId myId, uint16_t /*numReplicas*/, const std::pair<Key, KeyFormat>& mySigPrivateKey,
                       const std::vector<std::pair<Key, KeyFormat>>& publickeys,
                       const std::map<PrincipalId, KeyIndex>& publicKeysMapping, bool clientTransactionSigningEnabled,
                       ReplicasInfo& replicasInfo)
    : myId_(myId), clientTransactionSigningEnabled_(clientTransactionSigningEnabled), replicasInfo_(replicasInfo) {
  if (!mySigPrivateKey.first.empty()) {
    // an Ed25519 seed (hex / PEM) or an RSA private key (the reference's replicas sign with RSA)
    try {
      mySigner_ = std::make_unique<EdDSASigner>(mySigPrivateKey.first, mySigPrivateKey.second);
    } catch (const std::invalid_argument&) {
      mySigner_ = std::make_unique<RSASigner>(mySigPrivateKey.first, mySigPrivateKey.second);
    }
  }
  // one verifier object per distinct key index, shared by every principal mapped to it
  // (SigManager.cpp:139-150); Ed25519 or RSA by key type
  std::map<KeyIndex, std::shared_ptr<IVerifier>> byIndex;
  for (const auto& [pid, idx] : publicKeysMapping) {
    if (idx >= publickeys.size()) throw std::invalid_argument("SigManager: key index out of range");
    auto it = byIndex.find(idx);
    if (it == byIndex.end())
      it = byIndex.emplace(idx, concord::util::crypto::makeVerifier(publickeys[idx].first, publickeys[idx].second))
               .first;
    verifiers_[pid] = it->second;
  }
}

uint16_t SigManager::getSigLength(PrincipalId pid) const {
  if (pid == myId_) return getMySigLength();
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
  std::shared_ptr<IVerifier> v;
  {
    std::shared_lock lock(mutex_);
    auto it = verifiers_.find(pid);
    if (it != verifiers_.end()) v = it->second;
  }
  if (!v) {
    metrics_.signature_verification_failed_on_unrecognized_participant_id++;
    return false;
  }
  // IVerifier::verify: Ed25519 requests from concurrent threads are coalesced into GPU batches
  const bool result = v->verify(std::string(data, dataLength), std::string(sig, sigLength));
  account(pid, result);
  return result;
}

size_t SigManager::verifySigBatch(const std::vector<SigBatchItem>& items, std::vector<bool>& out,
                                  bool stopAtFirstFailure) const {
  out.assign(items.size(), false);
  std::vector<VerifyRequest> reqs(items.size());
  std::vector<std::shared_ptr<IVerifier>> hold(items.size());
  {
    std::shared_lock lock(mutex_);
    for (size_t i = 0; i < items.size(); i++) {
      auto it = verifiers_.find(items[i].pid);
      if (it != verifiers_.end()) hold[i] = it->second;  // kept alive past a concurrent key rotation
    }
  }
  for (size_t i = 0; i < items.size(); i++)
    reqs[i] = hold[i] ? VerifyRequest{hold[i].get(), items[i].data, items[i].dataLength, items[i].sig,
                                      items[i].sigLength}
                      : VerifyRequest{nullptr, nullptr, 0, nullptr, 0};
  concord::util::crypto::verifyBatch(reqs, out);
  size_t first = items.size();
  for (size_t i = 0; i < items.size(); i++) {
    if (!hold[i]) {
      out[i] = false;
      metrics_.signature_verification_failed_on_unrecognized_participant_id++;
    } else {
      account(items[i].pid, out[i]);
    }
    if (!out[i] && first == items.size()) {
      first = i;
      if (stopAtFirstFailure) break;
    }
  }
  return first;
}

void SigManager::sign(const char* data, size_t dataLength, char* outSig, uint16_t outSigLength) const {
  if (!mySigner_) throw std::runtime_error("SigManager::sign: no private key");
  std::string s = mySigner_->sign(std::string(data, dataLength));
  std::memcpy(outSig, s.data(), std::min<size_t>(s.size(), outSigLength));
}

uint16_t SigManager::getMySigLength() const { return mySigner_ ? (uint16_t)mySigner_->signatureLength() : 0; }

void SigManager::setClientPublicKey(const std::string& key, PrincipalId id, KeyFormat fmt) {
  if (!replicasInfo_.isIdOfExternalClient(id) && !replicasInfo_.isIdOfClientService(id)) return;  // :252, :262
  auto v = concord::util::crypto::makeVerifier(key, fmt);  // throws on a bad key, like the reference (:258)
  std::unique_lock lock(mutex_);
  verifiers_.insert_or_assign(id, std::move(v));
}

bool SigManager::hasVerifier(PrincipalId pid) const {
  std::shared_lock lock(mutex_);
  return verifiers_.count(pid) != 0;
}

std::string SigManager::getPublicKeyOfVerifier(uint32_t id) const {
  std::shared_lock lock(mutex_);
  auto it = verifiers_.find(id);
  return it == verifiers_.end() ? std::string() : it->second->getPubKey();
}

std::string SigManager::getSelfPrivKey() const { return mySigner_ ? mySigner_->getPrivKey() : std::string(); }

}  // namespace bftEngine::impl

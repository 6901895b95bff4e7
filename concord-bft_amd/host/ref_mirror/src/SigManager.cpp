// Standalone-build restatement of bftengine/src/bftengine/SigManager.cpp:27-265 (see
// ref_mirror/include/SigManager.hpp).  Behaviour kept: principal ids mapped to key indices
// (replica keys one each, client keys one per id set), one verifier object per distinct key,
// RSAVerifier / RSASigner as the reference builds them, the five counters of the
// "signature_manager" component with the aggregator pushed on every failure and on every 1,000th
// success, and ClientsPublicKeys in CMF encoding for getClientsPublicKeys().  ConcordAssert /
// std::terminate on bad ids become std::invalid_argument.
#include "SigManager.hpp"

#include <cstring>
#include <stdexcept>

#include "ReplicaConfig.hpp"
#include "ReplicasInfo.hpp"
#include "keys_and_signatures.cmf.hpp"

namespace bftEngine {
namespace impl {

using concord::util::crypto::KeyFormat;

// keys_and_signatures.cmf's ClientsPublicKeys, a namespace-scope global as in the reference
// (SigManager.cpp:25): HipSigManager::setClientPublicKey updates it too.  CMF encoding: integers
// big-endian, strings and maps u32-length prefixed (messages/compiler/cpp/serialize.cpp).
concord::messages::keys_and_signatures::ClientsPublicKeys clientsPublicKeys_;

namespace {
void putBE(std::vector<uint8_t>& o, uint64_t v, int bytes) {
  for (int i = bytes - 1; i >= 0; i--) o.push_back((uint8_t)(v >> (8 * i)));
}
}  // namespace

std::string SigManager::getClientsPublicKeys() {
  std::shared_lock lock(mutex_);
  std::vector<uint8_t> out;
  putBE(out, clientsPublicKeys_.ids_to_keys.size(), 4);
  for (const auto& [id, k] : clientsPublicKeys_.ids_to_keys) {
    putBE(out, id, 2);
    putBE(out, k.key.size(), 4);
    out.insert(out.end(), k.key.begin(), k.key.end());
    out.push_back(k.format);
  }
  putBE(out, clientsPublicKeys_.version, 2);
  return std::string(out.begin(), out.end());
}

SigManager* SigManager::initImpl(ReplicaId myId, const Key& mySigPrivateKey, const ReplicaKeys& publicKeysOfReplicas,
                                 KeyFormat replicasKeysFormat, const ClientKeys* publicKeysOfClients,
                                 KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo) {
  std::vector<std::pair<Key, KeyFormat>> keys;
  std::map<PrincipalId, KeyIndex> mapping;
  KeyIndex next = 0;
  const uint32_t lastReplica = replicasInfo.getNumberOfReplicas() + replicasInfo.getNumberOfRoReplicas() - 1;
  for (const auto& [id, key] : publicKeysOfReplicas) {
    if (id > lastReplica) throw std::invalid_argument("SigManager: replica key for id " + std::to_string(id));
    keys.emplace_back(key, replicasKeysFormat);
    mapping.insert({id, next++});
  }
  if (publicKeysOfClients) {
    const uint32_t lo = replicasInfo.getNumberOfRoReplicas() + replicasInfo.getNumberOfReplicas() +
                        replicasInfo.getNumOfClientProxies();
    const uint32_t hi = lo + replicasInfo.getNumberOfExternalClients() + replicasInfo.getNumberOfInternalClients() +
                        replicasInfo.getNumberOfClientServices() - 1;
    for (const auto& [key, ids] : *publicKeysOfClients) {
      if (key.empty()) throw std::invalid_argument("SigManager: empty client key");
      keys.emplace_back(key, clientsKeysFormat);
      for (const uint16_t e : ids) {
        if (e < lo || e > hi) throw std::invalid_argument("SigManager: invalid participant id " + std::to_string(e));
        mapping.insert({e, next});
      }
      ++next;
    }
  }
  const bool signing = ReplicaConfig::instance().clientTransactionSigningEnabled && publicKeysOfClients != nullptr;
  return new SigManager(myId, replicasInfo.getNumberOfReplicas(), {mySigPrivateKey, replicasKeysFormat}, keys,
                        mapping, signing, replicasInfo);
}

SigManager* SigManager::init(ReplicaId myId, const Key& mySigPrivateKey, const ReplicaKeys& publicKeysOfReplicas,
                             KeyFormat replicasKeysFormat, const ClientKeys* publicKeysOfClients,
                             KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo) {
  return instance(initImpl(myId, mySigPrivateKey, publicKeysOfReplicas, replicasKeysFormat, publicKeysOfClients,
                           clientsKeysFormat, replicasInfo));
}

SigManager::SigManager(PrincipalId myId, uint16_t, const std::pair<Key, KeyFormat>& mySigPrivateKey,
                       const std::vector<std::pair<Key, KeyFormat>>& publickeys,
                       const std::map<PrincipalId, KeyIndex>& publicKeysMapping, bool clientTransactionSigningEnabled,
                       ReplicasInfo& replicasInfo)
    : myId_(myId),
      clientTransactionSigningEnabled_(clientTransactionSigningEnabled),
      replicasInfo_(replicasInfo),
      metrics_component_{"signature_manager", std::make_shared<concordMetrics::Aggregator>()},
      metrics_{metrics_component_.RegisterAtomicCounter("external_client_request_signature_verification_failed"),
               metrics_component_.RegisterAtomicCounter("external_client_request_signatures_verified"),
               metrics_component_.RegisterAtomicCounter("peer_replicas_signature_verification_failed"),
               metrics_component_.RegisterAtomicCounter("peer_replicas_signatures_verified"),
               metrics_component_.RegisterAtomicCounter(
                   "signature_verification_failed_on_unrecognized_participant_id")} {
  if (publicKeysMapping.size() < publickeys.size()) throw std::invalid_argument("SigManager: unmapped keys");
  if (!mySigPrivateKey.first.empty())
    mySigner_.reset(new concord::util::crypto::RSASigner(mySigPrivateKey.first, mySigPrivateKey.second));
  std::map<KeyIndex, std::shared_ptr<concord::util::crypto::IVerifier>> byIndex;
  for (const auto& [pid, idx] : publicKeysMapping) {
    if (idx >= publickeys.size()) throw std::invalid_argument("SigManager: key index out of range");
    auto it = byIndex.find(idx);
    if (it == byIndex.end())
      it = byIndex
               .emplace(idx, std::make_shared<concord::util::crypto::RSAVerifier>(publickeys[idx].first,
                                                                                  publickeys[idx].second))
               .first;
    verifiers_[pid] = it->second;
    if (replicasInfo_.isIdOfExternalClient(pid))
      clientsPublicKeys_.ids_to_keys[pid] = {publickeys[idx].first, (uint8_t)publickeys[idx].second};
  }
  clientsPublicKeys_.version = 1;  // 1 = RSAVerifier
  metrics_component_.Register();
}

uint16_t SigManager::getSigLength(PrincipalId pid) const {
  if (pid == myId_) return (uint16_t)mySigner_->signatureLength();
  std::shared_lock lock(mutex_);
  auto it = verifiers_.find(pid);
  return it == verifiers_.end() ? 0 : (uint16_t)it->second->signatureLength();
}

bool SigManager::verifySig(PrincipalId pid, const char* data, size_t dataLength, const char* sig,
                           uint16_t sigLength) const {
  bool ok = false;
  {
    const std::string d(data, dataLength), s(sig, sigLength);
    std::shared_lock lock(mutex_);
    auto it = verifiers_.find(pid);
    if (it == verifiers_.end()) {
      metrics_.sigVerificationFailedOnUnrecognizedParticipantId_++;
      metrics_component_.UpdateAggregator();
      return false;
    }
    ok = it->second->verify(d, s);
  }
  const bool external = replicasInfo_.isIdOfExternalClient(pid);
  if (!external && !replicasInfo_.isIdOfReplica(pid) && !replicasInfo_.isIdOfPeerRoReplica(pid))
    throw std::logic_error("SigManager::verifySig: pid is neither a replica nor an external client");
  if (!ok) {
    (external ? metrics_.externalClientReqSigVerificationFailed_ : metrics_.replicaSigVerificationFailed_)++;
    metrics_component_.UpdateAggregator();
  } else {
    auto& c = external ? metrics_.externalClientReqSigVerified_ : metrics_.replicaSigVerified_;
    c++;
    if (c.Get().Get() % updateMetricsAggregatorThresh == 0) metrics_component_.UpdateAggregator();
  }
  return ok;
}

void SigManager::sign(const char* data, size_t dataLength, char* outSig, uint16_t) const {
  const std::string s = mySigner_->sign(std::string(data, dataLength));
  std::memcpy(outSig, s.data(), s.size());
}

uint16_t SigManager::getMySigLength() const { return (uint16_t)mySigner_->signatureLength(); }

void SigManager::setClientPublicKey(const std::string& key, PrincipalId id, KeyFormat format) {
  if (!replicasInfo_.isIdOfExternalClient(id) && !replicasInfo_.isIdOfClientService(id)) return;  // "Illegal id"
  {
    std::unique_lock lock(mutex_);
    verifiers_.insert_or_assign(id, std::make_shared<concord::util::crypto::RSAVerifier>(key, format));
  }
  clientsPublicKeys_.ids_to_keys[id] = {key, (uint8_t)format};
}

bool SigManager::hasVerifier(PrincipalId pid) { return verifiers_.find(pid) != verifiers_.end(); }

}  // namespace impl
}  // namespace bftEngine

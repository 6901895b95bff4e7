// Standalone-build restatement of bftEngine::impl::SigManager (bftengine/src/bftengine/
// SigManager.hpp:32-142, SigManager.cpp:27-265): the reference's public API and protected member
// names/types, so that concord::hip::HipSigManager, which derives from the reference's class,
// compiles unchanged against either.  The reference's SigManager.cpp is not buildable here (it
// includes the CMF-generated keys_and_signatures.cmf.hpp).  See ../README.md.
#pragma once
#include <map>
#include <memory>
#include <set>
#include <shared_mutex>
#include <string>
#include <utility>
#include <vector>

#include "Metrics.hpp"
#include "PrimitiveTypes.hpp"
#include "crypto_utils.hpp"

using concordMetrics::AtomicCounterHandle;

namespace bftEngine {
namespace impl {

class ReplicasInfo;

class SigManager {
  using KeyFormat = concord::util::crypto::KeyFormat;
  using ReplicaKeys = std::set<std::pair<PrincipalId, const std::string>>;
  using ClientKeys = std::set<std::pair<const std::string, std::set<uint16_t>>>;

 public:
  typedef std::string Key;
  typedef uint16_t KeyIndex;

  // process-wide instance; a non-null sm replaces it (tests), the caller deletes the object
  static SigManager* instance(SigManager* sm = nullptr) {
    static SigManager* current = nullptr;
    if (sm) current = sm;
    return current;
  }
  static SigManager* init(ReplicaId myId, const Key& mySigPrivateKey, const ReplicaKeys& publicKeysOfReplicas,
                          KeyFormat replicasKeysFormat, const ClientKeys* publicKeysOfClients,
                          KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo);

  bool verifySig(PrincipalId pid, const char* data, size_t dataLength, const char* sig, uint16_t sigLength) const;
  uint16_t getSigLength(PrincipalId pid) const;  // 0 for an unknown pid
  void sign(const char* data, size_t dataLength, char* outSig, uint16_t outSigLength) const;
  uint16_t getMySigLength() const;
  std::string getSelfPrivKey() const { return mySigner_->getPrivKey(); }
  bool isClientTransactionSigningEnabled() { return clientTransactionSigningEnabled_; }
  void setClientPublicKey(const std::string& key, PrincipalId, KeyFormat);
  bool hasVerifier(PrincipalId pid);
  std::string getPublicKeyOfVerifier(uint32_t id) const {
    auto it = verifiers_.find((PrincipalId)id);
    return it == verifiers_.end() ? std::string() : it->second->getPubKey();
  }
  std::string getClientsPublicKeys();  // CMF ClientsPublicKeys (keys_and_signatures.cmf)
  void SetAggregator(std::shared_ptr<concordMetrics::Aggregator> aggregator) {
    metrics_component_.SetAggregator(aggregator);
  }

  SigManager(const SigManager&) = delete;
  SigManager(SigManager&&) = delete;
  SigManager& operator=(const SigManager&) = delete;
  SigManager& operator=(SigManager&&) = delete;

 protected:
  static constexpr uint16_t updateMetricsAggregatorThresh = 1000;

  SigManager(PrincipalId myId, uint16_t numReplicas, const std::pair<Key, KeyFormat>& mySigPrivateKey,
             const std::vector<std::pair<Key, KeyFormat>>& publickeys,
             const std::map<PrincipalId, KeyIndex>& publicKeysMapping, bool clientTransactionSigningEnabled,
             ReplicasInfo& replicasInfo);
  static SigManager* initImpl(ReplicaId myId, const Key& mySigPrivateKey, const ReplicaKeys& publicKeysOfReplicas,
                              KeyFormat replicasKeysFormat, const ClientKeys* publicKeysOfClients,
                              KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo);

  const PrincipalId myId_;
  std::unique_ptr<concord::util::crypto::ISigner> mySigner_;
  std::map<PrincipalId, std::shared_ptr<concord::util::crypto::IVerifier>> verifiers_;
  bool clientTransactionSigningEnabled_ = true;
  ReplicasInfo& replicasInfo_;

  struct Metrics {  // the five counters of the "signature_manager" component
    AtomicCounterHandle externalClientReqSigVerificationFailed_, externalClientReqSigVerified_;
    AtomicCounterHandle replicaSigVerificationFailed_, replicaSigVerified_;
    AtomicCounterHandle sigVerificationFailedOnUnrecognizedParticipantId_;
  };
  mutable concordMetrics::Component metrics_component_;
  mutable Metrics metrics_;
  mutable std::shared_mutex mutex_;

#ifdef CONCORD_BFT_TESTING
 public:
  static SigManager* initInTesting(ReplicaId myId, const Key& mySigPrivateKey, const ReplicaKeys& publicKeysOfReplicas,
                                   KeyFormat replicasKeysFormat, const ClientKeys* publicKeysOfClients,
                                   KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo) {
    return initImpl(myId, mySigPrivateKey, publicKeysOfReplicas, replicasKeysFormat, publicKeysOfClients,
                    clientsKeysFormat, replicasInfo);
  }
#endif
};

}  // namespace impl
}  // namespace bftEngine

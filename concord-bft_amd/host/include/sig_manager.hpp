// bftEngine::impl::SigManager and the ReplicasInfo id space it reads, with the reference's API
// (bftengine/src/bftengine/SigManager.hpp:31-140, SigManager.cpp:34-265; ReplicasInfo.hpp:27-90,
// ReplicasInfo.cpp:50-140) plus one batch entry point.
//
// Same contract as the reference: principal id -> shared verifier under a shared_mutex; one
// verifier object per distinct key, shared by every principal mapped to it; verifySig() returns
// false on a bad signature OR an unknown principal; the five metric counters of
// SigManager.cpp:124-132 move exactly as there.  Verifiers are EdDSAVerifier or RSAVerifier
// by key type (the reference builds RSAVerifiers only, SigManager.cpp:138,146,255; its
// key-format "version" tag is where Ed25519 would be selected, :156).
//
// New: verifySigBatch(), which the serial loops of PrePrepareMsg::validate
// (PrePrepareMsg.cpp:116-125), PreProcessor::checkClientBatchMsgCorrectness
// (PreProcessor.cpp:557-590) and PreProcessResultMsg (PreProcessResultMsg.cpp:79-96) call once per
// batch instead of once per request (request_batch.hpp walks those messages).  Verdicts and
// counter increments equal calling verifySig() on each item in order — or, with
// stopAtFirstFailure, on each item up to and including the first failing one, as a loop that
// throws at the first failure does.
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <set>
#include <shared_mutex>
#include <string>
#include <utility>
#include <vector>

#include "crypto_utils.hpp"

namespace bftEngine::impl {

using PrincipalId = uint32_t;
using ReplicaId = uint16_t;
using NodeIdType = uint16_t;

// The ReplicaConfig fields ReplicasInfo and SigManager read (ReplicaConfig.hpp; ReplicasInfo.cpp:50-65;
// clientTransactionSigningEnabled, ReplicaConfig.hpp:90).
struct ReplicaIdsConfig {
  ReplicaId replicaId = 0;
  uint16_t fVal = 1;
  uint16_t cVal = 0;
  uint16_t numReplicas = 4;  // must be 3f + 2c + 1
  uint16_t numRoReplicas = 0;
  uint16_t numOfClientProxies = 0;
  uint16_t numOfExternalClients = 0;
  uint16_t numOfClientServices = 0;
  bool operatorEnabled = false;
  bool clientTransactionSigningEnabled = true;
};

// Principal ids in the reference's order (ReplicasInfo.cpp:71-140): [replicas][ro-replicas]
// [client proxies][external clients (the last one the operator when enabled)][client services]
// [internal clients: one per replica].
class ReplicasInfo {
 public:
  explicit ReplicasInfo(const ReplicaIdsConfig& config);  // throws std::invalid_argument if n != 3f+2c+1

  ReplicaId myId() const { return myId_; }
  uint16_t fVal() const { return cfg_.fVal; }
  uint16_t cVal() const { return cfg_.cVal; }
  bool isIdOfReplica(PrincipalId id) const { return id < cfg_.numReplicas; }
  bool isIdOfPeerReplica(PrincipalId id) const { return id < cfg_.numReplicas && id != myId_; }
  bool isIdOfPeerRoReplica(PrincipalId id) const { return roReplicas_.count(id) != 0; }
  bool isIdOfClientProxy(PrincipalId id) const { return clientProxies_.count(id) != 0; }
  bool isIdOfExternalClient(PrincipalId id) const { return externalClients_.count(id) != 0; }
  bool isIdOfInternalClient(PrincipalId id) const { return internalClients_.count(id) != 0; }
  bool isIdOfClientService(PrincipalId id) const { return clientServices_.count(id) != 0; }
  bool isValidPrincipalId(PrincipalId id) const { return id <= maxValidPrincipalId_; }
  uint16_t getNumberOfReplicas() const { return cfg_.numReplicas; }
  uint16_t getNumberOfRoReplicas() const { return cfg_.numRoReplicas; }
  uint16_t getNumOfClientProxies() const { return cfg_.numOfClientProxies; }
  uint16_t getNumberOfExternalClients() const { return cfg_.numOfExternalClients; }
  uint16_t getNumberOfInternalClients() const { return cfg_.numReplicas; }
  uint16_t getNumberOfClientServices() const { return cfg_.numOfClientServices; }
  bool clientTransactionSigningEnabled() const { return cfg_.clientTransactionSigningEnabled; }

 private:
  ReplicaIdsConfig cfg_;
  ReplicaId myId_;
  PrincipalId maxValidPrincipalId_;
  std::set<PrincipalId> roReplicas_, clientProxies_, externalClients_, clientServices_, internalClients_;
};

struct SigBatchItem {
  PrincipalId pid;
  const char* data;
  size_t dataLength;
  const char* sig;
  uint16_t sigLength;
};

class SigManager {
 public:
  typedef std::string Key;
  typedef uint16_t KeyIndex;

  // The process-wide instance (SigManager.hpp:40-48): sm != nullptr sets it (testing); the
  // caller owns (deletes) the object.
  static SigManager* instance(SigManager* sm = nullptr);

  // SigManager.cpp:96-111: builds the verifiers and sets the instance.  publicKeysOfReplicas:
  // (replica id, key) with ids in [0, numReplicas + numRoReplicas); publicKeysOfClients: (key,
  // principal ids sharing it) with ids in [numReplicas + numRoReplicas + numOfClientProxies,
  // ... + externalClients + internalClients + clientServices).  An id outside its range throws
  // std::invalid_argument (the reference asserts / terminates, SigManager.cpp:58,76-79); a key
  // that does not parse throws std::invalid_argument.
  static SigManager* init(ReplicaId myId, const Key& mySigPrivateKey,
                          const std::set<std::pair<PrincipalId, const std::string>>& publicKeysOfReplicas,
                          concord::util::crypto::KeyFormat replicasKeysFormat,
                          const std::set<std::pair<const std::string, std::set<uint16_t>>>* publicKeysOfClients,
                          concord::util::crypto::KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo);
  // the same without touching the instance (SigManager.hpp:119-137, CONCORD_BFT_TESTING)
  static SigManager* initInTesting(ReplicaId myId, const Key& mySigPrivateKey,
                                   const std::set<std::pair<PrincipalId, const std::string>>& publicKeysOfReplicas,
                                   concord::util::crypto::KeyFormat replicasKeysFormat,
                                   const std::set<std::pair<const std::string, std::set<uint16_t>>>* publicKeysOfClients,
                                   concord::util::crypto::KeyFormat clientsKeysFormat, ReplicasInfo& replicasInfo);

  // 0 if pid is unknown; pid == myId: this replica's own signature length (SigManager.cpp:183-195)
  uint16_t getSigLength(PrincipalId pid) const;
  bool verifySig(PrincipalId pid, const char* data, size_t dataLength, const char* sig, uint16_t sigLength) const;
  // out[i] == verifySig(items[i]...) for every item, one GPU launch per algorithm for the whole
  // batch.  stopAtFirstFailure: counters move only for items[0 .. f] where f is the first
  // failing item (the serial loops throw there); returns f, or items.size() if none failed.
  size_t verifySigBatch(const std::vector<SigBatchItem>& items, std::vector<bool>& out,
                        bool stopAtFirstFailure = false) const;
  void sign(const char* data, size_t dataLength, char* outSig, uint16_t outSigLength) const;
  uint16_t getMySigLength() const;
  bool isClientTransactionSigningEnabled() const { return clientTransactionSigningEnabled_; }
  // Replaces an external client's or client service's key (SigManager.cpp:250-264); other ids
  // are ignored (the reference logs "Illegal id for client"); a bad key throws.
  void setClientPublicKey(const std::string& key, PrincipalId id, concord::util::crypto::KeyFormat fmt);
  bool hasVerifier(PrincipalId pid) const;
  std::string getPublicKeyOfVerifier(uint32_t id) const;
  std::string getSelfPrivKey() const;
  const ReplicasInfo& replicasInfo() const { return replicasInfo_; }

  SigManager(const SigManager&) = delete;
  SigManager& operator=(const SigManager&) = delete;

  // metric counters (names as in SigManager.cpp:124-132)
  struct Metrics {
    std::atomic<uint64_t> external_client_request_signature_verification_failed{0};
    std::atomic<uint64_t> external_client_request_signatures_verified{0};
    std::atomic<uint64_t> peer_replicas_signature_verification_failed{0};
    std::atomic<uint64_t> peer_replicas_signatures_verified{0};
    std::atomic<uint64_t> signature_verification_failed_on_unrecognized_participant_id{0};
  };
  const Metrics& metrics() const { return metrics_; }

 protected:
  SigManager(PrincipalId myId, uint16_t numReplicas,
             const std::pair<Key, concord::util::crypto::KeyFormat>& mySigPrivateKey,
             const std::vector<std::pair<Key, concord::util::crypto::KeyFormat>>& publickeys,
             const std::map<PrincipalId, KeyIndex>& publicKeysMapping, bool clientTransactionSigningEnabled,
             ReplicasInfo& replicasInfo);

 private:
  void account(PrincipalId pid, bool result) const;

  const PrincipalId myId_;
  std::unique_ptr<concord::util::crypto::ISigner> mySigner_;
  std::map<PrincipalId, std::shared_ptr<concord::util::crypto::IVerifier>> verifiers_;
  bool clientTransactionSigningEnabled_ = true;
  ReplicasInfo& replicasInfo_;
  mutable Metrics metrics_;
  mutable std::shared_mutex mutex_;
};

}  // namespace bftEngine::impl

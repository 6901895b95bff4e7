// bftEngine::impl::SigManager with a batch entry point.
//
// Mirrors the reference's SigManager (bftengine/src/bftengine/SigManager.hpp:31-140,
// SigManager.cpp:96-265): principal id -> shared verifier map under a shared_mutex, the same
// verifySig() contract (false on a bad signature OR an unknown principal) and the same metric
// counters, named as in SigManager.cpp:124-132.  New: verifySigBatch(), which the serial loops
// of PrePrepareMsg::validate (PrePrepareMsg.cpp:116-125), PreProcessor::
// checkClientBatchMsgCorrectness (PreProcessor.cpp:557-590) and PreProcessResultMsg
// (PreProcessResultMsg.cpp:79-96) call once per batch instead of once per request.  Verdicts and
// counter increments are exactly those of calling verifySig() on each item in order.
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

// The id-space facts SigManager needs from ReplicasInfo (ReplicasInfo.hpp): replicas are
// [0, numReplicas), read-only replicas follow, external clients are the listed ids.
struct ReplicasInfo {
  uint16_t numReplicas = 4;
  uint16_t numRoReplicas = 0;
  std::set<PrincipalId> externalClients;
  bool isIdOfReplica(PrincipalId id) const { return id < numReplicas; }
  bool isIdOfPeerRoReplica(PrincipalId id) const { return id >= numReplicas && id < numReplicas + numRoReplicas; }
  bool isIdOfExternalClient(PrincipalId id) const { return externalClients.count(id) != 0; }
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
  using Key = std::string;

  // publicKeys: (principal ids sharing the key, key string); each key builds an EdDSAVerifier or
  // an RSAVerifier by its type (makeVerifier; the reference builds RSAVerifiers,
  // SigManager.cpp:138,146, and its key-format "version" tag would select Ed25519, :156).
  SigManager(PrincipalId myId, const std::pair<Key, concord::util::crypto::KeyFormat>& mySigPrivateKey,
             const std::vector<std::pair<std::set<PrincipalId>, Key>>& publicKeys,
             concord::util::crypto::KeyFormat keysFormat, const ReplicasInfo& replicasInfo);

  uint16_t getSigLength(PrincipalId pid) const;
  bool verifySig(PrincipalId pid, const char* data, size_t dataLength, const char* sig, uint16_t sigLength) const;
  // out[i] == verifySig(items[i]...); one GPU launch for the whole batch
  void verifySigBatch(const std::vector<SigBatchItem>& items, std::vector<bool>& out) const;
  void sign(const char* data, size_t dataLength, char* outSig, uint16_t outSigLength) const;
  uint16_t getMySigLength() const;
  void setClientPublicKey(const std::string& key, PrincipalId id, concord::util::crypto::KeyFormat fmt);
  bool hasVerifier(PrincipalId pid) const;

  // metric counters (names as in SigManager.cpp:124-132)
  struct Metrics {
    std::atomic<uint64_t> external_client_request_signature_verification_failed{0};
    std::atomic<uint64_t> external_client_request_signatures_verified{0};
    std::atomic<uint64_t> peer_replicas_signature_verification_failed{0};
    std::atomic<uint64_t> peer_replicas_signatures_verified{0};
    std::atomic<uint64_t> signature_verification_failed_on_unrecognized_participant_id{0};
  };
  const Metrics& metrics() const { return metrics_; }

 private:
  void account(PrincipalId pid, bool result) const;

  const PrincipalId myId_;
  std::unique_ptr<concord::util::crypto::ISigner> mySigner_;
  std::map<PrincipalId, std::shared_ptr<concord::util::crypto::IVerifier>> verifiers_;
  ReplicasInfo replicasInfo_;
  mutable Metrics metrics_;
  mutable std::shared_mutex mutex_;
};

}  // namespace bftEngine::impl

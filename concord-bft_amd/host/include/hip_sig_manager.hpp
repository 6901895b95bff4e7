// concord::hip::HipSigManager — the reference's bftEngine::impl::SigManager
// (bftengine/src/bftengine/SigManager.hpp:32-142) extended, by derivation, with the batch entry
// point the engine exists for and GPU verifiers for every principal.
//
// It derives from the reference's own class and uses only its public API and protected members
// (verifiers_, mutex_, metrics_, metrics_component_, replicasInfo_, mySigner_, ...), so it
// compiles against the reference's SigManager.hpp (tests/test_reference_boundary.py) and links
// into corebft beside the reference's SigManager.cpp without redefining anything; header-only,
// no data members of its own.
//
//   init(...)          SigManager::init's signature and key mapping (SigManager.cpp:34-111): replica
//                      keys one index each, client keys one index per id set; every principal
//                      gets a GPU verifier (HipEdDSAVerifier / HipRSAVerifier, one object per
//                      distinct key as the reference shares them, :139-150).  The base class is
//                      constructed without verification keys when the CMF client-key map is
//                      available (the external clients' keys are recorded for
//                      getClientsPublicKeys as :151-156 records them), else with the RSA keys
//                      only (its constructor then builds and records them, :146-156).  An Ed25519 own key
//                      signs with EdDSASigner; an RSA one with the reference's RSASigner (:138).
//   verifySig          inherited unchanged: it calls IVerifier::verify, i.e. the GPU verifier
//                      (concurrent Ed25519 calls are coalesced into batches by the engine).
//   verifySigBatch     out[i] == verifySig(items[i]...) for every item, one GPU launch per
//                      algorithm; the five counters and the aggregator pushes move exactly as
//                      SigManager.cpp:197-238 moves them per call (a push on every failure and on
//                      every 1,000th success of each counter); with stopAtFirstFailure only the
//                      items up to the first failure are counted (the serial loops throw there).
//   setClientPublicKey SigManager.cpp:250-264 with a GPU verifier of the key's type (the base's
//                      version builds an RSAVerifier), and the key recorded in the CMF
//                      ClientsPublicKeys map exactly as the reference records it (:260).  The
//                      base method is NOT virtual: through a SigManager* the base's runs.  Key
//                      exchange therefore calls setClientPublicKeyOf(SigManager::instance(), ...)
//                      (the KeyExchangeManager.cpp:310-320 patch in INTEGRATION.md), which routes
//                      to this version when the instance is the HipSigManager that init() made.
//
// The CMF map: clientsPublicKeys_ is a namespace-scope global of the reference's SigManager.cpp
// (:25) whose type comes from the generated keys_and_signatures.cmf.hpp; builds that have that
// header (corebft, and the standalone build's restatement in ref_mirror/) define
// CBFT_WITH_CLIENT_KEYS_MAP.  Its version tag stays the reference's "1 = RSAVerifier" (:156): a
// reader of an Ed25519 entry must tell the key type from the key itself (32 raw bytes / 64 hex).
#pragma once

#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ReplicaConfig.hpp"
#include "ReplicasInfo.hpp"
#include "SigManager.hpp"
#include "hip_crypto.hpp"

#if defined(CBFT_WITH_CLIENT_KEYS_MAP)
#include "keys_and_signatures.cmf.hpp"
namespace bftEngine::impl {
extern concord::messages::keys_and_signatures::ClientsPublicKeys clientsPublicKeys_;  // SigManager.cpp:25
}
#endif

namespace concord::hip {

struct SigBatchItem {
  bftEngine::impl::PrincipalId pid;
  const char* data;
  size_t dataLength;
  const char* sig;
  uint16_t sigLength;
};

class HipSigManager : public bftEngine::impl::SigManager {
  using Base = bftEngine::impl::SigManager;
  using PrincipalId = bftEngine::impl::PrincipalId;
  using ReplicaId = bftEngine::impl::ReplicaId;
  using ReplicasInfo = bftEngine::impl::ReplicasInfo;
  using Fmt = concord::util::crypto::KeyFormat;
  using KeyList = std::vector<std::pair<std::string, Fmt>>;
  using Mapping = std::map<PrincipalId, uint16_t>;

 public:
  using ReplicaKeys = std::set<std::pair<PrincipalId, const std::string>>;
  using ClientKeys = std::set<std::pair<const std::string, std::set<uint16_t>>>;

  // SigManager::init (SigManager.cpp:96-111): builds the manager and makes it the process-wide
  // SigManager::instance(); the caller owns it.  Bad principal ids throw std::invalid_argument
  // (the reference asserts / terminates); keys that do not parse throw std::invalid_argument.
  static HipSigManager* init(ReplicaId myId, const std::string& mySigPrivateKey,
                             const ReplicaKeys& publicKeysOfReplicas, Fmt replicasKeysFormat,
                             const ClientKeys* publicKeysOfClients, Fmt clientsKeysFormat, ReplicasInfo& replicasInfo) {
    HipSigManager* sm = initInTesting(myId, mySigPrivateKey, publicKeysOfReplicas, replicasKeysFormat,
                                      publicKeysOfClients, clientsKeysFormat, replicasInfo);
    Base::instance(sm);
    registered() = sm;
    return sm;
  }
  ~HipSigManager() {
    if (registered() == this) registered() = nullptr;
  }

  // Key exchange's entry (KeyExchangeManager::loadClientPublicKey, KeyExchangeManager.cpp:316-322):
  // `sm` is SigManager::instance().  When it is the HipSigManager init() registered, the rotation
  // gets a GPU verifier of the key's type; otherwise the reference's own method runs.
  static void setClientPublicKeyOf(Base* sm, const std::string& key, PrincipalId id, Fmt format) {
    if (sm != nullptr && sm == static_cast<Base*>(registered()))
      registered()->setClientPublicKey(key, id, format);
    else if (sm != nullptr)
      sm->setClientPublicKey(key, id, format);
  }
  // the same without touching the instance (SigManager::initInTesting)
  static HipSigManager* initInTesting(ReplicaId myId, const std::string& mySigPrivateKey,
                                      const ReplicaKeys& publicKeysOfReplicas, Fmt replicasKeysFormat,
                                      const ClientKeys* publicKeysOfClients, Fmt clientsKeysFormat,
                                      ReplicasInfo& replicasInfo) {
    KeyList keys;
    Mapping mapping;
    uint16_t next = 0;
    const uint32_t lastReplica = replicasInfo.getNumberOfReplicas() + replicasInfo.getNumberOfRoReplicas() - 1;
    for (const auto& [id, key] : publicKeysOfReplicas) {
      if (id > lastReplica) throw std::invalid_argument("HipSigManager: replica key for id " + std::to_string(id));
      keys.emplace_back(key, replicasKeysFormat);
      mapping.insert({id, next++});
    }
    if (publicKeysOfClients) {
      const uint32_t lo = replicasInfo.getNumberOfRoReplicas() + replicasInfo.getNumberOfReplicas() +
                          replicasInfo.getNumOfClientProxies();
      const uint32_t hi = lo + replicasInfo.getNumberOfExternalClients() + replicasInfo.getNumberOfInternalClients() +
                          replicasInfo.getNumberOfClientServices() - 1;
      for (const auto& [key, ids] : *publicKeysOfClients) {
        if (key.empty()) throw std::invalid_argument("HipSigManager: empty client key");
        keys.emplace_back(key, clientsKeysFormat);
        for (const uint16_t e : ids) {
          if (e < lo || e > hi) throw std::invalid_argument("HipSigManager: invalid participant id " + std::to_string(e));
          mapping.insert({e, next});
        }
        ++next;
      }
    }
    const bool signing =
        bftEngine::ReplicaConfig::instance().clientTransactionSigningEnabled && publicKeysOfClients != nullptr;
    return new HipSigManager(myId, replicasInfo.getNumberOfReplicas(), {mySigPrivateKey, replicasKeysFormat}, keys,
                             mapping, signing, replicasInfo, rsaOnly({mySigPrivateKey, replicasKeysFormat}, keys, mapping));
  }

  // See the header comment.  Returns the index of the first failing item (items.size() if none).
  size_t verifySigBatch(const std::vector<SigBatchItem>& items, std::vector<bool>& out,
                        bool stopAtFirstFailure = false) const {
    LatencyHistogram::Scope timer(recorders().sig_manager_batch);
    const size_t n = items.size();
    out.assign(n, false);
    std::vector<std::shared_ptr<concord::util::crypto::IVerifier>> hold(n);
    {
      std::shared_lock lock(mutex_);
      for (size_t i = 0; i < n; i++) {
        auto it = verifiers_.find(items[i].pid);
        if (it != verifiers_.end()) hold[i] = it->second;  // alive past a concurrent key rotation
      }
    }
    std::vector<VerifyRequest> reqs(n);
    for (size_t i = 0; i < n; i++)
      reqs[i] = hold[i] ? VerifyRequest{hold[i].get(), items[i].data, items[i].dataLength, items[i].sig,
                                        items[i].sigLength}
                        : VerifyRequest{nullptr, nullptr, 0, nullptr, 0};
    verifyBatch(reqs, out);
    size_t first = n;
    for (size_t i = 0; i < n; i++) {
      if (!hold[i]) {
        out[i] = false;
        metrics_.sigVerificationFailedOnUnrecognizedParticipantId_++;
        metrics_component_.UpdateAggregator();
      } else {
        account(items[i].pid, out[i]);
      }
      if (!out[i] && first == n) {
        first = i;
        if (stopAtFirstFailure) break;
      }
    }
    return first;
  }

  // SigManager::setClientPublicKey with a GPU verifier of the key's type.
  void setClientPublicKey(const std::string& key, PrincipalId id, Fmt format) {
    if (!replicasInfo_.isIdOfExternalClient(id) && !replicasInfo_.isIdOfClientService(id)) return;  // "Illegal id"
    auto v = makeVerifier(key, format);  // throws on a bad key, like the reference (:258)
    std::unique_lock lock(mutex_);
    verifiers_.insert_or_assign(id, std::move(v));
#if defined(CBFT_WITH_CLIENT_KEYS_MAP)
    bftEngine::impl::clientsPublicKeys_.ids_to_keys[id] =
        concord::messages::keys_and_signatures::PublicKey{key, (uint8_t)format};  // SigManager.cpp:260
#endif
  }

  // The verifier object a principal's signatures go to (nullptr: unknown principal).
  std::shared_ptr<concord::util::crypto::IVerifier> verifierOf(PrincipalId id) const {
    std::shared_lock lock(mutex_);
    auto it = verifiers_.find(id);
    return it == verifiers_.end() ? nullptr : it->second;
  }

  // isClientTransactionSigningEnabled() is non-const in the reference
  bool clientSigningEnabled() const { return clientTransactionSigningEnabled_; }

  // Live values of the five counters (the aggregator only sees them at its pushes).
  struct CounterValues {
    uint64_t externalFailed, externalVerified, replicaFailed, replicaVerified, unrecognizedPid;
  };
  CounterValues counterValues() const {
    return {metrics_.externalClientReqSigVerificationFailed_.Get().Get(),
            metrics_.externalClientReqSigVerified_.Get().Get(), metrics_.replicaSigVerificationFailed_.Get().Get(),
            metrics_.replicaSigVerified_.Get().Get(), metrics_.sigVerificationFailedOnUnrecognizedParticipantId_.Get().Get()};
  }

 private:
  static HipSigManager*& registered() {
    static HipSigManager* sm = nullptr;
    return sm;
  }
  struct RsaSubset {  // what the base constructor may see: RSA keys only
    std::pair<std::string, Fmt> myKey;
    KeyList keys;
    Mapping mapping;
  };
  static RsaSubset rsaOnly(const std::pair<std::string, Fmt>& myKey, const KeyList& keys, const Mapping& mapping) {
    RsaSubset r;
    r.myKey = myKey;
    if (!myKey.first.empty() && privateKeyKind(myKey.first, myKey.second) != KeyKind::RSA) r.myKey.first.clear();
    std::map<uint16_t, uint16_t> renum;
    for (size_t k = 0; k < keys.size(); k++)
      if (publicKeyKind(keys[k].first, keys[k].second) == KeyKind::RSA) {
        renum[(uint16_t)k] = (uint16_t)r.keys.size();
        r.keys.push_back(keys[k]);
      }
    for (const auto& [pid, k] : mapping)
      if (auto it = renum.find(k); it != renum.end()) r.mapping.insert({pid, it->second});
    return r;
  }

  // With the CMF client-key map at hand (CBFT_WITH_CLIENT_KEYS_MAP) the base is constructed with
  // NO verification keys -- it would build a Crypto++ RSAVerifier per RSA key (SigManager.cpp:146)
  // only for this constructor to replace it -- and the external clients' keys are entered into
  // the map here, as SigManager.cpp:151-156 enters them.  Without the map the base gets the RSA
  // subset, which it records itself.
  HipSigManager(PrincipalId myId, uint16_t numReplicas, const std::pair<std::string, Fmt>& myKey, const KeyList& keys,
                const Mapping& mapping, bool signing, ReplicasInfo& replicasInfo, const RsaSubset& rsa)
#if defined(CBFT_WITH_CLIENT_KEYS_MAP)
      : Base(myId, numReplicas, rsa.myKey, KeyList{}, Mapping{}, signing, replicasInfo) {
    for (const auto& [pid, k] : mapping)
      if (k < keys.size() && replicasInfo_.isIdOfExternalClient(pid))
        bftEngine::impl::clientsPublicKeys_.ids_to_keys[pid] =
            concord::messages::keys_and_signatures::PublicKey{keys[k].first, (uint8_t)keys[k].second};
#else
      : Base(myId, numReplicas, rsa.myKey, rsa.keys, rsa.mapping, signing, replicasInfo) {
#endif
    if (!myKey.first.empty() && !mySigner_) mySigner_ = makeSigner(myKey.first, myKey.second);
    std::map<uint16_t, std::shared_ptr<concord::util::crypto::IVerifier>> byIndex;
    for (const auto& [pid, k] : mapping) {
      if (k >= keys.size()) throw std::invalid_argument("HipSigManager: key index out of range");
      auto it = byIndex.find(k);
      if (it == byIndex.end()) it = byIndex.emplace(k, makeVerifier(keys[k].first, keys[k].second)).first;
      verifiers_[pid] = it->second;
    }
  }

  // SigManager.cpp:213-236, per item
  void account(PrincipalId pid, bool result) const {
    const bool external = replicasInfo_.isIdOfExternalClient(pid);
    if (!external && !replicasInfo_.isIdOfReplica(pid) && !replicasInfo_.isIdOfPeerRoReplica(pid))
      throw std::logic_error("HipSigManager: pid is neither a replica nor an external client");  // ConcordAssert
    if (!result) {
      (external ? metrics_.externalClientReqSigVerificationFailed_ : metrics_.replicaSigVerificationFailed_)++;
      metrics_component_.UpdateAggregator();
    } else {
      auto& c = external ? metrics_.externalClientReqSigVerified_ : metrics_.replicaSigVerified_;
      c++;
      if ((c.Get().Get() % updateMetricsAggregatorThresh) == 0) metrics_component_.UpdateAggregator();
    }
  }
};

}  // namespace concord::hip

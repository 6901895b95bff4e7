// Standalone-build restatement of bftengine/src/bftengine/ReplicasInfo.hpp:23-110 /
// ReplicasInfo.cpp:50-140: the principal-id space (replicas, read-only replicas, client proxies,
// external clients with the operator last, client services, one internal client per replica)
// and the id predicates SigManager and ClientRequestMsg::validate use, with the reference's
// names and constness.  The reference builds it from ReplicaConfig; this restatement from the
// same fields (ReplicaIdsConfig).  See ../README.md.
#pragma once

#include <cstdint>
#include <set>

#include "PrimitiveTypes.hpp"

namespace bftEngine {
namespace impl {

// The ReplicaConfig fields ReplicasInfo reads (ReplicaConfig.hpp; ReplicasInfo.cpp:50-65).
struct ReplicaIdsConfig {
  ReplicaId replicaId = 0;
  uint16_t fVal = 1;
  uint16_t cVal = 0;
  uint16_t numReplicas = 4;  // must be 3f + 2c + 1
  uint16_t numRoReplicas = 0;
  uint16_t numOfClientProxies = 0;
  uint16_t numOfExternalClients = 0;
  uint16_t numOfClientServices = 0;
  bool operatorEnabled_ = false;
};

class ReplicasInfo {
 public:
  explicit ReplicasInfo(const ReplicaIdsConfig& config);  // throws std::invalid_argument if n != 3f+2c+1
  ReplicaId myId() const { return _myId; }
  int16_t numberOfReplicas() const { return _numberOfReplicas; }
  int16_t fVal() const { return _fVal; }
  int16_t cVal() const { return _cVal; }
  bool isIdOfReplica(NodeIdType id) const { return id < _numberOfReplicas; }
  bool isIdOfPeerReplica(NodeIdType id) const { return id < _numberOfReplicas && id != _myId; }
  bool isIdOfPeerRoReplica(NodeIdType id) const { return _idsOfPeerROReplicas.count(id) != 0; }
  bool isIdOfClientProxy(PrincipalId id) const { return _idsOfClientProxies.count(id) != 0; }
  bool isIdOfExternalClient(PrincipalId id) const { return _idsOfExternalClients.count(id) != 0; }
  bool isIdOfInternalClient(PrincipalId id) const { return _idsOfInternalClients.count(id) != 0; }
  bool isIdOfClientService(NodeIdType id) { return _idsOfClientServices.count(id) != 0; }
  bool isValidPrincipalId(PrincipalId id) const { return id <= _maxValidPrincipalId; }
  uint16_t getNumberOfReplicas() { return _numberOfReplicas; }
  uint16_t getNumberOfRoReplicas() { return _numberOfRoReplicas; }
  uint16_t getNumOfClientProxies() { return _numOfClientProxies; }
  uint16_t getNumberOfExternalClients() { return _numberOfExternalClients; }
  uint16_t getNumberOfInternalClients() { return _numberOfInternalClients; }
  uint16_t getNumberOfClientServices() { return _numberOfClientServices; }

 private:
  const ReplicaId _myId;
  const uint16_t _numberOfReplicas, _numberOfRoReplicas, _numOfClientProxies, _numberOfExternalClients,
      _numberOfClientServices, _numberOfInternalClients, _maxValidPrincipalId, _fVal, _cVal;
  std::set<PrincipalId> _idsOfPeerROReplicas, _idsOfClientProxies, _idsOfExternalClients, _idsOfClientServices,
      _idsOfInternalClients;
};

}  // namespace impl
}  // namespace bftEngine

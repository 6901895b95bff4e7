// Standalone-build restatement of ReplicasInfo.cpp:50-143 (see ReplicasInfo.hpp).
#include "ReplicasInfo.hpp"

#include <stdexcept>

namespace bftEngine {
namespace impl {

ReplicasInfo::ReplicasInfo(const ReplicaIdsConfig& c)
    : _myId(c.replicaId),
      _numberOfReplicas(c.numReplicas),
      _numberOfRoReplicas(c.numRoReplicas),
      _numOfClientProxies(c.numOfClientProxies),
      _numberOfExternalClients(c.numOfExternalClients),
      _numberOfClientServices(c.numOfClientServices),
      _numberOfInternalClients(c.numReplicas),
      _maxValidPrincipalId((uint16_t)(c.numReplicas + c.numRoReplicas + c.numOfClientProxies +
                                      c.numOfExternalClients + c.numReplicas + c.numOfClientServices - 1)),
      _fVal(c.fVal),
      _cVal(c.cVal) {
  if (c.numReplicas != 3 * c.fVal + 2 * c.cVal + 1)
    throw std::invalid_argument("ReplicasInfo: numReplicas != 3f + 2c + 1");  // ReplicasInfo.cpp:143
  const uint32_t n = c.numReplicas, ro = c.numRoReplicas, px = c.numOfClientProxies, ext = c.numOfExternalClients,
                 svc = c.numOfClientServices, op = c.operatorEnabled_ ? 1u : 0u;
  for (uint32_t i = n; i < n + ro; i++) _idsOfPeerROReplicas.insert((PrincipalId)i);
  for (uint32_t i = n + ro; i < n + ro + px; i++) _idsOfClientProxies.insert((PrincipalId)i);
  const uint32_t es = n + ro + px, ee = es + ext;
  for (uint32_t i = es; i < ee - op; i++) _idsOfExternalClients.insert((PrincipalId)i);
  _idsOfExternalClients.insert((PrincipalId)(ee + svc - 1));  // :115 (the operator's id when enabled)
  for (uint32_t i = ee - op; i < ee - op + svc; i++) _idsOfClientServices.insert((PrincipalId)i);
  for (uint32_t i = ee + svc; i < ee + svc + n; i++) _idsOfInternalClients.insert((PrincipalId)i);
}

}  // namespace impl
}  // namespace bftEngine

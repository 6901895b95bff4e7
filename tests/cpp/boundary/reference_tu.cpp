// Compiled against the REFERENCE's headers (not ref_mirror/) by tests/test_reference_boundary.py:
// the integration a concord-bft maintainer would build.  It instantiates everything header-only
// in the product (HipSigManager derives from the reference's bftEngine::impl::SigManager) and
// uses the product through the reference's own types, and pins the wire restatements in
// request_batch.hpp to the reference's packed structs (bftengine/include/bftengine/ClientMsgs.hpp).
#include <cstddef>
#include <memory>

#include "ClientMsgs.hpp"
#include "PreProcessBatchRequestMsg.hpp"
#include "messages/PrePrepareMsg.hpp"
#include "ReplicasInfo.hpp"
#include "SigManager.hpp"
#include "crypto_utils.hpp"
#include "hip_crypto.hpp"
#include "hip_sig_manager.hpp"
#include "request_batch.hpp"
#include "threshsign/IThresholdVerifier.h"
#include "threshsign/bls_hip.hpp"

#define SAME_FIELD(A, B, f) static_assert(offsetof(A, f) == offsetof(B, f) && sizeof(A::f) == sizeof(B::f), #f)
using RefReq = bftEngine::ClientRequestMsgHeader;
using OurReq = concord::hip::wire::ClientRequestMsgHeader;
static_assert(sizeof(RefReq) == sizeof(OurReq), "ClientRequestMsgHeader size");
SAME_FIELD(RefReq, OurReq, msgType);
SAME_FIELD(RefReq, OurReq, spanContextSize);
SAME_FIELD(RefReq, OurReq, idOfClientProxy);
SAME_FIELD(RefReq, OurReq, flags);
SAME_FIELD(RefReq, OurReq, result);
SAME_FIELD(RefReq, OurReq, reqSeqNum);
SAME_FIELD(RefReq, OurReq, requestLength);
SAME_FIELD(RefReq, OurReq, timeoutMilli);
SAME_FIELD(RefReq, OurReq, cidLength);
SAME_FIELD(RefReq, OurReq, reqSignatureLength);
SAME_FIELD(RefReq, OurReq, extraDataLength);
using RefBatch = bftEngine::ClientBatchRequestMsgHeader;
using OurBatch = concord::hip::wire::ClientBatchRequestMsgHeader;
static_assert(sizeof(RefBatch) == sizeof(OurBatch), "ClientBatchRequestMsgHeader size");
SAME_FIELD(RefBatch, OurBatch, msgType);
SAME_FIELD(RefBatch, OurBatch, cidSize);
SAME_FIELD(RefBatch, OurBatch, clientId);
SAME_FIELD(RefBatch, OurBatch, numOfMessagesInBatch);
SAME_FIELD(RefBatch, OurBatch, dataSize);

// PreProcessRequestMsg::Header is public; the batch's and PrePrepareMsg's headers are protected,
// reached through a derived class as the reference's own sizeOfHeader<> friends do.
struct RefPPBatch : preprocessor::PreProcessBatchRequestMsg {
  using H = Header;
};
struct RefPrePrepare : bftEngine::impl::PrePrepareMsg {
  using H = Header;
  static constexpr uint32_t kMaxBatch = MAX_BATCH_SIZE;  // MessageBase's, protected
};
using RefPPReq = preprocessor::PreProcessRequestMsg::Header;
using OurPPReq = concord::hip::wire::PreProcessRequestMsgHeader;
static_assert(sizeof(RefPPReq) == sizeof(OurPPReq), "PreProcessRequestMsg::Header size");
SAME_FIELD(RefPPReq, OurPPReq, header);
SAME_FIELD(RefPPReq, OurPPReq, reqType);
SAME_FIELD(RefPPReq, OurPPReq, reqSeqNum);
SAME_FIELD(RefPPReq, OurPPReq, clientId);
SAME_FIELD(RefPPReq, OurPPReq, reqOffsetInBatch);
SAME_FIELD(RefPPReq, OurPPReq, senderId);
SAME_FIELD(RefPPReq, OurPPReq, requestLength);
SAME_FIELD(RefPPReq, OurPPReq, cidLength);
SAME_FIELD(RefPPReq, OurPPReq, spanContextSize);
SAME_FIELD(RefPPReq, OurPPReq, reqRetryId);
SAME_FIELD(RefPPReq, OurPPReq, reqSignatureLength);
SAME_FIELD(RefPPReq, OurPPReq, primaryBlockId);
SAME_FIELD(RefPPReq, OurPPReq, result);
SAME_FIELD(RefPPReq, OurPPReq, viewNum);
using RefPPB = RefPPBatch::H;
using OurPPB = concord::hip::wire::PreProcessBatchRequestMsgHeader;
static_assert(sizeof(RefPPB) == sizeof(OurPPB), "PreProcessBatchRequestMsg::Header size");
SAME_FIELD(RefPPB, OurPPB, header);
SAME_FIELD(RefPPB, OurPPB, reqType);
SAME_FIELD(RefPPB, OurPPB, clientId);
SAME_FIELD(RefPPB, OurPPB, senderId);
SAME_FIELD(RefPPB, OurPPB, cidLength);
SAME_FIELD(RefPPB, OurPPB, numOfMessagesInBatch);
SAME_FIELD(RefPPB, OurPPB, requestsSize);
SAME_FIELD(RefPPB, OurPPB, viewNum);
using RefPP = RefPrePrepare::H;
using OurPP = concord::hip::wire::PrePrepareMsgHeader;
static_assert(sizeof(RefPP) == sizeof(OurPP), "PrePrepareMsg::Header size");
SAME_FIELD(RefPP, OurPP, viewNum);
SAME_FIELD(RefPP, OurPP, seqNum);
SAME_FIELD(RefPP, OurPP, epochNum);
SAME_FIELD(RefPP, OurPP, flags);
SAME_FIELD(RefPP, OurPP, batchCidLength);
SAME_FIELD(RefPP, OurPP, time);
SAME_FIELD(RefPP, OurPP, digestOfRequests);
SAME_FIELD(RefPP, OurPP, numberOfRequests);
SAME_FIELD(RefPP, OurPP, endLocationOfLastRequest);
static_assert((int)bftEngine::impl::MsgCode::PreProcessRequest == concord::hip::wire::kPreProcessRequestMsgType &&
                  (int)bftEngine::impl::MsgCode::PreProcessBatchRequest == concord::hip::wire::kPreProcessBatchRequestMsgType,
              "message codes");
static_assert(RefPrePrepare::kMaxBatch == concord::hip::wire::kMaxClientBatchSize, "MAX_BATCH_SIZE");

// The GPU verifiers are the reference's IVerifier; the manager is the reference's SigManager.
static_assert(std::is_base_of_v<concord::util::crypto::IVerifier, concord::hip::HipEdDSAVerifier>);
static_assert(std::is_base_of_v<concord::util::crypto::IVerifier, concord::hip::HipRSAVerifier>);
static_assert(std::is_base_of_v<concord::util::crypto::ISigner, concord::hip::EdDSASigner>);
static_assert(std::is_base_of_v<bftEngine::impl::SigManager, concord::hip::HipSigManager>);
static_assert(std::is_base_of_v<IThresholdVerifier, BLS::Hip::BlsThresholdVerifier>);
static_assert(std::is_base_of_v<IThresholdAccumulator, BLS::Hip::BlsAccumulatorBase>);
static_assert(std::is_base_of_v<IThresholdSigner, BLS::Hip::BlsThresholdSigner>);

namespace concord::hip::boundary {
// What bftengine does with the plugin, spelled with the reference's types (never run here).
bool useThroughReferenceTypes(bftEngine::impl::ReplicasInfo& ri, const std::string& key, const char* msg, size_t len,
                              const char* sig) {
  std::shared_ptr<concord::util::crypto::IVerifier> v = makeVerifier(key, concord::util::crypto::KeyFormat::PemFormat);
  HipSigManager::ReplicaKeys replicas{{0, key}};
  bftEngine::impl::SigManager* sm = HipSigManager::init(0, "", replicas, concord::util::crypto::KeyFormat::PemFormat,
                                                        nullptr, concord::util::crypto::KeyFormat::PemFormat, ri);
  auto* hip = static_cast<HipSigManager*>(sm);
  std::vector<bool> out;
  hip->verifySigBatch({{0, msg, len, sig, 64}}, out);
  validatePrePrepareRequests(msg, len, ri, *hip);
  // PreProcessor's non-primary batch (PreProcessor.cpp:877-902), through the batched walker
  validatePreProcessBatchRequestMsg(msg, len, 1, ri, *hip);
  checkPreProcessBatchReqMsgCorrectness(msg, len, PreProcessReplicaState{}, ri, *hip);
  // KeyExchangeManager::loadClientPublicKey (KeyExchangeManager.cpp:316-322), patched as in
  // the rotation reaches the GPU verifiers through SigManager::instance()
  HipSigManager::setClientPublicKeyOf(bftEngine::impl::SigManager::instance(), key, 5,
                                      concord::util::crypto::KeyFormat::PemFormat);
  return v->verify(std::string(msg, len), std::string(sig, 64)) && sm->verifySig(0, msg, len, sig, 64);
}
}  // namespace concord::hip::boundary

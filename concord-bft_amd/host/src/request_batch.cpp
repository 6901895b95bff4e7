// Batched signature checks over the reference's message layouts (see request_batch.hpp).
#include "request_batch.hpp"

#include <openssl/evp.h>

#include <cstring>
#include <set>

namespace concord::hip {

using namespace wire;

uint64_t clientRequestMsgSize(const ClientRequestMsgHeader& h) {
  return sizeof(ClientRequestMsgHeader) + (uint64_t)h.spanContextSize + h.requestLength + h.cidLength +
         h.reqSignatureLength + h.extraDataLength;
}

namespace {

ClientRequestMsgHeader readHeader(const char* p) {
  ClientRequestMsgHeader h;
  std::memcpy(&h, p, sizeof h);  // packed wire struct, possibly unaligned in a batch
  return h;
}

enum class Check { Fail, Accept, Verify };

// ClientRequestMsg::validateImp (ClientRequestMsg.cpp:99-214) without the signature itself:
// Fail (with the reference's message), Accept (no signature to check) or Verify (item filled).
Check checkRequest(const ClientRequestView& r, const ReplicasInfo& repInfo, const HipSigManager& sm, std::string& err,
                   SigBatchItem& item) {
  const uint64_t msgSize = r.size;
  if (msgSize < sizeof(ClientRequestMsgHeader)) {
    err = "Invalid Message Size";
    return Check::Fail;
  }
  const ClientRequestMsgHeader h = readHeader(r.body);
  if (msgSize < sizeof(ClientRequestMsgHeader) + (uint64_t)h.spanContextSize) {
    err = "Invalid Message Size";
    return Check::Fail;
  }
  const PrincipalId clientId = h.idOfClientProxy;
  if ((h.flags & RECONFIG_FLAG) == 0 && r.senderId == repInfo.myId()) {  // a ConcordAssert there
    err = "request sent by this replica";
    return Check::Fail;
  }
  const uint64_t minMsgSize =
      sizeof(ClientRequestMsgHeader) + (uint64_t)h.cidLength + h.spanContextSize + h.reqSignatureLength;
  if (msgSize < minMsgSize) {
    err = "Invalid msgSize";
    return Check::Fail;
  }
  uint16_t expectedSigLen = 0;
  const bool signing = sm.clientSigningEnabled();
  const bool external = repInfo.isIdOfExternalClient(clientId);
  bool doSigVerify = false;
  const bool emptyReq = h.requestLength == 0;
  if ((h.flags & RECONFIG_FLAG) != 0 && (repInfo.isIdOfReplica(clientId) || repInfo.isIdOfPeerRoReplica(clientId)))
    return Check::Accept;  // verified by the reconfiguration handler
  if (!repInfo.isValidPrincipalId(clientId)) {
    err = "Invalid clientId " + std::to_string(clientId);
    return Check::Fail;
  }
  if (!repInfo.isValidPrincipalId(r.senderId)) {
    err = "Invalid senderId " + std::to_string(r.senderId);
    return Check::Fail;
  }
  if (external) {
    if ((h.flags & RECONFIG_FLAG) != 0) {
      expectedSigLen = h.reqSignatureLength;  // the operator's own signature, checked elsewhere
    } else if (signing) {
      if (!emptyReq) {
        expectedSigLen = sm.getSigLength(clientId);
        if (expectedSigLen == 0) {
          err = "Invalid expectedSigLen";
          return Check::Fail;
        }
        if ((h.flags & HAS_PRE_PROCESSED_FLAG) == 0) doSigVerify = true;
      }
    }
  }
  if (expectedSigLen != h.reqSignatureLength) {
    err = "Unexpected request signature length";
    return Check::Fail;
  }
  const uint64_t expectedMsgSize = sizeof(ClientRequestMsgHeader) + (uint64_t)h.requestLength + h.cidLength +
                                   h.spanContextSize + expectedSigLen + h.extraDataLength;
  if (msgSize != expectedMsgSize) {
    err = "Invalid msgSize";
    return Check::Fail;
  }
  if (!doSigVerify) return Check::Accept;
  const char* req = r.body + sizeof(ClientRequestMsgHeader) + h.spanContextSize;  // requestBuf()
  item = SigBatchItem{clientId, req, h.requestLength, req + h.requestLength + h.cidLength,  // requestSignature()
                      h.reqSignatureLength};
  return Check::Verify;
}

}  // namespace

RequestValidation validateClientRequests(const std::vector<ClientRequestView>& reqs, const ReplicasInfo& repInfo,
                                         const HipSigManager& sm, bool stopAtFirstFailure) {
  RequestValidation out;
  const size_t n = reqs.size();
  out.ok.assign(n, false);
  out.error.assign(n, std::string());
  out.firstFailure = n;
  std::vector<SigBatchItem> items;
  std::vector<size_t> owner;
  for (size_t i = 0; i < n; i++) {
    SigBatchItem it{};
    const Check c = checkRequest(reqs[i], repInfo, sm, out.error[i], it);
    if (c == Check::Fail) {
      if (out.firstFailure == n) out.firstFailure = i;
      if (stopAtFirstFailure) break;
      continue;
    }
    out.ok[i] = true;
    if (c == Check::Verify) {
      items.push_back(it);
      owner.push_back(i);
    }
  }
  // one signature batch; with stopAtFirstFailure only the requests before the first structural
  // failure were collected, and the counters stop at the first bad signature (the serial loop
  // throws there)
  std::vector<bool> verdict;
  if (!items.empty()) sm.verifySigBatch(items, verdict, stopAtFirstFailure);
  for (size_t k = 0; k < items.size(); k++) {
    if (verdict[k]) continue;
    const size_t i = owner[k];
    out.ok[i] = false;
    out.error[i] = "Signature verification failed for: clientId " + std::to_string(items[k].pid);
    if (i < out.firstFailure) out.firstFailure = i;
  }
  if (stopAtFirstFailure)
    for (size_t i = out.firstFailure + 1; i < n; i++) {  // never validated by the serial loop
      out.ok[i] = false;
      out.error[i] = "not validated (an earlier request failed)";
    }
  return out;
}

size_t validatePrePrepareRequests(const char* body, uint64_t size, const ReplicasInfo& repInfo,
                                  const HipSigManager& sm) {
  if (size < sizeof(PrePrepareMsgHeader)) throw std::runtime_error("PrePrepareMsg::validate: basic");
  PrePrepareMsgHeader h;
  std::memcpy(&h, body, sizeof h);
  if (size < sizeof(PrePrepareMsgHeader) + (uint64_t)h.header.spanContextSize)
    throw std::runtime_error("PrePrepareMsg::validate: basic");
  const uint64_t end = h.endLocationOfLastRequest;
  const uint64_t shift = sizeof(PrePrepareMsgHeader) + h.batchCidLength + h.header.spanContextSize;  // payloadShift
  // the structural conditions of PrePrepareMsg::validate that the request walk relies on
  // (PrePrepareMsg.cpp:106-108) and checkRequests (:258-283)
  bool good = end <= size && h.numberOfRequests != 0 && h.numberOfRequests < end && shift < end;
  std::vector<ClientRequestView> reqs;
  if (good) {
    uint64_t i = shift;
    for (uint16_t remain = h.numberOfRequests; remain > 0; remain--) {
      if (i + sizeof(ClientRequestMsgHeader) > end) {
        good = false;
        break;
      }
      const ClientRequestMsgHeader rh = readHeader(body + i);
      const uint64_t rs = clientRequestMsgSize(rh);
      reqs.push_back({body + i, rs, rh.idOfClientProxy});  // ClientRequestMsg(ClientRequestMsgHeader*)
      i += rs;
      if (remain > 1 ? i >= end : i != end) {
        good = false;
        break;
      }
    }
  }
  if (!good) throw std::runtime_error("PrePrepareMsg::validate: advanced");
  if (sm.clientSigningEnabled()) {
    RequestValidation v = validateClientRequests(reqs, repInfo, sm, true);
    if (v.firstFailure < reqs.size()) throw std::runtime_error(v.error[v.firstFailure]);
  }
  return reqs.size();
}

RequestValidation validateClientBatchRequestMsg(const char* body, uint64_t size, const ReplicasInfo& repInfo,
                                                const HipSigManager& sm) {
  // ClientBatchRequestMsg::validate + checkElements
  if (size < sizeof(ClientBatchRequestMsgHeader)) throw std::runtime_error("ClientBatchRequestMsg::validate");
  ClientBatchRequestMsgHeader h;
  std::memcpy(&h, body, sizeof h);
  if (size < sizeof(ClientBatchRequestMsgHeader) + (uint64_t)h.dataSize)
    throw std::runtime_error("ClientBatchRequestMsg::validate");
  if (!h.numOfMessagesInBatch || h.numOfMessagesInBatch > kMaxClientBatchSize)
    throw std::runtime_error("ClientBatchRequestMsg::validate: checkElements");
  const bool signing = sm.clientSigningEnabled();
  uint64_t pos = sizeof(ClientBatchRequestMsgHeader) + h.cidSize;
  std::vector<ClientRequestView> reqs;
  for (uint32_t k = 0; k < h.numOfMessagesInBatch; k++) {
    if (pos + sizeof(ClientRequestMsgHeader) > size) throw std::runtime_error("ClientBatchRequestMsg: truncated");
    const ClientRequestMsgHeader rh = readHeader(body + pos);
    const uint16_t expectedSigLen = signing ? sm.getSigLength(rh.idOfClientProxy) : 0;
    if (expectedSigLen != rh.reqSignatureLength || size < rh.requestLength || size < rh.cidLength)
      throw std::runtime_error("ClientBatchRequestMsg::validate: checkElements");
    // elements carry no extra data (ClientBatchRequestMsg.cpp: dataPosition advances by header,
    // span, request, cid and signature); each is rebuilt as its own message whose sender is the
    // batch's sender
    const uint64_t rs = sizeof(ClientRequestMsgHeader) + (uint64_t)rh.spanContextSize + rh.requestLength +
                        rh.cidLength + rh.reqSignatureLength;
    if (pos + rs > size || rh.extraDataLength != 0) throw std::runtime_error("ClientBatchRequestMsg: truncated");
    reqs.push_back({body + pos, rs, h.clientId});
    pos += rs;
  }
  return validateClientRequests(reqs, repInfo, sm, false);
}

namespace {

// One element of a PreProcessBatchRequestMsg: its header and where it starts.
struct PreProcessElement {
  PreProcessRequestMsgHeader h;
  const char* start;
};

// Walk the elements of a PreProcessBatchRequestMsg (getPreProcessRequestMsgs,
// PreProcessBatchRequestMsg.cpp:114-147), bounds-checked: each element is its header, span,
// request, cid and signature.  Throws when an element does not fit in the message.
std::vector<PreProcessElement> preProcessElements(const char* body, uint64_t size,
                                                  const PreProcessBatchRequestMsgHeader& bh) {
  std::vector<PreProcessElement> out;
  out.reserve(bh.numOfMessagesInBatch);
  uint64_t pos = sizeof(PreProcessBatchRequestMsgHeader) + (uint64_t)bh.cidLength;
  for (uint32_t k = 0; k < bh.numOfMessagesInBatch; k++) {
    if (pos + sizeof(PreProcessRequestMsgHeader) > size)
      throw std::runtime_error("PreProcessBatchRequestMsg: element header outside the message");
    PreProcessElement e;
    std::memcpy(&e.h, body + pos, sizeof e.h);
    e.start = body + pos;
    const uint64_t es = sizeof(PreProcessRequestMsgHeader) + (uint64_t)e.h.spanContextSize + e.h.requestLength +
                        e.h.cidLength + e.h.reqSignatureLength;
    if (pos + es > size) throw std::runtime_error("PreProcessBatchRequestMsg: element outside the message");
    out.push_back(e);
    pos += es;
  }
  return out;
}

}  // namespace

void validatePreProcessBatchRequestMsg(const char* body, uint64_t size, PrincipalId networkSender,
                                       const ReplicasInfo& repInfo, const HipSigManager& sm) {
  static const char* kWhat = "void preprocessor::PreProcessBatchRequestMsg::validate(const ReplicasInfo&) const";
  if (size < sizeof(PreProcessBatchRequestMsgHeader)) throw std::runtime_error(kWhat);
  PreProcessBatchRequestMsgHeader bh;
  std::memcpy(&bh, body, sizeof bh);
  if (size < sizeof(PreProcessBatchRequestMsgHeader) + (uint64_t)bh.requestsSize) throw std::runtime_error(kWhat);
  if (bh.header.msgType != kPreProcessBatchRequestMsgType) throw std::runtime_error(kWhat);
  if (networkSender == repInfo.myId()) throw std::runtime_error(kWhat);
  // checkElements (PreProcessBatchRequestMsg.cpp:63-89)
  if (!bh.numOfMessagesInBatch || bh.numOfMessagesInBatch > kMaxClientBatchSize) throw std::runtime_error(kWhat);
  const bool signing = sm.clientSigningEnabled();
  for (const PreProcessElement& e : preProcessElements(body, size, bh)) {
    const uint16_t expectedSigLen = signing ? sm.getSigLength(e.h.clientId) : 0;
    if (expectedSigLen != e.h.reqSignatureLength || size < e.h.requestLength || size < e.h.cidLength)
      throw std::runtime_error(kWhat);
  }
}

PreProcessBatchValidation checkPreProcessBatchReqMsgCorrectness(const char* body, uint64_t size,
                                                                const PreProcessReplicaState& state,
                                                                const ReplicasInfo& repInfo,
                                                                const HipSigManager& sm) {
  PreProcessBatchValidation out;
  if (size < sizeof(PreProcessBatchRequestMsgHeader))
    throw std::runtime_error("PreProcessBatchRequestMsg: shorter than its header");
  PreProcessBatchRequestMsgHeader bh;
  std::memcpy(&bh, body, sizeof bh);
  const std::vector<PreProcessElement> elems = preProcessElements(body, size, bh);  // getPreProcessRequestMsgs
  if (bh.viewNum != state.currentView) {
    out.viewMismatch = true;
    return out;
  }
  const size_t n = elems.size();
  out.outcome.assign(n, PreProcessOutcome::Valid);
  out.error.assign(n, std::string());
  // checkPreProcessReqPrerequisites (PreProcessor.cpp:848-873): replica state only
  const bool prerequisites = !state.collectingState && !state.isCurrentPrimary && state.currentViewIsActive;
  std::vector<SigBatchItem> items;
  std::vector<size_t> owner;
  for (size_t k = 0; k < n; k++) {
    if (!prerequisites) {
      out.outcome[k] = PreProcessOutcome::Ignored;
      out.ignored++;
      continue;
    }
    // PreProcessRequestMsg::validate (PreProcessRequestMsg.cpp:80-113) on the rebuilt message:
    // its size and type hold by construction; its sender is the batch header's senderId
    const PreProcessRequestMsgHeader& h = elems[k].h;
    if (bh.senderId == repInfo.myId()) {
      out.outcome[k] = PreProcessOutcome::Invalid;
      out.error[k] = "void preprocessor::PreProcessRequestMsg::validate(const ReplicasInfo&) const";
      out.invalid++;
      continue;
    }
    if (h.reqSignatureLength == 0) continue;  // no signature: valid
    if (!sm.clientSigningEnabled())           // a ConcordAssert in the reference
      throw std::logic_error("PreProcessRequestMsg::validate: signed request with client signing disabled");
    const char* req = elems[k].start + sizeof(PreProcessRequestMsgHeader) + h.spanContextSize;  // requestBuf()
    // verifySig(header->clientId, ...): the rebuilt message's clientId is the batch's
    items.push_back(SigBatchItem{bh.clientId, req, h.requestLength, req + h.requestLength + h.cidLength,
                                 h.reqSignatureLength});
    owner.push_back(k);
  }
  std::vector<bool> verdict;
  if (!items.empty()) sm.verifySigBatch(items, verdict, false);  // every element is validated
  for (size_t j = 0; j < items.size(); j++) {
    if (verdict[j]) continue;
    const size_t k = owner[j];
    const PreProcessRequestMsgHeader& h = elems[k].h;
    out.outcome[k] = PreProcessOutcome::Invalid;
    // the reference's text: "Signature verification failed for: " << KVLOG(header->clientId, ...),
    // KVARGS naming each argument by its source text and KvLog opening with a space
    // (PreProcessRequestMsg.cpp:108-109, util/include/kvstream.h, util/include/macros.h)
    out.error[k] = "Signature verification failed for:  header->clientId: " + std::to_string(bh.clientId) +
                   ", header->reqSeqNum: " + std::to_string(h.reqSeqNum) + ", header->requestLength: " +
                   std::to_string(h.requestLength) +
                   ", header->reqSignatureLength: " + std::to_string(h.reqSignatureLength);
    out.invalid++;
  }
  out.valid = out.ignored == 0 && out.invalid == 0;
  return out;
}

std::string preProcessResultHash(const char* result, uint32_t len, uint32_t resultCode, uint16_t clientId,
                                 uint64_t reqSeqNum) {
  unsigned char md[32];
  unsigned int mdlen = 0;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  bool ok = ctx && EVP_DigestInit_ex(ctx, EVP_sha3_256(), nullptr) == 1;
  if (ok && resultCode == 0) ok = EVP_DigestUpdate(ctx, result, len) == 1;  // OperationResult::SUCCESS
  ok = ok && EVP_DigestUpdate(ctx, &resultCode, sizeof resultCode) == 1 &&
       EVP_DigestUpdate(ctx, &clientId, sizeof clientId) == 1 && EVP_DigestUpdate(ctx, &reqSeqNum, sizeof reqSeqNum) == 1 &&
       EVP_DigestFinal_ex(ctx, md, &mdlen) == 1;
  EVP_MD_CTX_free(ctx);
  if (!ok || mdlen != 32) throw std::runtime_error("SHA3-256 failed");
  return std::string(reinterpret_cast<char*>(md), 32);
}

namespace {
uint32_t be32(const char* p) {
  const auto* u = reinterpret_cast<const uint8_t*>(p);
  return (uint32_t)u[0] << 24 | (uint32_t)u[1] << 16 | (uint32_t)u[2] << 8 | u[3];
}
struct ResultSig {
  uint16_t sender;
  uint32_t result;
  std::string sig;
  bool operator<(const ResultSig& o) const { return sender < o.sender; }  // PreProcessResultMsg.hpp:78
};
}  // namespace

std::optional<std::string> validatePreProcessResultSignatures(const char* body, uint64_t size, ReplicaId myReplicaId,
                                                              int16_t fVal, const HipSigManager& sm) {
  if (size < sizeof(ClientRequestMsgHeader)) throw std::runtime_error("PreProcessResultMsg: short message");
  const ClientRequestMsgHeader h = readHeader(body);
  if (clientRequestMsgSize(h) > size) throw std::runtime_error("PreProcessResultMsg: short message");
  // getExtraBufPtr(): the last extraDataLength bytes of the message (ClientRequestMsg.hpp:85-87)
  const char* buf = body + clientRequestMsgSize(h) - h.extraDataLength;
  const size_t len = h.extraDataLength;
  // deserializeResultSignatures (PreProcessResultMsg.cpp:124-160): a std::set keyed by sender
  std::set<ResultSig> sigs;
  for (size_t pos = 0;;) {
    if (2 + 4 + 4 > len - pos)
      throw std::runtime_error("Deserialization error - remaining buffer length is less than fixed size values size");
    ResultSig s;
    s.sender = (uint16_t)(((uint8_t)buf[pos] << 8) | (uint8_t)buf[pos + 1]);
    s.result = be32(buf + pos + 2);
    const uint32_t sl = be32(buf + pos + 6);
    pos += 10;
    if (sl > len - pos)
      throw std::runtime_error("Deserialization error - remaining buffer length is less than a signature size");
    s.sig.assign(buf + pos, sl);
    pos += sl;
    sigs.insert(std::move(s));
    if (len - pos == 0) break;
  }
  const size_t expected = (size_t)(fVal + 1);
  if (sigs.size() != expected)
    return std::string("PreProcessResult signatures validation failure - unexpected number of signatures received");
  const char* req = body + sizeof(ClientRequestMsgHeader) + h.spanContextSize;
  const std::string hash =
      preProcessResultHash(req, h.requestLength, sigs.begin()->result, h.idOfClientProxy, h.reqSeqNum);
  // the replicas' signatures in one batch, in sender order; the serial loop returns at the first
  // bad one, so counters stop there (stopAtFirstFailure)
  std::vector<SigBatchItem> items;
  std::vector<const ResultSig*> order;
  for (const ResultSig& s : sigs) order.push_back(&s);
  size_t firstBad = order.size();
  for (size_t k = 0; k < order.size(); k++) {
    const ResultSig& s = *order[k];
    if (s.sender == myReplicaId) {  // own signature: recompute and compare (deterministic signers)
      std::string mine(sm.getMySigLength(), '\0');
      sm.sign(hash.data(), hash.size(), &mine[0], (uint16_t)mine.size());
      if (mine != s.sig) {
        firstBad = k;
        break;
      }
    } else {
      items.push_back({s.sender, hash.data(), hash.size(), s.sig.data(), (uint16_t)s.sig.size()});
    }
  }
  // `items` holds the replicas' signatures before any own-signature mismatch (the serial loop
  // never reaches those after it)
  std::vector<bool> verdict;
  const size_t bad = items.empty() ? 0 : sm.verifySigBatch(items, verdict, true);
  if (bad < items.size() || firstBad < order.size())
    return std::string("PreProcessResult signatures validation failure - invalid signature received from replica");
  return std::nullopt;
}

}  // namespace concord::hip

// Batch extraction from the reference's wire formats: the
// serial per-request signature loops of bftengine, each replaced by a walk over the message
// bytes that applies the reference's non-cryptographic checks per request and then verifies every
// signature with ONE SigManager::verifySigBatch call.
//
//   ClientRequestMsg::validateImp        ClientRequestMsg.cpp:99-214   (per request: size, ids,
//                                        expected signature length, HAS_PRE_PROCESSED_FLAG skip,
//                                        expectedMsgSize; signed region = the request payload,
//                                        ClientRequestMsg.hpp:65, signature after the cid,
//                                        ClientRequestMsg.cpp:242-248)
//   PrePrepareMsg::validate's loop       PrePrepareMsg.cpp:116-125 over RequestsIterator
//                                        (PrePrepareMsg.cpp:258-350); the loop throws at the first
//                                        invalid request
//   ClientBatchRequestMsg                ClientBatchRequestMsg.cpp (checkElements, then one
//                                        ClientRequestMsg per element) validated by
//                                        PreProcessor::checkClientBatchMsgCorrectness
//                                        (PreProcessor.cpp:557-590): every element is validated,
//                                        the loop does not stop at an invalid one
//   PreProcessor::checkPreProcessBatchReqMsgCorrectness  PreProcessor.cpp:877-902: the non-primary's
//                                        pre-execution batch; validateMessage per embedded
//                                        PreProcessRequestMsg (PreProcessRequestMsg.cpp:80-113, one
//                                        verifySig each), after PreProcessBatchRequestMsg::validate
//                                        + checkElements (PreProcessBatchRequestMsg.cpp:44-89);
//                                        every element is validated, invalid ones are counted
//   PreProcessResultMsg::validatePreProcessResultSignatures  PreProcessResultMsg.cpp:57-99: f+1
//                                        replica signatures over SHA3-256(result || result code ||
//                                        client id || seq num) (PreProcessResultHashCreator.hpp:19-35)
//
// Wire structs are packed little-endian restatements of the reference's (ClientMsgs.hpp:23-50,
// PrePrepareMsg.hpp:33-53, MessageBase.hpp:30-33, PreProcessRequestMsg.hpp:65-81,
// PreProcessBatchRequestMsg.hpp:45-55) in namespace concord::hip::wire (their layout is
// checked against the reference's own structs by tests/test_reference_boundary.py).  Outcomes
// equal the serial reference loop's: the same request fails first with the same kind of error,
// and SigManager's counters move for exactly the signatures the serial loop would have verified.
// The ReplicasInfo and SigManager types are the reference's (bftEngine::impl::ReplicasInfo and
// HipSigManager, derived from bftEngine::impl::SigManager).
#pragma once

#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "hip_sig_manager.hpp"

namespace concord::hip {

using bftEngine::impl::PrincipalId;
using bftEngine::impl::ReplicaId;
using bftEngine::impl::ReplicasInfo;

namespace wire {

#pragma pack(push, 1)
struct MessageBaseHeader {  // MessageBase.hpp:30-33
  uint16_t msgType;
  uint32_t spanContextSize;
};

struct ClientRequestMsgHeader {  // ClientMsgs.hpp:33-50
  uint16_t msgType;              // REQUEST_MSG_TYPE (700)
  uint32_t spanContextSize;
  uint16_t idOfClientProxy;
  uint64_t flags;
  uint32_t result;
  uint64_t reqSeqNum;
  uint32_t requestLength;
  uint64_t timeoutMilli;
  uint32_t cidLength;
  uint16_t reqSignatureLength;
  uint32_t extraDataLength;
};

struct ClientBatchRequestMsgHeader {  // ClientMsgs.hpp:25-31
  uint16_t msgType;                   // BATCH_REQUEST_MSG_TYPE (750)
  uint32_t cidSize;
  uint16_t clientId;
  uint32_t numOfMessagesInBatch;
  uint32_t dataSize;
};

// preprocessor::PreProcessRequestMsg::Header (PreProcessRequestMsg.hpp:65-81); RequestType is a
// plain enum (4 B), SeqNum / ViewNum int64_t, NodeIdType uint16_t (PrimitiveTypes.hpp:29-36)
struct PreProcessRequestMsgHeader {
  MessageBaseHeader header;  // msgType PreProcessRequest (501)
  uint32_t reqType;
  int64_t reqSeqNum;
  uint16_t clientId;
  uint16_t reqOffsetInBatch;
  uint16_t senderId;
  uint32_t requestLength;
  uint32_t cidLength;
  uint32_t spanContextSize;
  uint64_t reqRetryId;
  uint16_t reqSignatureLength;
  uint64_t primaryBlockId;
  uint32_t result;
  int64_t viewNum;
};

// preprocessor::PreProcessBatchRequestMsg::Header (PreProcessBatchRequestMsg.hpp:45-55)
struct PreProcessBatchRequestMsgHeader {
  MessageBaseHeader header;  // msgType PreProcessBatchRequest (503)
  uint32_t reqType;
  uint16_t clientId;
  uint16_t senderId;
  uint32_t cidLength;
  uint32_t numOfMessagesInBatch;
  uint32_t requestsSize;
  int64_t viewNum;
};

struct PrePrepareMsgHeader {  // PrePrepareMsg.hpp:34-46
  MessageBaseHeader header;
  int64_t viewNum;
  int64_t seqNum;
  int64_t epochNum;
  uint16_t flags;
  uint64_t batchCidLength;
  int64_t time;
  uint8_t digestOfRequests[32];
  uint16_t numberOfRequests;
  uint32_t endLocationOfLastRequest;
};
#pragma pack(pop)
static_assert(sizeof(ClientRequestMsgHeader) == 50, "ClientRequestMsgHeader is 50 B");
static_assert(sizeof(ClientBatchRequestMsgHeader) == 16, "ClientBatchRequestMsgHeader is 16 B");
static_assert(sizeof(PrePrepareMsgHeader) == 86, "PrePrepareMsg::Header is 86 B");
static_assert(sizeof(PreProcessRequestMsgHeader) == 66, "PreProcessRequestMsg::Header is 66 B");
static_assert(sizeof(PreProcessBatchRequestMsgHeader) == 34, "PreProcessBatchRequestMsg::Header is 34 B");

// MsgCode.hpp:46-51
enum : uint16_t { kPreProcessRequestMsgType = 501, kPreProcessBatchRequestMsgType = 503 };

// Flag bits (Replica.hpp:44-51, SimpleClient.hpp:43-51)
enum : uint64_t {
  READ_ONLY_REQ = 0x1,
  PRE_PROCESS_REQ = 0x2,
  HAS_PRE_PROCESSED_FLAG = 0x4,
  KEY_EXCHANGE_FLAG = 0x8,
  EMPTY_CLIENT_REQ = 0x10,
  RECONFIG_FLAG = 0x20,
};
constexpr uint32_t kMaxClientBatchSize = 1024;  // MAX_BATCH_SIZE of ClientBatchRequestMsg::checkElements
}  // namespace wire
using wire::ClientRequestMsgHeader;

// Total size of a packed ClientRequestMsg as the reference computes it (compRequestMsgSize,
// ClientRequestMsg.cpp:26-29), from its header.
uint64_t clientRequestMsgSize(const ClientRequestMsgHeader& h);

// One ClientRequestMsg to validate: its bytes [body, body + size) (size = the message's size(),
// for an embedded request = clientRequestMsgSize) and its sender (the node the message came from;
// for a request embedded in a PrePrepare the reference uses idOfClientProxy, ClientRequestMsg.cpp:24).
struct ClientRequestView {
  const char* body;
  uint64_t size;
  PrincipalId senderId;
};

// Outcome of validating a list of requests: ok[i] = validate() of request i would not throw;
// error[i] = the message it would throw with (empty when ok).  firstFailure = index of the first
// request that fails (or size when all pass).
struct RequestValidation {
  std::vector<bool> ok;
  std::vector<std::string> error;
  size_t firstFailure = 0;
};

// ClientRequestMsg::validateImp over many requests with one signature batch.  stopAtFirstFailure
// = the caller's loop throws at the first invalid request (PrePrepareMsg::validate): requests after
// it are not validated and their signatures not counted.  Otherwise (PreProcessor's client batch
// loop) every request is validated and counted.
RequestValidation validateClientRequests(const std::vector<ClientRequestView>& reqs, const ReplicasInfo& repInfo,
                                         const HipSigManager& sigManager, bool stopAtFirstFailure);

// PrePrepareMsg::validate's request loop (PrePrepareMsg.cpp:116-125) for the PrePrepare message
// bytes [body, body + size): the requests between payloadShift() and endLocationOfLastRequest,
// numberOfRequests of them (checkRequests, PrePrepareMsg.cpp:258-306, must hold: else
// std::runtime_error("... advanced")).  With client transaction signing enabled, every embedded
// request is validated as ClientRequestMsg::validate; throws std::runtime_error with the first
// failing request's error, exactly where the serial loop would.  Returns the number of requests.
size_t validatePrePrepareRequests(const char* body, uint64_t size, const ReplicasInfo& repInfo,
                                  const HipSigManager& sigManager);

// The requests of a ClientBatchRequestMsg [body, body + size) (ClientBatchRequestMsg.cpp:
// checkElements, then getClientPreProcessRequestMsgs): throws std::runtime_error if the batch
// itself is malformed (ClientBatchRequestMsg::validate); else validates every element like
// PreProcessor::checkClientBatchMsgCorrectness does (all of them, in one signature batch) and
// returns the per-element outcome.
RequestValidation validateClientBatchRequestMsg(const char* body, uint64_t size, const ReplicasInfo& repInfo,
                                                const HipSigManager& sigManager);

// PreProcessBatchRequestMsg::validate (PreProcessBatchRequestMsg.cpp:44-61) with checkElements
// (:63-89) for the message [body, body + size) received from networkSender: throws
// std::runtime_error where the reference throws.  The reference reads every element header
// without a bounds check (checkElements, getPreProcessRequestMsgs:114-147); here an element that
// does not fit in the message also throws (the reference's behaviour there is undefined).
void validatePreProcessBatchRequestMsg(const char* body, uint64_t size, PrincipalId networkSender,
                                       const ReplicasInfo& repInfo, const HipSigManager& sigManager);

// The replica state PreProcessor::checkPreProcessBatchReqMsgCorrectness consults
// (PreProcessor.cpp:848-873, 877-885): the current view and the three prerequisites of
// checkPreProcessReqPrerequisites.  None depends on the message.
struct PreProcessReplicaState {
  int64_t currentView = 0;
  bool collectingState = false;
  bool isCurrentPrimary = false;
  bool currentViewIsActive = true;
};

// Per-element outcome of checkPreProcessBatchReqMsgCorrectness.
enum class PreProcessOutcome : uint8_t {
  Valid,
  Ignored,  // checkPreProcessReqPrerequisites failed (metric preProcReqIgnored)
  Invalid,  // validateMessage failed: PreProcessRequestMsg::validate threw (metric preProcReqInvalid)
};

struct PreProcessBatchValidation {
  bool valid = false;         // the function's return value
  bool viewMismatch = false;  // batch viewNum != current view: rejected before any element
  std::vector<PreProcessOutcome> outcome;
  std::vector<std::string> error;  // PreProcessRequestMsg::validate's message for Invalid elements
  uint32_t ignored = 0;            // preProcReqIgnored increments
  uint32_t invalid = 0;            // preProcReqInvalid increments
};

// PreProcessor::checkPreProcessBatchReqMsgCorrectness (PreProcessor.cpp:877-902) for a batch that
// passed validatePreProcessBatchRequestMsg.  The serial loop rebuilds every element as a
// PreProcessRequestMsg (sender and client = the batch header's, getPreProcessRequestMsgs) and calls
// validateMessage → PreProcessRequestMsg::validate (PreProcessRequestMsg.cpp:80-113), i.e.
// SigManager::verifySig once per signed element, and does not stop at an invalid one.  Here every
// element's non-cryptographic checks run first, then the signatures of the elements that reach
// the signature check are verified in ONE SigManager::verifySigBatch; outcomes, metric increments
// and SigManager's counters equal the serial loop's.
PreProcessBatchValidation checkPreProcessBatchReqMsgCorrectness(const char* body, uint64_t size,
                                                                const PreProcessReplicaState& state,
                                                                const ReplicasInfo& repInfo,
                                                                const HipSigManager& sigManager);

// PreProcessResultMsg::validatePreProcessResultSignatures (PreProcessResultMsg.cpp:57-99) for the
// ClientRequestMsg-format message [body, body + size) whose extra data holds the serialized result
// signatures (sender u16 BE, result u32 BE, length u32 BE, signature; PreProcessResultMsg.cpp:
// 101-160).  Returns the reference's error text, or nullopt when all f+1 signatures verify (own
// signature: recomputed and compared, as there).  Throws std::runtime_error on a malformed
// signature buffer (deserializeResultSignatures).
std::optional<std::string> validatePreProcessResultSignatures(const char* body, uint64_t size, ReplicaId myReplicaId,
                                                              int16_t fVal, const HipSigManager& sigManager);

// SHA3-256(result bytes (only when resultCode == SUCCESS = 0) || resultCode u32 || clientId u16
// || reqSeqNum u64), host byte order as the reference's update(&x, sizeof x)
// (PreProcessResultHashCreator.hpp:21-34).
std::string preProcessResultHash(const char* result, uint32_t len, uint32_t resultCode, uint16_t clientId,
                                 uint64_t reqSeqNum);

}  // namespace concord::hip

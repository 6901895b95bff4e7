// C++ host-side tests of the plugin layer (run on the GPU box by tests/test_cpp_host.py).
// Pattern of the reference's bftengine/tests/SigManager/SigManager_test.cpp:70-114: sign with
// one principal's key, verify through SigManager, corrupt a byte (++), expect failure and exact
// counter movements; plus the batch path against single verifies.
#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>

#include <atomic>
#include <cassert>
#include <chrono>
#include <cstdio>
#include <memory>
#include <thread>
#include <tuple>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "Metrics.hpp"
#include "ReplicaConfig.hpp"
#include "hip_crypto.hpp"
#include "hip_sig_manager.hpp"
#include "request_batch.hpp"

using namespace concord::hip;
using namespace concord::hip::wire;
using bftEngine::impl::PrincipalId;
using bftEngine::impl::ReplicaIdsConfig;
using bftEngine::impl::ReplicasInfo;
using concord::util::crypto::KeyFormat;
using concord::util::crypto::RSASigner;
using SigManager = concord::hip::HipSigManager;

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                    \
    }                                                              \
  } while (0)

static std::string seedHex(int i) {
  std::string s;
  std::mt19937 g(1000 + i);
  uint8_t b[32];
  for (auto& x : b) x = (uint8_t)g();
  return toHex(b, 32);
}

// RSA-2048 key pair as (private PKCS#8 hex DER, public SubjectPublicKeyInfo hex DER, public PEM),
// the formats crypto_utils.cpp:141-176 loads (Crypto++ Save / PEM_Load)
struct RsaKeys {
  std::string privHex, pubHex, pubPem;
};
static RsaKeys genRsa(unsigned e) {
  EVP_PKEY_CTX* c = EVP_PKEY_CTX_new_id(EVP_PKEY_RSA, nullptr);
  EVP_PKEY* k = nullptr;
  BIGNUM* be = BN_new();
  BN_set_word(be, e);
  EVP_PKEY_keygen_init(c);
  EVP_PKEY_CTX_set_rsa_keygen_bits(c, 2048);
  EVP_PKEY_CTX_set1_rsa_keygen_pubexp(c, be);
  EVP_PKEY_keygen(c, &k);
  RsaKeys r;
  unsigned char* der = nullptr;
  int n = i2d_PrivateKey(k, &der);
  r.privHex = toHex(der, n);
  OPENSSL_free(der);
  der = nullptr;
  n = i2d_PUBKEY(k, &der);
  r.pubHex = toHex(der, n);
  OPENSSL_free(der);
  BIO* b = BIO_new(BIO_s_mem());
  PEM_write_bio_PUBKEY(b, k);
  char* pem = nullptr;
  long pl = BIO_get_mem_data(b, &pem);
  r.pubPem.assign(pem, pl);
  BIO_free(b);
  BN_free(be);
  EVP_PKEY_free(k);
  EVP_PKEY_CTX_free(c);
  return r;
}

static int testRsa() {
  // --- RSAVerifier / RSASigner (crypto_utils.cpp:101-168): hex DER and PEM keys
  RsaKeys kc = genRsa(65537), kr = genRsa(17);
  RSASigner sc(kc.privHex, KeyFormat::HexaDecimalStrippedFormat);
  HipRSAVerifier vc(kc.pubHex, KeyFormat::HexaDecimalStrippedFormat), vcp(kc.pubPem, KeyFormat::PemFormat);
  CHECK(vc.signatureLength() == 256 && sc.signatureLength() == 256);
  std::string msg = "client request signed with RSA-2048";
  std::string sig = sc.sign(msg);
  CHECK(sig.size() == 256);
  CHECK(vc.verify(msg, sig) && vcp.verify(msg, sig));
  std::string bad = msg;
  bad[3]++;
  CHECK(!vc.verify(bad, sig));
  std::string bs = sig;
  bs[100] ^= 4;
  CHECK(!vc.verify(msg, bs));
  CHECK(vc.verify(msg, std::string(3, '\0') + sig));  // Crypto++ reads the signature as an Integer
  CHECK(!vc.verify(msg, sig.substr(1)) || sig[0] == 0);
  bool threw = false;
  try {
    HipRSAVerifier broken("3000", KeyFormat::HexaDecimalStrippedFormat);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);

  // --- SigManager with RSA replicas (e = 17, as bftengine/tests/messages/helper.cpp) and RSA +
  // Ed25519 clients in one batch: verdicts and counters as with single verifies.  Id space
  // (ReplicasInfo.cpp:71-140): replicas 0..3, external clients 4..7, internal clients 8..11.
  EdDSASigner ed(seedHex(50), KeyFormat::HexaDecimalStrippedFormat);
  ReplicaIdsConfig cfg;
  cfg.replicaId = 1;
  cfg.numOfExternalClients = 4;
  ReplicasInfo ri(cfg);
  std::set<std::pair<PrincipalId, const std::string>> replicaKeys;
  for (PrincipalId r = 0; r < 4; r++) replicaKeys.insert({r, kr.pubHex});
  std::set<std::pair<const std::string, std::set<uint16_t>>> clientKeys = {{kc.pubHex, {4}}, {ed.getPubKeyHex(), {5}}};
  std::unique_ptr<SigManager> smp(SigManager::initInTesting(1, kr.privHex, replicaKeys,
                                                            KeyFormat::HexaDecimalStrippedFormat, &clientKeys,
                                                            KeyFormat::HexaDecimalStrippedFormat, ri));
  SigManager& sm = *smp;
  const PrincipalId C_RSA = 4, C_ED = 5;
  CHECK(sm.getSigLength(0) == 256 && sm.getSigLength(C_ED) == 64 && sm.getMySigLength() == 256);
  CHECK(sm.getSigLength(1) == 256);  // own id: this replica's signer (SigManager.cpp:183-186)
  CHECK(sm.isClientTransactionSigningEnabled());
  RSASigner sr(kr.privHex, KeyFormat::HexaDecimalStrippedFormat);
  std::vector<std::string> datas, sigs;
  std::vector<PrincipalId> who;
  std::vector<bool> expect;
  std::mt19937 g(17);
  for (int i = 0; i < 120; i++) {
    const PrincipalId p = (i % 3 == 0) ? (PrincipalId)(i % 4) : (i % 3 == 1 ? C_RSA : C_ED);
    std::string d(1 + g() % 400, '\0');
    for (auto& ch : d) ch = (char)g();
    std::string s = p < 4 ? sr.sign(d) : (p == C_RSA ? sc.sign(d) : ed.sign(d));
    bool ok = true;
    if (i % 5 == 0) {
      d[0]++;
      ok = false;
    }
    datas.push_back(d);
    sigs.push_back(s);
    who.push_back(p);
    expect.push_back(ok);
  }
  std::vector<SigBatchItem> items;
  for (size_t i = 0; i < datas.size(); i++)
    items.push_back({who[i], datas[i].data(), datas[i].size(), sigs[i].data(), (uint16_t)sigs[i].size()});
  std::vector<bool> out;
  sm.verifySigBatch(items, out);
  uint64_t okC = 0, okR = 0, badC = 0, badR = 0;
  for (size_t i = 0; i < items.size(); i++) {
    CHECK(out[i] == expect[i]);
    const bool client = ri.isIdOfExternalClient(who[i]);
    (expect[i] ? (client ? okC : okR) : (client ? badC : badR))++;
  }
  const auto m = sm.counterValues();
  CHECK(m.externalVerified == okC && m.replicaVerified == okR);
  CHECK(m.externalFailed == badC);
  CHECK(m.replicaFailed == badR);
  for (size_t i = 0; i < 12; i++)
    CHECK(sm.verifySig(who[i], datas[i].data(), datas[i].size(), sigs[i].data(), (uint16_t)sigs[i].size()) ==
          expect[i]);
  char os[256];
  sm.sign(msg.data(), msg.size(), os, 256);  // replica 1 signs with its RSA key
  CHECK(sm.verifySig(2, msg.data(), msg.size(), os, 256));
  std::printf("test_host: RSA checks passed (%zu mixed batch items)\n", items.size());
  return 0;
}

// Key exchange (KeyExchangeManager::loadClientPublicKey, KeyExchangeManager.cpp:316-322) calls
// SigManager::instance()->setClientPublicKey, a NON-virtual method: with the INTEGRATION.md patch
// it goes through HipSigManager::setClientPublicKeyOf(SigManager::instance(), ...).  A rotation
// must stay on the GPU (RSA -> HipRSAVerifier, Ed25519 -> HipEdDSAVerifier), verify signatures
// of the new key only, and enter the key into the CMF ClientsPublicKeys map (SigManager.cpp:260).
static int testKeyRotation() {
  using Base = bftEngine::impl::SigManager;
  RsaKeys k0 = genRsa(65537), k1 = genRsa(65537), kr = genRsa(17);
  EdDSASigner e0(seedHex(60), KeyFormat::HexaDecimalStrippedFormat), e1(seedHex(61), KeyFormat::HexaDecimalStrippedFormat);
  ReplicaIdsConfig cfg;
  cfg.replicaId = 0;
  cfg.numOfExternalClients = 4;
  ReplicasInfo ri(cfg);
  std::set<std::pair<PrincipalId, const std::string>> replicaKeys;
  for (PrincipalId r = 0; r < 4; r++) replicaKeys.insert({r, kr.pubHex});
  std::set<std::pair<const std::string, std::set<uint16_t>>> clientKeys = {{k0.pubHex, {4}}, {e0.getPubKeyHex(), {5}}};
  std::unique_ptr<SigManager> smp(SigManager::init(0, kr.privHex, replicaKeys, KeyFormat::HexaDecimalStrippedFormat,
                                                   &clientKeys, KeyFormat::HexaDecimalStrippedFormat, ri));
  Base* base = Base::instance();
  CHECK(base == static_cast<Base*>(smp.get()));
  const std::string m = "request after key exchange";
  RSASigner s0(k0.privHex, KeyFormat::HexaDecimalStrippedFormat), s1(k1.privHex, KeyFormat::HexaDecimalStrippedFormat);
  const std::string rs0 = s0.sign(m), rs1 = s1.sign(m), es0 = e0.sign(m), es1 = e1.sign(m);
  CHECK(base->verifySig(4, m.data(), m.size(), rs0.data(), (uint16_t)rs0.size()));
  CHECK(!base->verifySig(4, m.data(), m.size(), rs1.data(), (uint16_t)rs1.size()));
  // RSA rotation through the base pointer: the new verifier is a GPU one, the new key verifies
  SigManager::setClientPublicKeyOf(base, k1.pubHex, 4, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(dynamic_cast<HipRSAVerifier*>(smp->verifierOf(4).get()) != nullptr);
  CHECK(base->verifySig(4, m.data(), m.size(), rs1.data(), (uint16_t)rs1.size()));
  CHECK(!base->verifySig(4, m.data(), m.size(), rs0.data(), (uint16_t)rs0.size()));
  // Ed25519 rotation (the base's method would throw: it builds an RSAVerifier)
  SigManager::setClientPublicKeyOf(base, e1.getPubKeyHex(), 5, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(dynamic_cast<HipEdDSAVerifier*>(smp->verifierOf(5).get()) != nullptr);
  CHECK(base->verifySig(5, m.data(), m.size(), es1.data(), (uint16_t)es1.size()));
  CHECK(!base->verifySig(5, m.data(), m.size(), es0.data(), (uint16_t)es0.size()));
  // an RSA client rotated to Ed25519, and a replica id refused ("Illegal id": unchanged)
  SigManager::setClientPublicKeyOf(base, e0.getPubKeyHex(), 4, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(base->verifySig(4, m.data(), m.size(), es0.data(), (uint16_t)es0.size()));
  auto replicaVerifier = smp->verifierOf(2);
  SigManager::setClientPublicKeyOf(base, e1.getPubKeyHex(), 2, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(smp->verifierOf(2) == replicaVerifier);
  // the CMF map carries the rotated keys, as SigManager.cpp:260 records them
  const std::string cmf = base->getClientsPublicKeys();
  CHECK(cmf.find(e0.getPubKeyHex()) != std::string::npos && cmf.find(e1.getPubKeyHex()) != std::string::npos);
  CHECK(cmf.find(k1.pubHex) == std::string::npos);  // client 4's RSA key was replaced again
  // a manager that init() did not register gets the reference's own method (RSA only)
  std::unique_ptr<SigManager> other(SigManager::initInTesting(0, kr.privHex, replicaKeys,
                                                              KeyFormat::HexaDecimalStrippedFormat, &clientKeys,
                                                              KeyFormat::HexaDecimalStrippedFormat, ri));
  bool threw = false;
  try {
    SigManager::setClientPublicKeyOf(other.get(), e1.getPubKeyHex(), 5, KeyFormat::HexaDecimalStrippedFormat);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  std::printf("test_host: key rotation through SigManager::instance() stays on the GPU\n");
  return 0;
}

// ------------------------------------------------------------------ reference wire formats
// A packed ClientRequestMsg: header (ClientMsgs.hpp:33-50) | span | request | cid | sig | extra
static std::string clientRequest(uint16_t client, uint64_t flags, uint64_t seq, const std::string& req,
                                 const std::string& cid, const std::string& sig, const std::string& extra = "") {
  ClientRequestMsgHeader h{};
  h.msgType = 700;
  h.idOfClientProxy = client;
  h.flags = flags;
  h.result = 1;
  h.reqSeqNum = seq;
  h.requestLength = (uint32_t)req.size();
  h.cidLength = (uint32_t)cid.size();
  h.reqSignatureLength = (uint16_t)sig.size();
  h.extraDataLength = (uint32_t)extra.size();
  return std::string(reinterpret_cast<const char*>(&h), sizeof h) + req + cid + sig + extra;
}

// A PrePrepareMsg (PrePrepareMsg.hpp:33-53) carrying the given packed requests
static std::string prePrepare(const std::vector<std::string>& reqs) {
  PrePrepareMsgHeader h{};
  h.header.msgType = 3;
  h.seqNum = 1;
  h.flags = 0x3;
  const std::string cid = "batch-cid";
  h.batchCidLength = cid.size();
  h.numberOfRequests = (uint16_t)reqs.size();
  std::string body;
  for (auto& r : reqs) body += r;
  h.endLocationOfLastRequest = (uint32_t)(sizeof h + cid.size() + body.size());
  return std::string(reinterpret_cast<const char*>(&h), sizeof h) + cid + body;
}

static std::string clientBatch(uint16_t sender, const std::vector<std::string>& reqs) {
  ClientBatchRequestMsgHeader h{};
  h.msgType = 750;
  const std::string cid = "cb";
  h.cidSize = (uint32_t)cid.size();
  h.clientId = sender;
  h.numOfMessagesInBatch = (uint32_t)reqs.size();
  std::string body;
  for (auto& r : reqs) body += r;
  h.dataSize = (uint32_t)body.size();
  return std::string(reinterpret_cast<const char*>(&h), sizeof h) + cid + body;
}

static uint64_t verifiedTotal(const SigManager& sm) {
  const auto m = sm.counterValues();
  return m.externalVerified + m.externalFailed + m.replicaVerified + m.replicaFailed;
}

// Message-level batch checks (request_batch.hpp) against what the reference's serial loops do.
template <class SignerOf>
static int testMessages(SigManager& sm, const ReplicasInfo& ri, std::vector<EdDSASigner>& signers, SignerOf signerOf) {
  (void)signers;
  std::mt19937 g(99);
  auto payload = [&](size_t n) {
    std::string p(n, '\0');
    for (auto& ch : p) ch = (char)g();
    return p;
  };
  // 60 requests from clients 4..11 (client 8's key was rotated above: it signs with seed 99)
  EdDSASigner rotated(seedHex(99), KeyFormat::HexaDecimalStrippedFormat);
  std::vector<std::string> reqs;
  std::vector<std::string> payloads;
  for (int i = 0; i < 60; i++) {
    const uint16_t c = (uint16_t)(4 + i % 8);
    std::string p = payload(32 + (size_t)(g() % 900));
    EdDSASigner& s = c == 8 ? rotated : signerOf(c);
    reqs.push_back(clientRequest(c, 0, 1000 + i, p, "cid-" + std::to_string(i), s.sign(p)));
    payloads.push_back(p);
  }
  // (1) a valid PrePrepare: every signature verified in one batch
  uint64_t before = verifiedTotal(sm);
  std::string pp = prePrepare(reqs);
  CHECK(validatePrePrepareRequests(pp.data(), pp.size(), ri, sm) == 60);
  CHECK(verifiedTotal(sm) - before == 60);
  // (2) a bad signature at request 23: throws there; the serial loop verified 0..23 only
  {
    std::vector<std::string> r2 = reqs;
    r2[23][sizeof(ClientRequestMsgHeader) + 5] ^= 1;  // a payload byte: the signature no longer matches
    std::string pp2 = prePrepare(r2);
    before = verifiedTotal(sm);
    const uint64_t failBefore = sm.counterValues().externalFailed;
    bool threw = false;
    try {
      validatePrePrepareRequests(pp2.data(), pp2.size(), ri, sm);
    } catch (const std::runtime_error& e) {
      threw = std::string(e.what()).find("Signature verification failed") != std::string::npos;
    }
    CHECK(threw);
    CHECK(verifiedTotal(sm) - before == 24);
    CHECK(sm.counterValues().externalFailed - failBefore == 1);
  }
  // (3) a wrong signature length at request 10 and a bad signature at 40: the length error wins
  // and no signature after request 9 is counted
  {
    std::vector<std::string> r3 = reqs;
    r3[10] = clientRequest(5, 0, 7, payloads[10], "x", std::string(63, 'a'));
    r3[40][sizeof(ClientRequestMsgHeader) + 2] ^= 1;
    std::string pp3 = prePrepare(r3);
    before = verifiedTotal(sm);
    std::string what;
    try {
      validatePrePrepareRequests(pp3.data(), pp3.size(), ri, sm);
    } catch (const std::runtime_error& e) {
      what = e.what();
    }
    CHECK(what.find("Unexpected request signature length") != std::string::npos);
    CHECK(verifiedTotal(sm) - before == 10);
  }
  // (4) HAS_PRE_PROCESSED_FLAG: the signature length is still checked, the signature is not
  // verified (ClientRequestMsg.cpp:172-174); an empty request carries no signature
  {
    std::vector<std::string> r4 = {reqs[0], clientRequest(6, HAS_PRE_PROCESSED_FLAG, 5, "payload", "c",
                                                          std::string(64, '\x01')),
                                   clientRequest(7, 0, 6, "", "c", "")};
    std::string pp4 = prePrepare(r4);
    before = verifiedTotal(sm);
    CHECK(validatePrePrepareRequests(pp4.data(), pp4.size(), ri, sm) == 3);
    CHECK(verifiedTotal(sm) - before == 1);
  }
  // (5) structural errors: a request count that does not match the bytes
  {
    std::string pp5 = prePrepare(reqs);
    PrePrepareMsgHeader h;
    std::memcpy(&h, pp5.data(), sizeof h);
    h.numberOfRequests = 61;
    std::memcpy(&pp5[0], &h, sizeof h);
    bool threw = false;
    try {
      validatePrePrepareRequests(pp5.data(), pp5.size(), ri, sm);
    } catch (const std::runtime_error& e) {
      threw = std::string(e.what()).find("advanced") != std::string::npos;
    }
    CHECK(threw);
  }
  // (6) a client batch (PreProcessor::checkClientBatchMsgCorrectness): every element validated,
  // the bad ones reported individually, every signature counted
  {
    std::vector<std::string> r6(reqs.begin(), reqs.begin() + 10);
    r6[3][sizeof(ClientRequestMsgHeader) + 1] ^= 1;
    r6[8][sizeof(ClientRequestMsgHeader) + 1] ^= 1;
    std::string cb = clientBatch(4, r6);
    before = verifiedTotal(sm);
    RequestValidation v = validateClientBatchRequestMsg(cb.data(), cb.size(), ri, sm);
    CHECK(v.ok.size() == 10 && v.firstFailure == 3);
    for (int i = 0; i < 10; i++) CHECK(v.ok[i] == (i != 3 && i != 8));
    CHECK(verifiedTotal(sm) - before == 10);
    std::string bad = clientBatch(4, {clientRequest(5, 0, 1, "p", "c", std::string(10, 'x'))});
    bool threw = false;
    try {
      validateClientBatchRequestMsg(bad.data(), bad.size(), ri, sm);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);  // checkElements: signature length != getSigLength(client)
  }
  return 0;
}

// A PreProcessRequestMsg as PreProcessBatchRequestMsg embeds it: header (PreProcessRequestMsg.hpp:
// 65-81) | span | request | cid | signature
static std::string preProcessElement(uint16_t client, int64_t seq, const std::string& span, const std::string& req,
                                     const std::string& cid, const std::string& sig) {
  PreProcessRequestMsgHeader h{};
  h.header.msgType = kPreProcessRequestMsgType;
  h.header.spanContextSize = (uint32_t)span.size();
  h.reqSeqNum = seq;
  h.clientId = client;
  h.senderId = 1;
  h.requestLength = (uint32_t)req.size();
  h.cidLength = (uint32_t)cid.size();
  h.spanContextSize = (uint32_t)span.size();
  h.reqSignatureLength = (uint16_t)sig.size();
  h.result = 1;
  h.viewNum = 3;
  return std::string(reinterpret_cast<const char*>(&h), sizeof h) + span + req + cid + sig;
}

// A PreProcessBatchRequestMsg (PreProcessBatchRequestMsg.hpp:45-55) from replica `sender`
static std::string preProcessBatch(uint16_t client, uint16_t sender, int64_t view, const std::vector<std::string>& elems) {
  PreProcessBatchRequestMsgHeader h{};
  h.header.msgType = kPreProcessBatchRequestMsgType;
  h.clientId = client;
  h.senderId = sender;
  const std::string cid = "pp-batch-cid";
  h.cidLength = (uint32_t)cid.size();
  h.numOfMessagesInBatch = (uint32_t)elems.size();
  std::string body;
  for (auto& e : elems) body += e;
  h.requestsSize = (uint32_t)body.size();
  h.viewNum = view;
  return std::string(reinterpret_cast<const char*>(&h), sizeof h) + cid + body;
}

// PreProcessor::checkPreProcessBatchReqMsgCorrectness on a non-primary: the batched walk against
// the serial loop it replaces (validateMessage → PreProcessRequestMsg::validate → verifySig per
// element, PreProcessor.cpp:877-902): same per-element outcomes, same metric increments, same
// SigManager counters.
template <class SignerOf>
static int testPreProcessBatch(SigManager& sm, const ReplicasInfo& ri, SignerOf signerOf) {
  std::mt19937 g(2024);
  const uint16_t client = 9;
  const int n = 48;
  std::vector<std::string> reqs, elems;
  for (int i = 0; i < n; i++) {
    std::string p(16 + g() % 700, '\0');
    for (auto& ch : p) ch = (char)g();
    reqs.push_back(p);
    const std::string span = i % 5 == 0 ? std::string(i % 3 + 1, 's') : std::string();
    elems.push_back(preProcessElement(client, 500 + i, span, p, "cid-" + std::to_string(i), signerOf(client).sign(p)));
  }
  PreProcessReplicaState st;
  st.currentView = 3;
  // the serial loop, element by element, through SigManager::verifySig
  auto serial = [&](const std::vector<std::string>& es, std::vector<PreProcessOutcome>& out) {
    out.clear();
    for (const std::string& e : es) {
      PreProcessRequestMsgHeader h;
      std::memcpy(&h, e.data(), sizeof h);
      const char* req = e.data() + sizeof h + h.spanContextSize;
      out.push_back(sm.verifySig(client, req, h.requestLength, req + h.requestLength + h.cidLength,
                                 h.reqSignatureLength)
                        ? PreProcessOutcome::Valid
                        : PreProcessOutcome::Invalid);
    }
  };
  // (1) a valid batch: one signature batch, every element verified
  {
    const std::string b = preProcessBatch(client, 1, 3, elems);
    validatePreProcessBatchRequestMsg(b.data(), b.size(), 1, ri, sm);
    const auto before = sm.counterValues();
    PreProcessBatchValidation v = checkPreProcessBatchReqMsgCorrectness(b.data(), b.size(), st, ri, sm);
    CHECK(v.valid && v.outcome.size() == (size_t)n && v.ignored == 0 && v.invalid == 0);
    CHECK(sm.counterValues().externalVerified - before.externalVerified == (uint64_t)n);
  }
  // (2) bad signatures at elements 3, 17 and 47, a corrupted request at 30: those are Invalid,
  // the rest Valid, every element verified (the loop does not stop); outcomes and counters equal
  // the serial loop's
  {
    std::vector<std::string> e2 = elems;
    for (int k : {3, 17, 47}) e2[k][e2[k].size() - 9] ^= 0x40;  // a signature byte
    e2[30][sizeof(PreProcessRequestMsgHeader) + 2] ^= 1;        // a request byte
    const std::string b = preProcessBatch(client, 1, 3, e2);
    validatePreProcessBatchRequestMsg(b.data(), b.size(), 1, ri, sm);
    auto c0 = sm.counterValues();
    std::vector<PreProcessOutcome> ref;
    serial(e2, ref);
    auto c1 = sm.counterValues();
    PreProcessBatchValidation v = checkPreProcessBatchReqMsgCorrectness(b.data(), b.size(), st, ri, sm);
    auto c2 = sm.counterValues();
    CHECK(!v.valid && v.invalid == 4 && v.ignored == 0);
    CHECK(v.outcome == ref);
    for (int k = 0; k < n; k++) CHECK((v.outcome[k] == PreProcessOutcome::Invalid) == (k == 3 || k == 17 || k == 30 || k == 47));
    {  // the whole text, as PreProcessRequestMsg::validate builds it with KVLOG
      PreProcessRequestMsgHeader h17;
      std::memcpy(&h17, e2[17].data(), sizeof h17);
      const std::string want = "Signature verification failed for:  header->clientId: " + std::to_string(client) +
                               ", header->reqSeqNum: 517, header->requestLength: " + std::to_string(reqs[17].size()) +
                               ", header->reqSignatureLength: " + std::to_string(h17.reqSignatureLength);
      CHECK(v.error[17] == want);
    }
    CHECK(c2.externalVerified - c1.externalVerified == c1.externalVerified - c0.externalVerified);
    CHECK(c2.externalFailed - c1.externalFailed == c1.externalFailed - c0.externalFailed);
    CHECK(c2.externalFailed - c1.externalFailed == 4);
  }
  // (3) PreProcessBatchRequestMsg::validate / checkElements failures throw, nothing is verified
  {
    const auto before = sm.counterValues();
    auto throws = [&](const std::string& b, uint16_t netSender) {
      try {
        validatePreProcessBatchRequestMsg(b.data(), b.size(), netSender, ri, sm);
      } catch (const std::runtime_error&) {
        return true;
      }
      return false;
    };
    std::vector<std::string> e3 = elems;
    e3[7] = preProcessElement(client, 7, "", reqs[7], "c", std::string(63, 'x'));  // signature length != 64
    CHECK(throws(preProcessBatch(client, 1, 3, e3), 1));
    CHECK(throws(preProcessBatch(client, 1, 3, elems), 0));                 // sent by this replica
    CHECK(throws(preProcessBatch(client, 1, 3, {}), 1));                    // empty batch
    std::string wrongType = preProcessBatch(client, 1, 3, elems);
    wrongType[0] = 1;
    CHECK(throws(wrongType, 1));
    std::string truncated = preProcessBatch(client, 1, 3, elems);
    truncated.resize(truncated.size() - 10);
    CHECK(throws(truncated, 1));
    std::vector<std::string> unsigned_ = {preProcessElement(client, 1, "", "payload", "c", "")};
    CHECK(throws(preProcessBatch(client, 1, 3, unsigned_), 1));  // signing on: 64 B expected
    CHECK(verifiedTotal(sm) == before.externalVerified + before.externalFailed + before.replicaVerified +
                                   before.replicaFailed);
  }
  // (4) the batch's own replica sender is this replica: every element Invalid, none verified;
  // (5) a view mismatch or an unmet prerequisite: rejected / Ignored, none verified
  {
    const uint64_t before = verifiedTotal(sm);
    const std::string self = preProcessBatch(client, 0, 3, elems);
    PreProcessBatchValidation v = checkPreProcessBatchReqMsgCorrectness(self.data(), self.size(), st, ri, sm);
    CHECK(!v.valid && v.invalid == (uint32_t)n);
    const std::string b = preProcessBatch(client, 1, 4, elems);
    v = checkPreProcessBatchReqMsgCorrectness(b.data(), b.size(), st, ri, sm);
    CHECK(!v.valid && v.viewMismatch && v.outcome.empty());
    PreProcessReplicaState collecting = st;
    collecting.collectingState = true;
    const std::string b3 = preProcessBatch(client, 1, 3, elems);
    v = checkPreProcessBatchReqMsgCorrectness(b3.data(), b3.size(), collecting, ri, sm);
    CHECK(!v.valid && v.ignored == (uint32_t)n && v.invalid == 0);
    PreProcessReplicaState primary = st;
    primary.isCurrentPrimary = true;
    v = checkPreProcessBatchReqMsgCorrectness(b3.data(), b3.size(), primary, ri, sm);
    CHECK(v.ignored == (uint32_t)n);
    CHECK(verifiedTotal(sm) == before);
  }
  std::printf("test_host: PreProcessBatchRequestMsg checks batched, outcomes and counters equal the serial loop\n");
  return 0;
}

// PreProcessResultMsg::validatePreProcessResultSignatures with f + 1 = 2 replica signatures.
static int testPreProcessResult(const SigManager& sm, std::vector<EdDSASigner>& signers) {
  const std::string result = "pre-execution result bytes";
  const uint16_t client = 5;
  const uint64_t seq = 77;
  const std::string hash = preProcessResultHash(result.data(), (uint32_t)result.size(), 0, client, seq);
  auto ser = [](const std::vector<std::tuple<uint16_t, uint32_t, std::string>>& sigs) {
    std::string o;
    for (auto& [sender, res, sig] : sigs) {
      o += (char)(sender >> 8);
      o += (char)sender;
      for (int k = 3; k >= 0; k--) o += (char)(res >> (8 * k));
      const uint32_t l = (uint32_t)sig.size();
      for (int k = 3; k >= 0; k--) o += (char)(l >> (8 * k));
      o += sig;
    }
    return o;
  };
  auto msg = [&](const std::string& extra) { return clientRequest(client, 0, seq, result, "cid", "", extra); };
  std::string good = msg(ser({{2, 0, signers[2].sign(hash)}, {1, 0, signers[1].sign(hash)}}));
  CHECK(!validatePreProcessResultSignatures(good.data(), good.size(), 3, 1, sm).has_value());
  // own signature (replica 0 = this SigManager's signer) is recomputed and compared
  std::string own = msg(ser({{0, 0, signers[0].sign(hash)}, {3, 0, signers[3].sign(hash)}}));
  CHECK(!validatePreProcessResultSignatures(own.data(), own.size(), 0, 1, sm).has_value());
  std::string badsig = signers[1].sign(hash);
  badsig[7] ^= 1;
  std::string bad = msg(ser({{2, 0, signers[2].sign(hash)}, {1, 0, badsig}}));
  auto r = validatePreProcessResultSignatures(bad.data(), bad.size(), 3, 1, sm);
  CHECK(r.has_value() && r->find("invalid signature") != std::string::npos);
  std::string three = msg(ser({{1, 0, signers[1].sign(hash)}, {2, 0, signers[2].sign(hash)},
                               {3, 0, signers[3].sign(hash)}}));
  r = validatePreProcessResultSignatures(three.data(), three.size(), 0, 1, sm);
  CHECK(r.has_value() && r->find("unexpected number") != std::string::npos);
  std::string dup = msg(ser({{2, 0, signers[2].sign(hash)}, {2, 0, signers[2].sign(hash)}}));  // a set: one sender
  r = validatePreProcessResultSignatures(dup.data(), dup.size(), 0, 1, sm);
  CHECK(r.has_value());
  return 0;
}

// 64 threads call HipEdDSAVerifier::verify concurrently (the reference's pool threads) while new
// client keys are registered: verdicts exact, calls coalesced into fewer GPU batches.
static int testConcurrent() {
  const int T = 64, K = 24;
  std::vector<std::unique_ptr<EdDSASigner>> sg;
  std::vector<std::unique_ptr<HipEdDSAVerifier>> vf;
  for (int k = 0; k < 8; k++) {
    sg.emplace_back(new EdDSASigner(seedHex(300 + k), KeyFormat::HexaDecimalStrippedFormat));
    vf.emplace_back(new HipEdDSAVerifier(sg.back()->getPubKeyHex(), KeyFormat::HexaDecimalStrippedFormat));
  }
  std::vector<std::vector<std::string>> msgs(T), sigs(T);
  std::vector<std::vector<bool>> expect(T);
  for (int t = 0; t < T; t++) {
    std::mt19937 g(5000 + t);
    for (int k = 0; k < K; k++) {
      std::string m(16 + g() % 500, '\0');
      for (auto& ch : m) ch = (char)g();
      std::string s = sg[(t + k) % 8]->sign(m);
      const bool ok = (t * K + k) % 9 != 0;
      if (!ok) s[3] ^= 0x20;
      msgs[t].push_back(m);
      sigs[t].push_back(s);
      expect[t].push_back(ok);
    }
  }
  std::atomic<int> bad{0};
  const uint64_t b0 = ed25519EngineStats().batches;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      for (int k = 0; k < K; k++)
        if (vf[(t + k) % 8]->verify(msgs[t][k], sigs[t][k]) != expect[t][k]) bad++;
    });
  // meanwhile: new clients join (keys appended to the live device table)
  std::vector<std::unique_ptr<HipEdDSAVerifier>> late;
  for (int k = 0; k < 6; k++) {
    EdDSASigner s(seedHex(400 + k), KeyFormat::HexaDecimalStrippedFormat);
    late.emplace_back(new HipEdDSAVerifier(s.getPubKeyHex(), KeyFormat::HexaDecimalStrippedFormat));
    std::string m = "late client " + std::to_string(k);
    if (!late.back()->verify(m, s.sign(m))) bad++;
  }
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const uint64_t batches = ed25519EngineStats().batches - b0;
  CHECK(bad == 0);
  CHECK(batches < (uint64_t)(T * K + 6));
  std::printf("test_host: %d concurrent verify() calls in %llu GPU batches, %.0f verifies/s\n", T * K + 6,
              (unsigned long long)batches, (T * K + 6) / secs);
  return 0;
}

// Metrics idiom of the reference (SigManager.hpp:65-67,83; SigManager.cpp:208-236): counters on
// a "signature_manager" component, pushed to the aggregator on every failure and on every
// 1,000th success.  Then client key rotation reusing freed device key slots.
static int testAggregatorAndKeySlots() {
  ReplicaIdsConfig cfg;
  cfg.replicaId = 0;
  cfg.numOfExternalClients = 2;
  ReplicasInfo ri(cfg);
  std::vector<EdDSASigner> rs;
  HipSigManager::ReplicaKeys replicaKeys;
  for (int r = 0; r < 4; r++) {
    rs.emplace_back(seedHex(600 + r), KeyFormat::HexaDecimalStrippedFormat);
    replicaKeys.insert({(PrincipalId)r, rs.back().getPubKeyHex()});
  }
  EdDSASigner c4(seedHex(610), KeyFormat::HexaDecimalStrippedFormat), c5(seedHex(611), KeyFormat::HexaDecimalStrippedFormat);
  HipSigManager::ClientKeys clientKeys = {{c4.getPubKeyHex(), {4}}, {c5.getPubKeyHex(), {5}}};
  std::unique_ptr<HipSigManager> sm(HipSigManager::initInTesting(0, seedHex(600), replicaKeys,
                                                                 KeyFormat::HexaDecimalStrippedFormat, &clientKeys,
                                                                 KeyFormat::HexaDecimalStrippedFormat, ri));
  auto agg = std::make_shared<concordMetrics::Aggregator>();
  sm->SetAggregator(agg);
  auto ctr = [&](const char* name) { return (uint64_t)agg->GetCounter("signature_manager", name).Get(); };
  std::vector<std::string> d(1001), sg(1001);
  std::vector<SigBatchItem> items;
  for (int i = 0; i < 1001; i++) {
    d[i] = "replica message " + std::to_string(i);
    sg[i] = rs[1].sign(d[i]);
  }
  for (int i = 0; i < 999; i++) items.push_back({1, d[i].data(), d[i].size(), sg[i].data(), 64});
  std::vector<bool> out;
  CHECK(sm->verifySigBatch(items, out) == 999);
  CHECK(ctr("peer_replicas_signatures_verified") == 0 && agg->Pushes("signature_manager") == 0);
  CHECK(sm->verifySig(1, d[999].data(), d[999].size(), sg[999].data(), 64));  // the 1,000th success
  CHECK(ctr("peer_replicas_signatures_verified") == 1000 && agg->Pushes("signature_manager") == 1);
  std::string badsig = sg[1000];
  badsig[9] ^= 1;
  items.assign(1, {1, d[1000].data(), d[1000].size(), badsig.data(), 64});
  CHECK(sm->verifySigBatch(items, out) == 0 && !out[0]);
  CHECK(ctr("peer_replicas_signature_verification_failed") == 1 && agg->Pushes("signature_manager") == 2);
  items.assign(1, {77, d[0].data(), d[0].size(), sg[0].data(), 64});  // unknown principal
  sm->verifySigBatch(items, out);
  CHECK(ctr("signature_verification_failed_on_unrecognized_participant_id") == 1);
  CHECK(agg->Pushes("signature_manager") == 3);
  std::string cpk = sm->getClientsPublicKeys();  // CMF-encoded, every external client's key (SigManager.cpp:151-156)
  CHECK(cpk.size() >= 6);
  CHECK(cpk.find(c4.getPubKeyHex()) != std::string::npos);

  // key rotation: the new key is registered while the old one is still referenced, then the old
  // slot is freed; the second rotation therefore reuses a freed slot and the table does not grow
  const std::string m = "rotated client request";
  CHECK(sm->verifySig(4, m.data(), m.size(), c4.sign(m).data(), 64));
  const auto s0 = ed25519EngineStats();
  EdDSASigner k1(seedHex(620), KeyFormat::HexaDecimalStrippedFormat), k2(seedHex(621), KeyFormat::HexaDecimalStrippedFormat);
  sm->setClientPublicKey(k1.getPubKeyHex(), 4, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(sm->verifySig(4, m.data(), m.size(), k1.sign(m).data(), 64));
  const auto s1 = ed25519EngineStats();
  // one key in, one out; the new key took a free slot or one new slot (the engine is process-wide:
  // earlier tests may have left free slots)
  CHECK(s1.table_keys <= s0.table_keys + 1 && s1.live_keys == s0.live_keys);
  sm->setClientPublicKey(k2.getPubKeyHex(), 4, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(sm->verifySig(4, m.data(), m.size(), k2.sign(m).data(), 64));
  CHECK(!sm->verifySig(4, m.data(), m.size(), k1.sign(m).data(), 64));
  CHECK(!sm->verifySig(4, m.data(), m.size(), c4.sign(m).data(), 64));
  CHECK(sm->verifySig(5, m.data(), m.size(), c5.sign(m).data(), 64));  // the other slots are untouched
  const auto s2 = ed25519EngineStats();
  CHECK(s2.table_keys == s1.table_keys && s2.live_keys == s1.live_keys);
  CHECK(s2.gpu_errors == 0);
  std::printf("test_host: aggregator pushes and key-slot reuse passed (%u device key slots)\n", s2.table_keys);
  return 0;
}

int main() {
  bftEngine::ReplicaConfig::instance().clientTransactionSigningEnabled = true;
  if (testRsa() != 0) return 1;
  if (testKeyRotation() != 0) return 1;
  // --- IVerifier/ISigner round trip, hex and PEM key formats
  EdDSASigner signer(seedHex(0), KeyFormat::HexaDecimalStrippedFormat);
  std::string pkhex = signer.getPubKeyHex();
  HipEdDSAVerifier vhex(pkhex, KeyFormat::HexaDecimalStrippedFormat);
  std::vector<uint8_t> raw;
  fromHex(pkhex, raw);
  HipEdDSAVerifier vpem(ed25519PublicKeyToPem(raw.data()), KeyFormat::PemFormat);
  CHECK(vhex.signatureLength() == 64 && signer.signatureLength() == 64);
  std::string msg = "concord client request payload";
  std::string sig = signer.sign(msg);
  CHECK(sig.size() == 64);
  CHECK(vhex.verify(msg, sig));
  CHECK(vpem.verify(msg, sig));
  std::string bad = msg;
  bad[0]++;
  CHECK(!vhex.verify(bad, sig));
  CHECK(!vhex.verify(msg, sig.substr(0, 63)));  // length gate
  bool threw = false;
  try {
    HipEdDSAVerifier broken("zz", KeyFormat::HexaDecimalStrippedFormat);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);

  // --- SigManager: 4 replicas + 8 external clients 4..11 (ReplicasInfo layout), clients 4..7
  // share one key (SigManager.cpp:66-85: one key, many principals)
  ReplicaIdsConfig cfg;
  cfg.replicaId = 0;
  cfg.numOfExternalClients = 8;
  ReplicasInfo ri(cfg);
  std::set<std::pair<PrincipalId, const std::string>> replicaKeys;
  std::set<std::pair<const std::string, std::set<uint16_t>>> clientKeys;
  std::vector<EdDSASigner> signers;
  signers.reserve(16);
  for (int r = 0; r < 4; r++) {
    signers.emplace_back(seedHex(10 + r), KeyFormat::HexaDecimalStrippedFormat);
    replicaKeys.insert({(PrincipalId)r, signers.back().getPubKeyHex()});
  }
  for (int c = 0; c < 5; c++) {
    signers.emplace_back(seedHex(20 + c), KeyFormat::HexaDecimalStrippedFormat);
    std::set<uint16_t> ids;
    if (c == 0)
      ids = {4, 5, 6, 7};
    else
      ids = {(uint16_t)(7 + c)};
    clientKeys.insert({signers.back().getPubKeyHex(), ids});
  }
  std::unique_ptr<SigManager> smp(SigManager::initInTesting(0, seedHex(10), replicaKeys,
                                                            KeyFormat::HexaDecimalStrippedFormat, &clientKeys,
                                                            KeyFormat::HexaDecimalStrippedFormat, ri));
  SigManager& sm = *smp;
  CHECK(sm.getSigLength(0) == 64 && sm.getSigLength(999) == 0 && sm.getSigLength(4) == 64);
  {  // ids outside their ranges are refused (the reference asserts, SigManager.cpp:58,76-79)
    bool threw = false;
    std::set<std::pair<const std::string, std::set<uint16_t>>> badClients = {{signers[4].getPubKeyHex(), {2}}};
    try {
      delete SigManager::initInTesting(0, "", replicaKeys, KeyFormat::HexaDecimalStrippedFormat, &badClients,
                                       KeyFormat::HexaDecimalStrippedFormat, ri);
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    CHECK(threw);
  }
  auto signerOf = [&](PrincipalId p) -> EdDSASigner& { return p < 4 ? signers[p] : (p <= 7 ? signers[4] : signers[4 + (p - 7)]); };

  std::vector<PrincipalId> pids = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  std::vector<std::string> datas, sigs;
  std::mt19937 g(7);
  for (int i = 0; i < 300; i++) {
    PrincipalId p = pids[i % pids.size()];
    std::string d(1 + g() % 600, '\0');
    for (auto& ch : d) ch = (char)g();
    datas.push_back(d);
    sigs.push_back(signerOf(p).sign(d));
  }
  // corrupt every 7th: ++ a data byte (reference corruption model), every 11th a sig byte
  std::vector<bool> expect(300, true);
  for (int i = 0; i < 300; i++) {
    if (i % 7 == 0) {
      datas[i][0]++;
      expect[i] = false;
    } else if (i % 11 == 0) {
      sigs[i][5]++;
      expect[i] = false;
    }
  }
  std::vector<SigBatchItem> items;
  for (int i = 0; i < 300; i++)
    items.push_back({pids[i % pids.size()], datas[i].data(), datas[i].size(), sigs[i].data(), 64});
  items.push_back({999, datas[1].data(), datas[1].size(), sigs[1].data(), 64});  // unknown principal
  expect.push_back(false);

  std::vector<bool> out;
  sm.verifySigBatch(items, out);
  CHECK(out.size() == items.size());
  for (size_t i = 0; i < items.size(); i++) CHECK(out[i] == expect[i]);
  uint64_t okC = 0, okR = 0, badC = 0, badR = 0;
  for (size_t i = 0; i < 300; i++) {
    bool client = ri.isIdOfExternalClient(items[i].pid);
    CHECK(client == (items[i].pid >= 4));
    (expect[i] ? (client ? okC : okR) : (client ? badC : badR))++;
  }
  const auto m = sm.counterValues();
  CHECK(m.externalVerified == okC);
  CHECK(m.replicaVerified == okR);
  CHECK(m.externalFailed == badC);
  CHECK(m.replicaFailed == badR);
  CHECK(m.unrecognizedPid == 1);

  // single-item path agrees with the batch
  for (size_t i = 0; i < 40; i++)
    CHECK(sm.verifySig(items[i].pid, items[i].data, items[i].dataLength, items[i].sig, items[i].sigLength) ==
          expect[i]);

  // key rotation: client 8 gets a new key; old signatures fail, new ones pass
  EdDSASigner rotated(seedHex(99), KeyFormat::HexaDecimalStrippedFormat);
  sm.setClientPublicKey(rotated.getPubKeyHex(), 8, KeyFormat::HexaDecimalStrippedFormat);
  std::string d = "after rotation";
  CHECK(sm.verifySig(8, d.data(), d.size(), rotated.sign(d).data(), 64));
  CHECK(!sm.verifySig(8, d.data(), d.size(), signerOf(8).sign(d).data(), 64));
  // only external clients / client services may be rotated (SigManager.cpp:252): a replica id
  // is ignored
  sm.setClientPublicKey(rotated.getPubKeyHex(), 2, KeyFormat::HexaDecimalStrippedFormat);
  CHECK(sm.verifySig(2, d.data(), d.size(), signers[2].sign(d).data(), 64));
  CHECK(sm.getPublicKeyOfVerifier(8) == rotated.getPubKeyHex());

  // own signature
  char os[64];
  sm.sign(d.data(), d.size(), os, 64);
  CHECK(sm.verifySig(0, d.data(), d.size(), os, 64));
  if (testMessages(sm, ri, signers, signerOf) != 0) return 1;
  if (testPreProcessBatch(sm, ri, signerOf) != 0) return 1;
  if (testPreProcessResult(sm, signers) != 0) return 1;
  if (testConcurrent() != 0) return 1;
  if (testAggregatorAndKeySlots() != 0) return 1;
  std::printf("test_host: all checks passed (%zu batch items)\n", items.size());
  return 0;
}

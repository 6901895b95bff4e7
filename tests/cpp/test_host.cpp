// C++ host-side tests of the plugin layer (run on the GPU box by tests/test_cpp_host.py).
// Pattern of the reference's bftengine/tests/SigManager/SigManager_test.cpp:70-114: sign with
// one principal's key, verify through SigManager, corrupt a byte (++), expect failure and exact
// counter movements; plus the batch path against single verifies.
#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>

#include <cassert>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "crypto_utils.hpp"
#include "sig_manager.hpp"

using namespace concord::util::crypto;
using namespace bftEngine::impl;

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
  RSAVerifier vc(kc.pubHex, KeyFormat::HexaDecimalStrippedFormat), vcp(kc.pubPem, KeyFormat::PemFormat);
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
    RSAVerifier broken("3000", KeyFormat::HexaDecimalStrippedFormat);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);

  // --- SigManager with RSA replicas (e = 17, as bftengine/tests/messages/helper.cpp) and RSA +
  // Ed25519 clients in one batch: verdicts and counters as with single verifies
  EdDSASigner ed(seedHex(50), KeyFormat::HexaDecimalStrippedFormat);
  ReplicasInfo ri;
  ri.numReplicas = 4;
  ri.externalClients = {200, 201};
  std::vector<std::pair<std::set<PrincipalId>, std::string>> keys = {
      {{0, 1, 2, 3}, kr.pubHex}, {{200}, kc.pubHex}, {{201}, ed.getPubKeyHex()}};
  SigManager sm(1, {kr.privHex, KeyFormat::HexaDecimalStrippedFormat}, keys, KeyFormat::HexaDecimalStrippedFormat,
                ri);
  CHECK(sm.getSigLength(0) == 256 && sm.getSigLength(201) == 64 && sm.getMySigLength() == 256);
  RSASigner sr(kr.privHex, KeyFormat::HexaDecimalStrippedFormat);
  std::vector<std::string> datas, sigs;
  std::vector<PrincipalId> who;
  std::vector<bool> expect;
  std::mt19937 g(17);
  for (int i = 0; i < 120; i++) {
    const PrincipalId p = (i % 3 == 0) ? (PrincipalId)(i % 4) : (i % 3 == 1 ? 200 : 201);
    std::string d(1 + g() % 400, '\0');
    for (auto& ch : d) ch = (char)g();
    std::string s = p < 4 ? sr.sign(d) : (p == 200 ? sc.sign(d) : ed.sign(d));
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
  const auto& m = sm.metrics();
  CHECK(m.external_client_request_signatures_verified == okC && m.peer_replicas_signatures_verified == okR);
  CHECK(m.external_client_request_signature_verification_failed == badC);
  CHECK(m.peer_replicas_signature_verification_failed == badR);
  for (size_t i = 0; i < 12; i++)
    CHECK(sm.verifySig(who[i], datas[i].data(), datas[i].size(), sigs[i].data(), (uint16_t)sigs[i].size()) ==
          expect[i]);
  char os[256];
  sm.sign(msg.data(), msg.size(), os, 256);  // replica 1 signs with its RSA key
  CHECK(sm.verifySig(2, msg.data(), msg.size(), os, 256));
  std::printf("test_host: RSA checks passed (%zu mixed batch items)\n", items.size());
  return 0;
}

int main() {
  if (testRsa() != 0) return 1;
  // --- IVerifier/ISigner round trip, hex and PEM key formats
  EdDSASigner signer(seedHex(0), KeyFormat::HexaDecimalStrippedFormat);
  std::string pkhex = signer.getPubKeyHex();
  EdDSAVerifier vhex(pkhex, KeyFormat::HexaDecimalStrippedFormat);
  std::vector<uint8_t> raw;
  fromHex(pkhex, raw);
  EdDSAVerifier vpem(ed25519PublicKeyToPem(raw.data()), KeyFormat::PemFormat);
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
    EdDSAVerifier broken("zz", KeyFormat::HexaDecimalStrippedFormat);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);

  // --- SigManager: 4 replicas + 8 clients, clients 100..103 share one key
  ReplicasInfo ri;
  ri.numReplicas = 4;
  std::vector<std::pair<std::set<PrincipalId>, std::string>> keys;
  std::vector<EdDSASigner> signers;
  signers.reserve(16);
  for (int r = 0; r < 4; r++) {
    signers.emplace_back(seedHex(10 + r), KeyFormat::HexaDecimalStrippedFormat);
    keys.push_back({{(PrincipalId)r}, signers.back().getPubKeyHex()});
  }
  for (int c = 0; c < 5; c++) {
    signers.emplace_back(seedHex(20 + c), KeyFormat::HexaDecimalStrippedFormat);
    std::set<PrincipalId> ids;
    if (c == 0)
      ids = {100, 101, 102, 103};
    else
      ids = {(PrincipalId)(103 + c)};
    for (auto id : ids) ri.externalClients.insert(id);
    keys.push_back({ids, signers.back().getPubKeyHex()});
  }
  SigManager sm(0, {seedHex(10), KeyFormat::HexaDecimalStrippedFormat}, keys, KeyFormat::HexaDecimalStrippedFormat,
                ri);
  CHECK(sm.getSigLength(0) == 64 && sm.getSigLength(999) == 0);
  auto signerOf = [&](PrincipalId p) -> EdDSASigner& { return p < 4 ? signers[p] : (p <= 103 ? signers[4] : signers[4 + (p - 103)]); };

  std::vector<PrincipalId> pids = {0, 1, 2, 3, 100, 101, 102, 103, 104, 105, 106, 107};
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
    (expect[i] ? (client ? okC : okR) : (client ? badC : badR))++;
  }
  const auto& m = sm.metrics();
  CHECK(m.external_client_request_signatures_verified == okC);
  CHECK(m.peer_replicas_signatures_verified == okR);
  CHECK(m.external_client_request_signature_verification_failed == badC);
  CHECK(m.peer_replicas_signature_verification_failed == badR);
  CHECK(m.signature_verification_failed_on_unrecognized_participant_id == 1);

  // single-item path agrees with the batch
  for (size_t i = 0; i < 40; i++)
    CHECK(sm.verifySig(items[i].pid, items[i].data, items[i].dataLength, items[i].sig, items[i].sigLength) ==
          expect[i]);

  // key rotation: client 104 gets a new key; old signatures fail, new ones pass
  EdDSASigner rotated(seedHex(99), KeyFormat::HexaDecimalStrippedFormat);
  sm.setClientPublicKey(rotated.getPubKeyHex(), 104, KeyFormat::HexaDecimalStrippedFormat);
  std::string d = "after rotation";
  CHECK(sm.verifySig(104, d.data(), d.size(), rotated.sign(d).data(), 64));
  CHECK(!sm.verifySig(104, d.data(), d.size(), signerOf(104).sign(d).data(), 64));

  // own signature
  char os[64];
  sm.sign(d.data(), d.size(), os, 64);
  CHECK(sm.verifySig(0, d.data(), d.size(), os, 64));
  std::printf("test_host: all checks passed (%zu batch items)\n", items.size());
  return 0;
}

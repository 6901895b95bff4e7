// C++ host-side tests of the plugin layer (run on the GPU box by tests/test_cpp_host.py).
// Pattern of the reference's bftengine/tests/SigManager/SigManager_test.cpp:70-114: sign with
// one principal's key, verify through SigManager, corrupt a byte (++), expect failure and exact
// counter movements; plus the batch path against single verifies.
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

int main() {
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

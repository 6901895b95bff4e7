// C++ host-side tests of the threshsign mirror (BLS::Hip over libcbft_hipcrypto), run on the GPU
// box by tests/test_cpp_host.py.  Modelled on the reference's threshsign tests:
//   TestThresholdBls.cpp:41-84      sign -> accumulate -> combine -> verify for (n, k) pairs,
//                                   threshold and multisig schemes
//   TestBlsBatchVerifier.cpp:42-106 a bad share is detected and reported by id
//   ThresholdAccumulatorBase.cpp    pending/valid/invalid bookkeeping, digest immutability
// Key sets and expected combined signatures: tests/golden/bls_sets.txt (gen_bls_fixtures.py): the
// reference's RELIC-generated cryptosystems (set{A,B}_replica_* key files) first, then larger
// oracle-generated sets.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "threshsign/bls_hip.hpp"

using namespace BLS::Hip;

#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

struct KeySet {
  int n = 0, k = 0;
  bool multisig = false;  // independent keys, PK = sum of vks (no Lagrange combination)
  std::string sk, pk, msgHex, sigHex;
  std::vector<std::string> vk, ski;
};

static std::vector<uint8_t> unhex(const std::string& h) {
  std::vector<uint8_t> o(h.size() / 2);
  for (size_t i = 0; i < o.size(); i++) o[i] = (uint8_t)std::stoi(h.substr(2 * i, 2), nullptr, 16);
  return o;
}
static std::string hex(const char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; i++) {
    s += d[((uint8_t)p[i]) >> 4];
    s += d[((uint8_t)p[i]) & 15];
  }
  return s;
}

static std::vector<KeySet> load(const std::string& path) {
  std::vector<KeySet> sets;
  std::ifstream f(path);
  std::string line;
  KeySet cur;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string tag;
    is >> tag;
    if (tag == "set") {
      cur = KeySet();
      is >> cur.n >> cur.k;
    } else if (tag == "scheme") {
      std::string v;
      is >> v;
      cur.multisig = v == "multisig";
    } else if (tag == "sk") {
      is >> cur.sk;
    } else if (tag == "pk") {
      is >> cur.pk;
    } else if (tag == "vk") {
      int i;
      std::string h;
      is >> i >> h;
      cur.vk.push_back(h);
    } else if (tag == "ski") {
      int i;
      std::string d;
      is >> i >> d;
      cur.ski.push_back(d);
    } else if (tag == "msg") {
      is >> cur.msgHex;
    } else if (tag == "sig") {
      is >> cur.sigHex;
    } else if (tag == "end") {
      sets.push_back(cur);
    }
  }
  return sets;
}

static std::string share(const KeySet& ks, int id, const std::vector<uint8_t>& msg) {
  BlsThresholdSigner s(id, ks.ski[(size_t)id - 1], ks.vk[(size_t)id - 1]);
  std::string out(37, '\0');
  s.signData(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), &out[0], 37);
  return out;
}

static int testThreshold(const KeySet& ks) {
  const auto msg = unhex(ks.msgHex);
  std::vector<uint8_t> other = msg;
  other[0] ^= 1;
  BlsThresholdVerifier v(ks.pk, ks.k, ks.n, ks.vk);
  CHECK(v.requiredLengthForSignedData() == 33);
  CHECK(v.getPublicKey().toString() == ks.pk);
  CHECK(v.getShareVerificationKey(1).toString() == ks.vk[0]);
  {  // the signer derives its verification key on the GPU: sk_i * g2 == the fixture's vk_i
    BlsThresholdSigner s(2, ks.ski[1]);
    CHECK(s.getShareVerificationKey().toString() == ks.vk[1]);
  }

  // signer output: 4-byte big-endian id || 33-byte point
  std::string s3 = share(ks, 3, msg);
  CHECK((uint8_t)s3[0] == 0 && (uint8_t)s3[1] == 0 && (uint8_t)s3[2] == 0 && (uint8_t)s3[3] == 3);

  // group signer (sk on the fixture) signs exactly the expected combined signature
  {
    BlsThresholdSigner g(1, ks.sk, "");
    std::string out(37, '\0');
    g.signData(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), &out[0], 37);
    CHECK(hex(out.data() + 4, 33) == ks.sigHex);
  }

  const bool almost = (ks.k == ks.n - 1);
  // (1) with share verification: shares added before the digest are pending; one bad share
  // (signed over another digest, like the reference's doubled share) must be reported.
  {
    std::unique_ptr<IThresholdAccumulator> acc(v.newAccumulator(true));
    CHECK(acc->hasShareVerificationEnabled() == !almost);
    const int bad = 2;
    for (int id = 1; id <= ks.n; id++) {
      std::string sh = id == bad ? share(ks, id, other) : share(ks, id, msg);
      int c = acc->add(sh.data(), (int)sh.size());
      if (!almost) CHECK(c == id);  // pending count
    }
    if (!almost) CHECK(acc->getNumValidShares() == 0);
    acc->setExpectedDigest(msg.data(), (int)msg.size());
    acc->setExpectedDigest(msg.data(), (int)msg.size());  // same digest again: allowed
    bool threw = false;
    try {
      acc->setExpectedDigest(other.data(), (int)other.size());
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
    if (!almost && ks.n - 1 < ks.k) {  // n-of-n: one bad share leaves the set short
      CHECK(acc->getNumValidShares() == ks.n - 1);
      auto inv = acc->getInvalidShareIds();
      CHECK(inv.size() == 1 && *inv.begin() == bad);
    } else if (!almost) {
      CHECK(acc->getNumValidShares() == ks.k);
      auto inv = acc->getInvalidShareIds();
      CHECK(inv.size() == 1 && *inv.begin() == bad);
      std::string sig(33, '\0');
      acc->getFullSignedData(&sig[0], 33);
      CHECK(hex(sig.data(), 33) == ks.sigHex);
      CHECK(v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), sig.data(), 33));
      CHECK(!v.verify(reinterpret_cast<const char*>(other.data()), (int)other.size(), sig.data(), 33));
      CHECK(!v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), sig.data(), 32));
      threw = false;
      try {
        acc->getFullSignedData(&sig[0], 32);
      } catch (const std::runtime_error&) {
        threw = true;
      }
      CHECK(threw);
    }
  }
  // (2) without verification: the last k signers, added after the digest; extra shares ignored
  {
    std::unique_ptr<IThresholdAccumulator> acc(v.newAccumulator(false));
    acc->setExpectedDigest(msg.data(), (int)msg.size());
    int c = 0;
    for (int id = ks.n; id >= 1; id--) {
      std::string sh = share(ks, id, msg);
      c = acc->add(sh.data(), (int)sh.size());
      std::string dup = share(ks, id, msg);  // the same signer twice: not counted again
      CHECK(acc->add(dup.data(), (int)dup.size()) == c);
    }
    CHECK(c == ks.k && acc->getNumValidShares() == ks.k);
    std::string sig(33, '\0');
    acc->getFullSignedData(&sig[0], 33);
    CHECK(hex(sig.data(), 33) == ks.sigHex);
  }
  // (3) verification on, digest first: each add verifies; a bad share is not counted
  if (!almost) {
    std::unique_ptr<IThresholdAccumulator> acc(v.newAccumulator(true));
    acc->setExpectedDigest(msg.data(), (int)msg.size());
    std::string badsh = share(ks, 1, other);
    CHECK(acc->add(badsh.data(), (int)badsh.size()) == 0);
    for (int id = 1; id <= ks.k; id++) {
      std::string sh = share(ks, id, msg);
      CHECK(acc->add(sh.data(), (int)sh.size()) == id);
    }
    std::string sig(33, '\0');
    acc->getFullSignedData(&sig[0], 33);
    CHECK(hex(sig.data(), 33) == ks.sigHex);
  }
  return 0;
}

static int testMultisig(const KeySet& ks) {
  const auto msg = unhex(ks.msgHex);
  BlsMultisigVerifier v(ks.k, ks.n, ks.vk);
  const bool nofn = ks.k == ks.n;
  CHECK(v.requiredLengthForSignedData() == (nofn ? 33 : 33 + 256));
  std::unique_ptr<IThresholdAccumulator> acc(v.newAccumulator(false));
  acc->setExpectedDigest(msg.data(), (int)msg.size());
  for (int id = 1; id <= ks.k; id++) {
    std::string sh = share(ks, id, msg);
    acc->add(sh.data(), (int)sh.size());
  }
  std::string sig((size_t)v.requiredLengthForSignedData(), '\0');
  acc->getFullSignedData(&sig[0], (int)sig.size());
  CHECK(v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), sig.data(), (int)sig.size()));
  std::string wrong = sig;
  wrong[5] ^= 1;
  CHECK(!v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), wrong.data(), (int)wrong.size()));
  if (!nofn) {
    // bitmap = signers 1..k, LSB first (VectorOfShares::toBytes)
    CHECK((uint8_t)sig[33] == (uint8_t)((1u << ks.k) - 1));
    std::string fewer = sig;
    fewer[33] = (char)((uint8_t)fewer[33] & ~(1u << (ks.k - 1)));  // k - 1 signers: below threshold
    CHECK(!v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), fewer.data(), (int)fewer.size()));
    std::string other = sig;
    other[33] = (char)(((uint8_t)other[33] & ~1u) | (1u << ks.k));  // another signer set
    CHECK(!v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), other.data(), (int)other.size()));
    bool threw = false;
    try {
      v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), sig.data(), 33);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
  }
  return 0;
}

// A RELIC multisig cryptosystem (independent keys): the n-of-n verifier's key is the sum of the
// vks and must equal the file's group key; the n-share aggregate equals group_sk * H(m) and
// verifies under that key (BlsMultisigVerifier.cpp:33-38,75-105).
static int testMultisigKeys(const KeySet& ks) {
  const auto msg = unhex(ks.msgHex);
  BlsMultisigVerifier v(ks.n, ks.n, ks.vk);
  CHECK(v.getPublicKey().toString() == ks.pk);
  std::unique_ptr<IThresholdAccumulator> acc(v.newAccumulator(true));
  acc->setExpectedDigest(msg.data(), (int)msg.size());
  for (int id = 1; id <= ks.n; id++) {
    std::string sh = share(ks, id, msg);
    CHECK(acc->add(sh.data(), (int)sh.size()) == id);
  }
  std::string sig(33, '\0');
  acc->getFullSignedData(&sig[0], 33);
  CHECK(hex(sig.data(), 33) == ks.sigHex);
  CHECK(v.verify(reinterpret_cast<const char*>(msg.data()), (int)msg.size(), sig.data(), 33));
  return 0;
}

int main(int argc, char** argv) {
  const std::string path = argc > 1 ? argv[1] : "tests/golden/bls_sets.txt";
  auto sets = load(path);
  CHECK(sets.size() >= 4);
  for (const auto& ks : sets) {
    std::printf("set n=%d k=%d %s\n", ks.n, ks.k, ks.multisig ? "multisig" : "threshold");
    if (!ks.multisig && testThreshold(ks)) return 1;
    if (ks.multisig && testMultisigKeys(ks)) return 1;
    if (testMultisig(ks)) return 1;
  }
  // key parsing errors throw
  bool threw = false;
  try {
    BlsPublicKey bad("abcd");
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  threw = false;
  try {
    BlsSecretKey bad("12x4");
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  std::printf("all checks passed\n");
  return 0;
}

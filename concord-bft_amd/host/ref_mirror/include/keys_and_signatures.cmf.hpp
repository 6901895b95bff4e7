// Standalone-build restatement of the CMF-generated keys_and_signatures.cmf.hpp
// (bftengine/src/bftengine/messages/keys_and_signatures.cmf: PublicKey { string key; uint8 format },
// ClientsPublicKeys { map uint16 PublicKey ids_to_keys; uint16 version }).  The reference build
// generates this header from the .cmf file; only the two structs HipSigManager writes are here.
#pragma once

#include <cstdint>
#include <map>
#include <string>

namespace concord::messages::keys_and_signatures {
struct PublicKey {
  std::string key;
  uint8_t format{};
};
struct ClientsPublicKeys {
  std::map<uint16_t, PublicKey> ids_to_keys;
  uint16_t version{};
};
}  // namespace concord::messages::keys_and_signatures

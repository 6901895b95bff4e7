// Standalone-build restatement of the one ReplicaConfig field the signature path reads:
// clientTransactionSigningEnabled (bftengine/include/bftengine/ReplicaConfig.hpp:38-44,90-91),
// through the reference's process-wide ReplicaConfig::instance().  See ../README.md.
#pragma once

namespace bftEngine {
class ReplicaConfig {
 public:
  static ReplicaConfig& instance() {
    static ReplicaConfig config_;
    return config_;
  }
  bool clientTransactionSigningEnabled = false;
};
}  // namespace bftEngine

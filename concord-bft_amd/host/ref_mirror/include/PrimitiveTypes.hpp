// Standalone-build restatement of bftengine/src/bftengine/PrimitiveTypes.hpp:29-40 (the id and
// size typedefs the SigManager path uses).  See ../README.md.
#pragma once

#include <cstdint>

namespace bftEngine {
namespace impl {
typedef int64_t SeqNum;
typedef int64_t ViewNum;
typedef uint16_t PrincipalId;  // ReplicaId or NodeIdType
typedef uint16_t ReplicaId;
typedef uint16_t NodeIdType;
typedef uint32_t MsgSize;
typedef uint16_t MsgType;
typedef uint32_t SpanContextSize;
}  // namespace impl
}  // namespace bftEngine

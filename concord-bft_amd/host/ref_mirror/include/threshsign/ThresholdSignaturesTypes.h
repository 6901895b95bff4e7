// Mirror of threshsign/include/threshsign/ThresholdSignaturesTypes.h:25-28 (the types the
// threshold interfaces use).  The reference's Cryptosystem class (same file, :41-294) is the
// injection point: its virtual createThresholdVerifier/createThresholdSigner are overridden to
// return the BLS::Hip objects of bls_hip.hpp.
#pragma once

#include <cstdint>

typedef int ShareID;
typedef ShareID NumSharesType;

#define MAX_NUM_OF_SHARES 2048

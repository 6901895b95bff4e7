// Internal state of libcbft_hipcrypto shared by the Ed25519 (cbft_hipcrypto.cpp) and BLS
// (cbft_bls.cpp) halves of the C ABI.  Not installed; not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cbft_hipcrypto.h"
#include "ed25519_verify.h"
#include "rsa_verify.h"

// Pinned host staging buffer (hipHostMalloc): the host-buffer entry points pack their inputs
// into it and move them with one DMA copy instead of one pageable copy per array.
struct HostBuf {
  void* p = nullptr;
  void* dev = nullptr;  // the same memory as kernels address it (zero-copy reads and writes)
  size_t cap = 0;
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dev, p, 0);
    if (e != hipSuccess) {
      if (p) (void)hipHostFree(p);
      p = dev = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    cap = 0;
  }
  template <class T>
  T* as(size_t off = 0) const { return reinterpret_cast<T*>(static_cast<uint8_t*>(p) + off); }
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // (re)allocate to at least `bytes`; contents are not preserved
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      (void)hipDeviceSynchronize();  // an earlier async launch may still read the old buffer
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// An Ed25519 key table: chunks of CBFT_KEY_CHUNK keys (comb tables of -A, raw keys, decode
// status; ed25519_verify.h KeyChunks).  Keys are appended into the last chunk / new chunks while
// verifies against the already published keys keep running; `nkeys` (read and written under the
// context's mutex) is raised only once the new keys' tables are built.
struct KeyTable {
  uint32_t nkeys = 0;     // published keys
  CombGeom geo{};         // radix of the per-key comb tables
  std::vector<DevBuf> chunks;
  DevBuf chunk_ptrs;      // CBFT_MAX_KEY_CHUNKS device pointers (only appended)
  std::mutex append_mu;   // one append (or the unload) at a time
  KeyChunks view() const { return KeyChunks{chunk_ptrs.as<const uint32_t* const>(), geo.words_per_unit()}; }
};

// BLS verifier key set: group public key + n share verification keys, decoded and with their
// Miller-loop lines precomputed (slot 0 = PK, slot i = vk_i)
struct BlsKeySet {
  uint32_t n = 0;
  DevBuf keys65, lines, ok, aff;  // aff: decoded affine keys (BLS_G2A_WORDS each)
};

// Per-batch intermediate state of one in-flight verify (h, S<L flags, R' coordinates, the
// per-signature key tables).  A context rotates over work_slots (<= CBFT_MAX_WORK_SLOTS) of them
// so that consecutive device-path batches on different streams overlap (batch i's finish and
// batch i+1's hash run together, each alone would leave the SIMDs half idle); a slot's `done`
// event orders its reuse after its previous batch.  With two streams two slots are enough (each
// stream's order already serialises its own batches); callers with more streams in flight
// (config #3's long-message tails) use more (CBFT_OPT_WORK_SLOTS, default 4).
#define CBFT_MAX_WORK_SLOTS 8
struct WorkSlot {
  DevBuf h, flags, xyz, ps_tbl, ps_aok;
  DevBuf perm, buckets;  // hash order of a variable-length batch (counting sort by SHA-512 blocks)
  hipStream_t aux = nullptr;                        // long-message hash stream (ed25519_hash_long_kernel)
  hipEvent_t fork = nullptr, join = nullptr;
  hipEvent_t done = nullptr;
  bool used = false;
};

// One in-flight host-buffer batch (cbft_ed25519_verify_batch_async and the blocking calls built on
// it).  Inputs are DMA'd from the caller's pinned memory (cbft_host_alloc) straight into `in`,
// or packed into `pack` first when they are pageable; the copy runs on the context's copy stream
// while earlier batches' kernels run on the compute streams.  A slot is reused only after its
// previous batch was collected (verdict words copied to that batch's bitmap).
#define CBFT_HOST_SLOTS 16
struct HostSlot {
  DevBuf in, verd;      // packed device inputs, device verdict words
  HostBuf pack, hverd;  // pinned packing image for pageable inputs, pinned verdict words
  hipEvent_t copied = nullptr, done = nullptr;
  // fused small batches complete on a blocking-sync event: their waiters sleep instead of
  // spinning, so dozens of concurrent per-request callers do not burn the host's cores
  hipEvent_t done_blk = nullptr;
  hipEvent_t wait_ev = nullptr;  // the event the pending batch completes on
  std::mutex m;         // guards the fields below (collect vs. reuse)
  uint64_t ticket = 0;  // batch currently owning the slot
  bool pending = false; // submitted, verdicts not yet delivered
  int status = 0;       // CBFT_* of the submission
  uint8_t* bitmap = nullptr;
  size_t n = 0;
};

// RSA verifier key table: per-key records (modulus, R^2 mod n, n0inv, e, validity) built on the
// GPU at load time (one verifier per key, SigManager.cpp:139-150)
struct RsaKeyTable {
  uint32_t nkeys = 0;
  DevBuf rec;
};

struct cbft_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // multi-GPU context (cbft_open_mask): one child context per device, static contiguous shards
  std::vector<cbft_ctx*> kids;
  std::mutex group_mu;
  std::unordered_map<uint64_t, std::vector<std::pair<size_t, uint64_t>>> group_tickets;  // ticket -> (kid, kid ticket)
  // host-buffer pipeline
  hipStream_t copy_stream = nullptr;
  hipStream_t compute[2] = {nullptr, nullptr};
  // fused small batches (the per-request path) rotate over their own streams, created on first
  // use, so that concurrent callers' batches run side by side instead of queueing on compute[]
  // (4 streams: kernels of different streams overlap only as far as the process has hardware
  // queues, GPU_MAX_HW_QUEUES = 4 by default)
#define CBFT_SMALL_STREAMS 4
  hipStream_t small_streams[CBFT_SMALL_STREAMS] = {};
  HostSlot hslots[CBFT_HOST_SLOTS];
  uint64_t next_ticket = 0;
  DevBuf base_table, base_comb;
  std::unordered_map<uint32_t, std::shared_ptr<KeyTable>> tables;
  hipStream_t build_stream = nullptr;  // key-table builds (appends), apart from the verify streams
  uint32_t next_table_id = 1;
  // per-batch work buffers
  WorkSlot slots[CBFT_MAX_WORK_SLOTS];
  int work_slots = 4;  // CBFT_OPT_WORK_SLOTS (1 .. CBFT_MAX_WORK_SLOTS)
  // the next batch's hash waits for this batch's SHORT-message hash only, not for the long tail
  // hashing on the slot's aux stream (CBFT_OPT_HASH_ORDER_EARLY, default 1)
  int hash_order_early = 1;
  unsigned next_slot = 0;
  int finish_k = 0;  // signatures per finish lane (CBFT_OPT_FINISH_K; 0 = 2 from 16K, else 1)
  // Stage order across batches (any streams): batch i+1's hash starts after batch i's hash and
  // its ladder after batch i's ladder, so the pipeline runs hash(i+1) / finish(i) beside
  // ladder-to-ladder instead of two streams marching in phase (both finishes together, 7/8 of
  // the SIMDs idle).  CBFT_OPT_STAGE_ORDER: 0 off, 1 hash + ladder, 2 ladder only.
  int stage_order = 1;
  // the same for variable-length (block-count sorted) batches: ladders only, so consecutive
  // batches' hash stages (whose long-message tails set their latency) overlap (config #3 A/B:
  // hash + ladder 219, ladders only 228-231 M/s)
  static constexpr int stage_order_var = 2;
  // streams of the last ordered-size batches: with three or more distinct streams in flight each
  // stream's hash -> ladder -> finish chain already covers three batches, and the order only
  // serialises them (headline at 20 steps, 3 streams: unordered 461-493 vs ordered 451-471 M/s);
  // batches below 4,096 signatures (latency-bound single waves per stage) always run unordered
  hipStream_t recent_streams[4] = {};
  unsigned recent_n = 0;
  static constexpr int order_max_streams = 2;
  static constexpr size_t stage_order_min = 4096;
  // key-table batches up to this size run as one fused launch (ed25519_small3_kernel;
  // CBFT_OPT_SMALL_MAX, 0 = never): the per-request coalescer's batches
  size_t small_max = 1024;
  size_t sha_sort_min = 4096;  // variable-length batches from this size hash in block-count order
  int b_radix = CBFT_COMB_B_RADIX;  // radix of B's comb table (CBFT_OPT_B_RADIX, 16..26)
  int ladder_lanes = 0;             // comb ladder lanes per signature (CBFT_OPT_LADDER_LANES 2 | 4; 0 = by batch)
  hipEvent_t stage_done[2] = {nullptr, nullptr};  // last hash, last ladder
  bool stage_used = false;
  DevBuf verdicts;
  DevBuf sig, msg, off, len, kidx, pk;
  std::vector<uint64_t> host_verdicts;
  std::vector<uint64_t> host_off;  // rebased message offsets of a host RSA batch
  HostBuf hstage;  // packed host inputs + verdict words of the host-buffer path
  DevBuf dstage;   // the same packing on the device
  // profiling: events around K1 (hash), K3 (ladder), K4 (finish) of the last verify
  bool profiling = false;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool ev_valid = false;
  // profiling mode 2: a ring of per-batch event quads, so pipelined batches keep their own
  // timings (cbft_stage_times_avg_ms averages them)
  std::vector<hipEvent_t> ring;
  size_t ring_n = 0;
  int prof_mode = 0;
  // BLS
  std::unordered_map<uint32_t, BlsKeySet> bls_sets;
  uint32_t next_bls_id = 1;
  // RSA
  std::unordered_map<uint32_t, RsaKeyTable> rsa_tables;
  uint32_t next_rsa_id = 1;
  DevBuf rsa_scratch, rsa_sig, rsa_kidx;
  hipEvent_t rsa_done = nullptr;  // orders reuse of rsa_scratch across streams
  bool rsa_used = false;
  hipEvent_t rsa_ev[2] = {nullptr, nullptr};  // around the last RSA kernel when profiling
  bool rsa_ev_valid = false;
  DevBuf bls_gen_lines, bls_msg, bls_H, bls_shares, bls_valid, bls_sig, bls_ids, bls_use, bls_lambda,
      bls_partial, bls_out, bls_ms_ok, bls_bitmap, bls_inv, bls_first, bls_flag, bls_g2tmp;
  DevBuf bls_aff;      // the last combine's signature as an affine point (BLS_SIG_WORDS)
  DevBuf bls_pub_tbl;  // fixed-base comb of g2 for cbft_bls_public_key (built at its first call)
};

int cbft_fail(hipError_t e, const char* what, const char* file, int line);
// the context BLS / RSA / profiling calls run on (a multi-GPU context's first device)
cbft_ctx* cbft_dev0(cbft_ctx* c);

#define CBFT_HIP(expr)                                                          \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) return cbft_fail(_e, #expr, __FILE__, __LINE__);      \
  } while (0)

// Run f(kid index) for every device of a multi-GPU context, one host thread per device (each
// device's calls take its own context mutex, so the devices work concurrently); the first
// failure's code is returned.
template <class F>
static int for_each_kid(cbft_ctx* c, F f) {
  const size_t G = c->kids.size();
  std::vector<int> rc(G, CBFT_OK);
  std::vector<std::thread> th;
  th.reserve(G);
  for (size_t g = 0; g < G; g++) th.emplace_back([&, g] { rc[g] = f(g); });
  for (auto& t : th) t.join();
  for (int r : rc)
    if (r) return r;
  return CBFT_OK;
}

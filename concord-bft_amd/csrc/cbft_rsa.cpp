// libcbft_hipcrypto, RSA half of the C ABI (include/cbft_hipcrypto.h).
//
// Replaces concord::util::crypto::RSAVerifier (util/src/crypto_utils.cpp:101-117,155-168):
// SigManager builds one verifier per replica / client key (SigManager.cpp:138,146,255); here a
// key table is loaded once (records built on the GPU) and every verify is a batch on the GPU.
//
// Multi-GPU contexts (cbft_open_mask / cbft_open_devices): key tables are loaded on every device
// (concurrently, table ids in step) and a host-buffer batch is cut into contiguous shards of whole
// 64-signature verdict words, one per device, verified concurrently (one host thread per device),
// each shard's verdicts landing in place in the caller's bitmap -- as for Ed25519 (SURVEY.md
// §8(e)).  The _device entry point needs a single-GPU context (CBFT_EINVAL otherwise).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cbft_internal.h"

static_assert(CBFT_RSA_MODULUS_BYTES == RSA_MOD_BYTES, "modulus size");

static int rsa_launch_locked(cbft_ctx* c, RsaKeyTable& kt, const uint32_t* d_kidx, const uint8_t* d_sig,
                             const uint8_t* d_msg, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                             uint64_t* d_verdicts, hipStream_t s) {
  CBFT_HIP(c->rsa_scratch.reserve(cbft_rsa_scratch_words(n) * sizeof(uint32_t)));
  if (!c->rsa_done) CBFT_HIP(hipEventCreateWithFlags(&c->rsa_done, hipEventDisableTiming));
  if (c->rsa_used) CBFT_HIP(hipStreamWaitEvent(s, c->rsa_done, 0));  // scratch reuse across streams
  RsaBatch b{n, kt.rec.as<uint32_t>(), kt.nkeys, d_kidx, d_sig, d_msg, d_off, d_len};
  if (c->profiling) {
    if (!c->rsa_ev[0])
      for (hipEvent_t& e : c->rsa_ev) CBFT_HIP(hipEventCreate(&e));
    CBFT_HIP(hipEventRecord(c->rsa_ev[0], s));
  }
  CBFT_HIP(cbft_rsa_launch_verify(b, c->rsa_scratch.as<uint32_t>(), d_verdicts, s));
  if (c->profiling) CBFT_HIP(hipEventRecord(c->rsa_ev[1], s));
  CBFT_HIP(hipEventRecord(c->rsa_done, s));
  c->rsa_used = true;
  c->rsa_ev_valid = c->profiling;
  return CBFT_OK;
}

extern "C" {

// One device's key records under `want_id` (chosen by a multi-device parent, so every device
// holds the table under the same id) or under the device's next id when want_id == 0.
static int rsa_load_on(cbft_ctx* c, const uint8_t* moduli, const uint32_t* exponents, uint32_t nkeys,
                       uint32_t want_id, uint32_t* out_id) {
  std::lock_guard<std::mutex> g(c->mu);
  if (want_id && c->rsa_tables.count(want_id)) return CBFT_EIO;
  CBFT_HIP(hipSetDevice(c->device));
  RsaKeyTable kt;
  kt.nkeys = nkeys;
  const size_t nk = std::max<uint32_t>(nkeys, 1);
  CBFT_HIP(kt.rec.reserve(nk * RSA_KEY_WORDS * sizeof(uint32_t)));
  if (nkeys) {
    DevBuf mod, ex;
    hipError_t e = mod.reserve((size_t)nkeys * RSA_MOD_BYTES);
    if (e == hipSuccess) e = ex.reserve((size_t)nkeys * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(mod.p, moduli, (size_t)nkeys * RSA_MOD_BYTES, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ex.p, exponents, (size_t)nkeys * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = cbft_rsa_launch_keys(mod.as<uint8_t>(), ex.as<uint32_t>(), nkeys, kt.rec.as<uint32_t>(), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    mod.release();
    ex.release();
    if (e != hipSuccess) {
      kt.rec.release();
      return cbft_fail(e, "rsa key records", __FILE__, __LINE__);
    }
  }
  const uint32_t id = want_id ? want_id : c->next_rsa_id++;
  c->rsa_tables.emplace(id, std::move(kt));
  *out_id = id;
  return CBFT_OK;
}

int cbft_rsa_load_keys(cbft_ctx* c, const uint8_t* moduli, const uint32_t* exponents, uint32_t nkeys,
                       uint32_t* out_id) {
  if (!c || !out_id || (nkeys && (!moduli || !exponents))) return CBFT_EINVAL;
  if (c->kids.empty()) return rsa_load_on(c, moduli, exponents, nkeys, 0, out_id);
  // every device, concurrently, under one id the parent allocates; a device that failed leaves
  // no table behind on the others (they unload theirs), so ids stay in step for later loads
  uint32_t id;
  {
    std::lock_guard<std::mutex> g(c->mu);
    id = c->next_rsa_id++;
  }
  std::vector<int> rcs(c->kids.size(), CBFT_OK);
  (void)for_each_kid(c, [&](size_t g) {
    uint32_t got = 0;
    return rcs[g] = rsa_load_on(c->kids[g], moduli, exponents, nkeys, id, &got);
  });
  int rc = CBFT_OK;
  for (int r : rcs)
    if (r && !rc) rc = r;
  if (rc) {
    for (size_t g = 0; g < c->kids.size(); g++)
      if (rcs[g] == CBFT_OK) (void)cbft_rsa_unload_keys(c->kids[g], id);
    return rc;
  }
  *out_id = id;
  return CBFT_OK;
}

int cbft_rsa_unload_keys(cbft_ctx* c, uint32_t id) {
  if (!c) return CBFT_EINVAL;
  if (!c->kids.empty()) {
    int rc = CBFT_OK;
    for (cbft_ctx* k : c->kids) {
      const int r = cbft_rsa_unload_keys(k, id);
      if (r && !rc) rc = r;
    }
    return rc;
  }
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->rsa_tables.find(id);
  if (it == c->rsa_tables.end()) return CBFT_EINVAL;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();  // in-flight device-path batches on caller streams read it
  it->second.rec.release();
  c->rsa_tables.erase(it);
  return CBFT_OK;
}

int cbft_rsa_key_status(cbft_ctx* c, uint32_t id, uint8_t* out_ok) {
  c = cbft_dev0(c);
  if (!c || !out_ok) return CBFT_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->rsa_tables.find(id);
  if (it == c->rsa_tables.end()) return CBFT_EINVAL;
  CBFT_HIP(hipSetDevice(c->device));
  std::vector<uint32_t> rec((size_t)it->second.nkeys * RSA_KEY_WORDS);
  if (!rec.empty())
    CBFT_HIP(hipMemcpy(rec.data(), it->second.rec.p, rec.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t k = 0; k < it->second.nkeys; k++) out_ok[k] = rec[(size_t)k * RSA_KEY_WORDS + RSA_KEY_OK] ? 1 : 0;
  return CBFT_OK;
}

int cbft_rsa_verify_batch(cbft_ctx* c, uint32_t id, const uint32_t* key_idx, const uint8_t* sig,
                          const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                          uint8_t* bitmap) {
  if (!c || (n && (!key_idx || !sig || !msg_off || !msg_len || !bitmap))) return CBFT_EINVAL;
  if (n == 0) return CBFT_OK;
  if (!c->kids.empty()) {  // contiguous shards of whole 64-signature words, one per device
    const size_t G = c->kids.size();
    const size_t per = (((n + G - 1) / G) + 63) / 64 * 64;
    return for_each_kid(c, [&](size_t g) {
      const size_t lo = g * per;
      if (lo >= n) return (int)CBFT_OK;
      const size_t m = std::min(n, lo + per) - lo;
      return cbft_rsa_verify_batch(c->kids[g], id, key_idx + lo, sig + lo * RSA_MOD_BYTES, msg_blob, msg_off + lo,
                                   msg_len + lo, m, bitmap + lo / 8);
    });
  }
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->rsa_tables.find(id);
  if (it == c->rsa_tables.end()) return CBFT_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (key_idx[i] >= it->second.nkeys) return CBFT_EINVAL;
  // the batch's messages are the blob range [lo, hi) its offsets span: only that range moves
  // (a shard of a multi-GPU batch carries its own part of the caller's blob), offsets rebased
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t i = 0; i < n; i++) {
    lo = std::min<uint64_t>(lo, msg_off[i]);
    hi = std::max<uint64_t>(hi, msg_off[i] + msg_len[i]);
  }
  if (hi > lo && !msg_blob) return CBFT_EINVAL;
  const uint64_t blob = hi > lo ? hi - lo : 0;
  c->host_off.resize(n);
  for (size_t i = 0; i < n; i++) c->host_off[i] = msg_off[i] - lo;
  CBFT_HIP(hipSetDevice(c->device));
  CBFT_HIP(c->rsa_kidx.reserve(n * 4));
  CBFT_HIP(c->rsa_sig.reserve(n * RSA_MOD_BYTES));
  CBFT_HIP(c->msg.reserve(blob + 16));
  CBFT_HIP(c->off.reserve(n * 8));
  CBFT_HIP(c->len.reserve(n * 4));
  CBFT_HIP(c->verdicts.reserve(((n + 63) / 64) * 8));
  CBFT_HIP(hipMemcpyAsync(c->rsa_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c->stream));
  CBFT_HIP(hipMemcpyAsync(c->rsa_sig.p, sig, n * RSA_MOD_BYTES, hipMemcpyHostToDevice, c->stream));
  if (blob) CBFT_HIP(hipMemcpyAsync(c->msg.p, msg_blob + lo, blob, hipMemcpyHostToDevice, c->stream));
  CBFT_HIP(hipMemcpyAsync(c->off.p, c->host_off.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  CBFT_HIP(hipMemcpyAsync(c->len.p, msg_len, n * 4, hipMemcpyHostToDevice, c->stream));
  int rc = rsa_launch_locked(c, it->second, c->rsa_kidx.as<uint32_t>(), c->rsa_sig.as<uint8_t>(),
                             c->msg.as<uint8_t>(), c->off.as<uint64_t>(), c->len.as<uint32_t>(), n,
                             c->verdicts.as<uint64_t>(), c->stream);
  if (rc) return rc;
  const size_t nw = (n + 63) / 64;
  c->host_verdicts.resize(nw);
  CBFT_HIP(hipMemcpyAsync(c->host_verdicts.data(), c->verdicts.p, nw * 8, hipMemcpyDeviceToHost, c->stream));
  CBFT_HIP(hipStreamSynchronize(c->stream));
  const size_t nbytes = (n + 7) / 8;
  std::memcpy(bitmap, c->host_verdicts.data(), nbytes);  // little-endian host: words == bytes
  if (n % 8) bitmap[nbytes - 1] &= (uint8_t)((1u << (n % 8)) - 1);
  return CBFT_OK;
}

int cbft_rsa_verify_batch_device(cbft_ctx* c, uint32_t id, const uint32_t* d_key_idx, const uint8_t* d_sig,
                                 const uint8_t* d_msg, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                                 uint64_t* d_verdicts, void* stream) {
  if (c && !c->kids.empty()) return CBFT_EINVAL;  // device pointers belong to one GPU: use its own context
  if (!c || (n && (!d_key_idx || !d_sig || !d_off || !d_len || !d_verdicts))) return CBFT_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_sig) & 3) return CBFT_EINVAL;  // signatures are read as words
  if (n == 0) return CBFT_OK;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->rsa_tables.find(id);
  if (it == c->rsa_tables.end()) return CBFT_EINVAL;
  CBFT_HIP(hipSetDevice(c->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  return rsa_launch_locked(c, it->second, d_key_idx, d_sig, d_msg, d_off, d_len, n, d_verdicts, s);
}

int cbft_rsa_kernel_ms(cbft_ctx* c, float* out_ms) {
  c = cbft_dev0(c);
  if (!c || !out_ms) return CBFT_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->rsa_ev_valid) return CBFT_EINVAL;
  CBFT_HIP(hipSetDevice(c->device));
  CBFT_HIP(hipEventSynchronize(c->rsa_ev[1]));
  CBFT_HIP(hipEventElapsedTime(out_ms, c->rsa_ev[0], c->rsa_ev[1]));
  return CBFT_OK;
}

}  // extern "C"

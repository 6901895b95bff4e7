/* Host-CPU Ed25519 path of the reference idiom: OpenSSL EVP_DigestVerify(ED25519), success only
 * on == 1 (util/src/openssl_crypto.cpp:229-253), one EVP_PKEY cached per public key (as
 * SigManager caches one verifier per key, SigManager.cpp:139-150), T pthreads over static
 * contiguous ranges (BASELINE.md "CPU-baseline plan").  Also signs (fixture generation).
 *
 * This is the measured CPU baseline (bench.py cpu_baseline, kind "reference") and a test-side
 * signer/ground truth; it is never linked into libcbft_hipcrypto. */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  EVP_PKEY** keys;
  const uint32_t* key_idx;
  const uint8_t* sig;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint8_t* out;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi; i++) {
    EVP_PKEY* k = j->keys[j->key_idx ? j->key_idx[i] : i];
    int ok = 0;
    if (k && EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, k) == 1)
      ok = EVP_DigestVerify(ctx, j->sig + 64 * i, 64, j->blob + j->off[i], j->len[i]) == 1;
    j->out[i] = (uint8_t)ok;
    EVP_MD_CTX_reset(ctx);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

/* Returns an opaque key cache for nkeys raw 32-byte public keys. */
void* cbft_cpu_keys_new(const uint8_t* pk, uint32_t nkeys) {
  EVP_PKEY** keys = (EVP_PKEY**)calloc(nkeys ? nkeys : 1, sizeof(EVP_PKEY*));
  for (uint32_t i = 0; i < nkeys; i++) keys[i] = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pk + 32 * i, 32);
  return keys;
}
void cbft_cpu_keys_free(void* h, uint32_t nkeys) {
  EVP_PKEY** keys = (EVP_PKEY**)h;
  for (uint32_t i = 0; i < nkeys; i++) EVP_PKEY_free(keys[i]);
  free(keys);
}

/* Verify n signatures on `threads` threads; out[i] = 0/1. */
int cbft_cpu_verify(void* keycache, const uint32_t* key_idx, const uint8_t* sig, const uint8_t* blob,
                    const uint64_t* off, const uint32_t* len, size_t n, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  job_t* jobs = (job_t*)calloc(threads, sizeof(job_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){(EVP_PKEY**)keycache, key_idx, sig, blob, off, len, n * t / threads, n * (t + 1) / threads, out};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/* Key derivation and signing from 32-byte seeds (RFC 8032 §5.1.5-6 via OpenSSL). */
int cbft_cpu_pubkey(const uint8_t sk[32], uint8_t pk[32]) {
  EVP_PKEY* k = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, sk, 32);
  if (!k) return -1;
  size_t l = 32;
  int rc = EVP_PKEY_get_raw_public_key(k, pk, &l) == 1 ? 0 : -1;
  EVP_PKEY_free(k);
  return rc;
}

typedef struct {
  EVP_PKEY** sks;
  const uint32_t* key_idx;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint8_t* sig;
} sjob_t;

static void* sworker(void* arg) {
  sjob_t* j = (sjob_t*)arg;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi; i++) {
    size_t sl = 64;
    EVP_DigestSignInit(ctx, NULL, NULL, NULL, j->sks[j->key_idx[i]]);
    EVP_DigestSign(ctx, j->sig + 64 * i, &sl, j->blob + j->off[i], j->len[i]);
    EVP_MD_CTX_reset(ctx);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

int cbft_cpu_sign_many(const uint8_t* sk, uint32_t nkeys, const uint32_t* key_idx, const uint8_t* blob,
                       const uint64_t* off, const uint32_t* len, size_t n, uint8_t* sig, int threads) {
  EVP_PKEY** sks = (EVP_PKEY**)calloc(nkeys, sizeof(EVP_PKEY*));
  for (uint32_t i = 0; i < nkeys; i++) sks[i] = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, sk + 32 * i, 32);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  sjob_t* jobs = (sjob_t*)calloc(threads, sizeof(sjob_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (sjob_t){sks, key_idx, blob, off, len, n * t / threads, n * (t + 1) / threads, sig};
    pthread_create(&th[t], NULL, sworker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  for (uint32_t i = 0; i < nkeys; i++) EVP_PKEY_free(sks[i]);
  free(sks);
  free(th);
  free(jobs);
  return 0;
}

/* ---- RSA-2048 PKCS#1 v1.5 / SHA-256 (the verifier SigManager instantiates today,
 * util/src/crypto_utils.cpp:101-117 — Crypto++ there, OpenSSL's RSA here as the host baseline;
 * identical verdicts on modulus-length signatures with s < n). */
#include <openssl/bn.h>
#include <openssl/rsa.h>

typedef struct {
  EVP_PKEY** keys;
  const uint32_t* key_idx;
  const uint8_t* sig;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint8_t* out;
} rjob_t;

static void* rworker(void* arg) {
  rjob_t* j = (rjob_t*)arg;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi; i++) {
    EVP_PKEY* k = j->keys[j->key_idx[i]];
    int ok = 0;
    if (k && EVP_DigestVerifyInit(ctx, NULL, EVP_sha256(), NULL, k) == 1)
      ok = EVP_DigestVerify(ctx, j->sig + 256 * i, 256, j->blob + j->off[i], j->len[i]) == 1;
    j->out[i] = (uint8_t)ok;
    EVP_MD_CTX_reset(ctx);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

/* key cache from nkeys big-endian 256-byte moduli and 32-bit exponents */
void* cbft_cpu_rsa_keys_new(const uint8_t* mod, const uint32_t* exps, uint32_t nkeys) {
  EVP_PKEY** keys = (EVP_PKEY**)calloc(nkeys ? nkeys : 1, sizeof(EVP_PKEY*));
  for (uint32_t i = 0; i < nkeys; i++) {
    RSA* r = RSA_new();
    BIGNUM* n = BN_bin2bn(mod + 256 * (size_t)i, 256, NULL);
    BIGNUM* e = BN_new();
    BN_set_word(e, exps[i]);
    RSA_set0_key(r, n, e, NULL);
    keys[i] = EVP_PKEY_new();
    EVP_PKEY_assign_RSA(keys[i], r);
  }
  return keys;
}

int cbft_cpu_rsa_verify(void* keycache, const uint32_t* key_idx, const uint8_t* sig, const uint8_t* blob,
                        const uint64_t* off, const uint32_t* len, size_t n, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  rjob_t* jobs = (rjob_t*)calloc(threads, sizeof(rjob_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (rjob_t){(EVP_PKEY**)keycache, key_idx, sig, blob, off, len, n * t / threads, n * (t + 1) / threads, out};
    pthread_create(&th[t], NULL, rworker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/*
 * tkv_amq_oracle.c -- CPU ORACLE (test infrastructure only; see tkv_amq_oracle.h).
 *
 * Plain C restatement of the tkv-amq v1 spec.  It is written
 * independently of the HIP product code (turtle_kv_amd/csrc/) on purpose: the VQF
 * here is the literal in-place insert (shift tags / insert a metadata zero, one key at
 * a time, as vqf_insert does), while the GPU uses an equivalent counting-sort
 * formulation.  Agreement between the two is what the parity tests check.
 */
#include "tkv_amq_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------
 * XXH64 (xxHash spec 0.8.x), as called by vqf_hash_val (vqf_filter_page_view.hpp:32-35).
 * ---------------------------------------------------------------------------------- */
#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline void wr64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }

static inline uint64_t xxh_round(uint64_t acc, uint64_t in)
{
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
static inline uint64_t xxh_merge(uint64_t acc, uint64_t v)
{
  acc ^= xxh_round(0, v);
  return acc * P1 + P4;
}

uint64_t tkvo_xxh64(const void* data, size_t len, uint64_t seed)
{
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xxh_round(v1, rd64(p));
      v2 = xxh_round(v2, rd64(p + 8));
      v3 = xxh_round(v3, rd64(p + 16));
      v4 = xxh_round(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge(h, v1);
    h = xxh_merge(h, v2);
    h = xxh_merge(h, v3);
    h = xxh_merge(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xxh_round(0, rd64(p));
    h = rotl64(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl64(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P5;
    h = rotl64(h, 11) * P1;
    ++p;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

/* splitmix64: output n (n >= 1) of the stream seeded with `seed` */
static inline uint64_t sm64_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
uint64_t tkvo_splitmix64_at(uint64_t seed, uint64_t n)
{
  return sm64_mix(seed + n * 0x9E3779B97F4A7C15ULL);
}

void tkvo_gen_keys16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out)
{
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t g = first + i;
    wr64(out + 16 * i, tkvo_splitmix64_at(seed, 2 * g + 1));
    wr64(out + 16 * i + 8, tkvo_splitmix64_at(seed, 2 * g + 2));
  }
}

static int cmp_key16(const void* a, const void* b) { return memcmp(a, b, 16); }

/* ------------------------------------------------------------------------------------
 * generic segment-parallel driver (build_all_pages-style worker pool)
 * ---------------------------------------------------------------------------------- */
typedef struct par_ctx {
  uint32_t n_items;
  uint32_t next;
  void (*fn)(struct par_ctx*, uint32_t);
  void* arg;
  int status;
} par_ctx;

static void* par_worker(void* p)
{
  par_ctx* c = (par_ctx*)p;
  for (;;) {
    uint32_t i = __atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (i >= c->n_items) return NULL;
    c->fn(c, i);
  }
}

static int par_run(uint32_t n_items, int n_threads, void (*fn)(par_ctx*, uint32_t), void* arg)
{
  par_ctx c = {n_items, 0, fn, arg, TKVO_OK};
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  int started = 0;
  for (int t = 1; t < n_threads; ++t) {
    if (pthread_create(&th[t], NULL, par_worker, &c) == 0) started = t;
    else break;
  }
  par_worker(&c);
  for (int t = 1; t <= started; ++t) pthread_join(th[t], NULL);
  return c.status;
}

typedef struct { uint8_t* keys; const uint64_t* seg_begin; } sort_arg;
static void sort_one(par_ctx* c, uint32_t s)
{
  sort_arg* a = (sort_arg*)c->arg;
  uint64_t b = a->seg_begin[s], e = a->seg_begin[s + 1];
  qsort(a->keys + 16 * b, (size_t)(e - b), 16, cmp_key16);
}
void tkvo_sort_keys16_segments(uint8_t* keys, const uint64_t* seg_begin, uint32_t n_segs,
                               int n_threads)
{
  sort_arg a = {keys, seg_begin};
  par_run(n_segs, n_threads, sort_one, &a);
}

static inline void key_at(const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                          uint64_t i, const uint8_t** kp, size_t* kl)
{
  if (offsets) {
    *kp = keys + offsets[i];
    *kl = (size_t)(offsets[i + 1] - offsets[i]);
  } else {
    *kp = keys + (uint64_t)stride * i;
    *kl = stride;
  }
}

/* ------------------------------------------------------------------------------------
 * Bloom, Blocked-512 layout (restates llfs::build_bloom_filter_page(..., kBlocked512,
 * bits_per_key, opt_hash_count=None, src_page_id, ComputeChecksum{false}, buffer) as
 * called at tree/filter_builder.hpp:126-135; sizing consistent with
 * tree/tree_options.hpp:183-191: round_up_bits(9, items * bits_per_key)).
 *
 *   hash_count k   = clamp(floor(bpk * ln 2 + 0.5), 1, 32)
 *   block_count    = max(1, ceil(n * bpk / 512))            (512-bit blocks)
 *   h_i            = XXH64(key, len, seed_i), i = 0..k-1
 *   seed_i         = splitmix64 mix of (0x243F6A8885A308D3 + i * 0x9E3779B97F4A7C15)
 *   block          = (h_0 * block_count) >> 64   (128-bit product, "fast range")
 *   bit_i          = h_i & 511 inside that block; word = bit_i >> 6, LE u64 words
 *
 * payload (PackedBloomFilterPage, 64-byte header, then words[8 * block_count]):
 *   0 magic u64 | 8 bit_count u64 | 16 src_page_id u64 | 24 xxh3_checksum u64 (=0)
 *  32 word_count u64 | 40 block_count u32 | 44 hash_count u16 | 46 layout u8 (=2) |
 *  47 reserved u8 | 48 item_count u64 | 56 reserved u64
 * ---------------------------------------------------------------------------------- */
#define BLOOM_MAGIC 0xca6f49a0f3f8a4b0ULL
#define BLOOM_HEADER 64

uint32_t tkvo_bloom_hash_count(uint32_t bpk)
{
  uint32_t k = (uint32_t)((double)bpk * 0.69314718055994530942 + 0.5);
  if (k < 1) k = 1;
  if (k > 32) k = 32;
  return k;
}

uint64_t tkvo_bloom_seed(uint32_t i)
{
  return sm64_mix(0x243F6A8885A308D3ULL + (uint64_t)i * 0x9E3779B97F4A7C15ULL);
}

uint32_t tkvo_bloom_block_count(uint64_t n, uint32_t bpk)
{
  uint64_t bits = n * (uint64_t)bpk;
  uint64_t blocks = (bits + 511) / 512;
  return blocks == 0 ? 1u : (uint32_t)blocks;
}

uint64_t tkvo_bloom_payload_size(uint64_t n, uint32_t bpk)
{
  return BLOOM_HEADER + 64ull * tkvo_bloom_block_count(n, bpk);
}

int tkvo_bloom_build_payload(const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                             uint64_t n, uint32_t bpk, uint64_t src_page_id, uint8_t* out,
                             uint64_t cap)
{
  if (bpk == 0) return TKVO_OK; /* filter_builder.hpp:115-117 */
  if (bpk > 64) return TKVO_INVALID_ARGUMENT;
  const uint32_t nb = tkvo_bloom_block_count(n, bpk);
  const uint32_t k = tkvo_bloom_hash_count(bpk);
  if (tkvo_bloom_payload_size(n, bpk) > cap) return TKVO_RESOURCE_EXHAUSTED;

  memset(out, 0, BLOOM_HEADER + 64ull * nb);
  wr64(out + 0, BLOOM_MAGIC);
  wr64(out + 8, 512ull * nb);
  wr64(out + 16, src_page_id);
  wr64(out + 24, 0);
  wr64(out + 32, 8ull * nb);
  uint32_t nb32 = nb;
  memcpy(out + 40, &nb32, 4);
  uint16_t k16 = (uint16_t)k;
  memcpy(out + 44, &k16, 2);
  out[46] = 2;
  wr64(out + 48, n);

  uint64_t* words = (uint64_t*)(out + BLOOM_HEADER);
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* kp;
    size_t kl;
    key_at(keys, offsets, stride, i, &kp, &kl);
    const uint64_t h0 = tkvo_xxh64(kp, kl, tkvo_bloom_seed(0));
    const uint64_t blk = (uint64_t)(((u128)h0 * nb) >> 64);
    uint64_t* bw = words + 8 * blk;
    for (uint32_t j = 0; j < k; ++j) {
      const uint64_t h = j == 0 ? h0 : tkvo_xxh64(kp, kl, tkvo_bloom_seed(j));
      const uint32_t bit = (uint32_t)(h & 511);
      bw[bit >> 6] |= 1ull << (bit & 63);
    }
  }
  return TKVO_OK;
}

int tkvo_bloom_query_payload(const uint8_t* payload, const uint8_t* key, size_t len)
{
  if (rd64(payload) != BLOOM_MAGIC) return -1;
  uint32_t nb;
  memcpy(&nb, payload + 40, 4);
  uint16_t k;
  memcpy(&k, payload + 44, 2);
  const uint8_t* words = payload + BLOOM_HEADER;
  const uint64_t h0 = tkvo_xxh64(key, len, tkvo_bloom_seed(0));
  const uint64_t blk = (uint64_t)(((u128)h0 * nb) >> 64);
  for (uint32_t j = 0; j < k; ++j) {
    const uint64_t h = j == 0 ? h0 : tkvo_xxh64(key, len, tkvo_bloom_seed(j));
    const uint32_t bit = (uint32_t)(h & 511);
    const uint64_t w = rd64(words + 64 * blk + 8 * (bit >> 6));
    if (!((w >> (bit & 63)) & 1)) return 0;
  }
  return 1;
}

/* Sampled block windows of the Bloom filter over the n splitmix keys tkvo_gen_keys16(seed,
 * first, n) would produce, without materialising the keys or the filter (the check of a
 * filter too large to build on one host thread in a test's time, e.g. BASELINE config 5's
 * 1B keys): every key is generated and its h0 computed; a key whose block falls in one of
 * the windows [blk0[i], blk1[i]) (ascending, disjoint) has its k bits set there, exactly as
 * tkvo_bloom_build_payload would.  out: the windows' 64-byte blocks concatenated, zeroed by
 * the caller.  Keys are spread over n_threads threads in chunks; bits are ORed atomically.
 * One window [0, block_count) is the whole filter: the multithreaded whole-filter check of
 * BASELINE config 5 (1B keys) against the GPU build. */
typedef struct {
  uint64_t seed, first, n;
  uint32_t nb, k, n_win;
  const uint64_t* blk0;
  const uint64_t* blk1;
  const uint64_t* wbase; /* first word of window i in out */
  uint64_t* words;
} sample_arg;

#define SAMPLE_CHUNK (1u << 20)

static void sample_chunk(par_ctx* c, uint32_t ci)
{
  const sample_arg* a = (const sample_arg*)c->arg;
  const uint64_t b = (uint64_t)ci * SAMPLE_CHUNK;
  const uint64_t e = b + SAMPLE_CHUNK < a->n ? b + SAMPLE_CHUNK : a->n;
  for (uint64_t i = b; i < e; ++i) {
    uint8_t key[16];
    const uint64_t g = a->first + i;
    wr64(key, tkvo_splitmix64_at(a->seed, 2 * g + 1));
    wr64(key + 8, tkvo_splitmix64_at(a->seed, 2 * g + 2));
    const uint64_t h0 = tkvo_xxh64(key, 16, tkvo_bloom_seed(0));
    const uint64_t blk = (uint64_t)(((u128)h0 * a->nb) >> 64);
    /* the last window starting at or before blk (binary search: windows are ascending) */
    uint32_t lo = 0, hi = a->n_win;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (a->blk0[mid] <= blk) lo = mid;
      else hi = mid;
    }
    if (a->n_win == 0 || blk < a->blk0[lo] || blk >= a->blk1[lo]) continue;
    uint64_t* bw = a->words + a->wbase[lo] + 8 * (blk - a->blk0[lo]);
    for (uint32_t j = 0; j < a->k; ++j) {
      const uint64_t h = j == 0 ? h0 : tkvo_xxh64(key, 16, tkvo_bloom_seed(j));
      const uint32_t bit = (uint32_t)(h & 511);
      __atomic_fetch_or(bw + (bit >> 6), 1ull << (bit & 63), __ATOMIC_RELAXED);
    }
  }
}

int tkvo_bloom_sample_blocks_gen16(uint64_t seed, uint64_t first, uint64_t n, uint32_t bpk,
                                   const uint64_t* blk0, const uint64_t* blk1, uint32_t n_win,
                                   uint8_t* out, int n_threads)
{
  if (bpk == 0 || bpk > 64 || n_win > TKVO_SAMPLE_MAX_WINDOWS) return TKVO_INVALID_ARGUMENT;
  uint64_t* wbase = (uint64_t*)malloc(sizeof(uint64_t) * (n_win ? n_win : 1));
  if (!wbase) return TKVO_RESOURCE_EXHAUSTED;
  uint64_t words = 0;
  for (uint32_t w = 0; w < n_win; ++w) {
    if (blk1[w] < blk0[w] || (w && blk0[w] < blk1[w - 1])) {
      free(wbase);
      return TKVO_INVALID_ARGUMENT;
    }
    wbase[w] = words;
    words += 8 * (blk1[w] - blk0[w]);
  }
  sample_arg a = {seed, first, n, tkvo_bloom_block_count(n, bpk), tkvo_bloom_hash_count(bpk),
                  n_win, blk0, blk1, wbase, (uint64_t*)out};
  const int st = par_run((uint32_t)((n + SAMPLE_CHUNK - 1) / SAMPLE_CHUNK), n_threads, sample_chunk, &a);
  free(wbase);
  return st;
}

/* ------------------------------------------------------------------------------------
 * VQF (restates the vqf 0.2.4 operations called at tree/filter_builder.hpp:193-211 and
 * vqf_filter_page_view.hpp:113-125; upstream design: Pandey et al., SIGMOD'21).
 *
 *  TAG_BITS 8 : 64-byte block = md[2] (128 bits) + 48 x u8 tags; 80 buckets;  CHECK_ALT 92
 *  TAG_BITS 16: 64-byte block = md    ( 64 bits) + 28 x u16 tags; 36 buckets; CHECK_ALT 43
 *  md: bucket o ends at the o-th set bit; its tags are the zeros before it.
 *  vqf_metadata (48 B): total_size_in_bytes, key_remainder_bits, range, nblocks, nelts, nslots
 * ---------------------------------------------------------------------------------- */
#define VQF_MAGIC 0x16015305e0f43a7dULL /* vqf_filter_page_view.hpp:66 */
#define VQF_SEED 0x9d0924dc03e79a75ULL  /* vqf_filter_page_view.hpp:26 */
#define VQF_HDR 32                      /* sizeof(PackedVqfFilter) - sizeof(vqf_metadata) */
#define VQF_MD 48                       /* sizeof(vqf_metadata) */
#define VQF_ALT_MUL 0x5bd1e995ULL

static inline uint32_t vqf_slots(int t) { return t == 8 ? 48u : 28u; }
static inline uint32_t vqf_buckets(int t) { return t == 8 ? 80u : 36u; }
static inline uint32_t vqf_check_alt(int t) { return t == 8 ? 92u : 43u; }

/* vqf_filter_page_view.hpp:39-59 */
double tkvo_vqf_load_factor(int tag_bits, uint64_t bpk)
{
  if (bpk == 0) return 0;
  const double b = (double)bpk;
  return tag_bits == 8 ? 10.2 / b : 18.0 / b;
}

uint64_t tkvo_vqf_required_size(int t, uint64_t nslots)
{
  const uint64_t s = vqf_slots(t);
  return VQF_MD + 64ull * ((nslots + s) / s);
}

uint64_t tkvo_vqf_nslots_for_size(int t, uint64_t bytes)
{
  if (bytes < VQF_MD + 64) return 0;
  const uint64_t nb = (bytes - VQF_MD) / 64;
  return nb * vqf_slots(t) - 1;
}

uint64_t tkvo_tree_filter_bits_per_key(uint64_t requested, int use_qf)
{
  /* tree_options.hpp:155-164 */
  if (!use_qf) return requested;
  return requested == 0 ? 0 : (requested < 12 ? 12 : requested);
}

/* build_quotient_filter_for_leaf sizing, filter_builder.hpp:241-290 */
int tkvo_vqf_plan_segment(uint64_t n, uint64_t bpk, uint64_t payload_capacity, tkvo_vqf_plan* o)
{
  memset(o, 0, sizeof(*o));
  if (bpk == 0) return TKVO_OK;                    /* :227-229 */
  if (bpk < 12) return TKVO_INVALID_ARGUMENT;      /* vqf_filter_page_view.hpp:46 CHECK */
  if (payload_capacity < VQF_HDR + VQF_MD + 64) return TKVO_RESOURCE_EXHAUSTED;

  const uint64_t max8 = tkvo_vqf_nslots_for_size(8, payload_capacity - VQF_HDR);
  const uint64_t max16 = tkvo_vqf_nslots_for_size(16, payload_capacity - VQF_HDR);
  const double n_keys = (double)n;
  const double lf8 = tkvo_vqf_load_factor(8, bpk);
  const double lf16 = tkvo_vqf_load_factor(16, bpk);
  const uint64_t n8 = (uint64_t)floor(n_keys / lf8);
  const uint64_t n16 = (uint64_t)floor(n_keys / lf16);
  if (!(lf8 <= 0.85)) return TKVO_INVALID_ARGUMENT; /* :265 CHECK */

  if (lf16 <= 0.85 && n16 <= max16) {
    o->tag_bits = 16;
    o->nslots = n16;
  } else if (n8 <= max8) {
    o->tag_bits = 8;
    o->nslots = n8;
  } else {
    if (!(max8 > max16)) return TKVO_INTERNAL; /* :278 CHECK */
    uint32_t shift = 1;
    while ((double)(n >> shift) / lf8 > (double)max8) ++shift;
    o->tag_bits = 8;
    o->hash_val_shift = shift;
    o->nslots = max8;
  }
  const uint64_t s = vqf_slots((int)o->tag_bits);
  o->nblocks = (o->nslots + s) / s;
  o->filter_size = tkvo_vqf_required_size((int)o->tag_bits, o->nslots);
  o->payload_used = VQF_HDR + o->filter_size;
  return TKVO_OK;
}

typedef struct vqf_view {
  int t;
  uint64_t nblocks;
  uint8_t* blocks;
} vqf_view;

static inline u128 md_get(const vqf_view* v, uint64_t b)
{
  const uint8_t* p = v->blocks + 64 * b;
  if (v->t == 8) return (u128)rd64(p) | ((u128)rd64(p + 8) << 64);
  return (u128)rd64(p);
}
static inline void md_put(vqf_view* v, uint64_t b, u128 md)
{
  uint8_t* p = v->blocks + 64 * b;
  wr64(p, (uint64_t)md);
  if (v->t == 8) wr64(p + 8, (uint64_t)(md >> 64));
}
static inline int popc128(u128 x)
{
  return __builtin_popcountll((uint64_t)x) + __builtin_popcountll((uint64_t)(x >> 64));
}
static inline int select128(u128 x, int r) /* position of the r-th (0-based) set bit */
{
  for (int i = 0; i < 128; ++i)
    if ((x >> i) & 1) {
      if (r == 0) return i;
      --r;
    }
  return -1;
}

static void vqf_locate(int t, uint64_t nblocks, uint64_t hash, uint64_t* prim, uint64_t* alt,
                       uint64_t* tag)
{
  const uint64_t R = nblocks * vqf_buckets(t); /* range >> TAG_BITS */
  const uint64_t tg = hash & ((1ull << t) - 1);
  *tag = tg;
  *prim = (hash >> t) % R;
  *alt = ((hash ^ (tg * VQF_ALT_MUL)) >> t) % R;
}

/* vqf_insert: returns 1 on success, 0 if the chosen block is full */
static int vqf_insert(vqf_view* v, uint64_t hash)
{
  const int t = v->t;
  const uint32_t B = vqf_buckets(t), S = vqf_slots(t);
  uint64_t pi, ai, tag;
  vqf_locate(t, v->nblocks, hash, &pi, &ai, &tag);
  uint64_t use = pi;
  const uint64_t pb = pi / B, ab = ai / B;
  const int pop_p = popc128(md_get(v, pb));
  if (pop_p < (int)vqf_check_alt(t) && pb != ab) {
    const int pop_a = popc128(md_get(v, ab));
    if (pop_a > pop_p) use = ai;
  }
  const uint64_t blk = use / B;
  const int o = (int)(use % B);
  u128 md = md_get(v, blk);
  if (popc128(md) == (int)B) return 0; /* block full */
  const int s = select128(md, o);
  const int p = s - o;
  uint8_t* tags = v->blocks + 64 * blk + (t == 8 ? 16 : 8);
  const int tb = t / 8;
  memmove(tags + tb * (p + 1), tags + tb * p, (size_t)tb * (S - 1 - p));
  if (t == 8) {
    tags[p] = (uint8_t)tag;
  } else {
    uint16_t t16 = (uint16_t)tag;
    memcpy(tags + 2 * p, &t16, 2);
  }
  const u128 low = (((u128)1) << s) - 1;
  u128 nmd = (md & low) | ((md & ~low) << 1);
  if (t == 16) nmd &= (u128)~0ull;
  md_put(v, blk, nmd);
  return 1;
}

static int vqf_bucket_has(const vqf_view* v, uint64_t idx, uint64_t tag)
{
  const int t = v->t;
  const uint32_t B = vqf_buckets(t);
  const uint64_t blk = idx / B;
  const int o = (int)(idx % B);
  const u128 md = md_get(v, blk);
  const int start = o == 0 ? 0 : select128(md, o - 1) - (o - 1);
  const int end = select128(md, o) - o;
  const uint8_t* tags = v->blocks + 64 * blk + (t == 8 ? 16 : 8);
  for (int i = start; i < end; ++i) {
    uint64_t tv;
    if (t == 8) {
      tv = tags[i];
    } else {
      uint16_t t16;
      memcpy(&t16, tags + 2 * i, 2);
      tv = t16;
    }
    if (tv == tag) return 1;
  }
  return 0;
}

int tkvo_vqf_build_payload(const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                           uint64_t n, uint64_t bpk, uint64_t src_page_id, uint8_t* out,
                           uint64_t cap, tkvo_vqf_plan* plan_out)
{
  tkvo_vqf_plan pl;
  int st = tkvo_vqf_plan_segment(n, bpk, cap, &pl);
  if (plan_out) *plan_out = pl;
  if (st != TKVO_OK || pl.tag_bits == 0) return st;

  const int t = (int)pl.tag_bits;
  const uint64_t mask = ~0ull << pl.hash_val_shift; /* filter_builder.hpp:187 */
  /* PackedVqfFilter::initialize (vqf_filter_page_view.hpp:87-94) */
  memset(out, 0, pl.payload_used);
  wr64(out + 0, VQF_MAGIC);
  wr64(out + 8, src_page_id);
  wr64(out + 16, VQF_SEED);
  wr64(out + 24, mask);
  /* vqf_init_in_place(filter, nslots) */
  const uint64_t nb = pl.nblocks;
  uint8_t* md = out + VQF_HDR;
  wr64(md + 0, 64ull * nb);
  wr64(md + 8, (uint64_t)t);
  wr64(md + 16, nb * vqf_buckets(t) * (1ull << t));
  wr64(md + 24, nb);
  wr64(md + 32, 0);
  wr64(md + 40, nb * vqf_slots(t));
  vqf_view v = {t, nb, out + VQF_HDR + VQF_MD};
  for (uint64_t b = 0; b < nb; ++b) {
    u128 init = ~(u128)0;
    if (t == 8) init &= ~(((u128)1) << 127);
    else init = (u128)(~0ull & ~(1ull << 63));
    md_put(&v, b, init);
  }
  /* insert loop, filter_builder.hpp:204-214 */
  uint64_t nelts = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* kp;
    size_t kl;
    key_at(keys, offsets, stride, i, &kp, &kl);
    const uint64_t h = tkvo_xxh64(kp, kl, VQF_SEED);
    if ((h & mask) == h) {
      if (!vqf_insert(&v, h)) return TKVO_INTERNAL; /* BATT_CHECK(vqf_insert) :211 */
      ++nelts;
    }
  }
  wr64(md + 32, nelts);
  return TKVO_OK;
}

/* PackedVqfFilter::is_present, vqf_filter_page_view.hpp:113-125 */
int tkvo_vqf_is_present_payload(const uint8_t* payload, uint64_t hash)
{
  if (rd64(payload) != VQF_MAGIC) return -1;
  const uint64_t mask = rd64(payload + 24);
  if ((hash & mask) != hash) return 1;
  const int t = (int)rd64(payload + VQF_HDR + 8);
  if (t != 8 && t != 16) return -1;
  vqf_view v = {t, rd64(payload + VQF_HDR + 24), (uint8_t*)payload + VQF_HDR + VQF_MD};
  uint64_t pi, ai, tag;
  vqf_locate(t, v.nblocks, hash, &pi, &ai, &tag);
  return vqf_bucket_has(&v, pi, tag) || vqf_bucket_has(&v, ai, tag);
}

/* ------------------------------------------------------------------------------------
 * batched build / probe
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int kind;
  const uint8_t* keys;
  const uint64_t* offsets; /* variable-length keys (key i = keys[offsets[i], offsets[i+1])) */
  uint32_t stride;         /* fixed-size keys (offsets == NULL) */
  const uint64_t* seg_begin;
  uint32_t bpk;
  const uint64_t* src;
  uint8_t* out;
  const uint64_t* off;
  const uint64_t* cap;
} build_arg;

static void build_one(par_ctx* c, uint32_t s)
{
  build_arg* a = (build_arg*)c->arg;
  const uint64_t b = a->seg_begin[s], e = a->seg_begin[s + 1];
  const uint64_t src = a->src ? a->src[s] : s;
  /* leaf s's keys: a pointer at its first key (fixed size), or its offsets (variable) */
  const uint8_t* k = a->offsets ? a->keys : a->keys + (uint64_t)a->stride * b;
  const uint64_t* o = a->offsets ? a->offsets + b : NULL;
  int st;
  if (a->kind == 0)
    st = tkvo_bloom_build_payload(k, o, a->stride, e - b, a->bpk, src, a->out + a->off[s], a->cap[s]);
  else
    st = tkvo_vqf_build_payload(k, o, a->stride, e - b, a->bpk, src, a->out + a->off[s], a->cap[s], NULL);
  if (st != TKVO_OK) __atomic_store_n(&c->status, st, __ATOMIC_RELAXED);
}

int tkvo_build_segments(int kind, const uint8_t* keys16, const uint64_t* seg_begin,
                        uint32_t n_segs, uint32_t bpk, const uint64_t* src_page_id,
                        uint8_t* out, const uint64_t* out_offset, const uint64_t* out_capacity,
                        int n_threads)
{
  return tkvo_build_segments_ex(kind, keys16, NULL, 16, seg_begin, n_segs, bpk, src_page_id, out,
                                out_offset, out_capacity, n_threads);
}

int tkvo_build_segments_ex(int kind, const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                           const uint64_t* seg_begin, uint32_t n_segs, uint32_t bpk,
                           const uint64_t* src_page_id, uint8_t* out, const uint64_t* out_offset,
                           const uint64_t* out_capacity, int n_threads)
{
  build_arg a = {kind, keys, offsets, stride, seg_begin, bpk, src_page_id, out, out_offset, out_capacity};
  return par_run(n_segs, n_threads, build_one, &a);
}

typedef struct {
  int kind;
  const uint8_t* filters;
  const uint64_t* off;
  const uint8_t* q;
  const uint32_t* qs;
  uint64_t n;
  uint8_t* res;
} probe_arg;

#define PROBE_CHUNK 65536
static void probe_chunk(par_ctx* c, uint32_t ci)
{
  probe_arg* a = (probe_arg*)c->arg;
  const uint64_t b = (uint64_t)ci * PROBE_CHUNK;
  uint64_t e = b + PROBE_CHUNK;
  if (e > a->n) e = a->n;
  for (uint64_t i = b; i < e; ++i) {
    const uint8_t* f = a->filters + a->off[a->qs[i]];
    int r;
    if (a->kind == 0) r = tkvo_bloom_query_payload(f, a->q + 16 * i, 16);
    else r = tkvo_vqf_is_present_payload(f, tkvo_xxh64(a->q + 16 * i, 16, VQF_SEED));
    if (r < 0) {
      __atomic_store_n(&c->status, TKVO_INTERNAL, __ATOMIC_RELAXED);
      r = 1;
    }
    a->res[i] = (uint8_t)r;
  }
}

int tkvo_probe_segments(int kind, const uint8_t* filters, const uint64_t* out_offset,
                        const uint8_t* queries16, const uint32_t* query_seg, uint64_t n,
                        uint8_t* result, int n_threads)
{
  probe_arg a = {kind, filters, out_offset, queries16, query_seg, n, result};
  return par_run((uint32_t)((n + PROBE_CHUNK - 1) / PROBE_CHUNK), n_threads, probe_chunk, &a);
}

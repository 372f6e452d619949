/*
 * tkv_amq_baseline.c -- CPU BASELINE for the VQF build (test infrastructure only: timed by
 * bench.py's cpu_baseline leg, never shipped, never part of the product path).
 *
 * The literal oracle (tkv_amq_oracle.c) inserts one key at a time the way the tkv-amq v1
 * spec reads: a bit-by-bit select over the block metadata and a generic XXH64.  The reference
 * compiles vqf 0.2.4 with -mbmi2 -mavx2 (CMakeLists.txt:46-48), i.e. select by pdep/tzcnt,
 * so timing the literal oracle would overstate the GPU's edge.  This is the same insert
 * (tree/filter_builder.hpp:204-214 -> vqf_insert) written the way an optimised CPU build
 * runs it:
 *   - XXH64 of a 16-byte key unrolled (two lane steps and the avalanche; vqf_hash_val,
 *     vqf_filter_page_view.hpp:32-35);
 *   - the bucket index by a multiply-high with the precomputed floor((2^64-1)/R) and one
 *     fix-up step instead of a 64-bit division (the same remainder);
 *   - select of the o-th set metadata bit by _pdep_u64 + _tzcnt_u64 on each 64-bit half;
 *   - popcounts by the POPCNT instruction, the tag shift by memmove.
 * Its output is byte-identical to the oracle's (tests/test_oracle.py::test_vqf_bmi2_baseline).
 */
#include "tkv_amq_oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <string.h>

typedef unsigned __int128 u128;

#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL
#define VQF_MAGIC 0x16015305e0f43a7dULL
#define VQF_SEED 0x9d0924dc03e79a75ULL
#define VQF_HDR 32
#define VQF_MD 48
#define VQF_ALT_MUL 0x5bd1e995ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void wr64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }

static inline uint64_t xxh64_16(const uint8_t* p, uint64_t seed)
{
  uint64_t h = seed + P5 + 16;
  uint64_t k = rd64(p) * P2;
  h ^= rotl64(k, 31) * P1;
  h = rotl64(h, 27) * P1 + P4;
  k = rd64(p + 8) * P2;
  h ^= rotl64(k, 31) * P1;
  h = rotl64(h, 27) * P1 + P4;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

/* x % R from q = floor(x * magic / 2^64), magic = floor((2^64-1) / R): q is x/R or one less */
static inline uint64_t mod_fast(uint64_t x, uint64_t R, uint64_t magic)
{
  const uint64_t q = (uint64_t)(((u128)x * magic) >> 64);
  uint64_t r = x - q * R;
  if (r >= R) r -= R;
  return r;
}

static inline int select64(uint64_t x, int r) { return (int)_tzcnt_u64(_pdep_u64(1ull << r, x)); }

/* one insert into a block array of 8- or 16-bit tags; 1 on success, 0 if the block is full */
static inline int insert(int t, uint8_t* blocks, uint64_t R, uint64_t magic, uint64_t h)
{
  const uint32_t B = t == 8 ? 80u : 36u, S = t == 8 ? 48u : 28u, CHECK_ALT = t == 8 ? 92u : 43u;
  const uint64_t tag = h & ((1ull << t) - 1);
  const uint64_t pi = mod_fast(h >> t, R, magic);
  const uint64_t ai = mod_fast((h ^ (tag * VQF_ALT_MUL)) >> t, R, magic);
  const uint64_t pb = pi / B, ab = ai / B;
  const uint8_t* mp = blocks + 64 * pb;
  const int pop_p = t == 8 ? _mm_popcnt_u64(rd64(mp)) + _mm_popcnt_u64(rd64(mp + 8))
                           : (int)_mm_popcnt_u64(rd64(mp));
  uint64_t use = pi;
  if (pop_p < (int)CHECK_ALT && pb != ab) {
    const uint8_t* ma = blocks + 64 * ab;
    const int pop_a = t == 8 ? _mm_popcnt_u64(rd64(ma)) + _mm_popcnt_u64(rd64(ma + 8))
                             : (int)_mm_popcnt_u64(rd64(ma));
    if (pop_a > pop_p) use = ai;
  }
  const uint64_t blk = use / B;
  const int o = (int)(use - blk * B);
  uint8_t* bp = blocks + 64 * blk;
  if (t == 8) {
    const uint64_t lo = rd64(bp), hi = rd64(bp + 8);
    const int pl = (int)_mm_popcnt_u64(lo);
    if (pl + (int)_mm_popcnt_u64(hi) == (int)B) return 0;
    const int s = o < pl ? select64(lo, o) : 64 + select64(hi, o - pl);
    const int p = s - o;
    uint8_t* tags = bp + 16;
    memmove(tags + p + 1, tags + p, (size_t)(S - 1 - p));
    tags[p] = (uint8_t)tag;
    /* insert a 0 at bit s of the 128-bit metadata */
    const u128 md = (u128)lo | ((u128)hi << 64);
    const u128 low = (((u128)1) << s) - 1;
    const u128 nmd = (md & low) | ((md & ~low) << 1);
    wr64(bp, (uint64_t)nmd);
    wr64(bp + 8, (uint64_t)(nmd >> 64));
  } else {
    const uint64_t md = rd64(bp);
    if ((int)_mm_popcnt_u64(md) == (int)B) return 0;
    const int s = select64(md, o);
    const int p = s - o;
    uint8_t* tags = bp + 8;
    memmove(tags + 2 * (p + 1), tags + 2 * p, (size_t)2 * (S - 1 - p));
    const uint16_t t16 = (uint16_t)tag;
    memcpy(tags + 2 * p, &t16, 2);
    const uint64_t low = (1ull << s) - 1;
    wr64(bp, (md & low) | ((md & ~low) << 1));
  }
  return 1;
}

/* The same payload tkvo_vqf_build_payload writes, for n 16-byte keys (leaf order). */
int tkvb_vqf_build_payload16(const uint8_t* keys, uint64_t n, uint64_t bpk, uint64_t src_page_id,
                             uint8_t* out, uint64_t cap)
{
  tkvo_vqf_plan pl;
  const int st = tkvo_vqf_plan_segment(n, bpk, cap, &pl);
  if (st != TKVO_OK || pl.tag_bits == 0) return st;
  const int t = (int)pl.tag_bits;
  const uint32_t B = t == 8 ? 80u : 36u, S = t == 8 ? 48u : 28u;
  const uint64_t mask = ~0ull << pl.hash_val_shift; /* filter_builder.hpp:187 */
  memset(out, 0, pl.payload_used);
  wr64(out + 0, VQF_MAGIC); /* PackedVqfFilter::initialize, vqf_filter_page_view.hpp:87-94 */
  wr64(out + 8, src_page_id);
  wr64(out + 16, VQF_SEED);
  wr64(out + 24, mask);
  const uint64_t nb = pl.nblocks;
  uint8_t* md = out + VQF_HDR;
  wr64(md + 0, 64ull * nb);
  wr64(md + 8, (uint64_t)t);
  wr64(md + 16, nb * B * (1ull << t));
  wr64(md + 24, nb);
  wr64(md + 40, nb * S);
  uint8_t* blocks = out + VQF_HDR + VQF_MD;
  for (uint64_t b = 0; b < nb; ++b) {
    if (t == 8) {
      wr64(blocks + 64 * b, ~0ull);
      wr64(blocks + 64 * b + 8, ~0ull >> 1);
    } else {
      wr64(blocks + 64 * b, ~0ull >> 1);
    }
  }
  const uint64_t R = nb * B, magic = ~0ull / R;
  uint64_t nelts = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t h = xxh64_16(keys + 16 * i, VQF_SEED);
    if ((h & mask) == h) {
      if (!insert(t, blocks, R, magic, h)) return TKVO_INTERNAL; /* BATT_CHECK :211 */
      ++nelts;
    }
  }
  wr64(md + 32, nelts);
  return TKVO_OK;
}

/* leaves spread over n_threads threads, one leaf per thread at a time (build_all_pages) */
typedef struct {
  const uint8_t* keys;
  const uint64_t* seg_begin;
  uint32_t n_segs;
  uint64_t bpk;
  const uint64_t* src;
  uint8_t* out;
  const uint64_t* off;
  const uint64_t* cap;
  uint32_t next;
  int status;
} seg_arg;

static void* seg_worker(void* p)
{
  seg_arg* a = (seg_arg*)p;
  for (;;) {
    const uint32_t s = __atomic_fetch_add(&a->next, 1, __ATOMIC_RELAXED);
    if (s >= a->n_segs) return NULL;
    const uint64_t b = a->seg_begin[s], e = a->seg_begin[s + 1];
    const int st = tkvb_vqf_build_payload16(a->keys + 16 * b, e - b, a->bpk, a->src ? a->src[s] : s,
                                            a->out + a->off[s], a->cap[s]);
    if (st != TKVO_OK) __atomic_store_n(&a->status, st, __ATOMIC_RELAXED);
  }
}

int tkvb_vqf_build_segments(const uint8_t* keys16, const uint64_t* seg_begin, uint32_t n_segs,
                            uint32_t bpk, const uint64_t* src_page_id, uint8_t* out,
                            const uint64_t* out_offset, const uint64_t* out_capacity, int n_threads)
{
  seg_arg a = {keys16, seg_begin, n_segs, bpk, src_page_id, out, out_offset, out_capacity, 0, TKVO_OK};
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  int started = 0;
  for (int i = 1; i < n_threads; ++i) {
    if (pthread_create(&th[i], NULL, seg_worker, &a) == 0) started = i;
    else break;
  }
  seg_worker(&a);
  for (int i = 1; i <= started; ++i) pthread_join(th[i], NULL);
  return a.status;
}

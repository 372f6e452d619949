/*
 * tkv_amq_oracle.h -- CPU ORACLE for the tkv-amq v1 filter spec.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (libtkv_amq.so) never links or calls it.
 *
 * This is a plain-C restatement of TurtleKV's per-leaf AMQ filter path:
 *   - vqf_hash_val                      src/turtle_kv/vqf_filter_page_view.hpp:32-35
 *   - vqf_filter_load_factor<T>         src/turtle_kv/vqf_filter_page_view.hpp:39-59
 *   - PackedVqfFilter (header, mask)    src/turtle_kv/vqf_filter_page_view.hpp:63-126
 *   - build_bloom_filter_for_leaf       src/turtle_kv/tree/filter_builder.hpp:109-152
 *   - build_vqf_filter<TAG_BITS>        src/turtle_kv/tree/filter_builder.hpp:176-217
 *   - build_quotient_filter_for_leaf    src/turtle_kv/tree/filter_builder.hpp:221-301
 *   - TreeOptions::filter_bits_per_key  src/turtle_kv/tree/tree_options.hpp:155-164
 *   - KeyQuery::reject_page             src/turtle_kv/tree/key_query.hpp:149-247
 *
 * PARITY STATUS.  The filter arithmetic itself lives in two third-party packages that
 * are NOT present in /root/reference: llfs 0.42.1-devel (Bloom, conanfile.py:60) and
 * vqf 0.2.4 (conanfile.py:62).  No reference test pins filter bytes.  The Bloom
 * Blocked-512 bit layout and the VQF block layout below are therefore a frozen
 * restatement of the published designs ("tkv-amq v1"):
 *   XXH64 is pinned against python-xxhash 3.8.1 / libxxhash 0.8.2 (tests/golden);
 *   the turtle_kv sizing/selection arithmetic is pinned line-by-line to the files above;
 *   the Bloom/VQF bit layouts are PARITY UNPINNED against llfs/vqf (self-pinned by
 *   tests/golden SHA-256 fixtures produced from this file).
 */
#ifndef TKV_AMQ_ORACLE_H
#define TKV_AMQ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: same numbering as include/tkv_amq.h (batt/absl StatusCode values) */
#define TKVO_OK 0
#define TKVO_INVALID_ARGUMENT 3
#define TKVO_RESOURCE_EXHAUSTED 8
#define TKVO_INTERNAL 13

uint64_t tkvo_xxh64(const void* data, size_t len, uint64_t seed);
uint64_t tkvo_splitmix64_at(uint64_t seed, uint64_t n);
/* fill n 16-byte keys: key i = (splitmix64_at(seed, 2(first+i)+1), splitmix64_at(seed, 2(first+i)+2)) LE */
void tkvo_gen_keys16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out);
/* sort each segment's 16-byte keys by memcmp order (leaf key order) */
void tkvo_sort_keys16_segments(uint8_t* keys, const uint64_t* seg_begin, uint32_t n_segs,
                               int n_threads);

/* ---------------- Bloom (Blocked-512) ---------------- */
uint32_t tkvo_bloom_hash_count(uint32_t bits_per_key);
uint64_t tkvo_bloom_seed(uint32_t i);
uint32_t tkvo_bloom_block_count(uint64_t n_items, uint32_t bits_per_key);
uint64_t tkvo_bloom_payload_size(uint64_t n_items, uint32_t bits_per_key);
/* keys: fixed stride when offsets == NULL, else offsets[n+1] byte offsets */
int tkvo_bloom_build_payload(const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                             uint64_t n, uint32_t bits_per_key, uint64_t src_page_id,
                             uint8_t* out_payload, uint64_t out_capacity);
int tkvo_bloom_query_payload(const uint8_t* payload, const uint8_t* key, size_t len);
/* the blocks of sampled windows [blk0[i], blk1[i]) of the filter over tkvo_gen_keys16(seed,
 * first, n), keys generated and hashed on the fly (no key array); ascending, disjoint, at most
 * TKVO_SAMPLE_MAX_WINDOWS; one window [0, block_count) is the whole filter */
#define TKVO_SAMPLE_MAX_WINDOWS 65536
int tkvo_bloom_sample_blocks_gen16(uint64_t seed, uint64_t first, uint64_t n, uint32_t bpk,
                                   const uint64_t* blk0, const uint64_t* blk1, uint32_t n_win,
                                   uint8_t* out, int n_threads);

/* ---------------- VQF ---------------- */
typedef struct tkvo_vqf_plan {
  uint32_t tag_bits;       /* 8 or 16; 0 => no filter (bpk == 0) */
  uint32_t hash_val_shift; /* filter_builder.hpp:280-283 */
  uint64_t nslots;         /* argument to vqf_init_in_place */
  uint64_t nblocks;
  uint64_t filter_size;    /* vqf_required_size<T>(nslots) */
  uint64_t payload_used;   /* 32 + filter_size */
} tkvo_vqf_plan;

double tkvo_vqf_load_factor(int tag_bits, uint64_t bits_per_key);
uint64_t tkvo_vqf_required_size(int tag_bits, uint64_t nslots);
uint64_t tkvo_vqf_nslots_for_size(int tag_bits, uint64_t bytes);
int tkvo_vqf_plan_segment(uint64_t n_items, uint64_t bits_per_key, uint64_t payload_capacity,
                          tkvo_vqf_plan* out);
int tkvo_vqf_build_payload(const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                           uint64_t n, uint64_t bits_per_key, uint64_t src_page_id,
                           uint8_t* out_payload, uint64_t payload_capacity,
                           tkvo_vqf_plan* plan_out);
int tkvo_vqf_is_present_payload(const uint8_t* payload, uint64_t hash_val);

/* TreeOptions::filter_bits_per_key() clamp (tree_options.hpp:155-164) */
uint64_t tkvo_tree_filter_bits_per_key(uint64_t requested, int use_quotient_filter);

/* ---------------- batched (checkpoint-level) CPU build ----------------
 * One filter per segment, single-threaded per filter (WorkerPool::null_pool(),
 * filter_builder.hpp:127); segments spread over n_threads as build_all_pages does
 * (tree_serialize_context.cpp:65-75).  kind: 0 = Bloom, 1 = VQF.
 * Segment s covers keys [seg_begin[s], seg_begin[s+1]); its payload is written at
 * out + out_offset[s] with capacity out_capacity[s].  src_page_id[s] may be NULL (=> s). */
int tkvo_build_segments(int kind, const uint8_t* keys16, const uint64_t* seg_begin,
                        uint32_t n_segs, uint32_t bits_per_key, const uint64_t* src_page_id,
                        uint8_t* out, const uint64_t* out_offset, const uint64_t* out_capacity,
                        int n_threads);
/* the same over keys of any fixed size (offsets NULL, `stride` bytes each) or variable-length
 * keys (key i = keys[offsets[i], offsets[i+1]), offsets indexed by global key) */
int tkvo_build_segments_ex(int kind, const uint8_t* keys, const uint64_t* offsets, uint32_t stride,
                           const uint64_t* seg_begin, uint32_t n_segs, uint32_t bpk,
                           const uint64_t* src_page_id, uint8_t* out, const uint64_t* out_offset,
                           const uint64_t* out_capacity, int n_threads);

/* batched probe: query i probes segment query_seg[i]; result[i] = 1 maybe-present, 0 absent */
int tkvo_probe_segments(int kind, const uint8_t* filters, const uint64_t* out_offset,
                        const uint8_t* queries16, const uint32_t* query_seg, uint64_t n_queries,
                        uint8_t* result, int n_threads);

/* tkv_amq_baseline.c: the VQF build as an optimised CPU build runs it (BMI2 pdep/tzcnt select,
 * POPCNT, unrolled 16-byte XXH64, multiply-high remainder) -- the cpu_baseline bench.py times;
 * byte-identical to tkvo_vqf_build_payload for 16-byte keys */
int tkvb_vqf_build_payload16(const uint8_t* keys, uint64_t n, uint64_t bpk, uint64_t src_page_id,
                             uint8_t* out, uint64_t cap);
int tkvb_vqf_build_segments(const uint8_t* keys16, const uint64_t* seg_begin, uint32_t n_segs,
                            uint32_t bpk, const uint64_t* src_page_id, uint8_t* out,
                            const uint64_t* out_offset, const uint64_t* out_capacity, int n_threads);

#ifdef __cplusplus
}
#endif
#endif

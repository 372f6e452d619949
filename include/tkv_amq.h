/*
 * tkv_amq.h -- C ABI of the MI355X-native AMQ filter engine for TurtleKV (libtkv_amq.so).
 *
 * This is the drop-in boundary for TurtleKV's per-leaf filter build/probe path.  Each
 * entry point names the reference interface it replaces (paths relative to the
 * mathworks/turtle_kv source tree):
 *
 *   tkv_amq_plan            build_{bloom,quotient}_filter_for_leaf sizing
 *                           (src/turtle_kv/tree/filter_builder.hpp:121-135, 241-290) and
 *                           TreeOptions::filter_bits_per_key (tree/tree_options.hpp:155-164)
 *   tkv_amq_build           build_filter_for_leaf_in_job (tree/filter_builder.hpp:307-331),
 *                           batched over every leaf of one TreeSerializeContext::build_all_pages
 *                           queue (tree/tree_serialize_context.cpp:62-115); per leaf it does what
 *                           build_bloom_filter_for_leaf (:109-152) or build_vqf_filter<T> (:176-217)
 *                           writes into the filter page payload
 *   tkv_amq_probe           KeyQuery::reject_page filter test (tree/key_query.hpp:149-247):
 *                           PackedBloomFilter::query (:216-219) / PackedVqfFilter::is_present
 *                           (vqf_filter_page_view.hpp:113-125); result 0 == "reject" (kTrue)
 *   tkv_amq_vqf_hash        vqf_hash_val (vqf_filter_page_view.hpp:32-35), hash-once per query
 *                           (tree/key_query.hpp:82)
 *   tkv_amq_vqf_probe_hashed PackedVqfFilter::is_present(hash_val) for pre-hashed queries
 *   tkv_amq_bloom_hash /    BloomFilterQuery<KeyView> hash cache (tree/key_query.hpp:78,97)
 *   tkv_amq_bloom_probe_hashed   and PackedBloomFilter::query on it (:219)
 *   tkv_amq_vqf_*sizing     vqf_filter_load_factor<T> (vqf_filter_page_view.hpp:39-59),
 *                           vqf_required_size<T> / vqf_nslots_for_size (vqf 0.2.4, used at
 *                           tree/filter_builder.hpp:243-244,270,274)
 *   tkv_amq_filter_page_size_log2, tkv_amq_expected_items_per_leaf, tkv_amq_leaf_data_size
 *                           TreeOptions::filter_page_size_log2 / expected_items_per_leaf /
 *                           leaf_data_size (tree/tree_options.hpp:177-258, tree_options.cpp:57-60,
 *                           tree/packed_leaf_page.hpp:307-311, core/packed_sizeof_edit.hpp:13-15)
 *   tkv_amq_bloom_route / tkv_amq_bloom_build_range (and their _records forms)
 *   tkv_amq_bloom_route_plan / _route_blocks / _build_part_blocks (the pipelined form)
 *                           one monolithic Bloom filter sharded by hash range over GPUs
 *                           (BASELINE config 5; the llfs build_bloom_filter_page it replaces is
 *                           called at tree/filter_builder.hpp:126-135)
 *   tkv_amq_plan_pages      FilterPageAlloc + the page header fields the builders set:
 *                           layout_id (filter_builder.hpp:237), unused_begin / unused_end
 *                           (:293-296), in one page-sized slot per leaf
 *   tkv_amq_probe_ex / tkv_amq_*_probe_hashed_ex
 *                           the same probes with KeyQuery::reject_page's page-id check
 *                           (tree/key_query.hpp:205-212,227-232) and KeyQuery::Metrics counters
 *                           (:36-60, updated at :154,157,210,231,243 and key_query.cpp:41,77)
 *   tkv_amq_stage_keys      the EditView key range build_filter_for_leaf_in_job iterates
 *                           (core/merge_compactor.hpp:107-139) gathered into one contiguous
 *                           host key buffer for the H2D copy (host only)
 *
 * Conventions
 *  - Plain pointers and sizes only.  Pointers documented "device" are HIP device pointers
 *    (hipMalloc / framework-owned HBM); `stream` is a hipStream_t passed as void* (NULL =
 *    the default stream).  Launch functions never allocate, copy synchronously or
 *    synchronise, so they can be captured into a hipGraph.
 *  - The caller owns every buffer (the reference writes into a PageCache page buffer it
 *    does not own, tree/filter_builder.hpp:76-84,189-193).
 *  - Return values are status codes numbered like batt::StatusCode / absl::StatusCode.
 *    On error the output is undefined and must not be committed (reference: a failed build
 *    leaves the leaf without a filter, tree/filter_builder.hpp:323-325).
 *  - Thread-safe: no global mutable state; concurrent calls on different streams are fine.
 *  - Filter bit layouts follow the frozen "tkv-amq v1" spec.
 */
#ifndef TKV_AMQ_H
#define TKV_AMQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TKV_AMQ_ABI_VERSION 2

/* status codes (batt::StatusCode values) */
#define TKV_AMQ_OK 0
#define TKV_AMQ_INVALID_ARGUMENT 3
#define TKV_AMQ_RESOURCE_EXHAUSTED 8
#define TKV_AMQ_INTERNAL 13
#define TKV_AMQ_UNAVAILABLE 14

/* filter kinds (config.hpp:20-24 compile-time switch, made a runtime argument) */
#define TKV_AMQ_BLOOM 0
#define TKV_AMQ_VQF 1

/* One leaf's filter ("segment"), produced on the host by tkv_amq_plan and read by the
 * device kernels.  64 bytes, little-endian, no padding.  The first 32 bytes are what a
 * probe needs (two 16-byte loads). */
typedef struct tkv_amq_segment {
  uint64_t out_offset;    /* byte offset of the filter page payload in the output array */
  uint32_t n_blocks;      /* Bloom: 512-bit blocks; VQF: 64-byte vqf blocks */
  uint16_t hash_count;    /* Bloom k; VQF 0 */
  uint8_t tag_bits;       /* VQF 8 | 16; Bloom 0 */
  uint8_t hash_val_shift; /* VQF hash truncation (filter_builder.hpp:280-283) */
  uint64_t mod_magic;     /* VQF: floor((2^64-1) / (n_blocks * buckets_per_block)); Bloom: 0 */
  uint64_t key_begin;     /* first key index of this leaf's (sorted) item range */
  uint64_t src_page_id;   /* leaf PageId stored in the filter header (reject_page check) */
  uint64_t block_base;    /* prefix sum of n_blocks (VQF workspace addressing) */
  uint32_t n_keys;        /* items in the leaf (tombstones included) */
  uint32_t payload_bytes; /* bytes of payload the build writes (header + filter) */
  uint32_t bits_per_key;  /* effective bits/key after the TreeOptions clamp */
  uint32_t page_flags;    /* TKV_AMQ_PAGE_IMAGE | page_size_log2 << 8 (tkv_amq_plan_pages); 0 */
} tkv_amq_segment;

/* page_flags bit: the build also writes the 64-byte llfs PackedPageHeader fields the filter
 * builders set, at out_offset - 64 (the page starts there) */
#define TKV_AMQ_PAGE_IMAGE 0x1u

const char* tkv_amq_version(void);
const char* tkv_amq_status_string(int status);
/* number of visible HIP devices; 0 => every device entry point returns TKV_AMQ_UNAVAILABLE */
int tkv_amq_device_count(void);

/* TreeOptions::filter_bits_per_key(): VQF clamps any nonzero bpk to >= 12 */
uint64_t tkv_amq_filter_bits_per_key(int kind, uint64_t requested_bits_per_key);

double tkv_amq_vqf_load_factor(int tag_bits, uint64_t bits_per_key);
uint64_t tkv_amq_vqf_required_size(int tag_bits, uint64_t nslots);
uint64_t tkv_amq_vqf_nslots_for_size(int tag_bits, uint64_t bytes);

/* TreeOptions filter page sizing (tree/tree_options.hpp:177-258).
 *  leaf_size              TreeOptions::leaf_size() (default 2 MiB)
 *  key/value_size_hint    defaults 24 / 100 (tree_options.hpp:58-59)
 *  bits_per_key           as set (the VQF clamp of filter_bits_per_key() is applied here)
 * tkv_amq_filter_page_size_log2 returns the derived log2 page size (0 for VQF with bpk 0, where
 * the reference would divide by a zero load factor).  The filter page payload capacity the
 * builders see is (1 << log2) - 64 (the llfs PackedPageHeader). */
uint64_t tkv_amq_leaf_data_size(uint64_t leaf_size);
uint64_t tkv_amq_expected_items_per_leaf(uint64_t leaf_size, uint32_t key_size_hint,
                                         uint32_t value_size_hint);
uint32_t tkv_amq_filter_page_size_log2(int kind, uint64_t leaf_size, uint32_t key_size_hint,
                                       uint32_t value_size_hint, uint64_t bits_per_key);

/* Host-side plan for a batch of n_segs leaves.
 *  seg_key_counts[n_segs]  items per leaf (keys are laid out leaf after leaf)
 *  src_page_ids[n_segs]    leaf page ids (NULL => segment index)
 *  bits_per_key            as passed to build_filter_for_leaf_in_job (0 => no filters)
 *  payload_capacity        filter page payload bytes (page size - page header); 0 => unlimited
 *                          (VQF needs a capacity: it drives vqf_nslots_for_size)
 *  out_stride              0 => payloads packed back to back (64-byte aligned); otherwise each
 *                          segment s starts at s * out_stride (e.g. the filter page size)
 *  segs[n_segs]            (out) plan; upload it to the device before tkv_amq_build
 *  total_out_bytes         (out) size of the output array
 *  workspace_bytes         (out) device workspace tkv_amq_build needs (0 for Bloom)
 *  max_seg_blocks          (out) largest n_blocks of any segment (launch geometry) */
int tkv_amq_plan(int kind, const uint64_t* seg_key_counts, const uint64_t* src_page_ids,
                 uint32_t n_segs, uint32_t bits_per_key, uint64_t payload_capacity,
                 uint64_t out_stride, tkv_amq_segment* segs, uint64_t* total_out_bytes,
                 uint64_t* workspace_bytes, uint32_t* max_seg_blocks);

/* Plan whole filter pages: leaf s owns bytes [s << page_size_log2, (s+1) << page_size_log2) of
 * the output array, laid out as the page buffer FilterPageAlloc hands the builder
 * (filter_builder.hpp:70-88): a 64-byte PackedPageHeader, then the payload (capacity =
 * page size - 64, which drives the VQF sizing).  tkv_amq_build then also writes the header
 * fields the filter builders set -- layout_id ("vqf_filt", :237 / vqf_filter_page_view.hpp:142;
 * Bloom "bloomflt"), unused_begin = 64 + payload bytes, unused_end = page size (:293-296) --
 * and the page size.  Magic, page id and crc are the PageCache's (llfs) and are written as 0.
 * Header field offsets follow llfs 0.42's PackedPageHeader and are UNPINNED (llfs is absent).
 * Bytes between unused_begin and unused_end are not written. */
int tkv_amq_plan_pages(int kind, const uint64_t* seg_key_counts, const uint64_t* src_page_ids,
                       uint32_t n_segs, uint32_t bits_per_key, uint32_t page_size_log2,
                       tkv_amq_segment* segs, uint64_t* total_out_bytes, uint64_t* workspace_bytes,
                       uint32_t* max_seg_blocks);

/* Device build of every planned filter.
 *  keys         device; fixed-length keys (key_offsets == NULL: key i at keys + i*key_stride,
 *               length key_stride) or variable-length (key_offsets[n_keys+1], device)
 *  d_segs       device copy of the plan; max_seg_blocks as returned by tkv_amq_plan
 *  d_out        device output array (total_out_bytes)
 *  d_workspace  device workspace (workspace_bytes, 16-byte aligned)
 * Asynchronous on `stream`.  VQF insert failures (the reference BATT_CHECKs,
 * filter_builder.hpp:211) are recorded in the workspace; read them with
 * tkv_amq_build_check after the stream completes.  VQF workspace header (written by every
 * build, so no clearing is needed between builds): bytes [4, 8) = the build's n_segs; bytes
 * [64 + 4*s, 68 + 4*s) = leaf s's element count, with TKV_AMQ_VQF_FLAG_OVERFLOW set if one of
 * its inserts failed and TKV_AMQ_VQF_FLAG_WORKSPACE if the workspace was short (a caller may
 * copy these words back with its own results instead of calling tkv_amq_build_check). */
#define TKV_AMQ_VQF_NELTS_OFFSET 64u
#define TKV_AMQ_VQF_FLAG_OVERFLOW 0x80000000u
#define TKV_AMQ_VQF_FLAG_WORKSPACE 0x40000000u
int tkv_amq_build(int kind, const uint8_t* keys, const uint64_t* key_offsets,
                  uint32_t key_stride, uint64_t n_keys, const tkv_amq_segment* d_segs,
                  uint32_t n_segs, uint32_t max_seg_blocks, uint8_t* d_out,
                  void* d_workspace, uint64_t workspace_bytes, void* stream);

/* tkv_amq_build with the host copy of the plan's segments (h_segs: the n_segs entries
 * tkv_amq_plan filled; d_segs is their device copy).  With it a Bloom batch of 16- or 24-byte
 * keys builds its leaves of more than 5 LDS windows (images past 800 KB; tree/tree_options.hpp:
 * 177-215 sizes any leaf) through the tiled build, up to 40 of them per launch, and the other
 * leaves through the batch kernels; with other key shapes (variable-length, other strides) only
 * the leaves past 16 windows (2.5 MB) leave the batch kernels, each hashed into bit records by
 * a pass of its own and built by the tiled build (k <= 8; above, device atomics); tkv_amq_build
 * of such a batch sets those leaves' bits with device atomics.  The workspace tkv_amq_plan
 * sizes covers either key shape.
 * h_segs == NULL, a single leaf, or a batch without such leaves: exactly tkv_amq_build. */
int tkv_amq_build_ex(int kind, const uint8_t* keys, const uint64_t* key_offsets, uint32_t key_stride,
                     uint64_t n_keys, const tkv_amq_segment* d_segs, const tkv_amq_segment* h_segs,
                     uint32_t n_segs, uint32_t max_blocks, uint8_t* d_out, void* d_workspace,
                     uint64_t workspace_bytes, void* stream);

/* Synchronises `stream`; returns TKV_AMQ_OK, TKV_AMQ_INTERNAL (a VQF block overflowed) or
 * TKV_AMQ_INVALID_ARGUMENT (the workspace was smaller than the plan).  Bloom builds cannot
 * fail on the device. */
int tkv_amq_build_check(int kind, const void* d_workspace, uint64_t workspace_bytes,
                        void* stream);

/* Hash-range sharding of ONE monolithic Bloom filter over several GPUs (BASELINE config 5,
 * SURVEY.md 8(e); no reference counterpart: the reference builds each filter on one CPU
 * thread, filter_builder.hpp:126-135).  The filter planned by tkv_amq_plan for the whole key
 * set (one segment of n_blocks blocks) is cut into T = ceil(n_blocks / tile_blocks) tiles of
 * tkv_amq_bloom_tile_blocks() blocks (2048: one 128 KiB LDS image); part p of n_parts owns
 * tiles [p*q, min((p+1)*q, T)), q = ceil(T / n_parts), i.e. a contiguous byte range of the
 * bitmap.  A key belongs to the tile of its block (h0).  A rank may own several consecutive
 * parts (its range is then their union, built part by part).
 *
 * tkv_amq_bloom_route: rank-local step 1.  Reorders this rank's n_keys 16-byte keys by owning
 * part into d_routed16 (part 0's keys first) and writes the per-part counts
 * (d_part_counts[n_parts], u32, device) -- the send counts of the all-to-all that follows.
 * d_seg is the whole filter's segment (device), n_blocks its n_blocks (host copy). */
uint32_t tkv_amq_bloom_tile_blocks(void);
/* the most tiles one range build takes, from records (records != 0) or from 16-byte keys: the
 * partition's LDS tile table (6,400 tiles) */
uint32_t tkv_amq_bloom_range_max_tiles(int records);
uint64_t tkv_amq_bloom_route_ws_bytes(uint64_t n_keys, uint32_t n_parts);
int tkv_amq_bloom_route(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                        uint32_t n_blocks, uint32_t n_parts, uint8_t* d_routed16,
                        uint32_t* d_part_counts, void* d_workspace, uint64_t workspace_bytes,
                        void* stream);

/* tkv_amq_bloom_build_range: rank-local step 2, after the all-to-all.  Builds tiles
 * [tile_begin, tile_end) of the filter from the keys this rank received (all of whose tiles
 * must fall in the range; others are ignored) into d_out at the segment's out_offset, exactly
 * where tkv_amq_build puts them, and writes the filter header too.  Bytes of other tiles are
 * not touched, so the ranks' ranges are disjoint and one all-gather of them is the filter.
 * An empty range (tile_begin == tile_end: a rank past the last tile when ceil(T/q) < ranks)
 * writes the header only.  Keys are 16 bytes (route and range build alike); a range holds at
 * most tkv_amq_bloom_range_max_tiles(0) tiles. */
uint64_t tkv_amq_bloom_build_range_ws_bytes(uint64_t n_keys, uint32_t tile_begin, uint32_t tile_end);
int tkv_amq_bloom_build_range(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                              uint32_t n_blocks, uint32_t tile_begin, uint32_t tile_end,
                              uint8_t* d_out, void* d_workspace, uint64_t workspace_bytes,
                              void* stream);

/* The same two steps with 12-byte bit records in place of the keys (hash_count <= 8, i.e.
 * bits_per_key <= 12; InvalidArgument otherwise): tkv_amq_bloom_route_records hashes each key
 * once and writes its record (block in tile, the k bit indices, the tile relative to its
 * owner's first tile) into d_recs12 ordered by owner, so the all-to-all carries 12 bytes per key
 * instead of 16 and the owner does not hash again; tkv_amq_bloom_build_range_records builds the
 * owner's tiles from the records it received.  The record carries its tile relative to its
 * part, so a part -- and a range built from records -- holds at most
 * tkv_amq_bloom_range_max_tiles(1) tiles (6,400: 800 MiB of filter); a route with larger parts
 * is refused (InvalidArgument). */
uint64_t tkv_amq_bloom_route_records_ws_bytes(uint64_t n_keys, uint32_t n_parts);
int tkv_amq_bloom_route_records(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                                uint32_t n_blocks, uint32_t hash_count, uint32_t n_parts,
                                uint8_t* d_recs12, uint32_t* d_part_counts, void* d_workspace,
                                uint64_t workspace_bytes, void* stream);
/* tkv_amq_bloom_route_records_ex: the same with key_bytes 16 or 24 (24-byte keys 8-byte
 * aligned: TurtleKV's default key size, tree/tree_options.hpp:58); the records, and so the
 * exchange and tkv_amq_bloom_build_range_records, do not depend on the key size.  Same
 * workspace as tkv_amq_bloom_route_records_ws_bytes. */
int tkv_amq_bloom_route_records_ex(const uint8_t* d_keys, uint32_t key_bytes, uint64_t n_keys,
                                   const tkv_amq_segment* d_seg, uint32_t n_blocks,
                                   uint32_t hash_count, uint32_t n_parts, uint8_t* d_recs12,
                                   uint32_t* d_part_counts, void* d_workspace,
                                   uint64_t workspace_bytes, void* stream);
uint64_t tkv_amq_bloom_build_range_records_ws_bytes(uint64_t n_recs, uint32_t tile_begin,
                                                    uint32_t tile_end);
int tkv_amq_bloom_build_range_records(const uint8_t* d_recs12, uint64_t n_recs,
                                      const tkv_amq_segment* d_seg, uint32_t n_blocks,
                                      uint32_t hash_count, uint32_t tile_begin, uint32_t tile_end,
                                      uint8_t* d_out, void* d_workspace, uint64_t workspace_bytes,
                                      void* stream);

/* The pipelined hash-range build (hash_count <= 8): the route writes fixed-capacity part
 * blocks, so the exchange needs no counts first.  Parts of q tiles are owned round-robin: part p
 * belongs to rank p % world as its part j = p / world, so round j (parts [j*world, (j+1)*world))
 * is one contiguous byte range of the bitmap and can be all-gathered in place as soon as every
 * rank has built its part of it.  Per step, each rank:
 *   1. routes its keys in n_chunks chunks (tkv_amq_bloom_route_blocks): every key hashed once
 *      into its 12-byte bit record, counting-sorted by part on chip, and appended to its route
 *      workgroup's region of that part's block.  Chunk c's send buffer holds n_parts blocks in
 *      global part order (part p at p * block_bytes), so round j's blocks -- one per
 *      destination -- are one slice;
 *   2. exchanges round j of chunk c with one all-to-all of equal splits (block_bytes per peer):
 *      the chunks' rounds as their routes finish, the last chunk round by round;
 *   3. builds its part j from the n_chunks * world blocks of round j it received, laid out
 *      contiguously (tkv_amq_bloom_build_part_blocks), as soon as they have landed, writing the
 *      part's tiles where tkv_amq_build puts them (and the header);
 *   4. all-gathers round j as soon as its part of round j is built, while the next rounds
 *      are exchanged and built.
 * Records beyond a region's capacity travel as (record, part) entries in its block's overflow area, at
 * most ovf_cap per block; tkv_amq_bloom_blocks_lost reports a block that needed more (keys far
 * from uniform, e.g. one key repeated), after which the caller must build through the exact
 * exchange (tkv_amq_bloom_route_records + tkv_amq_bloom_build_range_records) instead. */
typedef struct tkv_amq_route_plan {
  uint32_t n_tiles;          /* T = ceil(n_blocks / tile_blocks) */
  uint32_t n_parts;          /* world * parts_per_rank */
  uint32_t parts_per_rank;   /* g */
  uint32_t part_tiles;       /* q: part p owns tiles [p*q, min((p+1)*q, T)) */
  uint32_t world;
  uint32_t n_chunks;
  uint32_t route_wgs;        /* P: route workgroups per chunk (= a part build's workgroups) */
  uint32_t region_cap;       /* records per (part block, route workgroup) region */
  uint32_t ovf_cap;          /* overflow entries per part block */
  uint32_t hash_count;
  uint64_t chunk_keys;       /* keys per chunk the capacities are sized for (fewer is fine) */
  uint64_t block_bytes;      /* one (chunk, sender, part) block */
  uint64_t counts_off, ovf_n_off, regions_off, ovf_off;  /* block layout */
  uint64_t route_ws_bytes;   /* workspace of one tkv_amq_bloom_route_blocks call */
  uint64_t part_ws_bytes;    /* workspace of one tkv_amq_bloom_build_part_blocks call */
  uint64_t part_bytes;       /* bitmap bytes per part (q tiles; parts past the last tile pad) */
  uint64_t n_blocks;         /* the filter's blocks */
} tkv_amq_route_plan;

/* chunk_keys: the most keys a rank routes per chunk (the capacities assume a uniform hash) */
int tkv_amq_bloom_route_plan(uint64_t chunk_keys, uint32_t n_chunks, uint32_t n_blocks,
                             uint32_t hash_count, uint32_t world, tkv_amq_route_plan* plan);
/* d_keys: n_keys keys of key_bytes 16 (16-byte aligned) or 24 (8-byte aligned), n_keys <=
 * plan->chunk_keys.  Part p's block goes to d_dst + (p / world) * round_stride + (p % world) *
 * block_bytes; round_stride 0 means world * block_bytes (a send buffer: n_parts * block_bytes,
 * part p at p * block_bytes).  A rank that exchanges nothing (world 1) routes chunk c straight
 * into its receive layout with d_dst = recv + c * block_bytes, round_stride = n_chunks *
 * block_bytes. */
int tkv_amq_bloom_route_blocks(const uint8_t* d_keys, uint32_t key_bytes, uint64_t n_keys,
                               const tkv_amq_segment* d_seg, const tkv_amq_route_plan* plan,
                               uint8_t* d_dst, uint64_t round_stride, void* d_workspace,
                               uint64_t workspace_bytes, void* stream);
/* part: the global part index (this rank's part j is j * world + rank); d_recv: the part's
 * n_recv blocks, block_bytes apart (n_chunks * world after the exchange of its round); d_out:
 * the whole filter payload (header + bitmap, padded to 64 + n_parts * part_bytes) */
int tkv_amq_bloom_build_part_blocks(const uint8_t* d_recv, uint32_t n_recv,
                                    const tkv_amq_segment* d_seg, const tkv_amq_route_plan* plan,
                                    uint32_t part, uint8_t* d_out, void* d_workspace,
                                    uint64_t workspace_bytes, void* stream);
/* synchronises `stream`; returns 1 if any of the n_recv blocks lost overflow entries (the
 * exact exchange must be used), 0 if none, < 0 on error */
int tkv_amq_bloom_blocks_lost(const uint8_t* d_recv, uint32_t n_recv, const tkv_amq_route_plan* plan,
                              void* stream);

/* Batched probe: query i tests the filter of segment d_query_seg[i].  d_result[i] = 1 if
 * the key may be present, 0 if the filter rejects it (reject_page == kTrue).  A segment index
 * >= n_segs, like a segment without a filter, answers 1 (kUnknown: cannot reject). */
int tkv_amq_probe(int kind, const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                  uint32_t n_segs, const uint8_t* queries, const uint64_t* query_offsets,
                  uint32_t query_stride, uint64_t n_queries, const uint32_t* d_query_seg,
                  uint8_t* d_result, void* stream);

/* KeyQuery::Metrics counters (tree/key_query.hpp:36-60) a probe launch adds to (device
 * memory, u64 each, accumulated with atomics across launches; zero them to reset). */
typedef struct tkv_amq_probe_metrics {
  uint64_t total_filter_query_count;    /* every (query, leaf) test (:154) */
  uint64_t no_filter_page_count;        /* leaf without a filter / outside the plan (:157) */
  uint64_t page_id_mismatch_count;      /* filter's src_page_id != the leaf asked about (:210,231) */
  uint64_t filter_reject_count;         /* definitely absent, kTrue (:243) */
  uint64_t filter_positive_count;       /* filter says maybe, kFalse (key_query.cpp:41) */
  uint64_t filter_false_positive_count; /* positive, but ground truth says absent (:77) */
} tkv_amq_probe_metrics;

/* Optional per-query inputs and outputs of the _ex probes (any field may be NULL):
 *  d_query_page_id[i]  the leaf page id query i asks about (reject_page's page_id_to_reject);
 *                      if it differs from the filter's src_page_id the answer is 1 (kUnknown)
 *  d_truth[i]          1 if the key is in the leaf (the leaf search's answer), for the
 *                      false-positive count; NULL => filter_false_positive_count untouched
 *  d_metrics           counters to add to */
typedef struct tkv_amq_probe_opts {
  const uint64_t* d_query_page_id;
  const uint8_t* d_truth;
  tkv_amq_probe_metrics* d_metrics;
} tkv_amq_probe_opts;

int tkv_amq_probe_ex(int kind, const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                     uint32_t n_segs, const uint8_t* queries, const uint64_t* query_offsets,
                     uint32_t query_stride, uint64_t n_queries, const uint32_t* d_query_seg,
                     uint8_t* d_result, const tkv_amq_probe_opts* opts, void* stream);

/* vqf_hash_val for n keys -> d_hash[n] (device) */
int tkv_amq_vqf_hash(const uint8_t* keys, const uint64_t* key_offsets, uint32_t key_stride,
                     uint64_t n_keys, uint64_t* d_hash, void* stream);

/* PackedVqfFilter::is_present(hash_val) for pre-hashed queries (hash once, probe many).
 * Pair i probes leaf d_pair_leaf[i] with hash d_hash[d_pair_query ? d_pair_query[i] : i]:
 * one query's hash serves every filter on its root-to-leaf path (tree/algo/nodes.hpp:165-178). */
int tkv_amq_vqf_probe_hashed(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                             uint32_t n_segs, const uint64_t* d_hash,
                             const uint32_t* d_pair_query, uint64_t n_pairs,
                             const uint32_t* d_pair_leaf, uint8_t* d_result, void* stream);
/* opts fields are indexed by pair i */
int tkv_amq_vqf_probe_hashed_ex(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                                uint32_t n_segs, const uint64_t* d_hash,
                                const uint32_t* d_pair_query, uint64_t n_pairs,
                                const uint32_t* d_pair_leaf, uint8_t* d_result,
                                const tkv_amq_probe_opts* opts, void* stream);

/* BloomFilterQuery<KeyView> (tree/key_query.hpp:78,97,219): the hashes one query needs,
 * computed once and reused for every Bloom filter it is tested against.  Record i lives at
 * d_query + i * tkv_amq_bloom_query_stride(k_max): u64 h0 (block selector and bit 0), then
 * u16 bit index of hash j for j = 1 .. k_max-1.  k_max <= 32; a filter whose hash_count
 * exceeds k_max cannot reject (result 1). */
uint32_t tkv_amq_bloom_query_stride(uint32_t k_max);
int tkv_amq_bloom_hash(const uint8_t* keys, const uint64_t* key_offsets, uint32_t key_stride,
                       uint64_t n_keys, uint32_t k_max, uint8_t* d_query, void* stream);
int tkv_amq_bloom_probe_hashed(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                               uint32_t n_segs, const uint8_t* d_query, uint32_t k_max,
                               const uint32_t* d_pair_query, uint64_t n_pairs,
                               const uint32_t* d_pair_leaf, uint8_t* d_result, void* stream);
int tkv_amq_bloom_probe_hashed_ex(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                                  uint32_t n_segs, const uint8_t* d_query, uint32_t k_max,
                                  const uint32_t* d_pair_query, uint64_t n_pairs,
                                  const uint32_t* d_pair_leaf, uint8_t* d_result,
                                  const tkv_amq_probe_opts* opts, void* stream);

/* Key staging, host only (no device needed): the H2D front end.  The reference passes the
 * build a flattened range of EditView whose keys are KeyView = std::string_view into leaf /
 * edit memory (core/merge_compactor.hpp:107-139, tree/filter_builder.hpp:307-331).  This
 * gathers the viewed key bytes into one contiguous, caller-owned (normally pinned) buffer
 * with up to n_threads host threads (<= 0: min(hardware threads, 16)).
 *  views, view_stride  view i is the tkv_amq_key_view at (const uint8_t*)views + i*view_stride;
 *                      the struct has the libstdc++ std::string_view layout {size, data}, so
 *                      &edits[0].key with stride sizeof(EditView) is read in place
 *  fixed_len > 0       every key must be fixed_len bytes (else InvalidArgument); key i lands
 *                      at dst + i*fixed_len (the fixed-stride key form of tkv_amq_build)
 *  fixed_len == 0      variable length: dst_offsets[n+1] (out) byte offsets into dst
 *  dst_capacity        bytes available at dst (ResourceExhausted if the keys do not fit) */
typedef struct tkv_amq_key_view {
  uint64_t size;
  const uint8_t* data;
} tkv_amq_key_view;
int tkv_amq_stage_keys(const void* views, uint64_t view_stride, uint64_t n_keys, uint32_t fixed_len,
                       uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_offsets, int n_threads);

/* Synthetic 16-byte keys on the device: key i = (splitmix64_at(seed, 2(first+i)+1),
 * splitmix64_at(seed, 2(first+i)+2)), little-endian (the bench input). */
int tkv_amq_gen_keys16(uint64_t seed, uint64_t first, uint64_t n_keys, uint8_t* d_keys,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TKV_AMQ_H */

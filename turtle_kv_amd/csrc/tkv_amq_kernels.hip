// tkv_amq_kernels.hip -- CDNA4 (gfx950) kernels for TurtleKV's per-leaf AMQ filters.
//
// Hot path:
//   bloom_build_lds      one workgroup per leaf filter ("segment"); 16-byte keys streamed with
//                        global_load_dwordx4, k XXH64 hashes in registers (seed-independent
//                        lane rounds shared), bits set in an LDS image of the whole filter with
//                        ds_or_b32, image written out with 16-byte coalesced stores.  Other key
//                        shapes: 24-byte lanes, or XxhShort for any key under 32 bytes.
//   bloom_part_* / bloom_tile   one filter larger than LDS (the monolithic variant, and a rank's
//                        tile range of a hash-range sharded filter): each key hashed once into
//                        a 12-byte bit record, ranked in its 128 KiB tile's run by an LDS
//                        histogram and stored straight to its per-(tile, workgroup) region,
//                        then each tile built in LDS from its records (route_*: the parts of
//                        a filter beyond one partition's tile table, and hash-range shards).
//   vqf_decide           one wave per segment replays the reference's insert order exactly
//                        (power-of-two-choice decisions depend only on per-block counts, kept
//                        in LDS); per 64-key chunk every conflict-free lane decides in the same
//                        round.  Emits one coalesced (block, rank, bucket, tag) record per key.
//   vqf_decide_ring      batches of <= 768 segments: producer waves hash, locate and match each
//                        64-key chunk into an LDS ring; one decider wave replays the order from
//                        it (a lone segment's serial chain, not the VALU rate, sets the time).
//   vqf_place_fused      one workgroup per segment: the records land at [block][rank] of an LDS
//                        image, then one thread per 64-byte block runs the stable counting sort
//                        by bucket offset and writes the block (vqf_scatter + vqf_place: the
//                        same through HBM for segments whose image does not fit LDS).
//   *_probe              one lane per (query, segment) test; *_hash + *_probe_hashed hash each
//                        query once for many segments.
// No MFMA anywhere: this is hashing and bit-set, not a contraction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>
#include <vector>

#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include "tkv_amq.h"
#include "tkv_amq_device.h"

// The one diagnostic build option (TKV_DIAG_RING: per-step timestamps of vqf_ring_place's
// decider, read by tools/ring_diag.py) is for experiment libraries only; the shipped library
// refuses it, and no option changes what a kernel computes.
#if defined(TKV_DIAG_RING) && !defined(TKV_AMQ_EXPERIMENT_BUILD)
#error "TKV_DIAG_RING is a diagnostic: build it only as an experiment library (-DTKV_AMQ_EXPERIMENT_BUILD)"
#endif

namespace tkv {

// ---------------------------------------------------------------------------------------
// constant tables
// ---------------------------------------------------------------------------------------
struct BloomSeeds {
  uint64_t seed[kMaxBloomHashes];
  uint64_t rhinit16[kMaxBloomHashes];  // rotl(seed + P5 + 16, 27), see Xxh16
  uint64_t seed_p5[kMaxBloomHashes];   // seed + P5, see XxhShort
};

constexpr BloomSeeds make_bloom_seeds()
{
  BloomSeeds t{};
  for (uint32_t i = 0; i < kMaxBloomHashes; ++i) {
    t.seed[i] = bloom_seed(i);
    t.rhinit16[i] = xxh16_rhinit(t.seed[i]);
    t.seed_p5[i] = t.seed[i] + kP5;
  }
  return t;
}

// constant-initialised at load: no host upload, so every entry point is graph-capturable
__constant__ BloomSeeds c_bloom = make_bloom_seeds();

// ---------------------------------------------------------------------------------------
// key access
// ---------------------------------------------------------------------------------------
// kKey24: fixed 24-byte keys, 8-byte aligned (Bloom build fast path; other kernels hash them
// through the generic fixed-stride path)
// kKeyLoc: not a key shape -- the small-batch VQF path's located keys (vqf_locate_keys writes
// one 8-byte record per key: vqf_loc_encode), read by vqf_ring_place in place of the keys
enum KeyMode : int { kKey16 = 0, kKeyFixed = 1, kKeyVar = 2, kKey24 = 3, kKeyLoc = 4 };

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// streaming (non-temporal) loads/stores for data touched exactly once, so it does not
// evict reused data (the probe's filter array) from L2 / the Infinity Cache
__device__ inline uint4 load_nt16(const void* p)
{
  const u32x4_t v = __builtin_nontemporal_load(static_cast<const u32x4_t*>(p));
  return uint4{v.x, v.y, v.z, v.w};
}

// key i of a fixed-stride or offset-indexed key array: its bytes and length
template <int MODE>
__device__ inline const uint8_t* key_at(const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                                        uint64_t i, uint32_t& len)
{
  if constexpr (MODE == kKeyFixed || MODE == kKey24) {
    len = stride;
    return keys + i * stride;
  } else {
    const uint64_t b = offs[i];
    len = (uint32_t)(offs[i + 1] - b);
    return keys + b;
  }
}

template <int MODE>
__device__ inline uint64_t hash_key(const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                                    uint64_t i, uint64_t seed)
{
  uint32_t len;
  const uint8_t* p = key_at<MODE>(keys, offs, stride, i, len);
  if (len < 32) return XxhShort(p, len).finish(seed + kP5);
  return xxh64_bytes(p, len, seed);
}

// Workgroup barrier for LDS hazards only: this wave's LDS operations are complete, its global
// loads and stores stay in flight (__syncthreads() also drains vmcnt, stores included).
__device__ inline void lds_barrier()
{
  // (the memory clobber keeps the compiler from moving LDS accesses across it)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------------------
// Bloom build (LDS image per segment)
// ---------------------------------------------------------------------------------------
__device__ inline void lds_set_bit(uint32_t* blk, uint32_t bit)
{
  // `bit`: bits 0..8 are the index, higher bits are ignored.  word = bits 5..8 (v_bfe_u32
  // in asm: LLVM would re-canonicalize the extract-then-scale into lshr + and + add); the
  // shift amount uses bits 0..4 only.
  uint32_t word;
  asm("v_bfe_u32 %0, %1, 5, 4" : "=v"(word) : "v"(bit));
  atomicOr(blk + word, 1u << (bit & 31));
}

// Bloom insert of one fixed/variable-length key: keys under 32 bytes share the seed-independent
// lane rounds over all k hashes (XxhShort); longer keys hash from scratch per seed.
template <int K, int MODE>
__device__ inline void bloom_insert_any(uint32_t* s_bits, uint32_t nb, uint32_t k,
                                        const uint8_t* p, uint32_t len)
{
  if (len < 32) {
    const XxhShort x(p, len);
    const uint64_t h0 = x.finish(c_bloom.seed_p5[0]);
    uint32_t* blk = s_bits + 16 * (uint32_t)__umul64hi(h0, (uint64_t)nb);
    lds_set_bit(blk, (uint32_t)h0 & 511u);
    if constexpr (K != 0) {
#pragma unroll
      for (uint32_t j = 1; j < (uint32_t)K; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.seed_p5[j]));
    } else {
      for (uint32_t j = 1; j < k; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.seed_p5[j]));
    }
  } else {
    const uint64_t h0 = xxh64_bytes(p, len, c_bloom.seed[0]);
    uint32_t* blk = s_bits + 16 * (uint32_t)__umul64hi(h0, (uint64_t)nb);
    lds_set_bit(blk, (uint32_t)h0 & 511u);
    for (uint32_t j = 1; j < k; ++j) lds_set_bit(blk, (uint32_t)xxh64_bytes(p, len, c_bloom.seed[j]) & 511u);
  }
}

__device__ inline void write_bloom_header(uint8_t* payload, const tkv_amq_segment& sg, int part)
{
  // 64-byte PackedBloomFilterPage header, written as 4 x 16 bytes
  uint64_t w0, w1;
  const uint64_t nb = sg.n_blocks;
  switch (part) {
    case 0: w0 = kBloomMagic; w1 = 512ull * nb; break;
    case 1: w0 = sg.src_page_id; w1 = 0; break;
    case 2: w0 = 8ull * nb; w1 = nb | ((uint64_t)sg.hash_count << 32) | (2ull << 48); break;
    default: w0 = sg.n_keys; w1 = 0; break;
  }
  ulonglong2 v;
  v.x = w0;
  v.y = w1;
  reinterpret_cast<ulonglong2*>(payload)[part] = v;
}

// The llfs PackedPageHeader fields the filter builders set, for segments planned by
// tkv_amq_plan_pages (page_flags & TKV_AMQ_PAGE_IMAGE): layout_id @16 (filter_builder.hpp:237),
// unused_begin @28 = 64 + payload bytes and unused_end @32 = page size (:293-296), size @60.
// The PageCache's own fields (magic, page_id, crc32, user slot) are written as 0.  Offsets
// follow llfs 0.42's PackedPageHeader and are UNPINNED (llfs is absent).
// part = 0..3: one 16-byte piece each.
constexpr uint64_t kLayoutVqf = 0x746c69665f667176ull;    // "vqf_filt" (vqf_filter_page_view.hpp:142)
constexpr uint64_t kLayoutBloom = 0x746c666d6f6f6c62ull;  // "bloomflt" (tkv-amq v1; llfs's unpinned)

__device__ inline void write_page_header(uint8_t* out, const tkv_amq_segment& sg, uint64_t layout,
                                         uint32_t part)
{
  if (!(sg.page_flags & TKV_AMQ_PAGE_IMAGE)) return;
  uint8_t* page = out + sg.out_offset - kPackedPageHeaderBytes;
  const uint32_t size = 1u << ((sg.page_flags >> 8) & 31u);
  uint4 v = {0, 0, 0, 0};
  if (part == 1) {
    v.x = (uint32_t)layout;
    v.y = (uint32_t)(layout >> 32);
    v.w = (uint32_t)kPackedPageHeaderBytes + sg.payload_bytes;  // unused_begin
  } else if (part == 2) {
    v.x = size;  // unused_end
  } else if (part == 3) {
    v.w = size;  // size
  }
  reinterpret_cast<uint4*>(page)[part] = v;
}

// `first`: block index of s_bits[0] (0 for a whole leaf image; a tile's first block for the
// monolithic build's tile images)
template <int K>
__device__ inline void bloom_insert16(uint32_t* s_bits, uint32_t nb, uint32_t k, const uint4& kv,
                                      uint32_t first)
{
  const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
  const uint64_t h0 = x.finish(c_bloom.rhinit16[0]);
  uint32_t* blk = s_bits + 16 * ((uint32_t)__umul64hi(h0, (uint64_t)nb) - first);
  lds_set_bit(blk, (uint32_t)h0 & 511u);
  if constexpr (K != 0) {
#pragma unroll
    for (uint32_t j = 1; j < (uint32_t)K; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.rhinit16[j]));
  } else {
    for (uint32_t j = 1; j < k; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.rhinit16[j]));
  }
}

template <int K, uint32_t NT = 256>
__device__ inline void bloom_keys16_lds(const uint4* __restrict__ kp, uint32_t n, uint32_t nb,
                                        uint32_t k, uint32_t* s_bits, uint32_t first = 0)
{
  const uint32_t tid = threadIdx.x;
  constexpr int U = 4;  // 4 x 16-byte loads in flight per lane
  for (uint32_t base = 0; base < n; base += NT * U) {
    uint4 kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * NT + tid;
      if (i < n) kv[u] = kp[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * NT + tid;
      if (i < n) bloom_insert16<K>(s_bits, nb, k, kv[u], first);
    }
  }
}

template <int K, int L, uint32_t NT>
__device__ inline void bloom_keysL_lds(const uint64_t* __restrict__ kp, uint32_t n, uint32_t nb,
                                       uint32_t k, uint32_t* s_bits)
{
  constexpr int N = L / 8;
  const uint32_t tid = threadIdx.x;
  constexpr int U = 2;
  for (uint32_t base = 0; base < n; base += NT * U) {
    uint64_t lanes[U][N];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = min(base + u * NT + tid, n - 1);
#pragma unroll
      for (int w = 0; w < N; ++w) lanes[u][w] = kp[(uint64_t)i * N + w];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u * NT + tid < n) {
        const XxhFixed<L> x(lanes[u]);
        const uint64_t h0 = x.finish(xxh_fixed_rc<L>(c_bloom.seed[0]));
        uint32_t* blk = s_bits + 16 * (uint32_t)__umul64hi(h0, (uint64_t)nb);
        lds_set_bit(blk, (uint32_t)h0 & 511u);
        if constexpr (K != 0) {
#pragma unroll
          for (uint32_t j = 1; j < (uint32_t)K; ++j)
            lds_set_bit(blk, x.finish_lo9(xxh_fixed_rc<L>(c_bloom.seed[j])));
        } else {
          for (uint32_t j = 1; j < k; ++j)
            lds_set_bit(blk, x.finish_lo9(xxh_fixed_rc<L>(c_bloom.seed[j])));
        }
      }
    }
  }
}

// Keys [kb, ke) of one leaf into its LDS image s_bits (NT threads).
template <int MODE, uint32_t NT>
__device__ inline void bloom_leaf_image(const uint8_t* __restrict__ keys,
                                        const uint64_t* __restrict__ offs, uint32_t stride,
                                        const tkv_amq_segment& sg, uint32_t kb, uint32_t ke,
                                        uint32_t* s_bits)
{
  const uint32_t n = ke - kb, nb = sg.n_blocks, k = sg.hash_count;
  if constexpr (MODE == kKey16) {
    const uint4* kp = reinterpret_cast<const uint4*>(keys) + sg.key_begin + kb;
    // k = 7 / 8 are the hash counts at 10 / 12 bits per key: fully unrolled variants
    if (k == 7) bloom_keys16_lds<7, NT>(kp, n, nb, k, s_bits);
    else if (k == 8) bloom_keys16_lds<8, NT>(kp, n, nb, k, s_bits);
    else bloom_keys16_lds<0, NT>(kp, n, nb, k, s_bits);
  } else if constexpr (MODE == kKey24) {
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys) + 3 * (sg.key_begin + kb);
    if (n != 0) {
      if (k == 7) bloom_keysL_lds<7, 24, NT>(kp, n, nb, k, s_bits);
      else if (k == 8) bloom_keysL_lds<8, 24, NT>(kp, n, nb, k, s_bits);
      else bloom_keysL_lds<0, 24, NT>(kp, n, nb, k, s_bits);
    }
  } else {
    // one key per thread per iteration (two in flight measured 2% slower: the loop is
    // VALU-bound, every lane paying for the longest key of its wave)
    for (uint32_t i = kb + threadIdx.x; i < ke; i += NT) {
      uint32_t len;
      const uint8_t* p = key_at<MODE>(keys, offs, stride, sg.key_begin + i, len);
      if (k == 7) bloom_insert_any<7, MODE>(s_bits, nb, k, p, len);
      else if (k == 8) bloom_insert_any<8, MODE>(s_bits, nb, k, p, len);
      else bloom_insert_any<0, MODE>(s_bits, nb, k, p, len);
    }
  }
}

// Variable-length keys, sorted by length before they are hashed.  XXH64 of a short key runs a
// different number of lane, 4-byte and byte steps per length, and a wave pays for every step
// any of its lanes needs (8..31-byte keys in one wave: ~71 VALU per seed instead of ~47 on
// average).  The Bloom filter does not depend on the order of its keys, so each chunk of
// kVarChunk(NT) keys is counting-sorted by exact length in LDS, as (offset, length) pairs, and
// hashed in that order: a wave then holds one or two lengths.  The hash loop runs two keys
// deep: the next key's bytes (XxhShort's lanes, 4-byte tail, tail bytes) are loaded while the
// current one is hashed.
template <uint32_t NT>
constexpr uint32_t kVarChunk = 4 * NT;
constexpr uint32_t kVarBins = 64;  // lengths 0..31 and ">= 32" (bin 32); 64 for the scan wave
template <uint32_t NT>
constexpr uint32_t kVarAuxWords = 2 * kVarBins + 2 * kVarChunk<NT>;

// Short keys through a buffer resource.  A resource covers a range of the key array (a chunk
// or a leaf) plus the 32 bytes after it, clipped to the array's end; every key under 32 bytes
// is read as one 32-byte window (two 16-byte loads, the offset relative to the resource, no
// per-load address arithmetic), the window's start clamped into the resource, so every lane
// issues the same two loads and none reads past the array.  A clamped window (a key among the
// array's last 32 bytes) is realigned after the loads arrive.  Bytes past a key are never
// used.  The 4-byte tail and the tail bytes are then picked out of word n8 = len / 8.
typedef uint32_t u32x4_b __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t byte_rsrc(const uint8_t* base, uint32_t bytes)
{
  // word 3 = 0x00020000: DATA_FORMAT 32, as raw buffer loads need on gfx9
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)bytes, 0x00020000);
}

struct VarRsrc {
  __amdgpu_buffer_rsrc_t r;
  uint64_t base;  // key-array offset of the resource's first byte
  uint32_t nrec;  // bytes it covers; 0: not usable (fewer than 32 bytes, or a range >= 2 GiB)
};

// keys [.., ..) whose bytes are [base, end) of an array of key_end bytes
__device__ inline VarRsrc var_rsrc(const uint8_t* keys, uint64_t base, uint64_t end, uint64_t key_end)
{
  const uint64_t want = end - base + 32, avail = key_end - base;
  const uint64_t n = want < avail ? want : avail;
  VarRsrc v;
  v.base = base;
  v.nrec = (n >= 32 && n < (1ull << 31)) ? (uint32_t)n : 0u;
  v.r = byte_rsrc(keys + base, v.nrec);
  return v;
}

struct KeyWin {  // 32 bytes of a key as loaded: starting d bytes before it when clamped
  u32x4_b a, b;
  uint32_t d;
};

__device__ inline void key_win_load(const VarRsrc& v, uint32_t rel, KeyWin& w)
{
  const uint32_t relc = min(rel, v.nrec - 32);
  w.a = __builtin_amdgcn_raw_buffer_load_b128(v.r, relc, 0, 0);
  w.b = __builtin_amdgcn_raw_buffer_load_b128(v.r, relc + 16, 0, 0);
  w.d = rel - relc;
}

// the window's key as XxhShort's lanes, 4-byte tail word and tail bytes (len < 32)
__device__ inline void key_win_parts(const KeyWin& w, uint32_t len, uint64_t (&l)[3], uint32_t& t4,
                                     uint32_t& tb)
{
  uint32_t x[8] = {w.a.x, w.a.y, w.a.z, w.a.w, w.b.x, w.b.y, w.b.z, w.b.w};
  if (w.d != 0) {  // (divergent, rare: shift the window down by d bytes)
    asm volatile("");  // (a branch, not if-converted into every key's instruction stream)
    const uint32_t d = w.d;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (d & 16) ? (i + 4 < 8 ? x[i + 4] : 0u) : x[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (d & 8) ? (i + 2 < 8 ? x[i + 2] : 0u) : x[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (d & 4) ? (i + 1 < 8 ? x[i + 1] : 0u) : x[i];
    const uint32_t r = d & 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_alignbyte(i + 1 < 8 ? x[i + 1] : 0u, x[i], r);
  }
  l[0] = mk64(x[0], x[1]);
  l[1] = mk64(x[2], x[3]);
  l[2] = mk64(x[4], x[5]);
  const uint32_t n8 = len >> 3;
  const uint32_t tlo = n8 == 0 ? x[0] : n8 == 1 ? x[2] : n8 == 2 ? x[4] : x[6];
  const uint32_t thi = n8 == 0 ? x[1] : n8 == 1 ? x[3] : n8 == 2 ? x[5] : x[7];
  t4 = tlo;
  tb = (len & 4) ? thi : tlo;
}

// Without a usable resource: the key's full 8-byte lanes, its 4-byte tail and its tail bytes
// loaded one by one (clamped to `safe`, >= 16 readable bytes, past the key), packed as the
// window key_win_parts reads (the tail word at word n8).
__device__ inline void key_win_load_clamped(const uint8_t* p, uint32_t len, const uint8_t* safe, KeyWin& w)
{
  const bool sh = len < 32;
  const uint32_t n8 = len >> 3, nb = len & 3;
  uint64_t l[3];
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) l[j] = ld64_unaligned(sh && j < n8 ? p + 8 * j : safe);
  const uint8_t* q = p + 8 * n8;
  const uint32_t t4 = ld32_unaligned(sh && (len & 4) ? q : safe);
  q += len & 4;
  const uint32_t c0 = *(sh && nb > 0 ? q : safe), c1 = *(sh && nb > 1 ? q + 1 : safe),
                 c2 = *(sh && nb > 2 ? q + 2 : safe);
  const uint32_t tb = c0 | c1 << 8 | c2 << 16;
  const uint32_t tlo = (len & 4) ? t4 : tb;  // word n8 as key_win_parts reads it
  w.a = u32x4_b{lo32(l[0]), hi32(l[0]), lo32(l[1]), hi32(l[1])};
  w.b = u32x4_b{lo32(l[2]), hi32(l[2]), tlo, tb};
  if (n8 == 0) { w.a.x = tlo; w.a.y = tb; }
  else if (n8 == 1) { w.a.z = tlo; w.a.w = tb; }
  else if (n8 == 2) { w.b.x = tlo; w.b.y = tb; }
  w.d = 0;
}

struct VarKey {  // a key under 32 bytes as its window (a longer one: its address)
  KeyWin w;
  uint32_t len;
  const uint8_t* p;
};

template <int K>
__device__ inline void var_key_insert(uint32_t* s_bits, uint32_t nb, uint32_t k, const VarKey& v)
{
  if (v.len < 32) {
    uint64_t l[3];
    uint32_t t4, tb;
    key_win_parts(v.w, v.len, l, t4, tb);
    const XxhShort x(v.len, l, t4, tb);
    const uint64_t h0 = x.finish(c_bloom.seed_p5[0]);
    uint32_t* blk = s_bits + 16 * (uint32_t)__umul64hi(h0, (uint64_t)nb);
    lds_set_bit(blk, (uint32_t)h0 & 511u);
    if constexpr (K != 0) {
#pragma unroll
      for (uint32_t j = 1; j < (uint32_t)K; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.seed_p5[j]));
    } else {
      for (uint32_t j = 1; j < k; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.seed_p5[j]));
    }
  } else {
    bloom_insert_any<K, kKeyVar>(s_bits, nb, k, v.p, v.len);
  }
}

// key_end: offset one past the key array's last byte (offs[batch keys])
template <uint32_t NT, int K>
__device__ void bloom_var_sorted_image(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                       const tkv_amq_segment& sg, uint32_t kb, uint32_t ke,
                                       uint32_t* s_bits, uint32_t* s_aux, uint64_t key_end)
{
  constexpr uint32_t C = kVarChunk<NT>, U = C / NT;
  uint32_t* bins = s_aux;                        // [kVarBins] counts of this chunk
  uint32_t* start = s_aux + kVarBins;            // [kVarBins] their exclusive prefix
  uint2* kl = reinterpret_cast<uint2*>(s_aux + 2 * kVarBins);  // [C] (offset - base, length), sorted
  const uint32_t tid = threadIdx.x, nb = sg.n_blocks, k = sg.hash_count;
  const uint64_t* o = offs + sg.key_begin;
  const uint8_t* safe = reinterpret_cast<const uint8_t*>(offs);  // >= 16 readable bytes
  for (uint32_t c0 = kb; c0 < ke; c0 += C) {
    const uint32_t cn = min(C, ke - c0);
    const uint64_t base = o[c0];
    if (tid < kVarBins) bins[tid] = 0;
    __syncthreads();
    uint32_t bin[U], rank[U], rel[U], len[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t j = u * NT + tid;
      const uint32_t i = c0 + min(j, cn - 1);
      const uint64_t b = o[i];
      const uint64_t l = o[i + 1] - b;
      rel[u] = (uint32_t)(b - base);
      len[u] = (uint32_t)l;
      bin[u] = l < 32 ? (uint32_t)l : 32u;
      rank[u] = j < cn ? atomicAdd(bins + bin[u], 1u) : 0u;
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: exclusive scan of the bins
      const uint32_t v = bins[tid];
      uint32_t inc = v;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (tid >= d) inc += y;
      }
      start[tid] = inc - v;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t j = u * NT + tid;
      if (j < cn) kl[start[bin[u]] + rank[u]] = make_uint2(rel[u], len[u]);
    }
    __syncthreads();
    const uint8_t* kbase = keys + base;
    // the chunk's bytes through a buffer resource (KeyWin) when they span < 2 GiB (always,
    // but for keys of megabytes)
    const VarRsrc vr = var_rsrc(keys, base, o[c0 + cn], key_end);
    VarKey A, B;
    auto load = [&](uint32_t q, VarKey& v) {
      const uint2 e = kl[min(q, cn - 1)];
      if (vr.nrec) key_win_load(vr, e.x, v.w);  // (uniform)
      else key_win_load_clamped(kbase + e.x, e.y, safe, v.w);
      v.len = e.y;
      v.p = kbase + e.x;
    };
    load(tid, A);
    for (uint32_t q = tid; q < cn; q += 2 * NT) {
      load(q + NT, B);
      var_key_insert<K>(s_bits, nb, k, A);
      if (q + NT >= cn) break;
      load(q + 2 * NT, A);
      var_key_insert<K>(s_bits, nb, k, B);
    }
    __syncthreads();  // (the next chunk rewrites bins and the pairs)
  }
}

// One workgroup per leaf filter (batches of >= kBloomSplitSegs leaves).  Variable-length keys
// (var_sort): the length sort's scratch comes first in the dynamic LDS, then the image.
template <int MODE, uint32_t NT>
__global__ __launch_bounds__(NT) void bloom_build_lds(const uint8_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ offs,
                                                       uint32_t stride,
                                                       const tkv_amq_segment* __restrict__ segs,
                                                       uint8_t* __restrict__ out, uint32_t var_sort)
{
  extern __shared__ uint32_t s_lds[];
  const bool sorted = MODE == kKeyVar && var_sort;
  uint32_t* s_bits = s_lds + (sorted ? kVarAuxWords<NT> : 0u);
  const tkv_amq_segment sg = segs[blockIdx.x];
  const uint32_t n = sg.n_keys, nb = sg.n_blocks, k = sg.hash_count;
  if (k == 0) return;  // bits_per_key == 0: no filter (filter_builder.hpp:115-117)
  const uint32_t tid = threadIdx.x;
  const uint32_t nwords = nb * 16;

  for (uint32_t w = tid; w < nwords; w += NT) s_bits[w] = 0;
  __syncthreads();
  if constexpr (MODE == kKeyVar) {
    if (sorted) {
      // (one workgroup per leaf: the batch's last leaf ends the key array)
      const tkv_amq_segment& last = segs[gridDim.x - 1];
      const uint64_t key_end = offs[last.key_begin + last.n_keys];
      if (k == 7) bloom_var_sorted_image<NT, 7>(keys, offs, sg, 0, n, s_bits, s_lds, key_end);
      else if (k == 8) bloom_var_sorted_image<NT, 8>(keys, offs, sg, 0, n, s_bits, s_lds, key_end);
      else bloom_var_sorted_image<NT, 0>(keys, offs, sg, 0, n, s_bits, s_lds, key_end);
    } else {
      bloom_leaf_image<MODE, NT>(keys, offs, stride, sg, 0, n, s_bits);
    }
  } else {
    bloom_leaf_image<MODE, NT>(keys, offs, stride, sg, 0, n, s_bits);
  }
  __syncthreads();

  uint8_t* payload = out + sg.out_offset;
  if (tid < 4) write_bloom_header(payload, sg, tid);
  else if (tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
  uint4* dst = reinterpret_cast<uint4*>(payload + kBloomHeader);
  const uint4* src = reinterpret_cast<const uint4*>(s_bits);
  for (uint32_t q = tid; q < nb * 4; q += NT) dst[q] = src[q];
}

// Batches too small to fill the chip with one workgroup per leaf (one leaf per call, or a
// checkpoint of a few hundred leaves): each leaf's keys are split over `parts` workgroups,
// each building the image of its key range in LDS and writing it to the workspace
// (bloom_build_split); bloom_split_merge then ORs a leaf's part images into the filter.  The
// bits set do not depend on which workgroup set them, so the filter equals the one-workgroup
// build.  Two kernels, not a last-workgroup merge: the parts of a leaf run on different XCDs,
// and an agent-scope fence per workgroup (an L2 writeback plus invalidate on each XCD) made
// the merge pattern 4-9x slower than this.  Workspace: image (s, p) at
// ((s * parts) + p) * img_stride.
constexpr uint32_t kSplitThreads = 512;
constexpr uint32_t kSplitMaxParts = 16;
constexpr uint32_t kMergeThreads = 256;

template <int MODE>
__global__ __launch_bounds__(kSplitThreads) void bloom_build_split(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t stride,
    const tkv_amq_segment* __restrict__ segs, uint32_t parts, uint8_t* __restrict__ ws,
    uint64_t img_stride)
{
  constexpr uint32_t NT = kSplitThreads;
  extern __shared__ uint32_t s_bits[];
  const uint32_t seg = blockIdx.x / parts, part = blockIdx.x - seg * parts;
  const tkv_amq_segment sg = segs[seg];
  const uint32_t n = sg.n_keys, nb = sg.n_blocks;
  if (sg.hash_count == 0) return;  // no filter
  const uint32_t tid = threadIdx.x;
  for (uint32_t w = tid; w < nb * 16; w += NT) s_bits[w] = 0;
  __syncthreads();
  const uint32_t chunk = (n + parts - 1) / parts;
  const uint32_t kb = min(n, part * chunk), ke = min(n, kb + chunk);
  bloom_leaf_image<MODE, NT>(keys, offs, stride, sg, kb, ke, s_bits);
  __syncthreads();
  const uint4* img = reinterpret_cast<const uint4*>(s_bits);
  uint4* dst = reinterpret_cast<uint4*>(ws + (uint64_t)blockIdx.x * img_stride);
  for (uint32_t q = tid; q < nb * 4; q += NT) dst[q] = img[q];
}

// one thread per 16-byte word of a leaf's image, kMergeThreads words per workgroup: all the
// parts' loads are issued together (up to kSplitMaxParts, predicated), then ORed
__global__ __launch_bounds__(kMergeThreads) void bloom_split_merge(
    const tkv_amq_segment* __restrict__ segs, uint32_t parts, uint32_t chunks,
    const uint8_t* __restrict__ ws, uint64_t img_stride, uint8_t* __restrict__ out)
{
  const uint32_t seg = blockIdx.x / chunks, c = blockIdx.x - seg * chunks;
  const tkv_amq_segment sg = segs[seg];
  if (sg.hash_count == 0) return;
  const uint32_t tid = threadIdx.x, nq = sg.n_blocks * 4;
  uint8_t* payload = out + sg.out_offset;
  if (c == 0 && tid < 4) write_bloom_header(payload, sg, tid);
  else if (c == 0 && tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
  const uint32_t q = c * kMergeThreads + tid;
  if (q >= nq) return;
  const uint8_t* base = ws + (uint64_t)seg * parts * img_stride + 16ull * q;
  uint4 o[kSplitMaxParts];
#pragma unroll
  for (uint32_t p = 0; p < kSplitMaxParts; ++p)
    o[p] = p < parts ? load_nt16(base + (uint64_t)p * img_stride) : make_uint4(0, 0, 0, 0);
  uint4 v = o[0];
#pragma unroll
  for (uint32_t p = 1; p < kSplitMaxParts; ++p) {
    v.x |= o[p].x;
    v.y |= o[p].y;
    v.z |= o[p].z;
    v.w |= o[p].w;
  }
  reinterpret_cast<uint4*>(payload + kBloomHeader)[q] = v;
}

// ---------------------------------------------------------------------------------------
// Bloom build, leaves whose image exceeds one CU's LDS, in batches of any size
// (bloom_build_window).  The image of a leaf of nb blocks is cut into W windows of at most
// win_blocks blocks (<= kBloomLeafLdsBudget bytes); workgroup (leaf, window, part) streams the
// keys of its part of the leaf, computes each key's block (h0) and keeps only the keys whose
// block falls in its window.  Those are packed densely across the wave: each step's in-window
// lanes are pushed (ds_permute, a full permutation of the 64 lanes) behind the c keys still
// pending, and whenever 64 are pending the wave computes their other k - 1 hashes and sets
// their bits.  So only the seed-0 hash is repeated per window (~70 VALU of the ~280 a k = 8
// key costs); a window never hashes another window's keys.  A key moves as its hash state
// (16-byte keys: the two lane rounds; 24-byte keys: the three) plus its window block and
// bit 0; other key shapes move as their index and are re-hashed.  With one part per leaf
// the window is written straight into the filter; with several, each part writes its
// windows into a full-size partial image and bloom_split_merge ORs them.
// ---------------------------------------------------------------------------------------
constexpr uint32_t kWinThreads = 1024;
constexpr uint32_t kWinMaxWindows = 16;

template <int MODE>
struct WinItem {  // any key shape: the key's index in its leaf, then loc
  static constexpr int N = 2;
  uint32_t d[N];
};
template <>
struct WinItem<kKey16> {  // Xxh16 state (rk1, k2), then loc
  static constexpr int N = 5;
  uint32_t d[N];
};
template <>
struct WinItem<kKey24> {  // XxhFixed<24> state (rk0, k[0], k[1]), then loc
  static constexpr int N = 7;
  uint32_t d[N];
};
// loc = block in the window (< 4096) | bit index 0 << 12

template <int MODE>
struct WinKey {};
template <>
struct WinKey<kKey16> {
  uint4 v;
};
template <>
struct WinKey<kKey24> {
  uint64_t w[3];
};

template <int MODE>
__device__ inline void win_load(const uint8_t* __restrict__ keys, uint64_t gi, WinKey<MODE>& kb)
{
  if constexpr (MODE == kKey16) {
    kb.v = load_nt16(keys + 16 * gi);
  } else if constexpr (MODE == kKey24) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(keys) + 3 * gi;
#pragma unroll
    for (int i = 0; i < 3; ++i) kb.w[i] = p[i];
  }
}

// the key's block in its leaf (from h0) and its item (loc holds bit 0 only)
template <int MODE>
__device__ inline uint32_t win_hash(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                    uint32_t stride, const tkv_amq_segment& sg, uint32_t i,
                                    const WinKey<MODE>& kb, WinItem<MODE>& it)
{
  uint64_t h0;
  if constexpr (MODE == kKey16) {
    const Xxh16 x((uint64_t)kb.v.x | ((uint64_t)kb.v.y << 32), (uint64_t)kb.v.z | ((uint64_t)kb.v.w << 32));
    h0 = x.finish(c_bloom.rhinit16[0]);
    it.d[0] = lo32(x.rk1);
    it.d[1] = hi32(x.rk1);
    it.d[2] = lo32(x.k2);
    it.d[3] = hi32(x.k2);
  } else if constexpr (MODE == kKey24) {
    const XxhFixed<24> x(kb.w);
    h0 = x.finish(xxh_fixed_rc<24>(c_bloom.seed[0]));
    it.d[0] = lo32(x.rk0);
    it.d[1] = hi32(x.rk0);
    it.d[2] = lo32(x.k[0]);
    it.d[3] = hi32(x.k[0]);
    it.d[4] = lo32(x.k[1]);
    it.d[5] = hi32(x.k[1]);
  } else {
    h0 = hash_key<MODE>(keys, offs, stride, sg.key_begin + i, c_bloom.seed[0]);
    it.d[0] = i;
  }
  it.d[WinItem<MODE>::N - 1] = ((uint32_t)h0 & 511u) << 12;
  return (uint32_t)__umul64hi(h0, (uint64_t)sg.n_blocks);
}

// the other k - 1 bits of a packed key, and bit 0
template <int MODE, int K>
__device__ inline void win_insert(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                  uint32_t stride, const tkv_amq_segment& sg, uint32_t k,
                                  const WinItem<MODE>& it, uint32_t* s_bits)
{
  const uint32_t loc = it.d[WinItem<MODE>::N - 1];
  uint32_t* blk = s_bits + 16 * (loc & 0xfffu);
  lds_set_bit(blk, loc >> 12);
  const uint32_t kk = K != 0 ? (uint32_t)K : k;
  if constexpr (MODE == kKey16) {
    Xxh16 x;
    x.rk1 = mk64(it.d[0], it.d[1]);
    x.k2 = mk64(it.d[2], it.d[3]);
    if constexpr (K != 0) {
#pragma unroll
      for (uint32_t j = 1; j < (uint32_t)K; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.rhinit16[j]));
    } else {
      for (uint32_t j = 1; j < kk; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.rhinit16[j]));
    }
  } else if constexpr (MODE == kKey24) {
    XxhFixed<24> x;
    x.rk0 = mk64(it.d[0], it.d[1]);
    x.k[0] = mk64(it.d[2], it.d[3]);
    x.k[1] = mk64(it.d[4], it.d[5]);
    if constexpr (K != 0) {
#pragma unroll
      for (uint32_t j = 1; j < (uint32_t)K; ++j)
        lds_set_bit(blk, x.finish_lo9(xxh_fixed_rc<24>(c_bloom.seed[j])));
    } else {
      for (uint32_t j = 1; j < kk; ++j) lds_set_bit(blk, x.finish_lo9(xxh_fixed_rc<24>(c_bloom.seed[j])));
    }
  } else {
    uint32_t len;
    const uint8_t* p = key_at<MODE>(keys, offs, stride, sg.key_begin + it.d[0], len);
    if (len < 32) {
      const XxhShort x(p, len);
      for (uint32_t j = 1; j < kk; ++j) lds_set_bit(blk, x.finish_lo9(c_bloom.seed_p5[j]));
    } else {
      for (uint32_t j = 1; j < kk; ++j) lds_set_bit(blk, (uint32_t)xxh64_bytes(p, len, c_bloom.seed[j]));
    }
  }
}

__device__ inline uint32_t mbcnt64(uint64_t m)
{
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// keys [kb, ke) of the leaf, the ones in blocks [wb, wb + wn) into the window image s_bits
template <int MODE, int K>
__device__ void bloom_window_keys(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                  uint32_t stride, const tkv_amq_segment& sg, uint32_t wb, uint32_t wn,
                                  uint32_t kb, uint32_t ke, uint32_t* s_bits)
{
  constexpr int N = WinItem<MODE>::N;
  constexpr uint32_t NW = kWinThreads / 64;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t k = sg.hash_count;
  if (ke <= kb) return;
  WinItem<MODE> pend;
#pragma unroll
  for (int d = 0; d < N; ++d) pend.d[d] = 0;
  uint32_t c = 0;  // pending keys, in lanes [0, c)
  // one 64-key step of this wave; `cur` holds its keys (16 / 24 bytes, loaded a step ahead)
  auto step = [&](uint32_t base, const WinKey<MODE>& cur) {
    const uint32_t i = base + lane;
    WinItem<MODE> it;
    const uint32_t lb = win_hash<MODE>(keys, offs, stride, sg, min(i, ke - 1), cur, it) - wb;
    const bool in = i < ke && lb < wn;
    it.d[N - 1] |= lb & 0xfffu;
    const uint64_t mask = __ballot(in);
    const uint32_t m = (uint32_t)__popcll(mask);
    if (m == 0) return;
    // a permutation of the lanes: in-window lanes go (in order) behind the pending keys
    const uint32_t rank = mbcnt64(in ? mask : ~mask) + (in ? 0u : m);
    const int dest = (int)(((c + rank) & 63u) << 2);
    WinItem<MODE> pm;
#pragma unroll
    for (int d = 0; d < N; ++d) pm.d[d] = (uint32_t)__builtin_amdgcn_ds_permute(dest, (int)it.d[d]);
    if (c + m >= 64) {
      WinItem<MODE> full;
#pragma unroll
      for (int d = 0; d < N; ++d) full.d[d] = lane < c ? pend.d[d] : pm.d[d];
      win_insert<MODE, K>(keys, offs, stride, sg, k, full, s_bits);
      pend = pm;  // the keys that wrapped, in lanes [0, c + m - 64)
      c = c + m - 64;
    } else {
#pragma unroll
      for (int d = 0; d < N; ++d) pend.d[d] = lane < c ? pend.d[d] : pm.d[d];
      c += m;
    }
  };
  constexpr bool kPre = MODE == kKey16 || MODE == kKey24;
  auto load = [&](uint32_t base, WinKey<MODE>& kv) {
    if constexpr (kPre) win_load<MODE>(keys, sg.key_begin + min(base + lane, ke - 1), kv);
  };
  // unrolled by two with the buffers swapping roles (no register copy of a load in flight)
  WinKey<MODE> A{}, B{};
  uint32_t base = kb + wave * 64;
  load(base, A);
  for (; base < ke; base += 2 * NW * 64) {
    load(base + NW * 64, B);
    step(base, A);
    if (base + NW * 64 >= ke) break;
    load(base + 2 * NW * 64, A);
    step(base + NW * 64, B);
  }
  if (lane < c) win_insert<MODE, K>(keys, offs, stride, sg, k, pend, s_bits);
}

template <int MODE>
__global__ __launch_bounds__(kWinThreads) void bloom_build_window(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t stride,
    const tkv_amq_segment* __restrict__ segs, uint32_t n_win, uint32_t win_blocks, uint32_t parts,
    uint8_t* __restrict__ ws, uint64_t img_stride, uint8_t* __restrict__ out)
{
  extern __shared__ uint32_t s_bits[];
  const uint32_t per_seg = n_win * parts;
  const uint32_t seg = blockIdx.x / per_seg, r = blockIdx.x - seg * per_seg;
  const uint32_t w = r / parts, part = r - w * parts;
  const tkv_amq_segment sg = segs[seg];
  const uint32_t nb = sg.n_blocks, n = sg.n_keys, k = sg.hash_count;
  const uint32_t wb = w * win_blocks;
  if (k == 0 || wb >= nb) return;  // no filter, or a window past this leaf's image
  const uint32_t wn = min(win_blocks, nb - wb);
  const uint32_t tid = threadIdx.x;
  for (uint32_t q = tid; q < wn * 16; q += kWinThreads) s_bits[q] = 0;
  __syncthreads();
  const uint32_t chunk = (n + parts - 1) / parts;
  const uint32_t kb = min(n, part * chunk), ke = min(n, kb + chunk);
  if (nb <= win_blocks) {  // the whole image in one window: every key (the leaf kernel's loop)
    bloom_leaf_image<MODE, kWinThreads>(keys, offs, stride, sg, kb, ke, s_bits);
  } else if (k == 7) {
    bloom_window_keys<MODE, 7>(keys, offs, stride, sg, wb, wn, kb, ke, s_bits);
  } else if (k == 8) {
    bloom_window_keys<MODE, 8>(keys, offs, stride, sg, wb, wn, kb, ke, s_bits);
  } else {
    bloom_window_keys<MODE, 0>(keys, offs, stride, sg, wb, wn, kb, ke, s_bits);
  }
  __syncthreads();
  uint8_t* dst8;
  if (parts == 1) {
    uint8_t* payload = out + sg.out_offset;
    if (w == 0 && tid < 4) write_bloom_header(payload, sg, tid);
    else if (w == 0 && tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
    dst8 = payload + kBloomHeader + 64ull * wb;
  } else {
    dst8 = ws + (uint64_t)(seg * parts + part) * img_stride + 64ull * wb;
  }
  uint4* dst = reinterpret_cast<uint4*>(dst8);
  const uint4* src = reinterpret_cast<const uint4*>(s_bits);
  for (uint32_t q = tid; q < wn * 4; q += kWinThreads) dst[q] = src[q];
}

// ---------------------------------------------------------------------------------------
// Bloom build, global-memory fallback for segments whose image exceeds the LDS budget
// (monolithic filters).  Pass 1 zeroes + headers, pass 2 sets bits with device atomics.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bloom_global_init(const tkv_amq_segment* __restrict__ segs,
                                                         uint8_t* __restrict__ out)
{
  const tkv_amq_segment sg = segs[blockIdx.x];
  if (sg.hash_count == 0) return;
  uint8_t* payload = out + sg.out_offset;
  const uint32_t tid = threadIdx.x;
  if (tid < 4) write_bloom_header(payload, sg, tid);
  else if (tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
  uint4* dst = reinterpret_cast<uint4*>(payload + kBloomHeader);
  const uint4 z = {0, 0, 0, 0};
  for (uint64_t q = tid; q < 4ull * sg.n_blocks; q += 256) dst[q] = z;
}

__device__ inline uint32_t find_segment(const tkv_amq_segment* segs, uint32_t n_segs,
                                        uint64_t key)
{
  uint32_t lo = 0, hi = n_segs;  // last s with key_begin <= key
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].key_begin <= key) lo = mid;
    else hi = mid;
  }
  return lo;
}

template <int MODE>
__global__ __launch_bounds__(256) void bloom_global_set(const uint8_t* __restrict__ keys,
                                                        const uint64_t* __restrict__ offs,
                                                        uint32_t stride,
                                                        const tkv_amq_segment* __restrict__ segs,
                                                        uint32_t n_segs, uint64_t n_keys,
                                                        uint8_t* __restrict__ out, uint64_t first = 0)
{
  for (uint64_t i = first + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_keys;
       i += (uint64_t)gridDim.x * 256) {
    const uint32_t s = find_segment(segs, n_segs, i);
    const tkv_amq_segment& sg = segs[s];
    // (a leaf list need not cover every key: tkv_amq_build_ex hands the batch kernels the
    // leaves other than the oversize ones)
    if (sg.hash_count == 0 || i < sg.key_begin || i >= sg.key_begin + sg.n_keys) continue;
    uint32_t* words = reinterpret_cast<uint32_t*>(out + sg.out_offset + kBloomHeader);
    uint64_t h0;
    if constexpr (MODE == kKey16) {
      const uint4 kv = reinterpret_cast<const uint4*>(keys)[i];
      const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
      h0 = x.finish(c_bloom.rhinit16[0]);
      uint32_t* blk = words + 16 * (uint64_t)__umul64hi(h0, (uint64_t)sg.n_blocks);
      const uint32_t b0 = (uint32_t)h0 & 511u;
      atomicOr(blk + (b0 >> 5), 1u << (b0 & 31));
      for (uint32_t j = 1; j < sg.hash_count; ++j) {
        const uint32_t b = x.finish_lo9(c_bloom.rhinit16[j]) & 511u;
        atomicOr(blk + (b >> 5), 1u << (b & 31));
      }
    } else {
      h0 = hash_key<MODE>(keys, offs, stride, i, c_bloom.seed[0]);
      uint32_t* blk = words + 16 * (uint64_t)__umul64hi(h0, (uint64_t)sg.n_blocks);
      const uint32_t b0 = (uint32_t)h0 & 511u;
      atomicOr(blk + (b0 >> 5), 1u << (b0 & 31));
      for (uint32_t j = 1; j < sg.hash_count; ++j) {
        const uint32_t b = (uint32_t)hash_key<MODE>(keys, offs, stride, i, c_bloom.seed[j]) & 511u;
        atomicOr(blk + (b >> 5), 1u << (b & 31));
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Bloom build, monolithic filter: one filter larger than the window path takes (SURVEY.md
// 8(d)'s single-filter variant, the reference's build_bloom_filter_page over one item range,
// tree/filter_builder.hpp:126-135), and one rank's tile range of a hash-range sharded filter
// (BASELINE config 5).  The filter is cut into tiles of kTileBlocks 512-bit blocks (128 KiB,
// one LDS image each).  Every key is hashed once, where it is read, and what its tile needs of
// the hashes -- its 12-byte bit record -- travels instead of the key:
//   bloom_part      one 1024-thread workgroup per CU over a contiguous key range, in batches
//                   of kPartBatch: each key is hashed into its record and ranked in its tile's
//                   run of the batch by a returning ds_add on an LDS histogram (two u16
//                   counters per word); the batch is counting-sorted by tile in LDS planes and
//                   each tile's run is appended to this workgroup's region of that tile, so a
//                   store instruction writes a few long runs.  Region (t, w) holds `cap`
//                   records (mean + 6 sigma of a uniform hash); records beyond it go to the
//                   workgroup's overflow list (LDS counter).  LDS per tile beside the planes:
//                   two u16 histograms (double-buffered over batches), the u16 run starts and
//                   a u32 cursor, 10 bytes, so one pass takes up to kDirectMaxTiles tiles.
//   bloom_tile      one workgroup per tile: every region of the tile through ds_or into the
//                   128 KiB image, then 16-byte stores.
//   bloom_overflow  the overflow lists with device-scope atomicOr into the finished filter
//                   (empty unless the keys are not spread by the hash, e.g. duplicates).
// Partition sources: 16- and 24-byte keys (hashed here), 12-byte records routed by
// tkv_amq_bloom_route_records (not hashed again; the tile relative to the part is in the
// record), and, with k > 8, 16-byte keys as 16-byte records (the tile kernel hashes them).
// A filter of more than kDirectMaxTiles tiles is first routed into parts of at most
// kRecPartMaxTiles tiles (tkv_amq_bloom_route_records' kernels), and each part is built from
// its records, its count read on the device.  The bits set do not depend on which kernel or
// workgroup sets them, so the filter is byte-identical to the leaf kernel's and the oracle's.
// Record: w0 = blk | b0 << 11 | b1 << 20 | tile[0:2] << 29
//         w1 = b2 | b3 << 9 | b4 << 18 | tile[3:7] << 27
//         w2 = b5 | b6 << 9 | b7 << 18 | tile[8:12] << 27      (b_j = b_0 for j >= k)
// The tile field is the tile relative to the record's part (routed records); a partition's
// own region records leave it unused.  Overflow entries are 16 bytes: the record and its
// tile (relative to the build's first tile), or the 16-byte key.
// ---------------------------------------------------------------------------------------
constexpr uint32_t kTileBlocks = 2048;   // 128 KiB LDS image per tile
constexpr uint32_t kTileShift = 11;
constexpr uint32_t kTileThreads = 1024;  // one workgroup per CU
constexpr uint32_t kPartThreads = 1024;  // (two 512-thread workgroups per CU: 1.18 vs 1.03 ms)
constexpr uint32_t kPartU = 8;                              // items per thread per batch
constexpr uint32_t kPartBatch = kPartThreads * kPartU;      // < 65536: u16 ranks
constexpr uint32_t kPartMaxWgs = 256;  // one per CU
constexpr uint32_t kPartPlaneBytes = 12 * kPartBatch;       // the batch's records, sorted by tile
constexpr uint32_t kDirectMaxTiles = 6400;                  // LDS: 10 bytes per tile beside the planes
constexpr uint32_t kRecPartMaxTiles = kDirectMaxTiles;      // (< 2^13: a record's tile field)
constexpr uint32_t kRouteMaxParts = 2048;                   // tkv_amq_bloom_route(_records)
constexpr uint32_t kRouteMaxWgs = 1792;                     // route count / scatter workgroups
static_assert(kRouteMaxWgs % 256 == 0, "route_scan_cols: kRouteMaxWgs / 256 rows per thread");
// kSrcSeg12: the most route blocks one part build reads (chunks x senders)
constexpr uint32_t kMaxSrcSegs = 256;
// bloom_route_part (part_body bucketing by part): parts per route, and its LDS -- the three
// record planes, a u16 plane of each record's part, the histograms / starts / cursors of the
// parts, the wave sums and the overflow counter
__host__ __device__ constexpr inline uint32_t route_lds_bytes(uint32_t n_parts)
{
  return kPartPlaneBytes + 2u * kPartBatch + 20u * ((n_parts + 1) / 2) + 4u * (kPartThreads / 64 + 1) +
         8u + 12u * n_parts;  // + the per-part store pointers and limits of the batch
}
static_assert(route_lds_bytes(kRouteMaxParts) <= 160 * 1024, "one route workgroup per CU");

__host__ __device__ constexpr inline uint32_t part_lds_bytes(uint32_t n_tiles)
{
  // the planes; H0, H1, start: (T+1)/2 words each (u16 pairs); cursor: 2 * ((T+1)/2) words;
  // 16 wave sums and the overflow counter
  return kPartPlaneBytes + 20u * ((n_tiles + 1) / 2) + 4u * (kPartThreads / 64 + 1) +
         4u * (kMaxSrcSegs + 2);
}
static_assert(part_lds_bytes(kDirectMaxTiles) <= 160 * 1024, "one workgroup per CU");
// a partition with the store table (12 bytes per tile beside the rest) when it fits the CU's LDS
__host__ __device__ constexpr inline uint32_t part_tbl_lds_bytes(uint32_t n_tiles)
{
  return part_lds_bytes(n_tiles) + 8u + 12u * n_tiles;
}
__host__ __device__ constexpr inline bool part_tbl_fits(uint32_t n_tiles)
{
  return part_tbl_lds_bytes(n_tiles) <= 160u * 1024u;
}
static_assert(kRecPartMaxTiles <= 8192, "a record's 13-bit tile field");
static_assert(kPartBatch < 65536, "u16 ranks");

enum PartSrc : int { kSrcKey16 = 0, kSrcKey24 = 1, kSrcRec12 = 2, kSrcRaw16 = 3, kSrcSeg12 = 4 };
// what part_body buckets by: the filter's tiles (the partition, ahead of bloom_tile), or the
// route's parts (bloom_route_part: the one-pass route of a filter past kDirectMaxTiles tiles,
// and of a hash-range sharded filter's keys to their owners)
enum PartDst : int { kDstTiles = 0, kDstParts = 1 };


struct PartGeom {
  uint32_t P;        // partition workgroups
  uint32_t n_tiles;
  uint32_t per;      // items per partition workgroup at most (overflow list capacity)
  uint32_t cap;      // records per (tile, workgroup) region
  uint32_t rb;       // record bytes, 12 or 16
  uint64_t counts_off;   // u32 [n_tiles][P]: records in each region
  uint64_t ovf_n_off;    // u32 [P]: entries in each workgroup's overflow list
  uint64_t regions_off;  // region (t, w) at regions_off + (t * P + w) * cap * rb
  uint64_t ovf_off;      // workgroup w's overflow list at ovf_off + w * per * 16
  uint64_t bytes;
};

// the workspace layout of a partition from its P, n_tiles, per, cap and rb (the multi-leaf
// launch recomputes it on the device from the same five numbers)
__host__ __device__ inline void part_layout(PartGeom& g)
{
  const uint64_t regions = (uint64_t)g.n_tiles * g.P;
  g.counts_off = 256;
  g.ovf_n_off = g.counts_off + 4 * regions;
  g.regions_off = (g.ovf_n_off + 4ull * g.P + 255) & ~255ull;
  g.ovf_off = g.regions_off + (uint64_t)g.rb * regions * g.cap;
  g.bytes = g.ovf_off + 16ull * g.P * g.per;
}

// n_max: items the build may receive (the overflow lists' capacity); n_exp: the expected
// count (the regions' capacity; equal to n_max unless the count is only known on the device);
// wg_items: items per workgroup aimed at (the workgroups: at most one per CU)
inline PartGeom part_geom(uint64_t n_max, uint64_t n_exp, uint32_t n_tiles, uint32_t rb,
                          uint64_t wg_items = 32ull * kPartThreads)
{
  PartGeom g;
  g.n_tiles = n_tiles ? n_tiles : 1;
  g.rb = rb;
  const uint64_t p = (n_exp + wg_items - 1) / wg_items;
  g.P = (uint32_t)(p < 1 ? 1 : (p > kPartMaxWgs ? kPartMaxWgs : p));
  g.per = (uint32_t)((n_max + g.P - 1) / g.P);
  const double e = (double)((n_exp + g.P - 1) / g.P) / g.n_tiles;
  g.cap = ((uint32_t)(e + 6.0 * sqrt(e) + 16.0) + 15) & ~15u;
  part_layout(g);
  return g;
}

__device__ inline uint32_t bloom_tile_of(const uint4& kv, uint32_t nb)
{
  const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
  const uint64_t h0 = x.finish(c_bloom.rhinit16[0]);
  return (uint32_t)__umul64hi(h0, (uint64_t)nb) >> kTileShift;
}

// 24-byte keys (TurtleKV's default key size, 8-byte aligned) where the hash-once paths take
// them: the partition of a monolithic filter and the hash-range route's count and record
// passes.  (16-byte keys stay uint4.)
struct Key24 {
  uint64_t w[3];
};

__device__ inline Key24 load_key24(const uint8_t* keys, uint32_t i)
{
  const uint64_t* p = reinterpret_cast<const uint64_t*>(keys) + 3ull * i;
  return Key24{{__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                __builtin_nontemporal_load(p + 2)}};
}

__device__ inline uint32_t bloom_tile_of(const Key24& kv, uint32_t nb)
{
  const XxhFixed<24> x(kv.w);
  const uint64_t h0 = x.finish(xxh_fixed_rc<24>(c_bloom.seed[0]));
  return (uint32_t)__umul64hi(h0, (uint64_t)nb) >> kTileShift;
}

// key i of a 16- or 24-byte key array
template <int KB>
__device__ inline auto load_rec_key(const uint8_t* keys, uint32_t i)
{
  if constexpr (KB == 24) return load_key24(keys, i);
  else return load_nt16(keys + 16ull * i);
}

__device__ inline void rec_pack(uint32_t blk, uint32_t tile, const uint32_t (&b)[8], uint32_t& w0,
                                uint32_t& w1, uint32_t& w2)
{
  w0 = blk | b[0] << 11 | b[1] << 20 | (tile & 7u) << 29;
  w1 = b[2] | b[3] << 9 | b[4] << 18 | ((tile >> 3) & 31u) << 27;
  w2 = b[5] | b[6] << 9 | b[7] << 18 | ((tile >> 8) & 31u) << 27;
}

__device__ inline uint32_t rec_tile(uint32_t w0, uint32_t w1, uint32_t w2)
{
  return (w0 >> 29) | ((w1 >> 27) << 3) | ((w2 >> 27) << 8);
}

// a 16-byte key's block in the filter and its k <= 8 bit indices (b_j = b_0 for j >= k)
template <int K>
__device__ inline uint32_t rec_hash_bits(const uint4& kv, uint32_t nb, uint32_t k, uint32_t (&b)[8])
{
  const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
  const uint64_t h0 = x.finish(c_bloom.rhinit16[0]);
  b[0] = (uint32_t)h0 & 511u;
#pragma unroll
  for (uint32_t j = 1; j < 8; ++j) {
    if (K != 0 ? j < (uint32_t)K : j < k) b[j] = x.finish_lo9(c_bloom.rhinit16[j]) & 511u;
    else b[j] = b[0];
  }
  return (uint32_t)__umul64hi(h0, (uint64_t)nb);
}

// a 24-byte key's block and its bit indices (k > 8: the first eight; bloom_overflow sets the
// others)
template <int K>
__device__ inline uint32_t rec_hash_bits(const Key24& kv, uint32_t nb, uint32_t k, uint32_t (&b)[8])
{
  const XxhFixed<24> x(kv.w);
  const uint64_t h0 = x.finish(xxh_fixed_rc<24>(c_bloom.seed[0]));
  b[0] = (uint32_t)h0 & 511u;
#pragma unroll
  for (uint32_t j = 1; j < 8; ++j) {
    if (K != 0 ? j < (uint32_t)K : j < k) b[j] = x.finish_lo9(xxh_fixed_rc<24>(c_bloom.seed[j])) & 511u;
    else b[j] = b[0];
  }
  return (uint32_t)__umul64hi(h0, (uint64_t)nb);
}

// a key of any other shape (bloom_any_records): its bytes and length
struct KeyRef {
  const uint8_t* p;
  uint32_t len;
};

// its block and bit indices (k <= 8): under 32 bytes the seed-independent lane rounds are
// shared by the k hashes (XxhShort), longer keys hash from scratch per seed
__device__ inline uint32_t rec_hash_bits_any(const KeyRef& kr, uint32_t nb, uint32_t k, uint32_t (&b)[8])
{
  uint64_t h0;
  if (kr.len < 32) {
    const XxhShort x(kr.p, kr.len);
    h0 = x.finish(c_bloom.seed_p5[0]);
    b[0] = (uint32_t)h0 & 511u;
#pragma unroll
    for (uint32_t j = 1; j < 8; ++j) b[j] = j < k ? x.finish_lo9(c_bloom.seed_p5[j]) & 511u : b[0];
  } else {
    h0 = xxh64_bytes(kr.p, kr.len, c_bloom.seed[0]);
    b[0] = (uint32_t)h0 & 511u;
    for (uint32_t j = 1; j < 8; ++j) b[j] = j < k ? (uint32_t)xxh64_bytes(kr.p, kr.len, c_bloom.seed[j]) & 511u : b[0];
  }
  return (uint32_t)__umul64hi(h0, (uint64_t)nb);
}

// ---------------------------------------------------------------------------------------
// The route (hash-range sharding, and the parts of a filter beyond kDirectMaxTiles): part p
// of n_parts owns tiles [p*q, (p+1)*q).  A count pass (h0 -> part, LDS histogram, one row of
// H[P][n_parts] per workgroup), two scans (each workgroup's offset in each part's run, the
// part bases), and a scatter pass over the same key ranges that writes each key -- or, with
// k <= 8, its 12-byte bit record with its tile relative to its part -- to its slot.
// ---------------------------------------------------------------------------------------
struct RouteGeom {
  uint32_t P;         // route workgroups
  uint32_t n_parts;
  uint32_t per;       // keys per route workgroup
  uint64_t h_words;   // P * n_parts
  uint64_t bytes;     // workspace bytes: [H][part totals][part bases (n_parts + 1)]
};

inline RouteGeom route_geom(uint64_t n_keys, uint32_t n_parts)
{
  RouteGeom g;
  g.n_parts = n_parts;
  const uint64_t p = (n_keys + 4095) / 4096;
  g.P = (uint32_t)(p < 1 ? 1 : (p > kRouteMaxWgs ? kRouteMaxWgs : p));
  g.per = (uint32_t)((n_keys + g.P - 1) / g.P);
  g.h_words = (uint64_t)g.P * n_parts;
  g.bytes = (4 * (g.h_words + 2ull * n_parts + 1) + 255) & ~255ull;
  return g;
}

// PASS 0: histogram of the parts; PASS 1: the keys themselves to their slots (16-byte keys;
// nothing when the filter's k < min_k: the monolithic build routes records up to k = 8).
// Both walk the same key ranges in the same way.
template <int PASS, uint32_t NT, int KB = 16>
__global__ __launch_bounds__(NT) void route_keys(const uint8_t* __restrict__ keys,
                                                 const tkv_amq_segment* __restrict__ segs,
                                                 uint32_t* __restrict__ ws, uint32_t n_parts,
                                                 uint32_t per, uint32_t n, uint32_t q,
                                                 uint4* __restrict__ out, uint32_t min_k)
{
  extern __shared__ uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  if (sg.hash_count < min_k) return;
  const uint32_t tid = threadIdx.x, w = blockIdx.x, nb = sg.n_blocks;
  uint32_t* H = ws + (uint64_t)w * n_parts;
  const uint32_t* base = ws + (uint64_t)gridDim.x * n_parts + n_parts;
  for (uint32_t t = tid; t < n_parts; t += NT) s_part[t] = PASS == 0 ? 0u : base[t] + H[t];
  __syncthreads();
  const uint32_t b = min(n, w * per), e = min(n, b + per);
  static_assert(KB == 16 || (KB == 24 && PASS == 0), "24-byte keys: the count pass only");
  constexpr int U = 4;
  for (uint32_t i0 = b; i0 < e; i0 += NT * U) {
    decltype(load_rec_key<KB>(keys, 0)) kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * NT + tid;
      if (i < e) kv[u] = load_rec_key<KB>(keys, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * NT + tid;
      if (i < e) {
        const uint32_t p = bloom_tile_of(kv[u], nb) / q;
        if (p >= n_parts) continue;
        if constexpr (PASS == 0) {
          atomicAdd(s_part + p, 1u);
        } else if constexpr (KB == 16) {
          out[atomicAdd(s_part + p, 1u)] = kv[u];
        }
      }
    }
  }
  if constexpr (PASS == 0) {
    __syncthreads();
    for (uint32_t t = tid; t < n_parts; t += NT) H[t] = s_part[t];
  }
}

// exclusive scan of 256 per-thread values in a 256-thread block; returns this thread's prefix
// and sets *total
__device__ inline uint32_t block_exclusive_scan256(uint32_t v, uint32_t* s, uint32_t* total)
{
  const uint32_t tid = threadIdx.x;
  s[tid] = v;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    const uint32_t a = tid >= d ? s[tid - d] : 0u;
    __syncthreads();
    s[tid] += a;
    __syncthreads();
  }
  *total = s[255];
  const uint32_t r = s[tid] - v;
  __syncthreads();
  return r;
}

// One workgroup per part: H[w][p] <- sum of H[w'][p] over w' < w; totals[p] <- column sum.
__global__ __launch_bounds__(256) void route_scan_cols(uint32_t* __restrict__ ws, uint32_t P,
                                                       uint32_t n_parts)
{
  __shared__ uint32_t s[256];
  const uint32_t t = blockIdx.x, tid = threadIdx.x;
  constexpr uint32_t R = kRouteMaxWgs / 256;  // rows per thread
  uint32_t v[R];
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t w = tid * R + r;
    v[r] = w < P ? ws[(uint64_t)w * n_parts + t] : 0u;
    sum += v[r];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan256(sum, s, &total);
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t w = tid * R + r;
    if (w < P) ws[(uint64_t)w * n_parts + t] = run;
    run += v[r];
  }
  if (tid == 0) ws[(uint64_t)P * n_parts + t] = total;
}

// One workgroup: bases[p] = sum of totals[p'] over p' < p, bases[n_parts] = key count.
__global__ __launch_bounds__(256) void route_scan_parts(uint32_t* __restrict__ ws, uint32_t P,
                                                        uint32_t n_parts)
{
  __shared__ uint32_t s[256];
  const uint32_t* tot = ws + (uint64_t)P * n_parts;
  uint32_t* base = ws + (uint64_t)P * n_parts + n_parts;
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (n_parts + 255) / 256;  // consecutive parts per thread
  const uint32_t t0 = min(n_parts, tid * per), t1 = min(n_parts, t0 + per);
  uint32_t sum = 0;
  for (uint32_t t = t0; t < t1; ++t) sum += tot[t];
  uint32_t total;
  uint32_t run = block_exclusive_scan256(sum, s, &total);
  for (uint32_t t = t0; t < t1; ++t) {
    base[t] = run;
    run += tot[t];
  }
  if (tid == 0) base[n_parts] = total;
}

// the route's record scatter pass (k <= 8): the same key ranges and slots as route_keys<1>
// (after the same count pass), each key leaving as its 12-byte bit record with its tile
// relative to its part's first tile
template <uint32_t NT, int K, int KB>
__device__ void route_recs_body(const uint8_t* __restrict__ keys, const tkv_amq_segment& sg,
                                uint32_t n_parts, uint32_t per, uint32_t n, uint32_t q,
                                uint32_t* __restrict__ out, uint32_t* s_part)
{
  const uint32_t tid = threadIdx.x, w = blockIdx.x, nb = sg.n_blocks, k = sg.hash_count;
  const uint32_t b = min(n, w * per), e = min(n, b + per);
  constexpr int U = 4;
  for (uint32_t i0 = b; i0 < e; i0 += NT * U) {
    decltype(load_rec_key<KB>(keys, 0)) kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * NT + tid;
      if (i < e) kv[u] = load_rec_key<KB>(keys, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * NT + tid;
      if (i >= e) continue;
      uint32_t bits[8], r0, r1, r2;
      const uint32_t blk = rec_hash_bits<K>(kv[u], nb, k, bits);
      const uint32_t tg = blk >> kTileShift;
      const uint32_t p = tg / q;
      if (p >= n_parts) continue;
      rec_pack(blk & (kTileBlocks - 1), tg - p * q, bits, r0, r1, r2);
      const uint32_t slot = atomicAdd(s_part + p, 1u);
      uint3 v;
      v.x = r0;
      v.y = r1;
      v.z = r2;
      reinterpret_cast<uint3*>(out)[slot] = v;
    }
  }
}

template <uint32_t NT, int KB>
__global__ __launch_bounds__(NT) void route_recs(const uint8_t* __restrict__ keys,
                                                 const tkv_amq_segment* __restrict__ segs,
                                                 uint32_t* __restrict__ ws, uint32_t n_parts,
                                                 uint32_t per, uint32_t n, uint32_t q,
                                                 uint32_t* __restrict__ out)
{
  extern __shared__ uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  const uint32_t tid = threadIdx.x, w = blockIdx.x;
  const uint32_t* H = ws + (uint64_t)w * n_parts;
  const uint32_t* base = ws + (uint64_t)gridDim.x * n_parts + n_parts;
  for (uint32_t t = tid; t < n_parts; t += NT) s_part[t] = base[t] + H[t];
  __syncthreads();
  const uint32_t k = sg.hash_count;
  if (k == 0 || k > 8) return;  // (the ABI refuses k > 8: a record holds 8 bit indices)
  if (k == 7) route_recs_body<NT, 7, KB>(keys, sg, n_parts, per, n, q, out, s_part);
  else if (k == 8) route_recs_body<NT, 8, KB>(keys, sg, n_parts, per, n, q, out, s_part);
  else route_recs_body<NT, 0, KB>(keys, sg, n_parts, per, n, q, out, s_part);
}

// ---------------------------------------------------------------------------------------
// partition, tile build, overflow
// ---------------------------------------------------------------------------------------
// The route's output (bloom_route_part) and a part build's input (kSrcSeg12): fixed-size
// PART blocks, one per (route chunk, sender, part).  Block layout:
//   counts_off   u32 [P]: records in region w (<= cap)
//   ovf_n_off    u32: overflow entries appended to the block (> ovf_cap: entries were lost)
//   regions_off  region w at regions_off + w * cap * 12: route workgroup w's 12-byte records of
//                the part, in its batches' order (no atomics: each workgroup owns its region)
//   ovf_off      ovf_cap 16-byte entries (record, global part): records whose region was full
// Part p belongs to rank p % world as its part jl = p / world (round-robin: round jl's parts of
// all ranks are one contiguous byte range of the bitmap, all-gathered in place).  The route
// writes part p's block at dst + jl * jstride + (p % world) * bytes: with jstride = world *
// bytes a chunk's send buffer holds the parts in global order, so round jl's blocks (one per
// destination) are one contiguous slice -- one all-to-all of equal splits per (chunk, round),
// no host synchronisation to size it, and a part can be built as soon as its round has landed.
struct RouteBlock {
  uint64_t bytes;
  uint64_t jstride;         // the route's destination: bytes from round jl to jl + 1
  uint64_t counts_off;
  uint64_t ovf_n_off;
  uint64_t regions_off;
  uint64_t ovf_off;
  uint32_t P;               // route workgroups (= the part builds' partition workgroups)
  uint32_t cap;             // records per region
  uint32_t ovf_cap;         // overflow entries per block
  uint32_t pad;
};

struct PartArgs {
  const uint8_t* src;  // keys (16 or 24 bytes), routed 12-byte records, or routed 16-byte keys;
                       // kSrcSeg12: the first route block of the part's inputs
  uint32_t n;          // items [0, n) of src (from_seg: the segment's keys, n capped by it)
  uint32_t tile0;      // global tile of local tile 0
  uint32_t from_seg;
  uint32_t kb;         // key bytes of hashed keys, 16 or 24 (24 with k > 8: the first eight bits
                       // in the records, the others set by bloom_overflow from the keys)
  const uint32_t* cnt; // routed parts built on the device: items = cnt[part] at the offset
  uint32_t part;       // sum(cnt[0..part)) of src (n and from_seg unused)
  uint8_t* ws;
  PartGeom g;
  uint32_t src_kind;   // PartSrc of the partition (kSrcRec12: routed items), for bloom_overflow
  // kDstParts: the route blocks (one per destination rank), tiles per part, ranks, and the
  // multiply-high reciprocals of q and world (x / q = (x * q_magic) >> 32 for x < 2^21)
  uint8_t* dst;
  uint32_t q;
  uint32_t world;
  uint64_t q_magic;
  uint64_t w_magic;
  RouteBlock blk;
  // kSrcSeg12: the part blocks holding this part (n_src_segs of them, blk.bytes apart)
  uint32_t n_src_segs;
  uint32_t seg_part;  // (unused)
  // a partition (kDstTiles) with the per-tile store table: part_tbl_fits(n_tiles), and the
  // launch's LDS is part_tbl_lds_bytes
  uint32_t tbl;
  // the build's first workgroup in its grid (0 but in a multi-leaf launch, whose grid holds the
  // workgroups of several builds back to back)
  uint32_t wg0;
  // a filter of few tiles: each tile's regions split over `split` tile workgroups (> 1), each
  // writing a partial image at part_img + (t * split + s) * 128 KiB, ORed by bloom_tile_merge
  uint32_t split;
  uint8_t* part_img;
};

__host__ __device__ inline uint64_t div_magic(uint32_t d) { return (0x100000000ull / d) + 1; }
static_assert(sizeof(tkv_amq_route_plan) == 120, "abi.RoutePlan");
__device__ inline uint32_t div_by_magic(uint32_t x, uint64_t m) { return (uint32_t)(((uint64_t)x * m) >> 32); }

// (nontemporal, as the tile kernel's record loads: the records are read once)
typedef uint32_t u32x3_nt_t __attribute__((ext_vector_type(3)));
__device__ inline uint4 load_rec12(const uint8_t* recs, uint32_t i)
{
  const u32x3_nt_t r = __builtin_nontemporal_load(reinterpret_cast<const u32x3_nt_t*>(recs + 12ull * i));
  return make_uint4(r.x, r.y, r.z, 0u);
}

// items [b, e) of the build's source and its base pointer (SRC: item bytes)
__device__ inline void part_items(const tkv_amq_segment& sg, const PartArgs& a, uint32_t item_bytes,
                                  const uint8_t*& src, uint32_t& n)
{
  if (a.cnt) {
    uint64_t off = 0;
    for (uint32_t p = 0; p < a.part; ++p) off += a.cnt[p];
    n = a.cnt[a.part];
    src = a.src + (uint64_t)item_bytes * off;
  } else {
    n = a.from_seg ? min(a.n, sg.n_keys) : a.n;
    src = a.src + (uint64_t)item_bytes * (a.from_seg ? sg.key_begin : 0);
  }
}

// Per-batch tile bookkeeping of part_body over the tiles' packed u16 counters (word j holds
// tiles 2j and 2j+1; thread i owns words [i*c, (i+1)*c)): cursor[t] += prev[t] (the previous
// batch's run lengths), prev[t] = 0 (the next batch's histogram), start[t] = exclusive scan of
// cur[t].  Returns the batch's record count.  Two LDS barriers inside.
__device__ inline uint32_t part_scan(const uint32_t* cur, uint32_t* prev, uint32_t* start,
                                     uint32_t* cursor, uint32_t HW, uint32_t* wsum)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t c = (HW + kPartThreads - 1) / kPartThreads;
  // only the waves holding counter words scan (one for the route's parts, eight for a
  // 954-tile partition); the others skip to the barriers
  const uint32_t nwa = ((HW + c - 1) / c + 63) / 64;
  const uint32_t j0 = min(HW, tid * c), j1 = min(HW, j0 + c);
  uint32_t s = 0, inc = 0;
  if (wave < nwa) {
    for (uint32_t j = j0; j < j1; ++j) {
      const uint32_t x = cur[j], y = prev[j];
      if (y) {
        cursor[2 * j] += y & 0xffffu;
        cursor[2 * j + 1] += y >> 16;
        prev[j] = 0;
      }
      s += (x & 0xffffu) + (x >> 16);
    }
    inc = s;  // inclusive scan over the wave
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
  }
  lds_barrier();
  uint32_t before = 0, total = 0;
  for (uint32_t q = 0; q < nwa; ++q) {
    const uint32_t t = wsum[q];
    before += q < wave ? t : 0u;
    total += t;
  }
  if (wave < nwa) {
    uint32_t run = before + inc - s;
    for (uint32_t j = j0; j < j1; ++j) {
      const uint32_t x = cur[j], lo = x & 0xffffu;
      start[j] = run | (run + lo) << 16;
      run += lo + (x >> 16);
    }
  }
  lds_barrier();  // start / cursor complete; wsum is reused by the next call
  return total;
}

__device__ inline uint32_t lds_u16(const uint32_t* words, uint32_t t)
{
  return (words[t >> 1] >> ((t & 1u) << 4)) & 0xffffu;
}

// Per batch: hash U items per thread into records, each ranked in its bucket's run (its tile;
// DST == kDstParts: its part) by a returning ds_add on the packed histogram (the next batch's
// items are then loaded, in flight until its hash); LDS barrier; scan (two barriers); every
// record placed at its sorted position in the LDS planes; LDS barrier; the planes written out
// in order, each bucket's run to the end of this workgroup's region of that bucket, so a
// store instruction covers a few long runs (the L2 merges them into whole lines) instead of
// 64 scattered records.  Every lane issues the same loads and stores per batch (clamped loads;
// lanes without a record store to a sink in the workspace header).  Overflow entries are the
// records themselves (their tile is in the record: T <= kDirectMaxTiles < 2^13), RAW the
// 16-byte keys, kDstParts the record and its part (16 bytes).
template <int K, int SRC, int DST = kDstTiles, bool TBL = DST == kDstParts>
__device__ void part_body(const tkv_amq_segment& sg, const PartArgs& a, uint32_t* lds)
{
  constexpr bool RAW = SRC == kSrcRaw16;
  constexpr bool ROUTE = DST == kDstParts;
  static_assert(TBL || !ROUTE, "the route stores through its table");
  constexpr bool ROUTED = SRC == kSrcRec12 || SRC == kSrcSeg12;  // records with their tile in part
  static_assert(!(ROUTE && (RAW || ROUTED)), "the route hashes keys");
  // 16-byte records: four key words and the tile per item in LDS, half the items per batch
  constexpr uint32_t RB = RAW ? 16 : 12, U = RAW ? kPartU / 2 : kPartU, NT = kPartThreads, B = U * NT;
  constexpr uint32_t NPL = RAW ? 5 : 3;  // LDS planes (ROUTE: + a u16 plane of parts)
  static_assert(NPL * B * 4 <= kPartPlaneBytes, "planes");
  constexpr uint32_t IB = SRC == kSrcKey24 ? 24 : (ROUTED ? 12 : 16);  // item bytes
  const uint32_t tid = threadIdx.x, w = blockIdx.x - a.wg0, P = a.g.P, T = a.g.n_tiles, cap = a.g.cap;
  const uint32_t nb = sg.n_blocks, k = sg.hash_count;
  const uint32_t HW = (T + 1) >> 1;
  uint32_t* pl = lds;  // plane j at pl + j * B
  uint16_t* plp = reinterpret_cast<uint16_t*>(lds + kPartPlaneBytes / 4);  // ROUTE: parts
  uint32_t* H0 = lds + (kPartPlaneBytes + (ROUTE ? 2 * B : 0)) / 4;
  uint32_t* H1 = H0 + HW;
  uint32_t* start = H1 + HW;
  uint32_t* cursor = start + HW;
  uint32_t* wsum = cursor + 2 * HW;  // 16 wave sums
  uint32_t* ovf_n = wsum + NT / 64;
  uint32_t* pre = ovf_n + 1;         // kSrcSeg12: the item prefix over the source blocks
  // TBL: per bucket, for the batch in the planes: where its run's record j goes (the region
  // base + roff + RB j) and the first j past its region (rlim), so a record's store address is
  // one table read (the route always; a partition whose tiles leave room: part_tbl_fits).
  // (index arithmetic on lds, not an integer round trip: the pointer must stay an LDS pointer)
  uint64_t* roff = reinterpret_cast<uint64_t*>(
      lds + ((uint32_t)(ovf_n - lds) + (ROUTE ? 0u : kMaxSrcSegs + 2u) + 2u & ~1u));
  int32_t* rlim = reinterpret_cast<int32_t*>(roff + T);
  uint8_t* const rbase = ROUTE ? a.dst : a.ws;  // what roff is relative to
  for (uint32_t i = tid; i < 2 * HW; i += NT) {
    H0[i] = 0;  // (H0 and H1)
    cursor[i] = 0;
  }
  if (tid == 0) *ovf_n = 0;
  if constexpr (ROUTE) {
    // the part blocks' overflow counters, appended to by bloom_route_ovf_pack after this
    // kernel (a later launch on the same stream)
    if (w == 0)
      for (uint32_t t = tid; t < T; t += NT) {
        const uint32_t jl = div_by_magic(t, a.w_magic), dr = t - jl * a.world;
        *reinterpret_cast<uint32_t*>(a.dst + (uint64_t)jl * a.blk.jstride + (uint64_t)dr * a.blk.bytes +
                                     a.blk.ovf_n_off) = 0;
      }
  }
  const uint8_t* src;
  uint32_t n;
  uint64_t seg_reg = 0;  // kSrcSeg12: this workgroup's region inside a part block
  if constexpr (SRC == kSrcSeg12) {
    const uint32_t S = a.n_src_segs;
    seg_reg = a.blk.regions_off + (uint64_t)w * a.blk.cap * 12ull;
    const uint64_t cnt_off = a.blk.counts_off + 4ull * w;
    if (tid < 64) {  // one wave: the inclusive scan of the S counts, 64 at a time
      uint32_t run = 0;
      for (uint32_t s0 = 0; s0 < S; s0 += 64) {
        const uint32_t sidx = s0 + tid;
        uint32_t c = sidx < S ? *reinterpret_cast<const uint32_t*>(a.src + (uint64_t)sidx * a.blk.bytes + cnt_off) : 0u;
        c = min(c, a.blk.cap);
        uint32_t inc = c;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
          const uint32_t v = __shfl_up(inc, d, 64);
          if (tid >= d) inc += v;
        }
        if (sidx < S) pre[sidx + 1] = run + inc;
        run += __shfl(inc, 63, 64);
      }
      if (tid == 0) pre[0] = 0;
    }
  }
  __syncthreads();
  uint32_t kb, ke;
  if constexpr (SRC == kSrcSeg12) {
    src = a.src;
    n = pre[a.n_src_segs];
    kb = 0;  // this workgroup's own regions, whole
    ke = n;
  } else {
    part_items(sg, a, IB, src, n);
    const uint32_t per = a.cnt ? (n + P - 1) / P : a.g.per;
    kb = min(n, w * per);
    ke = min(n, kb + per);
  }
  const uint64_t ovf_base = a.g.ovf_off + (uint64_t)w * a.g.per * 16;  // (lists 16 B per item apart)
  const uint32_t last_item = ke > 0 ? ke - 1 : 0;
  uint32_t cs = 0;  // kSrcSeg12: the block of this thread's last item (items rise per thread)
  using In = typename std::conditional<SRC == kSrcKey24, Key24, uint4>::type;
  auto load_in = [&](uint32_t i) -> In {
    if constexpr (SRC == kSrcSeg12) {
      while (i >= pre[cs + 1]) ++cs;
      return load_rec12(src + (uint64_t)cs * a.blk.bytes + seg_reg, i - pre[cs]);
    } else if constexpr (SRC == kSrcRec12) {
      return load_rec12(src, i);
    } else if constexpr (SRC == kSrcKey24) {
      return load_key24(src, i);
    } else {
      return load_nt16(src + 16ull * i);
    }
  };
  In in[U];
  // the store phase: the previous batch's sorted records (LDS planes) to the regions
  uint32_t total = 0;  // records in the planes
  auto write_out = [&]() {
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t j0 = u * NT + tid;
      const bool v = j0 < total;
      const uint32_t j = v ? j0 : 0u;
      const uint32_t x0 = pl[j], x1 = pl[B + j], x2 = pl[2 * B + j];
      uint32_t x3 = 0, t;
      if constexpr (RAW) {
        x3 = pl[3 * B + j];
        t = pl[4 * B + j];
      } else if constexpr (ROUTE) {
        t = plp[j];
      } else {
        t = rec_tile(x0, x1, x2);
      }
      t = v ? t : 0u;
      uint8_t* d = a.ws;  // the sink
      bool ovf = false;
      if (v) {
        bool in_region;
        if constexpr (TBL) {
          in_region = (int32_t)j < rlim[t];
        } else {
          const uint32_t c = cursor[t] + (j - lds_u16(start, t));
          in_region = c < cap;
          d = a.ws + a.g.regions_off + ((uint64_t)t * P + w) * cap * a.g.rb + (uint64_t)c * RB;
        }
        if (in_region) {
          // (relative to a kernel-argument pointer, so the store stays a global store, not a
          // flat one; the asm keeps the compiler from hoisting base + RB j for every u into
          // spilled registers)
          if constexpr (TBL) {
            uint32_t jj = j;
            asm volatile("" : "+v"(jj));
            d = rbase + (roff[t] + RB * jj);
          }
        } else {
          ovf = true;  // LDS atomic: this workgroup's list
          d = a.ws + ovf_base + (uint64_t)(ROUTE ? 16 : RB) * atomicAdd(ovf_n, 1u);
        }
      }
      uint32_t* dw = reinterpret_cast<uint32_t*>(d);
      if constexpr (RAW) {
        *reinterpret_cast<uint4*>(dw) = make_uint4(x0, x1, x2, x3);
      } else {
        dw[0] = x0;
        dw[1] = x1;
        dw[2] = x2;
        if constexpr (ROUTE)
          if (ovf) dw[3] = t;
      }
    }
  };
  if (ke > kb) {  // (no items: src may be null)
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) in[u] = load_in(min(kb + u * NT + tid, last_item));
  }
  uint32_t par = 0;
  // Per iteration: hash batch b; write out batch b - 1 (its stores then drain while this
  // batch is scanned and sorted: the compiler waits for every outstanding load and store
  // before the next hash, vmcnt(0), since loads and stores share the counter); load batch
  // b + 1; LDS barrier; scan; place batch b in the planes; LDS barrier.
  for (uint32_t b0 = kb; b0 < ke; b0 += B, par ^= 1) {
    uint32_t* hist = par ? H1 : H0;
    uint32_t* prev = par ? H0 : H1;
    // per item: its record and (bucket << 16 | rank in the bucket's run), ~0: no record
    uint32_t r0[U], r1[U], r2[U], r3[RAW ? U : 1], tr[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = b0 + u * NT + tid;
      // (under a branch: the hashes of the U items are not interleaved by the scheduler,
      // whose register demand would then spill)
      uint32_t t = ~0u;
      if (i < ke) {
        if constexpr (RAW) {
          t = bloom_tile_of(in[u], nb) - a.tile0;  // wraps below the window
          r0[u] = in[u].x;
          r1[u] = in[u].y;
          r2[u] = in[u].z;
          r3[u] = in[u].w;
        } else if constexpr (ROUTED) {
          r0[u] = in[u].x;
          r1[u] = in[u].y;
          r2[u] = in[u].z;
          t = rec_tile(r0[u], r1[u], r2[u]);
        } else {
          uint32_t bits[8];
          const uint32_t blk = rec_hash_bits<K>(in[u], nb, k, bits);
          const uint32_t tg = blk >> kTileShift;
          if constexpr (ROUTE) {
            t = div_by_magic(tg, a.q_magic);  // the key's part; its record's tile is in the part
            rec_pack(blk & (kTileBlocks - 1), tg - t * a.q, bits, r0[u], r1[u], r2[u]);
          } else {
            t = tg - a.tile0;
            rec_pack(blk & (kTileBlocks - 1), t, bits, r0[u], r1[u], r2[u]);
          }
        }
      }
      if (t >= T) {
        tr[u] = ~0u;
      } else {
        const uint32_t sh = (t & 1u) << 4;
        const uint32_t rank = (atomicAdd(hist + (t >> 1), 1u << sh) >> sh) & 0xffffu;
        tr[u] = t << 16 | rank;
      }
    }
    write_out();  // batch b - 1 (total = 0 before the first batch: sink stores only)
#pragma unroll
    for (uint32_t u = 0; u < U; ++u)  // the next batch's items
      in[u] = load_in(min(b0 + B + u * NT + tid, last_item));
    lds_barrier();
    total = part_scan(hist, prev, start, cursor, HW, wsum);
    if constexpr (TBL) {
      // this batch's store table (read by its write-out, after the barrier below)
      for (uint32_t t = tid; t < T; t += NT) {
        const uint32_t st = lds_u16(start, t), cu = cursor[t];
        uint64_t base;
        if constexpr (ROUTE) {
          const uint32_t jl = div_by_magic(t, a.w_magic), dr = t - jl * a.world;
          base = (uint64_t)jl * a.blk.jstride + (uint64_t)dr * a.blk.bytes + a.blk.regions_off +
                 (uint64_t)w * cap * 12ull;
        } else {
          base = a.g.regions_off + ((uint64_t)t * P + w) * cap * a.g.rb;
        }
        roff[t] = base + (uint64_t)RB * cu - (uint64_t)RB * st;
        rlim[t] = (int32_t)(cap + st) - (int32_t)cu;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if (tr[u] == ~0u) continue;
      const uint32_t t = tr[u] >> 16;
      const uint32_t pos = lds_u16(start, t) + (tr[u] & 0xffffu);
      pl[pos] = r0[u];
      pl[B + pos] = r1[u];
      pl[2 * B + pos] = r2[u];
      if constexpr (RAW) {
        pl[3 * B + pos] = r3[u];
        pl[4 * B + pos] = t;
      }
      if constexpr (ROUTE) plp[pos] = (uint16_t)t;
    }
    lds_barrier();
  }
  write_out();  // the last batch
  __syncthreads();
  // the last batch's run lengths (its histogram is the one the loop's last batch counted into)
  const uint32_t* last = par ? H0 : H1;
  if constexpr (ROUTE) {
    for (uint32_t t = tid; t < T; t += NT) {
      const uint32_t jl = div_by_magic(t, a.w_magic), dr = t - jl * a.world;
      *reinterpret_cast<uint32_t*>(a.dst + (uint64_t)jl * a.blk.jstride + (uint64_t)dr * a.blk.bytes +
                                   a.blk.counts_off + 4ull * w) = min(cursor[t] + lds_u16(last, t), cap);
    }
  } else {
    uint32_t* counts = reinterpret_cast<uint32_t*>(a.ws + a.g.counts_off);
    for (uint32_t t = tid; t < T; t += NT)
      counts[(uint64_t)t * P + w] = min(cursor[t] + lds_u16(last, t), cap);
  }
  if (tid == 0) reinterpret_cast<uint32_t*>(a.ws + a.g.ovf_n_off)[w] = *ovf_n;
}

// 16-byte keys: bit records for k <= 8, the keys themselves above
__device__ __attribute__((always_inline)) inline void part_keys16(const tkv_amq_segment& sg, const PartArgs& a, uint32_t* s_part)
{
  const uint32_t k = sg.hash_count;
  if (k == 0) return;
  if (k == 7 && a.tbl) part_body<7, kSrcKey16, kDstTiles, true>(sg, a, s_part);
  else if (k == 7) part_body<7, kSrcKey16>(sg, a, s_part);
  else if (k == 8 && a.tbl) part_body<8, kSrcKey16, kDstTiles, true>(sg, a, s_part);
  else if (k == 8) part_body<8, kSrcKey16>(sg, a, s_part);
  else if (k < 8) part_body<0, kSrcKey16>(sg, a, s_part);
  else part_body<0, kSrcRaw16>(sg, a, s_part);
}

__global__ __launch_bounds__(kPartThreads) void bloom_part_keys16(const tkv_amq_segment* __restrict__ segs,
                                                                  PartArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  part_keys16(sg, a, s_part);
}

// 24-byte keys (a kernel of its own: their six key words per prefetched key would raise the
// 16-byte kernel's register count): always bit records (k > 8: the first eight bits)
__device__ __attribute__((always_inline)) inline void part_keys24(const tkv_amq_segment& sg, const PartArgs& a, uint32_t* s_part)
{
  const uint32_t k = sg.hash_count;
  if (k == 0) return;
  // (the store-table variant: 62.0 vs 61.8 Gkeys/s, bloom10monok24, profiles/r05/k24tbl/ -- not kept)
  if (k == 7) part_body<7, kSrcKey24>(sg, a, s_part);
  else if (k == 8) part_body<8, kSrcKey24>(sg, a, s_part);
  else part_body<0, kSrcKey24>(sg, a, s_part);
}

__global__ __launch_bounds__(kPartThreads) void bloom_part_keys24(const tkv_amq_segment* __restrict__ segs,
                                                                  PartArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  part_keys24(sg, a, s_part);
}

// routed items: 12-byte bit records for k <= 8, 16-byte keys above (tkv_amq_bloom_route)
__global__ __launch_bounds__(kPartThreads) void bloom_part_routed(const tkv_amq_segment* __restrict__ segs,
                                                                  PartArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  const uint32_t k = sg.hash_count;
  if (k == 0) return;
  if (k <= 8) part_body<0, kSrcRec12>(sg, a, s_part);
  else part_body<0, kSrcRaw16>(sg, a, s_part);
}

// Keys of any other shape (variable-length through offsets, or a fixed stride; k <= 8) for the
// tiled build: one thread per key hashes it into its 12-byte bit record, the tile in the
// record's tile field (the filter has <= kDirectMaxTiles tiles), and the partition then sorts
// the records (kSrcRec12) as it sorts routed ones.  A pass of its own, at full occupancy, hides
// the latency of the keys' scattered byte loads, which the partition's batch loop could not
// (round 6: hashing them inside the partition ran at 97.5 us for 3M variable-length keys).
// (Round 5: such a leaf past the window path set its bits with device atomics, 3.6 Gkeys/s.)
template <int MODE>
__global__ __launch_bounds__(256) void bloom_any_records(const uint8_t* __restrict__ keys,
                                                         const uint64_t* __restrict__ offs, uint32_t stride,
                                                         const tkv_amq_segment* __restrict__ segs, uint32_t n,
                                                         uint32_t* __restrict__ recs)
{
  const tkv_amq_segment sg = segs[0];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t k = sg.hash_count;
  if (i >= n || i >= sg.n_keys || k == 0 || k > 8) return;
  // the leaf's bytes through a buffer resource: a key under 32 bytes as one 32-byte window
  // (two 16-byte loads; KeyWin, as the VQF producers read them) instead of its lanes, tail
  // word and tail bytes one load each
  const uint64_t n_all = min(n, sg.n_keys);
  const uint64_t b0 = MODE == kKeyVar ? offs[sg.key_begin] : sg.key_begin * stride;
  const uint64_t b1 = MODE == kKeyVar ? offs[sg.key_begin + n_all] : (sg.key_begin + n_all) * stride;
  const VarRsrc vr = var_rsrc(keys, b0, b1, b1);
  uint32_t len;
  const uint8_t* p = key_at<MODE>(keys, offs, stride, sg.key_begin + i, len);
  uint32_t bits[8], r0, r1, r2;
  uint32_t blk;
  if (len < 32 && vr.nrec) {
    KeyWin kw;
    key_win_load(vr, (uint32_t)(p - keys - vr.base), kw);
    uint64_t l[3];
    uint32_t t4, tb;
    key_win_parts(kw, len, l, t4, tb);
    const XxhShort x(len, l, t4, tb);
    const uint64_t h0 = x.finish(c_bloom.seed_p5[0]);
    bits[0] = (uint32_t)h0 & 511u;
#pragma unroll
    for (uint32_t j = 1; j < 8; ++j) bits[j] = j < k ? x.finish_lo9(c_bloom.seed_p5[j]) & 511u : bits[0];
    blk = (uint32_t)__umul64hi(h0, (uint64_t)sg.n_blocks);
  } else {
    blk = rec_hash_bits_any(KeyRef{p, len}, sg.n_blocks, k, bits);
  }
  rec_pack(blk & (kTileBlocks - 1), blk >> kTileShift, bits, r0, r1, r2);
  uint3 v;
  v.x = r0;
  v.y = r1;
  v.z = r2;
  reinterpret_cast<uint3*>(recs)[i] = v;
}

// The one-pass route (k <= 8): every key hashed once into its 12-byte bit record, counting-
// sorted by part in LDS and appended to this workgroup's region of the part in the part's
// destination block (part p -> rank p % world), whole runs per store; records beyond a region's
// capacity go to this workgroup's overflow list as (record, part).  No count pass: the regions
// have a fixed capacity.
// (one 1024-thread workgroup per CU -- its LDS -- so four waves per SIMD: the compiler may take
// 128 VGPRs instead of assuming two workgroups per CU and spilling at 64).  One kernel per
// (k, key bytes) variant, chosen on the host, so each gets its own register allocation.
template <int K, int KB>
__global__ __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void bloom_route_part(
    const tkv_amq_segment* __restrict__ segs, PartArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  const uint32_t k = sg.hash_count;
  if (k == 0 || k > 8 || (K != 0 && k != (uint32_t)K)) return;  // (the host passes the plan's k)
  part_body<K, KB == 24 ? kSrcKey24 : kSrcKey16, kDstParts>(sg, a, s_part);
}

// a part's partition from the route blocks that hold it (kSrcSeg12): workgroup w reads region
// (jl, w) of every block, back to back
__global__ __launch_bounds__(kPartThreads) void bloom_part_segs(const tkv_amq_segment* __restrict__ segs,
                                                                PartArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const tkv_amq_segment sg = segs[0];
  if (sg.hash_count == 0 || sg.hash_count > 8) return;
  if (a.tbl) part_body<0, kSrcSeg12, kDstTiles, true>(sg, a, s_part);
  else part_body<0, kSrcSeg12>(sg, a, s_part);
}

// Route overflow entries (record, part) of each route workgroup's list into the destination
// blocks' fixed-capacity overflow areas; a block's counter past ovf_cap records the loss (the
// caller then rebuilds through the exact exchange).  Empty lists: one count read per workgroup.
__global__ __launch_bounds__(256) void bloom_route_ovf_pack(PartArgs a)
{
  const uint32_t w = blockIdx.x;
  const uint32_t n = reinterpret_cast<const uint32_t*>(a.ws + a.g.ovf_n_off)[w];
  const uint4* list = reinterpret_cast<const uint4*>(a.ws + a.g.ovf_off + (uint64_t)w * a.g.per * 16);
  for (uint32_t e = threadIdx.x; e < n; e += 256) {
    const uint4 x = list[e];
    const uint32_t jl = div_by_magic(x.w, a.w_magic), dr = x.w - jl * a.world;
    uint8_t* b = a.dst + (uint64_t)jl * a.blk.jstride + (uint64_t)dr * a.blk.bytes;
    const uint32_t slot = atomicAdd(reinterpret_cast<uint32_t*>(b + a.blk.ovf_n_off), 1u);
    if (slot < a.blk.ovf_cap) reinterpret_cast<uint4*>(b + a.blk.ovf_off)[slot] = x;
  }
}

// Overflow entries (record, part) into the finished filter with device-scope atomicOr, for the
// parts [p0, p1) (after their bloom_tile): n_lists lists, list l's count at cnt + l * cnt_stride
// (at most cap entries used), its entries at ent + l * ent_stride.  Per-workgroup route lists
// (one GPU) and received blocks' overflow areas (hash-range shards) alike.
__global__ __launch_bounds__(256) void bloom_route_ovf_apply(const tkv_amq_segment* __restrict__ segs,
                                                             const uint8_t* cnt, uint64_t cnt_stride,
                                                             const uint8_t* ent, uint64_t ent_stride,
                                                             uint32_t cap, uint32_t q, uint32_t p0, uint32_t p1,
                                                             uint8_t* __restrict__ out)
{
  const tkv_amq_segment sg = segs[0];
  const uint32_t k = sg.hash_count, l = blockIdx.x;
  if (k == 0) return;
  const uint32_t n = min(*reinterpret_cast<const uint32_t*>(cnt + (uint64_t)l * cnt_stride), cap);
  const uint4* list = reinterpret_cast<const uint4*>(ent + (uint64_t)l * ent_stride);
  uint32_t* words = reinterpret_cast<uint32_t*>(out + sg.out_offset + kBloomHeader);
  const uint32_t kk = k < 8 ? k : 8u;
  for (uint32_t e = threadIdx.x; e < n; e += 256) {
    const uint4 x = list[e];
    if (x.w < p0 || x.w >= p1) continue;
    const uint64_t blk = ((uint64_t)x.w * q + rec_tile(x.x, x.y, x.z)) * kTileBlocks + (x.x & (kTileBlocks - 1));
    const uint32_t b[8] = {x.x >> 11, x.x >> 20, x.y, x.y >> 9, x.y >> 18, x.z, x.z >> 9, x.z >> 18};
    uint32_t* bw = words + 16ull * blk;
    for (uint32_t j = 0; j < kk; ++j) {
      const uint32_t bj = b[j] & 511u;
      atomicOr(bw + (bj >> 5), 1u << (bj & 31u));
    }
  }
}

// the tile and overflow kernels' records are 16-byte keys when the partition had them
__device__ inline bool part_raw(const tkv_amq_segment& sg, const PartArgs& a)
{
  return sg.hash_count > 8 && a.kb != 24;
}

template <int K>
__device__ inline void rec_insert(uint32_t* img, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t k)
{
  uint32_t* blk = img + 16 * (w0 & (kTileBlocks - 1));
  const uint32_t b[8] = {w0 >> 11, w0 >> 20, w1, w1 >> 9, w1 >> 18, w2, w2 >> 9, w2 >> 18};
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j)
    if (K != 0 ? j < (uint32_t)K : j < k) lds_set_bit(blk, b[j]);
}

// one workgroup per local tile t: region (t, w) of every partition workgroup w.  Each wave
// walks its regions (w = wave, wave + 16, ...) in pieces of 64 * V records, V per lane, and
// loads the next piece before it inserts the current one (two register sets, unrolled by two:
// no copy of an in-flight load), so every wave has one piece in flight at all times.
template <int K, bool RAW>
__device__ void tile_body(const tkv_amq_segment& sg, const PartArgs& a, uint32_t* img, uint32_t t,
                          uint32_t w_lo, uint32_t w_hi)
{
  constexpr uint32_t RB = RAW ? 16 : 12, NW = kTileThreads / 64, V = 8, PIECE = 64 * V;
  // wave-uniform in an SGPR: region counts are scalar loads (lgkmcnt), so waiting for one
  // never waits for the record loads in flight
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t P = a.g.P, cap = a.g.cap;
  const uint32_t k = sg.hash_count, nb = sg.n_blocks, first = (a.tile0 + t) * kTileBlocks;
  const uint32_t* counts = reinterpret_cast<const uint32_t*>(a.ws + a.g.counts_off) + (uint64_t)t * P;
  const uint64_t rstride = (uint64_t)cap * a.g.rb;  // bytes per region
  const uint8_t* regions = a.ws + a.g.regions_off + (uint64_t)t * P * rstride;
  struct Piece {
    uint32_t w, i0, c;  // region, first record, records in the region
    uint32_t x[V][4];
  };
  auto count = [&](uint32_t w) { return w < w_hi ? counts[w] : 0u; };
  auto load = [&](Piece& q) {
    const uint8_t* reg = q.w < w_hi ? regions + (uint64_t)q.w * rstride : a.ws;
    const uint32_t lastr = q.c ? q.c - 1 : 0u;
#pragma unroll
    for (uint32_t v = 0; v < V; ++v) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(reg + (uint64_t)min(q.i0 + v * 64 + lane, lastr) * RB);
      if constexpr (RAW) {
        const u32x4_t e = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
        q.x[v][0] = e.x; q.x[v][1] = e.y; q.x[v][2] = e.z; q.x[v][3] = e.w;
      } else {
        // one 12-byte load per record, nontemporal: the records are read once (plain loads
        // ran 20% slower, 0.351 vs 0.292 ms per 100M keys), and 16 bytes at the 12-byte
        // stride -- until round 6 -- took 77 instead of 68.7 us per config-5 part
        const u32x3_nt_t e = __builtin_nontemporal_load(reinterpret_cast<const u32x3_nt_t*>(p));
        q.x[v][0] = e.x; q.x[v][1] = e.y; q.x[v][2] = e.z; q.x[v][3] = 0;
      }
    }
  };
  // the piece after `q`: the next PIECE records of its region, else the wave's next region
  auto advance = [&](const Piece& q, Piece& n) {
    if (q.i0 + PIECE < q.c) {
      n.w = q.w;
      n.i0 = q.i0 + PIECE;
      n.c = q.c;
    } else {
      n.w = q.w + NW;
      n.i0 = 0;
      n.c = count(n.w);
    }
    load(n);
  };
  auto insert = [&](const Piece& q) {
#pragma unroll
    for (uint32_t v = 0; v < V; ++v) {
      if (q.i0 + v * 64 + lane >= q.c) continue;
      if constexpr (RAW) bloom_insert16<0>(img, nb, k, make_uint4(q.x[v][0], q.x[v][1], q.x[v][2], q.x[v][3]), first);
      else rec_insert<K>(img, q.x[v][0], q.x[v][1], q.x[v][2], k);
    }
  };
  Piece A, B;
  A.w = w_lo + wave;
  A.i0 = 0;
  A.c = count(A.w);
  load(A);
  while (A.w < w_hi) {
    advance(A, B);
    insert(A);
    if (B.w >= w_hi) break;
    advance(B, A);
    insert(B);
  }
  (void)P;
}

// (wg0: the build's first tile workgroup in the grid)
__device__ __attribute__((always_inline)) inline void tile_run(const tkv_amq_segment& sg, const PartArgs& a, uint8_t* __restrict__ out,
                                uint32_t hdr_always, uint32_t* s_img, uint32_t wg0)
{
  const uint32_t x = blockIdx.x - wg0, tid = threadIdx.x, k = sg.hash_count;
  if (k == 0) return;
  const uint32_t S = a.split > 1 ? a.split : 1u;
  const uint32_t t = x / S, sp = x - t * S;  // tile, and its share of the regions
  const uint32_t w_lo = (uint32_t)((uint64_t)a.g.P * sp / S), w_hi = (uint32_t)((uint64_t)a.g.P * (sp + 1) / S);
  const bool raw = part_raw(sg, a);
  const uint32_t first = (a.tile0 + t) * kTileBlocks;
  const uint32_t tb = min(kTileBlocks, sg.n_blocks - first);
  for (uint32_t w = tid; w < tb * 16; w += kTileThreads) s_img[w] = 0;
  __syncthreads();
  if (raw) tile_body<0, true>(sg, a, s_img, t, w_lo, w_hi);
  else if (k == 7) tile_body<7, false>(sg, a, s_img, t, w_lo, w_hi);
  else if (k == 8) tile_body<8, false>(sg, a, s_img, t, w_lo, w_hi);
  else tile_body<0, false>(sg, a, s_img, t, w_lo, w_hi);  // (k > 8 with 24-byte keys: eight bits)
  __syncthreads();
  uint8_t* payload = out + sg.out_offset;
  const bool hdr = t == 0 && sp == 0 && (a.tile0 == 0 || hdr_always);
  if (hdr && tid < 4) write_bloom_header(payload, sg, tid);
  else if (hdr && tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
  uint4* dst = reinterpret_cast<uint4*>(S > 1 ? a.part_img + ((uint64_t)(t * S + sp) << 17)
                                              : payload + kBloomHeader + 64ull * first);
  const uint4* src = reinterpret_cast<const uint4*>(s_img);
  for (uint32_t q = tid; q < tb * 4; q += kTileThreads) dst[q] = src[q];
}

// a split tile's partial images ORed into the filter: workgroup (t, c) merges uint4s
// [c * 256, (c + 1) * 256) of tile t, one per thread, its S partial loads issued together
constexpr uint32_t kMergeChunks = kTileBlocks * 4 / 256;  // 32 per tile
constexpr uint32_t kMaxSplit = 16;
__device__ __attribute__((always_inline)) inline void tile_merge_run(const tkv_amq_segment& sg, const PartArgs& a,
                                                                     uint8_t* __restrict__ out, uint32_t wg0)
{
  const uint32_t x = blockIdx.x - wg0, t = x / kMergeChunks, c = x - t * kMergeChunks;
  const uint32_t S = a.split, first = (a.tile0 + t) * kTileBlocks;
  const uint32_t tb = min(kTileBlocks, sg.n_blocks - first);
  const uint32_t q = c * 256 + threadIdx.x;
  if (q >= tb * 4) return;
  const uint4* src = reinterpret_cast<const uint4*>(a.part_img + ((uint64_t)t * S << 17)) + q;
  uint4 w[kMaxSplit];
#pragma unroll
  for (uint32_t sp = 0; sp < kMaxSplit; ++sp)
    w[sp] = sp < S ? load_nt16(src + ((uint64_t)sp << 13)) : make_uint4(0, 0, 0, 0);
  uint4 v = w[0];
#pragma unroll
  for (uint32_t sp = 1; sp < kMaxSplit; ++sp) {
    v.x |= w[sp].x;
    v.y |= w[sp].y;
    v.z |= w[sp].z;
    v.w |= w[sp].w;
  }
  reinterpret_cast<uint4*>(out + sg.out_offset + kBloomHeader + 64ull * first)[q] = v;
}

__global__ __launch_bounds__(256) void bloom_tile_merge(const tkv_amq_segment* __restrict__ segs, PartArgs a,
                                                         uint8_t* __restrict__ out)
{
  const tkv_amq_segment sg = segs[0];
  if (sg.hash_count == 0) return;
  tile_merge_run(sg, a, out, 0u);
}

__global__ __launch_bounds__(kTileThreads) void bloom_tile(const tkv_amq_segment* __restrict__ segs,
                                                           PartArgs a, uint8_t* __restrict__ out,
                                                           uint32_t hdr_always)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_img[];
  const tkv_amq_segment sg = segs[0];
  tile_run(sg, a, out, hdr_always, s_img, 0u);
}

// the filter header alone (a hash-range shard that owns no tile still returns a whole header)
__global__ __launch_bounds__(64) void bloom_header_only(const tkv_amq_segment* __restrict__ segs,
                                                        uint8_t* __restrict__ out)
{
  const tkv_amq_segment sg = segs[0];
  const uint32_t tid = threadIdx.x;
  if (sg.hash_count == 0) return;
  if (tid < 4) write_bloom_header(out + sg.out_offset, sg, tid);
  else if (tid < 8) write_page_header(out, sg, kLayoutBloom, tid - 4);
}

// one workgroup per partition workgroup's overflow list; device-scope atomics into the filter
// (runs after bloom_tile has stored every tile).  An entry is a record whose region was full
// (the 16-byte key itself when the records were keys).  24-byte keys with k > 8 (bits_per_key
// >= 13): the bits past the eighth of the workgroup's keys, also with atomics.
__device__ __attribute__((always_inline)) inline void overflow_run(const tkv_amq_segment& sg, const PartArgs& a, uint8_t* __restrict__ out)
{
  const uint32_t k = sg.hash_count, w = blockIdx.x - a.wg0, nb = sg.n_blocks;
  if (k == 0) return;
  const bool raw = part_raw(sg, a);
  const uint32_t n = reinterpret_cast<const uint32_t*>(a.ws + a.g.ovf_n_off)[w];
  const uint8_t* list = a.ws + a.g.ovf_off + (uint64_t)w * a.g.per * 16;
  uint32_t* words = reinterpret_cast<uint32_t*>(out + sg.out_offset + kBloomHeader);
  const uint32_t ib = a.src_kind == kSrcKey24 ? 24 : (a.src_kind == kSrcRec12 ? (raw ? 16 : 12) : 16);
  const uint8_t* src;
  uint32_t n_items;
  part_items(sg, a, ib, src, n_items);
  if (a.src_kind == kSrcKey24 && k > 8) {
    const uint32_t per = a.g.per;
    const uint32_t kb = min(n_items, w * per), ke = min(n_items, kb + per);
    for (uint32_t i = kb + threadIdx.x; i < ke; i += 256) {
      const XxhFixed<24> x(load_key24(src, i).w);
      const uint64_t h0 = x.finish(xxh_fixed_rc<24>(c_bloom.seed[0]));
      const uint32_t blk = (uint32_t)__umul64hi(h0, (uint64_t)nb);
      if ((blk >> kTileShift) - a.tile0 >= a.g.n_tiles) continue;  // (outside the window)
      uint32_t* bw = words + 16ull * blk;
      for (uint32_t j = 8; j < k; ++j) {
        const uint32_t bj = x.finish_lo9(xxh_fixed_rc<24>(c_bloom.seed[j])) & 511u;
        atomicOr(bw + (bj >> 5), 1u << (bj & 31u));
      }
    }
  }
  for (uint32_t e = threadIdx.x; e < n; e += 256) {
    if (raw) {
      const uint4 q = *reinterpret_cast<const uint4*>(list + 16ull * e);
      const Xxh16 x((uint64_t)q.x | ((uint64_t)q.y << 32), (uint64_t)q.z | ((uint64_t)q.w << 32));
      const uint64_t h0 = x.finish(c_bloom.rhinit16[0]);
      uint32_t* bw = words + 16 * (uint64_t)__umul64hi(h0, (uint64_t)nb);
      atomicOr(bw + ((h0 & 511u) >> 5), 1u << (h0 & 31u));
      for (uint32_t j = 1; j < k; ++j) {
        const uint32_t bj = x.finish_lo9(c_bloom.rhinit16[j]) & 511u;
        atomicOr(bw + (bj >> 5), 1u << (bj & 31u));
      }
      continue;
    }
    // a record whose region was full (its tile relative to the build's first tile is in it)
    const uint3 r = *reinterpret_cast<const uint3*>(list + 12ull * e);
    const uint64_t blk = (uint64_t)(a.tile0 + rec_tile(r.x, r.y, r.z)) * kTileBlocks + (r.x & (kTileBlocks - 1));
    const uint32_t b[8] = {r.x >> 11, r.x >> 20, r.y, r.y >> 9, r.y >> 18, r.z, r.z >> 9, r.z >> 18};
    uint32_t* bw = words + 16ull * blk;
    const uint32_t kk = k < 8 ? k : 8u;
    for (uint32_t j = 0; j < kk; ++j) {
      const uint32_t bj = b[j] & 511u;
      atomicOr(bw + (bj >> 5), 1u << (bj & 31u));
    }
  }
}

__global__ __launch_bounds__(256) void bloom_overflow(const tkv_amq_segment* __restrict__ segs,
                                                      PartArgs a, uint8_t* __restrict__ out)
{
  const tkv_amq_segment sg = segs[0];
  overflow_run(sg, a, out);
}

// ---------------------------------------------------------------------------------------
// Several monolithic builds in one launch each of partition, tile and overflow (the oversize
// leaves of a tkv_amq_build_ex batch, each of at most kDirectMaxTiles tiles): one leaf alone
// holds a few tiles -- a 3M-key leaf at 12 bits/key 35 -- so its tile kernel would leave most
// CUs idle; back to back in one grid the leaves' workgroups fill the chip.  The leaves'
// PartArgs are in the kernel argument (constant memory: the partition re-reads its fields
// instead of holding them in registers), with the first tile workgroup and the segment of
// each; a workgroup finds its leaf by a binary search over the first workgroups.
// ---------------------------------------------------------------------------------------
// Per leaf, what its PartArgs need beyond the launch's shared fields, all precomputed on the
// host: the kernels copy them from the kernel argument (constant memory, re-read rather than
// held in registers), never compute them
struct MultiLeaf {
  uint8_t* ws;
  uint8_t* part_img;
  uint64_t counts_off, ovf_n_off, regions_off, ovf_off;
  uint32_t n, P, n_tiles, per, cap, tbl, split;
  uint32_t wg0, tg0, mg0;  // the leaf's first partition / tile / merge workgroup
  uint32_t seg;            // its segment in the batch
};
constexpr uint32_t kMultiMaxLeaves = 40;
struct MultiParts {
  const uint8_t* keys;
  uint32_t kb, n;
  MultiLeaf l[kMultiMaxLeaves];
};
static_assert(sizeof(MultiParts) <= 4096 - 32, "kernel argument");

__device__ __attribute__((always_inline)) inline PartArgs multi_args(const MultiParts& m, const MultiLeaf& l)
{
  PartArgs a{};
  a.src = m.keys;
  a.n = l.n;
  a.from_seg = 1;
  a.kb = m.kb;
  a.ws = l.ws;
  a.g.P = l.P;
  a.g.n_tiles = l.n_tiles;
  a.g.per = l.per;
  a.g.cap = l.cap;
  a.g.rb = 16;
  a.g.counts_off = l.counts_off;
  a.g.ovf_n_off = l.ovf_n_off;
  a.g.regions_off = l.regions_off;
  a.g.ovf_off = l.ovf_off;
  a.src_kind = m.kb == 24 ? kSrcKey24 : kSrcKey16;
  a.tbl = l.tbl;
  a.wg0 = l.wg0;
  a.split = l.split;
  a.part_img = l.part_img;
  return a;
}

// GRID 0: partition / overflow, 1: tile, 2: merge
template <int GRID>
__device__ inline uint32_t multi_find(const MultiParts& m)
{
  uint32_t lo = 0, hi = m.n;  // the last leaf whose first workgroup is <= blockIdx.x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    const MultiLeaf& x = m.l[mid];
    if ((GRID == 1 ? x.tg0 : GRID == 2 ? x.mg0 : x.wg0) <= blockIdx.x) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kPartThreads) void bloom_part_multi16(const tkv_amq_segment* __restrict__ segs,
                                                                   MultiParts m)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const MultiLeaf& l = m.l[multi_find<0>(m)];
  const tkv_amq_segment sg = segs[l.seg];
  part_keys16(sg, multi_args(m, l), s_part);
}

__global__ __launch_bounds__(kPartThreads) void bloom_part_multi24(const tkv_amq_segment* __restrict__ segs,
                                                                   MultiParts m)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_part[];
  const MultiLeaf& l = m.l[multi_find<0>(m)];
  const tkv_amq_segment sg = segs[l.seg];
  part_keys24(sg, multi_args(m, l), s_part);
}

__global__ __launch_bounds__(kTileThreads) void bloom_tile_multi(const tkv_amq_segment* __restrict__ segs,
                                                                 MultiParts m, uint8_t* __restrict__ out)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_img[];
  const MultiLeaf& l = m.l[multi_find<1>(m)];
  const tkv_amq_segment sg = segs[l.seg];
  tile_run(sg, multi_args(m, l), out, 0u, s_img, l.tg0);
}

__global__ __launch_bounds__(256) void bloom_tile_merge_multi(const tkv_amq_segment* __restrict__ segs,
                                                              MultiParts m, uint8_t* __restrict__ out)
{
  const MultiLeaf& l = m.l[multi_find<2>(m)];
  const tkv_amq_segment sg = segs[l.seg];
  tile_merge_run(sg, multi_args(m, l), out, l.mg0);
}

__global__ __launch_bounds__(256) void bloom_overflow_multi(const tkv_amq_segment* __restrict__ segs,
                                                            MultiParts m, uint8_t* __restrict__ out)
{
  const MultiLeaf& l = m.l[multi_find<0>(m)];
  const tkv_amq_segment sg = segs[l.seg];
  overflow_run(sg, multi_args(m, l), out);
}

// ---------------------------------------------------------------------------------------
// Bloom probe
// ---------------------------------------------------------------------------------------
// Probe-side view of a segment: the first 16 bytes of tkv_amq_segment in one load.
struct ProbeDesc {
  uint64_t out_offset;
  uint32_t n_blocks;
  uint32_t hash_count, tag_bits, hash_val_shift;
};

// A leaf index outside the plan reads as "no filter" (the probe answers "maybe", like
// reject_page's kUnknown for a page it cannot check, tree/key_query.hpp:156-159): nothing is
// read out of bounds.
__device__ inline ProbeDesc load_probe_desc(const tkv_amq_segment* segs, uint32_t s, uint32_t n_segs)
{
  const bool in = s < n_segs;
  const uint4 v = reinterpret_cast<const uint4*>(segs + (in ? s : 0u))[0];
  ProbeDesc d;
  d.out_offset = (uint64_t)v.x | ((uint64_t)v.y << 32);
  d.n_blocks = v.z;
  d.hash_count = in ? v.w & 0xffffu : 0u;
  d.tag_bits = in ? (v.w >> 16) & 0xffu : 0u;
  d.hash_val_shift = v.w >> 24;
  return d;
}

// One lane per (query, leaf).  The 64-byte filter block is fetched with four 16-byte loads
// (instead of k divergent 8-byte loads) and staged in a per-lane LDS slot; the k bit tests
// are then LDS reads.  Stride 20 dwords keeps the slots 16-byte aligned and spreads banks.
constexpr uint32_t kProbeSlotWords = 20;

// The block's four 16-byte loads are issued first and the remaining k-1 bit indices are
// hashed while they are in flight; only then is the block staged in the lane's LDS slot.
template <int K>
__device__ inline uint32_t probe_block16(const Xxh16& x, uint64_t h0, const uint4* blk, uint4* slot,
                                         uint32_t k_rt = K)
{
  const uint4 b0 = blk[0], b1 = blk[1], b2 = blk[2], b3 = blk[3];
  const uint32_t* slot32 = reinterpret_cast<const uint32_t*>(slot);
  uint32_t ok = 1;
  if constexpr (K > 0) {
    uint32_t bit[K];
    bit[0] = (uint32_t)h0 & 511u;
#pragma unroll
    for (int j = 1; j < K; ++j) bit[j] = x.finish_lo9(c_bloom.rhinit16[j]) & 511u;
    slot[0] = b0;
    slot[1] = b1;
    slot[2] = b2;
    slot[3] = b3;
#pragma unroll
    for (int j = 0; j < K; ++j) ok &= slot32[bit[j] >> 5] >> (bit[j] & 31);
  } else {
    slot[0] = b0;
    slot[1] = b1;
    slot[2] = b2;
    slot[3] = b3;
    uint32_t b = (uint32_t)h0 & 511u;
    ok &= slot32[b >> 5] >> (b & 31);
    for (uint32_t j = 1; j < k_rt; ++j) {
      b = x.finish_lo9(c_bloom.rhinit16[j]) & 511u;
      ok &= slot32[b >> 5] >> (b & 31);
    }
  }
  return ok;
}

// KeyQuery::Metrics tallies of one lane (tkv_amq_probe_ex): per query, the class of its
// reject_page answer (tree/key_query.hpp:149-247).  Reduced over the wave with shuffles and
// added to the caller's counters with one atomic per counter per wave.
enum ProbeClass : uint32_t { kNoFilter = 0, kIdMismatch = 1, kChecked = 2 };

struct ProbeTally {
  uint32_t total = 0, no_filter = 0, mismatch = 0, reject = 0, positive = 0, false_pos = 0;
  // r: result bit (1 = maybe present) | class << 1
  __device__ inline void add(uint32_t r, const uint8_t* truth, uint64_t i)
  {
    const uint32_t cls = r >> 1;
    ++total;
    no_filter += cls == kNoFilter;
    mismatch += cls == kIdMismatch;
    const bool checked = cls == kChecked;
    reject += checked && !(r & 1u);
    const bool pos = checked && (r & 1u);
    positive += pos;
    if (pos && truth) false_pos += truth[i] == 0;
  }
};

__device__ inline uint32_t wave_sum(uint32_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ inline void flush_tally(const ProbeTally& t, tkv_amq_probe_metrics* m, bool has_truth)
{
  const uint32_t v[6] = {wave_sum(t.total), wave_sum(t.no_filter), wave_sum(t.mismatch),
                         wave_sum(t.reject), wave_sum(t.positive), wave_sum(t.false_pos)};
  if (__lane_id() == 0 && m) {
    unsigned long long* c = reinterpret_cast<unsigned long long*>(m);
    if (v[0]) atomicAdd(&c[0], (unsigned long long)v[0]);
    if (v[1]) atomicAdd(&c[1], (unsigned long long)v[1]);
    if (v[2]) atomicAdd(&c[2], (unsigned long long)v[2]);
    if (v[3]) atomicAdd(&c[3], (unsigned long long)v[3]);
    if (v[4]) atomicAdd(&c[4], (unsigned long long)v[4]);
    if (has_truth && v[5]) atomicAdd(&c[5], (unsigned long long)v[5]);
  }
}

// filter header's src_page_id (PackedBloomFilterPage / PackedVqfFilter) vs the leaf the query
// asks about (reject_page, tree/key_query.hpp:205-212,227-232): the filter bytes decide, as in
// the reference
__device__ inline bool page_id_matches(const uint8_t* payload, uint32_t id_off, const uint64_t* ids,
                                       uint64_t i)
{
  return ids == nullptr || *reinterpret_cast<const uint64_t*>(payload + id_off) == ids[i];
}

// One Bloom (query, leaf) test: result bit | class << 1 (the class only with kOpts).  Without
// kOpts the control flow is the plain probe's: no early exit, so the key load is issued
// side by side with the segment index and descriptor loads (an early "no filter" return
// made the compiler sink it behind them: 11% slower).
template <int MODE, bool kOpts>
__device__ inline uint32_t bloom_probe_item(const uint8_t* __restrict__ filters,
                                            const tkv_amq_segment* __restrict__ segs, uint32_t n_segs,
                                            const uint8_t* __restrict__ q,
                                            const uint64_t* __restrict__ qoffs, uint32_t stride,
                                            uint64_t i, uint32_t sidx, uint4* slot,
                                            const uint64_t* page_ids)
{
  uint32_t ok = 1;
  if constexpr (MODE == kKey16) {
    // the key load, the descriptor and the first hash do not depend on the "has a filter"
    // test, so they are issued before it: one dependent chain qseg -> descriptor -> block
    const uint4 kv = load_nt16(q + 16 * i);
    const ProbeDesc d = load_probe_desc(segs, sidx, n_segs);
    const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
    const uint64_t h0 = x.finish(c_bloom.rhinit16[0]);
    const uint4* blk = reinterpret_cast<const uint4*>(filters + d.out_offset + kBloomHeader +
                                                      64 * __umul64hi(h0, (uint64_t)d.n_blocks));
    // hash_count 0: no filter page => reject_page returns kUnknown => cannot reject
    uint32_t cls = d.hash_count == 0 ? kNoFilter : kChecked;
    if constexpr (kOpts) {
      if (cls == kChecked && !page_id_matches(filters + d.out_offset, 16, page_ids, i)) cls = kIdMismatch;
    }
    if (!kOpts || cls == kChecked) {
      if (d.hash_count == 7) ok = probe_block16<7>(x, h0, blk, slot);
      else if (d.hash_count == 8) ok = probe_block16<8>(x, h0, blk, slot);
      else if (d.hash_count != 0) ok = probe_block16<0>(x, h0, blk, slot, d.hash_count);
    }
    return (ok & 1u) | (cls << 1);
  } else {
    const ProbeDesc d = load_probe_desc(segs, sidx, n_segs);
    if (d.hash_count == 0) return 1u | (kNoFilter << 1);
    if (!page_id_matches(filters + d.out_offset, 16, page_ids, i)) return 1u | (kIdMismatch << 1);
    const uint8_t* words = filters + d.out_offset + kBloomHeader;
    uint32_t len;
    const uint8_t* p = key_at<MODE>(q, qoffs, stride, i, len);
    if (len < 32) {  // seed-independent lane rounds shared by the k hashes
      const XxhShort x(p, len);
      const uint64_t h0 = x.finish(c_bloom.seed_p5[0]);
      const uint64_t* blk = reinterpret_cast<const uint64_t*>(words + 64 * __umul64hi(h0, (uint64_t)d.n_blocks));
      uint32_t b = (uint32_t)h0 & 511u;
      ok &= (uint32_t)(blk[b >> 6] >> (b & 63));
      for (uint32_t j = 1; j < d.hash_count; ++j) {
        b = x.finish_lo9(c_bloom.seed_p5[j]) & 511u;
        ok &= (uint32_t)(blk[b >> 6] >> (b & 63));
      }
    } else {
      const uint64_t h0 = xxh64_bytes(p, len, c_bloom.seed[0]);
      const uint64_t* blk = reinterpret_cast<const uint64_t*>(words + 64 * __umul64hi(h0, (uint64_t)d.n_blocks));
      uint32_t b = (uint32_t)h0 & 511u;
      ok &= (uint32_t)(blk[b >> 6] >> (b & 63));
      for (uint32_t j = 1; j < d.hash_count; ++j) {
        b = (uint32_t)xxh64_bytes(p, len, c_bloom.seed[j]) & 511u;
        ok &= (uint32_t)(blk[b >> 6] >> (b & 63));
      }
    }
  }
  return (ok & 1u) | (kChecked << 1);
}

// kOpts = false: one lane per query (the plain probe).  kOpts = true (tkv_amq_probe_ex): a
// grid-stride loop over a bounded grid with the page-id check and the metrics tallies.
template <int MODE, bool kOpts>
__global__ __launch_bounds__(256) void bloom_probe(const uint8_t* __restrict__ filters,
                                                   const tkv_amq_segment* __restrict__ segs, uint32_t n_segs,
                                                   const uint8_t* __restrict__ q,
                                                   const uint64_t* __restrict__ qoffs,
                                                   uint32_t stride, uint64_t n,
                                                   const uint32_t* __restrict__ qseg,
                                                   uint8_t* __restrict__ result, tkv_amq_probe_opts opts)
{
  __shared__ uint4 s_blk[256 * kProbeSlotWords / 4];
  uint4* slot = s_blk + threadIdx.x * (kProbeSlotWords / 4);
  if constexpr (!kOpts) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = bloom_probe_item<MODE, false>(filters, segs, n_segs, q, qoffs, stride, i,
                                                     __builtin_nontemporal_load(qseg + i), slot, nullptr);
    __builtin_nontemporal_store((uint8_t)(r & 1u), result + i);
  } else {
    ProbeTally t;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
      const uint32_t r = bloom_probe_item<MODE, true>(filters, segs, n_segs, q, qoffs, stride, i,
                                                      qseg[i], slot, opts.d_query_page_id);
      result[i] = (uint8_t)(r & 1u);
      t.add(r, opts.d_truth, i);
    }
    flush_tally(t, opts.d_metrics, opts.d_truth != nullptr);
  }
}

// ---------------------------------------------------------------------------------------
// VQF constants (tkv-amq v1)
// ---------------------------------------------------------------------------------------
template <int T>
struct Vqf;
template <>
struct Vqf<8> {
  static constexpr uint32_t kSlots = 48, kBuckets = 80, kThreshold = 37, kMdBytes = 16;
  static constexpr uint32_t kOffsetBits = 7;
  using Entry = uint16_t;  // (bucket offset << 8) | tag
};
template <>
struct Vqf<16> {
  static constexpr uint32_t kSlots = 28, kBuckets = 36, kThreshold = 22, kMdBytes = 8;
  static constexpr uint32_t kOffsetBits = 6;
  using Entry = uint32_t;  // (bucket offset << 16) | tag
};
// kThreshold: the reference-side vqf consults the alternate block only when the primary's
// metadata popcount is below CHECK_ALT (92 / 43), i.e. when its count >= kThreshold.

constexpr uint32_t kVqfTempStride = 128;  // workspace bytes per block (>= slots * entry)
constexpr uint32_t kVqfMaxLdsBlocks = 16384;
constexpr uint32_t kVqfMatchLdsBlocks = 2048;  // vqf_decide's LDS lane-mask table (8 B/block)

// workspace: [header u32 x8][record sink u64 x4][nelts u32 x n_segs][pad to 256]
//            [128-byte record per block]
//            [u64 placement record per key]
// header[1] = n_segs of the last build (written by every decide workgroup; read by
// tkv_amq_build_check); nelts[s] = leaf s's element count | its failure flags (below).  Every
// build rewrites both for every leaf, so no memset precedes a build.
// block record = slots x Entry (insertion order) ... u32 final count at byte 124
// key record (written by vqf_decide in key order, coalesced; scattered by vqf_scatter):
//   hi 32 = global block * 64 + rank in the block, or ~0 for a key that is not inserted
//   lo 32 = Entry ((bucket offset << T) | tag), bit 31 set for 32-bit entries (T = 16)
struct VqfWorkspace {
  uint32_t* hdr;
  uint32_t* nelts;
  uint8_t* temp;
  uint64_t* sink;  // write-only target of vqf_decide's stores for lanes with no record
};
constexpr uint32_t kVqfCountByte = 124;

__host__ __device__ inline uint64_t vqf_temp_offset(uint32_t n_segs)
{
  return (64 + 4ull * n_segs + 255) & ~255ull;
}

__host__ __device__ inline VqfWorkspace vqf_workspace(void* base, uint32_t n_segs)
{
  uint8_t* p = static_cast<uint8_t*>(base);
  VqfWorkspace w;
  w.hdr = reinterpret_cast<uint32_t*>(p);
  w.nelts = reinterpret_cast<uint32_t*>(p + TKV_AMQ_VQF_NELTS_OFFSET);
  w.sink = reinterpret_cast<uint64_t*>(p + 32);
  w.temp = p + vqf_temp_offset(n_segs);
  return w;
}

// the key records follow the last segment's blocks
__device__ inline uint64_t* vqf_records(VqfWorkspace ws, const tkv_amq_segment* segs, uint32_t n_segs)
{
  const tkv_amq_segment& last = segs[n_segs - 1];
  return reinterpret_cast<uint64_t*>(ws.temp + kVqfTempStride * (last.block_base + last.n_blocks));
}

// Bytes of workspace the plan's VQF kernels touch (tkv_amq_plan's workspace_bytes minus the
// tail pad).  Every VQF kernel checks it against the size the caller passed and, if the
// workspace is too small, flags its leaf kVqfFlagWorkspace and writes nothing else.
constexpr uint32_t kVqfFlagOverflow = TKV_AMQ_VQF_FLAG_OVERFLOW;    // a block overflowed (vqf_insert failed)
constexpr uint32_t kVqfFlagWorkspace = TKV_AMQ_VQF_FLAG_WORKSPACE;  // workspace smaller than the plan needs
static_assert(kVqfFlagOverflow == 1u << 31 && kVqfFlagWorkspace == 1u << 30, "");
constexpr uint32_t kVqfNeltsMask = kVqfFlagWorkspace - 1;

// seg: the leaf whose nelts word takes the flag (~0u: none, e.g. a per-key kernel)
__device__ inline bool vqf_ws_ok(const tkv_amq_segment* segs, uint32_t n_segs, uint64_t ws_bytes,
                                 VqfWorkspace ws, uint32_t seg)
{
  const tkv_amq_segment& last = segs[n_segs - 1];
  const uint64_t need = vqf_temp_offset(n_segs) + kVqfTempStride * (last.block_base + last.n_blocks) +
                        8 * (last.key_begin + last.n_keys);
  if (need <= ws_bytes) return true;
  if (threadIdx.x == 0 && seg != ~0u) ws.nelts[seg] = kVqfFlagWorkspace;
  return false;
}

// the first thing every decide workgroup does: the build's leaf count for tkv_amq_build_check
// (the header lies inside the part of the workspace the host checks).
// INVARIANT (no memset precedes a VQF build): every decide-class kernel (vqf_decide,
// vqf_decide_big, vqf_decide_ring, vqf_ring_place) calls this for every leaf and then writes
// that leaf's nelts word -- flags included -- on every path, including the early exits
// (vqf_ws_ok's short-workspace flag, bits_per_key 0); tkv_amq_build's max_blocks == 0 path
// clears the header word itself.  A kernel that skipped either would let tkv_amq_build_check,
// LeafBatcher and HostFilterPipeline read a previous build's flags
// (test_gpu_robustness.py::test_vqf_failed_build_then_clean_build_on_one_workspace).
__device__ inline void vqf_mark_build(VqfWorkspace ws, uint32_t n_segs)
{
  if (threadIdx.x == 0) ws.hdr[1] = n_segs;
}

__device__ inline uint32_t vqf_nelts_word(uint32_t nelts, bool fail)
{
  return (nelts & kVqfNeltsMask) | (fail ? kVqfFlagOverflow : 0u);
}

__device__ inline uint32_t& vqf_count(VqfWorkspace ws, uint64_t block)
{
  return *reinterpret_cast<uint32_t*>(ws.temp + block * kVqfTempStride + kVqfCountByte);
}

// vqf_decide's per-block element counts, by leaf size:
//   kCntU32     u32 in LDS (leaves of <= kVqfMaxLdsBlocks blocks: the fast path)
//   kCntU8      u8 in LDS, 4 per dword (<= kVqfU8LdsBlocks blocks, ~10 MB of filter).  A count
//               passes 255 (and carries into its neighbour) only after its block overflowed
//               at the 49th insert, which already fails the leaf (Internal, no filter)
//   kCntGlobal  u32 at byte kVqfCountByte of the leaf's block records in the workspace, with
//               agent-scope atomics (any larger leaf: one memory round trip per 64-key step)
enum VqfCountMode : int { kCntU32 = 0, kCntU8 = 1, kCntGlobal = 2 };
constexpr uint32_t kVqfU8LdsBlocks = 160 * 1024;
constexpr uint32_t kVqfMaxBlocks = 1u << 24;  // block ids fit the 24-bit ballot match

template <int CNT>
struct VqfCounts;
template <>
struct VqfCounts<kCntU32> {
  uint32_t* p;
  __device__ inline uint32_t get(uint32_t b) const { return p[b]; }
  __device__ inline void add(uint32_t b, uint32_t v) const { atomicAdd(p + b, v); }
  __device__ inline void clear(uint32_t nb, uint32_t lane) const
  {
    for (uint32_t b = lane; b < nb; b += 64) p[b] = 0;
  }
};
template <>
struct VqfCounts<kCntU8> {
  uint32_t* p;
  __device__ inline uint32_t get(uint32_t b) const { return reinterpret_cast<const uint8_t*>(p)[b]; }
  __device__ inline void add(uint32_t b, uint32_t v) const { atomicAdd(p + (b >> 2), v << (8 * (b & 3))); }
  __device__ inline void clear(uint32_t nb, uint32_t lane) const
  {
    for (uint32_t w = lane; w < (nb + 3) / 4; w += 64) p[w] = 0;
  }
};
template <>
struct VqfCounts<kCntGlobal> {
  uint8_t* rec;  // the leaf's first block record
  __device__ inline uint32_t* at(uint32_t b) const
  {
    return reinterpret_cast<uint32_t*>(rec + (uint64_t)b * kVqfTempStride + kVqfCountByte);
  }
  __device__ inline uint32_t get(uint32_t b) const
  {
    return __hip_atomic_load(at(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // acquire-release: the wave waits for the add before its next step reads the counts
  __device__ inline void add(uint32_t b, uint32_t v) const
  {
    __hip_atomic_fetch_add(at(b), v, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ inline void clear(uint32_t nb, uint32_t lane) const
  {
    for (uint32_t b = lane; b < nb; b += 64)
      __hip_atomic_store(at(b), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  }
};

// A key the VQF kernels load one or two chunks ahead of hashing it (16- and 24-byte keys;
// other shapes are read where they are hashed)
template <int MODE>
struct VqfKeyBuf {
  uint4 v;
};
template <>
struct VqfKeyBuf<kKey24> {
  uint64_t w[3];
};
// Variable-length keys (the reference's KeyView ranges): the bytes of a key under 32 bytes
// (XxhShort's lanes, 4-byte tail, tail bytes) and the offsets of the key this lane loads
// next, so a step's byte loads need no offset load of their own: the offsets run one load
// ahead of the bytes.  Keys of 32 bytes or more are hashed from memory where they are hashed.
template <>
struct VqfKeyBuf<kKeyVar> {
  KeyWin w;  // the key's bytes (a key under 32 bytes)
  uint32_t len;
  uint64_t off;
  uint64_t noff;
  uint32_t nlen;
};
template <>
struct VqfKeyBuf<kKeyLoc> {
  uint2 v;  // the key's located record (vqf_loc_encode)
};
template <int MODE>
constexpr bool kVqfPrefetch = MODE == kKey16 || MODE == kKey24 || MODE == kKeyVar;
// vqf_decide_ring's producers prefetch 16- and 24-byte keys (and located records) only (three
// rotating buffers of variable-length keys would cost the ring kernel its three workgroups
// per CU)
template <int MODE>
constexpr bool kVqfRingPrefetch = MODE == kKey16 || MODE == kKey24 || MODE == kKeyLoc;

// the bytes of the key whose offsets `prev` holds, and the offsets of key gi_next.  Every lane
// issues the same loads (clamped to a safe address when the key is shorter: the offsets
// array holds >= 16 bytes; or the leaf's buffer resource, KeyWin), so the count in flight is
// fixed.
__device__ inline void vqf_load_var(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                    uint64_t gi_next, const VqfKeyBuf<kKeyVar>& prev,
                                    VqfKeyBuf<kKeyVar>& kb, const VarRsrc& vr)
{
  const uint64_t off = prev.noff;
  const uint32_t len = prev.nlen;
  if (vr.nrec) key_win_load(vr, (uint32_t)(off - vr.base), kb.w);  // (uniform per leaf)
  else key_win_load_clamped(keys + off, len, reinterpret_cast<const uint8_t*>(offs), kb.w);
  kb.len = len;
  kb.off = off;
  kb.noff = offs[gi_next];
  kb.nlen = (uint32_t)(offs[gi_next + 1] - kb.noff);
}

template <int MODE>
__device__ inline void vqf_load_key(const uint8_t* __restrict__ keys, uint64_t gi, VqfKeyBuf<MODE>& kb)
{
  if constexpr (MODE == kKey16) {
    kb.v = reinterpret_cast<const uint4*>(keys)[gi];
  } else if constexpr (MODE == kKey24) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(keys) + 3 * gi;
#pragma unroll
    for (int i = 0; i < 3; ++i) kb.w[i] = p[i];
  } else if constexpr (MODE == kKeyLoc) {
    kb.v = reinterpret_cast<const uint2*>(keys)[gi];
  }
}

template <int MODE>
__device__ inline uint64_t vqf_key_hash(const uint8_t* __restrict__ keys,
                                        const uint64_t* __restrict__ offs, uint32_t stride,
                                        uint64_t gi, const VqfKeyBuf<MODE>& kb)
{
  if constexpr (MODE == kKey16) {
    const uint4 kv = kb.v;
    const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
    return x.finish(xxh16_rhinit(kVqfHashSeed));
  } else if constexpr (MODE == kKey24) {
    const XxhFixed<24> x(kb.w);
    return x.finish(xxh_fixed_rc<24>(kVqfHashSeed));
  } else if constexpr (MODE == kKeyVar) {
    if (kb.len < 32) {
      uint64_t l[3];
      uint32_t t4, tb;
      key_win_parts(kb.w, kb.len, l, t4, tb);
      return XxhShort(kb.len, l, t4, tb).finish(kVqfHashSeed + kP5);
    }
    return xxh64_bytes(keys + kb.off, kb.len, kVqfHashSeed);
  } else {
    return hash_key<MODE>(keys, offs, stride, gi, kVqfHashSeed);
  }
}

// Per-lane location of one key: primary block and bucket offset, tag, and the hash (the
// alternate block is derived from it only when a step needs it: vqf_locate_alt).
struct VqfLoc {
  uint64_t h;
  uint32_t pb, po, tag;
  bool kept;
};

template <int T>
__device__ inline VqfLoc vqf_locate(uint64_t h, bool valid, uint64_t mask, uint64_t R,
                                    uint64_t magic)
{
  using C = Vqf<T>;
  VqfLoc l;
  l.h = h;
  l.kept = valid && ((h & mask) == h);  // filter_builder.hpp:210
  l.tag = (uint32_t)(h & ((1ull << T) - 1));
  const uint32_t pi = (uint32_t)mod_by_magic(h >> T, R, magic);
  l.pb = pi / C::kBuckets;
  l.po = pi - l.pb * C::kBuckets;
  return l;
}

// alternate bucket ((h ^ tag * 0x5bd1e995) >> T) mod R -> (block, offset)
template <int T>
__device__ inline void vqf_locate_alt(const VqfLoc& l, uint64_t R, uint64_t magic, uint32_t& ab,
                                      uint32_t& ao)
{
  using C = Vqf<T>;
  const uint32_t ai = (uint32_t)mod_by_magic((l.h ^ ((uint64_t)l.tag * kVqfAltMul)) >> T, R, magic);
  ab = ai / C::kBuckets;
  ao = ai - ab * C::kBuckets;
}

// A located key (kKeyLoc; leaves of <= 2,048 blocks): x = primary block | alternate block << 11
// | primary bucket offset << 22 | kept << 31, y = tag | alternate bucket offset << 16
template <int T>
__device__ inline uint2 vqf_loc_encode(uint64_t h, const tkv_amq_segment& sg)
{
  using C = Vqf<T>;
  const uint64_t R = (uint64_t)sg.n_blocks * C::kBuckets;
  const VqfLoc l = vqf_locate<T>(h, true, ~0ull << sg.hash_val_shift, R, sg.mod_magic);
  uint32_t ab, ao;
  vqf_locate_alt<T>(l, R, sg.mod_magic, ab, ao);
  return make_uint2(l.pb | ab << 11 | l.po << 22 | (l.kept ? 1u << 31 : 0u), l.tag | ao << 16);
}
__device__ inline void vqf_loc_decode(uint2 r, bool valid, VqfLoc& l, uint32_t& ab, uint32_t& ao)
{
  l.h = 0;
  l.pb = r.x & 2047u;
  ab = (r.x >> 11) & 2047u;
  l.po = (r.x >> 22) & 127u;
  l.kept = valid && (r.x >> 31) != 0;
  l.tag = r.y & 0xffffu;
  ao = r.y >> 16;
}
constexpr uint32_t kVqfLocMaxBlocks = 2048;

// Exact replay of the reference insert order (build_vqf_filter<T>, filter_builder.hpp:204-214)
// for one leaf, 64 keys per step.  The power-of-two-choice decision of key i depends only on
// the element counts of its two candidate blocks at the time of its insertion, so a chunk is
// resolved as follows: every lane starts from the counts it would see if all earlier lanes of
// the chunk took their primary block (two bit-sliced ballot matches); the first lane whose
// exact decision is "alternate" is found with one ballot, its move is applied to the later
// lanes, and the scan repeats -- one round per alternate choice, not per key.  The count of
// the chosen block at decision time is the key's insertion rank inside that block.
// NBITS >= ceil(log2(n_blocks)) is a compile-time bound (extra high bits are zero in every
// lane and leave the matches unchanged), so the match loop unrolls into the same basic
// block as the next chunk's hashing and the two interleave.
// kLdsMatch: the four lane-match masks come from an LDS table of 64-bit lane masks, one per
// block (each lane ORs its bit into its block's entry, then reads the entries it needs,
// then clears): a handful of LDS operations instead of ~7 VALU per block-id bit.  Needs
// 8 B of LDS per block, so it is used for leaves of <= kVqfMatchLdsBlocks blocks.
// kCompact (T = 8, <= 512 blocks, fused place): 4-byte key records
//   block << 21 | rank << 15 | (bucket offset << 8 | tag), or ~0 for a key not inserted
template <int T, int MODE, int NBITS, bool kLdsMatch, bool kCompact, int CNT = kCntU32>
__device__ void vqf_decide_body(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                uint32_t stride, const tkv_amq_segment& sg, uint32_t seg_index,
                                VqfWorkspace ws, uint64_t* __restrict__ recs, uint32_t* s_lds,
                                bool fused, uint64_t key_end)
{
  static_assert(!kLdsMatch || CNT == kCntU32, "the lane-mask table follows u32 counts");
  using C = Vqf<T>;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = sg.n_keys, nb = sg.n_blocks;
  const uint64_t R = (uint64_t)nb * C::kBuckets;
  const uint64_t magic = sg.mod_magic;
  const uint64_t mask = ~0ull << sg.hash_val_shift;  // filter_builder.hpp:187
  const uint64_t lt = lanemask_lt();
  using Rec = typename std::conditional<kCompact, uint32_t, uint64_t>::type;
  Rec* rec = reinterpret_cast<Rec*>(recs + sg.key_begin);
  using KB = VqfKeyBuf<MODE>;
  // variable-length keys: the leaf's bytes through a buffer resource (KeyWin)
  VarRsrc vr{};
  if constexpr (MODE == kKeyVar)
    if (n > 0) vr = var_rsrc(keys, offs[sg.key_begin], offs[sg.key_begin + n], key_end);

  VqfCounts<CNT> cnt;
  if constexpr (CNT == kCntGlobal) cnt.rec = ws.temp + sg.block_base * kVqfTempStride;
  else cnt.p = s_lds;
  unsigned long long* mt = reinterpret_cast<unsigned long long*>(s_lds + ((nb + 1) & ~1u));
  cnt.clear(nb, lane);
  if constexpr (kLdsMatch)
    for (uint32_t b = lane; b < nb; b += 64) mt[b] = 0;
  // one wave: its LDS operations execute in order, so no workgroup barrier (the body also
  // runs in wave 0 of vqf_decide_ring's workgroup after the other waves have left)
  asm volatile("" ::: "memory");
  const unsigned long long mybit = 1ull << lane;

  uint32_t nelts = 0;
  uint32_t fail = 0;

  // One 64-key step.  `cur` = located keys of this chunk; `kv_hash` = raw keys of the next
  // chunk (loaded one step earlier); `kv_load` receives the chunk after that.  The loop
  // below is unrolled by two with the key buffers swapping roles, so no register copy of an
  // in-flight load exists and the compiler waits only for that load, never for the scatter
  // store issued after it.
  // The chunk's placement records are one coalesced 512-byte store, issued at the start of
  // the next step (after that step's loads), so a wait for the key prefetch never waits
  // for a store issued just before it.  (Scattering each tag straight into its block's
  // record from here made every step wait on partial-line writes: 2.1x slower.)
  // The store is unconditional (lanes with nothing to write hit a sink word), so the number
  // of memory operations issued after each key load is fixed and the compiler's wait for
  // that load (s_waitcnt vmcnt counts loads and stores in issue order) lets the later load
  // and the stores stay in flight; a skippable store made it wait for the newest load too.
  Rec* const sink = reinterpret_cast<Rec*>(ws.sink);
  Rec* pend_ptr = sink;
  Rec pend_val = 0;
  auto step = [&](uint32_t base, VqfLoc& cur, const KB& kv_hash, KB& kv_load) {
    const VqfLoc L = cur;
    // primary block counts before this chunk (every lane reads: an invalid lane's block is 0)
    const uint32_t cnt_p = cnt.get(L.pb);
    const uint32_t inext = base + 64 + lane;
    const bool vnext = inext < n;
    uint64_t hn;
    if constexpr (kVqfPrefetch<MODE>) {
      // branch-free (clamped index, select on the result): straight-line code lets the
      // compiler count vmcnt exactly instead of draining every outstanding access
      if constexpr (MODE == kKeyVar)  // bytes of chunk + 2 (offsets in kv_hash), offsets of + 3
        vqf_load_var(keys, offs, sg.key_begin + min(inext + 128, n - 1), kv_hash, kv_load, vr);
      else
        vqf_load_key<MODE>(keys, sg.key_begin + min(inext + 64, n - 1), kv_load);
      *pend_ptr = pend_val;
      const uint64_t hh = vqf_key_hash<MODE>(keys, offs, stride, 0, kv_hash);
      hn = vnext ? hh : 0;
    } else {
      *pend_ptr = pend_val;
      hn = vnext ? vqf_key_hash<MODE>(keys, offs, stride, sg.key_begin + inext, kv_hash) : 0;
    }

    const uint64_t keptmask = __ballot(L.kept);
    nelts += __popcll(keptmask);
    // lanes with pb_j == my pb: one LDS lane-mask table round trip, or one ballot per
    // block-id bit, each 32-bit half of the match mask updated with one v_bitop3
    // (m & ~(ballot ^ sext(bit)))
    uint32_t mpp_lo = (uint32_t)keptmask, mpp_hi = (uint32_t)(keptmask >> 32);
    // LDS operations are never skipped (lanes with no key OR 0, add 0 and clear an entry no
    // kept lane set in this phase), so the compiler's count of them in flight is exact
    if constexpr (kLdsMatch) {
      atomicOr(mt + L.pb, L.kept ? mybit : 0ull);
      asm volatile("" ::: "memory");
      const uint64_t a = mt[L.pb];
      asm volatile("" ::: "memory");
      mt[L.pb] = 0;
      mpp_lo &= (uint32_t)a;
      mpp_hi &= (uint32_t)(a >> 32);
    }
#pragma unroll
    for (int j = 0; j < (kLdsMatch ? 0 : NBITS); ++j) {
      const uint32_t xp = (uint32_t)__builtin_amdgcn_sbfe((int32_t)L.pb, j, 1);  // 0 or ~0
      const uint64_t bp = __ballot(xp != 0);
      mpp_lo &= ~((uint32_t)bp ^ xp);
      mpp_hi &= ~((uint32_t)(bp >> 32) ^ xp);
    }
    cur = vqf_locate<T>(hn, vnext, mask, R, magic);
    const uint64_t Mpp = ((uint64_t)mpp_hi << 32) | mpp_lo;
    // count of my primary block if every earlier lane of the chunk took its primary
    uint32_t cp = L.kept ? cnt_p + __popcll(Mpp & lt) : 0u;
    const uint32_t pb = L.pb;
    uint32_t ab = pb, ao = L.po, ca = 0;
    uint64_t altmask = 0;
    // No lane at the threshold: every key of the chunk stays primary (a lane moves only when
    // its primary holds >= kThreshold elements, and with all earlier lanes primary it holds
    // cp).  This is most steps of a leaf (blocks fill towards ~0.85 x slots), and they skip
    // the alternate block entirely.
    if (bal(cp >= C::kThreshold) != 0) {  // (cp = 0 for a key not inserted)
      vqf_locate_alt<T>(L, R, magic, ab, ao);
      const uint32_t cnt_a = cnt.get(ab);
      // lanes with pb_j == my ab
      uint32_t mpa_lo = (uint32_t)keptmask, mpa_hi = (uint32_t)(keptmask >> 32);
      if constexpr (kLdsMatch) {
        atomicOr(mt + pb, L.kept ? mybit : 0ull);
        asm volatile("" ::: "memory");
        const uint64_t b = mt[ab];
        asm volatile("" ::: "memory");
        mt[pb] = 0;
        mpa_lo &= (uint32_t)b;
        mpa_hi &= (uint32_t)(b >> 32);
      }
#pragma unroll
      for (int j = 0; j < (kLdsMatch ? 0 : NBITS); ++j) {
        const uint32_t xp = (uint32_t)__builtin_amdgcn_sbfe((int32_t)pb, j, 1);
        const uint32_t xa = (uint32_t)__builtin_amdgcn_sbfe((int32_t)ab, j, 1);
        const uint64_t bp = __ballot(xp != 0);
        mpa_lo &= ~((uint32_t)bp ^ xa);
        mpa_hi &= ~((uint32_t)(bp >> 32) ^ xa);
      }
      const uint64_t Mpa = ((uint64_t)mpa_hi << 32) | mpa_lo;
      ca = L.kept ? cnt_a + __popcll(Mpa & lt) : 0u;
      // Decisions in insertion order, resolved in rounds.  Lane k's choice depends only on
      // the counts of its two blocks, which an earlier lane j changes only by moving
      // (pb_j -> ab_j) and only if {pb_j, ab_j} meets {pb_k, ab_k}.  So every undecided lane
      // with no undecided earlier lane sharing a block is final now: all of them decide in
      // one round and the movers' effects are applied to later lanes with four masked
      // popcounts.
      uint64_t U = bal(L.kept && pb != ab);  // blocks differ (vqf_insert alt test)
      // (cp >= threshold and ca < cp) as one compare: max(ca, threshold - 1) < cp
      uint64_t F = bal(max(ca, C::kThreshold - 1) < cp) & U;
      if (F != 0) {
        // lanes whose alternate block is my primary / my alternate
        uint32_t map_lo = (uint32_t)keptmask, map_hi = (uint32_t)(keptmask >> 32);
        uint32_t maa_lo = map_lo, maa_hi = map_hi;
        if constexpr (kLdsMatch) {
          atomicOr(mt + ab, L.kept ? mybit : 0ull);
          asm volatile("" ::: "memory");
          const uint64_t a = mt[pb], b = mt[ab];
          asm volatile("" ::: "memory");
          mt[ab] = 0;
          map_lo &= (uint32_t)a;
          map_hi &= (uint32_t)(a >> 32);
          maa_lo &= (uint32_t)b;
          maa_hi &= (uint32_t)(b >> 32);
        }
#pragma unroll
        for (int j = 0; j < (kLdsMatch ? 0 : NBITS); ++j) {
          const uint32_t xp = (uint32_t)__builtin_amdgcn_sbfe((int32_t)pb, j, 1);
          const uint32_t xa = (uint32_t)__builtin_amdgcn_sbfe((int32_t)ab, j, 1);
          const uint64_t ba = __ballot(xa != 0);
          const uint32_t bl = (uint32_t)ba, bh = (uint32_t)(ba >> 32);
          map_lo &= ~(bl ^ xp);
          map_hi &= ~(bh ^ xp);
          maa_lo &= ~(bl ^ xa);
          maa_hi &= ~(bh ^ xa);
        }
        const uint64_t Map = ((uint64_t)map_hi << 32) | map_lo;
        const uint64_t Maa = ((uint64_t)maa_hi << 32) | maa_lo;
        const uint64_t conf = (Mpp | Mpa | Map | Maa) & lt;  // earlier lanes sharing a block
        // a lane whose primary cannot reach the threshold even if every earlier lane with
        // its alternate there moved in stays primary: it is decided already
        U &= bal(cp + (uint32_t)__popcll(Map & lt) >= C::kThreshold);
        F &= U;
        while (F != 0) {
          const uint64_t res = bal((conf & U) == 0) & U;
          const uint64_t A = res & F;
          altmask |= A;
          U &= ~res;
          const uint64_t Al = A & lt;
          cp = cp + (uint32_t)__popcll(Map & Al) - (uint32_t)__popcll(Mpp & Al);
          ca = ca + (uint32_t)__popcll(Maa & Al) - (uint32_t)__popcll(Mpa & Al);
          F = bal(max(ca, C::kThreshold - 1) < cp) & U;
        }
      }
    }
    const uint32_t chosen = sel_mask(altmask, ab, pb);
    const uint32_t cho = sel_mask(altmask, ao, L.po);
    const uint32_t r = sel_mask(altmask, ca, cp);  // count of the chosen block when this key is inserted
    fail |= (uint32_t)(bal(L.kept && r >= C::kSlots) != 0);
    pend_ptr = base + lane < n ? rec + base + lane : sink;
    if constexpr (kCompact) {
      pend_val = (L.kept && r < C::kSlots) ? (chosen << 21) | (r << 15) | (cho << T) | L.tag
                                           : 0xffffffffu;
    } else {
      const uint32_t slot_hi = (L.kept && r < C::kSlots)
                                   ? (uint32_t)((sg.block_base + chosen) * 64 + r) : 0xffffffffu;
      pend_val = ((uint64_t)slot_hi << 32) | ((cho << T) | L.tag) | (T == 16 ? 0x80000000u : 0u);
    }
    cnt.add(chosen, L.kept ? 1u : 0u);
  };

  KB kv0{}, kvA{}, kvB{};
  if constexpr (kVqfPrefetch<MODE>) {
    if (n > 0) {
      if constexpr (MODE == kKeyVar) {
        KB first{};
        const uint64_t g0 = sg.key_begin + min(lane, n - 1);
        first.noff = offs[g0];
        first.nlen = (uint32_t)(offs[g0 + 1] - first.noff);
        vqf_load_var(keys, offs, sg.key_begin + min(lane + 64, n - 1), first, kv0, vr);
        vqf_load_var(keys, offs, sg.key_begin + min(lane + 128, n - 1), kv0, kvA, vr);
      } else {
        vqf_load_key<MODE>(keys, sg.key_begin + min(lane, n - 1), kv0);
        vqf_load_key<MODE>(keys, sg.key_begin + min(lane + 64, n - 1), kvA);
      }
    }
  }
  VqfLoc cur = vqf_locate<T>(lane < n ? vqf_key_hash<MODE>(keys, offs, stride, sg.key_begin + lane, kv0) : 0,
                             lane < n, mask, R, magic);
  for (uint32_t base = 0; base < n; base += 128) {
    step(base, cur, kvA, kvB);
    if (base + 64 >= n) break;
    step(base + 64, cur, kvB, kvA);
  }
  if (pend_ptr != sink) *pend_ptr = pend_val;
  asm volatile("" ::: "memory");
  // the final per-block counts feed only the unfused place path (the fused one recounts in
  // LDS): 4 bytes per 128-byte block record, so skip them when they are not read
  if (!fused && CNT != kCntGlobal) {  // (global counts are in the block records already)
    for (uint32_t b = lane; b < nb; b += 64) {
      const uint32_t c = cnt.get(b);
      vqf_count(ws, sg.block_base + b) = c < C::kSlots ? c : C::kSlots;
    }
  }
  if (lane == 0) ws.nelts[seg_index] = vqf_nelts_word(nelts, fail);
}

// variable-length keys: one past the key array's last byte (the batch's last leaf ends it)
template <int MODE>
__device__ inline uint64_t vqf_key_end(const uint64_t* offs, const tkv_amq_segment* segs, uint32_t n_segs)
{
  if constexpr (MODE != kKeyVar) return 0;
  const tkv_amq_segment& last = segs[n_segs - 1];
  return offs[last.key_begin + last.n_keys];
}

template <int T, int MODE>
__device__ inline void vqf_decide_dispatch(const uint8_t* keys, const uint64_t* offs,
                                           uint32_t stride, const tkv_amq_segment& sg,
                                           uint32_t seg_index, VqfWorkspace ws, uint64_t* recs,
                                           uint32_t* cnt, bool match_lds, bool compact_ok,
                                           uint64_t key_end)
{
  // kVqfMaxLdsBlocks = 16384 -> at most 14 block-id bits
  if (sg.n_blocks <= 512) {
    if (T == 8 && compact_ok) {
      if (match_lds) vqf_decide_body<T, MODE, 9, true, T == 8>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
      else vqf_decide_body<T, MODE, 9, false, T == 8>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
    } else {
      if (match_lds) vqf_decide_body<T, MODE, 9, true, false>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
      else vqf_decide_body<T, MODE, 9, false, false>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
    }
  } else if (match_lds) {
    vqf_decide_body<T, MODE, 14, true, false>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
  } else {
    vqf_decide_body<T, MODE, 14, false, false>(keys, offs, stride, sg, seg_index, ws, recs, cnt, compact_ok, key_end);
  }
}

// (74 VGPRs, 6 waves per SIMD.  Forcing 7 or 8 waves per SIMD spills -- 12 / 48 bytes per
// lane for 16-byte keys -- and ran slower: 498 -> 544 / 546 us per 100M keys, variable-length
// keys 986 -> 1241 / 1590 us; profiles/r04/experiments/vqf_decide_waves_per_eu.txt)
template <int MODE>
__global__ __launch_bounds__(64) void vqf_decide(const uint8_t* __restrict__ keys,
                                                 const uint64_t* __restrict__ offs, uint32_t stride,
                                                 const tkv_amq_segment* __restrict__ segs,
                                                 void* ws_base, uint64_t ws_bytes, uint32_t n_segs,
                                                 int flags)
{
  const bool match_lds = flags & 1, compact_ok = flags & 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t s_cnt[];
  const tkv_amq_segment sg = segs[blockIdx.x];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  vqf_mark_build(ws, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, blockIdx.x)) return;
  uint64_t* recs = vqf_records(ws, segs, n_segs);
  const uint64_t key_end = vqf_key_end<MODE>(offs, segs, n_segs);
  if (sg.tag_bits == 8)
    vqf_decide_dispatch<8, MODE>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_cnt, match_lds, compact_ok, key_end);
  else if (sg.tag_bits == 16)
    vqf_decide_dispatch<16, MODE>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_cnt, match_lds, compact_ok, key_end);
  else if (threadIdx.x == 0)
    ws.nelts[blockIdx.x] = 0;  // no filter (bits_per_key 0)
}

// Batches with a leaf past kVqfMaxLdsBlocks (VqfCountMode kCntU8 / kCntGlobal): a kernel of
// their own, so the wider block-id matches do not raise vqf_decide's registers (and cut its
// waves per SIMD) for every batch.
template <int MODE, int CNT>
__global__ __launch_bounds__(64) void vqf_decide_big(const uint8_t* __restrict__ keys,
                                                     const uint64_t* __restrict__ offs, uint32_t stride,
                                                     const tkv_amq_segment* __restrict__ segs,
                                                     void* ws_base, uint64_t ws_bytes, uint32_t n_segs)
{
  constexpr int NBITS = CNT == kCntU8 ? 18 : 24;  // kVqfU8LdsBlocks / kVqfMaxBlocks
  extern __shared__ __attribute__((aligned(16))) uint32_t s_cnt[];
  const tkv_amq_segment sg = segs[blockIdx.x];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  vqf_mark_build(ws, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, blockIdx.x)) return;
  uint64_t* recs = vqf_records(ws, segs, n_segs);
  const uint64_t key_end = vqf_key_end<MODE>(offs, segs, n_segs);
  if (sg.tag_bits == 8)
    vqf_decide_body<8, MODE, NBITS, false, false, CNT>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_cnt, false, key_end);
  else if (sg.tag_bits == 16)
    vqf_decide_body<16, MODE, NBITS, false, false, CNT>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_cnt, false, key_end);
  else if (threadIdx.x == 0)
    ws.nelts[blockIdx.x] = 0;
}

// the fused place's LDS image (vqf_place_fused_body; vqf_ring_place writes it from the decider)
constexpr uint32_t kFusedLdsBudget = 160 * 1024;  // 1,241 blocks per workgroup (one per CU at the top)
constexpr uint32_t kFusedMaxParts = 4;            // workgroups per leaf: leaves up to 4,964 blocks
constexpr uint32_t kFusedRegionWords = 33;
constexpr uint32_t kFusedCountWord = 32;

// ---------------------------------------------------------------------------------------
// Small batches: vqf_decide_ring.  A lone leaf's decide is a serial chain of 64-key steps, so
// a batch too small to fill the chip is bound by that chain's latency.  Here one 512-thread
// workgroup per leaf splits the work: waves 1..7 (producers) hash and locate the leaf's
// chunks of 64 keys in order and compute every chunk's four lane-match masks (lanes with
// my primary as primary / as alternate, with my alternate as primary / as alternate) with
// ballots; wave 0 (the decider) replays the insertion order from them.  Per step the
// decider reads the chunk's slot and the two block counts in one LDS round trip and runs
// only the decision logic of vqf_decide_body.  Chunks pass through a ring of kRingSlots slots:
// a producer fills a slot when the decider has freed it and then publishes it (ready word =
// chunk + 1); the decider frees a slot once its words are in registers.  LDS operations of
// a CU take effect in issue order per wave, so a decider that sees the ready word written
// after the slot's words reads those words.  ~70 KB of LDS: two workgroups per CU.
// A batch with a leaf of more than kRingMaxBlocks blocks takes vqf_decide instead.
// Same decisions, same key records as vqf_decide (test_gpu_parity: small and large batches).
constexpr uint32_t kRingThreads = 512;
constexpr uint32_t kRingProducers = kRingThreads / 64 - 1;
constexpr uint32_t kRingSlots = 10;
constexpr uint32_t kRingPlaceSlots = 8;  // vqf_ring_place, one workgroup per CU
// A slot holds, per lane of its chunk, these u32 words (plane w at [w * 64 + lane]), all the
// producers can know, so the decider's step is the decision and nothing else:
enum VqfSlotWord : uint32_t {
  kSwPb4 = 0,            // LDS address of the primary block's count (a key not inserted: the
                         // dummy block n_blocks, whose count stays 0)
  kSwAb4 = 1,            // LDS address of the alternate block's count (dummy likewise)
  kSwRanks = 2,          // r_pp | r_pa << 8 | r_ap << 16 | kept << 24 | eligible << 25
  kSwRecP = 3,           // the key's record with its primary block, rank bits 0 (VqfRecMode)
  kSwRecA = 4,           // ... with its alternate block
  kSwImgP = 5,           // kRecImage: LDS address of the primary block's image region
  kSwMpp = 6,            // lo, hi: earlier kept lanes with my primary as their primary
  kSwMpa = kSwMpp + 2,   // ... with my alternate as their primary
  kSwMap = kSwMpa + 2,   // ... with my primary as their alternate
  kSwMaa = kSwMap + 2,   // ... with my alternate as their alternate
  kSwConf = kSwMaa + 2,  // union of the four: earlier lanes sharing a block
  kSwCount = kSwConf + 2
};
// r_pp / r_pa / r_ap: popcounts of Mpp / Mpa / Map (0 for a key not inserted); eligible: kept
// and its two blocks differ (vqf_insert's alternate test).  The decider uses the LDS addresses
// as they are (ds_read / ds_add with no address arithmetic).
constexpr uint32_t kRingSlotU32 = kSwCount * 64;
static_assert(kSwCount == 16, "a 4 KiB slot");

// LDS byte addresses (the low word of a generic pointer to LDS is its LDS address)
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) uint16_t lds_u16_t;
__device__ inline uint32_t lds_addr(const void* p)
{
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}
__device__ inline uint32_t lds_rd(uint32_t a)
{
  return *reinterpret_cast<const lds_u32_t*>((uintptr_t)a);
}
__device__ inline void lds_add(uint32_t a, uint32_t v)
{
  __atomic_fetch_add(reinterpret_cast<lds_u32_t*>((uintptr_t)a), v, __ATOMIC_RELAXED);
}
constexpr uint32_t kRingMaxBlocks = 2048;
// ring | ready[NS] | freed (+1 spare): the count table starts here
__host__ __device__ constexpr inline uint32_t ring_base_bytes(uint32_t NS)
{
  return NS * kRingSlotU32 * 4 + 4 * NS + 8;
}
constexpr uint32_t kRingBaseBytes = ring_base_bytes(kRingSlots);
constexpr uint32_t kRingLdsBytes = kRingBaseBytes + 4 * (kRingMaxBlocks + 1);
constexpr uint32_t kVqfRingMaxSegs = 768;
constexpr uint32_t kVqfRingMaxSegsOther = 4096;  // keys other than 16 bytes (tkv_amq_build)
static_assert(kRingLdsBytes <= 160 * 1024 / 3, "three workgroups per CU");

// Ring hand-off words: relaxed workgroup-scope atomics, so they stay LDS operations (a
// volatile access through a generic pointer is compiled as a system-coherent flat access).
__device__ inline uint32_t lds_load_relaxed(uint32_t* p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline void lds_store_relaxed(uint32_t* p, uint32_t v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Where vqf_ring_decide puts each key's (block, rank, bucket, tag):
//   kRecWide     8-byte key records in the workspace (vqf_decide_body's form)
//   kRecCompact  4-byte key records (T = 8, <= 512 blocks)
//   kRecImage    straight into the leaf's LDS image, entry at [block][rank] (vqf_ring_place:
//                the place's sort then runs in the same workgroup; no key records at all)
enum VqfRecMode : int { kRecWide = 0, kRecCompact = 1, kRecImage = 2 };

// kSwRecP / kSwRecA by record mode: compact: block << 21 | bucket << 8 | tag (~0 for a key not
// inserted: OR-ing the rank keeps it ~0); wide / image: the entry (bucket << T | tag; wide
// sets bit 31 for 32-bit entries)
template <int T, int REC>
__device__ inline uint32_t vqf_ring_rec(bool kept, uint32_t block, uint32_t bucket, uint32_t tag)
{
  if constexpr (REC == kRecCompact) return kept ? (block << 21) | (bucket << 8) | tag : ~0u;
  else if constexpr (REC == kRecWide) return (bucket << T) | tag | (T == 16 ? 0x80000000u : 0u);
  else return (bucket << T) | tag;
}

// kTbl (vqf_ring_place, leaves of <= kRingTblBlocks blocks): the four lane-match masks from two
// LDS tables of 64-bit lane masks per producer (P[block]: lanes with that primary, A[block]:
// with that alternate; each lane ORs its bit into P[pb] and A[ab], reads P[pb], P[ab], A[pb],
// A[ab], clears its two entries): eight LDS operations instead of ~12 VALU per block-id bit,
// which made the producers, not the decider, set a lone leaf's time.  Six producers (waves 1-3
// and 5-7): wave 4 idles so the decider has its SIMD to itself (a workgroup's waves are
// placed on the CU's four SIMDs in turn).  Otherwise seven producers and block-id ballots.
constexpr uint32_t kRingTblBlocks = 512;
constexpr uint32_t kRingTblProducers = 7;

template <int T, int MODE, int NBITS, int REC, bool kTbl, uint32_t NS>
__device__ __attribute__((always_inline)) void vqf_ring_produce(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs,
                                 uint32_t stride, const tkv_amq_segment& sg, uint32_t* ring,
                                 uint32_t* ready, uint32_t* freed, uint64_t* tbl, uint64_t key_end,
                                 const uint32_t* cnt, const uint32_t* img)
{
  const uint32_t cnt_base = lds_addr(cnt), img_base = lds_addr(img);
  using C = Vqf<T>;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x / 64;
  // (with six table producers wave 4 idles: the decider's SIMD without a producer)
  if (kTbl && kRingTblProducers == 6 && wave == 4) return;
  const uint32_t w = (kTbl && kRingTblProducers == 6) ? (wave < 4 ? wave - 1 : wave - 2) : wave - 1;
  const uint32_t n = sg.n_keys, nb = sg.n_blocks;
  const uint32_t n_chunks = (n + 63) / 64;
  const uint64_t R = (uint64_t)nb * C::kBuckets;
  const uint64_t magic = sg.mod_magic;
  const uint64_t mask = ~0ull << sg.hash_val_shift;  // filter_builder.hpp:187
  const uint64_t lt = lanemask_lt();
  // (variable-length keys are read where they are hashed here: kVqfRingPrefetch)
  using KB = typename std::conditional<kVqfRingPrefetch<MODE>, VqfKeyBuf<MODE>, VqfKeyBuf<kKeyFixed>>::type;
  // a producer's next three chunks of keys are in flight (one chunk's load latency is longer
  // than the time to produce it); the loop is unrolled by three so the buffers rotate
  constexpr uint32_t kDepth = 3, kStep = kTbl ? kRingTblProducers : kRingProducers;
  uint64_t* const tp = tbl + (kTbl ? w * 2 * (nb + 1) : 0);  // this producer's P, then A
  uint64_t* const ta = tp + nb + 1;
  auto load = [&](uint32_t q, KB& kv) {  // clamped, not skipped: a fixed count in flight
    if constexpr (kVqfRingPrefetch<MODE>) vqf_load_key<MODE>(keys, sg.key_begin + min(q * 64 + lane, n - 1), kv);
  };
  // variable-length keys: the leaf's bytes through a buffer resource (KeyWin)
  VarRsrc vr{};
  if constexpr (MODE == kKeyVar)
    if (n > 0) vr = var_rsrc(keys, offs[sg.key_begin], offs[sg.key_begin + n], key_end);
  auto produce = [&](uint32_t q, KB& kv) {
    const uint32_t i = q * 64 + lane;
    const bool valid = i < n;
    VqfLoc l;
    uint32_t ab, ao;
    if constexpr (MODE == kKeyLoc) {
      vqf_loc_decode(kv.v, valid, l, ab, ao);
      load(q + kDepth * kStep, kv);
    } else {
    uint64_t h = 0;
    if constexpr (MODE == kKey16 || MODE == kKey24) {
      h = valid ? vqf_key_hash<MODE>(keys, offs, stride, sg.key_begin + i, kv) : 0;
    } else if constexpr (MODE == kKeyVar) {
      const uint64_t gi = sg.key_begin + min(i, n - 1), o0 = offs[gi];
      const uint32_t len = (uint32_t)(offs[gi + 1] - o0);
      if (vr.nrec) {  // (uniform per leaf; every lane loads its window, valid or not)
        KeyWin kw;
        key_win_load(vr, (uint32_t)(o0 - vr.base), kw);
        if (valid && len < 32) {
          uint64_t l[3];
          uint32_t t4, tb;
          key_win_parts(kw, len, l, t4, tb);
          h = XxhShort(len, l, t4, tb).finish(kVqfHashSeed + kP5);
        } else if (valid) {
          h = xxh64_bytes(keys + o0, len, kVqfHashSeed);
        }
      } else {
        h = valid ? hash_key<MODE>(keys, offs, stride, gi, kVqfHashSeed) : 0;
      }
    } else {
      h = valid ? hash_key<MODE>(keys, offs, stride, sg.key_begin + i, kVqfHashSeed) : 0;
    }
    load(q + kDepth * kStep, kv);
    l = vqf_locate<T>(h, valid, mask, R, magic);
    vqf_locate_alt<T>(l, R, magic, ab, ao);
    }
    const uint64_t keptmask = __ballot(l.kept);
    uint32_t pp_lo = (uint32_t)keptmask, pp_hi = (uint32_t)(keptmask >> 32);
    uint32_t pa_lo = pp_lo, pa_hi = pp_hi, ap_lo = pp_lo, ap_hi = pp_hi, aa_lo = pp_lo, aa_hi = pp_hi;
    if constexpr (kTbl) {
      // (LDS operations of a wave complete in order: every lane's OR lands before any read,
      // every read before any clear; lanes without a key OR 0, so the masks hold kept lanes)
      const uint64_t mybit = l.kept ? 1ull << lane : 0ull;
      atomicOr(reinterpret_cast<unsigned long long*>(tp + l.pb), mybit);
      atomicOr(reinterpret_cast<unsigned long long*>(ta + ab), mybit);
      asm volatile("" ::: "memory");
      const uint64_t xpp = tp[l.pb], xpa = tp[ab], xap = ta[l.pb], xaa = ta[ab];
      asm volatile("" ::: "memory");
      tp[l.pb] = 0;
      ta[ab] = 0;
      pp_lo &= lo32(xpp);
      pp_hi &= hi32(xpp);
      pa_lo &= lo32(xpa);
      pa_hi &= hi32(xpa);
      ap_lo &= lo32(xap);
      ap_hi &= hi32(xap);
      aa_lo &= lo32(xaa);
      aa_hi &= hi32(xaa);
    }
#pragma unroll
    for (int j = 0; j < (kTbl ? 0 : NBITS); ++j) {
      const uint32_t xp = (uint32_t)__builtin_amdgcn_sbfe((int32_t)l.pb, j, 1);  // 0 or ~0
      const uint32_t xa = (uint32_t)__builtin_amdgcn_sbfe((int32_t)ab, j, 1);
      const uint64_t bp = __ballot(xp != 0), ba = __ballot(xa != 0);
      const uint32_t bpl = (uint32_t)bp, bph = (uint32_t)(bp >> 32);
      const uint32_t bal = (uint32_t)ba, bah = (uint32_t)(ba >> 32);
      pp_lo &= ~(bpl ^ xp);
      pp_hi &= ~(bph ^ xp);
      pa_lo &= ~(bpl ^ xa);
      pa_hi &= ~(bph ^ xa);
      ap_lo &= ~(bal ^ xp);
      ap_hi &= ~(bah ^ xp);
      aa_lo &= ~(bal ^ xa);
      aa_hi &= ~(bah ^ xa);
    }
    // only earlier lanes matter to a lane (later lanes' moves cannot change its counts)
    const uint64_t Mpp = mk64(pp_lo, pp_hi) & lt, Mpa = mk64(pa_lo, pa_hi) & lt;
    const uint64_t Map = mk64(ap_lo, ap_hi) & lt, Maa = mk64(aa_lo, aa_hi) & lt;
    const uint64_t conf = Mpp | Mpa | Map | Maa;
    const bool kept = l.kept;
    const uint32_t ranks = kept ? (uint32_t)__popcll(Mpp) | ((uint32_t)__popcll(Mpa) << 8) |
                                      ((uint32_t)__popcll(Map) << 16) | (1u << 24) |
                                      (l.pb != ab ? 1u << 25 : 0u)
                                : 0u;
    const uint32_t pbk = kept ? l.pb : nb;
    const uint32_t pb4 = cnt_base + 4 * pbk, ab4 = cnt_base + 4 * (kept ? ab : nb);
    const uint32_t imgP = img_base + 4 * kFusedRegionWords * pbk;
    const uint32_t recP = vqf_ring_rec<T, REC>(kept, l.pb, l.po, l.tag);
    const uint32_t recA = vqf_ring_rec<T, REC>(kept, ab, ao, l.tag);
    // the slot is free once the decider has taken chunk q - NS
    while (q >= NS && lds_load_relaxed(freed) < q - NS + 1) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");  // no slot write above the wait, none below the publish
    uint32_t* slot = ring + (q % NS) * kRingSlotU32 + lane;
    slot[64 * kSwPb4] = pb4;
    slot[64 * kSwAb4] = ab4;
    slot[64 * kSwRanks] = ranks;
    slot[64 * kSwRecP] = recP;
    slot[64 * kSwRecA] = recA;
    slot[64 * kSwImgP] = imgP;
    slot[64 * kSwMpp] = lo32(Mpp);
    slot[64 * (kSwMpp + 1)] = hi32(Mpp);
    slot[64 * kSwMpa] = lo32(Mpa);
    slot[64 * (kSwMpa + 1)] = hi32(Mpa);
    slot[64 * kSwMap] = lo32(Map);
    slot[64 * (kSwMap + 1)] = hi32(Map);
    slot[64 * kSwMaa] = lo32(Maa);
    slot[64 * (kSwMaa + 1)] = hi32(Maa);
    slot[64 * kSwConf] = lo32(conf);
    slot[64 * (kSwConf + 1)] = hi32(conf);
    asm volatile("" ::: "memory");
    if (lane == 0) lds_store_relaxed(ready + q % NS, q + 1);
  };
  if (w >= n_chunks) return;
  KB kv0{}, kv1{}, kv2{};
  if constexpr (!kVqfRingPrefetch<MODE>) {
    // other key shapes are read where they are hashed: no buffers to rotate, and one copy of
    // the (long) hash code keeps the kernel at three workgroups per CU
    for (uint32_t q = w; q < n_chunks; q += kStep) produce(q, kv0);
    return;
  }
  load(w, kv0);
  load(w + kStep, kv1);
  load(w + 2 * kStep, kv2);
  for (uint32_t q = w; q < n_chunks; q += kDepth * kStep) {
    produce(q, kv0);
    if (q + kStep >= n_chunks) break;
    produce(q + kStep, kv1);
    if (q + 2 * kStep >= n_chunks) break;
    produce(q + 2 * kStep, kv2);
  }
}

#ifdef TKV_DIAG_RING
// per step of leaf 0: wait, count read, decision, spins | slow << 32; then (g_diag[4 * 4096 +])
// the kernel's stamps: start, decider done, place sort done
__device__ uint64_t g_diag[4 * 4096 + 8];
extern "C" int tkv_amq_diag_read(void* host)
{
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), sizeof(g_diag)) == hipSuccess ? 0 : 13;
}
__device__ inline void diag_stamp(int i)
{
  if (blockIdx.x == 0 && threadIdx.x == 0) g_diag[4 * 4096 + i] = __builtin_amdgcn_s_memtime();
}
#else
__device__ inline void diag_stamp(int) {}
#endif

// NS steps of the decider's loop with compile-time slot indices (no modulo, no slot address
// arithmetic): f(c + I, integral_constant<I>) for I = 0.. while c + I < n
template <uint32_t I, uint32_t NS, typename F>
__device__ inline bool ring_unroll(F& f, uint32_t c, uint32_t n)
{
  if constexpr (I == NS) {
    return true;
  } else {
    if (c + I >= n) return false;
    f(c + I, std::integral_constant<uint32_t, I>{});
    return ring_unroll<I + 1, NS>(f, c, n);
  }
}

// The decider wave.  Per 64-key step: the two block counts (one LDS round trip at the LDS
// addresses the producers wrote; the next slot is read a step ahead), then -- in the steps
// where no lane's primary has reached the threshold, most of a leaf -- a handful of
// instructions: every key takes its primary at rank cp, its record is recP | cp (kRecImage:
// its entry lands at imgP + cp).  Otherwise the rounds of vqf_decide_body, with every mask at
// hand.  The loop is unrolled by the ring's NS slots, so every slot offset is an immediate.
// (always inlined: out of line, the unrolled loop of the larger instantiations became a call
// with a scratch frame -- 768 leaves of variable-length keys 253 -> 384 us)
template <int T, int REC, uint32_t NS>
__device__ __attribute__((always_inline)) void vqf_ring_decide(const tkv_amq_segment& sg, uint32_t seg_index, VqfWorkspace ws,
                                uint64_t* __restrict__ recs, const uint32_t* ring,
                                uint32_t* ready, uint32_t* freed, uint32_t* cnt, bool fused,
                                uint8_t* img8, uint32_t* img_sink, uint32_t* s_nelts)
{
  using C = Vqf<T>;
  static_assert(NS % 2 == 0, "two slot register sets alternate");
  constexpr bool kCompact = REC == kRecCompact;
  constexpr uint32_t kE = sizeof(typename C::Entry);
  const uint32_t lane = threadIdx.x;
  const uint32_t n = sg.n_keys, nb = sg.n_blocks;
  const uint32_t n_chunks = (n + 63) / 64;
  using Rec = typename std::conditional<kCompact, uint32_t, uint64_t>::type;
  Rec* rec = reinterpret_cast<Rec*>(recs + sg.key_begin);
  Rec* const sink = reinterpret_cast<Rec*>(ws.sink);  // see vqf_decide_body
  Rec* pend_ptr = sink;
  Rec pend_val = 0;
  const uint32_t cnt_base = lds_addr(cnt), img_base = lds_addr(img8);
  const uint32_t sink_addr = lds_addr(img_sink);  // a full block's key writes its entry here
  // Two slot register sets alternate (even / odd steps), so no step copies the prefetched words.
  struct Slot {
    uint32_t rdy, pb4, ab4, ranks, recP, recA, imgP;
    uint64_t pp, pa, ap, aa, conf;
  };
  auto fetch = [&](uint32_t q, Slot& S) {  // slot q (compile-time in the unrolled loop)
    const uint32_t* slot = ring + q * kRingSlotU32 + lane;
    S.rdy = lds_load_relaxed(ready + q);
    asm volatile("" ::: "memory");  // the slot words are read after the ready word
    S.pb4 = slot[64 * kSwPb4];
    S.ab4 = slot[64 * kSwAb4];
    S.ranks = slot[64 * kSwRanks];
    S.recP = slot[64 * kSwRecP];
    S.recA = slot[64 * kSwRecA];
    S.imgP = slot[64 * kSwImgP];
    S.pp = mk64(slot[64 * kSwMpp], slot[64 * (kSwMpp + 1)]);
    S.pa = mk64(slot[64 * kSwMpa], slot[64 * (kSwMpa + 1)]);
    S.ap = mk64(slot[64 * kSwMap], slot[64 * (kSwMap + 1)]);
    S.aa = mk64(slot[64 * kSwMaa], slot[64 * (kSwMaa + 1)]);
    S.conf = mk64(slot[64 * kSwConf], slot[64 * (kSwConf + 1)]);
  };
  Slot A, B;
  auto step = [&](uint32_t c, auto I) {
    constexpr uint32_t q = decltype(I)::value;
    Slot& S = q % 2 == 0 ? A : B;
    Slot& next = q % 2 == 0 ? B : A;
    asm volatile("; ring step %0" ::"n"(q));  // (keeps the copies distinct)
#ifdef TKV_DIAG_RING
    const uint64_t d0 = __builtin_amdgcn_s_memtime();
    uint32_t spins = 0;
#endif
    while (S.rdy != c + 1) {
      __builtin_amdgcn_s_sleep(1);
      fetch(q, S);
#ifdef TKV_DIAG_RING
      ++spins;
#endif
    }
#ifdef TKV_DIAG_RING
    const uint64_t d1 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t cnt_p = lds_rd(S.pb4);
    const uint32_t cnt_a = lds_rd(S.ab4);
#ifdef TKV_DIAG_RING
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t d2 = __builtin_amdgcn_s_memtime();
#endif
    // LDS operations complete in issue order: the prefetch goes after the count reads, so
    // waiting for the counts does not wait for it.  Neither the hand-off write nor the
    // prefetch is skipped (every lane writes the same word; after the last chunk the prefetch
    // reads a slot no producer writes any more), so the compiler's count of LDS operations in
    // flight is exact on every path.
    asm volatile("" ::: "memory");
    lds_store_relaxed(freed, c + 1);  // the slot's words are in registers (LDS order)
    fetch((q + 1) % NS, next);
    if constexpr (REC != kRecImage) *pend_ptr = pend_val;
    const uint32_t ranks = S.ranks;
    // count of my primary if every earlier lane of the chunk takes its primary (a key not
    // inserted: 0, the dummy block's count and no ranks)
    uint32_t cp = cnt_p + (ranks & 0xffu);
    uint32_t chosen4 = S.pb4, r = cp, recx = S.recP;
    uint32_t dst = S.imgP + cp * kE;  // kRecImage: cp < threshold < slots on the fast path
#ifdef TKV_DIAG_RING
    uint64_t slow = 0;
#endif
    if (bal(cp >= C::kThreshold) != 0) {
#ifdef TKV_DIAG_RING
      slow = 1;
#endif
      uint32_t ca = cnt_a + ((ranks >> 8) & 0xffu);
      uint64_t U = bal(ranks >= (2u << 24));  // eligible
      // (cp >= threshold and ca < cp) as one compare: max(ca, threshold - 1) < cp
      uint64_t F = bal(max(ca, C::kThreshold - 1) < cp) & U;
      uint64_t altmask = 0;
      if (F != 0) {
        // a lane whose primary cannot reach the threshold even if every earlier lane with
        // its alternate there moved in stays primary: it is decided already
        U &= bal(cp + ((ranks >> 16) & 0xffu) >= C::kThreshold);
        F &= U;
        while (F != 0) {
          const uint64_t res = bal((S.conf & U) == 0) & U;
          const uint64_t Am = res & F;
          altmask |= Am;
          U &= ~res;
          cp = cp + (uint32_t)__popcll(S.ap & Am) - (uint32_t)__popcll(S.pp & Am);
          ca = ca + (uint32_t)__popcll(S.aa & Am) - (uint32_t)__popcll(S.pa & Am);
          F = bal(max(ca, C::kThreshold - 1) < cp) & U;
        }
      }
      // (selects on the mask itself: no per-lane bit test)
      chosen4 = sel_mask(altmask, S.ab4, S.pb4);
      r = sel_mask(altmask, ca, cp);  // a full block (r >= slots) shows in the final counts
      recx = sel_mask(altmask, S.recA, S.recP);
      if constexpr (REC == kRecImage)
        dst = r < C::kSlots ? img_base + (chosen4 - cnt_base) * kFusedRegionWords + r * kE : sink_addr;
    }
#ifdef TKV_DIAG_RING
    const uint64_t d3 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && blockIdx.x == 0 && c < 4096) {
      g_diag[4 * c] = d1 - d0;
      g_diag[4 * c + 1] = d2 - d1;
      g_diag[4 * c + 2] = d3 - d2;
      g_diag[4 * c + 3] = spins | (slow << 32);
    }
#endif
    const uint32_t kept = (ranks >> 24) & 1u;
    if constexpr (REC == kRecImage) {
      // entry at [chosen][r] of the image (vqf_place_fused_body's phase 1, done here); a key
      // not inserted lands in the dummy block's region, a full block's key on the sink word,
      // so every step issues the same LDS operations
      if constexpr (T == 8) *reinterpret_cast<lds_u16_t*>((uintptr_t)dst) = (uint16_t)recx;
      else *reinterpret_cast<lds_u32_t*>((uintptr_t)dst) = recx;
    } else {
      pend_ptr = c * 64 + lane < n ? rec + c * 64 + lane : sink;
      if constexpr (kCompact) {
        pend_val = r < C::kSlots ? recx | (r << 15) : 0xffffffffu;
      } else {
        const uint32_t slot_hi = (kept && r < C::kSlots)
                                     ? (uint32_t)((sg.block_base + (chosen4 - cnt_base) / 4) * 64 + r)
                                     : 0xffffffffu;
        pend_val = ((uint64_t)slot_hi << 32) | recx;
      }
    }
    lds_add(chosen4, kept);
  };
  if (n_chunks > 0) fetch(0, A);
  for (uint32_t c = 0; c < n_chunks; c += NS)
    if (!ring_unroll<0, NS>(step, c, n_chunks)) break;
  // a key found its block full (vqf_insert fails) iff that block's final count exceeds
  // slots; the element count is the sum of the counts (the dummy block's stays 0)
  uint32_t fail = 0, nelts = 0;
  for (uint32_t b = lane; b < nb; b += 64) {
    const uint32_t cb = cnt[b];
    fail |= cb > C::kSlots;
    nelts += cb;
  }
  if constexpr (REC != kRecImage) {
    if (pend_ptr != sink) *pend_ptr = pend_val;
  }
  asm volatile("" ::: "memory");
  if (REC != kRecImage && !fused) {  // block counts for the unfused place (as vqf_decide_body)
    for (uint32_t b = lane; b < nb; b += 64) {
      const uint32_t cb = cnt[b];
      vqf_count(ws, sg.block_base + b) = cb < C::kSlots ? cb : C::kSlots;
    }
  }
  const bool any_fail = __ballot(fail) != 0;
  nelts = wave_sum(nelts);
  if (lane == 0) {
    ws.nelts[seg_index] = vqf_nelts_word(nelts, any_fail);
    if constexpr (REC == kRecImage) *s_nelts = nelts;
  }
}

template <int T, int MODE, int REC, int NBITS, bool kTbl = false, uint32_t NS = kRingSlots>
__device__ __attribute__((always_inline)) void vqf_ring_body(const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                              const tkv_amq_segment& sg, uint32_t seg_index, VqfWorkspace ws,
                              uint64_t* recs, uint32_t* lds, bool fused, uint32_t cnt_words,
                              uint64_t key_end)
{
  uint32_t* ring = lds;
  uint32_t* ready = ring + NS * kRingSlotU32;
  uint32_t* freed = ready + NS;
  uint32_t* cnt = freed + 2;  // n_blocks + 1 counts: the last is the dummy block's
  // kRecImage: the image after the count table ((n_blocks + 1) regions: the dummy block's
  // last), then the sink word and the nelts word
  uint32_t* img = cnt + cnt_words;
  uint32_t* img_sink = img + (sg.n_blocks + 1) * kFusedRegionWords;
  // kTbl: the producers' match tables after the sink and nelts words (8-byte aligned)
  uint64_t* tbl = reinterpret_cast<uint64_t*>(img_sink + 2 + ((sg.n_blocks + 1) * kFusedRegionWords & 1));
  for (uint32_t i = threadIdx.x; i < NS + 1; i += kRingThreads) ready[i] = 0;  // + freed
  for (uint32_t b = threadIdx.x; b <= sg.n_blocks; b += kRingThreads) cnt[b] = 0;
  if constexpr (kTbl)
    for (uint32_t e = threadIdx.x; e < 2 * kRingTblProducers * (sg.n_blocks + 1); e += kRingThreads) tbl[e] = 0;
  __syncthreads();
  if (threadIdx.x < 64)
    vqf_ring_decide<T, REC, NS>(sg, seg_index, ws, recs, ring, ready, freed, cnt, fused,
                            reinterpret_cast<uint8_t*>(img), img_sink, img_sink + 1);
  else
    vqf_ring_produce<T, MODE, NBITS, REC, kTbl, NS>(keys, offs, stride, sg, ring, ready, freed, tbl, key_end,
                                                    cnt, img);
}

template <int MODE>
__global__ __launch_bounds__(kRingThreads) void vqf_decide_ring(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ offs, uint32_t stride,
    const tkv_amq_segment* __restrict__ segs, void* ws_base, uint64_t ws_bytes, uint32_t n_segs,
    int flags)
{
  const bool compact_ok = flags & 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
  const tkv_amq_segment sg = segs[blockIdx.x];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  vqf_mark_build(ws, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, blockIdx.x)) return;
  uint64_t* recs = vqf_records(ws, segs, n_segs);
  const uint64_t key_end = vqf_key_end<MODE>(offs, segs, n_segs);
  const uint32_t nb = sg.n_blocks;  // <= kRingMaxBlocks (tkv_amq_build)
  // compact records exactly where vqf_decide_dispatch writes them
  if (sg.tag_bits == 8) {
    if (nb <= 512 && compact_ok)
      vqf_ring_body<8, MODE, kRecCompact, 9>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_ring, compact_ok, 0, key_end);
    else if (nb <= 512)
      vqf_ring_body<8, MODE, kRecWide, 9>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_ring, compact_ok, 0, key_end);
    else
      vqf_ring_body<8, MODE, kRecWide, 11>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_ring, compact_ok, 0, key_end);
  } else if (sg.tag_bits == 16) {
    if (nb <= 512)
      vqf_ring_body<16, MODE, kRecWide, 9>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_ring, compact_ok, 0, key_end);
    else
      vqf_ring_body<16, MODE, kRecWide, 11>(keys, offs, stride, sg, blockIdx.x, ws, recs, s_ring, compact_ok, 0, key_end);
  } else if (threadIdx.x == 0) {
    ws.nelts[blockIdx.x] = 0;
  }
}

// One thread per key: moves the key's entry from its coalesced placement record into the
// block record (insertion rank = slot).  Fully parallel, so the partial-line writes overlap.
__global__ __launch_bounds__(256) void vqf_scatter(const tkv_amq_segment* __restrict__ segs,
                                                   void* ws_base, uint64_t ws_bytes, uint32_t n_segs,
                                                   uint64_t n_keys)
{
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const tkv_amq_segment& last = segs[n_segs - 1];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, ~0u)) return;
  if (i >= n_keys || i >= last.key_begin + last.n_keys) return;
  const uint64_t r = __builtin_nontemporal_load(vqf_records(ws, segs, n_segs) + i);
  const uint32_t hi = (uint32_t)(r >> 32), lo = (uint32_t)r;
  if (hi == 0xffffffffu) return;
  uint8_t* p = ws.temp + (uint64_t)(hi >> 6) * kVqfTempStride;
  const uint32_t rank = hi & 63u;
  if (lo >> 31) *reinterpret_cast<uint32_t*>(p + 4 * rank) = lo & 0x7fffffffu;
  else *reinterpret_cast<uint16_t*>(p + 2 * rank) = (uint16_t)lo;
}

// One thread per 64-byte VQF block: the block's records (bucket offset, tag) arrive in
// insertion order; vqf_insert appends each tag at the end of its bucket, so the final block
// is a stable counting sort by bucket offset.  Per-thread bucket counters are packed 4 per
// LDS dword (counts <= 48 never carry into the next byte), the exclusive prefix is a SWAR
// multiply, and the second pass takes each entry's slot with ds_add_rtn in insertion order.
constexpr uint32_t kPlaceThreads = 128;

template <int T>
__device__ void vqf_place_body(const tkv_amq_segment& sg, uint32_t seg_index, VqfWorkspace ws,
                               uint8_t* __restrict__ out, uint32_t* s_cnt, uint32_t* s_img,
                               uint32_t part, uint32_t parts)
{
  using C = Vqf<T>;
  using E = typename C::Entry;
  constexpr uint32_t kCntWords = (C::kBuckets + 3) / 4;  // 20 / 9
  constexpr uint32_t kCntStride = kCntWords | 1;         // odd stride: no bank conflicts
  constexpr uint32_t kImgStride = 17;
  constexpr uint32_t kRecWords = C::kSlots * sizeof(E) / 16;  // 16-byte loads per record: 6 / 7
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = sg.n_blocks;
  uint8_t* payload = out + sg.out_offset;

  if (part == 0 && tid < 5) {
    // PackedVqfFilter header (vqf_filter_page_view.hpp:79-94) + vqf_metadata
    uint64_t w0, w1;
    switch (tid) {
      case 0: w0 = kVqfMagic; w1 = sg.src_page_id; break;
      case 1: w0 = kVqfHashSeed; w1 = ~0ull << sg.hash_val_shift; break;
      case 2: w0 = 64ull * nb; w1 = T; break;
      case 3: w0 = (uint64_t)nb * C::kBuckets << T; w1 = nb; break;
      default: w0 = ws.nelts[seg_index] & kVqfNeltsMask; w1 = (uint64_t)nb * C::kSlots; break;
    }
    ulonglong2 v;
    v.x = w0;
    v.y = w1;
    reinterpret_cast<ulonglong2*>(payload)[tid] = v;
  } else if (part == 0 && tid < 9) {
    write_page_header(out, sg, kLayoutVqf, tid - 5);
  }

  uint32_t* cnt = s_cnt + tid * kCntStride;
  uint32_t* img = s_img + tid * kImgStride;
  uint4* dst_blocks = reinterpret_cast<uint4*>(payload + kVqfHeader + kVqfMetadata);

  for (uint32_t b = part * kPlaceThreads + tid; b < nb; b += parts * kPlaceThreads) {
    const uint8_t* rec = ws.temp + (sg.block_base + b) * kVqfTempStride;
    const uint32_t c = *reinterpret_cast<const uint32_t*>(rec + kVqfCountByte);
    uint4 rv[kRecWords];
#pragma unroll
    for (uint32_t q = 0; q < kRecWords; ++q) rv[q] = reinterpret_cast<const uint4*>(rec)[q];
    const E* ent = reinterpret_cast<const E*>(rv);

#pragma unroll
    for (uint32_t w = 0; w < kCntWords; ++w) cnt[w] = 0;
#pragma unroll
    for (uint32_t w = C::kMdBytes / 4; w < 16; ++w) img[w] = 0;
    // pass 1: bucket histogram.  Branch-free (slots >= c add 0 to bucket 0) so the LDS
    // atomics issue back to back instead of one waitcnt per predicated slot.
#pragma unroll
    for (uint32_t i = 0; i < C::kSlots; ++i) {
      const bool live = i < c;
      const uint32_t o = live ? (uint32_t)(ent[i] >> T) : 0u;
      atomicAdd(cnt + (o >> 2), live ? 1u << (8 * (o & 3)) : 0u);
    }
    // exclusive prefix over buckets (bytes): inclusive-in-dword = v * 0x01010101
    uint32_t run = 0;
#pragma unroll
    for (uint32_t w = 0; w < kCntWords; ++w) {
      const uint32_t v = cnt[w];
      const uint32_t incl = v * 0x01010101u;
      cnt[w] = (incl - v) + run * 0x01010101u;
      run += incl >> 24;
    }
    // pass 2: slot of each entry in insertion order; metadata zero at slot + offset.  Pass 1's
    // per-slot offsets and masks are recomputed, not kept live across the scan (as in
    // vqf_place_fused_sort: that kept the kernel at ~230 VGPRs)
#pragma unroll
    for (uint32_t q = 0; q < kRecWords; ++q)
      asm volatile("" : "+v"(rv[q].x), "+v"(rv[q].y), "+v"(rv[q].z), "+v"(rv[q].w));
    uint64_t md_lo = ~0ull, md_hi = T == 8 ? ~0ull : 0ull;
    // (branch-free as in pass 1; slots are distinct, so each tag is a plain byte/short store,
    // dead slots store into the image's pad dword)
    uint8_t* img8 = reinterpret_cast<uint8_t*>(img);
#pragma unroll
    for (uint32_t i = 0; i < C::kSlots; ++i) {
      const bool live = i < c;
      const uint32_t e = ent[i];
      const uint32_t o = live ? e >> T : 0u, tag = e & ((1u << T) - 1);
      const uint32_t old = atomicAdd(cnt + (o >> 2), live ? 1u << (8 * (o & 3)) : 0u);
      const uint32_t slot = (old >> (8 * (o & 3))) & 0xffu;
      const uint32_t z = slot + o;
      const uint64_t clr = live ? 1ull << (z & 63) : 0ull;
      if (z < 64) md_lo &= ~clr;
      else md_hi &= ~clr;
      const uint32_t byte = live ? C::kMdBytes + slot * (T / 8) : 64u;
      if constexpr (T == 8) {
        img8[byte] = (uint8_t)tag;
      } else {
        const uint16_t t16 = (uint16_t)tag;
        __builtin_memcpy(img8 + byte, &t16, 2);  // (memcpy: the image is read back as u32)
      }
    }
    if (c == 0) {  // an empty block keeps the init metadata: top bit clear
      if constexpr (T == 8) md_hi &= ~(1ull << 63);
      else md_lo &= ~(1ull << 63);
    }
    uint4 v0;
    v0.x = (uint32_t)md_lo;
    v0.y = (uint32_t)(md_lo >> 32);
    if constexpr (T == 8) {
      v0.z = (uint32_t)md_hi;
      v0.w = (uint32_t)(md_hi >> 32);
    } else {
      v0.z = img[2];
      v0.w = img[3];
    }
    uint4* dst = dst_blocks + (uint64_t)b * 4;
    dst[0] = v0;
#pragma unroll
    for (uint32_t q = 1; q < 4; ++q) {
      uint4 v;
      v.x = img[4 * q];
      v.y = img[4 * q + 1];
      v.z = img[4 * q + 2];
      v.w = img[4 * q + 3];
      dst[q] = v;
    }
  }
}

__global__ __launch_bounds__(kPlaceThreads) void vqf_place(const tkv_amq_segment* __restrict__ segs,
                                                           void* ws_base, uint64_t ws_bytes,
                                                           uint32_t n_segs, uint8_t* __restrict__ out,
                                                           uint32_t parts)
{
  __shared__ uint32_t s_cnt[kPlaceThreads * 21];
  __shared__ uint32_t s_img[kPlaceThreads * 17];
  const uint32_t seg = blockIdx.x / parts, part = blockIdx.x - seg * parts;
  const tkv_amq_segment sg = segs[seg];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, seg)) return;
  if (sg.tag_bits == 8) vqf_place_body<8>(sg, seg, ws, out, s_cnt, s_img, part, parts);
  else if (sg.tag_bits == 16) vqf_place_body<16>(sg, seg, ws, out, s_cnt, s_img, part, parts);
}

// Fused scatter + place for leaves whose block records fit in LDS (one workgroup per leaf, or
// up to kFusedMaxParts per leaf for a leaf of more than 1,241 blocks):
// the leaf's placement records stream in coalesced, each entry lands at [block][rank] of an
// LDS image (no partial-line global writes), then the per-block counting sort runs on it.
//
// LDS image: one 33-dword (132-byte) region per block -- an odd dword stride, so threads
// working on consecutive blocks at the same offset hit distinct banks.  Phase 1 writes the
// block's entries at [0, slots * entry bytes) and counts them in dword 32 (reading the counts
// vqf_decide could leave in the workspace instead cost 4-byte reads of 128-byte lines: +0.31 GB
// per 100M keys; on this path vqf_decide does not write them).  Phase 2 loads a block's
// entries and count into registers, then reuses the region: packed bucket counters
// in dwords [0, kCntWords), the tag image (bytes kMdBytes..63 of the output block) at
// kTagDword; the metadata stays in registers.  No per-thread scratch: a 402-block leaf takes
// 53 KB of LDS (registers, ~234 VGPRs, still hold the kernel to two workgroups per CU; forcing
// three spilled and ran 29% slower).
// (kFusedLdsBudget, kFusedMaxParts, kFusedRegionWords, kFusedCountWord: above vqf_decide_ring)

__host__ __device__ inline uint32_t vqf_fused_img_bytes(uint32_t nb)
{
  return nb * kFusedRegionWords * 4u;
}

__host__ __device__ inline uint32_t vqf_fused_lds_bytes(uint32_t max_nb)
{
  return vqf_fused_img_bytes(max_nb);
}

// Phase 2: one thread per block (NB > 1: NB blocks per thread interleaved; NB = 2 takes 173
// VGPRs, two workgroups per CU, and ran 9% slower: 0.760 vs 0.699 ms at 100M keys).  At 72
// VGPRs the LDS image sets three workgroups per CU.  Measured and not kept: a word-major image
// (dword w of block b at w * 480 + b, so the 32 threads of a bank group never conflict
// whatever bucket word they pick): 0.752 vs 0.730 ms -- bank conflicts (~59% of the LDS
// cycles, PMC) do not set this kernel's time.
template <int T, int NB, uint32_t NT>
__device__ void vqf_place_fused_sort(const tkv_amq_segment& sg, uint32_t nelts,
                                     uint8_t* __restrict__ out, uint32_t* lds,
                                     uint32_t lo, uint32_t nbl)
{
  using C = Vqf<T>;
  using E = typename C::Entry;
  constexpr uint32_t kCntWords = (C::kBuckets + 3) / 4;                // 20 / 9
  constexpr uint32_t kEntWords = C::kSlots * sizeof(E) / 4;            // 24 / 28
  constexpr uint32_t kTagDword = T == 8 ? 20 : 12;                     // tag image start
  constexpr uint32_t kTagWords = (64 - C::kMdBytes) / 4;               // 12 / 14
  static_assert(kTagDword + kTagWords <= kFusedCountWord && kEntWords <= kFusedCountWord, "");
  static_assert(kCntWords <= kTagDword, "");
  constexpr uint32_t kGroup = 12;
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = sg.n_blocks;
  uint8_t* payload = out + sg.out_offset;

  if (lo == 0 && tid < 5) {
    // PackedVqfFilter header (vqf_filter_page_view.hpp:79-94) + vqf_metadata
    uint64_t w0, w1;
    switch (tid) {
      case 0: w0 = kVqfMagic; w1 = sg.src_page_id; break;
      case 1: w0 = kVqfHashSeed; w1 = ~0ull << sg.hash_val_shift; break;
      case 2: w0 = 64ull * nb; w1 = T; break;
      case 3: w0 = (uint64_t)nb * C::kBuckets << T; w1 = nb; break;
      default: w0 = nelts; w1 = (uint64_t)nb * C::kSlots; break;
    }
    ulonglong2 v;
    v.x = w0;
    v.y = w1;
    reinterpret_cast<ulonglong2*>(payload)[tid] = v;
  } else if (lo == 0 && tid < 9) {
    write_page_header(out, sg, kLayoutVqf, tid - 5);
  }
  // this workgroup's blocks: LDS region b - lo, output block b
  uint4* dst_blocks = reinterpret_cast<uint4*>(payload + kVqfHeader + kVqfMetadata) + 4ull * lo;

  for (uint32_t b0 = tid; b0 < nbl; b0 += NB * NT) {
    uint32_t* reg[NB];
    uint32_t c[NB];
    bool live[NB];
    uint32_t ent[NB][kEntWords];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const uint32_t b = b0 + j * NT;
      live[j] = b < nbl;
      reg[j] = lds + (live[j] ? b : b0) * kFusedRegionWords;
      c[j] = live[j] ? reg[j][kFusedCountWord] : 0u;
#pragma unroll
      for (uint32_t w = 0; w < kEntWords; ++w) ent[j][w] = reg[j][w];
    }
    asm volatile("" ::: "memory");  // entries are in registers before their words are reused
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (!live[j]) continue;
#pragma unroll
      for (uint32_t w = 0; w < kCntWords; ++w) reg[j][w] = 0;
#pragma unroll
      for (uint32_t w = 0; w < kTagWords; ++w) reg[j][kTagDword + w] = 0;
    }
    // pass 1: bucket histogram (bytes, 4 buckets per dword).  Branch-free: dead slots add 0.
#pragma unroll
    for (uint32_t i = 0; i < C::kSlots; ++i) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const E e = reinterpret_cast<const E*>(ent[j])[i];
        const bool on = live[j] && i < c[j];
        const uint32_t o = on ? (uint32_t)(e >> T) : 0u;
        atomicAdd(reg[j] + (o >> 2), on ? 1u << (8 * (o & 3)) : 0u);
      }
    }
    // exclusive prefix over buckets: inclusive-in-dword = v * 0x01010101 (a dead j aliases
    // the thread's first block, whose counters must be scanned once)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (!live[j]) continue;
      uint32_t run = 0;
#pragma unroll
      for (uint32_t w = 0; w < kCntWords; ++w) {
        const uint32_t v = reg[j][w];
        const uint32_t incl = v * 0x01010101u;
        reg[j][w] = (incl - v) + run * 0x01010101u;
        run += incl >> 24;
      }
    }
    // pass 2: each entry's slot in insertion order (ds_add_rtn on its bucket counter), then
    // its metadata zero at slot + offset and its tag byte in the image.  Groups of kGroup
    // slots: the group's atomics are issued back to back (a store whose address depends on
    // a returned slot between them made every atomic wait for the previous one), then the
    // group's slots are consumed while the next group's atomics queue behind its stores.
    uint64_t md_lo[NB], md_hi[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      md_lo[j] = ~0ull;
      md_hi[j] = T == 8 ? ~0ull : 0ull;
      // the per-slot offsets and masks of pass 1 are recomputed below, not kept live across
      // the prefix scan (48 slots' worth of them set the register count)
#pragma unroll
      for (uint32_t w = 0; w < kEntWords; ++w) asm volatile("" : "+v"(ent[j][w]));
    }
#pragma unroll
    for (uint32_t g = 0; g < C::kSlots; g += kGroup) {
      uint32_t old[NB][kGroup];
#pragma unroll
      for (uint32_t u = 0; u < kGroup && g + u < C::kSlots; ++u) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const uint32_t i = g + u;
          const uint32_t e = reinterpret_cast<const E*>(ent[j])[i];
          const bool on = live[j] && i < c[j];
          const uint32_t o = on ? e >> T : 0u;
          old[j][u] = atomicAdd(reg[j] + (o >> 2), on ? 1u << (8 * (o & 3)) : 0u);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (uint32_t u = 0; u < kGroup && g + u < C::kSlots; ++u) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const uint32_t i = g + u;
          const uint32_t e = reinterpret_cast<const E*>(ent[j])[i];
          const bool on = live[j] && i < c[j];
          const uint32_t o = on ? e >> T : 0u, tag = e & ((1u << T) - 1);
          const uint32_t slot = (old[j][u] >> (8 * (o & 3))) & 0xffu;
          const uint32_t z = slot + o;
          const uint64_t clr = on ? 1ull << (z & 63) : 0ull;
          if (z < 64) md_lo[j] &= ~clr;
          else md_hi[j] &= ~clr;
          // dead slots store into the region's count word (no longer read)
          uint8_t* r8 = reinterpret_cast<uint8_t*>(reg[j]);
          const uint32_t byte = on ? 4 * kTagDword + slot * (T / 8) : 4 * kFusedCountWord;
          if constexpr (T == 8) {
            r8[byte] = (uint8_t)tag;
          } else {
            const uint16_t t16 = (uint16_t)tag;
            __builtin_memcpy(r8 + byte, &t16, 2);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (!live[j]) continue;
      if (c[j] == 0) {  // an empty block keeps the init metadata: top bit clear
        if constexpr (T == 8) md_hi[j] &= ~(1ull << 63);
        else md_lo[j] &= ~(1ull << 63);
      }
      const uint32_t* tg = reg[j] + kTagDword;
      uint4* dst = dst_blocks + (uint64_t)(b0 + j * NT) * 4;
      uint4 v0;
      v0.x = (uint32_t)md_lo[j];
      v0.y = (uint32_t)(md_lo[j] >> 32);
      if constexpr (T == 8) {
        v0.z = (uint32_t)md_hi[j];
        v0.w = (uint32_t)(md_hi[j] >> 32);
        dst[0] = v0;
#pragma unroll
        for (uint32_t q = 0; q < 3; ++q) dst[1 + q] = make_uint4(tg[4 * q], tg[4 * q + 1], tg[4 * q + 2], tg[4 * q + 3]);
      } else {
        v0.z = tg[0];
        v0.w = tg[1];
        dst[0] = v0;
#pragma unroll
        for (uint32_t q = 0; q < 3; ++q)
          dst[1 + q] = make_uint4(tg[2 + 4 * q], tg[3 + 4 * q], tg[4 + 4 * q], tg[5 + 4 * q]);
      }
    }
  }
}

// Blocks [lo, lo + nbl) of the leaf (a leaf whose LDS image exceeds the budget is placed by
// several workgroups, each reading all of the leaf's records and keeping its blocks' ones).
template <int T, uint32_t NT>
__device__ void vqf_place_fused_body(const tkv_amq_segment& sg, uint32_t seg_index,
                                     VqfWorkspace ws, const uint64_t* __restrict__ recs,
                                     uint8_t* __restrict__ out, uint32_t* lds, uint32_t lo,
                                     uint32_t nbl)
{
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = sg.n_blocks, n = sg.n_keys;
  for (uint32_t b = tid; b < nbl; b += NT) lds[b * kFusedRegionWords + kFusedCountWord] = 0;
  __syncthreads();
  const uint32_t gb0 = (uint32_t)sg.block_base;
  constexpr uint32_t kU = 16;  // 16-byte loads in flight per thread: 64 KB per workgroup
  auto put_entry = [&](uint32_t blk, uint32_t rank, uint32_t e) {
    uint32_t* r = lds + blk * kFusedRegionWords;
    if constexpr (T == 8) reinterpret_cast<uint16_t*>(r)[rank] = (uint16_t)e;
    else r[rank] = e;
    atomicAdd(r + kFusedCountWord, 1u);
  };
  if (T == 8 && nb <= 512) {
    // compact 4-byte records (vqf_decide kCompact), four per load (such a leaf has one
    // workgroup: lo = 0, nbl = nb)
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(recs + sg.key_begin);
    const uint32_t skip = (uint32_t)((reinterpret_cast<uintptr_t>(r32) & 15) >> 2);  // 0 or 2
    const uint4* r4 = reinterpret_cast<const uint4*>(r32 - skip);
    const uint32_t n_quads = (skip + n + 3) / 4;
    auto put = [&](uint32_t v, uint32_t k) {
      if (k >= skip && k < skip + n && v != 0xffffffffu) put_entry(v >> 21, (v >> 15) & 63u, v & 0x7fffu);
    };
    for (uint32_t q0 = 0; q0 < n_quads; q0 += NT * kU) {
      uint4 v[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t q = q0 + u * NT + tid;
        v[u] = q < n_quads ? load_nt16(r4 + q) : make_uint4(~0u, ~0u, ~0u, ~0u);
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t k = 4 * (q0 + u * NT + tid);
        put(v[u].x, k);
        put(v[u].y, k + 1);
        put(v[u].z, k + 2);
        put(v[u].w, k + 3);
      }
    }
  } else {
    // 8-byte records, two per load; records start 128-byte aligned in the workspace
    const uint64_t a0 = sg.key_begin & ~1ull;
    const uint4* r2 = reinterpret_cast<const uint4*>(recs + a0);
    const uint32_t lo_skip = (uint32_t)(sg.key_begin - a0);  // 0 or 1
    const uint32_t n_pairs = (lo_skip + n + 1) / 2;
    auto put = [&](uint64_t v, uint32_t k) {
      const uint32_t hi = (uint32_t)(v >> 32);
      const uint32_t blk = (hi >> 6) - gb0 - lo;  // (a key not inserted: hi = ~0, out of range)
      if (k >= lo_skip && k < lo_skip + n && hi != 0xffffffffu && blk < nbl)
        put_entry(blk, hi & 63u, (uint32_t)v & 0x7fffffffu);
    };
    for (uint32_t p0 = 0; p0 < n_pairs; p0 += NT * kU) {
      uint4 v[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t p = p0 + u * NT + tid;
        v[u] = p < n_pairs ? load_nt16(r2 + p) : make_uint4(0, ~0u, 0, ~0u);
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t k = 2 * (p0 + u * NT + tid);
        put((uint64_t)v[u].x | ((uint64_t)v[u].y << 32), k);
        put((uint64_t)v[u].z | ((uint64_t)v[u].w << 32), k + 1);
      }
    }
  }
  __syncthreads();
  vqf_place_fused_sort<T, 1, NT>(sg, lo == 0 ? ws.nelts[seg_index] & kVqfNeltsMask : 0u, out, lds, lo, nbl);
}

// grid: n_segs * parts workgroups; workgroup (s, p) places blocks [p * span, (p + 1) * span)
// of leaf s (parts = 1 unless a leaf's image exceeds kFusedLdsBudget)
template <uint32_t NT>
__global__ __launch_bounds__(NT) void vqf_place_fused(const tkv_amq_segment* __restrict__ segs,
                                                                 void* ws_base, uint64_t ws_bytes,
                                                                 uint32_t n_segs,
                                                                 uint8_t* __restrict__ out,
                                                                 uint32_t parts, uint32_t span)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_lds[];
  const uint32_t seg = blockIdx.x / parts, lo = (blockIdx.x - seg * parts) * span;
  const tkv_amq_segment sg = segs[seg];
  if (lo >= sg.n_blocks && lo != 0) return;
  const uint32_t nbl = sg.n_blocks - lo < span ? sg.n_blocks - lo : span;
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, seg)) return;
  const uint64_t* recs = vqf_records(ws, segs, n_segs);
  if (sg.tag_bits == 8) vqf_place_fused_body<8, NT>(sg, seg, ws, recs, out, s_lds, lo, nbl);
  else if (sg.tag_bits == 16) vqf_place_fused_body<16, NT>(sg, seg, ws, recs, out, s_lds, lo, nbl);
}

// ---------------------------------------------------------------------------------------
// vqf_ring_place: vqf_decide_ring and vqf_place_fused in one workgroup per leaf, for batches
// that do not fill the chip with one workgroup per CU (<= kRingPlaceMaxSegs leaves) of leaves
// whose LDS image fits beside the ring (<= kRingPlaceMaxBlocks blocks).  The decider writes
// each key's entry straight to [block][rank] of the leaf's LDS image (the rank is the block's
// count at the key's insertion), so no key record goes through HBM; once the decider is done,
// all eight waves run the place's per-block counting sort on the image and write the filter.
// One kernel instead of two (and no records written and read back): the small-batch latency.
// LDS: ring | ready/freed | counts [cnt_words] | image [nb x 33 dwords] | sink | nelts.
// ---------------------------------------------------------------------------------------
constexpr uint32_t kRingPlaceMaxSegs = 256;
// vqf_locate_keys before vqf_ring_place up to this many leaves (variable-length keys, other
// fixed sizes): measured crossovers, past which the chip is busy enough that hashing inside the
// producers, overlapped with the decider, beats writing and re-reading 8-byte located records
constexpr uint32_t kVqfLocMaxSegsVar = 64;
constexpr uint32_t kVqfLocMaxSegsFixed = 32;
__host__ __device__ inline uint32_t ring_place_cnt_words(uint32_t max_nb)
{
  return (max_nb + 1 + 3) & ~3u;  // + the dummy block
}

__host__ __device__ constexpr inline uint32_t ring_place_lds_bytes(uint32_t max_nb, uint32_t NS = kRingPlaceSlots,
                                                                  bool tbl = true)
{
  return ring_base_bytes(NS) + 4 * ((max_nb + 4) & ~3u) + 4 * kFusedRegionWords * (max_nb + 1) + 16 +
         (tbl && max_nb <= kRingTblBlocks ? 16 * kRingTblProducers * (max_nb + 1) : 0);
}

constexpr uint32_t kRingPlaceMaxBlocks =
    ((160 * 1024 - ring_base_bytes(kRingPlaceSlots) - 16 - 4 * kFusedRegionWords - 16) / (4 * kFusedRegionWords + 4)) & ~3u;
static_assert(kRingPlaceMaxBlocks == 960, "(DESIGN.md and test_vqf_ring_place_classes quote it)");
static_assert(ring_place_lds_bytes(kRingPlaceMaxBlocks) <= 160 * 1024, "vqf_ring_place LDS");
static_assert(ring_place_lds_bytes(kRingTblBlocks) <= 160 * 1024, "vqf_ring_place match tables");
// Batches of kRingPlaceMaxSegs..kRingPlace2MaxSegs leaves: two workgroups per CU, each with a
// ring of kRingPlace2Slots slots, no match tables, leaves of <= kRingPlace2MaxBlocks blocks
// (the bench layout's 402-block leaves: one round of 512 leaves instead of the unfused pair)
constexpr uint32_t kRingPlace2Slots = 6;
constexpr uint32_t kRingPlace2MaxSegs = 512;
constexpr uint32_t kRingPlace2MaxBlocks =
    ((80 * 1024 - ring_base_bytes(kRingPlace2Slots) - 16 - 4 * kFusedRegionWords - 16) / (4 * kFusedRegionWords + 4)) & ~3u;
static_assert(ring_place_lds_bytes(kRingPlace2MaxBlocks, kRingPlace2Slots, false) <= 80 * 1024,
              "two vqf_ring_place workgroups per CU");
static_assert(kRingPlace2MaxBlocks == 420, "(DESIGN.md and test_vqf_ring_place_classes quote it)");
static_assert(kRingPlaceMaxBlocks < kVqfLocMaxBlocks, "located records hold 11-bit block ids");

template <int T, int MODE, int NBITS, uint32_t NS>
__device__ __attribute__((always_inline)) void vqf_ring_place_body(const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                                    const tkv_amq_segment& sg, uint32_t seg_index, VqfWorkspace ws,
                                    uint8_t* out, uint32_t* lds, uint32_t cnt_words, bool tbl,
                                    uint64_t key_end)
{
  using C = Vqf<T>;
  diag_stamp(0);
  if (NBITS == 9 && NS == kRingPlaceSlots && tbl)  // (leaves <= kRingTblBlocks blocks: the host sized the tables)
    vqf_ring_body<T, MODE, kRecImage, NBITS, true, NS>(keys, offs, stride, sg, seg_index, ws, nullptr, lds,
                                                   true, cnt_words, key_end);
  else
    vqf_ring_body<T, MODE, kRecImage, NBITS, false, NS>(keys, offs, stride, sg, seg_index, ws, nullptr, lds,
                                                    true, cnt_words, key_end);
  const uint32_t nb = sg.n_blocks;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(lds) + ring_base_bytes(NS) / 4;
  uint32_t* img = cnt + cnt_words;
  __syncthreads();  // the decider is done (its LDS writes are visible to the workgroup)
  // the sort reads each block's count from its region (a full block keeps its slots)
  for (uint32_t b = threadIdx.x; b < nb; b += kRingThreads) {
    const uint32_t c = cnt[b];
    img[b * kFusedRegionWords + kFusedCountWord] = c < C::kSlots ? c : C::kSlots;
  }
  const uint32_t nelts = img[(nb + 1) * kFusedRegionWords + 1];
  __syncthreads();
  diag_stamp(1);
  vqf_place_fused_sort<T, 1, kRingThreads>(sg, nelts, out, img, 0, nb);
  __syncthreads();
  diag_stamp(2);
}

// every key of a small batch hashed and located on the whole chip, ahead of vqf_ring_place
// (kKeyLoc): the hashing leaves the ring's CU, whose producers then only read the records
template <int MODE>
__global__ __launch_bounds__(256) void vqf_locate_keys(const uint8_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ offs, uint32_t stride,
                                                       const tkv_amq_segment* __restrict__ segs,
                                                       void* ws_base, uint64_t ws_bytes, uint32_t n_segs,
                                                       uint64_t n_keys)
{
  const uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (gi >= n_keys) return;
  // the key's leaf: the last with key_begin <= gi (leaves lie in key order)
  uint32_t lo = 0, hi = n_segs;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (segs[mid].key_begin <= gi) lo = mid;
    else hi = mid;
  }
  const tkv_amq_segment sg = segs[lo];
  if (gi >= sg.key_begin + sg.n_keys || (sg.tag_bits != 8 && sg.tag_bits != 16)) return;
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, ~0u)) return;  // (vqf_ring_place flags the leaf)
  uint64_t h;
  if constexpr (MODE == kKey16 || MODE == kKey24) {
    VqfKeyBuf<MODE> kb;
    vqf_load_key<MODE>(keys, gi, kb);
    h = vqf_key_hash<MODE>(keys, offs, stride, gi, kb);
  } else {
    h = hash_key<MODE>(keys, offs, stride, gi, kVqfHashSeed);
  }
  reinterpret_cast<uint2*>(vqf_records(ws, segs, n_segs))[gi] =
      sg.tag_bits == 8 ? vqf_loc_encode<8>(h, sg) : vqf_loc_encode<16>(h, sg);
}

template <int MODE, uint32_t NS>
__global__ __launch_bounds__(kRingThreads) void vqf_ring_place(
    const uint8_t* keys, const uint64_t* __restrict__ offs, uint32_t stride,
    const tkv_amq_segment* __restrict__ segs, void* ws_base, uint64_t ws_bytes, uint32_t n_segs,
    uint8_t* __restrict__ out, uint32_t cnt_words, uint32_t tbl)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
  const tkv_amq_segment sg = segs[blockIdx.x];
  const VqfWorkspace ws = vqf_workspace(ws_base, n_segs);
  vqf_mark_build(ws, n_segs);
  if (!vqf_ws_ok(segs, n_segs, ws_bytes, ws, blockIdx.x)) return;
  const uint64_t key_end = vqf_key_end<MODE>(offs, segs, n_segs);
  const uint32_t nb = sg.n_blocks;  // <= kRingPlaceMaxBlocks (tkv_amq_build)
  // kKeyLoc: the located records vqf_locate_keys wrote, where vqf_decide_ring writes its records
  if constexpr (MODE == kKeyLoc) keys = reinterpret_cast<const uint8_t*>(vqf_records(ws, segs, n_segs));
  if (sg.tag_bits == 8) {
    if (nb <= 512) vqf_ring_place_body<8, MODE, 9, NS>(keys, offs, stride, sg, blockIdx.x, ws, out, s_ring, cnt_words, tbl != 0, key_end);
    else vqf_ring_place_body<8, MODE, 10, NS>(keys, offs, stride, sg, blockIdx.x, ws, out, s_ring, cnt_words, tbl != 0, key_end);
  } else if (sg.tag_bits == 16) {
    if (nb <= 512) vqf_ring_place_body<16, MODE, 9, NS>(keys, offs, stride, sg, blockIdx.x, ws, out, s_ring, cnt_words, tbl != 0, key_end);
    else vqf_ring_place_body<16, MODE, 10, NS>(keys, offs, stride, sg, blockIdx.x, ws, out, s_ring, cnt_words, tbl != 0, key_end);
  } else if (threadIdx.x == 0) {
    ws.nelts[blockIdx.x] = 0;
  }
}

// ---------------------------------------------------------------------------------------
// VQF probe (PackedVqfFilter::is_present, vqf_filter_page_view.hpp:113-125)
// ---------------------------------------------------------------------------------------
template <int T>
struct VqfBucketRef {
  const uint8_t* bp;  // the 64-byte block
  uint32_t o;         // bucket offset inside it
  uint64_t lo, hi;    // block metadata
};

template <int T>
__device__ inline VqfBucketRef<T> vqf_bucket_ref(const uint8_t* blocks, uint32_t idx)
{
  using C = Vqf<T>;
  VqfBucketRef<T> r;
  const uint32_t blk = idx / C::kBuckets;
  r.o = idx - blk * C::kBuckets;
  r.bp = blocks + (uint64_t)blk * 64;
  if constexpr (T == 8) {
    const ulonglong2 md = *reinterpret_cast<const ulonglong2*>(r.bp);
    r.lo = md.x;
    r.hi = md.y;
  } else {
    r.lo = *reinterpret_cast<const uint64_t*>(r.bp);
    r.hi = 0;
  }
  return r;
}

// exact per-byte / per-halfword equality mask (high bit of each lane set where x's lane is 0)
__device__ inline uint32_t zero_bytes(uint32_t x)
{
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}
__device__ inline uint32_t zero_halves(uint32_t x)
{
  return ~(((x & 0x7fff7fffu) + 0x7fff7fffu) | x | 0x7fff7fffu);
}

// Tags of bucket o are slots [start, end).  One 16-byte load of the tag area starting at the
// dword that holds slot `start` covers the bucket in almost every case (a bucket holds ~0.6
// tags on average); longer buckets finish with a per-slot loop.
template <int T>
__device__ inline bool vqf_bucket_has(const VqfBucketRef<T>& r, uint32_t tag)
{
  using C = Vqf<T>;
  const int o = (int)r.o;
  const int start = o == 0 ? 0 : select128(r.lo, r.hi, o - 1) - (o - 1);
  const int end = select128(r.lo, r.hi, o) - o;
  if (end <= start) return false;
  constexpr int kPer = 4 / (T / 8);                     // slots per dword: 4 / 2
  const int d0 = start / kPer;                          // first dword of the window
  const int last_dword = (C::kSlots * (T / 8)) / 4 - 1; // 11 / 13
  const int d = d0 + 3 <= last_dword ? d0 : last_dword - 3;
  const uint4 w = *reinterpret_cast<const uint4*>(r.bp + C::kMdBytes + 4 * d);
  const int s0 = start - d * kPer, s1 = end - d * kPer;  // window-relative slot range
  const uint32_t rep = T == 8 ? tag * 0x01010101u : tag * 0x00010001u;
  uint32_t m[4];
  const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) m[i] = T == 8 ? zero_bytes(wv[i] ^ rep) : zero_halves(wv[i] ^ rep);
  // pack one bit per slot: slot j of the window <-> bit j
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (T == 8) {
      const uint32_t b4 = ((m[i] >> 7) & 1u) | ((m[i] >> 14) & 2u) | ((m[i] >> 21) & 4u) | ((m[i] >> 28) & 8u);
      bits |= b4 << (4 * i);
    } else {
      const uint32_t b2 = ((m[i] >> 15) & 1u) | ((m[i] >> 30) & 2u);
      bits |= b2 << (2 * i);
    }
  }
  constexpr int kWin = 4 * kPer;  // 16 / 8 slots
  const int hi_in = s1 < kWin ? s1 : kWin;
  const uint32_t range = (hi_in > s0 ? ((1u << (hi_in - s0)) - 1u) : 0u) << s0;
  bool hit = (bits & range) != 0;
  for (int p = d * kPer + kWin; p < end; ++p) {  // rare: bucket runs past the window
    uint32_t tv;
    if constexpr (T == 8) tv = r.bp[C::kMdBytes + p];
    else tv = *reinterpret_cast<const uint16_t*>(r.bp + C::kMdBytes + 2 * p);
    hit |= tv == tag;
  }
  return hit;
}

template <int T>
__device__ inline bool vqf_present(const uint8_t* payload, uint32_t n_blocks, uint64_t magic,
                                   uint64_t h)
{
  using C = Vqf<T>;
  const uint64_t R = (uint64_t)n_blocks * C::kBuckets;
  const uint32_t tag = (uint32_t)(h & ((1ull << T) - 1));
  const uint32_t pi = (uint32_t)mod_by_magic(h >> T, R, magic);
  const uint32_t ai = (uint32_t)mod_by_magic((h ^ ((uint64_t)tag * kVqfAltMul)) >> T, R, magic);
  const uint8_t* blocks = payload + kVqfHeader + kVqfMetadata;
  // primary bucket first; only the lanes that did not find the tag there read the alternate
  // block (vqf_is_present's order, vqf_filter_page_view.hpp:120-124; loading both blocks up
  // front measured slower)
  if (vqf_bucket_has<T>(vqf_bucket_ref<T>(blocks, pi), tag)) return true;
  return vqf_bucket_has<T>(vqf_bucket_ref<T>(blocks, ai), tag);
}

// One VQF (hash, leaf) test: result bit | class << 1.
// (always inlined: out of line it was a real call in every probe kernel, with a stack frame)
template <bool kOpts>
__device__ __attribute__((always_inline)) inline uint32_t vqf_probe_one(const uint8_t* filters, const tkv_amq_segment* segs,
                                         uint32_t n_segs, uint32_t s, uint64_t h,
                                         const uint64_t* page_ids = nullptr, uint64_t i = 0)
{
  const ProbeDesc d = load_probe_desc(segs, s, n_segs);
  if (d.tag_bits == 0) return 1u | (kNoFilter << 1);  // no filter: cannot reject
  const uint8_t* payload = filters + d.out_offset;
  if constexpr (kOpts) {
    if (!page_id_matches(payload, 8, page_ids, i)) return 1u | (kIdMismatch << 1);
  }
  const uint64_t mask = ~0ull << d.hash_val_shift;  // == PackedVqfFilter::hash_mask
  // dropped hash values are always "maybe" (:115-117)
  if ((h & mask) != h) return 1u | (kChecked << 1);
  const uint64_t magic = segs[s].mod_magic;
  const bool p = d.tag_bits == 8 ? vqf_present<8>(payload, d.n_blocks, magic, h)
                                 : vqf_present<16>(payload, d.n_blocks, magic, h);
  return (uint32_t)p | (kChecked << 1);
}

template <int MODE>
__device__ inline uint64_t vqf_query_hash(const uint8_t* __restrict__ q, const uint64_t* __restrict__ qoffs,
                                          uint32_t stride, uint64_t i)
{
  if constexpr (MODE == kKey16) {
    const uint4 kv = load_nt16(q + 16 * i);
    const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
    return x.finish(xxh16_rhinit(kVqfHashSeed));
  } else {
    return hash_key<MODE>(q, qoffs, stride, i, kVqfHashSeed);
  }
}

template <int MODE, bool kOpts>
__global__ __launch_bounds__(256) void vqf_probe(const uint8_t* __restrict__ filters,
                                                 const tkv_amq_segment* __restrict__ segs, uint32_t n_segs,
                                                 const uint8_t* __restrict__ q,
                                                 const uint64_t* __restrict__ qoffs, uint32_t stride,
                                                 uint64_t n, const uint32_t* __restrict__ qseg,
                                                 uint8_t* __restrict__ result, tkv_amq_probe_opts opts)
{
  if constexpr (!kOpts) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = vqf_query_hash<MODE>(q, qoffs, stride, i);
    __builtin_nontemporal_store(
        (uint8_t)(vqf_probe_one<false>(filters, segs, n_segs, __builtin_nontemporal_load(qseg + i), h) & 1u),
        result + i);
  } else {
    ProbeTally t;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
      const uint32_t r = vqf_probe_one<true>(filters, segs, n_segs, qseg[i],
                                             vqf_query_hash<MODE>(q, qoffs, stride, i), opts.d_query_page_id, i);
      result[i] = (uint8_t)(r & 1u);
      t.add(r, opts.d_truth, i);
    }
    flush_tally(t, opts.d_metrics, opts.d_truth != nullptr);
  }
}

template <bool kOpts>
__global__ __launch_bounds__(256) void vqf_probe_hashed(const uint8_t* __restrict__ filters,
                                                        const tkv_amq_segment* __restrict__ segs, uint32_t n_segs,
                                                        const uint64_t* __restrict__ hashes,
                                                        const uint32_t* __restrict__ pair_query,
                                                        uint64_t n, const uint32_t* __restrict__ qseg,
                                                        uint8_t* __restrict__ result, tkv_amq_probe_opts opts)
{
  ProbeTally t;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t qi = pair_query ? pair_query[i] : i;
    const uint32_t r = vqf_probe_one<kOpts>(filters, segs, n_segs, qseg[i], hashes[qi],
                                            opts.d_query_page_id, i);
    result[i] = (uint8_t)(r & 1u);
    if constexpr (kOpts) t.add(r, opts.d_truth, i);
    else break;
  }
  if constexpr (kOpts) flush_tally(t, opts.d_metrics, opts.d_truth != nullptr);
}

// ---- Bloom query hash cache (BloomFilterQuery<KeyView>) ----
__host__ __device__ inline uint32_t bloom_query_stride(uint32_t k_max)
{
  return (8 + 2 * (k_max > 1 ? k_max - 1 : 0) + 15) & ~15u;
}

template <int MODE>
__global__ __launch_bounds__(256) void bloom_hash_kernel(const uint8_t* __restrict__ q,
                                                         const uint64_t* __restrict__ qoffs,
                                                         uint32_t stride, uint64_t n, uint32_t k_max,
                                                         uint8_t* __restrict__ out)
{
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint8_t* rec = out + i * bloom_query_stride(k_max);
  uint16_t* bits = reinterpret_cast<uint16_t*>(rec + 8);
  if constexpr (MODE == kKey16) {
    const uint4 kv = load_nt16(q + 16 * i);
    const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
    *reinterpret_cast<uint64_t*>(rec) = x.finish(c_bloom.rhinit16[0]);
    for (uint32_t j = 1; j < k_max; ++j) bits[j - 1] = (uint16_t)(x.finish_lo9(c_bloom.rhinit16[j]) & 511u);
  } else {
    uint32_t len;
    const uint8_t* p = key_at<MODE>(q, qoffs, stride, i, len);
    if (len < 32) {
      const XxhShort x(p, len);
      *reinterpret_cast<uint64_t*>(rec) = x.finish(c_bloom.seed_p5[0]);
      for (uint32_t j = 1; j < k_max; ++j) bits[j - 1] = (uint16_t)(x.finish_lo9(c_bloom.seed_p5[j]) & 511u);
    } else {
      *reinterpret_cast<uint64_t*>(rec) = xxh64_bytes(p, len, c_bloom.seed[0]);
      for (uint32_t j = 1; j < k_max; ++j)
        bits[j - 1] = (uint16_t)(xxh64_bytes(p, len, c_bloom.seed[j]) & 511u);
    }
  }
}

template <bool kOpts>
__global__ __launch_bounds__(256) void bloom_probe_hashed(const uint8_t* __restrict__ filters,
                                                          const tkv_amq_segment* __restrict__ segs, uint32_t n_segs,
                                                          const uint8_t* __restrict__ qrec,
                                                          uint32_t k_max,
                                                          const uint32_t* __restrict__ pair_query,
                                                          uint64_t n, const uint32_t* __restrict__ qseg,
                                                          uint8_t* __restrict__ result, tkv_amq_probe_opts opts)
{
  __shared__ uint4 s_blk[256 * kProbeSlotWords / 4];
  uint4* slot = s_blk + threadIdx.x * (kProbeSlotWords / 4);
  const uint32_t* slot32 = reinterpret_cast<const uint32_t*>(slot);
  ProbeTally t;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    // qseg[i] and pair_query[i], then the descriptor and the query record, are independent
    // loads issued side by side; only the block load waits for both
    const uint32_t sidx = qseg[i];
    const uint64_t qi = pair_query ? pair_query[i] : i;
    const uint8_t* rec = qrec + qi * bloom_query_stride(k_max);
    const ProbeDesc d = load_probe_desc(segs, sidx, n_segs);
    const uint64_t h0 = *reinterpret_cast<const uint64_t*>(rec);
    uint32_t r;
    // a filter whose hash_count exceeds the cached k_max cannot be tested: cannot reject
    if (d.hash_count == 0 || d.hash_count > k_max) {
      r = 1u | (kNoFilter << 1);
    } else if (kOpts && !page_id_matches(filters + d.out_offset, 16, opts.d_query_page_id, i)) {
      r = 1u | (kIdMismatch << 1);
    } else {
      const uint16_t* bits = reinterpret_cast<const uint16_t*>(rec + 8);
      const uint4* blk = reinterpret_cast<const uint4*>(filters + d.out_offset + kBloomHeader +
                                                        64 * __umul64hi(h0, (uint64_t)d.n_blocks));
      const uint4 b0 = blk[0], b1 = blk[1], b2 = blk[2], b3 = blk[3];
      slot[0] = b0;
      slot[1] = b1;
      slot[2] = b2;
      slot[3] = b3;
      uint32_t bit = (uint32_t)h0 & 511u;
      uint32_t ok = slot32[bit >> 5] >> (bit & 31);
      for (uint32_t j = 1; j < d.hash_count; ++j) {
        bit = bits[j - 1];
        ok &= slot32[bit >> 5] >> (bit & 31);
      }
      r = (ok & 1u) | (kChecked << 1);
    }
    result[i] = (uint8_t)(r & 1u);
    if constexpr (kOpts) t.add(r, opts.d_truth, i);
    else break;
  }
  if constexpr (kOpts) flush_tally(t, opts.d_metrics, opts.d_truth != nullptr);
}

template <int MODE>
__global__ __launch_bounds__(256) void vqf_hash_kernel(const uint8_t* __restrict__ q,
                                                       const uint64_t* __restrict__ qoffs,
                                                       uint32_t stride, uint64_t n,
                                                       uint64_t* __restrict__ out)
{
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if constexpr (MODE == kKey16) {
    const uint4 kv = reinterpret_cast<const uint4*>(q)[i];
    const Xxh16 x((uint64_t)kv.x | ((uint64_t)kv.y << 32), (uint64_t)kv.z | ((uint64_t)kv.w << 32));
    out[i] = x.finish(xxh16_rhinit(kVqfHashSeed));
  } else {
    out[i] = hash_key<MODE>(q, qoffs, stride, i, kVqfHashSeed);
  }
}

__global__ __launch_bounds__(256) void gen_keys16_kernel(uint64_t seed, uint64_t first, uint64_t n,
                                                         ulonglong2* __restrict__ out)
{
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t g = first + i;
    ulonglong2 v;
    v.x = splitmix64_at(seed, 2 * g + 1);
    v.y = splitmix64_at(seed, 2 * g + 2);
    out[i] = v;
  }
}

}  // namespace tkv

// =======================================================================================
// host side: planning (sizing restated from the reference) and the C ABI
// =======================================================================================
using namespace tkv;

namespace {

inline uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// The leaves of a Bloom batch other than the oversize ones (more than kWinMaxWindows windows),
// in order, into `dst` (tkv_amq_build_ex): one workgroup scans the flags chunk by chunk.
__global__ __launch_bounds__(1024) void bloom_compact_segs(const tkv_amq_segment* __restrict__ segs,
                                                           uint32_t n_segs, uint32_t max_small_blocks,
                                                           tkv_amq_segment* __restrict__ dst)
{
  // (256 or 1,024 threads: a short list launches narrow, a quarter of a CU's wave slots)
  __shared__ uint32_t s_w[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, nt = blockDim.x, nw = nt >> 6;
  uint32_t base = 0;
  for (uint32_t c0 = 0; c0 < n_segs; c0 += nt) {
    const uint32_t s = c0 + tid;
    const bool keep = s < n_segs && segs[s].n_blocks <= max_small_blocks;
    const uint64_t m = __ballot(keep);
    const uint32_t before = (uint32_t)__popcll(m & lanemask_lt());
    if (lane == 0) s_w[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = base, tot = 0;
    for (uint32_t w = 0; w < nw; ++w) {
      off += w < wave ? s_w[w] : 0u;
      tot += s_w[w];
    }
    if (keep) dst[off + before] = segs[s];
    base += tot;
    __syncthreads();
  }
}

constexpr uint32_t kBloomLdsBudget = 64 * 1024;  // dynamic LDS a launch gets without the attribute
// Leaf images are built in LDS up to the whole CU's LDS (a 160 KB image: 1.3M bits, ~130K
// keys at 10 bits/key; TurtleKV leaves of small items reach ~80K keys): one workgroup per
// leaf from kBloomSpreadSegs leaves, the split build below kBloomSplitSegs.  Images above
// kBloomWideLds take 1024-thread workgroups (fewer than five 256-thread workgroups would fit
// a CU).  Larger leaves take the window path (up to 16 windows of LDS); a single larger filter
// of 16- or 24-byte keys the tiled monolithic build (128 KiB tiles); anything else, device
// atomics.
constexpr uint32_t kBloomLeafLdsBudget = 160 * 1024;
constexpr uint32_t kBloomWideLds = 32 * 1024;
// The LDS build runs one workgroup per leaf, so a batch of a few leaves (the per-leaf call
// site, or a small LeafBatcher batch) keeps a few CUs busy for the whole leaf.  Below this many
// leaves the keys are spread over n_keys/256 workgroups that set bits with device atomics.
constexpr uint32_t kBloomSpreadSegs = 64;
// Below this many leaves (and with the workspace tkv_amq_plan sizes for it) each leaf's keys
// are split over several workgroups (bloom_build_split): about kSplitTargetWgs workgroups in
// all, at most kSplitMaxParts per leaf, at least kSplitMinKeys keys each.
constexpr uint32_t kBloomSplitSegs = 256;
constexpr uint32_t kSplitTargetWgs = 1024;
constexpr uint32_t kSplitMinKeys = 1024;
// From kBloomSplitSegs up to kBloomWideSegs leaves, one 1024-thread workgroup per leaf; from
// there one 256-thread workgroup per leaf (8 per CU).
constexpr uint32_t kBloomWideSegs = 2048;

// parts per leaf for a batch of n_segs leaves holding n_keys keys (1: no split)
inline uint32_t bloom_split_parts(uint32_t n_segs, uint64_t n_keys, uint64_t max_blocks)
{
  if (n_segs == 0 || n_segs >= kBloomSplitSegs || 64 * max_blocks > kBloomLeafLdsBudget) return 1;
  uint64_t p = (kSplitTargetWgs + n_segs - 1) / n_segs;
  const uint64_t per_leaf = n_keys / n_segs;
  const uint64_t by_keys = per_leaf / kSplitMinKeys;
  if (p > by_keys) p = by_keys;
  if (p > kSplitMaxParts) p = kSplitMaxParts;
  return p < 2 ? 1u : (uint32_t)p;
}

inline uint64_t bloom_split_ws_bytes(uint32_t n_segs, uint32_t parts, uint64_t max_blocks)
{
  return parts < 2 ? 0 : (uint64_t)n_segs * parts * 64 * max_blocks;
}

// The window path (bloom_build_window): leaves whose image exceeds kBloomLeafLdsBudget, cut
// into W windows.  A single 16- or 24-byte-key filter of more than kWinMonoMax windows takes
// the tiled monolithic build instead (it hashes each key once, whatever the tile count; since
// round 5 its few tiles are split over the chip, so it wins from two windows on: one 200K-key
// filter 53.3 vs 28.7 us, 500K 95.3 vs 34.3 us, profiles/r05/winmono/).
constexpr uint32_t kWinMonoMax = 1;
constexpr uint32_t kChipCUs = 256;  // MI355X; plans are made without a device

inline uint32_t bloom_window_count(uint64_t max_blocks)
{
  return (uint32_t)div_up(64 * max_blocks, kBloomLeafLdsBudget);
}

inline uint32_t bloom_window_blocks(uint64_t max_blocks)
{
  return (uint32_t)div_up(max_blocks, bloom_window_count(max_blocks));
}

// Parts per leaf: enough (leaf, window, part) workgroups to fill the chip in whole rounds,
// at >= kWinMinKeys keys per part; every extra part adds a partial image to write and merge
inline uint32_t bloom_window_parts(uint32_t n_segs, uint64_t n_keys, uint64_t max_blocks)
{
  constexpr uint32_t kWinMinKeys = 4096;
  if (n_segs == 0) return 1;
  const uint64_t W = bloom_window_count(max_blocks);
  const uint64_t per_cu = 64 * bloom_window_blocks(max_blocks) <= kBloomLeafLdsBudget / 2 ? 2 : 1;
  const uint64_t G = kChipCUs * per_cu;
  uint64_t max_p = n_keys / n_segs / kWinMinKeys;
  if (max_p > kSplitMaxParts) max_p = kSplitMaxParts;
  uint32_t best = 1;
  double best_cost = 1e30;
  for (uint64_t p = 1; p <= (max_p < 1 ? 1 : max_p); ++p) {
    const double rounds = (double)div_up((uint64_t)n_segs * W * p, G);
    const double cost = rounds / (double)p + (p > 1 ? 0.03 * (double)p : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = (uint32_t)p;
    }
  }
  return best;
}

// a batch the window path takes (n_keys: the batch's keys; mono16: one filter of 16-byte keys)
inline bool bloom_window_path(uint32_t n_segs, uint64_t max_blocks, bool mono16)
{
  const uint32_t W = bloom_window_count(max_blocks);
  if (W < 2 || W > kWinMaxWindows) return false;
  return !(n_segs == 1 && mono16 && W > kWinMonoMax);
}

template <uint32_t NT>
void launch_bloom_lds(int bmode, int mode, uint32_t n_segs, size_t lds, hipStream_t s,
                      const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                      const tkv_amq_segment* d_segs, uint8_t* d_out)
{
  const dim3 grid(n_segs), block(NT);
  if (bmode == kKey24)
    hipLaunchKernelGGL((bloom_build_lds<kKey24, NT>), grid, block, lds, s, keys, offs, stride, d_segs, d_out, 0u);
  else if (mode == kKey16)
    hipLaunchKernelGGL((bloom_build_lds<kKey16, NT>), grid, block, lds, s, keys, offs, stride, d_segs, d_out, 0u);
  else if (mode == kKeyFixed)
    hipLaunchKernelGGL((bloom_build_lds<kKeyFixed, NT>), grid, block, lds, s, keys, offs, stride, d_segs, d_out, 0u);
  else {
    // variable-length keys sorted by length per chunk when the scratch fits beside the image
    const size_t aux = 4ull * kVarAuxWords<NT>;
    const uint32_t sort = lds + aux <= kBloomLeafLdsBudget ? 1u : 0u;
    hipLaunchKernelGGL((bloom_build_lds<kKeyVar, NT>), grid, block, lds + (sort ? aux : 0), s, keys, offs,
                       stride, d_segs, d_out, sort);
  }
}

inline uint32_t vqf_slots(int t) { return t == 8 ? 48u : 28u; }
inline uint32_t vqf_buckets(int t) { return t == 8 ? 80u : 36u; }

uint32_t bloom_hash_count(uint32_t bpk)
{
  uint32_t k = (uint32_t)((double)bpk * 0.69314718055994530942 + 0.5);
  return k < 1 ? 1 : (k > kMaxBloomHashes ? kMaxBloomHashes : k);
}

inline int key_mode(const uint64_t* offs, uint32_t stride)
{
  if (offs) return kKeyVar;
  return stride == 16 ? kKey16 : kKeyFixed;
}

// the Bloom build additionally has a 24-byte fast path (needs 8-byte aligned keys)
inline int build_key_mode(const uint8_t* keys, const uint64_t* offs, uint32_t stride)
{
  if (!offs && stride == 24 && (reinterpret_cast<uintptr_t>(keys) & 7) == 0) return kKey24;
  return key_mode(offs, stride);
}

inline hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

inline tkv_amq_probe_opts probe_opts(const tkv_amq_probe_opts* o)
{
  tkv_amq_probe_opts r{nullptr, nullptr, nullptr};
  return o ? *o : r;
}

inline bool probe_opts_used(const tkv_amq_probe_opts& o)
{
  return o.d_query_page_id || o.d_truth || o.d_metrics;
}

// plain probes: one lane per query; with options: a grid-stride loop over a bounded grid, so
// the metrics take one atomic per counter per wave (8 waves per SIMD)
inline uint32_t probe_grid(uint64_t n, bool ex)
{
  const uint64_t g = (n + 255) / 256;
  const uint64_t cap = ex ? 8192 : 0xffffffffull;
  return (uint32_t)(g < cap ? g : cap);
}


// Kernel attributes (dynamic LDS above 64 KiB) are set once per device: a process may drive
// several GPUs from different threads.
constexpr int kMaxDevices = 64;
template <typename Fn>
inline void once_per_device(std::once_flag (&flags)[kMaxDevices], Fn&& fn)
{
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
    fn();
    return;
  }
  std::call_once(flags[dev], fn);
}

// Kernel attributes of the monolithic build (dynamic LDS above 64 KiB).
inline void set_mono_attributes()
{
  static std::once_flag lds_attr[kMaxDevices];
  once_per_device(lds_attr, [] {
    for (const void* f : {reinterpret_cast<const void*>(&bloom_part_keys16),
                          reinterpret_cast<const void*>(&bloom_part_keys24),
                          reinterpret_cast<const void*>(&bloom_part_routed)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(160 * 1024));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_tile),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(64 * kTileBlocks));
  });
}

inline uint32_t filter_tiles(uint64_t n_blocks) { return (uint32_t)div_up(n_blocks, kTileBlocks); }

inline uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

// partition -> tiles -> overflow.  src: kSrcKey16 / kSrcKey24 (keys, hashed), or kSrcRec12 for
// routed items (records, or 16-byte keys when k > 8)
inline void launch_part_build(int src, PartArgs a, hipStream_t s, const tkv_amq_segment* d_segs,
                              uint8_t* d_out, uint32_t hdr_always)
{
  set_mono_attributes();
  a.src_kind = (uint32_t)src;
  a.tbl = part_tbl_fits(a.g.n_tiles) ? 1u : 0u;
  const size_t lds = a.tbl ? part_tbl_lds_bytes(a.g.n_tiles) : part_lds_bytes(a.g.n_tiles);
  const dim3 grid(a.g.P), block(kPartThreads);
  if (src == kSrcKey24) hipLaunchKernelGGL(bloom_part_keys24, grid, block, lds, s, d_segs, a);
  else if (src == kSrcKey16) hipLaunchKernelGGL(bloom_part_keys16, grid, block, lds, s, d_segs, a);
  else hipLaunchKernelGGL(bloom_part_routed, grid, block, lds, s, d_segs, a);
  const uint32_t S = a.split > 1 ? a.split : 1u;
  hipLaunchKernelGGL(bloom_tile, dim3(a.g.n_tiles * S), dim3(kTileThreads), 64ull * kTileBlocks, s, d_segs, a,
                     d_out, hdr_always);
  if (S > 1) hipLaunchKernelGGL(bloom_tile_merge, dim3(a.g.n_tiles * kMergeChunks), dim3(256), 0, s, d_segs, a, d_out);
  hipLaunchKernelGGL(bloom_overflow, dim3(a.g.P), dim3(256), 0, s, d_segs, a, d_out);
}

// Tile workgroups per tile for a filter of T tiles: one tile per CU leaves most of the chip
// idle below 256 tiles (a tile's ~100K records take ~50 us of LDS ORs on one CU), so below 128
// each tile's regions are split over S workgroups (T * S <= 256), their partial images ORed
// by bloom_tile_merge; the partial images take T * S * 128 KiB <= kSplitImgBytes.
constexpr uint64_t kSplitImgBytes = 256ull << 17;
inline uint32_t tile_split(uint32_t T) { return T == 0 || T >= 128 ? 1u : std::min(kMaxSplit, 256u / T); }

// partition workgroups of a monolithic build of n keys (several leaves: all of them): the keys
// / 256 each, at least 1,024 and at most `most` -- every CU works, on fewer batches each
inline uint64_t mono_wg_items(uint64_t n, uint64_t most)
{
  return std::min<uint64_t>(most, std::max<uint64_t>(1024, n / kPartMaxWgs));
}

// The route of n keys (16 or 24 bytes) into g.n_parts parts of q tiles: the count pass, the two
// scans, then the scatter of the 12-byte records (out_recs; route_recs writes nothing for
// k > 8) and/or of the 16-byte keys themselves (out_keys; nothing for k < min_k).  The part
// totals are left at ws + g.P * n_parts (u32).
inline void launch_route(const RouteGeom& g, hipStream_t s, const uint8_t* keys, uint32_t kb, uint32_t n,
                         const tkv_amq_segment* d_seg, uint32_t q, uint32_t* ws, uint8_t* out_keys,
                         uint32_t min_k, uint8_t* out_recs)
{
  const size_t hl = 4ull * g.n_parts;
  const dim3 grid(g.P), block(256);
  if (kb == 24)
    hipLaunchKernelGGL((route_keys<0, 256, 24>), grid, block, hl, s, keys, d_seg, ws, g.n_parts, g.per, n,
                       q, nullptr, 0u);
  else
    hipLaunchKernelGGL((route_keys<0, 256, 16>), grid, block, hl, s, keys, d_seg, ws, g.n_parts, g.per, n,
                       q, nullptr, 0u);
  hipLaunchKernelGGL(route_scan_cols, dim3(g.n_parts), dim3(256), 0, s, ws, g.P, g.n_parts);
  hipLaunchKernelGGL(route_scan_parts, dim3(1), dim3(256), 0, s, ws, g.P, g.n_parts);
  if (out_recs) {
    uint32_t* r = reinterpret_cast<uint32_t*>(out_recs);
    if (kb == 24)
      hipLaunchKernelGGL((route_recs<256, 24>), grid, block, hl, s, keys, d_seg, ws, g.n_parts, g.per, n, q, r);
    else
      hipLaunchKernelGGL((route_recs<256, 16>), grid, block, hl, s, keys, d_seg, ws, g.n_parts, g.per, n, q, r);
  }
  if (out_keys && kb == 16)
    hipLaunchKernelGGL((route_keys<1, 256, 16>), grid, block, hl, s, keys, d_seg, ws, g.n_parts, g.per, n,
                       q, reinterpret_cast<uint4*>(out_keys), min_k);
}

// Tiles per routed part (a filter past kDirectMaxTiles): the fewer tiles a partition spreads
// a batch over, the longer each tile's run per store (fewer partial-line writes), until the
// route's output over that many parts pays more than the part builds save; and at most one
// tile per CU, so a part's tile kernel runs in one round.  Bit records (k <= 8), 1B keys at 12
// bits/key on one GPU, round 4's two-pass route: 1,431-tile parts 36.7 Gkeys/s, 800 39.2, 400
// 40.4, 294 39.8, 255 42.6, 229 41.9, 198 41.5, 127 37.1, 100 33.6 (profiles/r04/part_tiles/).
// 16-byte keys routed as themselves (k > 8) keep 1,600.  (turtle_kv_amd.dist.ROUTED_PART_TILES,
// ROUTED_KEY_PART_TILES)
constexpr uint32_t kRoutePartTiles = 256;
constexpr uint32_t kRouteKeyPartTiles = 1600;
static_assert(kRoutePartTiles <= kRecPartMaxTiles && kRouteKeyPartTiles <= kRecPartMaxTiles, "");
static_assert(kRoutePartTiles < 2048, "div_by_magic: exact for q < 2048 and tiles < 2^21");

// The route plan of tkv_amq_bloom_route_plan: parts, route workgroups, the part block layout.
// A region holds mean + 6 sigma + 16 records of a uniform hash when its overflow has nowhere to
// go but the route workgroup's own list (the one-GPU build), and mean + 2 sigma + 16 when the
// block carries an overflow area of ovf_cap entries (the exchange): the regions' slack is what
// crosses xGMI beside the records (round 5: 6 sigma, 14% at config 5's size on eight ranks; 2
// sigma: ~5%), and the ~2% of regions that fill send their few extra records as overflow
// entries (~0.4 per region of a uniform hash; the part build sets them with atomics).
inline int route_plan(uint64_t chunk_keys, uint32_t n_chunks, uint64_t n_blocks, uint32_t k, uint32_t world,
                      bool ovf_area, tkv_amq_route_plan& rp)
{
  if (world == 0 || n_chunks == 0 || n_blocks == 0 || n_blocks > 0xffffffffull || k == 0 || k > 8 ||
      chunk_keys > 0xffffffffull || (uint64_t)n_chunks * world > kMaxSrcSegs)
    return TKV_AMQ_INVALID_ARGUMENT;
  memset(&rp, 0, sizeof(rp));
  const uint32_t T = filter_tiles(n_blocks);
  const uint32_t per_rank = (uint32_t)div_up(T, world);
  const uint32_t g = (uint32_t)div_up(per_rank, kRoutePartTiles);
  const uint32_t q = (uint32_t)div_up(T, (uint64_t)world * g);
  if ((uint64_t)world * g > kRouteMaxParts) return TKV_AMQ_INVALID_ARGUMENT;
  rp.n_tiles = T;
  rp.n_blocks = n_blocks;
  rp.parts_per_rank = g;
  rp.n_parts = world * g;
  rp.part_tiles = q;
  rp.world = world;
  rp.n_chunks = n_chunks;
  rp.hash_count = k;
  rp.chunk_keys = chunk_keys;
  const uint64_t pw = div_up(chunk_keys, 32ull * kPartThreads);
  const uint32_t P = (uint32_t)(pw < 1 ? 1 : (pw > kPartMaxWgs ? kPartMaxWgs : pw));
  rp.route_wgs = P;
  const uint64_t per = div_up(chunk_keys, P);  // keys per route workgroup
  // a part's share of the keys is its blocks' share (q full tiles at most; the last tile may
  // be short, and the last parts may hold fewer tiles, or none when world * g * q > T)
  const double e = (double)per * std::min<uint64_t>((uint64_t)q * kTileBlocks, n_blocks) / n_blocks;
  // (2 sigma only where the blocks cross xGMI: one rank keeps 6 and sends nothing to the
  // overflow path)
  rp.region_cap = ((uint32_t)(e + (ovf_area && world > 1 ? 2.0 : 6.0) * sqrt(e) + 16.0) + 15) & ~15u;
  // overflow entries per block: the expected spill of 2-sigma regions (~0.4 per region) many
  // times over, plus room for keys that are not spread by the hash (duplicates)
  rp.ovf_cap = ovf_area ? (uint32_t)(4096 + 4 * P + chunk_keys / ((uint64_t)world * g * 256)) : 0u;
  rp.counts_off = 0;
  rp.ovf_n_off = align256(4ull * P);
  rp.regions_off = rp.ovf_n_off + 256;
  rp.ovf_off = align256(rp.regions_off + 12ull * P * rp.region_cap);
  rp.block_bytes = align256(rp.ovf_off + 16ull * rp.ovf_cap);
  // route workspace: [sink 256][u32 overflow count per workgroup][16-byte entries, per each]
  rp.route_ws_bytes = align256(512 + 4ull * P) + 16ull * P * per;
  // a part build: partition regions over the part's q tiles, overflow lists of what its
  // workgroup may receive (every source block's region at capacity)
  const uint64_t S = (uint64_t)n_chunks * world;
  const double ep = (double)chunk_keys * S / P * std::min<uint64_t>(kTileBlocks, n_blocks) / n_blocks;  // per (full tile, workgroup)
  const uint32_t capp = ((uint32_t)(ep + 6.0 * sqrt(ep) + 16.0) + 15) & ~15u;
  const uint64_t regions = (uint64_t)q * P;
  const uint64_t p_ovf_n = 256 + 4 * regions;
  const uint64_t p_regions = align256(p_ovf_n + 4ull * P);
  const uint64_t p_ovf = p_regions + 12ull * regions * capp;
  rp.part_ws_bytes = p_ovf + 16ull * P * S * rp.region_cap;
  rp.part_bytes = (uint64_t)q * kTileBlocks * 64;
  return TKV_AMQ_OK;
}

// PartGeom of a part build of tn tiles from S part blocks (its workgroups: the route's)
inline PartGeom route_part_geom(const tkv_amq_route_plan& rp, uint32_t tn, uint32_t S)
{
  PartGeom g{};
  const uint32_t P = rp.route_wgs;
  g.P = P;
  g.n_tiles = tn ? tn : 1;
  g.rb = 12;
  g.per = S * rp.region_cap;
  const double ep = (double)rp.chunk_keys * S / P * std::min<uint64_t>(kTileBlocks, rp.n_blocks) /
                    rp.n_blocks;  // records per (full tile, workgroup)
  g.cap = ((uint32_t)(ep + 6.0 * sqrt(ep) + 16.0) + 15) & ~15u;
  const uint64_t regions = (uint64_t)g.n_tiles * P;
  g.counts_off = 256;
  g.ovf_n_off = g.counts_off + 4 * regions;
  g.regions_off = (g.ovf_n_off + 4ull * P + 255) & ~255ull;
  g.ovf_off = g.regions_off + 12ull * regions * g.cap;
  g.bytes = g.ovf_off + 16ull * P * g.per;
  return g;
}

// jstride 0: the send-buffer layout, part p at p * block_bytes
inline RouteBlock route_block(const tkv_amq_route_plan& rp, uint64_t jstride = 0)
{
  RouteBlock b{};
  b.bytes = rp.block_bytes;
  b.jstride = jstride ? jstride : (uint64_t)rp.world * rp.block_bytes;
  b.counts_off = rp.counts_off;
  b.ovf_n_off = rp.ovf_n_off;
  b.regions_off = rp.regions_off;
  b.ovf_off = rp.ovf_off;
  b.P = rp.route_wgs;
  b.cap = rp.region_cap;
  b.ovf_cap = rp.ovf_cap;
  return b;
}

inline void set_route_attributes()
{
  static std::once_flag attr[kMaxDevices];
  once_per_device(attr, [] {
    for (const void* f : {reinterpret_cast<const void*>(&bloom_route_part<8, 16>),
                          reinterpret_cast<const void*>(&bloom_route_part<7, 16>),
                          reinterpret_cast<const void*>(&bloom_route_part<0, 16>),
                          reinterpret_cast<const void*>(&bloom_route_part<8, 24>),
                          reinterpret_cast<const void*>(&bloom_route_part<0, 24>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)route_lds_bytes(kRouteMaxParts));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_part_segs),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024));
  });
}

// the route of n keys (kb 16 or 24) into the part blocks at d_dst (part p at (p / world) *
// jstride + (p % world) * block_bytes; jstride 0: world * block_bytes) (from_seg: keys [0, n) of
// the segment, n capped by its count -- tkv_amq_build's plan; else exactly n keys)
inline PartArgs route_args(const tkv_amq_route_plan& rp, const uint8_t* keys, uint32_t kb, uint64_t n,
                           uint32_t from_seg, uint8_t* d_dst, uint8_t* ws, uint64_t jstride = 0)
{
  PartArgs a{};
  a.src = keys;
  a.n = (uint32_t)n;
  a.from_seg = from_seg;
  a.kb = kb;
  a.ws = ws;
  a.g.P = rp.route_wgs;
  a.g.n_tiles = rp.n_parts;
  a.g.per = (uint32_t)div_up(rp.chunk_keys, rp.route_wgs);
  a.g.cap = rp.region_cap;
  a.g.rb = 12;
  a.g.ovf_n_off = 512;
  a.g.ovf_off = align256(512 + 4ull * rp.route_wgs);
  a.dst = d_dst;
  a.q = rp.part_tiles;
  a.world = rp.world;
  a.q_magic = div_magic(rp.part_tiles);
  a.w_magic = div_magic(rp.world);
  a.blk = route_block(rp, jstride);
  return a;
}

inline void launch_route_blocks(const PartArgs& a, const tkv_amq_route_plan& rp, hipStream_t s,
                                const tkv_amq_segment* d_seg, bool pack)
{
  set_route_attributes();
  const dim3 g(rp.route_wgs), b(kPartThreads);
  const size_t lds = route_lds_bytes(rp.n_parts);
  if (a.kb == 24 && rp.hash_count == 8) hipLaunchKernelGGL((bloom_route_part<8, 24>), g, b, lds, s, d_seg, a);
  else if (a.kb == 24) hipLaunchKernelGGL((bloom_route_part<0, 24>), g, b, lds, s, d_seg, a);
  else if (rp.hash_count == 8) hipLaunchKernelGGL((bloom_route_part<8, 16>), g, b, lds, s, d_seg, a);
  else if (rp.hash_count == 7) hipLaunchKernelGGL((bloom_route_part<7, 16>), g, b, lds, s, d_seg, a);
  else hipLaunchKernelGGL((bloom_route_part<0, 16>), g, b, lds, s, d_seg, a);
  if (pack) hipLaunchKernelGGL(bloom_route_ovf_pack, dim3(rp.route_wgs), dim3(256), 0, s, a);
}

// part p's tiles from its n_recv part blocks at d_recv, block_bytes apart (partition -> tiles
// -> the partition's own overflow lists); the route overflow entries are applied by the caller
inline void launch_part_from_blocks(const tkv_amq_route_plan& rp, hipStream_t s, const uint8_t* d_recv,
                                    uint32_t n_recv, const tkv_amq_segment* d_seg, uint32_t p, uint8_t* d_out,
                                    uint8_t* ws)
{
  const uint32_t t0 = p * rp.part_tiles;
  if (t0 >= rp.n_tiles) return;
  const uint32_t tn = std::min(rp.part_tiles, rp.n_tiles - t0);
  set_mono_attributes();
  set_route_attributes();
  PartArgs a{};
  a.src = d_recv;
  a.tile0 = t0;
  a.kb = 16;
  a.ws = ws;
  a.g = route_part_geom(rp, tn, n_recv);
  a.src_kind = kSrcSeg12;
  a.blk = route_block(rp);
  a.n_src_segs = n_recv;
  a.seg_part = 0;
  a.tbl = part_tbl_fits(tn) ? 1u : 0u;
  hipLaunchKernelGGL(bloom_part_segs, dim3(a.g.P), dim3(kPartThreads),
                     a.tbl ? part_tbl_lds_bytes(tn) : part_lds_bytes(tn), s, d_seg, a);
  hipLaunchKernelGGL(bloom_tile, dim3(tn), dim3(kTileThreads), 64ull * kTileBlocks, s, d_seg, a, d_out, 1u);
  hipLaunchKernelGGL(bloom_overflow, dim3(a.g.P), dim3(256), 0, s, d_seg, a, d_out);
}

// The monolithic build of one filter (a one-leaf tkv_amq_build batch beyond the window path):
// up to kDirectMaxTiles tiles the partition reads the keys.  Beyond, with k <= 8 (bits_per_key
// <= 12): the one-pass route (bloom_route_part, one block) into parts of <= kRoutePartTiles
// tiles, each part built from its regions (bloom_part_segs -> bloom_tile), then the route
// workgroups' overflow lists applied (bloom_route_ovf_apply; empty for hashed keys).  k > 8
// (or k not derivable from n_keys and n_blocks): the 16-byte keys routed as themselves by the
// two-pass route (count, scan, scatter) into parts of <= kRouteKeyPartTiles tiles.
struct MonoPlan {
  uint32_t T, g, q;  // tiles, parts, tiles per part
  uint32_t k;        // hash count when known (the one-pass route needs 1..8)
  bool blocks;       // the one-pass route
  tkv_amq_route_plan rp;
  RouteGeom rg;      // (the two-pass route)
  uint64_t items_off, part_off;
  PartGeom pg;       // a part of q tiles (every part's own geometry is no larger)
  uint32_t split;    // g == 1: tile workgroups per tile (tile_split), partial images at img_off
  uint64_t img_off;
  uint64_t bytes;
};

inline uint32_t bloom_k_of(uint64_t n_keys, uint64_t n_blocks);

inline MonoPlan mono_plan(uint64_t n_keys, uint64_t n_blocks)
{
  MonoPlan m{};
  m.T = filter_tiles(n_blocks);
  m.k = bloom_k_of(n_keys, n_blocks);  // (0: unknown)
  if (m.T <= kDirectMaxTiles) {
    m.g = 1;
    m.q = m.T;
    m.pg = part_geom(n_keys, n_keys, m.T, 16, mono_wg_items(n_keys, 32ull * kPartThreads));
    m.split = tile_split(m.T);
    m.img_off = align256(m.pg.bytes);
    m.bytes = m.split > 1 ? m.img_off + (uint64_t)m.T * m.split * (64ull * kTileBlocks) : m.pg.bytes;
    return m;
  }
  if (m.k >= 1 && m.k <= 8 && route_plan(n_keys, 1, n_blocks, m.k, 1, false, m.rp) == TKV_AMQ_OK) {
    m.blocks = true;
    m.g = m.rp.n_parts;
    m.q = m.rp.part_tiles;
    m.items_off = align256(m.rp.route_ws_bytes);                  // the part blocks
    m.part_off = align256(m.items_off + (uint64_t)m.rp.n_parts * m.rp.block_bytes);  // a part build's workspace
    m.bytes = m.part_off + m.rp.part_ws_bytes;
    return m;
  }
  m.g = (uint32_t)div_up(m.T, kRouteKeyPartTiles);
  m.q = (uint32_t)div_up(m.T, m.g);
  m.rg = route_geom(n_keys, m.g);
  m.items_off = align256(m.rg.bytes);
  m.part_off = align256(m.items_off + 16ull * n_keys);
  m.pg = part_geom(n_keys, div_up(n_keys, m.g), m.q, 16);
  m.bytes = m.part_off + m.pg.bytes;
  return m;
}

// k of a one-leaf Bloom plan from its key and block counts (the host-side plan is gone by the
// time tkv_amq_build runs; for n >= 512 keys one bits-per-key value gives n_blocks); 0 if none
inline uint32_t bloom_k_of(uint64_t n_keys, uint64_t n_blocks)
{
  for (uint32_t b = 1; b <= 64; ++b) {
    const uint64_t nb = div_up(n_keys * b, 512);
    if ((nb == 0 ? 1 : nb) == n_blocks) return bloom_hash_count(b);
  }
  return 0;
}

// One filter of keys of any other shape (variable-length, or a fixed stride other than 16 and
// 24) with k <= 8 and at most kDirectMaxTiles tiles: the tiled build from bit records that
// bloom_any_records hashes, tiles split over the chip below 128 of them.  Workspace: the
// records, the partition's, the partial tile images.
struct AnyPlan {
  PartGeom pg;
  uint32_t split;
  uint64_t part_off, img_off, bytes;
};

inline bool any_tiled_ok(uint32_t k, uint64_t n_keys, uint64_t n_blocks)
{
  return k >= 1 && k <= 8 && filter_tiles(n_blocks) <= kDirectMaxTiles && n_keys <= 0xffffffffull;
}

inline AnyPlan any_plan(uint64_t n_keys, uint64_t n_blocks)
{
  AnyPlan p{};
  const uint32_t T = filter_tiles(n_blocks);
  p.pg = part_geom(n_keys, n_keys, T, 12, mono_wg_items(n_keys, 32ull * kPartThreads));
  p.split = tile_split(T);
  p.part_off = align256(12ull * n_keys);
  p.img_off = align256(p.part_off + p.pg.bytes);
  p.bytes = p.split > 1 ? p.img_off + (uint64_t)T * p.split * (64ull * kTileBlocks) : p.img_off;
  return p;
}

// keys [0, n) of segment 0 (from its key_begin), offs != nullptr: variable-length
inline void launch_any(const AnyPlan& p, hipStream_t s, const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                       uint32_t n, const tkv_amq_segment* d_seg, uint8_t* ws, uint8_t* d_out)
{
  uint32_t* recs = reinterpret_cast<uint32_t*>(ws);
  const uint32_t g = (uint32_t)div_up(n, 256);
  if (g) {
    if (offs) hipLaunchKernelGGL(bloom_any_records<kKeyVar>, dim3(g), dim3(256), 0, s, keys, offs, 0u, d_seg, n, recs);
    else hipLaunchKernelGGL(bloom_any_records<kKeyFixed>, dim3(g), dim3(256), 0, s, keys, offs, stride, d_seg, n, recs);
  }
  PartArgs a{reinterpret_cast<const uint8_t*>(recs), n, 0u, 0u, 16u, nullptr, 0u, ws + p.part_off, p.pg};
  a.split = p.split;
  a.part_img = ws + p.img_off;
  launch_part_build(kSrcRec12, a, s, d_seg, d_out, 0u);
}

// keys [0, n) of segment 0 (kb 16 or 24; routed 24-byte keys need the one-pass route, k <= 8)
inline void launch_mono(const MonoPlan& m, hipStream_t s, const uint8_t* keys, uint32_t kb, uint32_t n,
                        const tkv_amq_segment* d_segs, uint8_t* ws, uint8_t* d_out, uint64_t key0 = 0)
{
  // (key0: the segment's key_begin, for the two-pass route, which reads keys [0, n) of its
  // pointer; the other paths add the segment's key_begin themselves)
  if (m.g == 1) {
    PartArgs a{keys, n, 0u, 1u, kb, nullptr, 0u, ws, m.pg};
    a.split = m.split;
    a.part_img = ws + m.img_off;
    launch_part_build(kb == 24 ? kSrcKey24 : kSrcKey16, a, s, d_segs, d_out, 0u);
    return;
  }
  if (m.blocks) {
    const tkv_amq_route_plan& rp = m.rp;
    uint8_t* blk = ws + m.items_off;
    const PartArgs ra = route_args(rp, keys, kb, n, 1u, blk, ws);
    launch_route_blocks(ra, rp, s, d_segs, false);
    for (uint32_t p = 0; p < rp.n_parts; ++p)
      launch_part_from_blocks(rp, s, blk + (uint64_t)p * rp.block_bytes, 1, d_segs, p, d_out, ws + m.part_off);
    // the route workgroups' overflow lists (entries: record, part), every part at once
    hipLaunchKernelGGL(bloom_route_ovf_apply, dim3(rp.route_wgs), dim3(256), 0, s, d_segs, ws + ra.g.ovf_n_off,
                       4ull, ws + ra.g.ovf_off, 16ull * ra.g.per, ra.g.per, rp.part_tiles, 0u, rp.n_parts, d_out);
    return;
  }
  uint32_t* rws = reinterpret_cast<uint32_t*>(ws);
  uint8_t* items = ws + m.items_off;
  launch_route(m.rg, s, keys + (uint64_t)kb * key0, kb, n, d_segs, m.q, rws, kb == 16 ? items : nullptr, 9u, items);
  const uint32_t* cnt = rws + (uint64_t)m.rg.P * m.g;  // the part totals
  for (uint32_t j = 0; j < m.g; ++j) {
    const uint32_t t0 = j * m.q, tn = m.T - t0 < m.q ? m.T - t0 : m.q;
    const PartArgs a{items, 0u, t0, 0u, 16u, cnt, j, ws + m.part_off,
                     part_geom(n, div_up(n, m.g), tn, 16)};
    launch_part_build(kSrcRec12, a, s, d_segs, d_out, 0u);
  }
}

// a one-filter Bloom batch too large for one LDS image takes the monolithic build (it needs a
// workspace of mono_plan(n_keys, n_blocks).bytes and 16- or 24-byte keys)
inline bool bloom_partitioned(uint32_t n_segs, uint64_t max_blocks, uint64_t n_keys)
{
  return n_segs == 1 && 64 * max_blocks > kBloomLeafLdsBudget && n_keys <= 0xffffffffull;
}

// A Bloom batch with leaves of more than kWinMaxWindows windows (images past 2.5 MB) among
// others (tkv_amq_build_ex): the other leaves go through the batch kernels from a compacted
// leaf list, each oversize leaf through the monolithic build of its own.  Workspace: the
// compacted list, then the larger of the batch's and the biggest oversize leaf's needs.
inline bool bloom_oversize(uint64_t n_blocks) { return bloom_window_count(n_blocks) > kWinMaxWindows; }

// In a batch of 16- or 24-byte keys the tiled build takes over from the window path earlier:
// past kBatchMonoWindows windows (each window re-reads its part's keys and repeats their first
// hash, the tiled build hashes every key once).  Measured (tools/window_batch.py, 10 bits/key,
// Gkeys/s, window path vs tiled): 128 x 650K keys (5 windows) 44.4 vs 42.0, 64 x 1M (8) 31.5 vs
// 68.6, 48 x 1.5M (12) 25.3 vs 68.0, 32 x 2M (16) 18.4 vs 67.8.  Other key shapes keep the
// window path up to kWinMaxWindows.  (fixed: the batch's keys are 16 or 24 bytes)
constexpr uint32_t kBatchMonoWindows = 5;
inline uint32_t batch_window_max(bool fixed) { return fixed ? kBatchMonoWindows : kWinMaxWindows; }
inline bool batch_tiled(uint64_t n_blocks, bool fixed) { return bloom_window_count(n_blocks) > batch_window_max(fixed); }

inline uint64_t bloom_batch_ws_bytes(uint32_t n_segs, uint64_t n_keys, uint64_t max_blocks)
{
  if (bloom_window_path(n_segs, max_blocks, false))
    return bloom_split_ws_bytes(n_segs, bloom_window_parts(n_segs, n_keys, max_blocks), max_blocks);
  return bloom_split_ws_bytes(n_segs, bloom_split_parts(n_segs, n_keys, max_blocks), max_blocks);
}

// A tiled leaf of at most kDirectMaxTiles tiles joins a multi-leaf launch (bloom_part_multi).
// Its partition workgroups take the batch's tiled keys / 256 each, between 1,024 keys and 4
// batches: few keys still spread over every CU (a lone 3M-key leaf: 256 workgroups), many give
// each workgroup a pipeline of 4 batches and the chip several rounds of workgroups per launch,
// so a short last round idles little of it.  Measured against 8 batches (Gkeys/s): 64 x 1M
// keys 68.6 vs 64.2, 32 x 2M 67.8 vs 64.4, 8 x 3M + 200 x 16K 71.9 vs 63.4, 64 x 3M 70.6 vs
// 72.2; a workgroup size chosen per launch from its keys (launch keys / 768) measured no
// steadier (60.4 / 64.2 / 72.8 / 72.9).  The leaves of one launch share the workspace budget
// below (a leaf larger than it runs alone).
constexpr uint64_t kMultiWsBudget = 2ull << 30;

inline uint64_t multi_wg_items(uint64_t multi_keys) { return mono_wg_items(multi_keys, 4ull * kPartBatch); }

// (a batch of 16- or 24-byte keys)
inline bool multi_leaf(uint64_t n_keys, uint64_t n_blocks)
{
  return batch_tiled(n_blocks, true) && filter_tiles(n_blocks) <= kDirectMaxTiles && n_keys <= 0xffffffffull;
}

inline PartGeom multi_geom(uint64_t n_keys, uint64_t n_blocks, uint64_t wg_items)
{
  return part_geom(n_keys, n_keys, filter_tiles(n_blocks), 16, wg_items);
}

// the keys (and, in `count`, the number) of a batch's multi-leaf candidates
inline uint64_t multi_keys_of(const tkv_amq_segment* segs, uint32_t n_segs, uint32_t* count = nullptr)
{
  uint64_t n = 0;
  uint32_t c = 0;
  for (uint32_t i = 0; i < n_segs; ++i)
    if (segs[i].bits_per_key && multi_leaf(segs[i].n_keys, segs[i].n_blocks)) {
      n += segs[i].n_keys;
      ++c;
    }
  if (count) *count = c;
  return n;
}

inline size_t multi_lds_bytes(uint32_t n_tiles)
{
  return part_tbl_fits(n_tiles) ? part_tbl_lds_bytes(n_tiles) : part_lds_bytes(n_tiles);
}

// the leaves' tile grids (T_l * S each) and merge grids (T_l * kMergeChunks, split tiles only)
// for the group's tile split S, and its partial images from split_img
inline void multi_split(MultiParts& m, uint32_t n_tiles, uint8_t* split_img)
{
  const uint32_t S = tile_split(n_tiles);
  for (uint32_t i = 0; i < m.n; ++i) {
    MultiLeaf& l = m.l[i];
    const uint32_t t0 = l.tg0;
    l.split = S;
    l.part_img = split_img + ((uint64_t)t0 * S << 17);
    l.tg0 = t0 * S;
    l.mg0 = t0 * kMergeChunks;
  }
}

inline void launch_multi(const MultiParts& m, uint32_t kb, uint32_t n_wgs, uint32_t n_tiles, size_t lds, hipStream_t s,
                         const tkv_amq_segment* d_segs, uint8_t* d_out)
{
  static std::once_flag attr[kMaxDevices];
  once_per_device(attr, [] {
    for (const void* f : {reinterpret_cast<const void*>(&bloom_part_multi16),
                          reinterpret_cast<const void*>(&bloom_part_multi24)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_tile_multi),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(64 * kTileBlocks));
  });
  if (kb == 24) hipLaunchKernelGGL(bloom_part_multi24, dim3(n_wgs), dim3(kPartThreads), lds, s, d_segs, m);
  else hipLaunchKernelGGL(bloom_part_multi16, dim3(n_wgs), dim3(kPartThreads), lds, s, d_segs, m);
  const uint32_t S = m.n ? (m.l[0].split > 1 ? m.l[0].split : 1u) : 1u;
  hipLaunchKernelGGL(bloom_tile_multi, dim3(n_tiles * S), dim3(kTileThreads), 64ull * kTileBlocks, s, d_segs, m,
                     d_out);
  if (S > 1)
    hipLaunchKernelGGL(bloom_tile_merge_multi, dim3(n_tiles * kMergeChunks), dim3(256), 0, s, d_segs, m, d_out);
  hipLaunchKernelGGL(bloom_overflow_multi, dim3(n_wgs), dim3(256), 0, s, d_segs, m, d_out);
}

// The workspace of a tkv_amq_build_ex batch, for either key shape (the plan does not know
// it): 16- or 24-byte keys -- the leaves past kBatchMonoWindows windows tiled (multi-leaf
// launches, or alone past kDirectMaxTiles tiles), the others batched; other key shapes -- the
// leaves up to kWinMaxWindows windows batched (the window path), the larger ones with device
// atomics.  After the compacted leaf list.
inline uint64_t bloom_oversize_ws_bytes(const tkv_amq_segment* segs, uint32_t n_segs)
{
  uint64_t need = 0;
  for (const bool fixed : {true, false}) {
    uint32_t n_small = 0;
    uint64_t small_keys = 0, small_max = 0, big = 0, multi_sum = 0, multi_max = 0;
    const uint64_t wg_items = multi_wg_items(multi_keys_of(segs, n_segs));
    for (uint32_t i = 0; i < n_segs; ++i) {
      const tkv_amq_segment& g = segs[i];
      if (!batch_tiled(g.n_blocks, fixed)) {
        ++n_small;
        small_keys += g.n_keys;
        small_max = std::max<uint64_t>(small_max, g.n_blocks);
      } else if (fixed && multi_leaf(g.n_keys, g.n_blocks)) {
        const uint64_t b = align256(multi_geom(g.n_keys, g.n_blocks, wg_items).bytes);
        multi_sum += b;
        multi_max = std::max(multi_max, b);
      } else if (fixed) {
        big = std::max(big, mono_plan(g.n_keys, g.n_blocks).bytes);
      } else if (any_tiled_ok(g.hash_count, g.n_keys, g.n_blocks)) {
        big = std::max(big, any_plan(g.n_keys, g.n_blocks).bytes);  // (bloom_part_any)
      }
    }
    const uint64_t small = n_small ? bloom_batch_ws_bytes(n_small, small_keys, small_max) : 0;
    const uint64_t multi = multi_sum ? std::min(multi_sum, std::max(multi_max, kMultiWsBudget)) + kSplitImgBytes : 0;
    need = std::max(need, std::max(std::max(small, big), multi));
  }
  return align256(64ull * n_segs) + need;
}

}  // namespace

extern "C" {

const char* tkv_amq_version(void) { return "tkv-amq 0.1.0 (spec tkv-amq-v1, gfx950)"; }

const char* tkv_amq_status_string(int s)
{
  switch (s) {
    case TKV_AMQ_OK: return "OK";
    case TKV_AMQ_INVALID_ARGUMENT: return "InvalidArgument";
    case TKV_AMQ_RESOURCE_EXHAUSTED: return "ResourceExhausted";
    case TKV_AMQ_INTERNAL: return "Internal";
    case TKV_AMQ_UNAVAILABLE: return "Unavailable";
    default: return "Unknown";
  }
}

int tkv_amq_device_count(void)
{
  // the visible device set is fixed for the life of the process: ask the runtime once (every
  // entry point checks it, and the per-leaf path calls several entry points per leaf)
  static const int n = [] {
    int c = 0;
    return hipGetDeviceCount(&c) == hipSuccess ? c : 0;
  }();
  return n;
}

uint64_t tkv_amq_filter_bits_per_key(int kind, uint64_t bpk)
{
  // tree/tree_options.hpp:155-164
  if (kind != TKV_AMQ_VQF) return bpk;
  return bpk == 0 ? 0 : (bpk < 12 ? 12 : bpk);
}

double tkv_amq_vqf_load_factor(int tag_bits, uint64_t bpk)
{
  // vqf_filter_page_view.hpp:39-59
  if (bpk == 0) return 0;
  const double b = (double)bpk;
  return tag_bits == 8 ? 10.2 / b : 18.0 / b;
}

uint64_t tkv_amq_vqf_required_size(int tag_bits, uint64_t nslots)
{
  const uint64_t s = vqf_slots(tag_bits);
  return kVqfMetadata + 64ull * ((nslots + s) / s);
}

uint64_t tkv_amq_vqf_nslots_for_size(int tag_bits, uint64_t bytes)
{
  if (bytes < kVqfMetadata + 64) return 0;
  return (bytes - kVqfMetadata) / 64 * vqf_slots(tag_bits) - 1;
}

// ---- TreeOptions filter page sizing (tree/tree_options.hpp:177-258) ----
uint64_t tkv_amq_leaf_data_size(uint64_t leaf_size)
{
  // leaf_max_space_from_size (tree/packed_leaf_page.hpp:307-311)
  constexpr uint64_t kOverhead = kPackedPageHeaderBytes + kPackedLeafPageBytes + kPackedArrayBytes;
  return leaf_size > kOverhead ? leaf_size - kOverhead : 0;
}

uint64_t tkv_amq_expected_items_per_leaf(uint64_t leaf_size, uint32_t key_size_hint,
                                         uint32_t value_size_hint)
{
  // expected_item_size (:246-253), PackedSizeOfEdit (core/packed_sizeof_edit.hpp:13-15):
  // u32 key length + key + u32 value offset + 1 op byte + value
  const uint64_t item = 4ull + key_size_hint + 4ull + 1ull + value_size_hint;
  return tkv_amq_leaf_data_size(leaf_size) / item;
}

static uint32_t log2_ceil_u64(uint64_t x)
{
  uint32_t k = 0;
  while (k < 64 && (1ull << k) < x) ++k;
  return k;
}

uint32_t tkv_amq_filter_page_size_log2(int kind, uint64_t leaf_size, uint32_t key_size_hint,
                                       uint32_t value_size_hint, uint64_t bits_per_key)
{
  const uint64_t bpk = tkv_amq_filter_bits_per_key(kind, bits_per_key);
  const uint64_t items = tkv_amq_expected_items_per_leaf(leaf_size, key_size_hint, value_size_hint);
  uint64_t page;
  if (kind == TKV_AMQ_BLOOM) {
    // round_up_bits(9, items * bpk) / 8 + page header + PackedBloomFilterPage (:184-191)
    const uint64_t bits = (items * bpk + 511) & ~511ull;
    page = kPackedPageHeaderBytes + kBloomHeader + bits / 8;
  } else if (kind == TKV_AMQ_VQF) {
    if (bpk == 0) return 0;  // no filter pages (the reference would take ceil(n / 0.0))
    // (:195-209): ceil(items / load factor) slots at 8 and 16 tag bits, the larger size
    const double n = (double)items;
    const uint64_t s8 = (uint64_t)ceil(n / tkv_amq_vqf_load_factor(8, bpk));
    const uint64_t s16 = (uint64_t)ceil(n / tkv_amq_vqf_load_factor(16, bpk));
    const uint64_t f8 = tkv_amq_vqf_required_size(8, s8), f16 = tkv_amq_vqf_required_size(16, s16);
    page = (f8 > f16 ? f8 : f16) + kPackedPageHeaderBytes + kVqfHeader + kVqfMetadata;
  } else {
    return 0;
  }
  return log2_ceil_u64(page);
}

int tkv_amq_plan(int kind, const uint64_t* counts, const uint64_t* src_ids, uint32_t n_segs,
                 uint32_t bpk, uint64_t cap, uint64_t stride, tkv_amq_segment* segs,
                 uint64_t* total_out, uint64_t* ws_bytes, uint32_t* max_blocks_out)
{
  if ((kind != TKV_AMQ_BLOOM && kind != TKV_AMQ_VQF) || (n_segs && (!counts || !segs)))
    return TKV_AMQ_INVALID_ARGUMENT;
  if (kind == TKV_AMQ_BLOOM && bpk > 64) return TKV_AMQ_INVALID_ARGUMENT;
  if (kind == TKV_AMQ_VQF && bpk != 0 && bpk < 12) return TKV_AMQ_INVALID_ARGUMENT;  // :46
  if (stride && (stride % 64)) return TKV_AMQ_INVALID_ARGUMENT;
  if (kind == TKV_AMQ_VQF && bpk != 0 && cap == 0) return TKV_AMQ_INVALID_ARGUMENT;

  uint64_t off = 0, key_begin = 0, block_base = 0;
  uint32_t max_blocks = 0;
  for (uint32_t s = 0; s < n_segs; ++s) {
    tkv_amq_segment& g = segs[s];
    memset(&g, 0, sizeof(g));
    const uint64_t n = counts[s];
    if (n > 0xffffffffull) return TKV_AMQ_INVALID_ARGUMENT;
    g.key_begin = key_begin;
    g.src_page_id = src_ids ? src_ids[s] : s;
    g.n_keys = (uint32_t)n;
    g.bits_per_key = bpk;
    key_begin += n;
    uint64_t payload = 0;
    if (bpk != 0 && kind == TKV_AMQ_BLOOM) {
      // build_bloom_filter_for_leaf, filter_builder.hpp:126-135 (kBlocked512, k = None)
      const uint64_t nb = div_up(n * bpk, 512) == 0 ? 1 : div_up(n * bpk, 512);
      if (nb > 0xffffffffull) return TKV_AMQ_RESOURCE_EXHAUSTED;
      g.n_blocks = (uint32_t)nb;
      g.hash_count = (uint16_t)bloom_hash_count(bpk);
      payload = kBloomHeader + 64 * nb;
      if (cap && payload > cap) return TKV_AMQ_RESOURCE_EXHAUSTED;
    } else if (bpk != 0) {
      // build_quotient_filter_for_leaf sizing, filter_builder.hpp:241-290
      if (cap < kVqfHeader + kVqfMetadata + 64) return TKV_AMQ_RESOURCE_EXHAUSTED;
      const uint64_t max8 = tkv_amq_vqf_nslots_for_size(8, cap - kVqfHeader);
      const uint64_t max16 = tkv_amq_vqf_nslots_for_size(16, cap - kVqfHeader);
      const double n_keys = (double)n;
      const double lf8 = tkv_amq_vqf_load_factor(8, bpk);
      const double lf16 = tkv_amq_vqf_load_factor(16, bpk);
      const uint64_t n8 = (uint64_t)floor(n_keys / lf8);
      const uint64_t n16 = (uint64_t)floor(n_keys / lf16);
      if (!(lf8 <= 0.85)) return TKV_AMQ_INVALID_ARGUMENT;  // :265
      int t;
      uint64_t nslots;
      uint32_t shift = 0;
      if (lf16 <= 0.85 && n16 <= max16) {
        t = 16;
        nslots = n16;
      } else if (n8 <= max8) {
        t = 8;
        nslots = n8;
      } else {
        if (!(max8 > max16)) return TKV_AMQ_INTERNAL;  // :278
        shift = 1;
        while ((double)(n >> shift) / lf8 > (double)max8) ++shift;
        t = 8;
        nslots = max8;
      }
      const uint64_t sl = vqf_slots(t);
      const uint64_t nb = (nslots + sl) / sl;
      if (nb > kVqfMaxBlocks) return TKV_AMQ_RESOURCE_EXHAUSTED;
      g.n_blocks = (uint32_t)nb;
      g.tag_bits = (uint8_t)t;
      g.hash_val_shift = (uint8_t)shift;
      g.block_base = block_base;
      g.mod_magic = ~0ull / (nb * vqf_buckets(t));
      block_base += nb;
      payload = kVqfHeader + tkv_amq_vqf_required_size(t, nslots);
    }
    if (g.n_blocks > max_blocks) max_blocks = g.n_blocks;
    g.payload_bytes = (uint32_t)payload;
    if (stride) {
      if (payload > stride) return TKV_AMQ_RESOURCE_EXHAUSTED;
      g.out_offset = (uint64_t)s * stride;
    } else {
      g.out_offset = off;
      off += (payload + 63) & ~63ull;
    }
  }
  if (total_out) *total_out = stride ? stride * n_segs : off;
  if (ws_bytes) {
    *ws_bytes = 0;
    if (kind == TKV_AMQ_VQF && bpk != 0)
      *ws_bytes = vqf_temp_offset(n_segs) + kVqfTempStride * block_base + 8 * key_begin + 64;
    // (the window path for one 16- or 24-byte-key filter above kWinMonoMax windows is not
    // taken: the monolithic workspace below; any other window batch, its partial images.  The
    // plan does not know the key shape, so a single filter of kWinMonoMax+1 .. kWinMaxWindows
    // windows gets the larger of the two: other key shapes take the window path with it)
    const uint64_t win_ws =
        kind == TKV_AMQ_BLOOM && bpk != 0 && bloom_window_path(n_segs, max_blocks, false)
            ? bloom_split_ws_bytes(n_segs, bloom_window_parts(n_segs, key_begin, max_blocks), max_blocks)
            : 0;
    if (kind == TKV_AMQ_BLOOM && bpk != 0 && bloom_window_path(n_segs, max_blocks, true))
      *ws_bytes = win_ws;
    else if (kind == TKV_AMQ_BLOOM && bloom_partitioned(n_segs, max_blocks, key_begin))
      // (the plan does not know the key shape: other shapes take bloom_any_records' records)
      *ws_bytes = std::max<uint64_t>({mono_plan(key_begin, max_blocks).bytes, win_ws,
                                      any_tiled_ok(segs[0].hash_count, key_begin, max_blocks)
                                          ? any_plan(key_begin, max_blocks).bytes
                                          : uint64_t{0}});
    else if (kind == TKV_AMQ_BLOOM)
      *ws_bytes = bloom_split_ws_bytes(n_segs, bloom_split_parts(n_segs, key_begin, max_blocks),
                                       max_blocks);
    if (kind == TKV_AMQ_BLOOM && bpk != 0 && n_segs > 1 && batch_tiled(max_blocks, true))
      *ws_bytes = bloom_oversize_ws_bytes(segs, n_segs);
  }
  if (max_blocks_out) *max_blocks_out = max_blocks;
  return TKV_AMQ_OK;
}

int tkv_amq_plan_pages(int kind, const uint64_t* counts, const uint64_t* src_ids, uint32_t n_segs,
                       uint32_t bpk, uint32_t page_log2, tkv_amq_segment* segs, uint64_t* total_out,
                       uint64_t* ws_bytes, uint32_t* max_blocks_out)
{
  // FilterPageAlloc's page buffer: a 64-byte PackedPageHeader, then the payload the builders
  // size against (filter_builder.hpp:231-244)
  if (page_log2 < 7 || page_log2 > 31) return TKV_AMQ_INVALID_ARGUMENT;
  const uint64_t page = 1ull << page_log2;
  const int st = tkv_amq_plan(kind, counts, src_ids, n_segs, bpk, page - kPackedPageHeaderBytes,
                              page, segs, total_out, ws_bytes, max_blocks_out);
  if (st != TKV_AMQ_OK) return st;
  for (uint32_t s = 0; s < n_segs; ++s) {
    segs[s].out_offset += kPackedPageHeaderBytes;
    segs[s].page_flags = TKV_AMQ_PAGE_IMAGE | (page_log2 << 8);
  }
  return TKV_AMQ_OK;
}

// tkv_amq_build with the keys its leaves hold (sizing_keys: the Bloom launch heuristics and the
// monolithic plan) apart from the key array's count (n_keys: what the device-atomics fallback
// and VQF scan): tkv_amq_build_ex's compacted small leaves are a subset of the array's keys
static int build_batch(int kind, const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                       uint64_t n_keys, const tkv_amq_segment* d_segs, uint32_t n_segs,
                       uint32_t max_blocks, uint8_t* d_out, void* d_ws, uint64_t ws_bytes, void* stream,
                       uint64_t sizing_keys);

int tkv_amq_build(int kind, const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                  uint64_t n_keys, const tkv_amq_segment* d_segs, uint32_t n_segs,
                  uint32_t max_blocks, uint8_t* d_out, void* d_ws, uint64_t ws_bytes, void* stream)
{
  return build_batch(kind, keys, offs, stride, n_keys, d_segs, n_segs, max_blocks, d_out, d_ws, ws_bytes,
                     stream, n_keys);
}

static int build_batch(int kind, const uint8_t* keys, const uint64_t* offs, uint32_t stride,
                       uint64_t n_keys, const tkv_amq_segment* d_segs, uint32_t n_segs,
                       uint32_t max_blocks, uint8_t* d_out, void* d_ws, uint64_t ws_bytes, void* stream,
                       uint64_t sizing_keys)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n_segs == 0) return TKV_AMQ_OK;
  if (!d_segs || !d_out || (n_keys && !keys) || (!offs && stride == 0))
    return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  const int mode = key_mode(offs, stride);
  if (mode == kKey16 && (reinterpret_cast<uintptr_t>(keys) & 15)) return TKV_AMQ_INVALID_ARGUMENT;

  if (kind == TKV_AMQ_BLOOM) {
    const uint64_t lds = 64ull * max_blocks;
    if (max_blocks == 0) return TKV_AMQ_OK;
    const uint32_t parts = bloom_split_parts(n_segs, sizing_keys, max_blocks);
    const uint64_t split_ws = bloom_split_ws_bytes(n_segs, parts, max_blocks);
    if (parts > 1 && d_ws && ws_bytes >= split_ws) {
      // a small batch: each leaf's keys over `parts` workgroups, then their images ORed
      static std::once_flag split_attr[kMaxDevices];
      once_per_device(split_attr, [] {
        const int cap = (int)kBloomLeafLdsBudget;
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_build_split<kKey16>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, cap);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_build_split<kKey24>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, cap);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_build_split<kKeyFixed>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, cap);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bloom_build_split<kKeyVar>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, cap);
      });
      const int bmode = build_key_mode(keys, offs, stride);
      const dim3 grid(n_segs * parts), block(kSplitThreads);
      uint8_t* w = static_cast<uint8_t*>(d_ws);
      const uint64_t img = 64ull * max_blocks;
      if (bmode == kKey24)
        hipLaunchKernelGGL(bloom_build_split<kKey24>, grid, block, lds, s, keys, offs, stride, d_segs,
                           parts, w, img);
      else if (mode == kKey16)
        hipLaunchKernelGGL(bloom_build_split<kKey16>, grid, block, lds, s, keys, offs, stride, d_segs,
                           parts, w, img);
      else if (mode == kKeyFixed)
        hipLaunchKernelGGL(bloom_build_split<kKeyFixed>, grid, block, lds, s, keys, offs, stride,
                           d_segs, parts, w, img);
      else
        hipLaunchKernelGGL(bloom_build_split<kKeyVar>, grid, block, lds, s, keys, offs, stride, d_segs,
                           parts, w, img);
      const uint32_t chunks = (uint32_t)div_up(4ull * max_blocks, kMergeThreads);
      hipLaunchKernelGGL(bloom_split_merge, dim3(n_segs * chunks), dim3(kMergeThreads), 0, s, d_segs,
                         parts, chunks, w, img, d_out);
      return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
    }
    // one filter beyond the window path: 16- and 24-byte keys take the monolithic build (each
    // key hashed once); 24-byte keys with k > 8 only up to kDirectMaxTiles tiles (their records
    // hold eight bits, and the others are set from the keys, which the route does not carry)
    const int mono_mode = build_key_mode(keys, offs, stride);
    const bool mono_part = bloom_partitioned(n_segs, max_blocks, sizing_keys) && d_ws;
    const MonoPlan mp = mono_plan(sizing_keys, max_blocks);
    const bool mono16 = mono_part && mode == kKey16 && ws_bytes >= mp.bytes;
    // (routed 24-byte keys travel as bit records only: k must be known -- bloom_k_of 0 means
    // the plan does not match n_keys -- and at most 8)
    const uint32_t k_route = bloom_k_of(sizing_keys, max_blocks);
    const bool mono24 = mono_part && mono_mode == kKey24 && ws_bytes >= mp.bytes &&
                        (mp.g == 1 || (mp.blocks && k_route >= 1 && k_route <= 8));
    if (bloom_window_path(n_segs, max_blocks, mono16 || mono24)) {
      // leaves beyond one CU's LDS: windows of the image, parts of the keys
      const uint32_t W = bloom_window_count(max_blocks), wblk = bloom_window_blocks(max_blocks);
      uint32_t wparts = bloom_window_parts(n_segs, sizing_keys, max_blocks);
      if (wparts > 1 && (!d_ws || ws_bytes < bloom_split_ws_bytes(n_segs, wparts, max_blocks)))
        wparts = 1;  // no workspace for partial images: one part per leaf, no merge
      static std::once_flag win_attr[kMaxDevices];
      once_per_device(win_attr, [] {
        for (const void* f : {reinterpret_cast<const void*>(&bloom_build_window<kKey16>),
                              reinterpret_cast<const void*>(&bloom_build_window<kKey24>),
                              reinterpret_cast<const void*>(&bloom_build_window<kKeyFixed>),
                              reinterpret_cast<const void*>(&bloom_build_window<kKeyVar>)})
          (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kBloomLeafLdsBudget);
      });
      const int bmode = build_key_mode(keys, offs, stride);
      const dim3 grid(n_segs * W * wparts), block(kWinThreads);
      const size_t wl = 64ull * wblk;
      uint8_t* w = static_cast<uint8_t*>(d_ws);
      const uint64_t img = 64ull * max_blocks;
      if (bmode == kKey24)
        hipLaunchKernelGGL(bloom_build_window<kKey24>, grid, block, wl, s, keys, offs, stride, d_segs,
                           W, wblk, wparts, w, img, d_out);
      else if (mode == kKey16)
        hipLaunchKernelGGL(bloom_build_window<kKey16>, grid, block, wl, s, keys, offs, stride, d_segs,
                           W, wblk, wparts, w, img, d_out);
      else if (mode == kKeyFixed)
        hipLaunchKernelGGL(bloom_build_window<kKeyFixed>, grid, block, wl, s, keys, offs, stride, d_segs,
                           W, wblk, wparts, w, img, d_out);
      else
        hipLaunchKernelGGL(bloom_build_window<kKeyVar>, grid, block, wl, s, keys, offs, stride, d_segs,
                           W, wblk, wparts, w, img, d_out);
      if (wparts > 1) {
        const uint32_t chunks = (uint32_t)div_up(4ull * max_blocks, kMergeThreads);
        hipLaunchKernelGGL(bloom_split_merge, dim3(n_segs * chunks), dim3(kMergeThreads), 0, s, d_segs,
                           wparts, chunks, w, img, d_out);
      }
      return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
    }
    if (lds <= kBloomLeafLdsBudget && n_segs >= kBloomSpreadSegs) {
      const int bmode = build_key_mode(keys, offs, stride);
      // (variable-length keys add their length-sort scratch: kVarAuxWords)
      if (lds + (mode == kKeyVar ? 4ull * kVarAuxWords<1024> : 0ull) > kBloomLdsBudget) {
        static std::once_flag big_attr[kMaxDevices];
        once_per_device(big_attr, [] {
          for (const void* f : {reinterpret_cast<const void*>(&bloom_build_lds<kKey16, 1024>),
                                reinterpret_cast<const void*>(&bloom_build_lds<kKey24, 1024>),
                                reinterpret_cast<const void*>(&bloom_build_lds<kKeyFixed, 1024>),
                                reinterpret_cast<const void*>(&bloom_build_lds<kKeyVar, 1024>)})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kBloomLeafLdsBudget);
        });
      }
      if (n_segs < kBloomWideSegs || lds > kBloomWideLds)
        launch_bloom_lds<1024>(bmode, mode, n_segs, lds, s, keys, offs, stride, d_segs, d_out);
      else
        launch_bloom_lds<256>(bmode, mode, n_segs, lds, s, keys, offs, stride, d_segs, d_out);
      return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
    }
    const bool mono_any = mono_part && !mono16 && !mono24 && mode != kKey16 && mono_mode != kKey24 &&
                          any_tiled_ok(k_route, sizing_keys, max_blocks) &&
                          ws_bytes >= any_plan(sizing_keys, max_blocks).bytes;
    if (mono16 || mono24) {
      // one monolithic filter: every key hashed once into its bit record, records partitioned
      // by tile (routed into parts first beyond kDirectMaxTiles tiles), tiles built in LDS
      launch_mono(mp, s, keys, mono24 ? 24u : 16u, (uint32_t)sizing_keys, d_segs, static_cast<uint8_t*>(d_ws),
                  d_out);
    } else if (mono_any) {
      // one filter of variable-length or other fixed-size keys: the same, from bit records
      // (bloom_any_records)
      launch_any(any_plan(sizing_keys, max_blocks), s, keys, mode == kKeyVar ? offs : nullptr, stride,
                 (uint32_t)sizing_keys, d_segs, static_cast<uint8_t*>(d_ws), d_out);
    } else {
      // fewer than kBloomSpreadSegs leaves, leaves beyond the LDS budget in a multi-leaf batch,
      // or a monolithic filter whose keys are neither 16 nor 24 bytes (or 24-byte keys with
      // k > 8 beyond kDirectMaxTiles tiles): device atomics
      const dim3 g1(n_segs), b(256);
      hipLaunchKernelGGL(bloom_global_init, g1, b, 0, s, d_segs, d_out);
      const uint32_t g2 = (uint32_t)(div_up(n_keys, 256) < 8192 ? div_up(n_keys, 256) : 8192);
      if (g2) {
        if (mode == kKey16)
          hipLaunchKernelGGL(bloom_global_set<kKey16>, dim3(g2), b, 0, s, keys, offs, stride,
                             d_segs, n_segs, n_keys, d_out, 0ull);
        else if (mode == kKeyFixed)
          hipLaunchKernelGGL(bloom_global_set<kKeyFixed>, dim3(g2), b, 0, s, keys, offs, stride,
                             d_segs, n_segs, n_keys, d_out, 0ull);
        else
          hipLaunchKernelGGL(bloom_global_set<kKeyVar>, dim3(g2), b, 0, s, keys, offs, stride,
                             d_segs, n_segs, n_keys, d_out, 0ull);
      }
    }
    return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
  }

  if (kind != TKV_AMQ_VQF) return TKV_AMQ_INVALID_ARGUMENT;
  if (max_blocks == 0) {
    // no kernel runs: a later tkv_amq_build_check must not read an earlier build's flags
    if (d_ws && ws_bytes >= 64 && hipMemsetAsync(static_cast<uint8_t*>(d_ws) + 4, 0, 4, s) != hipSuccess)
      return TKV_AMQ_INTERNAL;
    return TKV_AMQ_OK;
  }
  if (max_blocks > kVqfMaxBlocks) return TKV_AMQ_RESOURCE_EXHAUSTED;
  if (!d_ws) return TKV_AMQ_INVALID_ARGUMENT;
  // the status word and leaf counts must be writable; the rest is checked on the device
  // against the plan (every leaf with a filter has >= 1 block record, every key one record)
  if (ws_bytes < vqf_temp_offset(n_segs) + kVqfTempStride * (uint64_t)max_blocks + 8 * n_keys)
    return TKV_AMQ_INVALID_ARGUMENT;
  // (no memset: every decide workgroup writes the header's leaf count and its leaf's nelts
  // word, flags included, so tkv_amq_build_check reads only this build's results)
  // LDS: u32 block counts (+ the u64 lane-mask table when every leaf is small enough)
  // The lane-mask table costs 8 B of LDS per block in every decide wave, and wins even where
  // it costs waves per CU: 6,104 leaves of 804 blocks 2.49 -> 2.14 ms (16 instead of 24 waves
  // per CU), 2,048 of 1,961 blocks 3.03 -> 2.52 ms, against block-id ballots
  const int match_lds = max_blocks <= kVqfMatchLdsBlocks;
  // a leaf whose LDS image exceeds the budget is placed by up to kFusedMaxParts workgroups
  const uint32_t place_parts =
      (uint32_t)div_up(max_blocks, kFusedLdsBudget / (4 * kFusedRegionWords));
  const uint32_t place_span = (uint32_t)div_up(max_blocks, place_parts);
  const uint32_t fused_lds = vqf_fused_lds_bytes(place_span);
  const bool fused = place_parts <= kFusedMaxParts;  // compact records are read only there
  // the count table: u32 in LDS up to kVqfMaxLdsBlocks, u8 in LDS up to kVqfU8LdsBlocks, else
  // in the workspace's block records (VqfCountMode)
  const int cnt_mode = max_blocks <= kVqfMaxLdsBlocks ? kCntU32
                       : (max_blocks <= kVqfU8LdsBlocks ? kCntU8 : kCntGlobal);
  const int flags = match_lds | (fused ? 2 : 0);
  const size_t lds = cnt_mode == kCntU8 ? (size_t)((max_blocks + 15) & ~15u)
                     : cnt_mode == kCntGlobal ? 16
                     : 4ull * ((max_blocks + 1) & ~1u) + (match_lds ? 8ull * max_blocks : 0);
  const int vmode = build_key_mode(keys, offs, stride);
  if (cnt_mode != kCntU32) {
    // a leaf past the u32 count table: vqf_decide_big for the whole batch (fused place is out
    // of reach for such a leaf, so the records are the 8-byte ones)
    static std::once_flag big_attr[kMaxDevices];
    once_per_device(big_attr, [] {
      for (const void* f : {reinterpret_cast<const void*>(&vqf_decide_big<kKey16, kCntU8>),
                            reinterpret_cast<const void*>(&vqf_decide_big<kKey24, kCntU8>),
                            reinterpret_cast<const void*>(&vqf_decide_big<kKeyFixed, kCntU8>),
                            reinterpret_cast<const void*>(&vqf_decide_big<kKeyVar, kCntU8>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    const dim3 g(n_segs), b(64);
#define TKV_DECIDE_BIG(CNT)                                                                         \
  do {                                                                                              \
    if (vmode == kKey16)                                                                            \
      hipLaunchKernelGGL((vqf_decide_big<kKey16, CNT>), g, b, lds, s, keys, offs, stride, d_segs, d_ws, \
                         ws_bytes, n_segs);                                                         \
    else if (vmode == kKey24)                                                                       \
      hipLaunchKernelGGL((vqf_decide_big<kKey24, CNT>), g, b, lds, s, keys, offs, stride, d_segs, d_ws, \
                         ws_bytes, n_segs);                                                         \
    else if (mode == kKeyFixed)                                                                     \
      hipLaunchKernelGGL((vqf_decide_big<kKeyFixed, CNT>), g, b, lds, s, keys, offs, stride, d_segs,    \
                         d_ws, ws_bytes, n_segs);                                                   \
    else                                                                                            \
      hipLaunchKernelGGL((vqf_decide_big<kKeyVar, CNT>), g, b, lds, s, keys, offs, stride, d_segs,      \
                         d_ws, ws_bytes, n_segs);                                                   \
  } while (0)
    if (cnt_mode == kCntU8) TKV_DECIDE_BIG(kCntU8);
    else TKV_DECIDE_BIG(kCntGlobal);
#undef TKV_DECIDE_BIG
  }
  // the ring kernel for small batches of leaves its count table holds (a batch with a larger
  // leaf takes vqf_decide: the one-wave body inside the ring kernel set its registers, and so
  // its workgroups per CU, for every batch).  Keys other than 16 bytes are read where they are
  // hashed, which puts their load latency on vqf_decide's serial chain: the ring kernel, whose
  // producers hash off the chain, stays faster up to ~4,096 leaves for them (1,024 leaves of
  // 24-byte keys 0.47 -> 0.29 ms, variable-length 0.66 -> 0.38 ms; at 6,104 leaves vqf_decide
  // wins, 1.25 vs 1.45 ms)
  // 24-byte keys (TurtleKV's default key size hint), 8-byte aligned, are loaded ahead of
  // their hash like 16-byte ones
  const bool prefetched = vmode == kKey16 || vmode == kKey24;
  const bool rp1 = n_segs <= kRingPlaceMaxSegs && max_blocks <= kRingPlaceMaxBlocks;
  const bool rp2 = !rp1 && n_segs <= kRingPlace2MaxSegs && max_blocks <= kRingPlace2MaxBlocks;
  if (cnt_mode == kCntU32 && (rp1 || rp2)) {
    // decide and place in one workgroup per leaf (vqf_ring_place): no key records, one launch;
    // up to 256 leaves one workgroup per CU (ring of kRingPlaceSlots, match tables), up to 512 two
    static std::once_flag rp_attr[kMaxDevices];
    once_per_device(rp_attr, [] {
      for (const void* f : {reinterpret_cast<const void*>(&vqf_ring_place<kKey16, kRingPlaceSlots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKey24, kRingPlaceSlots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyFixed, kRingPlaceSlots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyVar, kRingPlaceSlots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKey16, kRingPlace2Slots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKey24, kRingPlace2Slots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyFixed, kRingPlace2Slots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyVar, kRingPlace2Slots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyLoc, kRingPlaceSlots>),
                            reinterpret_cast<const void*>(&vqf_ring_place<kKeyLoc, kRingPlace2Slots>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    const dim3 g(n_segs), b(kRingThreads);
    const uint32_t cw = ring_place_cnt_words(max_blocks);
    const uint32_t tbl = rp1 && max_blocks <= kRingTblBlocks;  // (ring_place_lds_bytes sizes them)
    const size_t rl = rp1 ? ring_place_lds_bytes(max_blocks) : ring_place_lds_bytes(max_blocks, kRingPlace2Slots, false);
    // keys read where they are hashed (other than 16 or 24 bytes: the producers, not the
    // decider, set a lone leaf's time): every key hashed and located on the whole chip first
    // (vqf_locate_keys), the ring's producers then read 8-byte located records
    const bool loc = !prefetched && n_segs <= (mode == kKeyVar ? kVqfLocMaxSegsVar : kVqfLocMaxSegsFixed);
    if (loc && n_keys > 0) {
      const dim3 lg((uint32_t)div_up(n_keys, 256)), lb(256);
      if (mode == kKeyFixed)
        hipLaunchKernelGGL(vqf_locate_keys<kKeyFixed>, lg, lb, 0, s, keys, offs, stride, d_segs, d_ws, ws_bytes, n_segs,
                           n_keys);
      else
        hipLaunchKernelGGL(vqf_locate_keys<kKeyVar>, lg, lb, 0, s, keys, offs, stride, d_segs, d_ws, ws_bytes, n_segs,
                           n_keys);
    }
#define TKV_RING_PLACE(NS)                                                                              \
  do {                                                                                                  \
    if (loc)                                                                                            \
      hipLaunchKernelGGL((vqf_ring_place<kKeyLoc, NS>), g, b, rl, s, nullptr, nullptr, 0, d_segs, d_ws,   \
                         ws_bytes, n_segs, d_out, cw, tbl);                                             \
    else if (vmode == kKey16)                                                                           \
      hipLaunchKernelGGL((vqf_ring_place<kKey16, NS>), g, b, rl, s, keys, offs, stride, d_segs, d_ws,     \
                         ws_bytes, n_segs, d_out, cw, tbl);                                             \
    else if (vmode == kKey24)                                                                           \
      hipLaunchKernelGGL((vqf_ring_place<kKey24, NS>), g, b, rl, s, keys, offs, stride, d_segs, d_ws,     \
                         ws_bytes, n_segs, d_out, cw, tbl);                                             \
    else if (mode == kKeyFixed)                                                                         \
      hipLaunchKernelGGL((vqf_ring_place<kKeyFixed, NS>), g, b, rl, s, keys, offs, stride, d_segs, d_ws,  \
                         ws_bytes, n_segs, d_out, cw, tbl);                                             \
    else                                                                                                \
      hipLaunchKernelGGL((vqf_ring_place<kKeyVar, NS>), g, b, rl, s, keys, offs, stride, d_segs, d_ws,    \
                         ws_bytes, n_segs, d_out, cw, tbl);                                             \
  } while (0)
    if (rp1) TKV_RING_PLACE(kRingPlaceSlots);
    else TKV_RING_PLACE(kRingPlace2Slots);
#undef TKV_RING_PLACE
    return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
  }
  if (cnt_mode != kCntU32) {
    // (decided above)
  } else if (n_segs <= (prefetched ? kVqfRingMaxSegs : kVqfRingMaxSegsOther) &&
             max_blocks <= kRingMaxBlocks) {
    static std::once_flag ring_attr[kMaxDevices];
    once_per_device(ring_attr, [] {
      for (const void* f : {reinterpret_cast<const void*>(&vqf_decide_ring<kKey16>),
                            reinterpret_cast<const void*>(&vqf_decide_ring<kKey24>),
                            reinterpret_cast<const void*>(&vqf_decide_ring<kKeyFixed>),
                            reinterpret_cast<const void*>(&vqf_decide_ring<kKeyVar>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    const dim3 g(n_segs), b(kRingThreads);
    const size_t rl = lds > kRingLdsBytes ? lds : kRingLdsBytes;
    if (vmode == kKey16)
      hipLaunchKernelGGL(vqf_decide_ring<kKey16>, g, b, rl, s, keys, offs, stride, d_segs, d_ws,
                         ws_bytes, n_segs, flags);
    else if (vmode == kKey24)
      hipLaunchKernelGGL(vqf_decide_ring<kKey24>, g, b, rl, s, keys, offs, stride, d_segs, d_ws,
                         ws_bytes, n_segs, flags);
    else if (mode == kKeyFixed)
      hipLaunchKernelGGL(vqf_decide_ring<kKeyFixed>, g, b, rl, s, keys, offs, stride, d_segs, d_ws,
                         ws_bytes, n_segs, flags);
    else
      hipLaunchKernelGGL(vqf_decide_ring<kKeyVar>, g, b, rl, s, keys, offs, stride, d_segs, d_ws,
                         ws_bytes, n_segs, flags);
  } else if (vmode == kKey16)
    hipLaunchKernelGGL(vqf_decide<kKey16>, dim3(n_segs), dim3(64), lds, s, keys, offs, stride,
                       d_segs, d_ws, ws_bytes, n_segs, flags);
  else if (vmode == kKey24)
    hipLaunchKernelGGL(vqf_decide<kKey24>, dim3(n_segs), dim3(64), lds, s, keys, offs, stride,
                       d_segs, d_ws, ws_bytes, n_segs, flags);
  else if (mode == kKeyFixed)
    hipLaunchKernelGGL(vqf_decide<kKeyFixed>, dim3(n_segs), dim3(64), lds, s, keys, offs, stride,
                       d_segs, d_ws, ws_bytes, n_segs, flags);
  else
    hipLaunchKernelGGL(vqf_decide<kKeyVar>, dim3(n_segs), dim3(64), lds, s, keys, offs, stride,
                       d_segs, d_ws, ws_bytes, n_segs, flags);
  if (fused) {
    static std::once_flag lds_attr[kMaxDevices];
    once_per_device(lds_attr, [] {
      for (const void* f : {reinterpret_cast<const void*>(&vqf_place_fused<256>),
                            reinterpret_cast<const void*>(&vqf_place_fused<512>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFusedLdsBudget);
    });
    // 512 threads for a batch that does not fill the chip (the ring-decide sizes) or leaves of
    // more than 512 blocks: lone leaf 98 -> 95 us, 2,048 x 80K keys 2.51 -> 2.30 ms; 256 for a
    // full batch of small leaves (0.709 vs 0.697 ms at 100M keys)
    const dim3 pg(n_segs * place_parts);
    if (n_segs <= kVqfRingMaxSegs || max_blocks > 512)
      hipLaunchKernelGGL(vqf_place_fused<512>, pg, dim3(512), fused_lds, s, d_segs, d_ws, ws_bytes,
                         n_segs, d_out, place_parts, place_span);
    else
      hipLaunchKernelGGL(vqf_place_fused<256>, pg, dim3(256), fused_lds, s, d_segs, d_ws, ws_bytes,
                         n_segs, d_out, place_parts, place_span);
  } else {
    if (n_keys)
      hipLaunchKernelGGL(vqf_scatter, dim3((uint32_t)div_up(n_keys, 256)), dim3(256), 0, s,
                         d_segs, d_ws, ws_bytes, n_segs, n_keys);
    // several workgroups per leaf for large leaves (each takes every parts-th group of
    // kPlaceThreads blocks)
    const uint32_t parts = (uint32_t)(div_up(max_blocks, 4 * kPlaceThreads) < 256
                                          ? div_up(max_blocks, 4 * kPlaceThreads) : 256);
    hipLaunchKernelGGL(vqf_place, dim3(n_segs * parts), dim3(kPlaceThreads), 0, s, d_segs, d_ws,
                       ws_bytes, n_segs, d_out, parts);
  }
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_build_ex(int kind, const uint8_t* keys, const uint64_t* offs, uint32_t stride, uint64_t n_keys,
                     const tkv_amq_segment* d_segs, const tkv_amq_segment* h_segs, uint32_t n_segs,
                     uint32_t max_blocks, uint8_t* d_out, void* d_ws, uint64_t ws_bytes, void* stream)
{
  const int mode = key_mode(offs, stride), bmode = build_key_mode(keys, offs, stride);
  const bool fixed = mode == kKey16 || bmode == kKey24;  // the tiled build takes these keys
  if (kind != TKV_AMQ_BLOOM || !h_segs || n_segs < 2 || !batch_tiled(max_blocks, fixed))
    return tkv_amq_build(kind, keys, offs, stride, n_keys, d_segs, n_segs, max_blocks, d_out, d_ws, ws_bytes,
                         stream);
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (!d_segs || !d_out || (n_keys && !keys) || (!offs && stride == 0)) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  const uint64_t list_bytes = align256(64ull * n_segs);
  if (!d_ws || ws_bytes < list_bytes) return TKV_AMQ_INVALID_ARGUMENT;
  uint8_t* ws = static_cast<uint8_t*>(d_ws);
  uint8_t* rest = ws + list_bytes;
  const uint64_t rest_bytes = ws_bytes - list_bytes;
  uint32_t n_small = 0, small_max = 0;
  uint64_t small_keys = 0;  // (the inner build's launch heuristics size from these)
  for (uint32_t i = 0; i < n_segs; ++i)
    if (!batch_tiled(h_segs[i].n_blocks, fixed)) {
      ++n_small;
      small_max = std::max(small_max, h_segs[i].n_blocks);
      small_keys += h_segs[i].n_keys;
    }
  if (n_small) {
    tkv_amq_segment* list = reinterpret_cast<tkv_amq_segment*>(ws);
    const uint32_t small_blocks = batch_window_max(fixed) * (kBloomLeafLdsBudget / 64);
    hipLaunchKernelGGL(bloom_compact_segs, dim3(1), dim3(n_segs <= 4096 ? 256 : 1024), 0, s, d_segs, n_segs,
                       small_blocks, list);
    const int st = build_batch(kind, keys, offs, stride, n_keys, list, n_small, small_max, d_out, rest,
                               rest_bytes, stream, small_keys);
    if (st != TKV_AMQ_OK) return st;
  }
  // the tiled leaves of at most kDirectMaxTiles tiles: multi-leaf launches, as many leaves
  // per launch as the workspace holds
  MultiParts m{};
  const uint32_t mkb = mode == kKey16 ? 16u : 24u;
  m.keys = keys;
  m.kb = mkb;
  uint64_t used = 0;
  uint32_t wgs = 0, tiles = 0;
  size_t lds = 0;
  // the group's partial tile images first, then the leaves' workspaces
  uint8_t* const mrest = rest + kSplitImgBytes;
  const uint64_t mbudget = rest_bytes > kSplitImgBytes ? rest_bytes - kSplitImgBytes : 0;
  auto flush = [&] {
    if (m.n) {
      multi_split(m, tiles, rest);
      launch_multi(m, mkb, wgs, tiles, lds, s, d_segs, d_out);
    }
    m.n = 0;
    used = 0;
    wgs = tiles = 0;
    lds = 0;
  };
  const bool multi_keys = fixed;
  uint32_t n_multi = 0;
  const uint64_t tiled_keys = multi_keys_of(h_segs, n_segs, &n_multi);
  const uint64_t wg_items = multi_wg_items(tiled_keys);
  // leaves per launch: as even as the launches allow (no short last launch)
  const uint32_t per_launch = n_multi ? (uint32_t)div_up(n_multi, div_up(n_multi, kMultiMaxLeaves)) : 1u;
  for (uint32_t i = 0; i < n_segs; ++i) {
    const tkv_amq_segment& g = h_segs[i];
    if (!batch_tiled(g.n_blocks, fixed) || g.bits_per_key == 0) continue;
    if (multi_keys && multi_leaf(g.n_keys, g.n_blocks)) {
      const PartGeom pg = multi_geom(g.n_keys, g.n_blocks, wg_items);
      const uint64_t b = align256(pg.bytes);
      if (b <= mbudget) {
        if (m.n == per_launch || used + b > mbudget) flush();
        MultiLeaf& l = m.l[m.n];
        l = MultiLeaf{};
        l.ws = mrest + used;
        l.counts_off = pg.counts_off;
        l.ovf_n_off = pg.ovf_n_off;
        l.regions_off = pg.regions_off;
        l.ovf_off = pg.ovf_off;
        l.n = (uint32_t)g.n_keys;
        l.P = pg.P;
        l.n_tiles = pg.n_tiles;
        l.per = pg.per;
        l.cap = pg.cap;
        l.tbl = part_tbl_fits(pg.n_tiles) ? 1u : 0u;
        l.wg0 = wgs;
        l.tg0 = tiles;
        l.seg = i;
        ++m.n;
        used += b;
        wgs += pg.P;
        tiles += pg.n_tiles;
        lds = std::max(lds, multi_lds_bytes(pg.n_tiles));
        continue;
      }
    }
    const MonoPlan mp = mono_plan(g.n_keys, g.n_blocks);
    const uint32_t k = bloom_k_of(g.n_keys, g.n_blocks);
    const bool mono = rest_bytes >= mp.bytes &&
                      (mode == kKey16 || (bmode == kKey24 && (mp.g == 1 || (mp.blocks && k >= 1 && k <= 8))));
    const bool any = !mono && mode != kKey16 && bmode != kKey24 && any_tiled_ok(g.hash_count, g.n_keys, g.n_blocks) &&
                     rest_bytes >= any_plan(g.n_keys, g.n_blocks).bytes;
    if (mono) {
      launch_mono(mp, s, keys, mode == kKey16 ? 16u : 24u, g.n_keys, d_segs + i, rest, d_out, g.key_begin);
    } else if (any) {
      // variable-length or other fixed-size keys: hashed into bit records (bloom_any_records),
      // then the tiled build
      launch_any(any_plan(g.n_keys, g.n_blocks), s, keys, mode == kKeyVar ? offs : nullptr, stride,
                 (uint32_t)g.n_keys, d_segs + i, rest, d_out);
    } else {
      // other key shapes (or no room): device atomics for this leaf alone
      hipLaunchKernelGGL(bloom_global_init, dim3(1), dim3(256), 0, s, d_segs + i, d_out);
      const uint32_t g2 = (uint32_t)std::min<uint64_t>(div_up(g.n_keys, 256), 8192);
      if (g2) {
        const uint64_t end = g.key_begin + g.n_keys;
        if (mode == kKey16)
          hipLaunchKernelGGL(bloom_global_set<kKey16>, dim3(g2), dim3(256), 0, s, keys, offs, stride, d_segs + i, 1u,
                             end, d_out, g.key_begin);
        else if (mode == kKeyFixed)
          hipLaunchKernelGGL(bloom_global_set<kKeyFixed>, dim3(g2), dim3(256), 0, s, keys, offs, stride, d_segs + i,
                             1u, end, d_out, g.key_begin);
        else
          hipLaunchKernelGGL(bloom_global_set<kKeyVar>, dim3(g2), dim3(256), 0, s, keys, offs, stride, d_segs + i,
                             1u, end, d_out, g.key_begin);
      }
    }
  }
  flush();
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

uint32_t tkv_amq_bloom_tile_blocks(void) { return kTileBlocks; }

uint32_t tkv_amq_bloom_range_max_tiles(int records)
{
  return records ? kRecPartMaxTiles : kDirectMaxTiles;
}

uint64_t tkv_amq_bloom_route_ws_bytes(uint64_t n_keys, uint32_t n_parts)
{
  if (n_parts == 0 || n_parts > kRouteMaxParts) return 0;
  return route_geom(n_keys, n_parts).bytes;
}

int tkv_amq_bloom_route(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                        uint32_t n_blocks, uint32_t n_parts, uint8_t* d_routed16,
                        uint32_t* d_part_counts, void* d_ws, uint64_t ws_bytes, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n_parts == 0 || n_parts > kRouteMaxParts || n_blocks == 0 || !d_seg || !d_part_counts ||
      n_keys > 0xffffffffull)
    return TKV_AMQ_INVALID_ARGUMENT;
  if (n_keys && (!d_keys16 || !d_routed16 || (reinterpret_cast<uintptr_t>(d_keys16) & 15) ||
                 (reinterpret_cast<uintptr_t>(d_routed16) & 15)))
    return TKV_AMQ_INVALID_ARGUMENT;
  const RouteGeom g = route_geom(n_keys, n_parts);
  if (!d_ws || ws_bytes < g.bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  uint32_t* w = static_cast<uint32_t*>(d_ws);
  const uint32_t q = (uint32_t)div_up(filter_tiles(n_blocks), n_parts);
  launch_route(g, s, d_keys16, 16, (uint32_t)n_keys, d_seg, q, w, d_routed16, 0u, nullptr);
  // the per-part totals route_scan_cols left after the histogram
  if (hipMemcpyAsync(d_part_counts, w + g.h_words, 4ull * n_parts, hipMemcpyDeviceToDevice, s) !=
      hipSuccess)
    return TKV_AMQ_INTERNAL;
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

uint64_t tkv_amq_bloom_route_records_ws_bytes(uint64_t n_keys, uint32_t n_parts)
{
  return tkv_amq_bloom_route_ws_bytes(n_keys, n_parts);
}

int tkv_amq_bloom_route_records(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                                uint32_t n_blocks, uint32_t hash_count, uint32_t n_parts,
                                uint8_t* d_recs12, uint32_t* d_part_counts, void* d_ws, uint64_t ws_bytes,
                                void* stream)
{
  return tkv_amq_bloom_route_records_ex(d_keys16, 16, n_keys, d_seg, n_blocks, hash_count, n_parts,
                                        d_recs12, d_part_counts, d_ws, ws_bytes, stream);
}

int tkv_amq_bloom_route_records_ex(const uint8_t* d_keys, uint32_t key_bytes, uint64_t n_keys,
                                   const tkv_amq_segment* d_seg, uint32_t n_blocks, uint32_t hash_count,
                                   uint32_t n_parts, uint8_t* d_recs12, uint32_t* d_part_counts,
                                   void* d_ws, uint64_t ws_bytes, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n_parts == 0 || n_parts > kRouteMaxParts || n_blocks == 0 || !d_seg || !d_part_counts ||
      n_keys > 0xffffffffull || hash_count == 0 || hash_count > 8 || (key_bytes != 16 && key_bytes != 24))
    return TKV_AMQ_INVALID_ARGUMENT;
  // a record's tile field holds the tile relative to its part: parts of <= kRecPartMaxTiles
  const uint32_t q = (uint32_t)div_up(filter_tiles(n_blocks), n_parts);
  if (q > kRecPartMaxTiles) return TKV_AMQ_INVALID_ARGUMENT;
  const uintptr_t kalign = key_bytes == 16 ? 15 : 7;
  if (n_keys && (!d_keys || !d_recs12 || (reinterpret_cast<uintptr_t>(d_keys) & kalign) ||
                 (reinterpret_cast<uintptr_t>(d_recs12) & 3)))
    return TKV_AMQ_INVALID_ARGUMENT;
  const RouteGeom g = route_geom(n_keys, n_parts);
  if (!d_ws || ws_bytes < g.bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  uint32_t* w = static_cast<uint32_t*>(d_ws);
  launch_route(g, s, d_keys, key_bytes, (uint32_t)n_keys, d_seg, q, w, nullptr, 0u, d_recs12);
  if (hipMemcpyAsync(d_part_counts, w + g.h_words, 4ull * n_parts, hipMemcpyDeviceToDevice, s) !=
      hipSuccess)
    return TKV_AMQ_INTERNAL;
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

uint64_t tkv_amq_bloom_build_range_records_ws_bytes(uint64_t n_recs, uint32_t tile_begin, uint32_t tile_end)
{
  if (tile_end <= tile_begin || tile_end - tile_begin > kRecPartMaxTiles || n_recs > 0xffffffffull) return 0;
  return part_geom(n_recs, n_recs, tile_end - tile_begin, 12).bytes;
}

int tkv_amq_bloom_build_range_records(const uint8_t* d_recs12, uint64_t n_recs, const tkv_amq_segment* d_seg,
                                      uint32_t n_blocks, uint32_t hash_count, uint32_t tile_begin,
                                      uint32_t tile_end, uint8_t* d_out, void* d_ws, uint64_t ws_bytes,
                                      void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  const uint32_t T = filter_tiles(n_blocks);
  if (!d_seg || !d_out || n_blocks == 0 || tile_begin > tile_end || tile_end > T ||
      tile_end - tile_begin > kRecPartMaxTiles || n_recs > 0xffffffffull || hash_count == 0 ||
      hash_count > 8)
    return TKV_AMQ_INVALID_ARGUMENT;
  if (n_recs && (!d_recs12 || (reinterpret_cast<uintptr_t>(d_recs12) & 3))) return TKV_AMQ_INVALID_ARGUMENT;
  if (tile_begin == tile_end) {
    hipLaunchKernelGGL(bloom_header_only, dim3(1), dim3(64), 0, as_stream(stream), d_seg, d_out);
    return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
  }
  const PartGeom g = part_geom(n_recs, n_recs, tile_end - tile_begin, 12);
  if (!d_ws || ws_bytes < g.bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const PartArgs a{d_recs12, (uint32_t)n_recs, tile_begin, 0u, 16u, nullptr, 0u, static_cast<uint8_t*>(d_ws), g};
  launch_part_build(kSrcRec12, a, as_stream(stream), d_seg, d_out, 1u);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_bloom_route_plan(uint64_t chunk_keys, uint32_t n_chunks, uint32_t n_blocks,
                             uint32_t hash_count, uint32_t world, tkv_amq_route_plan* plan)
{
  if (!plan) return TKV_AMQ_INVALID_ARGUMENT;
  return route_plan(chunk_keys, n_chunks, n_blocks, hash_count, world, true, *plan);
}

int tkv_amq_bloom_route_blocks(const uint8_t* d_keys, uint32_t key_bytes, uint64_t n_keys,
                               const tkv_amq_segment* d_seg, const tkv_amq_route_plan* plan,
                               uint8_t* d_dst, uint64_t round_stride, void* d_ws, uint64_t ws_bytes,
                               void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (!plan || !d_seg || !d_dst || (key_bytes != 16 && key_bytes != 24) || n_keys > plan->chunk_keys ||
      plan->hash_count == 0 || plan->hash_count > 8 || plan->route_wgs == 0 || plan->world == 0)
    return TKV_AMQ_INVALID_ARGUMENT;
  // a round's world blocks must not overlap the next round's
  if (round_stride && round_stride < (uint64_t)plan->world * plan->block_bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const uintptr_t kalign = key_bytes == 16 ? 15 : 7;
  if (n_keys && (!d_keys || (reinterpret_cast<uintptr_t>(d_keys) & kalign))) return TKV_AMQ_INVALID_ARGUMENT;
  if (!d_ws || ws_bytes < plan->route_ws_bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const PartArgs a = route_args(*plan, d_keys, key_bytes, n_keys, 0u, d_dst, static_cast<uint8_t*>(d_ws),
                                round_stride);
  launch_route_blocks(a, *plan, as_stream(stream), d_seg, true);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_bloom_build_part_blocks(const uint8_t* d_recv, uint32_t n_recv, const tkv_amq_segment* d_seg,
                                    const tkv_amq_route_plan* plan, uint32_t part, uint8_t* d_out,
                                    void* d_ws, uint64_t ws_bytes, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (!plan || !d_seg || !d_out || !d_recv || n_recv == 0 || n_recv > kMaxSrcSegs || part >= plan->n_parts ||
      plan->hash_count == 0 || plan->hash_count > 8)
    return TKV_AMQ_INVALID_ARGUMENT;
  // the workspace sized for n_recv blocks (every source region full)
  tkv_amq_route_plan rp = *plan;
  const PartGeom g = route_part_geom(rp, rp.part_tiles, n_recv);
  if (!d_ws || ws_bytes < g.bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  if (part * rp.part_tiles >= rp.n_tiles) {  // a part past the last tile: the header only
    hipLaunchKernelGGL(bloom_header_only, dim3(1), dim3(64), 0, s, d_seg, d_out);
    return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
  }
  uint8_t* ws = static_cast<uint8_t*>(d_ws);
  launch_part_from_blocks(rp, s, d_recv, n_recv, d_seg, part, d_out, ws);
  // the part's overflow entries from every received block
  hipLaunchKernelGGL(bloom_route_ovf_apply, dim3(n_recv), dim3(256), 0, s, d_seg, d_recv + rp.ovf_n_off,
                     rp.block_bytes, d_recv + rp.ovf_off, rp.block_bytes, rp.ovf_cap, rp.part_tiles, part,
                     part + 1, d_out);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_bloom_blocks_lost(const uint8_t* d_recv, uint32_t n_recv, const tkv_amq_route_plan* plan,
                              void* stream)
{
  if (tkv_amq_device_count() == 0) return -TKV_AMQ_UNAVAILABLE;
  if (!plan || (n_recv && !d_recv)) return -TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  std::vector<uint32_t> n(n_recv ? n_recv : 1);
  if (n_recv && hipMemcpy2DAsync(n.data(), 4, d_recv + plan->ovf_n_off, plan->block_bytes, 4, n_recv,
                                 hipMemcpyDeviceToHost, s) != hipSuccess)
    return -TKV_AMQ_INTERNAL;
  if (hipStreamSynchronize(s) != hipSuccess) return -TKV_AMQ_INTERNAL;
  for (uint32_t i = 0; i < n_recv; ++i)
    if (n[i] > plan->ovf_cap) return 1;
  return 0;
}

uint64_t tkv_amq_bloom_build_range_ws_bytes(uint64_t n_keys, uint32_t tile_begin, uint32_t tile_end)
{
  if (tile_end <= tile_begin || tile_end - tile_begin > kDirectMaxTiles || n_keys > 0xffffffffull) return 0;
  return part_geom(n_keys, n_keys, tile_end - tile_begin, 16).bytes;
}

int tkv_amq_bloom_build_range(const uint8_t* d_keys16, uint64_t n_keys, const tkv_amq_segment* d_seg,
                              uint32_t n_blocks, uint32_t tile_begin, uint32_t tile_end,
                              uint8_t* d_out, void* d_ws, uint64_t ws_bytes, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  const uint32_t T = filter_tiles(n_blocks);
  if (!d_seg || !d_out || n_blocks == 0 || tile_begin > tile_end || tile_end > T ||
      tile_end - tile_begin > kDirectMaxTiles || n_keys > 0xffffffffull)
    return TKV_AMQ_INVALID_ARGUMENT;
  if (n_keys && (!d_keys16 || (reinterpret_cast<uintptr_t>(d_keys16) & 15)))
    return TKV_AMQ_INVALID_ARGUMENT;
  if (tile_begin == tile_end) {
    // a rank past the last tile range (ceil(T / q) < ranks): its part of the result is the
    // header, which every range build writes
    hipLaunchKernelGGL(bloom_header_only, dim3(1), dim3(64), 0, as_stream(stream), d_seg, d_out);
    return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
  }
  const PartGeom g = part_geom(n_keys, n_keys, tile_end - tile_begin, 16);
  if (!d_ws || ws_bytes < g.bytes) return TKV_AMQ_INVALID_ARGUMENT;
  const PartArgs a{d_keys16, (uint32_t)n_keys, tile_begin, 0u, 16u, nullptr, 0u, static_cast<uint8_t*>(d_ws), g};
  launch_part_build(kSrcKey16, a, as_stream(stream), d_seg, d_out, 1u);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_build_check(int kind, const void* d_ws, uint64_t ws_bytes, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  const hipStream_t s = as_stream(stream);
  if (hipStreamSynchronize(s) != hipSuccess) return TKV_AMQ_INTERNAL;
  if (kind != TKV_AMQ_VQF || !d_ws || ws_bytes < 64) return TKV_AMQ_OK;
  // the last build's leaf count, then every leaf's flags (VqfWorkspace)
  uint32_t hdr[2] = {0, 0};
  if (hipMemcpy(hdr, d_ws, 8, hipMemcpyDeviceToHost) != hipSuccess) return TKV_AMQ_INTERNAL;
  const uint64_t n_segs = hdr[1];
  if (n_segs == 0) return TKV_AMQ_OK;
  if (64 + 4 * n_segs > ws_bytes) return TKV_AMQ_INVALID_ARGUMENT;
  std::vector<uint32_t> nelts(n_segs);
  if (hipMemcpy(nelts.data(), static_cast<const uint8_t*>(d_ws) + 64, 4 * n_segs,
                hipMemcpyDeviceToHost) != hipSuccess)
    return TKV_AMQ_INTERNAL;
  uint32_t flags = 0;
  for (const uint32_t w : nelts) flags |= w;
  if (flags & kVqfFlagWorkspace) return TKV_AMQ_INVALID_ARGUMENT;
  return (flags & kVqfFlagOverflow) ? TKV_AMQ_INTERNAL : TKV_AMQ_OK;
}

int tkv_amq_probe(int kind, const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                  uint32_t n_segs, const uint8_t* q, const uint64_t* qoffs, uint32_t stride,
                  uint64_t n, const uint32_t* d_qseg, uint8_t* d_result, void* stream)
{
  return tkv_amq_probe_ex(kind, d_filters, d_segs, n_segs, q, qoffs, stride, n, d_qseg, d_result,
                          nullptr, stream);
}

int tkv_amq_probe_ex(int kind, const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                     uint32_t n_segs, const uint8_t* q, const uint64_t* qoffs, uint32_t stride,
                     uint64_t n, const uint32_t* d_qseg, uint8_t* d_result,
                     const tkv_amq_probe_opts* opts, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!d_filters || !d_segs || !q || !d_qseg || !d_result || n_segs == 0 || (!qoffs && !stride))
    return TKV_AMQ_INVALID_ARGUMENT;
  if (kind != TKV_AMQ_BLOOM && kind != TKV_AMQ_VQF) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  const int mode = key_mode(qoffs, stride);
  if (mode == kKey16 && (reinterpret_cast<uintptr_t>(q) & 15)) return TKV_AMQ_INVALID_ARGUMENT;
  const tkv_amq_probe_opts o = probe_opts(opts);
  const bool ex = probe_opts_used(o);
  const dim3 grid(probe_grid(n, ex)), block(256);
#define TKV_PROBE_LAUNCH(KERNEL, MODE)                                                         \
  do {                                                                                         \
    if (ex)                                                                                    \
      hipLaunchKernelGGL((KERNEL<MODE, true>), grid, block, 0, s, d_filters, d_segs, n_segs, q, \
                         qoffs, stride, n, d_qseg, d_result, o);                               \
    else                                                                                       \
      hipLaunchKernelGGL((KERNEL<MODE, false>), grid, block, 0, s, d_filters, d_segs, n_segs,  \
                         q, qoffs, stride, n, d_qseg, d_result, o);                            \
  } while (0)
  if (kind == TKV_AMQ_BLOOM) {
    if (mode == kKey16) TKV_PROBE_LAUNCH(bloom_probe, kKey16);
    else if (mode == kKeyFixed) TKV_PROBE_LAUNCH(bloom_probe, kKeyFixed);
    else TKV_PROBE_LAUNCH(bloom_probe, kKeyVar);
  } else {
    if (mode == kKey16) TKV_PROBE_LAUNCH(vqf_probe, kKey16);
    else if (mode == kKeyFixed) TKV_PROBE_LAUNCH(vqf_probe, kKeyFixed);
    else TKV_PROBE_LAUNCH(vqf_probe, kKeyVar);
  }
#undef TKV_PROBE_LAUNCH
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_vqf_hash(const uint8_t* q, const uint64_t* qoffs, uint32_t stride, uint64_t n,
                     uint64_t* d_hash, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!q || !d_hash || (!qoffs && !stride)) return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  const int mode = key_mode(qoffs, stride);
  if (mode == kKey16 && (reinterpret_cast<uintptr_t>(q) & 15)) return TKV_AMQ_INVALID_ARGUMENT;
  const dim3 grid((uint32_t)div_up(n, 256)), block(256);
  if (mode == kKey16)
    hipLaunchKernelGGL(vqf_hash_kernel<kKey16>, grid, block, 0, s, q, qoffs, stride, n, d_hash);
  else if (mode == kKeyFixed)
    hipLaunchKernelGGL(vqf_hash_kernel<kKeyFixed>, grid, block, 0, s, q, qoffs, stride, n, d_hash);
  else
    hipLaunchKernelGGL(vqf_hash_kernel<kKeyVar>, grid, block, 0, s, q, qoffs, stride, n, d_hash);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_vqf_probe_hashed(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                             uint32_t n_segs, const uint64_t* d_hash, const uint32_t* d_pair_query,
                             uint64_t n, const uint32_t* d_qseg, uint8_t* d_result, void* stream)
{
  return tkv_amq_vqf_probe_hashed_ex(d_filters, d_segs, n_segs, d_hash, d_pair_query, n, d_qseg,
                                     d_result, nullptr, stream);
}

int tkv_amq_vqf_probe_hashed_ex(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                                uint32_t n_segs, const uint64_t* d_hash,
                                const uint32_t* d_pair_query, uint64_t n, const uint32_t* d_qseg,
                                uint8_t* d_result, const tkv_amq_probe_opts* opts, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!d_filters || !d_segs || !d_hash || !d_qseg || !d_result || n_segs == 0)
    return TKV_AMQ_INVALID_ARGUMENT;
  const tkv_amq_probe_opts o = probe_opts(opts);
  const bool ex = probe_opts_used(o);
  if (ex)
    hipLaunchKernelGGL(vqf_probe_hashed<true>, dim3(probe_grid(n, true)), dim3(256), 0,
                       as_stream(stream), d_filters, d_segs, n_segs, d_hash, d_pair_query, n, d_qseg,
                       d_result, o);
  else
    hipLaunchKernelGGL(vqf_probe_hashed<false>, dim3(probe_grid(n, false)), dim3(256), 0,
                       as_stream(stream), d_filters, d_segs, n_segs, d_hash, d_pair_query, n, d_qseg,
                       d_result, o);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

uint32_t tkv_amq_bloom_query_stride(uint32_t k_max) { return bloom_query_stride(k_max); }

int tkv_amq_bloom_hash(const uint8_t* q, const uint64_t* qoffs, uint32_t stride, uint64_t n,
                       uint32_t k_max, uint8_t* d_query, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!q || !d_query || (!qoffs && !stride) || k_max == 0 || k_max > kMaxBloomHashes)
    return TKV_AMQ_INVALID_ARGUMENT;
  const hipStream_t s = as_stream(stream);
  const int mode = key_mode(qoffs, stride);
  if (mode == kKey16 && (reinterpret_cast<uintptr_t>(q) & 15)) return TKV_AMQ_INVALID_ARGUMENT;
  const dim3 grid((uint32_t)div_up(n, 256)), block(256);
  if (mode == kKey16)
    hipLaunchKernelGGL(bloom_hash_kernel<kKey16>, grid, block, 0, s, q, qoffs, stride, n, k_max, d_query);
  else if (mode == kKeyFixed)
    hipLaunchKernelGGL(bloom_hash_kernel<kKeyFixed>, grid, block, 0, s, q, qoffs, stride, n, k_max, d_query);
  else
    hipLaunchKernelGGL(bloom_hash_kernel<kKeyVar>, grid, block, 0, s, q, qoffs, stride, n, k_max, d_query);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_bloom_probe_hashed(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                               uint32_t n_segs, const uint8_t* d_query, uint32_t k_max,
                               const uint32_t* d_pair_query, uint64_t n, const uint32_t* d_qseg,
                               uint8_t* d_result, void* stream)
{
  return tkv_amq_bloom_probe_hashed_ex(d_filters, d_segs, n_segs, d_query, k_max, d_pair_query, n,
                                       d_qseg, d_result, nullptr, stream);
}

int tkv_amq_bloom_probe_hashed_ex(const uint8_t* d_filters, const tkv_amq_segment* d_segs,
                                  uint32_t n_segs, const uint8_t* d_query, uint32_t k_max,
                                  const uint32_t* d_pair_query, uint64_t n, const uint32_t* d_qseg,
                                  uint8_t* d_result, const tkv_amq_probe_opts* opts, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!d_filters || !d_segs || !d_query || !d_qseg || !d_result || n_segs == 0 || k_max == 0 ||
      k_max > kMaxBloomHashes)
    return TKV_AMQ_INVALID_ARGUMENT;
  const tkv_amq_probe_opts o = probe_opts(opts);
  const bool ex = probe_opts_used(o);
  if (ex)
    hipLaunchKernelGGL(bloom_probe_hashed<true>, dim3(probe_grid(n, true)), dim3(256), 0,
                       as_stream(stream), d_filters, d_segs, n_segs, d_query, k_max, d_pair_query, n,
                       d_qseg, d_result, o);
  else
    hipLaunchKernelGGL(bloom_probe_hashed<false>, dim3(probe_grid(n, false)), dim3(256), 0,
                       as_stream(stream), d_filters, d_segs, n_segs, d_query, k_max, d_pair_query, n,
                       d_qseg, d_result, o);
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

int tkv_amq_gen_keys16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* d_keys, void* stream)
{
  if (tkv_amq_device_count() == 0) return TKV_AMQ_UNAVAILABLE;
  if (n == 0) return TKV_AMQ_OK;
  if (!d_keys || (reinterpret_cast<uintptr_t>(d_keys) & 15)) return TKV_AMQ_INVALID_ARGUMENT;
  const uint32_t g = (uint32_t)(div_up(n, 256) < 16384 ? div_up(n, 256) : 16384);
  hipLaunchKernelGGL(gen_keys16_kernel, dim3(g), dim3(256), 0, as_stream(stream), seed, first, n,
                     reinterpret_cast<ulonglong2*>(d_keys));
  return hipGetLastError() == hipSuccess ? TKV_AMQ_OK : TKV_AMQ_INTERNAL;
}

}  // extern "C"

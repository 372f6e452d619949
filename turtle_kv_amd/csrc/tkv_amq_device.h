// tkv_amq_device.h -- gfx950 device helpers for the tkv-amq v1 filter kernels.
//
// XXH64 (xxHash spec; the reference hashes every key with it: vqf_hash_val,
// src/turtle_kv/vqf_filter_page_view.hpp:32-35, and llfs's Bloom hashes).  Three forms:
//   xxh64_bytes        any length / alignment (variable-length keys)
//   Xxh16              16-byte keys, split so that k seeds share the seed-independent work:
//                      for len < 32 the two 8-byte lane rounds do not depend on the seed,
//                      so a k-hash Bloom key costs 4 + 4k 64-bit multiplies instead of 8k.
// All arithmetic is u64 wrap-around, bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tkv {

constexpr uint64_t kP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t kP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t kP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t kP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t kP5 = 0x27D4EB2F165667C5ULL;

constexpr uint64_t kVqfHashSeed = 0x9d0924dc03e79a75ULL;  // vqf_filter_page_view.hpp:26
constexpr uint64_t kVqfMagic = 0x16015305e0f43a7dULL;     // vqf_filter_page_view.hpp:66
constexpr uint64_t kBloomMagic = 0xca6f49a0f3f8a4b0ULL;   // tkv-amq v1 PackedBloomFilterPage
constexpr uint64_t kVqfAltMul = 0x5bd1e995ULL;
constexpr uint32_t kBloomHeader = 64;
constexpr uint32_t kVqfHeader = 32;   // sizeof(PackedVqfFilter) - sizeof(vqf_metadata)
constexpr uint32_t kVqfMetadata = 48; // sizeof(vqf_metadata)
constexpr uint32_t kMaxBloomHashes = 32;
// page framing (TreeOptions sizing, tree/tree_options.hpp:177-258; filter page image):
constexpr uint64_t kPackedPageHeaderBytes = 64;  // sizeof(llfs::PackedPageHeader), pinned by
                                                 // tree/packed_node_page.hpp:472
constexpr uint64_t kPackedLeafPageBytes = 32;    // sizeof(PackedLeafPage), packed_leaf_page.hpp:303
constexpr uint64_t kPackedArrayBytes = 8;        // sizeof(llfs::PackedArray<T>): UNPINNED (llfs
                                                 // absent; u32 item_count + 4 reserved bytes)

__host__ __device__ constexpr inline uint64_t rotl64(uint64_t x, int r)
{
  return (x << r) | (x >> (64 - r));
}

__host__ __device__ inline uint64_t xxh_round(uint64_t acc, uint64_t in)
{
  acc += in * kP2;
  acc = rotl64(acc, 31);
  return acc * kP1;
}

__host__ __device__ inline uint64_t xxh_merge(uint64_t acc, uint64_t v)
{
  acc ^= xxh_round(0, v);
  return acc * kP1 + kP4;
}

__host__ __device__ inline uint64_t xxh_avalanche(uint64_t h)
{
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}

__host__ __device__ constexpr inline uint64_t sm64_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__host__ __device__ constexpr inline uint64_t splitmix64_at(uint64_t seed, uint64_t n)
{
  return sm64_mix(seed + n * 0x9E3779B97F4A7C15ULL);
}

// tkv-amq v1 Bloom seed table entry i
__host__ __device__ constexpr inline uint64_t bloom_seed(uint32_t i)
{
  return sm64_mix(0x243F6A8885A308D3ULL + (uint64_t)i * 0x9E3779B97F4A7C15ULL);
}

// ---- 64-bit ops spelled as 32-bit halves (gfx950 has no 64-bit rotate; the compiler
// otherwise emits v_lshlrev_b64 + v_lshrrev_b64 + 2 v_or per rotate) ----
__device__ inline uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ inline uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ inline uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

template <int R>
__device__ inline uint64_t drotl(uint64_t x)
{
  static_assert(R > 0 && R < 32, "rotate amount");
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(__builtin_amdgcn_alignbit(l, h, 32 - R), __builtin_amdgcn_alignbit(h, l, 32 - R));
}

template <int S>
__device__ inline uint64_t dshr(uint64_t x)
{
  if constexpr (S >= 32) {
    return (uint64_t)(hi32(x) >> (S - 32));
  } else {
    return mk64(__builtin_amdgcn_alignbit(hi32(x), lo32(x), S), hi32(x) >> S);
  }
}

__device__ inline uint64_t dround(uint64_t acc, uint64_t in)
{
  acc += in * kP2;
  acc = drotl<31>(acc);
  return acc * kP1;
}

__device__ inline uint64_t davalanche(uint64_t h)
{
  h ^= dshr<33>(h);
  h *= kP2;
  h ^= dshr<29>(h);
  h *= kP3;
  h ^= dshr<32>(h);
  return h;
}

// v_mul_u32_u24 (full rate).  Inline asm because LLVM's demanded-bits folding turns a
// masked 24-bit multiply whose result is later masked to 9 bits back into v_mul_lo_u32
// (quarter rate).
__device__ inline uint32_t mul_u24(uint32_t konst, uint32_t x)
{
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(konst), "v"(x));
  return r;
}

__device__ inline uint32_t mad_u24(uint32_t konst, uint32_t x, uint32_t addend)
{
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "s"(konst), "v"(x), "v"(addend));
  return r;
}

// davalanche(h) with the last multiply narrowed; only bits 0..8 of the result are valid
// (callers take `& 511` or a bitfield of them).  Bits 0..8 and 32..40 of y * P3 only need
// hi32(y_lo * P3_lo) and the low 9 bits of the two cross products, which 24-bit
// multiply-adds (full rate) give exactly.
__device__ inline uint32_t davalanche_lo9(uint64_t h)
{
  h ^= dshr<33>(h);
  h *= kP2;
  h ^= dshr<29>(h);
  const uint32_t yl = lo32(h), yh = hi32(h);
  constexpr uint32_t cl = (uint32_t)kP3, ch = (uint32_t)(kP3 >> 32);
  const uint64_t p = (uint64_t)yl * cl;  // both words in one v_mad_u64_u32
  const uint32_t h3_hi = mad_u24(cl, yh, mad_u24(ch, yl, hi32(p)));
  return lo32(p) ^ h3_hi;
}

// 16-byte key, seed-independent part precomputed once per key.  Rotation distributes over
// XOR, so rotl(hinit ^ k1, 27) = rotl(hinit, 27) ^ rotl(k1, 27): the per-seed part is the
// constant `rhinit` = rotl(seed + P5 + 16, 27) and rotl(k1, 27) is computed once per key.
struct Xxh16 {
  uint64_t rk1, k2;
  __device__ inline Xxh16(uint64_t lo, uint64_t hi) : rk1{drotl<27>(dround(0, lo))}, k2{dround(0, hi)} {}
  __device__ inline Xxh16() : rk1{0}, k2{0} {}  // (a state moved between lanes: set rk1, k2)
  // state before the avalanche
  __device__ inline uint64_t pre(uint64_t rhinit) const
  {
    uint64_t h = (rhinit ^ rk1) * kP1 + kP4;
    h ^= k2;
    return drotl<27>(h) * kP1 + kP4;
  }
  __device__ inline uint64_t finish(uint64_t rhinit) const { return davalanche(pre(rhinit)); }
  // bits 0..8 only are valid (Bloom bit index inside a 512-bit block)
  __device__ inline uint32_t finish_lo9(uint64_t rhinit) const { return davalanche_lo9(pre(rhinit)); }
};

// Fixed key length L (multiple of 8, 8 <= L < 32): the same split for any short key.  All L/8
// lane rounds are seed-independent; the per-seed constant is rotl(seed + P5 + L, 27).
// (TurtleKV's default key size hint is 24 bytes, tree/tree_options.hpp:58.)
template <int L>
struct XxhFixed {
  static_assert(L % 8 == 0 && L >= 8 && L < 32, "short fixed-length keys only");
  static constexpr int N = L / 8;
  uint64_t rk0;
  uint64_t k[N > 1 ? N - 1 : 1];
  __device__ inline XxhFixed() : rk0{0}, k{} {}  // (a state moved between lanes)
  __device__ inline explicit XxhFixed(const uint64_t (&lanes)[N])
  {
    rk0 = drotl<27>(dround(0, lanes[0]));
#pragma unroll
    for (int i = 1; i < N; ++i) k[i - 1] = dround(0, lanes[i]);
  }
  __device__ inline uint64_t pre(uint64_t rc) const
  {
    uint64_t h = (rc ^ rk0) * kP1 + kP4;
#pragma unroll
    for (int i = 1; i < N; ++i) {
      h ^= k[i - 1];
      h = drotl<27>(h) * kP1 + kP4;
    }
    return h;
  }
  __device__ inline uint64_t finish(uint64_t rc) const { return davalanche(pre(rc)); }
  __device__ inline uint32_t finish_lo9(uint64_t rc) const { return davalanche_lo9(pre(rc)); }
};

template <int L>
__host__ __device__ constexpr inline uint64_t xxh_fixed_rc(uint64_t seed)
{
  return rotl64(seed + kP5 + L, 27);
}

// rotl(seed + P5 + 16, 27): the per-seed constant Xxh16 takes
__host__ __device__ constexpr inline uint64_t xxh16_rhinit(uint64_t seed)
{
  return rotl64(seed + kP5 + 16, 27);
}

// Unaligned global loads: gfx950 (HSA, unaligned access mode) serves a dwordx2 / dword load
// at any byte address; memcpy from a byte pointer compiles to exactly that
// (tools/probe/unaligned_load.hip checks every byte offset on the device).
__device__ inline uint64_t ld64_unaligned(const uint8_t* p)
{
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

__device__ inline uint32_t ld32_unaligned(const uint8_t* p)
{
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// Any key shorter than 32 bytes (XXH64's short-input path), any alignment: the 8-byte lane
// rounds and the 4-byte / 1-byte tail products do not depend on the seed, so they are
// computed once per key; per seed only the chained rotate-multiply steps and the avalanche
// remain.  Lanes of one wave may have different lengths: the steps a key does not have are
// predicated off.
struct XxhShort {
  uint32_t len;
  uint64_t r[3];   // round(0, lane j), j < len / 8
  uint64_t t4;     // (4-byte tail) * P1, if len & 4
  uint64_t tb[3];  // byte k of the 1..3-byte tail * P5
  __device__ inline XxhShort(const uint8_t* p, uint32_t n) : len{n}
  {
    const uint32_t n8 = n >> 3;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) r[j] = j < n8 ? dround(0, ld64_unaligned(p + 8 * j)) : 0ull;
    const uint8_t* q = p + 8 * n8;
    t4 = (n & 4) ? (uint64_t)ld32_unaligned(q) * kP1 : 0ull;
    q += (n & 4);
    const uint32_t nb = n & 3;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) tb[k] = k < nb ? (uint64_t)q[k] * kP5 : 0ull;
  }
  // from bytes loaded ahead (VqfKeyBuf<kKeyVar>): the n >> 3 eight-byte lanes, the 4-byte
  // tail word and the 1..3 tail bytes packed low to high
  __device__ inline XxhShort(uint32_t n, const uint64_t (&lanes)[3], uint32_t tail4, uint32_t tail_bytes)
      : len{n}
  {
    const uint32_t n8 = n >> 3;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) r[j] = j < n8 ? dround(0, lanes[j]) : 0ull;
    t4 = (n & 4) ? (uint64_t)tail4 * kP1 : 0ull;
    const uint32_t nb = n & 3;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) tb[k] = k < nb ? (uint64_t)((tail_bytes >> (8 * k)) & 0xffu) * kP5 : 0ull;
  }
  // state before the avalanche; seed_p5 = seed + P5
  __device__ inline uint64_t pre(uint64_t seed_p5) const
  {
    uint64_t h = seed_p5 + len;
    const uint32_t n8 = len >> 3, nb = len & 3;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
      if (j < n8) {
        h ^= r[j];
        h = drotl<27>(h) * kP1 + kP4;
      }
    }
    if (len & 4) {
      h ^= t4;
      h = drotl<23>(h) * kP2 + kP3;
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      if (k < nb) {
        h ^= tb[k];
        h = drotl<11>(h) * kP1;
      }
    }
    return h;
  }
  __device__ inline uint64_t finish(uint64_t seed_p5) const { return davalanche(pre(seed_p5)); }
  __device__ inline uint32_t finish_lo9(uint64_t seed_p5) const { return davalanche_lo9(pre(seed_p5)); }
};

// XXH64 of an arbitrary byte string in device memory.
__device__ inline uint64_t xxh64_bytes(const uint8_t* p, uint64_t len, uint64_t seed)
{
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = dround(v1, ld64_unaligned(p));
      v2 = dround(v2, ld64_unaligned(p + 8));
      v3 = dround(v3, ld64_unaligned(p + 16));
      v4 = dround(v4, ld64_unaligned(p + 24));
      p += 32;
    } while (p <= limit);
    h = drotl<1>(v1) + drotl<7>(v2) + drotl<12>(v3) + drotl<18>(v4);
    h = (h ^ dround(0, v1)) * kP1 + kP4;
    h = (h ^ dround(0, v2)) * kP1 + kP4;
    h = (h ^ dround(0, v3)) * kP1 + kP4;
    h = (h ^ dround(0, v4)) * kP1 + kP4;
  } else {
    h = seed + kP5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= dround(0, ld64_unaligned(p));
    h = drotl<27>(h) * kP1 + kP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)ld32_unaligned(p) * kP1;
    h = drotl<23>(h) * kP2 + kP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * kP5;
    h = drotl<11>(h) * kP1;
    ++p;
  }
  return davalanche(h);
}

// x mod d for x < 2^64, d < 2^31, given m = floor((2^64 - 1) / d): q = umulhi(x, m) is at
// most 2 below floor(x / d), so x - q*d < 3d < 2^32 and the whole fix-up runs in 32 bits
// (min(r, r - d) subtracts d exactly when r >= d: otherwise r - d wraps above r).
__device__ inline uint32_t mod_by_magic(uint64_t x, uint32_t d, uint64_t m)
{
  const uint64_t q = __umul64hi(x, m);
  uint32_t r = (uint32_t)x - (uint32_t)q * d;
  r = min(r, r - d);
  r = min(r, r - d);
  return r;
}

// 64-lane wave helpers
__device__ inline uint64_t lanemask_lt()
{
  const uint32_t lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// 64-lane ballot of a bool (HIP's __ballot takes an int, and the int round trip can leave a
// compare mask materialised as 0/1 in a VGPR and compared again)
__device__ inline uint64_t bal(bool b)
{
  return __builtin_amdgcn_ballot_w64(b);
}

// per lane: bit `lane` of the wave-uniform mask m ? a : b, as one v_cndmask on the mask's SGPRs
__device__ inline uint32_t sel_mask(uint64_t m, uint32_t a, uint32_t b)
{
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}

// position of the r-th (0-based) set bit of x; x must have > r set bits
__device__ inline int select64(uint64_t x, int r)
{
  int pos = 0;
  int c = __popcll(x & 0xffffffffull);
  if (r >= c) { r -= c; x >>= 32; pos += 32; }
  c = __popc((uint32_t)(x & 0xffffu));
  if (r >= c) { r -= c; x >>= 16; pos += 16; }
  c = __popc((uint32_t)(x & 0xffu));
  if (r >= c) { r -= c; x >>= 8; pos += 8; }
  c = __popc((uint32_t)(x & 0xfu));
  if (r >= c) { r -= c; x >>= 4; pos += 4; }
  c = __popc((uint32_t)(x & 0x3u));
  if (r >= c) { r -= c; x >>= 2; pos += 2; }
  c = (int)(x & 1u);
  if (r >= c) { pos += 1; }
  return pos;
}

__device__ inline int select128(uint64_t lo, uint64_t hi, int r)
{
  const int c0 = __popcll(lo);
  return r < c0 ? select64(lo, r) : 64 + select64(hi, r - c0);
}

}  // namespace tkv

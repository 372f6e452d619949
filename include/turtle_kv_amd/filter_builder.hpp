// turtle_kv_amd/filter_builder.hpp -- C++ host mirror of TurtleKV's filter API over the
// tkv_amq C ABI (libtkv_amq.so, HIP/gfx950).  Header-only, C++17.
//
// Reference interface (mathworks/turtle_kv, src/turtle_kv/...) -> this header:
//   vqf_hash_val                          vqf_filter_page_view.hpp:32-35   (device: vqf_hash_val_batch)
//   vqf_filter_load_factor<TAG_BITS>      vqf_filter_page_view.hpp:39-59   vqf_filter_load_factor<T>
//   PackedVqfFilter                       vqf_filter_page_view.hpp:63-131  PackedVqfFilter (layout)
//   TreeOptions::filter_bits_per_key      tree/tree_options.hpp:155-164    filter_bits_per_key
//   build_bloom_filter_for_leaf           tree/filter_builder.hpp:109-152  build_bloom_filter_for_leaf
//   build_quotient_filter_for_leaf        tree/filter_builder.hpp:221-301  build_quotient_filter_for_leaf
//   build_filter_for_leaf_in_job          tree/filter_builder.hpp:307-331  build_filter_for_leaf_in_job
//   TreeSerializeContext::build_all_pages tree/tree_serialize_context.cpp:62-115 (filter half)
//                                                                          FilterBatchBuilder
//   KeyQuery::reject_page                 tree/key_query.hpp:149-247       KeyQuery::reject_page
//   KeyQuery::Metrics                     tree/key_query.hpp:36-60         KeyQuery::Metrics
//   TreeOptions (filter sizing)           tree/tree_options.hpp:149-258    TreeOptions
//   FilterPageAlloc page image            tree/filter_builder.hpp:58-105,231-237,293-296
//                                                                          FilterBatchBuilder::plan_pages
//
// The single-leaf functions take the leaf's keys as host string views (the reference's
// `items` range of EditView keys, tombstones included) and fill a host page payload
// buffer, staging through the device.  The batched FilterBatchBuilder works on
// device-resident keys and is the fast path.  There is no CPU implementation here: every
// filter byte is computed by the HIP kernels.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <optional>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "../tkv_amq.h"

namespace turtle_kv_amd {

using u8 = std::uint8_t;
using u16 = std::uint16_t;
using u32 = std::uint32_t;
using u64 = std::uint64_t;
using usize = std::size_t;

// ---------------------------------------------------------------------------------------
// Status (batt::Status numbering)
// ---------------------------------------------------------------------------------------
struct Status {
  int code = TKV_AMQ_OK;
  std::string what;
  bool ok() const { return code == TKV_AMQ_OK; }
  static Status from(int c, const char* w) { return Status{c, c == TKV_AMQ_OK ? "" : w}; }
  std::string to_string() const
  {
    return std::string(tkv_amq_status_string(code)) + (what.empty() ? "" : ": " + what);
  }
};
inline Status OkStatus() { return Status{}; }

#define TKV_AMQ_REQUIRE_OK(expr)          \
  do {                                    \
    ::turtle_kv_amd::Status s_ = (expr);  \
    if (!s_.ok()) return s_;              \
  } while (0)

// ---------------------------------------------------------------------------------------
// constants and sizing (config.hpp:20-24, vqf_filter_page_view.hpp:26-28)
// ---------------------------------------------------------------------------------------
enum class FilterKind : int { kBloom = TKV_AMQ_BLOOM, kQuotient = TKV_AMQ_VQF };
inline constexpr FilterKind kDefaultFilterKind = FilterKind::kQuotient;  // TURTLE_KV_USE_QUOTIENT_FILTER 1
inline constexpr u64 kVqfHashSeed = 0x9d0924dc03e79a75ull;
inline constexpr usize kMinQuotientFilterBitsPerKey = 12;
inline constexpr double kMaxQuotientFilterLoadFactor = 0.85;
inline constexpr u16 kDefaultFilterBitsPerKey = 12;
inline constexpr usize kPackedPageHeaderSize = 64;

template <int TAG_BITS>
inline double vqf_filter_load_factor(usize bits_per_key)
{
  static_assert(TAG_BITS == 8 || TAG_BITS == 16, "TAG_BITS must be 8 or 16");
  return tkv_amq_vqf_load_factor(TAG_BITS, bits_per_key);
}

inline usize filter_bits_per_key(std::optional<u16> requested,
                                 FilterKind kind = kDefaultFilterKind)
{
  return (usize)tkv_amq_filter_bits_per_key((int)kind, requested.value_or(kDefaultFilterBitsPerKey));
}

// The filter part of TreeOptions (tree/tree_options.hpp:43-395): bits per key with the VQF
// clamp, and the filter page size from the leaf size and key/value size hints.  `kind` stands
// for the compile-time filter switch (config.hpp:20-24).
class TreeOptions
{
 public:
  static constexpr u32 kDefaultKeySizeHint = 24;     // :58
  static constexpr u32 kDefaultValueSizeHint = 100;  // :59

  explicit TreeOptions(FilterKind kind = kDefaultFilterKind) : kind_{kind} {}
  static TreeOptions with_default_values(FilterKind kind = kDefaultFilterKind) { return TreeOptions{kind}; }

  u64 leaf_size() const { return u64{1} << leaf_size_log2_; }
  TreeOptions& set_leaf_size_log2(u8 size_log2) { leaf_size_log2_ = size_log2; return *this; }
  usize leaf_data_size() const { return (usize)tkv_amq_leaf_data_size(leaf_size()); }

  TreeOptions& set_filter_bits_per_key(std::optional<u16> bpk) { filter_bits_per_key_ = bpk; return *this; }
  usize filter_bits_per_key() const { return turtle_kv_amd::filter_bits_per_key(filter_bits_per_key_, kind_); }

  TreeOptions& set_key_size_hint(u32 n) { key_size_hint_ = n; return *this; }
  TreeOptions& set_value_size_hint(u32 n) { value_size_hint_ = n; return *this; }
  u32 key_size_hint() const { return key_size_hint_; }
  u32 value_size_hint() const { return value_size_hint_; }
  usize expected_items_per_leaf() const
  {
    return (usize)tkv_amq_expected_items_per_leaf(leaf_size(), key_size_hint_, value_size_hint_);
  }

  TreeOptions& set_filter_page_size_log2(u8 size_log2) { filter_page_size_log2_ = size_log2; return *this; }
  u32 filter_page_size_log2() const
  {
    if (filter_page_size_log2_) return *filter_page_size_log2_;
    return tkv_amq_filter_page_size_log2((int)kind_, leaf_size(), key_size_hint_, value_size_hint_,
                                         filter_bits_per_key_.value_or(kDefaultFilterBitsPerKey));
  }
  u64 filter_page_size() const { return u64{1} << filter_page_size_log2(); }
  // the payload the filter builders size against: the page minus the llfs PackedPageHeader
  u64 filter_page_payload_size() const { return filter_page_size() - kPackedPageHeaderSize; }

 private:
  FilterKind kind_;
  u8 leaf_size_log2_ = 21;  // 2 MiB (tree_options.cpp:20-21)
  std::optional<u16> filter_bits_per_key_;
  std::optional<u8> filter_page_size_log2_;
  u32 key_size_hint_ = kDefaultKeySizeHint;
  u32 value_size_hint_ = kDefaultValueSizeHint;
};

// payload capacity of the default TreeOptions' filter page at this bits/key
inline u64 default_filter_page_payload_size(usize bits_per_key, FilterKind kind)
{
  return TreeOptions{kind}.set_filter_bits_per_key((u16)bits_per_key).filter_page_payload_size();
}

// vqf_metadata + PackedVqfFilter on-page layout (little-endian)
struct VqfMetadata {
  u64 total_size_in_bytes;
  u64 key_remainder_bits;
  u64 range;
  u64 nblocks;
  u64 nelts;
  u64 nslots;
};
struct PackedVqfFilter {
  static constexpr u64 kMagic = 0x16015305e0f43a7dull;
  u64 magic;
  u64 src_page_id;
  u64 hash_seed;
  u64 hash_mask;
  VqfMetadata metadata;
};
static_assert(sizeof(PackedVqfFilter) == 32 + sizeof(VqfMetadata), "vqf_filter_page_view.hpp:128");

struct PackedBloomFilterPage {
  static constexpr u64 kMagic = 0xca6f49a0f3f8a4b0ull;
  u64 magic;
  u64 bit_count;
  u64 src_page_id;
  u64 xxh3_checksum;
  u64 word_count;
  u32 block_count;
  u16 hash_count;
  u8 layout;  // 2 = kBlocked512
  u8 reserved0;
  u64 item_count;
  u64 reserved1;
};
static_assert(sizeof(PackedBloomFilterPage) == 64, "tkv-amq v1 Bloom header");

// ---------------------------------------------------------------------------------------
// device buffer helper (RAII)
// ---------------------------------------------------------------------------------------
class DeviceBuffer
{
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(usize n) { resize(n); }
  ~DeviceBuffer() { reset(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : p_{o.p_}, n_{o.n_} { o.p_ = nullptr; o.n_ = 0; }

  bool resize(usize n)
  {
    if (n <= n_) return true;
    reset();
    if (hipMalloc(&p_, n ? n : 1) != hipSuccess) { p_ = nullptr; return false; }
    n_ = n;
    return true;
  }
  void reset()
  {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  template <typename T = u8>
  T* get() const { return static_cast<T*>(p_); }
  usize size() const { return n_; }

 private:
  void* p_ = nullptr;
  usize n_ = 0;
};

// ---------------------------------------------------------------------------------------
// FilterBatchBuilder: every leaf filter of one build_all_pages queue in one device call
// ---------------------------------------------------------------------------------------
class FilterBatchBuilder
{
 public:
  FilterBatchBuilder(FilterKind kind, usize bits_per_key, u64 page_payload_bytes,
                     u64 out_stride = 0)
      : kind_{kind}, bpk_{bits_per_key}, cap_{page_payload_bytes}, stride_{out_stride}
  {
  }

  // Whole filter pages of 2^page_size_log2 bytes, leaf s at s << log2: the PackedPageHeader
  // fields the builders set, then the payload (tkv_amq_plan_pages).
  static FilterBatchBuilder pages(FilterKind kind, usize bits_per_key, u32 page_size_log2)
  {
    FilterBatchBuilder b{kind, bits_per_key, (u64{1} << page_size_log2) - kPackedPageHeaderSize,
                         u64{1} << page_size_log2};
    b.page_log2_ = page_size_log2;
    return b;
  }

  // Queue one leaf whose keys occupy the next n_keys slots of the device key array.
  u32 add_leaf(u64 leaf_page_id, u64 n_keys)
  {
    counts_.push_back(n_keys);
    page_ids_.push_back(leaf_page_id);
    return (u32)(counts_.size() - 1);
  }

  Status plan()
  {
    segs_.resize(counts_.size());
    const int st =
        page_log2_ ? tkv_amq_plan_pages((int)kind_, counts_.data(), page_ids_.data(), (u32)counts_.size(),
                                        (u32)bpk_, page_log2_, segs_.data(), &total_out_, &ws_bytes_,
                                        &max_blocks_)
                   : tkv_amq_plan((int)kind_, counts_.data(), page_ids_.data(), (u32)counts_.size(),
                                  (u32)bpk_, cap_, stride_, segs_.data(), &total_out_, &ws_bytes_,
                                  &max_blocks_);
    if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_plan");
    if (!d_segs_.resize(segs_.size() * sizeof(tkv_amq_segment)) || !d_ws_.resize(ws_bytes_))
      return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipMalloc");
    if (hipMemcpy(d_segs_.get(), segs_.data(), segs_.size() * sizeof(tkv_amq_segment),
                  hipMemcpyHostToDevice) != hipSuccess)
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpy plan");
    planned_ = true;
    return OkStatus();
  }

  // Device keys: fixed length (d_key_offsets == nullptr, key_stride bytes each) or
  // variable length (d_key_offsets[n+1]).  Asynchronous on `stream`; call check().
  Status build_all(const u8* d_keys, u32 key_stride, const u64* d_key_offsets, u8* d_out,
                   hipStream_t stream = nullptr)
  {
    if (!planned_) TKV_AMQ_REQUIRE_OK(plan());
    u64 n = 0;
    for (u64 c : counts_) n += c;
    // (_ex with the host plan: in a Bloom batch, leaves of 16- or 24-byte keys past 5 LDS
    // windows -- other key shapes past 16 -- take the tiled build, up to 40 per launch)
    return Status::from(tkv_amq_build_ex((int)kind_, d_keys, d_key_offsets, key_stride, n,
                                         d_segs_.get<tkv_amq_segment>(), segs_.data(), (u32)segs_.size(),
                                         max_blocks_, d_out, d_ws_.get(), ws_bytes_, stream),
                        "tkv_amq_build_ex");
  }

  Status check(hipStream_t stream = nullptr) const
  {
    return Status::from(tkv_amq_build_check((int)kind_, d_ws_.get(), ws_bytes_, stream),
                        "vqf_insert (filter_builder.hpp:211)");
  }

  Status probe(const u8* d_filters, const u8* d_queries, u32 query_stride,
               const u64* d_query_offsets, u64 n_queries, const u32* d_query_leaf, u8* d_result,
               hipStream_t stream = nullptr) const
  {
    return Status::from(tkv_amq_probe((int)kind_, d_filters, d_segs_.get<tkv_amq_segment>(),
                                      (u32)segs_.size(), d_queries, d_query_offsets, query_stride,
                                      n_queries, d_query_leaf, d_result, stream),
                        "tkv_amq_probe");
  }

  const std::vector<tkv_amq_segment>& segments() const { return segs_; }
  u64 total_out_bytes() const { return total_out_; }
  const tkv_amq_segment* device_segments() const { return d_segs_.get<tkv_amq_segment>(); }

 private:
  FilterKind kind_;
  usize bpk_;
  u64 cap_, stride_;
  std::vector<u64> counts_, page_ids_;
  std::vector<tkv_amq_segment> segs_;
  u64 total_out_ = 0, ws_bytes_ = 0;
  u32 max_blocks_ = 0;
  u32 page_log2_ = 0;
  bool planned_ = false;
  DeviceBuffer d_segs_, d_ws_;
};

// ---------------------------------------------------------------------------------------
// single-leaf entry points (host keys -> host page payload)
// ---------------------------------------------------------------------------------------
namespace detail {

// std::string_view is read in place as tkv_amq_key_view when the layouts agree (libstdc++:
// {size, data}); otherwise the views are copied into tkv_amq_key_view records first.
inline bool string_view_is_key_view()
{
  static_assert(sizeof(std::string_view) == sizeof(tkv_amq_key_view), "string_view size");
  const char probe[2] = {'a', 0};
  const std::string_view sv(probe, 1);
  tkv_amq_key_view kv;
  std::memcpy(&kv, &sv, sizeof(kv));
  return kv.size == 1 && kv.data == reinterpret_cast<const u8*>(probe);
}

inline Status stage_keys(const std::vector<std::string_view>& items, DeviceBuffer& d_keys,
                         DeviceBuffer& d_offs, bool& fixed, u32& stride)
{
  const usize n = items.size();
  fixed = n > 0;
  stride = n ? (u32)items[0].size() : 16;
  u64 total = 0;
  for (usize i = 0; i < n; ++i) {
    total += items[i].size();
    fixed = fixed && items[i].size() == stride;
  }
  if (fixed && stride == 0) fixed = false;
  std::vector<tkv_amq_key_view> copied;
  const void* views = items.data();
  if (!string_view_is_key_view()) {
    copied.resize(n);
    for (usize i = 0; i < n; ++i)
      copied[i] = tkv_amq_key_view{items[i].size(), reinterpret_cast<const u8*>(items[i].data())};
    views = copied.data();
  }
  // tkv_amq_stage_keys: the host gather (the EditView key range -> one contiguous buffer)
  std::vector<u64> offs(n + 1, 0);
  std::vector<u8> blob(total ? total : 1);
  const int st = tkv_amq_stage_keys(views, sizeof(tkv_amq_key_view), n, fixed ? stride : 0,
                                    blob.data(), blob.size(), fixed ? nullptr : offs.data(), 0);
  if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_stage_keys");
  if (!d_keys.resize(blob.size()) || !d_offs.resize(offs.size() * 8))
    return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipMalloc");
  if (hipMemcpy(d_keys.get(), blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d_offs.get(), offs.data(), offs.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return Status::from(TKV_AMQ_INTERNAL, "hipMemcpy keys");
  return OkStatus();
}

// Per-thread scratch for the single-leaf entry points, which the reference calls once per
// leaf from its worker threads (tree/tree_serialize_context.cpp:71-75): a stream of the
// thread's own and grow-only device / pinned host buffers, so a call makes no hipMalloc /
// hipFree (hipFree synchronises the whole device, which would serialise the workers) and
// only waits for its own stream.
struct LeafScratch {
  hipStream_t stream = nullptr;
  DeviceBuffer d_keys, d_offs, d_segs, d_ws, d_out;
  u8* h_keys = nullptr;
  usize h_keys_cap = 0;
  u64* h_offs = nullptr;
  usize h_offs_cap = 0;
  u8* h_io = nullptr;  // pinned: [segment 64 B][status 4 B .. 64 B][payload]
  usize h_io_cap = 0;
  std::vector<tkv_amq_key_view> views;

  ~LeafScratch()
  {
    if (h_keys) (void)hipHostFree(h_keys);
    if (h_offs) (void)hipHostFree(h_offs);
    if (h_io) (void)hipHostFree(h_io);
    if (stream) (void)hipStreamDestroy(stream);
  }
  bool ensure_stream() { return stream || hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess; }
  template <typename T>
  static bool grow_pinned(T*& p, usize& cap, usize n)
  {
    if (n <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&p), n * sizeof(T)) != hipSuccess) return false;
    cap = n;
    return true;
  }
};

inline LeafScratch& leaf_scratch()
{
  thread_local LeafScratch s;
  return s;
}

inline Status build_one(FilterKind kind, usize bpk, u64 leaf_page_id,
                        const std::vector<std::string_view>& items,
                        std::vector<u8>& page_payload, u64 page_payload_bytes)
{
  if (bpk == 0) return OkStatus();  // filter_builder.hpp:115-117, :227-229
  if (tkv_amq_device_count() == 0) return Status::from(TKV_AMQ_UNAVAILABLE, "no HIP device");
  LeafScratch& sc = leaf_scratch();
  if (!sc.ensure_stream()) return Status::from(TKV_AMQ_INTERNAL, "hipStreamCreate");
  const u64 n = items.size();
  tkv_amq_segment seg{};
  u64 total_out = 0, ws_bytes = 0;
  u32 max_blocks = 0;
  int st = tkv_amq_plan((int)kind, &n, &leaf_page_id, 1, (u32)bpk, page_payload_bytes, 0, &seg,
                        &total_out, &ws_bytes, &max_blocks);
  if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_plan");

  // stage the keys (the EditView key range) into pinned memory: one fixed stride if every key
  // has the same length, else bytes + offsets
  u64 bytes = 0;
  bool fixed = n > 0;
  const u32 stride = n ? (u32)items[0].size() : 16;
  for (const auto& k : items) {
    bytes += k.size();
    fixed = fixed && k.size() == stride;
  }
  fixed = fixed && stride != 0;
  const void* views = items.data();
  if (!string_view_is_key_view()) {
    sc.views.resize(n);
    for (u64 i = 0; i < n; ++i)
      sc.views[i] = tkv_amq_key_view{items[i].size(), reinterpret_cast<const u8*>(items[i].data())};
    views = sc.views.data();
  }
  if (!LeafScratch::grow_pinned(sc.h_keys, sc.h_keys_cap, bytes ? bytes : 1) ||
      !LeafScratch::grow_pinned(sc.h_offs, sc.h_offs_cap, n + 1))
    return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipHostMalloc");
  st = tkv_amq_stage_keys(views, sizeof(tkv_amq_key_view), n, fixed ? stride : 0, sc.h_keys,
                          sc.h_keys_cap, fixed ? nullptr : sc.h_offs, 1);
  if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_stage_keys");
  if (!sc.d_keys.resize(bytes ? bytes : 1) || !sc.d_offs.resize(8 * (n + 1)) ||
      !sc.d_segs.resize(sizeof(seg)) || !sc.d_ws.resize(ws_bytes) || !sc.d_out.resize(total_out) ||
      !LeafScratch::grow_pinned(sc.h_io, sc.h_io_cap, 128 + (usize)seg.payload_bytes))
    return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipMalloc");
  // everything below is asynchronous on the thread's stream, from and to pinned memory, with
  // one synchronisation at the end (the VQF failure word comes back with the payload)
  std::memcpy(sc.h_io, &seg, sizeof(seg));
  u32* h_status = reinterpret_cast<u32*>(sc.h_io + 64);
  *h_status = 0;
  u8* h_payload = sc.h_io + 128;
  hipStream_t s = sc.stream;
  const u32 used = seg.payload_bytes;
  if (hipMemcpyAsync(sc.d_keys.get(), sc.h_keys, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      (!fixed && hipMemcpyAsync(sc.d_offs.get(), sc.h_offs, 8 * (n + 1), hipMemcpyHostToDevice, s) != hipSuccess) ||
      hipMemcpyAsync(sc.d_segs.get(), sc.h_io, sizeof(seg), hipMemcpyHostToDevice, s) != hipSuccess)
    return Status::from(TKV_AMQ_INTERNAL, "hipMemcpyAsync keys");
  st = tkv_amq_build((int)kind, sc.d_keys.get(), fixed ? nullptr : sc.d_offs.get<u64>(),
                     fixed ? stride : 0, n, sc.d_segs.get<tkv_amq_segment>(), 1, max_blocks,
                     sc.d_out.get(), sc.d_ws.get(), ws_bytes, s);
  if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_build");
  if (hipMemcpyAsync(h_payload, sc.d_out.get(), used, hipMemcpyDeviceToHost, s) != hipSuccess)
    return Status::from(TKV_AMQ_INTERNAL, "hipMemcpyAsync payload");
  // (the leaf's nelts word: its failure flags, tkv_amq.h)
  if ((kind == FilterKind::kQuotient && ws_bytes >= TKV_AMQ_VQF_NELTS_OFFSET + 4 &&
       hipMemcpyAsync(h_status, sc.d_ws.get<u8>() + TKV_AMQ_VQF_NELTS_OFFSET, 4, hipMemcpyDeviceToHost,
                      s) != hipSuccess) ||
      hipStreamSynchronize(s) != hipSuccess)
    return Status::from(TKV_AMQ_INTERNAL, "hipStreamSynchronize");
  if (*h_status & TKV_AMQ_VQF_FLAG_WORKSPACE) return Status::from(TKV_AMQ_INVALID_ARGUMENT, "workspace");
  if (*h_status & TKV_AMQ_VQF_FLAG_OVERFLOW)
    return Status::from(TKV_AMQ_INTERNAL, "vqf_insert (filter_builder.hpp:211)");
  page_payload.assign(page_payload_bytes ? page_payload_bytes : used, 0);
  std::memcpy(page_payload.data(), h_payload, used);
  return OkStatus();
}

}  // namespace detail

inline Status build_bloom_filter_for_leaf(usize filter_bits_per_key, u64 leaf_page_id,
                                          const std::vector<std::string_view>& items,
                                          std::vector<u8>& page_payload,
                                          u64 page_payload_bytes = 0)
{
  return detail::build_one(FilterKind::kBloom, filter_bits_per_key, leaf_page_id, items,
                           page_payload, page_payload_bytes);
}

inline Status build_quotient_filter_for_leaf(usize filter_bits_per_key, u64 leaf_page_id,
                                             const std::vector<std::string_view>& items,
                                             std::vector<u8>& page_payload,
                                             u64 page_payload_bytes)
{
  return detail::build_one(FilterKind::kQuotient, filter_bits_per_key, leaf_page_id, items,
                           page_payload, page_payload_bytes);
}

// Like the reference: a failed build is logged by the caller and the leaf gets no filter
// (filter_builder.hpp:323-325); the returned Status carries the reason.
// page_payload_bytes 0: the default TreeOptions' filter page payload at this bits/key
// (TreeOptions::filter_page_size(), tree/tree_options.hpp:177-220; 32,704 bytes at 12 bits/key)
inline Status build_filter_for_leaf_in_job(usize filter_bits_per_key, u64 leaf_page_id,
                                           const std::vector<std::string_view>& items,
                                           std::vector<u8>& page_payload,
                                           u64 page_payload_bytes = 0,
                                           FilterKind kind = kDefaultFilterKind)
{
  page_payload.clear();
  if (page_payload_bytes == 0 && filter_bits_per_key != 0)
    page_payload_bytes = default_filter_page_payload_size(filter_bits_per_key, kind);
  Status s = kind == FilterKind::kBloom
                 ? build_bloom_filter_for_leaf(filter_bits_per_key, leaf_page_id, items,
                                               page_payload, page_payload_bytes)
                 : build_quotient_filter_for_leaf(filter_bits_per_key, leaf_page_id, items,
                                                  page_payload, page_payload_bytes);
  if (!s.ok()) page_payload.clear();
  return s;
}

// ---------------------------------------------------------------------------------------
// LeafBatcher: the reference's per-leaf call pattern, built in batches
// ---------------------------------------------------------------------------------------
// build_all_pages runs build_filter_for_leaf_in_job once per leaf on its worker threads
// (tree/tree_serialize_context.cpp:71-75).  One GPU call per leaf pays a copy in, a build, a
// copy out and a synchronisation for one leaf.  LeafBatcher keeps that call site and batches
// the calls that arrive together:
//   - a call reserves its leaf's place in the open batch's pinned arena (keys, offsets) and
//     stages its keys there itself, in parallel with the other callers;
//   - the call that opened the batch (its leader) closes it after `linger`, or as soon as
//     the batch holds its share of the callers (below) or the arena is full, and the next call
//     opens another batch, which fills while this one is on the GPU;
//   - the leader waits for every member's keys, then builds the batch on its thread's stream:
//     one copy of the arena in, one plan, one build, one copy of the pages out;
//   - each caller copies its own page out of the batch's pinned output.
// A batch's share of the callers: the callers inside build() divided by `batches_in_flight`
// (at least 2, at most `max_batch`), so that several small batches run at once, each on its
// own stream, rather than one large one while the next collects.
// A batch holds leaves of one kind, bits/key, page size and key stride (0 = variable length);
// other calls open their own batch.  A leaf larger than the arena is built on its own.  If a
// batch's VQF build reports an insert failure, its leaves are rebuilt one by one so that only
// the failing leaf goes without a filter (filter_builder.hpp:323-325).
//
// Compile-time overrides for tools/leaf_bench.cpp sweeps (profiles/r06/leaf_sweep/, leaf_spin/):
// how long a member polls before it sleeps (16 VQF callers 1,046 Mkeys/s at 300 us, 930 at
// 200, ~750-860 at 0-100 or 400), and how many poll at once (16 / 32 VQF callers 942 / 1,272
// at 4, 878 / 1,105 at 8, 977 / 1,095 at 16; 2-6 within noise, sweep4)
#ifndef TKV_LEAF_SPIN_US
#define TKV_LEAF_SPIN_US 300
#endif
#ifndef TKV_LEAF_MAX_SPINNERS
#define TKV_LEAF_MAX_SPINNERS 4
#endif

class LeafBatcher
{
 public:
  struct Options {
    usize max_batch;  // leaves per batch at most
    std::chrono::microseconds linger;
    usize arena_bytes;  // pinned key bytes per batch (and as many bytes of offsets)
    usize batches_in_flight = 5;  // a batch closes at (callers in build()) / this many leaves
  };

  // (a batch collects callers for up to 60 us.  16 callers of 16K-key leaves, median of three
  // processes of five passes each, profiles/r06/leaf_sweep/: fixed batches of 3 leaves VQF
  // 1,046 Mkeys/s (members spinning 300 us), 4: 979, 5: 930, 8: 750-860, 16: 650-710; Bloom
  // 1,367-1,389 at 3, 1,259-1,279 at 4, 930-1,002 at 8.  32 callers at a fixed 3 fell to
  // 466-912 (VQF): hence a share of the callers, 16 / 5 -> 3, 32 / 5 -> 6.  With one wake-up
  // per batch instead of one for every waiting caller, 32 VQF callers run at 1,015-1,363
  // instead of swinging between ~450 and ~1,200; profiles/r06/leaf_default/, leaf_spin/)
  LeafBatcher() : LeafBatcher(Options{16, std::chrono::microseconds{60}, usize{8} << 20}) {}
  explicit LeafBatcher(Options o) : opt_{o}
  {
    if (opt_.max_batch == 0) opt_.max_batch = 1;
    if (opt_.batches_in_flight == 0) opt_.batches_in_flight = 1;
  }
  LeafBatcher(const LeafBatcher&) = delete;
  LeafBatcher& operator=(const LeafBatcher&) = delete;
  ~LeafBatcher()
  {
    for (Batch* b : all_) destroy(b);
  }

  Status build(FilterKind kind, usize bpk, u64 leaf_page_id, const std::vector<std::string_view>& items,
               std::vector<u8>& page_payload, u64 page_payload_bytes)
  {
    if (bpk == 0) {  // filter_builder.hpp:115-117, :227-229
      page_payload.clear();
      return OkStatus();
    }
    if (tkv_amq_device_count() == 0) return Status::from(TKV_AMQ_UNAVAILABLE, "no HIP device");
    const u64 n = items.size();
    u64 bytes = 0;
    bool fixed = n > 0;
    const u32 len0 = n ? (u32)items[0].size() : 0;
    for (const auto& k : items) {
      bytes += k.size();
      fixed = fixed && k.size() == len0;
    }
    const u32 stride = fixed && len0 ? len0 : 0;
    if (bytes > opt_.arena_bytes || n + 1 > key_cap()) {
      Status st = detail::build_one(kind, bpk, leaf_page_id, items, page_payload, page_payload_bytes);
      if (!st.ok()) page_payload.clear();
      return st;
    }

    Req r{&items, leaf_page_id, n, bytes};
    std::unique_lock<std::mutex> lk{mu_};
    ++active_;
    Batch* b = nullptr;
    bool leader = false;
    for (;;) {
      for (Batch* o : open_)
        if (o->kind == kind && o->bpk == bpk && o->cap == page_payload_bytes && o->stride == stride) b = o;
      if (b && (b->bytes + bytes > opt_.arena_bytes || b->n + n + 1 > key_cap())) {
        close(b);
        b = nullptr;
      }
      if (b || !free_.empty()) break;
      // a new batch's pinned arenas, stream and device buffers, allocated outside the lock
      lk.unlock();
      Batch* nb = create();
      lk.lock();
      if (!nb) {
        --active_;
        lk.unlock();
        Status st = detail::build_one(kind, bpk, leaf_page_id, items, page_payload, page_payload_bytes);
        if (!st.ok()) page_payload.clear();
        return st;
      }
      all_.push_back(nb);
      free_.push_back(nb);
    }
    if (!b) {
      leader = true;
      b = free_.back();
      free_.pop_back();
      b->kind = kind;
      b->bpk = bpk;
      b->cap = page_payload_bytes;
      b->stride = stride;
      open_.push_back(b);
    }
    r.key_off = b->n;
    r.byte_off = b->bytes;
    b->n += n;
    b->bytes += bytes;
    b->reqs.push_back(&r);
    ++b->users;
    if (b->reqs.size() >= batch_share()) close(b);
    lk.unlock();

    Status staged = stage(r, *b);
    // this leaf's keys (and offsets) to the device now, on the batch's stream: the copies of
    // the members overlap the collection window and each other's staging, so the leader's
    // build waits only for the last of them (round 6; they were one copy after the batch closed)
    // (a leaf whose staging failed copies too: its zero-length offsets keep the batch valid)
    if (n) {
      const Status c = copy_in(r, *b);
      if (staged.ok()) staged = c;
    }

    lk.lock();
    ++b->staged;
    b->cv.notify_all();
    if (leader) {
      const auto deadline = std::chrono::steady_clock::now() + opt_.linger;
      // no lingering once every caller inside build() has joined this batch (one thread alone
      // never waits)
      b->cv.wait_until(lk, deadline, [&] { return b->closed || b->reqs.size() >= active_; });
      if (!b->closed) close(b);
      b->cv.wait(lk, [&] { return b->staged == b->reqs.size(); });
      lk.unlock();
      run(*b);
      lk.lock();
      for (Req* q : b->reqs) {
        q->done = true;
        q->done_flag.store(true, std::memory_order_release);
      }
      b->cv.notify_all();
    } else {
      // a member first polls its flag (yielding) for about a batch's device time, then sleeps:
      // a condition-variable wake-up costs tens of microseconds on a busy host, about as long
      // as the batch's kernel.  At most kMaxSpinners poll at once (more callers than CPUs:
      // the pollers would take the CPUs the others stage their keys on)
      lk.unlock();
      if (spinners_.fetch_add(1, std::memory_order_relaxed) < kMaxSpinners) {
        const auto spin_until = std::chrono::steady_clock::now() + std::chrono::microseconds{kSpinUs};
        while (!r.done_flag.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < spin_until)
          std::this_thread::yield();
      }
      spinners_.fetch_sub(1, std::memory_order_relaxed);
      lk.lock();
      b->cv.wait(lk, [&] { return r.done; });
    }
    lk.unlock();

    // this leaf's page, from the batch's pinned output (or the per-leaf rebuild)
    Status st = staged.ok() ? r.st : staged;
    if (st.ok() && r.page) {
      page_payload.assign(page_payload_bytes ? page_payload_bytes : r.page_bytes, 0);
      std::memcpy(page_payload.data(), r.page, r.page_bytes);
    } else if (st.ok() && r.rebuilt) {
      page_payload.swap(r.rebuilt_page);
    } else {
      page_payload.clear();
    }
    lk.lock();
    if (--b->users == 0) release(b);
    --active_;
    for (Batch* o : open_) o->cv.notify_all();  // (their leaders' linger ends at every caller joined)
    return st;
  }

 private:
  struct Req {
    const std::vector<std::string_view>* items;
    u64 page_id;
    u64 n, bytes;
    u64 key_off = 0, byte_off = 0;  // this leaf's place in the batch arena
    Status st{};
    const u8* page = nullptr;  // into the batch's pinned output
    u64 page_bytes = 0;
    bool rebuilt = false;
    std::vector<u8> rebuilt_page;
    bool done = false;                 // under mu_
    std::atomic<bool> done_flag{false};  // the same, for the members' polling
  };

  static constexpr int kSpinUs = TKV_LEAF_SPIN_US;
  static constexpr int kMaxSpinners = TKV_LEAF_MAX_SPINNERS;

  struct Batch {
    FilterKind kind{};
    usize bpk = 0;
    u64 cap = 0;
    u32 stride = 0;
    u8* h_keys = nullptr;   // [arena_bytes + seg_area()]: the keys, then the segments (one copy in)
    u64* h_offs = nullptr;  // [arena_bytes / 8]
    u8* h_io = nullptr;     // [segments][status 64 B][pages]
    usize h_io_cap = 0;
    hipStream_t stream = nullptr;
    DeviceBuffer d_keys, d_offs, d_out;  // d_keys: keys then segments; d_out: pages then workspace
    u64 n = 0, bytes = 0;
    usize staged = 0, users = 0;
    bool closed = false;
    std::vector<Req*> reqs;
    std::condition_variable cv;  // this batch's leader and members wait here (under mu_)
  };

  usize key_cap() const { return opt_.arena_bytes / 8; }

  // under mu_: the leaves a batch closes at (Options::batches_in_flight)
  usize batch_share() const
  {
    const usize share = active_ / opt_.batches_in_flight;
    return std::min(opt_.max_batch, std::max<usize>(share, 2));
  }

  // under mu_
  void close(Batch* b)
  {
    b->closed = true;
    for (usize i = 0; i < open_.size(); ++i)
      if (open_[i] == b) {
        open_.erase(open_.begin() + i);
        break;
      }
    b->cv.notify_all();
  }

  // the segments after the batch's keys in the same buffers (256-byte aligned)
  usize seg_area() const { return 256 + opt_.max_batch * sizeof(tkv_amq_segment); }
  static u64 align256(u64 x) { return (x + 255) & ~u64{255}; }

  Batch* create()
  {
    Batch* b = new Batch;
    if (hipHostMalloc(reinterpret_cast<void**>(&b->h_keys), opt_.arena_bytes + seg_area()) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&b->h_offs), 8 * key_cap() + 8) != hipSuccess ||
        hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
        !b->d_keys.resize(opt_.arena_bytes + seg_area()) || !b->d_offs.resize(8 * key_cap() + 8)) {
      destroy(b);
      return nullptr;
    }
    return b;
  }

  static void destroy(Batch* b)
  {
    if (b->h_keys) (void)hipHostFree(b->h_keys);
    if (b->h_offs) (void)hipHostFree(b->h_offs);
    if (b->h_io) (void)hipHostFree(b->h_io);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
  }

  // grow-only, with headroom, so that steady state allocates nothing
  static bool reserve_device(DeviceBuffer& d, usize n) { return n <= d.size() || d.resize(n + n / 2); }

  void release(Batch* b)
  {
    b->reqs.clear();
    b->n = b->bytes = 0;
    b->staged = 0;
    b->closed = false;
    free_.push_back(b);
  }

  // the caller's keys into its reserved place in the arena; variable-length offsets are
  // staged leaf-relative into the thread's pinned scratch, then rebased into the arena
  static Status stage(const Req& r, Batch& b)
  {
    const auto& items = *r.items;
    const void* views = items.data();
    detail::LeafScratch& sc = detail::leaf_scratch();
    if (!detail::string_view_is_key_view()) {
      sc.views.resize(r.n);
      for (u64 i = 0; i < r.n; ++i)
        sc.views[i] = tkv_amq_key_view{items[i].size(), reinterpret_cast<const u8*>(items[i].data())};
      views = sc.views.data();
    }
    if (r.n == 0) return OkStatus();
    if (b.stride) {
      const int st = tkv_amq_stage_keys(views, sizeof(tkv_amq_key_view), r.n, b.stride,
                                        b.h_keys + r.byte_off, r.bytes, nullptr, 1);
      return st == TKV_AMQ_OK ? OkStatus() : Status::from(st, "tkv_amq_stage_keys");
    }
    u64* dst = b.h_offs + r.key_off;
    // on failure this leaf's slice of the batch offsets must not keep an earlier batch's
    // values (the batch is built anyway): zero-length keys at the leaf's own byte offset
    auto fail = [&](int code, const char* what) {
      for (u64 j = 0; j < r.n; ++j) dst[j] = r.byte_off;
      return Status::from(code, what);
    };
    if (!detail::LeafScratch::grow_pinned(sc.h_offs, sc.h_offs_cap, r.n + 1))
      return fail(TKV_AMQ_RESOURCE_EXHAUSTED, "hipHostMalloc");
    const int st = tkv_amq_stage_keys(views, sizeof(tkv_amq_key_view), r.n, 0, b.h_keys + r.byte_off,
                                      r.bytes, sc.h_offs, 1);
    if (st != TKV_AMQ_OK) return fail(st, "tkv_amq_stage_keys");
    for (u64 j = 0; j < r.n; ++j) dst[j] = sc.h_offs[j] + r.byte_off;
    return OkStatus();
  }

  // a member's staged keys (and its offsets) to the batch's device buffers, on its stream
  static Status copy_in(const Req& r, Batch& b)
  {
    if (hipMemcpyAsync(b.d_keys.get<u8>() + r.byte_off, b.h_keys + r.byte_off, r.bytes, hipMemcpyHostToDevice,
                       b.stream) != hipSuccess ||
        (b.stride == 0 && hipMemcpyAsync(b.d_offs.get<u8>() + 8 * r.key_off, b.h_offs + r.key_off, 8 * r.n,
                                         hipMemcpyHostToDevice, b.stream) != hipSuccess))
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpyAsync keys");
    return OkStatus();
  }

  // on the leader's thread: every member staged, nothing else touches the batch
  void run(Batch& b)
  {
    Status st = build_batch(b);
    if (!st.ok() && b.reqs.size() > 1 && st.code == TKV_AMQ_INTERNAL) {
      for (Req* q : b.reqs) {
        q->st = detail::build_one(b.kind, b.bpk, q->page_id, *q->items, q->rebuilt_page, b.cap);
        q->rebuilt = q->st.ok();
      }
    } else {
      for (Req* q : b.reqs) q->st = st;
    }
  }

  Status build_batch(Batch& b)
  {
    const usize n_segs = b.reqs.size();
    std::vector<u64> counts(n_segs), ids(n_segs);
    for (usize i = 0; i < n_segs; ++i) {
      counts[i] = b.reqs[i]->n;
      ids[i] = b.reqs[i]->page_id;
    }
    std::vector<tkv_amq_segment> segs(n_segs);
    u64 total_out = 0, ws_bytes = 0;
    u32 max_blocks = 0;
    int st = tkv_amq_plan((int)b.kind, counts.data(), ids.data(), (u32)n_segs, (u32)b.bpk, b.cap, 0,
                          segs.data(), &total_out, &ws_bytes, &max_blocks);
    if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_plan");
    const usize seg_bytes = n_segs * sizeof(tkv_amq_segment);
    // one copy out: the pages, then (VQF) the workspace header up to the leaves' nelts words,
    // the workspace placed after the pages in one device buffer
    const u64 ws_off = align256(total_out);
    const bool flags_out = b.kind == FilterKind::kQuotient && ws_bytes >= TKV_AMQ_VQF_NELTS_OFFSET + 4 * n_segs;
    const u64 out_bytes = flags_out ? ws_off + TKV_AMQ_VQF_NELTS_OFFSET + 4 * n_segs : total_out;
    const usize io_bytes = seg_bytes + out_bytes;
    if (!detail::LeafScratch::grow_pinned(b.h_io, b.h_io_cap, io_bytes <= b.h_io_cap ? io_bytes : io_bytes + io_bytes / 2))
      return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipHostMalloc");
    const u64 n = b.n, bytes = b.bytes;
    if (!reserve_device(b.d_out, ws_off + ws_bytes)) return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipMalloc");
    std::memcpy(b.h_io, segs.data(), seg_bytes);  // the host plan (tkv_amq_build_ex's h_segs)
    u8* h_out = b.h_io + seg_bytes;
    // the members copied their keys in (copy_in); the segments follow at the next 256-byte
    // boundary, and the offsets' closing entry
    const u64 seg_off = align256(bytes);
    std::memcpy(b.h_keys + seg_off, segs.data(), seg_bytes);
    if (b.stride == 0) b.h_offs[n] = bytes;
    hipStream_t s = b.stream;
    if (hipMemcpyAsync(b.d_keys.get<u8>() + seg_off, b.h_keys + seg_off, seg_bytes, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        (b.stride == 0 && hipMemcpyAsync(b.d_offs.get<u8>() + 8 * n, b.h_offs + n, 8, hipMemcpyHostToDevice, s) !=
                              hipSuccess))
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpyAsync segments");
    u8* d_ws = b.d_out.get<u8>() + ws_off;
    st = tkv_amq_build_ex((int)b.kind, b.d_keys.get(), b.stride ? nullptr : b.d_offs.get<u64>(), b.stride, n,
                          reinterpret_cast<const tkv_amq_segment*>(b.d_keys.get<u8>() + seg_off),
                          reinterpret_cast<const tkv_amq_segment*>(b.h_io), (u32)n_segs, max_blocks, b.d_out.get(),
                          ws_bytes ? d_ws : nullptr, ws_bytes, s);
    if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_build_ex");
    if (hipMemcpyAsync(h_out, b.d_out.get(), out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpyAsync pages");
    // (polled, yielding: a blocking synchronisation sleeps until an interrupt wakes it)
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady) std::this_thread::yield();
    if (q != hipSuccess) return Status::from(TKV_AMQ_INTERNAL, "hipStreamQuery");
    u32 flags = 0;
    if (flags_out) {
      const u32* h_flags = reinterpret_cast<const u32*>(h_out + ws_off + TKV_AMQ_VQF_NELTS_OFFSET);
      for (usize i = 0; i < n_segs; ++i) flags |= h_flags[i];
    }
    if (flags & TKV_AMQ_VQF_FLAG_WORKSPACE) return Status::from(TKV_AMQ_INVALID_ARGUMENT, "workspace");
    if (flags & TKV_AMQ_VQF_FLAG_OVERFLOW)
      return Status::from(TKV_AMQ_INTERNAL, "vqf_insert (filter_builder.hpp:211)");
    for (usize i = 0; i < n_segs; ++i) {
      b.reqs[i]->page = h_out + segs[i].out_offset;
      b.reqs[i]->page_bytes = segs[i].payload_bytes;
    }
    return OkStatus();
  }

  Options opt_;
  std::mutex mu_;
  std::atomic<int> spinners_{0};
  std::vector<Batch*> open_, free_, all_;
  usize active_ = 0;  // callers inside build() past their size check
};

// build_filter_for_leaf_in_job through a process-wide LeafBatcher: the reference's per-leaf
// call site, built in batches across the worker threads that call it concurrently.  The
// batcher is never destroyed, so no pinned memory is freed after the HIP runtime shuts down.
inline Status build_filter_for_leaf_in_job_batched(usize filter_bits_per_key, u64 leaf_page_id,
                                                   const std::vector<std::string_view>& items,
                                                   std::vector<u8>& page_payload,
                                                   u64 page_payload_bytes = 0,
                                                   FilterKind kind = kDefaultFilterKind)
{
  if (page_payload_bytes == 0 && filter_bits_per_key != 0)
    page_payload_bytes = default_filter_page_payload_size(filter_bits_per_key, kind);
  static LeafBatcher* batcher = new LeafBatcher;
  return batcher->build(kind, filter_bits_per_key, leaf_page_id, items, page_payload, page_payload_bytes);
}

// ---------------------------------------------------------------------------------------
// KeyQuery::reject_page for a batch of point queries against one filter page payload
// ---------------------------------------------------------------------------------------
enum class BoolStatus : int { kFalse = 0, kTrue = 1, kUnknown = 2 };

// FastCountMetric<u64>
struct CountMetric {
  std::atomic<u64> value{0};
  void add(u64 n) { value.fetch_add(n, std::memory_order_relaxed); }
  u64 get() const { return value.load(std::memory_order_relaxed); }
};

class KeyQuery
{
 public:
  // KeyQuery::Metrics, the filter counters (tree/key_query.hpp:36-60).  reject_page updates
  // total / no-filter / load-failed / page-id-mismatch / reject (:154,157,183,210,231,243);
  // positive / false positive are the caller's leaf search's (key_query.cpp:41,77):
  // reject_page counts them when the caller passes the ground truth.
  struct Metrics {
    CountMetric total_filter_query_count;
    CountMetric no_filter_page_count;
    CountMetric filter_page_load_failed_count;
    CountMetric page_id_mismatch_count;
    CountMetric filter_reject_count;
    CountMetric filter_positive_count;
    CountMetric filter_false_positive_count;

    double filter_false_positive_rate() const noexcept
    {
      const double positives = (double)filter_positive_count.get();
      if (positives == 0) return -1;
      return (double)filter_false_positive_count.get() / positives;
    }
  };

  static Metrics& metrics()
  {
    static Metrics metrics_;
    return metrics_;
  }

  explicit KeyQuery(std::vector<std::string_view> keys) : keys_{std::move(keys)} {}

  // per key: kTrue = definitely absent; kFalse = maybe present; kUnknown = no filter or the
  // filter belongs to another page (key_query.hpp:156-159, 207-212, 227-232).
  // truth (optional, one per key: 1 = the key is in the leaf) feeds the positive /
  // false-positive counters the reference's leaf search keeps (key_query.cpp:41,77).
  Status reject_page(u64 page_id_to_reject, const std::vector<u8>* filter_payload,
                     FilterKind kind, std::vector<BoolStatus>& out,
                     const std::vector<u8>* truth = nullptr)
  {
    Metrics& m = metrics();
    const u64 n = keys_.size();
    out.assign(n, BoolStatus::kUnknown);
    m.total_filter_query_count.add(n);
    if (!filter_payload) {
      m.no_filter_page_count.add(n);
      return OkStatus();
    }
    if (filter_payload->size() < 64) {  // cannot be read as a filter page: cannot reject
      m.filter_page_load_failed_count.add(n);
      return OkStatus();
    }
    u64 magic, src;
    std::memcpy(&magic, filter_payload->data(), 8);
    std::memcpy(&src, filter_payload->data() + (kind == FilterKind::kBloom ? 16 : 8), 8);
    const u64 want = kind == FilterKind::kBloom ? PackedBloomFilterPage::kMagic : PackedVqfFilter::kMagic;
    if (magic != want) return Status::from(TKV_AMQ_INTERNAL, "filter page magic");
    if (src != page_id_to_reject) {
      m.page_id_mismatch_count.add(n);
      return OkStatus();
    }
    if (keys_.empty()) return OkStatus();
    if (tkv_amq_device_count() == 0) return Status::from(TKV_AMQ_UNAVAILABLE, "no HIP device");

    // single-segment plan whose payload sits at offset 0 of the staged page
    tkv_amq_segment seg{};
    if (kind == FilterKind::kBloom) {
      PackedBloomFilterPage h;
      std::memcpy(&h, filter_payload->data(), sizeof(h));
      seg.n_blocks = h.block_count;
      seg.hash_count = h.hash_count;
    } else {
      if (filter_payload->size() < sizeof(PackedVqfFilter)) {
        m.filter_page_load_failed_count.add(n);
        return OkStatus();
      }
      PackedVqfFilter h;
      std::memcpy(&h, filter_payload->data(), sizeof(h));
      const u64 tb = h.metadata.key_remainder_bits;
      if ((tb != 8 && tb != 16) || h.metadata.nblocks == 0 || h.hash_mask == 0)
        return Status::from(TKV_AMQ_INTERNAL, "PackedVqfFilter metadata");
      // hash_mask = ~0 << hash_val_shift (filter_builder.hpp:187): truncated leaves answer
      // "maybe" for every hash with a low bit set (vqf_filter_page_view.hpp:115-117)
      const u32 shift = (u32)__builtin_ctzll(h.hash_mask);
      if (h.hash_mask != (~u64{0} << shift)) return Status::from(TKV_AMQ_INTERNAL, "hash_mask");
      const u64 buckets = tb == 8 ? 80 : 36;
      seg.n_blocks = (u32)h.metadata.nblocks;
      seg.tag_bits = (u8)tb;
      seg.hash_val_shift = (u8)shift;
      seg.mod_magic = ~0ull / (h.metadata.nblocks * buckets);
    }
    seg.out_offset = 0;
    DeviceBuffer d_keys, d_offs, d_page, d_seg, d_leaf, d_res;
    if (!d_page.resize(filter_payload->size()) || !d_seg.resize(sizeof(seg)) ||
        !d_leaf.resize(4 * n) || !d_res.resize(n))
      return Status::from(TKV_AMQ_RESOURCE_EXHAUSTED, "hipMalloc");
    bool fixed = false;
    u32 stride = 16;
    TKV_AMQ_REQUIRE_OK(detail::stage_keys(keys_, d_keys, d_offs, fixed, stride));
    if (hipMemcpy(d_page.get(), filter_payload->data(), filter_payload->size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_seg.get(), &seg, sizeof(seg), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d_leaf.get(), 0, 4 * n) != hipSuccess)
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpy page");
    const int st = tkv_amq_probe((int)kind, d_page.get(), d_seg.get<tkv_amq_segment>(), 1,
                                 d_keys.get(), fixed ? nullptr : d_offs.get<u64>(),
                                 fixed ? stride : 0, n, d_leaf.get<u32>(), d_res.get(), nullptr);
    if (st != TKV_AMQ_OK) return Status::from(st, "tkv_amq_probe");
    std::vector<u8> res(n);
    if (hipMemcpy(res.data(), d_res.get(), res.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return Status::from(TKV_AMQ_INTERNAL, "hipMemcpy result");
    u64 rejects = 0, fps = 0;
    for (usize i = 0; i < res.size(); ++i) {
      out[i] = res[i] ? BoolStatus::kFalse : BoolStatus::kTrue;
      rejects += res[i] == 0;
      if (truth && i < truth->size()) fps += res[i] != 0 && (*truth)[i] == 0;
    }
    m.filter_reject_count.add(rejects);
    m.filter_positive_count.add(n - rejects);
    if (truth) m.filter_false_positive_count.add(fps);
    return OkStatus();
  }

 private:
  std::vector<std::string_view> keys_;
};

}  // namespace turtle_kv_amd

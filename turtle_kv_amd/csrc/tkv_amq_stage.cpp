// tkv_amq_stage.cpp -- host key staging: the H2D front end of the filter build
// (SURVEY.md 8(f) row 4).
//
// The reference hands build_filter_for_leaf_in_job a range of EditView (key + value views)
// flattened out of a ResultSet's chunks (core/merge_compactor.hpp:107-139,
// tree/filter_builder.hpp:307-331); each key is a KeyView (std::string_view) pointing into
// leaf / edit memory.  The device build wants one contiguous key array, so this gathers the
// viewed bytes into a caller-owned (normally pinned) buffer with a few host threads.  The
// view array is read in place at any stride: `&edits[0].key` with stride sizeof(EditView)
// works without building a pointer list.  Host only: no HIP call, usable without a device.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "tkv_amq.h"

namespace {

inline const tkv_amq_key_view& view_at(const void* views, uint64_t stride, uint64_t i)
{
  return *reinterpret_cast<const tkv_amq_key_view*>(static_cast<const uint8_t*>(views) + i * stride);
}

// Splits [0, n) into `parts` contiguous ranges and runs fn(part, begin, end) on each, part 0
// on the calling thread.
template <typename Fn>
void parallel_ranges(uint64_t n, int parts, Fn&& fn)
{
  const uint64_t per = (n + parts - 1) / parts;
  std::vector<std::thread> pool;
  pool.reserve(parts - 1);
  for (int t = 1; t < parts; ++t) {
    const uint64_t b = std::min(n, per * t), e = std::min(n, b + per);
    pool.emplace_back([&fn, t, b, e] { fn(t, b, e); });
  }
  fn(0, 0, std::min(n, per));
  for (auto& th : pool) th.join();
}

// Threads for n keys: small batches stay on the calling thread.
int resolve_threads(int n_threads, uint64_t n)
{
  int t = n_threads;
  if (t <= 0) t = (int)std::min(std::max(1u, std::thread::hardware_concurrency()), 16u);
  t = std::min(t, 256);
  const uint64_t max_useful = std::max<uint64_t>(1, n / 16384);  // >= 16K keys per thread
  return (int)std::min<uint64_t>((uint64_t)t, max_useful);
}

}  // namespace

extern "C" {

int tkv_amq_stage_keys(const void* views, uint64_t view_stride, uint64_t n, uint32_t fixed_len,
                       uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_offsets, int n_threads)
{
  if (fixed_len == 0 && !dst_offsets) return TKV_AMQ_INVALID_ARGUMENT;
  if (n == 0) {
    if (fixed_len == 0) dst_offsets[0] = 0;
    return TKV_AMQ_OK;
  }
  if (!views || !dst || view_stride < sizeof(tkv_amq_key_view)) return TKV_AMQ_INVALID_ARGUMENT;
  const int parts = resolve_threads(n_threads, n);
  std::atomic<int> bad{0};

  if (fixed_len != 0) {
    // key i -> dst + i * fixed_len; every key must have exactly fixed_len bytes
    if (n > dst_capacity / fixed_len) return TKV_AMQ_RESOURCE_EXHAUSTED;
    parallel_ranges(n, parts, [&](int, uint64_t b, uint64_t e) {
      uint8_t* d = dst + b * fixed_len;
      for (uint64_t i = b; i < e; ++i, d += fixed_len) {
        const tkv_amq_key_view& v = view_at(views, view_stride, i);
        if (v.size != fixed_len || !v.data) {
          bad.store(1, std::memory_order_relaxed);
          return;
        }
        if (fixed_len == 16) memcpy(d, v.data, 16);  // the common case: one 16-byte move
        else memcpy(d, v.data, fixed_len);
      }
    });
    return bad.load() ? TKV_AMQ_INVALID_ARGUMENT : TKV_AMQ_OK;
  }

  // variable length: byte total per range, exclusive scan over the ranges, then the copy
  std::vector<uint64_t> base(parts + 1, 0);
  parallel_ranges(n, parts, [&](int t, uint64_t b, uint64_t e) {
    uint64_t s = 0;
    for (uint64_t i = b; i < e; ++i) {
      const tkv_amq_key_view& v = view_at(views, view_stride, i);
      if (!v.data && v.size) bad.store(1, std::memory_order_relaxed);
      s += v.size;
    }
    base[t + 1] = s;
  });
  if (bad.load()) return TKV_AMQ_INVALID_ARGUMENT;
  for (int t = 0; t < parts; ++t) base[t + 1] += base[t];
  if (base[parts] > dst_capacity) return TKV_AMQ_RESOURCE_EXHAUSTED;
  parallel_ranges(n, parts, [&](int t, uint64_t b, uint64_t e) {
    uint64_t off = base[t];
    for (uint64_t i = b; i < e; ++i) {
      const tkv_amq_key_view& v = view_at(views, view_stride, i);
      dst_offsets[i] = off;
      if (v.size) memcpy(dst + off, v.data, v.size);
      off += v.size;
    }
  });
  dst_offsets[n] = base[parts];
  return TKV_AMQ_OK;
}

}  // extern "C"

// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_host_sanitize.py):
// the sizing / plan entry points of libtkv_amq (host part of tkv_amq_kernels.hip), the key
// staging of tkv_amq_stage.cpp, and the CPU oracle.  Reads one case per stdin line and prints
// one result line per case; the test compares them with the same calls through the
// unsanitized libraries.  Needs no device (no HIP call is made).
//   plan <kind> <bpk> <cap> <stride> <page_log2> <n> <count>...  -> status total ws maxb fnv
//   size <kind> <leaf_size> <key_hint> <value_hint> <bpk>       -> log2 items data_size
//   bloom <n> <bpk> <seed>                                       -> status fnv negatives
//   vqf <n> <bpk> <cap> <seed>                                   -> status fnv used negatives
//   stage <fixed_len> <n> <threads> <seed>                       -> status ok
//   obuild <kind> <n_segs> <keys_per_seg> <bpk> <threads> <seed>  -> status fnv
//     (the oracle's threaded checkpoint-level build, tkvo_build_segments; VQF at 32704 B)
// Built twice by the test: AddressSanitizer + UBSan, and ThreadSanitizer (the threaded paths).
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../oracle/tkv_amq_oracle.h"
#include "tkv_amq.h"

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull)
{
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

static void plan_case(std::istringstream& in)
{
  int kind;
  uint32_t bpk, page_log2, n;
  uint64_t cap, stride;
  in >> kind >> bpk >> cap >> stride >> page_log2 >> n;
  std::vector<uint64_t> counts(n);
  for (auto& c : counts) in >> c;
  // exactly n segments: the sanitizer sees any write past them
  std::vector<tkv_amq_segment> segs(n);
  uint64_t total = 0, ws = 0;
  uint32_t maxb = 0;
  const int st = page_log2
                     ? tkv_amq_plan_pages(kind, n ? counts.data() : nullptr, nullptr, n, bpk, page_log2,
                                          n ? segs.data() : nullptr, &total, &ws, &maxb)
                     : tkv_amq_plan(kind, n ? counts.data() : nullptr, nullptr, n, bpk, cap, stride,
                                    n ? segs.data() : nullptr, &total, &ws, &maxb);
  const uint64_t h = st == TKV_AMQ_OK && n ? fnv(segs.data(), sizeof(tkv_amq_segment) * n) : 0;
  std::printf("plan %d %" PRIu64 " %" PRIu64 " %u %" PRIu64 "\n", st, total, ws, maxb, h);
}

static void size_case(std::istringstream& in)
{
  int kind;
  uint64_t leaf, bpk;
  uint32_t key, val;
  in >> kind >> leaf >> key >> val >> bpk;
  std::printf("size %u %" PRIu64 " %" PRIu64 "\n", tkv_amq_filter_page_size_log2(kind, leaf, key, val, bpk),
              tkv_amq_expected_items_per_leaf(leaf, key, val), tkv_amq_leaf_data_size(leaf));
}

static uint32_t false_negatives(int kind, const std::vector<uint8_t>& keys, uint64_t n,
                                const uint8_t* payload)
{
  uint32_t neg = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* k = keys.data() + 16 * i;
    const int r = kind == 0 ? tkvo_bloom_query_payload(payload, k, 16)
                            : tkvo_vqf_is_present_payload(payload, tkvo_xxh64(k, 16, 0x9D0924DC03E79A75ull));
    neg += r == 0;
  }
  return neg;
}

static void bloom_case(std::istringstream& in)
{
  uint64_t n, seed;
  uint32_t bpk;
  in >> n >> bpk >> seed;
  std::vector<uint8_t> keys(16 * n + 1);
  tkvo_gen_keys16(seed, 0, n, keys.data());
  const uint64_t cap = tkvo_bloom_payload_size(n, bpk);
  std::vector<uint8_t> out(cap);  // exactly the payload: the sanitizer sees any overrun
  const int st = tkvo_bloom_build_payload(keys.data(), nullptr, 16, n, bpk, 7, out.data(), cap);
  std::printf("bloom %d %" PRIu64 " %u\n", st, fnv(out.data(), cap),
              st == 0 && bpk ? false_negatives(0, keys, n, out.data()) : 0u);
}

static void vqf_case(std::istringstream& in)
{
  uint64_t n, bpk, cap, seed;
  in >> n >> bpk >> cap >> seed;
  std::vector<uint8_t> keys(16 * n + 1);
  tkvo_gen_keys16(seed, 0, n, keys.data());
  std::vector<uint64_t> seg = {0, n};
  tkvo_sort_keys16_segments(keys.data(), seg.data(), 1, 1);
  std::vector<uint8_t> out(cap);
  tkvo_vqf_plan plan;
  memset(&plan, 0, sizeof(plan));
  const int st = tkvo_vqf_build_payload(keys.data(), nullptr, 16, n, bpk, 9, out.data(), cap, &plan);
  const uint64_t used = st == 0 ? plan.payload_used : 0;
  // a truncated (hash-shifted) filter answers "maybe" for keys it did not insert; the
  // negatives are counted for full filters only
  std::printf("vqf %d %" PRIu64 " %" PRIu64 " %u\n", st, fnv(out.data(), used), used,
              st == 0 && plan.tag_bits && plan.hash_val_shift == 0 ? false_negatives(1, keys, n, out.data()) : 0u);
}

static void stage_case(std::istringstream& in)
{
  uint32_t fixed, threads;
  uint64_t n, seed;
  in >> fixed >> n >> threads >> seed;
  std::vector<uint8_t> blob(48 * n + 64);
  for (size_t i = 0; i < blob.size(); ++i) blob[i] = (uint8_t)tkvo_splitmix64_at(seed, i);
  std::vector<tkv_amq_key_view> views(n);
  uint64_t bytes = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = fixed ? fixed : tkvo_splitmix64_at(seed ^ 1, i) % 48;
    // views in reverse address order, lengths up to 47
    views[i].size = len;
    views[i].data = blob.data() + 48 * (n - 1 - i);
    bytes += len;
  }
  std::vector<uint8_t> dst(bytes);  // exactly the bytes needed
  std::vector<uint64_t> offs(fixed ? 0 : n + 1);
  const int st = tkv_amq_stage_keys(views.data(), sizeof(tkv_amq_key_view), n, fixed, dst.data(),
                                    dst.size(), fixed ? nullptr : offs.data(), (int)threads);
  bool ok = st == TKV_AMQ_OK;
  uint64_t off = 0;
  for (uint64_t i = 0; ok && i < n; ++i) {
    if (!fixed && offs[i] != off) ok = false;
    if (views[i].size && memcmp(dst.data() + off, views[i].data, views[i].size) != 0) ok = false;
    off += views[i].size;
  }
  if (ok && !fixed && offs[n] != bytes) ok = false;
  std::printf("stage %d %d\n", st, ok ? 1 : 0);
}

static void obuild_case(std::istringstream& in)
{
  int kind, threads;
  uint32_t n_segs, bpk;
  uint64_t per, seed;
  in >> kind >> n_segs >> per >> bpk >> threads >> seed;
  const uint64_t n = per * n_segs;
  std::vector<uint8_t> keys(16 * n + 1);
  tkvo_gen_keys16(seed, 0, n, keys.data());
  std::vector<uint64_t> begin(n_segs + 1), off(n_segs), capv(n_segs);
  uint64_t total = 0;
  for (uint32_t s = 0; s <= n_segs; ++s) begin[s] = per * s;
  for (uint32_t s = 0; s < n_segs; ++s) {
    capv[s] = kind == 0 ? tkvo_bloom_payload_size(per, bpk) : 32704;
    off[s] = total;
    total += capv[s];
  }
  if (kind == 1) tkvo_sort_keys16_segments(keys.data(), begin.data(), n_segs, threads);
  std::vector<uint8_t> out(total + 1);
  const int st = tkvo_build_segments(kind, keys.data(), begin.data(), n_segs, bpk, nullptr, out.data(),
                                     off.data(), capv.data(), threads);
  std::printf("obuild %d %" PRIu64 "\n", st, fnv(out.data(), total));
}

int main()
{
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op == "plan") plan_case(in);
    else if (op == "size") size_case(in);
    else if (op == "bloom") bloom_case(in);
    else if (op == "vqf") vqf_case(in);
    else if (op == "stage") stage_case(in);
    else if (op == "obuild") obuild_case(in);
    else if (!op.empty()) {
      std::fprintf(stderr, "unknown case %s\n", op.c_str());
      return 2;
    }
    std::fflush(stdout);
  }
  return 0;
}

// Per-leaf drop-in throughput: build_filter_for_leaf_in_job called once per leaf from T
// worker threads, as TreeSerializeContext::build_all_pages does (tree/tree_serialize_context.cpp
// :71-75, tree/filter_builder.hpp:307-331).  Host keys in, host filter pages out (PCIe
// included); the batched host pipeline's rate is bench.py's e2e_pcie_inclusive.
//   leaf_bench <threads> <leaves> [keys_per_leaf=16384] [kind: 0 bloom | 1 vqf] [batched: 0 | 1] [max_batch=16] [linger_us=60] [batches_in_flight=5]
#include <turtle_kv_amd/filter_builder.hpp>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

using namespace turtle_kv_amd;

static u64 splitmix(u64& s)
{
  u64 z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv)
{
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int leaves = argc > 2 ? std::atoi(argv[2]) : 512;
  const u64 per = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 16384;
  const FilterKind kind = (argc > 4 && std::atoi(argv[4]) == 1) ? FilterKind::kQuotient : FilterKind::kBloom;
  const bool batched = argc > 5 && std::atoi(argv[5]) == 1;
  LeafBatcher::Options bo{(usize)(argc > 6 ? std::atoi(argv[6]) : 16),
                          std::chrono::microseconds{argc > 7 ? std::atoi(argv[7]) : 60}, usize{8} << 20};
  if (argc > 8) bo.batches_in_flight = (usize)std::atoi(argv[8]);
  LeafBatcher batcher{bo};
  const usize bpk = kind == FilterKind::kBloom ? 10 : 12;
  const u64 page = 32768 - kPackedPageHeaderSize;
  if (tkv_amq_device_count() == 0) {
    std::printf("no device\n");
    return 2;
  }
  // keys: 16 bytes each, sorted within a leaf (VQF inserts in leaf order) and laid out one
  // leaf after another in one arena, as items of a leaf page sit in its page buffer
  std::vector<std::array<u64, 2>> raw(leaves * per);
  u64 seed = 42;
  for (auto& k : raw) k = {splitmix(seed), splitmix(seed)};
  auto key_less = [](const std::array<u64, 2>& a, const std::array<u64, 2>& b) {
    return std::memcmp(a.data(), b.data(), 16) < 0;
  };
  for (int l = 0; l < leaves; ++l) std::sort(raw.begin() + l * per, raw.begin() + (l + 1) * per, key_less);
  const char* arena = reinterpret_cast<const char*>(raw.data());
  std::vector<std::vector<std::string_view>> items(leaves);
  for (int l = 0; l < leaves; ++l) {
    items[l].reserve(per);
    for (u64 i = 0; i < per; ++i) items[l].emplace_back(arena + 16 * (l * per + i), 16);
  }
  std::vector<std::vector<u8>> pages(leaves);

  // each worker builds every leaf once untimed (its thread-local stream and buffers are
  // created then), waits for the others, then the timed pass builds every leaf again
  auto run = [&](int t_count) {
    std::atomic<int> next_warm{0}, next{0}, failed{0}, ready{0};
    std::atomic<bool> go{false};
    auto build = [&](int l) {
      return batched ? batcher.build(kind, bpk, 1000 + l, items[l], pages[l], page)
                     : build_filter_for_leaf_in_job(bpk, 1000 + l, items[l], pages[l], page, kind);
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < t_count; ++t)
      pool.emplace_back([&] {
        for (int l; (l = next_warm.fetch_add(1)) < leaves;) (void)build(l);
        ready.fetch_add(1);
        while (!go.load()) std::this_thread::yield();
        for (int l; (l = next.fetch_add(1)) < leaves;)
          if (!build(l).ok()) failed.fetch_add(1);
      });
    while (ready.load() < t_count) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true);
    for (auto& th : pool) th.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return std::make_pair(dt, failed.load());
  };
  // (the timed pass 5 times at `threads` callers, the median reported: one pass is ~40 ms)
  for (int t : {1, threads}) {
    std::vector<double> dts;
    int failed = 0;
    for (int rep = 0; rep < (t == 1 ? 1 : 5); ++rep) {
      auto [d, f] = run(t);
      dts.push_back(d);
      failed += f;
    }
    std::sort(dts.begin(), dts.end());
    const double dt = dts[dts.size() / 2];
    std::printf("per-leaf %s: %2d threads  %d leaves x %llu keys  %.2f ms  %.0f leaves/s  %.1f Mkeys/s%s\n",
                batched ? "batched " : "drop-in", t, leaves, (unsigned long long)per, dt * 1e3, leaves / dt, leaves * per / dt / 1e6,
                failed ? "  FAILED" : "");
    if (batched)
      std::printf("  (max_batch %zu, linger %d us, batches in flight %zu, member spin %d us; %zu passes %.1f-%.1f Mkeys/s)\n",
                  bo.max_batch, (int)bo.linger.count(), bo.batches_in_flight, TKV_LEAF_SPIN_US, dts.size(),
                  leaves * per / dts.back() / 1e6, leaves * per / dts.front() / 1e6);
  }
  return 0;
}

// C++ parity test of the header-only host mirror (include/turtle_kv_amd/filter_builder.hpp)
// over libtkv_amq.so.  Reads the golden fixtures; exits non-zero on any mismatch.
// Usage: test_mirror <tests/golden dir>
#include <turtle_kv_amd/filter_builder.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

using namespace turtle_kv_amd;

static int failures = 0;
#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                   \
    }                                                               \
  } while (0)

static std::vector<u8> read_file(const std::string& p)
{
  std::ifstream f(p, std::ios::binary);
  return std::vector<u8>(std::istreambuf_iterator<char>(f), {});
}

int main(int argc, char** argv)
{
  const std::string dir = argc > 1 ? argv[1] : "tests/golden";
  std::vector<std::string> keys;
  {
    std::ifstream f(dir + "/workload_e_keys.txt");
    for (std::string line; std::getline(f, line);)
      if (!line.empty()) keys.push_back(line);
  }
  std::vector<std::string_view> items(keys.begin(), keys.end());
  EXPECT(items.size() == 4096);
  EXPECT(filter_bits_per_key(std::nullopt) == 12);
  EXPECT(filter_bits_per_key(10) == 12);
  EXPECT(filter_bits_per_key(10, FilterKind::kBloom) == 10);
  EXPECT(vqf_filter_load_factor<8>(12) == 10.2 / 12.0);
  // TreeOptions filter page sizing (host only): defaults -> 32 KiB pages, 32,704 payload bytes
  {
    TreeOptions t = TreeOptions::with_default_values();
    EXPECT(t.leaf_size() == (u64{2} << 20) && t.leaf_data_size() == (usize{2} << 20) - 104);
    EXPECT(t.expected_items_per_leaf() == 15767);
    EXPECT(t.filter_page_size_log2() == 15 && t.filter_page_payload_size() == 32704);
    EXPECT(TreeOptions{FilterKind::kBloom}.set_filter_bits_per_key(10).filter_bits_per_key() == 10);
    EXPECT(TreeOptions{}.set_filter_bits_per_key(10).filter_bits_per_key() == 12);
    EXPECT(default_filter_page_payload_size(12, FilterKind::kQuotient) == 32704);
  }

  // build_filter_for_leaf_in_job, default kind = VQF (config.hpp:24)
  std::vector<u8> vqf_page;
  Status s = build_filter_for_leaf_in_job(12, 7, items, vqf_page);
  if (tkv_amq_device_count() == 0) {
    // no GPU: the device path must fail loudly, never fall back to a CPU build
    EXPECT(s.code == TKV_AMQ_UNAVAILABLE && vqf_page.empty());
    std::printf("%s (no device; %d failures)\n", failures ? "FAIL" : "NODEVICE-OK", failures);
    return failures ? 1 : 0;
  }
  EXPECT(s.ok());
  const std::vector<u8> want_vqf = read_file(dir + "/workload_e_vqf12.bin");
  EXPECT(vqf_page.size() == 32768 - 64);
  EXPECT(std::equal(want_vqf.begin(), want_vqf.end(), vqf_page.begin()));
  PackedVqfFilter hdr;
  std::memcpy(&hdr, vqf_page.data(), sizeof(hdr));
  EXPECT(hdr.magic == PackedVqfFilter::kMagic && hdr.src_page_id == 7 && hdr.hash_seed == kVqfHashSeed);
  EXPECT(hdr.metadata.key_remainder_bits == 8 && hdr.metadata.nelts == 4096);

  std::vector<u8> bloom_page;
  s = build_bloom_filter_for_leaf(10, 7, items, bloom_page);
  EXPECT(s.ok());
  EXPECT(bloom_page == read_file(dir + "/workload_e_bloom10.bin"));

  // bits_per_key == 0: no filter, OK
  std::vector<u8> none;
  EXPECT(build_filter_for_leaf_in_job(0, 7, items, none).ok() && none.empty());
  // VQF below the 12-bit minimum: InvalidArgument (vqf_filter_page_view.hpp:46)
  EXPECT(build_quotient_filter_for_leaf(10, 7, items, none, 32704).code == TKV_AMQ_INVALID_ARGUMENT);

  // reject_page: present keys are never rejected; wrong page => kUnknown
  KeyQuery q(items);
  std::vector<BoolStatus> r;
  EXPECT(q.reject_page(7, &vqf_page, FilterKind::kQuotient, r).ok());
  size_t n_false = 0;
  for (auto v : r) n_false += v == BoolStatus::kFalse;
  EXPECT(n_false == items.size());
  EXPECT(q.reject_page(8, &vqf_page, FilterKind::kQuotient, r).ok() && r[0] == BoolStatus::kUnknown);
  EXPECT(q.reject_page(7, &bloom_page, FilterKind::kBloom, r).ok() && r[5] == BoolStatus::kFalse);

  std::vector<std::string> miss;
  for (int i = 0; i < 4096; ++i) miss.push_back("miss" + std::to_string(1000000 + i * 7919) + "zz");
  KeyQuery qm(std::vector<std::string_view>(miss.begin(), miss.end()));
  EXPECT(qm.reject_page(7, &vqf_page, FilterKind::kQuotient, r).ok());
  size_t n_true = 0;
  for (auto v : r) n_true += v == BoolStatus::kTrue;
  EXPECT(n_true > 4000);

  // batched builder over device keys == per-leaf results
  {
    FilterBatchBuilder b{FilterKind::kQuotient, 12, 32704};
    b.add_leaf(7, 4096);
    b.add_leaf(8, 0);
    EXPECT(b.plan().ok());
    DeviceBuffer d_keys(4096 * 24), d_out(b.total_out_bytes());
    std::string blob;
    for (auto& k : keys) blob += k;
    (void)hipMemcpy(d_keys.get(), blob.data(), blob.size(), hipMemcpyHostToDevice);
    EXPECT(b.build_all(d_keys.get(), 24, nullptr, d_out.get()).ok());
    EXPECT(b.check().ok());
    std::vector<u8> out(want_vqf.size());
    (void)hipMemcpy(out.data(), d_out.get(), out.size(), hipMemcpyDeviceToHost);
    EXPECT(out == want_vqf);
  }
  // LeafBatcher: the per-leaf call site from 16 worker threads, built in batches.  Every page
  // equals the unbatched per-leaf build; leaves mix 24-byte and variable-length keys (one
  // batch then stages offsets), kinds and sizes, and include an empty leaf.
  {
    const int n_leaves = 96;
    std::vector<std::vector<std::string>> leaf_keys(n_leaves);
    uint64_t st = 12345;
    auto rnd = [&st] {
      st ^= st << 13;
      st ^= st >> 7;
      st ^= st << 17;
      return st;
    };
    for (int l = 0; l < n_leaves; ++l) {
      const int n = l == 5 ? 0 : 500 + (int)(rnd() % 4000);
      for (int i = 0; i < n; ++i) {
        const int len = (l % 3 == 0) ? 24 : 4 + (int)(rnd() % 40);
        std::string k(len, '\0');
        for (auto& c : k) c = (char)rnd();
        leaf_keys[l].push_back(k);
      }
      std::sort(leaf_keys[l].begin(), leaf_keys[l].end());
      leaf_keys[l].erase(std::unique(leaf_keys[l].begin(), leaf_keys[l].end()), leaf_keys[l].end());
    }
    std::vector<std::vector<std::string_view>> views(n_leaves);
    for (int l = 0; l < n_leaves; ++l) views[l].assign(leaf_keys[l].begin(), leaf_keys[l].end());
    // (the process-wide batcher from 16 and 32 threads: batches close at 3 and 6 leaves; a
    // batcher whose max_batch 4 caps the 32 threads' share of 16)
    LeafBatcher capped{LeafBatcher::Options{4, std::chrono::microseconds{60}, usize{8} << 20, 2}};
    for (FilterKind kind : {FilterKind::kQuotient, FilterKind::kBloom}) {
      const usize bpk = kind == FilterKind::kBloom ? 10 : 12;
      std::vector<std::vector<u8>> want(n_leaves);
      for (int l = 0; l < n_leaves; ++l)
        EXPECT(build_filter_for_leaf_in_job(bpk, 500 + l, views[l], want[l], 32768 - 64, kind).ok());
      for (const int threads : {16, 32, -32}) {
        std::vector<std::vector<u8>> got(n_leaves);
        std::vector<Status> got_st(n_leaves);
        std::vector<std::thread> pool;
        const int nt = threads < 0 ? -threads : threads;
        for (int t = 0; t < nt; ++t)
          pool.emplace_back([&, t] {
            for (int l = t; l < n_leaves; l += nt)
              got_st[l] = threads < 0 ? capped.build(kind, bpk, 500 + l, views[l], got[l], 32768 - 64)
                                      : build_filter_for_leaf_in_job_batched(bpk, 500 + l, views[l], got[l],
                                                                             32768 - 64, kind);
          });
        for (auto& th : pool) th.join();
        for (int l = 0; l < n_leaves; ++l) {
          EXPECT(got_st[l].ok());
          EXPECT(got[l] == want[l]);
        }
      }
      // one caller alone: its batch closes at once
      std::vector<u8> solo;
      EXPECT(build_filter_for_leaf_in_job_batched(bpk, 501, views[1], solo, 32768 - 64, kind).ok());
      EXPECT(solo == want[1]);
    }
  }
  // reject_page on a leaf whose hashes were truncated to fit the page (hash_val_shift > 0,
  // filter_builder.hpp:277-290): no inserted key may be rejected (the shift must
  // come from the page's hash_mask)
  {
    std::vector<u8> small;
    EXPECT(build_quotient_filter_for_leaf(12, 9, items, small, 4096 - 64).ok());
    PackedVqfFilter h;
    std::memcpy(&h, small.data(), sizeof(h));
    EXPECT(h.hash_mask == (~u64{0} << 1));
    KeyQuery qt(items);
    std::vector<BoolStatus> rt;
    EXPECT(qt.reject_page(9, &small, FilterKind::kQuotient, rt).ok());
    size_t rejected = 0;
    for (auto v : rt) rejected += v == BoolStatus::kTrue;
    EXPECT(rejected == 0);
  }
  // KeyQuery::Metrics (tree/key_query.hpp:36-60)
  {
    auto& m = KeyQuery::metrics();
    const u64 t0 = m.total_filter_query_count.get(), r0 = m.filter_reject_count.get(),
              p0 = m.filter_positive_count.get(), f0 = m.filter_false_positive_count.get(),
              x0 = m.page_id_mismatch_count.get(), z0 = m.no_filter_page_count.get();
    std::vector<u8> truth(miss.size(), 0);
    EXPECT(qm.reject_page(7, &vqf_page, FilterKind::kQuotient, r, &truth).ok());
    size_t rej = 0;
    for (auto v : r) rej += v == BoolStatus::kTrue;
    EXPECT(qm.reject_page(8, &vqf_page, FilterKind::kQuotient, r).ok());
    EXPECT(qm.reject_page(7, nullptr, FilterKind::kQuotient, r).ok());
    EXPECT(m.total_filter_query_count.get() - t0 == 3 * miss.size());
    EXPECT(m.filter_reject_count.get() - r0 == rej);
    EXPECT(m.filter_positive_count.get() - p0 == miss.size() - rej);
    EXPECT(m.filter_false_positive_count.get() - f0 == miss.size() - rej);
    EXPECT(m.page_id_mismatch_count.get() - x0 == miss.size());
    EXPECT(m.no_filter_page_count.get() - z0 == miss.size());
    EXPECT(m.filter_false_positive_rate() > 0);
  }
  // whole filter pages (tkv_amq_plan_pages): header fields the builders set, then the payload
  {
    FilterBatchBuilder b = FilterBatchBuilder::pages(FilterKind::kQuotient, 12, 15);
    b.add_leaf(7, 4096);
    EXPECT(b.plan().ok() && b.total_out_bytes() == 32768);
    DeviceBuffer d_keys(4096 * 24), d_out(b.total_out_bytes());
    std::string blob;
    for (auto& k : keys) blob += k;
    (void)hipMemcpy(d_keys.get(), blob.data(), blob.size(), hipMemcpyHostToDevice);
    EXPECT(b.build_all(d_keys.get(), 24, nullptr, d_out.get()).ok());
    EXPECT(b.check().ok());
    std::vector<u8> page(32768);
    (void)hipMemcpy(page.data(), d_out.get(), page.size(), hipMemcpyDeviceToHost);
    EXPECT(std::memcmp(page.data() + 16, "vqf_filt", 8) == 0);
    u32 ub, ue, sz;
    std::memcpy(&ub, page.data() + 28, 4);
    std::memcpy(&ue, page.data() + 32, 4);
    std::memcpy(&sz, page.data() + 60, 4);
    EXPECT(ub == 64 + want_vqf.size() && ue == 32768 && sz == 32768);
    EXPECT(std::equal(want_vqf.begin(), want_vqf.end(), page.begin() + 64));
  }
  std::printf("%s (%d failures)\n", failures ? "FAIL" : "OK", failures);
  return failures ? 1 : 0;
}

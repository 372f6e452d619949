// ubench_valu.hip -- issue rates of the integer VALU ops the filter hashes use on gfx950
// (v_mul_lo_u32, v_mad_u64_u32, v_mul_hi_u32, v_mul_u32_u24, v_alignbit_b32, v_xor_b32,
// v_lshlrev_b64) and v_fma_f32 for comparison with the guide's 2-cycle figure
// (MI355X_MICROARCH.md:54).  Not part of the product; grounds the VALU roofline in DESIGN.md.
//
// Each op runs in 8 independent chains per wave, 8 waves per SIMD (8 workgroups of 4 waves per
// CU), back to back for >= 2 s so the chip holds its clock under load (MI355X_MICROARCH.md
// "DVFS give-back"); then one stamped launch: every workgroup records s_memtime (shader
// cycles) and s_memrealtime (100 MHz) around its loop.  Reported per op (median over
// workgroups): the in-kernel clock = d(memtime) / d(memrealtime) x 100 MHz, and cycles per
// wave-instruction per SIMD = d(memtime) / (8 waves x ITERS x CHAINS).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHAINS 8
#define ITERS 4096
constexpr int kWavesPerSimd = 8;

template <int OP, bool STAMP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint64_t* stamps, uint32_t seed)
{
  uint32_t v[CHAINS];
  uint64_t w[CHAINS];
  float f[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    v[c] = seed + threadIdx.x * 7 + c;
    w[c] = v[c];
    f[c] = (float)v[c] * 1e-9f;
  }
  const uint32_t k = 0x85EBCA87u ^ seed;
  const float fk = 1.0000001f;
  uint64_t t0 = 0, r0 = 0;
  if constexpr (STAMP) {
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "s"(k));
      if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[c]) : "s"(k));
      if constexpr (OP == 2) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(w[c]) : "v"(v[c]), "s"(k) : "s0", "s1");
      if constexpr (OP == 3) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(v[c]) : "s"(k));
      if constexpr (OP == 4) asm volatile("v_alignbit_b32 %0, %0, %1, 5" : "+v"(v[c]) : "v"(v[(c + 1) % CHAINS]));
      if constexpr (OP == 5) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[c]) : "s"(k));
      if constexpr (OP == 6) asm volatile("v_lshlrev_b64 %0, 5, %0" : "+v"(w[c]));
      if constexpr (OP == 7) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "s"(fk));
      if constexpr (OP == 8) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v[c]) : "s"(k));
    }
  }
  if constexpr (STAMP) {
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      stamps[2 * blockIdx.x] = t1 - t0;
      stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
    acc ^= v[c] ^ (uint32_t)w[c] ^ (uint32_t)(w[c] >> 32) ^ __float_as_uint(f[c]);
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int OP>
void run(const char* name, uint32_t* d, uint64_t* st, int n_cu, int wps = kWavesPerSimd)
{
  const int blocks = n_cu * wps;  // wps workgroups of 4 waves per CU: wps waves per SIMD
  // >= 2 s of back-to-back launches: the clock the chip holds under this load
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(2000);
  int launches = 0;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  while (std::chrono::steady_clock::now() < t_end) {
    for (int r = 0; r < 16; ++r) kern<OP, false><<<blocks, 256>>>(d, st, r);
    launches += 16;
    hipDeviceSynchronize();
  }
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  kern<OP, true><<<blocks, 256>>>(d, st, 7);
  hipDeviceSynchronize();
  std::vector<uint64_t> h(2 * blocks);
  hipMemcpy(h.data(), st, 16ull * blocks, hipMemcpyDeviceToHost);
  std::vector<double> cyc, clk;
  for (int i = 0; i < blocks; ++i) {
    cyc.push_back((double)h[2 * i]);
    clk.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 100e6);
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(clk.begin(), clk.end());
  const double cyc_med = cyc[blocks / 2], clk_med = clk[blocks / 2];
  // all wps waves of a SIMD are resident together (<= 8 workgroups of 4 waves per CU at a
  // few VGPRs), so the SIMD issued wps x ITERS x CHAINS instructions in the loop's cycles
  const double per_instr = cyc_med / ((double)wps * ITERS * CHAINS);
  // wall-clock rate of the back-to-back launches (includes launch gaps)
  const double wave_instrs = (double)launches * blocks * 4 * (double)ITERS * CHAINS;
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"clock_ghz_in_kernel\": %.3f, "
         "\"cycles_per_wave_instr_per_simd\": %.3f, \"wall_G_wave_instr_per_s\": %.1f, "
         "\"launches\": %d}\n",
         name, wps, clk_med / 1e9, per_instr, wave_instrs / (ms * 1e-3) / 1e9, launches);
  fflush(stdout);
}

int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d}\n", p.gcnArchName, n_cu);
  uint32_t* d;
  uint64_t* st;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&st, 16ull * n_cu * 8);
  // occupancy sweep: cycles per instruction per SIMD with 1, 2, 4, 8 waves per SIMD
  for (int wps : {1, 2, 4}) {
    run<5>("v_xor_b32", d, st, n_cu, wps);
    run<7>("v_fma_f32", d, st, n_cu, wps);
  }
  run<5>("v_xor_b32", d, st, n_cu);
  run<8>("v_add_u32", d, st, n_cu);
  run<4>("v_alignbit_b32", d, st, n_cu);
  run<3>("v_mul_u32_u24", d, st, n_cu);
  run<6>("v_lshlrev_b64", d, st, n_cu);
  run<0>("v_mul_lo_u32", d, st, n_cu);
  run<1>("v_mul_hi_u32", d, st, n_cu);
  run<2>("v_mad_u64_u32", d, st, n_cu);
  run<7>("v_fma_f32", d, st, n_cu);
  hipFree(d);
  hipFree(st);
  return 0;
}

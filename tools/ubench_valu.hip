// ubench_valu.hip -- measure issue rates of the integer VALU ops the filter hashes use on
// gfx950 (v_mul_lo_u32, v_mad_u64_u32, v_mul_hi_u32, v_mul_u32_u24, v_alignbit_b32,
// v_xor_b32).  Not part of the product; grounds the VALU roofline in DESIGN.md.
// Build: hipcc -O3 --offload-arch=gfx950 -o ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS 8
#define ITERS 2048

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed)
{
  uint32_t v[CHAINS];
  uint64_t w[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    v[c] = seed + threadIdx.x * 7 + c;
    w[c] = v[c];
  }
  const uint32_t k = 0x85EBCA87u ^ seed;
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
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc ^= v[c] ^ (uint32_t)w[c] ^ (uint32_t)(w[c] >> 32);
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int OP>
double run(const char* name, uint32_t* d)
{
  const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU: 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<OP><<<blocks, 256>>>(d, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) kern<OP><<<blocks, 256>>>(d, r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double wave_instrs = 5.0 * blocks * 4 * (double)ITERS * CHAINS;
  const double per_simd = wave_instrs / 1024.0;
  // cycles per wave-instruction per SIMD at 2.4 GHz
  const double cyc = ms * 1e-3 * 2.4e9 / per_simd;
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_instr_per_simd_at_2.4GHz\": %.2f, "
         "\"Gops_per_s\": %.1f}\n",
         name, ms, cyc, wave_instrs * 64 / (ms * 1e-3) / 1e9);
  return cyc;
}

int main()
{
  uint32_t* d;
  hipMalloc(&d, 1 << 20);
  run<0>("v_mul_lo_u32", d);
  run<1>("v_mul_hi_u32", d);
  run<2>("v_mad_u64_u32", d);
  run<3>("v_mul_u32_u24", d);
  run<4>("v_alignbit_b32", d);
  run<5>("v_xor_b32", d);
  run<6>("v_lshlrev_b64", d);
  hipFree(d);
  return 0;
}

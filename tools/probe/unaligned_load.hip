// Checks that unaligned 8- and 4-byte global loads (what __builtin_memcpy from a byte
// pointer compiles to on gfx950) return the right bytes at every byte offset.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k(const uint8_t* __restrict__ p, uint64_t* out8, uint32_t* out4)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // byte offset
  uint64_t v;
  uint32_t w;
  __builtin_memcpy(&v, p + i, 8);
  __builtin_memcpy(&w, p + i + 8, 4);
  out8[i] = v;
  out4[i] = w;
}

int main()
{
  const int n = 4096;
  uint8_t h[n + 16];
  for (int i = 0; i < n + 16; ++i) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t* d;
  uint64_t* o8;
  uint32_t* o4;
  if (hipMalloc(&d, n + 16) || hipMalloc(&o8, 8 * n) || hipMalloc(&o4, 4 * n)) return 2;
  hipMemcpy(d, h, n + 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, o8, o4);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
  uint64_t r8[n];
  uint32_t r4[n];
  hipMemcpy(r8, o8, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(r4, o4, 4 * n, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t e8 = 0;
    uint32_t e4 = 0;
    for (int b = 0; b < 8; ++b) e8 |= (uint64_t)h[i + b] << (8 * b);
    for (int b = 0; b < 4; ++b) e4 |= (uint32_t)h[i + 8 + b] << (8 * b);
    bad += (r8[i] != e8) + (r4[i] != e4);
  }
  printf("%s: %d mismatches over %d byte offsets\n", bad ? "FAIL" : "OK", bad, n);
  return bad ? 1 : 0;
}

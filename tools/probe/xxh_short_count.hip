// ISA-level VALU count of the short-key XXH64 (XxhShort, csrc/tkv_amq_device.h) that the
// variable-length VQF key path runs: one runtime-length kernel (what a
// wave of mixed lengths executes: every lane round, the 4-byte step and every byte step,
// predicated) against one kernel per compile-time length (what a perfectly length-grouped wave
// would execute).  Compile only, count the v_ instructions of each body:
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only tools/probe/xxh_short_count.hip \
//     -Iturtle_kv_amd/csrc -o /tmp/xxh_short.s && python3 tools/probe/count_valu.py /tmp/xxh_short.s
#include <hip/hip_runtime.h>

#include "tkv_amq_device.h"

using namespace tkv;

constexpr uint64_t kSeedP5 = 0x9d0924dc03e79a75ull + kP5;

// the key as the VQF producers load it: the lanes, the 4-byte tail and the tail bytes
struct Win {
  uint64_t l[3];
  uint32_t t4, tb;
};

__device__ inline Win load_win(const uint64_t* w, uint32_t i)
{
  Win v;
  v.l[0] = w[4 * i];
  v.l[1] = w[4 * i + 1];
  v.l[2] = w[4 * i + 2];
  v.t4 = (uint32_t)w[4 * i + 3];
  v.tb = (uint32_t)(w[4 * i + 3] >> 32);
  return v;
}

extern "C" __global__ void xxh_short_var(const uint64_t* w, const uint32_t* lens, uint64_t* out)
{
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const Win v = load_win(w, i);
  out[i] = XxhShort(lens[i], v.l, v.t4, v.tb).finish(kSeedP5);
}

template <uint32_t N>
__global__ void xxh_short_len(const uint64_t* w, uint64_t* out)
{
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const Win v = load_win(w, i);
  out[i] = XxhShort(N, v.l, v.t4, v.tb).finish(kSeedP5);
}

#define L(n) template __global__ void xxh_short_len<n>(const uint64_t*, uint64_t*);
L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23)
L(24) L(25) L(26) L(27) L(28) L(29) L(30) L(31)

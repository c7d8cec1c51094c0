// ubench_gups2.hip — why C4's PolyRand update stream runs 12x below random
// atomicXor on the same 2^30-word table. Each variant
// does 1M streamers x 16 no-return 64-bit atomicXor per launch, table = 8
// updaters x 2^27 words, field-major (word * 8 + updater), as the engine's
// gups Updater state (engine_dev.h send_updater):
//   poly      the engine's stream: streamer i at PolyRand position i * 128
//   poly_rs   the same stream, streamers seeded at random positions
//   poly_perm the engine's streams, lanes dealt streamers i * 4099 mod 2^20
//   poly_mul  the engine's stream, word index scrambled by an odd multiplier
//             mod 2^27 (a bijection of the updater's fields)
//   poly_xsh  the engine's stream, word index ^= (word >> 13) * 0x5bd1 (bijection)
//   poly_rot  the engine's stream, word index rotated right by 9 within 27 bits
//   poly_fei  the engine's stream, word index through two Feistel rounds
//   poly_hash the engine's stream, word = splitmix(d) (not a bijection)
//   poly_u0   the engine's stream, every update to updater 0
//   rand      xorshift64 data, same launch shape
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_gups2 scripts/ubench_gups2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../ponyc_amd/csrc/rng_dev.h"

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

constexpr uint32_t kN = 1u << 20, kPer = 16;
constexpr uint64_t kSize = 1ull << 27;       // words per updater
constexpr uint32_t kShift = 28;              // size.bit_length()

__global__ void k_seed(uint64_t* st, uint64_t stride, int mode)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if(i >= kN) return;
  uint64_t pos = stride * i;
  if(mode == 1) pos = gpa::splitmix_mix(i) >> 8;                       // random positions
  if(mode == 2) pos = stride * ((uint64_t)i * 4099u % kN);             // lanes dealt apart
  st[i] = gpa::polyrand_seeded(pos);
}

template <int MODE>
__device__ __forceinline__ uint64_t word_of(uint64_t d)
{
  uint64_t w = d & (kSize - 1);
  if constexpr(MODE == 1) w = (w * 0x2545F49ull) & (kSize - 1);
  if constexpr(MODE == 2) w ^= ((w >> 13) * 0x5bd1ull) & 0x1FFFull;
  if constexpr(MODE == 3) w = ((w >> 9) | (w << 18)) & (kSize - 1);
  if constexpr(MODE == 4)
  {
    // two Feistel rounds over (13, 14)-bit halves with a multiplicative hash
    uint32_t hi = (uint32_t)(w >> 14), lo = (uint32_t)w & 0x3FFFu;
    lo ^= ((hi * 0x9E3779B1u) >> 18) & 0x3FFFu;
    hi ^= ((lo * 0x85EBCA77u) >> 19) & 0x1FFFu;
    w = ((uint64_t)hi << 14) | lo;
  }
  if constexpr(MODE == 5) w = gpa::splitmix_mix(d) & (kSize - 1);     // not a bijection: address study only
  return w;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_poly(unsigned long long* t, uint64_t* st)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if(i >= kN) return;
  uint64_t last = st[i];
  for(uint32_t k = 0; k < kPer; ++k)
  {
    const uint64_t d = gpa::polyrand_next(last);
    const uint64_t u = MODE == 6 ? 0 : (d >> kShift) & 7;
    atomicXor(&t[word_of<MODE>(d) * 8 + u], (unsigned long long)d);
  }
  st[i] = last;
}

__global__ void __launch_bounds__(256) k_rand(unsigned long long* t, uint64_t* st)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if(i >= kN) return;
  uint64_t x = st[i] | 1;
  for(uint32_t k = 0; k < kPer; ++k)
  {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    atomicXor(&t[x & (kSize * 8 - 1)], (unsigned long long)x);
  }
  st[i] = x;
}

template <class F>
static void time_it(const char* name, F launch, uint64_t* st, int seed_mode)
{
  hipLaunchKernelGGL(k_seed, dim3(kN / 256), dim3(256), 0, 0, st, (uint64_t)128, seed_mode);
  launch();                                           // warm
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for(int r = 0; r < 8; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("%-10s %7.2f G updates/s  %.3f ms/launch\n", name, 8.0 * kN * kPer / (ms * 1e-3) / 1e9, ms / 8);
  fflush(stdout);
}

int main(int argc, char** argv)
{
  unsigned long long* t; uint64_t* st;
  CK(hipMalloc(&t, kSize * 8 * 8));
  CK(hipMalloc(&st, kN * 8ull));
  CK(hipMemset(t, 0, kSize * 8 * 8));
  const dim3 g(kN / 256), b(256);
  time_it("poly", [&] { hipLaunchKernelGGL(k_poly<0>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_rs", [&] { hipLaunchKernelGGL(k_poly<0>, g, b, 0, 0, t, st); }, st, 1);
  time_it("poly_perm", [&] { hipLaunchKernelGGL(k_poly<0>, g, b, 0, 0, t, st); }, st, 2);
  time_it("poly_mul", [&] { hipLaunchKernelGGL(k_poly<1>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_xsh", [&] { hipLaunchKernelGGL(k_poly<2>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_rot", [&] { hipLaunchKernelGGL(k_poly<3>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_fei", [&] { hipLaunchKernelGGL(k_poly<4>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_hash", [&] { hipLaunchKernelGGL(k_poly<5>, g, b, 0, 0, t, st); }, st, 0);
  time_it("poly_u0", [&] { hipLaunchKernelGGL(k_poly<6>, g, b, 0, 0, t, st); }, st, 0);
  time_it("rand", [&] { hipLaunchKernelGGL(k_rand, g, b, 0, 0, t, st); }, st, 1);
  CK(hipFree(t)); CK(hipFree(st));
  return 0;
}

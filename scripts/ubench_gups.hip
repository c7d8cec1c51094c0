// ubench_gups.hip — the ceiling for C4 (gups): random 64-bit atomicXor (no
// return) over a table of 2^L u64 words, the device op a gups Updater apply
// becomes (engine_dev.h: send_updater). Reports G updates/s for several table
// sizes, so the engine's C4 rate can be read against the same access pattern.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_gups scripts/ubench_gups.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "../ponyc_amd/csrc/rng_dev.h"

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

__global__ void k_gups(unsigned long long* t, uint64_t mask, uint32_t per, uint64_t seed)
{
  uint64_t x = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B97F4A7C15ull);
  for(uint32_t k = 0; k < per; ++k)
  {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;           // xorshift64
    atomicXor(&t[x & mask], (unsigned long long)x);
  }
}

// The engine's C4 access pattern: streamer i = PolyRand jumped to i * stride
// (gups_basic/main.pony:93-143), update d goes to updater (d >> shift) & 7,
// word d & (size - 1), state field-major (word * 8 + updater).
__global__ void k_seed(uint64_t* st, uint32_t n, uint64_t stride)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if(i < n) st[i] = gpa::polyrand_seeded(stride * i);
}

__global__ void k_gups_poly(unsigned long long* t, uint64_t* st, uint32_t n, uint32_t per,
  uint64_t size_mask, uint32_t shift)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if(i >= n) return;
  uint64_t last = st[i];
  for(uint32_t k = 0; k < per; ++k)
  {
    const uint64_t d = gpa::polyrand_next(last);
    const uint64_t u = (d >> shift) & 7;
    atomicXor(&t[(d & size_mask) * 8 + u], (unsigned long long)d);
  }
  st[i] = last;
}

int main()
{
  {
    // 2^30-word table as 8 updaters of 2^27; 1M streamers x 16 updates, stride 128
    const uint32_t n = 1u << 20, per = 16;
    const uint64_t size = 1ull << 27;
    unsigned long long* t; uint64_t* st;
    CK(hipMalloc(&t, size * 8 * 8));
    CK(hipMalloc(&st, n * 8ull));
    CK(hipMemset(t, 0, size * 8 * 8));
    k_seed<<<n / 256, 256>>>(st, n, 128);
    k_gups_poly<<<n / 256, 256>>>(t, st, n, per, size - 1, 28);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for(int r = 0; r < 4; ++r) k_gups_poly<<<n / 256, 256>>>(t, st, n, per, size - 1, 28);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("PolyRand streams (engine C4 pattern, 1M x 16 per launch): %7.2f G updates/s, %.3f ms/launch\n",
      4.0 * n * per / (ms * 1e-3) / 1e9, ms / 4);
    CK(hipFree(t)); CK(hipFree(st));
  }
  const uint32_t threads = 256, blocks = 8192, per = 64;    // 134M updates per launch
  const double ups = (double)threads * blocks * per;
  for(int L = 20; L <= 30; L += 2)
  {
    const size_t words = (size_t)1 << L;
    unsigned long long* t;
    CK(hipMalloc(&t, words * 8));
    CK(hipMemset(t, 0, words * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    k_gups<<<blocks, threads>>>(t, words - 1, per, 1);     // warm (TLB, caches)
    CK(hipEventRecord(a));
    for(int r = 0; r < 3; ++r) k_gups<<<blocks, threads>>>(t, words - 1, per, 2 + r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("table 2^%d u64 (%8.1f MB): %7.2f G updates/s\n", L, words * 8 / 1e6,
      3 * ups / (ms * 1e-3) / 1e9);
    CK(hipFree(t));
  }
  return 0;
}

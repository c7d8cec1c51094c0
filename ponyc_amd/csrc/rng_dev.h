// rng_dev.h — device restatements of the workload RNGs the handler tables draw
// from (packages/random: xoroshiro.pony:1-42, random.pony:143-193,
// splitmix64.pony; PolyRand: examples/gups_basic/main.pony:167-216).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

namespace gpa {

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// XorOshiro128Plus.next — state kept in two registers.
__device__ __forceinline__ uint64_t xoro_next(uint64_t& x0, uint64_t& y0)
{
  const uint64_t x = x0;
  uint64_t y = y0;
  const uint64_t r = x + y;
  y ^= x;
  x0 = rotl64(x, 24) ^ y ^ (y << 16);
  y0 = rotl64(y, 37);
  return r;
}

__device__ __forceinline__ void xoro_create(uint64_t& x, uint64_t& y, uint64_t sx, uint64_t sy)
{
  x = sx;
  y = sy;
  (void)xoro_next(x, y);
}

// Random.int(n) on native128: high half of next() * n.
__device__ __forceinline__ uint64_t rand_int(uint64_t& x, uint64_t& y, uint64_t n)
{
  return mulhi64(xoro_next(x, y), n);
}

// Random._u64_unbiased(range) (Lemire).
__device__ __forceinline__ uint64_t rand_int_unbiased(uint64_t& x, uint64_t& y, uint64_t range)
{
  uint64_t v = xoro_next(x, y);
  uint64_t hi = mulhi64(v, range);
  uint64_t lo = v * range;
  if(lo < range)
  {
    uint64_t t = (uint64_t)0 - range;
    if(t >= range)
    {
      t -= range;
      if(t >= range)
        t %= range;
    }
    while(lo < t)
    {
      v = xoro_next(x, y);
      hi = mulhi64(v, range);
      lo = v * range;
    }
  }
  return hi;
}

__device__ __forceinline__ uint64_t splitmix_mix(uint64_t s)
{
  uint64_t z = s + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t polyrand_next(uint64_t& last)
{
  const uint64_t l = last;
  last = (l << 1) ^ ((int64_t)l < 0 ? 7ULL : 0ULL);
  return last;
}

// PolyRand's step is a product by x in GF(2)[x] / (x^64 + x^2 + x + 1), so n
// steps are one product by x^n: a * b mod that polynomial, b's bits high to
// low (the jump-ahead _seed makes through its squaring table, exact here in
// all 64 bits).
__host__ __device__ inline uint64_t polyrand_mulmod(uint64_t a, uint64_t b)
{
  uint64_t r = 0;
  for(int i = 63; i >= 0; --i)
  {
    r = (r << 1) ^ ((int64_t)r < 0 ? 7ULL : 0ULL);
    if((b >> i) & 1) r ^= a;
  }
  return r;
}

// x^n mod the PolyRand polynomial (square and multiply)
__host__ __device__ inline uint64_t polyrand_xpow(uint64_t n)
{
  uint64_t r = 1, b = 2;
  while(n)
  {
    if(n & 1) r = polyrand_mulmod(r, b);
    b = polyrand_mulmod(b, b);
    n >>= 1;
  }
  return r;
}

// PolyRand._seed: x^n style jump through the squaring table m2 (63 entries;
// the reference's m2(63) read is out of bounds and skipped inside `try`).
__device__ inline uint64_t polyrand_seeded(uint64_t seed)
{
  const uint64_t period = 1317624576693539401ULL;
  const uint64_t n = seed % period;
  if(n == 0)
    return 1;
  uint64_t m2[63];
  uint64_t last = 1;
#pragma unroll
  for(int i = 0; i < 63; i++)
  {
    m2[i] = last;
    (void)polyrand_next(last);
    (void)polyrand_next(last);
  }
  uint64_t i = 64 - (uint64_t)__clzll((long long)n);
  last = 2;
  while(i > 0)
  {
    uint64_t temp = 0;
#pragma unroll
    for(int j = 0; j < 63; j++)
      temp ^= ((last >> j) & 1) ? m2[j] : 0ULL;
    last = temp;
    i -= 1;
    if((n >> i) & 1)
      (void)polyrand_next(last);
  }
  return last;
}

} // namespace gpa

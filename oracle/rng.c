/*
 * rng.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the workload RNGs.
 * Pinned by tests/test_oracle_rng.py against the reference KATs in
 * packages/random/_test.pony (xoroshiro128+ seed 5489: 473-493; SplitMix64
 * seed 5489: 359-).
 */
#include "oracle.h"

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* Random.int on native128: ((next().u128() * n.u128()) >> 64) (random.pony:143-156) */
uint64_t or_mulhi(uint64_t a, uint64_t b)
{
  return (uint64_t)(((unsigned __int128)a * (unsigned __int128)b) >> 64);
}

/* XorOshiro128Plus.next (xoroshiro.pony:31-42) */
uint64_t or_xoro_next(or_xoro_t* r)
{
  uint64_t x = r->x;
  uint64_t y = r->y;
  uint64_t res = x + y;
  y = x ^ y;
  r->x = rotl64(x, 24) ^ y ^ (y << 16);
  r->y = rotl64(y, 37);
  return res;
}

/* XorOshiro128Plus.create(x, y): store, then next() once (xoroshiro.pony:22-29) */
void or_xoro_create(or_xoro_t* r, uint64_t x, uint64_t y)
{
  r->x = x;
  r->y = y;
  (void)or_xoro_next(r);
}

uint64_t or_rand_int(or_xoro_t* r, uint64_t n)
{
  return or_mulhi(or_xoro_next(r), n);
}

/* Random._u64_unbiased (random.pony:168-193), Lemire's nearly-divisionless. */
uint64_t or_rand_int_unbiased(or_xoro_t* r, uint64_t range)
{
  uint64_t x = or_xoro_next(r);
  unsigned __int128 m = (unsigned __int128)x * range;
  uint64_t l = (uint64_t)m;
  if(l < range)
  {
    uint64_t t = (uint64_t)0 - range;
    if(t >= range)
    {
      t -= range;
      if(t >= range)
        t = t % range;
    }
    while(l < t)
    {
      x = or_xoro_next(r);        /* u64() == next() for XorOshiro128Plus */
      m = (unsigned __int128)x * range;
      l = (uint64_t)m;
    }
  }
  return (uint64_t)(m >> 64);
}

/* SplitMix64.next (splitmix64.pony) */
uint64_t or_splitmix_next(uint64_t* s)
{
  *s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = *s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

uint64_t or_splitmix_mix(uint64_t x)
{
  uint64_t s = x;
  return or_splitmix_next(&s);
}

/* PolyRand.apply (gups_basic/main.pony:180-182): the condition reads the old
 * value of `last`. */
uint64_t or_polyrand_next(or_polyrand_t* r)
{
  uint64_t last = r->last;
  r->last = (last << 1) ^ ((last & (1ULL << 63)) != 0 ? 7ULL : 0ULL);
  return r->last;
}

static inline int clz64(uint64_t n) { return n == 0 ? 64 : __builtin_clzll(n); }

/* PolyRand.create/_seed (gups_basic/main.pony:173-216), restated literally:
 * m2 holds 63 entries (Range(0, 63)); the j loop runs to 63 and the
 * out-of-bounds m2(63)? read raises inside `try`, so bit 63 contributes
 * nothing. i starts at 64 - clz(n). */
void or_polyrand_create(or_polyrand_t* r, uint64_t seed)
{
  const uint64_t period = 1317624576693539401ULL;
  uint64_t n = seed % period;
  r->last = 1;
  if(n == 0)
    return;

  uint64_t m2[63];
  r->last = 1;
  for(int i = 0; i < 63; i++)
  {
    m2[i] = r->last;
    (void)or_polyrand_next(r);
    (void)or_polyrand_next(r);
  }

  uint64_t i = (uint64_t)(64 - clz64(n));
  r->last = 2;
  while(i > 0)
  {
    uint64_t temp = 0;
    for(int j = 0; j < 64; j++)
    {
      if(((r->last >> j) & 1) != 0 && j < 63)
        temp ^= m2[j];
    }
    r->last = temp;
    i = i - 1;
    if(((n >> i) & 1) != 0)
      (void)or_polyrand_next(r);
  }
}

/* XOR of every datum a gups_basic run streams (main.pony:67-68, 93-143):
 * streamer i is seeded PolyRand(chunk * iterate * i) and produces
 * chunk * (iterate + 1) values (apply(iterate) down to apply(0)); each value d
 * does t[d & (size-1)] ^= d at its updater (main.pony:157-161), so the XOR of
 * the whole table moves by the XOR of all of them. PolyRand's step is linear
 * over GF(2), so the XOR over streamers of their k-th values is the k-th value
 * of the XOR of their seeds: one stream of chunk * (iterate + 1) steps. */
uint64_t or_gups_update_xor(uint64_t streamers, uint64_t chunk, uint64_t iterate)
{
  uint64_t x = 0;
  for(uint64_t i = 0; i < streamers; i++)
  {
    or_polyrand_t r;
    or_polyrand_create(&r, chunk * iterate * i);
    x ^= r.last;
  }
  or_polyrand_t s = { x };
  uint64_t acc = 0;
  const uint64_t m = chunk * (iterate + 1);
  for(uint64_t k = 0; k < m; k++)
    acc ^= or_polyrand_next(&s);
  return acc;
}

/* The same XOR with every stream stepped one value at a time (small sizes:
 * pins the linearity argument above). */
uint64_t or_gups_update_xor_literal(uint64_t streamers, uint64_t chunk, uint64_t iterate)
{
  uint64_t acc = 0;
  const uint64_t m = chunk * (iterate + 1);
  for(uint64_t i = 0; i < streamers; i++)
  {
    or_polyrand_t r;
    or_polyrand_create(&r, chunk * iterate * i);
    for(uint64_t k = 0; k < m; k++)
      acc ^= or_polyrand_next(&r);
  }
  return acc;
}

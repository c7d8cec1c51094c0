// ubench_plan.hip — can k_step drop its HBM outbox? The data movement of one C2
// superstep's sends (MI355X), with destinations made on the fly (a hash, as a
// handler computes them) and every chunk position planned ahead (no
// reservation atomics in any variant, so only the staging differs):
//
//   outbox  — today's k_step: sends appended to the zone's outbox O in HBM,
//             read back in 4096-record tiles, counting-sorted by destination
//             zone in LDS, stored in runs (~8) at their chunk positions;
//   lds2    — 2 workgroups of 512 per CU: the zone's actors drained in rounds
//             of 512 (one per thread); a round's ~2560 sends are staged in
//             LDS (40 KB), sorted there, and stored in runs (~5) at the
//             zone's planned chunk for each destination (cursor per bucket);
//   lds1    — 1 workgroup of 1024 per CU: rounds of 1024 actors, ~5120 sends
//             (80 KB) staged per round, runs ~10;
//   direct  — each send stored at its planned position as it is made.
// State: 3 words per actor read and written, field-major, as the pinger's.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_plan scripts/ubench_plan.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

constexpr uint32_t NZ = 512, ACT = 2048, SENDS = 5, PER = ACT * SENDS, TILE = 4096;
constexpr uint32_t REGION = 16384;          // landing records per destination zone

__host__ __device__ inline uint32_t dest(uint32_t z, uint32_t a, uint32_t j)
{
  uint32_t h = (z * 2048u + a) * 5u + j;
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h % NZ;
}

__device__ __forceinline__ void state_rw(uint64_t* st, uint32_t a)
{
  uint64_t x = st[a], y = st[(size_t)NZ * ACT + a], c = st[2 * (size_t)NZ * ACT + a];
  x ^= y; c += SENDS;
  st[a] = x; st[(size_t)NZ * ACT + a] = y; st[2 * (size_t)NZ * ACT + a] = c;
}

// exclusive scan of the NZ bucket counts by wave 0 (the caller synchronises)
__device__ __forceinline__ void scan_nz(const uint32_t* s_cnt, uint32_t* s_st)
{
  const uint32_t tid = threadIdx.x;
  if(tid >= 64) return;
  uint32_t v[NZ / 64], sum = 0;
#pragma unroll
  for(uint32_t k = 0; k < NZ / 64; ++k) { v[k] = s_cnt[tid * (NZ / 64) + k]; sum += v[k]; }
  uint32_t incl = sum;
#pragma unroll
  for(int off = 1; off < 64; off <<= 1)
  {
    const uint32_t u = __shfl_up(incl, off);
    if(tid >= (uint32_t)off) incl += u;
  }
  uint32_t run = incl - sum;
#pragma unroll
  for(uint32_t k = 0; k < NZ / 64; ++k) { s_st[tid * (NZ / 64) + k] = run; run += v[k]; }
}

// base[z * NZ + b]: planned chunk start of (source zone z, destination b)
template <uint32_t T>
__global__ void __launch_bounds__(T) k_outbox(uint64_t* st, uint4* O, const uint32_t* base, uint4* land)
{
  __shared__ uint4 s_tile[TILE];
  __shared__ uint32_t s_cur[NZ], s_cnt[NZ], s_st[NZ];
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  __shared__ uint32_t s_n;
  if(tid == 0) s_n = 0;
  for(uint32_t b = tid; b < NZ; b += T) { s_cur[b] = base[z * NZ + b]; s_cnt[b] = 0; }
  __syncthreads();
  uint4* Oz = O + (size_t)z * PER;
  for(uint32_t a = tid; a < ACT; a += T)
  {
    state_rw(st, z * ACT + a);
    for(uint32_t j = 0; j < SENDS; ++j)
    {
      const uint32_t i = atomicAdd(&s_n, 1u);
      Oz[i] = uint4{dest(z, a, j), a, 42u, j};
    }
  }
  __syncthreads();
  constexpr uint32_t P = TILE / T;
  for(uint32_t t0 = 0; t0 < PER; t0 += TILE)
  {
    const uint32_t m = min(TILE, PER - t0);
    uint4 r[P];
    uint32_t rk[P];
#pragma unroll
    for(uint32_t u = 0; u < P; ++u) r[u] = Oz[t0 + min(u * T + tid, m - 1)];
#pragma unroll
    for(uint32_t u = 0; u < P; ++u)
      if(u * T + tid < m) rk[u] = atomicAdd(&s_cnt[r[u].x], 1u);
    __syncthreads();
    scan_nz(s_cnt, s_st);
    __syncthreads();
#pragma unroll
    for(uint32_t u = 0; u < P; ++u)
      if(u * T + tid < m) s_tile[s_st[r[u].x] + rk[u]] = r[u];
    __syncthreads();
    for(uint32_t p = tid; p < m; p += T)
    {
      const uint4 v = s_tile[p];
      land[(size_t)v.x * REGION + s_cur[v.x] + (p - s_st[v.x])] = v;
    }
    __syncthreads();
    for(uint32_t b = tid; b < NZ; b += T) { s_cur[b] += s_cnt[b]; s_cnt[b] = 0; }
    __syncthreads();
  }
}

// rounds of T actors; each round's sends staged in LDS, sorted, stored
template <uint32_t T>
__global__ void __launch_bounds__(T) k_lds(uint64_t* st, const uint32_t* base, uint4* land)
{
  constexpr uint32_t RT = T * SENDS;         // sends per round
  __shared__ uint4 s_tile[RT];
  __shared__ uint16_t s_idx[RT];
  __shared__ uint32_t s_cur[NZ], s_cnt[NZ], s_st[NZ];
  __shared__ uint32_t s_n;
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  for(uint32_t b = tid; b < NZ; b += T) { s_cur[b] = base[z * NZ + b]; s_cnt[b] = 0; }
  if(tid == 0) s_n = 0;
  __syncthreads();
  for(uint32_t a0 = 0; a0 < ACT; a0 += T)
  {
    const uint32_t a = a0 + tid;
    state_rw(st, z * ACT + a);
    uint32_t slot[SENDS], rk[SENDS], bk[SENDS];
#pragma unroll
    for(uint32_t j = 0; j < SENDS; ++j)
    {
      bk[j] = dest(z, a, j);
      slot[j] = atomicAdd(&s_n, 1u);
      rk[j] = atomicAdd(&s_cnt[bk[j]], 1u);
      s_tile[slot[j]] = uint4{bk[j], a, 42u, j};
    }
    __syncthreads();
    scan_nz(s_cnt, s_st);
    __syncthreads();
#pragma unroll
    for(uint32_t j = 0; j < SENDS; ++j) s_idx[s_st[bk[j]] + rk[j]] = (uint16_t)slot[j];
    __syncthreads();
    const uint32_t m = s_n;
    for(uint32_t p = tid; p < m; p += T)
    {
      const uint4 v = s_tile[s_idx[p]];
      land[(size_t)v.x * REGION + s_cur[v.x] + (p - s_st[v.x])] = v;
    }
    __syncthreads();
    for(uint32_t b = tid; b < NZ; b += T) { s_cur[b] += s_cnt[b]; s_cnt[b] = 0; }
    if(tid == 0) s_n = 0;
    __syncthreads();
  }
}

template <uint32_t T>
__global__ void __launch_bounds__(T) k_direct(uint64_t* st, const uint32_t* base, uint4* land)
{
  __shared__ uint32_t s_cur[NZ];
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  for(uint32_t b = tid; b < NZ; b += T) s_cur[b] = base[z * NZ + b];
  __syncthreads();
  for(uint32_t a = tid; a < ACT; a += T)
  {
    state_rw(st, z * ACT + a);
#pragma unroll
    for(uint32_t j = 0; j < SENDS; ++j)
    {
      const uint32_t b = dest(z, a, j);
      const uint32_t pos = atomicAdd(&s_cur[b], 1u);
      land[(size_t)b * REGION + pos] = uint4{b, a, 42u, j};
    }
  }
}

int main()
{
  // plan: every (source, destination) chunk sized exactly, packed per destination
  std::vector<uint32_t> cnt((size_t)NZ * NZ, 0), base((size_t)NZ * NZ);
  for(uint32_t z = 0; z < NZ; ++z)
    for(uint32_t a = 0; a < ACT; ++a)
      for(uint32_t j = 0; j < SENDS; ++j) cnt[(size_t)z * NZ + dest(z, a, j)]++;
  for(uint32_t b = 0; b < NZ; ++b)
  {
    uint32_t acc = 0;
    for(uint32_t z = 0; z < NZ; ++z) { base[(size_t)z * NZ + b] = acc; acc += cnt[(size_t)z * NZ + b]; }
    if(acc > REGION) { printf("region overflow\n"); return 1; }
  }
  uint64_t* st;
  uint4 *O, *land;
  uint32_t* d_base;
  CK(hipMalloc(&st, 3 * (size_t)NZ * ACT * 8));
  CK(hipMalloc(&O, (size_t)NZ * PER * 16));
  CK(hipMalloc(&land, (size_t)NZ * REGION * 16));
  CK(hipMalloc(&d_base, base.size() * 4));
  CK(hipMemcpy(d_base, base.data(), base.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(st, 1, 3 * (size_t)NZ * ACT * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto check = [&](const char* name) {
    // every landed record at its place: each destination region holds exactly
    // its records (the x field is the destination)
    std::vector<uint4> h((size_t)NZ * REGION);
    CK(hipMemcpy(h.data(), land, h.size() * 16, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for(uint32_t b = 0; b < NZ; ++b)
    {
      uint32_t tot = 0;
      for(uint32_t z = 0; z < NZ; ++z) tot += cnt[(size_t)z * NZ + b];
      for(uint32_t i = 0; i < tot; ++i) if(h[(size_t)b * REGION + i].x != b) ++bad;
    }
    printf("  %s: %zu misplaced\n", name, bad);
    CK(hipMemset(land, 0xFF, (size_t)NZ * REGION * 16));
  };
  auto timeit = [&](const char* name, auto launch) {
    CK(hipMemset(land, 0xFF, (size_t)NZ * REGION * 16));
    launch();
    CK(hipDeviceSynchronize());
    check(name);
    float best = 1e30f, sum = 0;
    for(int rep = 0; rep < 20; ++rep)
    {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      sum += ms;
    }
    printf("%-58s best %8.4f ms  mean %8.4f ms\n", name, best, sum / 20);
  };
  timeit("outbox (O in HBM, tile 4096, 2x512/CU)", [&] {
    hipLaunchKernelGGL(k_outbox<512>, dim3(NZ), dim3(512), 0, 0, st, O, d_base, land); });
  timeit("lds2 (rounds of 512 staged in LDS, 2x512/CU)", [&] {
    hipLaunchKernelGGL(k_lds<512>, dim3(NZ), dim3(512), 0, 0, st, d_base, land); });
  timeit("lds1 (rounds of 1024 staged in LDS, 1x1024/CU)", [&] {
    hipLaunchKernelGGL(k_lds<1024>, dim3(NZ), dim3(1024), 0, 0, st, d_base, land); });
  timeit("direct (stored as made, 2x512/CU)", [&] {
    hipLaunchKernelGGL(k_direct<512>, dim3(NZ), dim3(512), 0, 0, st, d_base, land); });
  timeit("direct (stored as made, 1x1024/CU)", [&] {
    hipLaunchKernelGGL(k_direct<1024>, dim3(NZ), dim3(1024), 0, 0, st, d_base, land); });
  return 0;
}

// ubench_scatter.hip — the outbox scatter of k_step in isolation (MI355X):
// 512 source zones x 10240 records of 16 B, each to one of 512 destination
// zones (uniform), landing in one contiguous chunk per (source, destination)
// pair (~20 records). Measures the store side for two record orders:
//   random  — outbox order (what the scatter phase writes today)
//   sorted  — records grouped by destination (consecutive lanes, consecutive
//             addresses within a chunk)
// plus a coalesced 16-B copy of the same bytes as the reference.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_scatter scripts/ubench_scatter.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

constexpr uint32_t NZ = 512, PER = 10240, REGION = 32768, THREADS = 512;

__global__ void __launch_bounds__(THREADS) k_scatter(const uint4* __restrict__ src,
  const uint32_t* __restrict__ pos, uint4* __restrict__ dst)
{
  const uint32_t base = blockIdx.x * PER;
  for(uint32_t i = threadIdx.x; i < PER; i += THREADS * 4)
  {
    uint4 r[4];
    uint32_t p[4];
#pragma unroll
    for(int u = 0; u < 4; ++u)
    {
      const uint32_t j = i + u * THREADS;
      if(j < PER) { r[u] = src[base + j]; p[u] = pos[base + j]; }
    }
#pragma unroll
    for(int u = 0; u < 4; ++u)
      if(i + u * THREADS < PER) dst[p[u]] = r[u];
  }
}

__global__ void __launch_bounds__(THREADS) k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst)
{
  const uint32_t base = blockIdx.x * PER;
  for(uint32_t i = threadIdx.x; i < PER; i += THREADS) dst[(size_t)blockIdx.x * REGION + i] = src[base + i];
}

// read-only pass over the source records (coalesced), folded into a sink
__global__ void __launch_bounds__(THREADS) k_read(const uint4* __restrict__ src, uint32_t* sink)
{
  const uint32_t base = blockIdx.x * PER;
  uint32_t acc = 0;
  for(uint32_t i = threadIdx.x; i < PER; i += THREADS) { const uint4 v = src[base + i]; acc ^= v.x ^ v.w; }
  if(acc == 0x12345678u) sink[0] = acc;
}

// gather: record i of the zone's output comes from src[perm[i]] (same zone)
__global__ void __launch_bounds__(THREADS) k_gather_scatter(const uint4* __restrict__ src,
  const uint32_t* __restrict__ perm, const uint32_t* __restrict__ pos, uint4* __restrict__ dst)
{
  const uint32_t base = blockIdx.x * PER;
  for(uint32_t i = threadIdx.x; i < PER; i += THREADS * 4)
  {
    uint4 r[4];
    uint32_t p[4];
#pragma unroll
    for(int u = 0; u < 4; ++u)
    {
      const uint32_t j = i + u * THREADS;
      if(j < PER) { r[u] = src[base + perm[base + j]]; p[u] = pos[base + j]; }
    }
#pragma unroll
    for(int u = 0; u < 4; ++u)
      if(i + u * THREADS < PER) dst[p[u]] = r[u];
  }
}

// every workgroup adds to each of NZ counters `reps` times (chunk reservations)
__global__ void __launch_bounds__(THREADS) k_reserve(uint32_t* ctr, uint32_t reps, uint32_t* sink)
{
  uint32_t acc = 0;
  for(uint32_t r = 0; r < reps; ++r)
    for(uint32_t b = threadIdx.x; b < NZ; b += THREADS) acc += atomicAdd(&ctr[b], 20u);
  if(acc == 0x12345678u) sink[0] = acc;
}

// pull: zone z gathers its chunk from every source zone's bucket-sorted outbox
// (start/count per (source, z)) into its own contiguous landing region
__global__ void __launch_bounds__(THREADS) k_pull(const uint4* __restrict__ src,
  const uint32_t* __restrict__ start, const uint32_t* __restrict__ count, uint4* __restrict__ dst)
{
  __shared__ uint32_t s_pre[NZ + 1];
  __shared__ uint32_t s_st[NZ];
  const uint32_t z = blockIdx.x;
  for(uint32_t s = threadIdx.x; s < NZ; s += THREADS)
  {
    s_pre[s + 1] = count[(size_t)s * NZ + z];
    s_st[s] = start[(size_t)s * NZ + z];
  }
  if(threadIdx.x == 0) s_pre[0] = 0;
  __syncthreads();
  if(threadIdx.x == 0)
    for(uint32_t s = 1; s <= NZ; ++s) s_pre[s] += s_pre[s - 1];
  __syncthreads();
  const uint32_t tot = s_pre[NZ];
  for(uint32_t j = threadIdx.x; j < tot; j += THREADS)
  {
    uint32_t lo = 0, hi = NZ;     // largest s with s_pre[s] <= j
    while(hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if(s_pre[m] <= j) lo = m; else hi = m; }
    dst[(size_t)z * REGION + j] = src[(size_t)lo * REGION + s_st[lo] + (j - s_pre[lo])];
  }
}

int main()
{
  std::mt19937 rng(1);
  std::vector<uint32_t> dstz((size_t)NZ * PER), cnt((size_t)NZ * NZ, 0);
  for(uint32_t s = 0; s < NZ; ++s)
    for(uint32_t i = 0; i < PER; ++i) { dstz[(size_t)s * PER + i] = rng() % NZ; cnt[(size_t)s * NZ + dstz[(size_t)s * PER + i]]++; }
  // chunk base of (s, b) inside region b: sources in a shuffled order (atomic order)
  std::vector<uint32_t> chunk((size_t)NZ * NZ);
  for(uint32_t b = 0; b < NZ; ++b)
  {
    std::vector<uint32_t> ord(NZ);
    std::iota(ord.begin(), ord.end(), 0);
    std::shuffle(ord.begin(), ord.end(), rng);
    uint32_t run = 0;
    for(uint32_t s : ord) { chunk[(size_t)s * NZ + b] = b * REGION + run; run += cnt[(size_t)s * NZ + b]; }
  }
  // the same with every chunk starting on a 128-B line (8 records)
  std::vector<uint32_t> chunk_a((size_t)NZ * NZ);
  for(uint32_t b = 0; b < NZ; ++b)
  {
    uint32_t run = 0;
    for(uint32_t s = 0; s < NZ; ++s) { chunk_a[(size_t)s * NZ + b] = b * REGION + run; run += (cnt[(size_t)s * NZ + b] + 7) & ~7u; }
  }
  auto positions = [&](const std::vector<uint32_t>& ch, std::vector<uint32_t>& pr, std::vector<uint32_t>& ps) {
    pr.resize((size_t)NZ * PER); ps.resize((size_t)NZ * PER);
    for(uint32_t s = 0; s < NZ; ++s)
    {
      std::vector<uint32_t> cur(NZ, 0);
      for(uint32_t i = 0; i < PER; ++i)
      {
        const uint32_t b = dstz[(size_t)s * PER + i];
        pr[(size_t)s * PER + i] = ch[(size_t)s * NZ + b] + cur[b]++;
      }
      std::vector<uint32_t> p(pr.begin() + (size_t)s * PER, pr.begin() + (size_t)(s + 1) * PER);
      std::sort(p.begin(), p.end());
      std::copy(p.begin(), p.end(), ps.begin() + (size_t)s * PER);
    }
  };
  std::vector<uint32_t> pos_ar, pos_as;
  positions(chunk_a, pos_ar, pos_as);
  std::vector<uint32_t> pos_r((size_t)NZ * PER), pos_s((size_t)NZ * PER);
  for(uint32_t s = 0; s < NZ; ++s)
  {
    std::vector<uint32_t> cur(NZ, 0);
    for(uint32_t i = 0; i < PER; ++i)
    {
      const uint32_t b = dstz[(size_t)s * PER + i];
      pos_r[(size_t)s * PER + i] = chunk[(size_t)s * NZ + b] + cur[b]++;
    }
    std::vector<uint32_t> p(pos_r.begin() + (size_t)s * PER, pos_r.begin() + (size_t)(s + 1) * PER);
    std::sort(p.begin(), p.end(), [&](uint32_t x, uint32_t y) { return x / REGION != y / REGION ? x / REGION < y / REGION : x < y; });
    std::copy(p.begin(), p.end(), pos_s.begin() + (size_t)s * PER);
  }
  uint4 *src, *dst;
  uint32_t *dpr, *dps;
  CK(hipMalloc(&src, (size_t)NZ * PER * 16));
  CK(hipMalloc(&dst, (size_t)NZ * REGION * 16));
  CK(hipMalloc(&dpr, (size_t)NZ * PER * 4));
  CK(hipMalloc(&dps, (size_t)NZ * PER * 4));
  CK(hipMemset(src, 7, (size_t)NZ * PER * 16));
  CK(hipMemcpy(dpr, pos_r.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dps, pos_s.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
  uint32_t *dpar, *dpas;
  CK(hipMalloc(&dpar, (size_t)NZ * PER * 4));
  CK(hipMalloc(&dpas, (size_t)NZ * PER * 4));
  CK(hipMemcpy(dpar, pos_ar.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpas, pos_as.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for(int rep = 0; rep < 10; ++rep)
    {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    const double recs = (double)NZ * PER;
    printf("%-34s %8.4f ms  %6.2f G rec/s  %7.1f GB/s of 16-B records\n", name, best, recs / best / 1e6,
      recs * 16 / best / 1e6);
  };
  timeit("scatter, outbox (random) order", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpr, dst); });
  timeit("scatter, sorted by destination", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dps, dst); });
  timeit("aligned chunks, random order", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpar, dst); });
  timeit("aligned chunks, sorted", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpas, dst); });
  {
    // local: each zone sorts its outbox into its OWN region by destination
    std::vector<uint32_t> pos_l((size_t)NZ * PER), st((size_t)NZ * NZ), cn((size_t)NZ * NZ);
    for(uint32_t s = 0; s < NZ; ++s)
    {
      std::vector<uint32_t> pre(NZ + 1, 0), cur(NZ, 0);
      for(uint32_t b = 0; b < NZ; ++b) pre[b + 1] = pre[b] + cnt[(size_t)s * NZ + b];
      for(uint32_t b = 0; b < NZ; ++b) { st[(size_t)s * NZ + b] = pre[b]; cn[(size_t)s * NZ + b] = cnt[(size_t)s * NZ + b]; }
      for(uint32_t i = 0; i < PER; ++i)
      {
        const uint32_t b = dstz[(size_t)s * PER + i];
        pos_l[(size_t)s * PER + i] = s * REGION + pre[b] + cur[b]++;
      }
    }
    uint32_t *dpl, *dst_, *dcn;
    uint4* dst2;
    CK(hipMalloc(&dpl, (size_t)NZ * PER * 4));
    CK(hipMalloc(&dst_, (size_t)NZ * NZ * 4));
    CK(hipMalloc(&dcn, (size_t)NZ * NZ * 4));
    CK(hipMalloc(&dst2, (size_t)NZ * REGION * 16));
    CK(hipMemcpy(dpl, pos_l.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dst_, st.data(), (size_t)NZ * NZ * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcn, cn.data(), (size_t)NZ * NZ * 4, hipMemcpyHostToDevice));
    timeit("local sort into own region", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpl, dst); });
    timeit("pull chunks into own region", [&] { hipLaunchKernelGGL(k_pull, dim3(NZ), dim3(THREADS), 0, 0, dst, dst_, dcn, dst2); });
  }
  {
    // tile-sorted: positions sorted within each tile of 4096 records
    std::vector<uint32_t> pos_t(pos_r);
    for(uint32_t s = 0; s < NZ; ++s)
      for(uint32_t t0 = 0; t0 < PER; t0 += 4096)
      {
        auto b0 = pos_t.begin() + (size_t)s * PER + t0;
        std::sort(b0, b0 + std::min<uint32_t>(4096, PER - t0));
      }
    uint32_t* dpt;
    CK(hipMalloc(&dpt, (size_t)NZ * PER * 4));
    CK(hipMemcpy(dpt, pos_t.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
    timeit("tile-sorted (4096) scatter", [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpt, dst); });
    // gather in bucket order from the zone's records, write sorted runs
    std::vector<uint32_t> perm((size_t)NZ * PER), pos_g((size_t)NZ * PER);
    for(uint32_t s = 0; s < NZ; ++s)
    {
      std::vector<uint32_t> id(PER);
      std::iota(id.begin(), id.end(), 0);
      std::stable_sort(id.begin(), id.end(), [&](uint32_t x, uint32_t y) { return pos_r[(size_t)s * PER + x] < pos_r[(size_t)s * PER + y]; });
      for(uint32_t i = 0; i < PER; ++i) { perm[(size_t)s * PER + i] = id[i]; pos_g[(size_t)s * PER + i] = pos_r[(size_t)s * PER + id[i]]; }
    }
    uint32_t *dperm, *dpg, *sink, *ctr;
    CK(hipMalloc(&dperm, (size_t)NZ * PER * 4));
    CK(hipMalloc(&dpg, (size_t)NZ * PER * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&ctr, NZ * 4));
    CK(hipMemcpy(dperm, perm.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpg, pos_g.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
    timeit("read only (coalesced)", [&] { hipLaunchKernelGGL(k_read, dim3(NZ), dim3(THREADS), 0, 0, src, sink); });
    timeit("gather by bucket + sorted runs", [&] { hipLaunchKernelGGL(k_gather_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dperm, dpg, dst); });
    for(uint32_t reps : {1u, 4u})
    {
      char nm[64];
      snprintf(nm, sizeof nm, "reservations: %u x 512 per zone", reps);
      timeit(nm, [&] { hipLaunchKernelGGL(k_reserve, dim3(NZ), dim3(THREADS), 0, 0, ctr, reps, sink); });
    }
  }
  timeit("coalesced copy (same bytes)", [&] { hipLaunchKernelGGL(k_copy, dim3(NZ), dim3(THREADS), 0, 0, src, dst); });
  return 0;
}

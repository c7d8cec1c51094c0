// ubench_pull.hip — push vs pull delivery of one C2 superstep's records in
// isolation (MI355X): 512 source zones x 10240 records of 16 B, each to one of
// 512 destination zones (uniform).
//
//   push, tile T  — each source zone sorts its records by destination inside
//                   tiles of T records and writes each tile's run for
//                   destination d into d's landing region (runs of T/512);
//   pull, tile T  — each source zone writes its tiles contiguously into its
//                   OWN region (coalesced), runs sorted by destination inside
//                   each tile; destination d then reads its run of every
//                   (source, tile) segment (runs of T/512 records).
// Pull timings are the read side only (the write side is the coalesced copy).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_pull scripts/ubench_pull.hip
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

__global__ void __launch_bounds__(THREADS) k_read(const uint4* __restrict__ src, uint32_t* sink)
{
  const uint32_t base = blockIdx.x * REGION;
  uint32_t acc = 0;
  for(uint32_t i = threadIdx.x; i < PER; i += THREADS * 4)
  {
    uint4 v[4];
#pragma unroll
    for(int u = 0; u < 4; ++u) v[u] = i + u * THREADS < PER ? src[base + i + u * THREADS] : uint4{0, 0, 0, 0};
#pragma unroll
    for(int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].w;
  }
  if(acc == 0x12345678u) sink[0] = acc;
}

// destination z reads its run of every segment g (nseg segments): start and
// count of (g, z) in segment-major tables; the reads are folded into a sink
__global__ void __launch_bounds__(THREADS) k_pull_read(const uint4* __restrict__ src,
  const uint32_t* __restrict__ start, const uint32_t* __restrict__ count, uint32_t nseg, uint32_t* sink)
{
  __shared__ uint32_t s_pre[NZ * 8 + 1];
  __shared__ uint32_t s_st[NZ * 8];
  __shared__ uint32_t s_tmp[THREADS / 64];
  const uint32_t z = blockIdx.x;
  // counts of every segment for z, then an exclusive scan (one pass, per-thread runs)
  const uint32_t per = (nseg + THREADS - 1) / THREADS;
  const uint32_t lo = min(threadIdx.x * per, nseg), hi = min(lo + per, nseg);
  uint32_t sum = 0;
  for(uint32_t g = lo; g < hi; ++g)
  {
    const uint32_t c = count[(size_t)z * nseg + g];
    s_pre[g + 1] = c;
    s_st[g] = start[(size_t)z * nseg + g];
    sum += c;
  }
  uint32_t incl = sum;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for(int off = 1; off < 64; off <<= 1) { const uint32_t u = __shfl_up(incl, off); if(lane >= (uint32_t)off) incl += u; }
  if(lane == 63) s_tmp[wv] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for(uint32_t w = 0; w < wv; ++w) run += s_tmp[w];
  for(uint32_t g = lo; g < hi; ++g) { const uint32_t c = s_pre[g + 1]; s_pre[g] = run; run += c; }
  if(threadIdx.x == THREADS - 1) s_pre[nseg] = run;
  __syncthreads();
  const uint32_t tot = s_pre[nseg];
  uint32_t acc = 0;
  for(uint32_t j0 = threadIdx.x; j0 < tot; j0 += THREADS * 4)
  {
    uint4 v[4];
#pragma unroll
    for(int u = 0; u < 4; ++u)
    {
      const uint32_t j = j0 + u * THREADS;
      if(j < tot)
      {
        uint32_t a = 0, b = nseg;     // largest g with s_pre[g] <= j
        while(b - a > 1) { const uint32_t m = (a + b) >> 1; if(s_pre[m] <= j) a = m; else b = m; }
        v[u] = src[s_st[a] + (j - s_pre[a])];
      }
      else
        v[u] = uint4{0, 0, 0, 0};
    }
#pragma unroll
    for(int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].w;
  }
  if(acc == 0x12345678u) sink[0] = acc;
}

int main()
{
  std::mt19937 rng(1);
  std::vector<uint32_t> dstz((size_t)NZ * PER);
  for(auto& d : dstz) d = rng() % NZ;
  uint4 *src, *dst;
  uint32_t* sink;
  CK(hipMalloc(&src, (size_t)NZ * REGION * 16));
  CK(hipMalloc(&dst, (size_t)NZ * REGION * 16));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(src, 7, (size_t)NZ * REGION * 16));
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
    printf("%-40s %8.4f ms  %7.1f GB/s of 16-B records\n", name, best, recs * 16 / best / 1e6);
  };
  timeit("coalesced copy (read + write)", [&] { hipLaunchKernelGGL(k_copy, dim3(NZ), dim3(THREADS), 0, 0, src, dst); });
  timeit("coalesced read", [&] { hipLaunchKernelGGL(k_read, dim3(NZ), dim3(THREADS), 0, 0, src, sink); });
  // xm = 1: destinations ordered XCD-major inside every tile (b' = (b % 8) * 64
  // + b / 8), so the 64 receivers an XCD runs read one contiguous stretch of
  // each tile and share its boundary lines in their own L2
  for(int xm = 0; xm < 2; ++xm)
  for(uint32_t T : {PER, 5120u, 4096u, 2560u, 2048u})
  {
    auto perm = [&](uint32_t b) { return xm ? (b % 8) * (NZ / 8) + b / 8 : b; };
    const uint32_t ntile = (PER + T - 1) / T, nseg = NZ * ntile;
    // push: chunk of (source s, dest d) inside d's region, sources in a shuffled order
    std::vector<uint32_t> cnt((size_t)NZ * NZ, 0);
    for(uint32_t s = 0; s < NZ; ++s)
      for(uint32_t i = 0; i < PER; ++i) cnt[(size_t)s * NZ + dstz[(size_t)s * PER + i]]++;
    std::vector<uint32_t> chunk((size_t)NZ * NZ);
    for(uint32_t b = 0; b < NZ; ++b)
    {
      std::vector<uint32_t> ord(NZ);
      std::iota(ord.begin(), ord.end(), 0);
      std::shuffle(ord.begin(), ord.end(), rng);
      uint32_t run = 0;
      for(uint32_t s : ord) { chunk[(size_t)s * NZ + b] = b * REGION + run; run += cnt[(size_t)s * NZ + b]; }
    }
    std::vector<uint32_t> pos_push((size_t)NZ * PER), pos_pull((size_t)NZ * PER);
    std::vector<uint32_t> st((size_t)NZ * nseg, 0), cn((size_t)NZ * nseg, 0);   // [dest][segment]
    for(uint32_t s = 0; s < NZ; ++s)
    {
      std::vector<uint32_t> cur(NZ, 0);
      for(uint32_t t = 0; t < ntile; ++t)
      {
        const uint32_t i0 = t * T, i1 = std::min(PER, i0 + T);
        std::vector<uint32_t> tc(NZ, 0), tpre(NZ + 1, 0), tcur(NZ, 0);
        for(uint32_t i = i0; i < i1; ++i) tc[perm(dstz[(size_t)s * PER + i])]++;
        for(uint32_t b = 0; b < NZ; ++b) tpre[b + 1] = tpre[b] + tc[b];
        std::vector<std::pair<uint32_t, uint32_t>> ps;
        for(uint32_t i = i0; i < i1; ++i)
        {
          const uint32_t b = dstz[(size_t)s * PER + i], bp = perm(b);
          ps.push_back({tpre[bp] + tcur[bp]++, chunk[(size_t)s * NZ + b] + cur[b]++});
        }
        // record at sorted slot k of the tile goes to push position / pull position
        std::sort(ps.begin(), ps.end());
        for(uint32_t k = 0; k < ps.size(); ++k)
        {
          pos_push[(size_t)s * PER + i0 + k] = ps[k].second;
          pos_pull[(size_t)s * PER + i0 + k] = s * REGION + i0 + k;
        }
        const uint32_t g = s * ntile + t;
        for(uint32_t b = 0; b < NZ; ++b)
        {
          st[(size_t)b * nseg + g] = s * REGION + i0 + tpre[perm(b)];
          cn[(size_t)b * nseg + g] = tc[perm(b)];
        }
      }
    }
    uint32_t *dpush, *dst_, *dcn;
    CK(hipMalloc(&dpush, (size_t)NZ * PER * 4));
    CK(hipMalloc(&dst_, (size_t)NZ * nseg * 4));
    CK(hipMalloc(&dcn, (size_t)NZ * nseg * 4));
    CK(hipMemcpy(dpush, pos_push.data(), (size_t)NZ * PER * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dst_, st.data(), (size_t)NZ * nseg * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcn, cn.data(), (size_t)NZ * nseg * 4, hipMemcpyHostToDevice));
    char nm[96];
    snprintf(nm, sizeof nm, "push, tile %u (runs ~%.1f)", T, (double)T / NZ);
    if(!xm) timeit(nm, [&] { hipLaunchKernelGGL(k_scatter, dim3(NZ), dim3(THREADS), 0, 0, src, dpush, dst); });
    if(nseg <= NZ * 8)
    {
      snprintf(nm, sizeof nm, "pull read%s, tile %u (runs ~%.1f)", xm ? " xcd-major" : "", T, (double)T / NZ);
      timeit(nm, [&] { hipLaunchKernelGGL(k_pull_read, dim3(NZ), dim3(THREADS), 0, 0, src, dst_, dcn, nseg, sink); });
    }
    CK(hipFree(dpush)); CK(hipFree(dst_)); CK(hipFree(dcn));
  }
  return 0;
}

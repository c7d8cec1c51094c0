// ubench_rounds.hip — the data movement of one C2 superstep's behaviours and
// delivery, in isolation, three ways (MI355X). 512 zones x 2048 actors, 10240
// sends per zone (uniform random destination zone), 16-B records, 24-B state
// per actor; 2 workgroups of 512 threads per CU (64 KB of LDS each, as k_step).
//
//   outbox  — k_step today: state r/w + the zone's 10240 sends appended to its
//             outbox O (HBM), then O read back tile by tile (4096 records,
//             sorted by destination) and stored in runs (~8) into the chunks;
//   rounds  — the same in 4 rounds of 512 actors: each round's ~2560 sends go
//             to a small per-zone O (40 KB, reused: stays in L2) and are
//             stored in runs (~5) into a chunk reserved per (zone, round, dest);
//   direct  — each send stored straight into its chunk as it is made (runs 1).
// Compute is left out; only the memory traffic pattern is modelled.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_rounds scripts/ubench_rounds.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

constexpr uint32_t NZ = 512, ACT = 2048, PER = 10240, THREADS = 512, ROUNDS = 4, TILE = 4096;
constexpr uint32_t REGION = 16384;          // landing records per destination zone
constexpr uint32_t RPER = PER / ROUNDS;     // sends per round

// state: field-major 3 words per actor, one pass over the zone's actors
__device__ __forceinline__ void state_rw(uint64_t* st, uint32_t a)
{
  uint64_t x = st[a], y = st[(size_t)NZ * ACT + a], c = st[2 * (size_t)NZ * ACT + a];
  x ^= y; c += 5;
  st[a] = x; st[(size_t)NZ * ACT + a] = y; st[2 * (size_t)NZ * ACT + a] = c;
}

// outbox: O written in production order, then read back in sorted tile order
// (perm: sorted slot -> O index, per tile) and stored at pos
__global__ void __launch_bounds__(THREADS) k_outbox(uint64_t* st, uint4* O, const uint32_t* perm,
  const uint32_t* pos, uint4* land)
{
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  for(uint32_t a = tid; a < ACT; a += THREADS) state_rw(st, z * ACT + a);
  uint4* Oz = O + (size_t)z * PER;
  for(uint32_t i = tid; i < PER; i += THREADS) Oz[i] = uint4{z, i, 42u, 0u};
  __syncthreads();
  for(uint32_t k = tid; k < PER; k += THREADS)
  {
    const uint32_t t0 = k / TILE * TILE;
    const uint4 r = Oz[t0 + perm[(size_t)z * PER + k]];
    land[pos[(size_t)z * PER + k]] = r;
  }
}

__global__ void __launch_bounds__(THREADS) k_rounds(uint64_t* st, uint4* O, const uint32_t* perm,
  const uint32_t* pos, uint4* land)
{
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  uint4* Oz = O + (size_t)z * RPER;
  for(uint32_t r = 0; r < ROUNDS; ++r)
  {
    state_rw(st, z * ACT + r * THREADS + tid);
    for(uint32_t i = tid; i < RPER; i += THREADS) Oz[i] = uint4{z, r * RPER + i, 42u, 0u};
    __syncthreads();
    for(uint32_t k = tid; k < RPER; k += THREADS)
    {
      const size_t g = (size_t)z * PER + r * RPER + k;
      land[pos[g]] = Oz[perm[g]];
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(THREADS) k_direct(uint64_t* st, const uint32_t* pos, uint4* land)
{
  const uint32_t z = blockIdx.x, tid = threadIdx.x;
  for(uint32_t a = tid; a < ACT; a += THREADS)
  {
    state_rw(st, z * ACT + a);
    // this actor's 5 sends, stored as made
    for(uint32_t j = 0; j < PER / ACT; ++j)
    {
      const uint32_t i = (a / THREADS) * (THREADS * PER / ACT) + j * THREADS + tid;
      land[pos[(size_t)z * PER + i]] = uint4{z, i, 42u, 0u};
    }
  }
}

int main()
{
  std::mt19937 rng(1);
  std::vector<uint32_t> dstz((size_t)NZ * PER);
  for(auto& d : dstz) d = rng() % NZ;
  // landing cursor per destination, sources reserving in a shuffled order
  auto layout = [&](uint32_t T, std::vector<uint32_t>& perm, std::vector<uint32_t>& pos) {
    perm.assign((size_t)NZ * PER, 0);
    pos.assign((size_t)NZ * PER, 0);
    std::vector<uint32_t> cur(NZ, 0);
    std::vector<uint32_t> ord(NZ);
    std::iota(ord.begin(), ord.end(), 0);
    std::shuffle(ord.begin(), ord.end(), rng);
    for(uint32_t s : ord)
      for(uint32_t t0 = 0; t0 < PER; t0 += T)
      {
        const uint32_t t1 = std::min(PER, t0 + T);
        std::vector<uint32_t> idx(t1 - t0);
        std::iota(idx.begin(), idx.end(), 0);
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
          return dstz[(size_t)s * PER + t0 + a] < dstz[(size_t)s * PER + t0 + b]; });
        for(uint32_t k = 0; k < idx.size(); ++k)
        {
          const uint32_t b = dstz[(size_t)s * PER + t0 + idx[k]];
          perm[(size_t)s * PER + t0 + k] = idx[k];
          pos[(size_t)s * PER + t0 + k] = b * REGION + (cur[b]++ % REGION);
        }
      }
  };
  std::vector<uint32_t> perm_o, pos_o, perm_r, pos_r, pos_d((size_t)NZ * PER);
  layout(TILE, perm_o, pos_o);
  layout(RPER, perm_r, pos_r);
  // direct: production order i -> its position (same chunks as the tiles)
  for(uint32_t s = 0; s < NZ; ++s)
    for(uint32_t t0 = 0; t0 < PER; t0 += TILE)
      for(uint32_t k = 0; k < std::min(TILE, PER - t0); ++k)
        pos_d[(size_t)s * PER + t0 + perm_o[(size_t)s * PER + t0 + k]] = pos_o[(size_t)s * PER + t0 + k];

  uint64_t* st;
  uint4 *O, *land;
  uint32_t *d_perm_o, *d_pos_o, *d_perm_r, *d_pos_r, *d_pos_d;
  CK(hipMalloc(&st, 3 * (size_t)NZ * ACT * 8));
  CK(hipMalloc(&O, (size_t)NZ * PER * 16));
  CK(hipMalloc(&land, (size_t)NZ * REGION * 16));
  const size_t pb = (size_t)NZ * PER * 4;
  CK(hipMalloc(&d_perm_o, pb)); CK(hipMalloc(&d_pos_o, pb));
  CK(hipMalloc(&d_perm_r, pb)); CK(hipMalloc(&d_pos_r, pb));
  CK(hipMalloc(&d_pos_d, pb));
  CK(hipMemcpy(d_perm_o, perm_o.data(), pb, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pos_o, pos_o.data(), pb, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_perm_r, perm_r.data(), pb, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pos_r, pos_r.data(), pb, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pos_d, pos_d.data(), pb, hipMemcpyHostToDevice));
  CK(hipMemset(st, 1, 3 * (size_t)NZ * ACT * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t lds = 64 * 1024;     // 2 workgroups per CU, as k_step
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
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
    printf("%-48s best %8.4f ms  mean %8.4f ms\n", name, best, sum / 20);
  };
  timeit("outbox (O in HBM, tile 4096, runs ~8)", [&] {
    hipLaunchKernelGGL(k_outbox, dim3(NZ), dim3(THREADS), lds, 0, st, O, d_perm_o, d_pos_o, land); });
  timeit("rounds (O 40 KB per zone, runs ~5)", [&] {
    hipLaunchKernelGGL(k_rounds, dim3(NZ), dim3(THREADS), lds, 0, st, O, d_perm_r, d_pos_r, land); });
  timeit("direct (stored as made, runs 1)", [&] {
    hipLaunchKernelGGL(k_direct, dim3(NZ), dim3(THREADS), lds, 0, st, d_pos_d, land); });
  return 0;
}

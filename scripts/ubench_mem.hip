// ubench_mem.hip — microbenchmarks of the primitives a superstep is made of,
// to place the drain kernel against what the hardware does (MI355X, gfx950):
//   1. random u32 atomicAdd WITH return on N counters        (slot reservation)
//   2. random u32 atomicAdd without return                    (counting)
//   3. random 16-B stores into a ring region (N x cap x 16 B) (record write)
//   4. random 16-B loads from the same region                 (record read)
//   5. the fused reservation: atomic-with-return then a dependent 16-B store
//   6. streaming 16-B copy (HBM roofline reference)
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_mem scripts/ubench_mem.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if(e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while(0)

__device__ __forceinline__ uint32_t hash32(uint32_t x)
{
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

__global__ void k_atomic_ret(uint32_t* ctr, uint32_t n, uint32_t ops, uint32_t* sink, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t t = hash32(i * 8u + k + seed) % n;
    acc += atomicAdd(&ctr[t], 1u);
  }
  if(acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ void k_atomic_noret(uint32_t* ctr, uint32_t n, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t t = hash32(i * 8u + k + seed) % n;
    __hip_atomic_fetch_add(&ctr[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_store16(uint4* ring, uint32_t n_slots, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t t = hash32(i * 8u + k + seed) % n_slots;
    ring[t] = make_uint4(i, k, t, seed);
  }
}

__global__ void k_load16(const uint4* ring, uint32_t n_slots, uint32_t ops, uint32_t* sink, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t t = hash32(i * 8u + k + seed) % n_slots;
    uint4 v = ring[t];
    acc += v.x ^ v.w;
  }
  if(acc == 0x12345678u) sink[0] = acc;
}

// reservation: slot = atomicAdd(tail[t]); ring[t*cap + (slot & cap-1)] = rec
__global__ void k_reserve_store(uint32_t* tail, uint4* ring, uint32_t n, uint32_t cap, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t t[4], s[4];
  for(uint32_t k = 0; k < ops; k += 4)
  {
#pragma unroll
    for(int u = 0; u < 4; ++u)
    {
      t[u] = hash32(i * 8u + k + u + seed) % n;
      s[u] = atomicAdd(&tail[t[u]], 1u);
    }
#pragma unroll
    for(int u = 0; u < 4; ++u)
      ring[(size_t)t[u] * cap + (s[u] & (cap - 1))] = make_uint4(i, k, t[u], s[u]);
  }
}

// same, 16 reservations in flight per lane before the dependent stores
__global__ void k_reserve_store16(uint32_t* tail, uint4* ring, uint32_t n, uint32_t cap, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t t[16], s[16];
  for(uint32_t k = 0; k < ops; k += 16)
  {
#pragma unroll
    for(int u = 0; u < 16; ++u)
    {
      t[u] = hash32(i * 16u + k + u + seed) % n;
      s[u] = atomicAdd(&tail[t[u]], 1u);
    }
#pragma unroll
    for(int u = 0; u < 16; ++u)
      ring[(size_t)t[u] * cap + (s[u] & (cap - 1))] = make_uint4(i, k, t[u], s[u]);
  }
}

// atomic and store to the same target, store NOT dependent on the atomic
__global__ void k_atomic_indep_store(uint32_t* tail, uint4* ring, uint32_t n, uint32_t cap, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t t = hash32(i * 8u + k + seed) % n;
    __hip_atomic_fetch_add(&tail[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ring[(size_t)t * cap + (k & (cap - 1))] = make_uint4(i, k, t, seed);
  }
}

// chunked writes: each wave writes one 256-B chunk (16 lanes x 16 B) per op
// at a random 256-B-aligned position (the bucketed-outbox flush pattern)
__global__ void k_chunk_store(uint4* ring, uint32_t n_chunks, uint32_t ops, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t grp = i >> 4, sub = i & 15;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
  {
    uint32_t c = hash32(grp * 8u + k + seed) % n_chunks;
    ring[(size_t)c * 16 + sub] = make_uint4(i, k, c, seed);
  }
}

// few-address contention: ops atomics spread over `n` hot counters
__global__ void k_atomic_hot(uint32_t* ctr, uint32_t n, uint32_t ops, uint32_t* sink, uint32_t seed)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 4
  for(uint32_t k = 0; k < ops; ++k)
    acc += atomicAdd(&ctr[hash32(i * 8u + k + seed) % n], 1u);
  if(acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ void k_copy(const uint4* a, uint4* b, size_t n)
{
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for(; i < n; i += stride) b[i] = a[i];
}

int main(int argc, char** argv)
{
  const uint32_t N = argc > 1 ? atoi(argv[1]) : (1u << 20);       // actors
  const uint32_t CAP = argc > 2 ? atoi(argv[2]) : 64;             // ring slots
  const uint32_t OPS = 8;
  const uint32_t threads = 5u << 20;                               // ~5M msgs per launch x OPS/...
  const uint32_t nthreads = threads / OPS;
  uint32_t *ctr, *sink;
  uint4 *ring, *a, *b;
  CK(hipMalloc(&ctr, (size_t)N * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&ring, (size_t)N * CAP * 16));
  const size_t ncopy = (size_t)1 << 26;   // 1 GiB
  CK(hipMalloc(&a, ncopy * 16));
  CK(hipMalloc(&b, ncopy * 16));
  CK(hipMemset(ctr, 0, (size_t)N * 4));
  CK(hipMemset(ring, 0, (size_t)N * CAP * 16));
  CK(hipMemset(a, 1, ncopy * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 blk(256), grd((nthreads + 255) / 256);
  const double ops_total = (double)nthreads * OPS;
  auto timeit = [&](const char* name, auto launch, double bytes_per_op) {
    launch(0);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for(int rep = 0; rep < 5; ++rep)
    {
      CK(hipEventRecord(e0));
      launch(rep + 1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if(ms < best) best = ms;
    }
    printf("%-28s %8.3f ms  %7.2f Gop/s  %8.1f GB/s(useful)\n", name, best,
      ops_total / best / 1e6, ops_total * bytes_per_op / best / 1e6);
  };
  printf("N=%u cap=%u ops/launch=%.0f\n", N, CAP, ops_total);
  timeit("atomicAdd u32 w/ return", [&](int r) {
    hipLaunchKernelGGL(k_atomic_ret, grd, blk, 0, 0, ctr, N, OPS, sink, (uint32_t)r * 7919u); }, 4);
  timeit("atomicAdd u32 no return", [&](int r) {
    hipLaunchKernelGGL(k_atomic_noret, grd, blk, 0, 0, ctr, N, OPS, (uint32_t)r * 7919u); }, 4);
  timeit("random 16B store", [&](int r) {
    hipLaunchKernelGGL(k_store16, grd, blk, 0, 0, ring, N * CAP, OPS, (uint32_t)r * 7919u); }, 16);
  timeit("random 16B load", [&](int r) {
    hipLaunchKernelGGL(k_load16, grd, blk, 0, 0, ring, N * CAP, OPS, sink, (uint32_t)r * 7919u); }, 16);
  timeit("reserve+store (atomic,16B)", [&](int r) {
    hipLaunchKernelGGL(k_reserve_store, grd, blk, 0, 0, ctr, ring, N, CAP, OPS, (uint32_t)r * 7919u); }, 20);
  timeit("reserve+store x16 in flight", [&](int r) {
    hipLaunchKernelGGL(k_reserve_store16, dim3((nthreads / 2 + 255) / 256), blk, 0, 0, ctr, ring, N, CAP, 16, (uint32_t)r * 7919u); }, 20);
  timeit("atomic + indep 16B store", [&](int r) {
    hipLaunchKernelGGL(k_atomic_indep_store, grd, blk, 0, 0, ctr, ring, N, CAP, OPS, (uint32_t)r * 7919u); }, 20);
  timeit("256B chunk store (per 16B)", [&](int r) {
    hipLaunchKernelGGL(k_chunk_store, grd, blk, 0, 0, ring, N * CAP / 16, OPS, (uint32_t)r * 7919u); }, 16);
  timeit("atomic on 4096 hot ctrs", [&](int r) {
    hipLaunchKernelGGL(k_atomic_hot, grd, blk, 0, 0, ctr, 4096, OPS, sink, (uint32_t)r * 7919u); }, 4);
  timeit("atomic on 256 hot ctrs", [&](int r) {
    hipLaunchKernelGGL(k_atomic_hot, grd, blk, 0, 0, ctr, 256, OPS, sink, (uint32_t)r * 7919u); }, 4);
  {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, a, b, ncopy);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, a, b, ncopy);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.3f ms  copy %.1f GB/s (read+write)\n", "stream copy 1 GiB", ms,
      2.0 * ncopy * 16 / ms / 1e6);
  }
  return 0;
}

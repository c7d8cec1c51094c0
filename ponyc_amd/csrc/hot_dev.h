// hot_dev.h — hot zones: a zone that lands more records in one step than its
// workgroup can count, place and sort at speed (a fan-in to non-commutative
// receivers: 100,000 FIFO sources -> 4 sinks) is prepared by the whole GPU
// before k_step runs it. The reference drains such a receiver
// on whichever scheduler thread holds it (actor.c:437-480); here its
// arrivals are put into canonical order by every CU instead of one.
//
// k_hot (kHotBlocks workgroups, launched right before k_step in engines that
// build backlogs: EngDev::hot_on) finds the zones whose landing count is at
// least kHotMin and takes the kMaxHot of them with the lowest indices (every
// workgroup the same list, by ballot in zone order), and for each, with a
// grid barrier between phases:
//   P1 count    each workgroup counts a slice of the landing buffer per actor
//               in LDS (and the senders' id range and largest sequence number
//               per actor), then adds its nonzero bins to the zone's globals;
//   P2 bins     every workgroup scans the counts (actor segments in S, as
//               k_step's scratch path lays them out) and gives each big
//               group (> kBigGroup arrivals) nb bins of its compressed key
//               ((from - fmin) << seq bits | seq), ~8 records a bin; the
//               slices' records of big groups are counted per bin;
//   P2.5 starts one workgroup per big group scans its bin counts;
//   P3 place    every record to its actor's segment of S (big groups: at its
//               bin, a cursor per bin; others anywhere in the segment: k_step
//               orders them);
//   P4 sort     one thread per bin sorts its records by key in place (<= 16
//               in registers), and the bins, counters and cursors are reset.
// The last workgroup to finish the zone marks it (hot_prep = step index + 1,
// its slot in hot_slot) if every workgroup ran every phase (hot_zone_done),
// and k_step then takes its arrival counts from hot_cnt, finds the records where
// its scratch path would have placed them, and its big groups sorted.
// Results are the same whichever workgroups did the work: records are placed
// by cursor order only inside a bin or a small group, which are sorted (by
// distinct keys) afterwards.
#pragma once
#include "engine_dev.h"

namespace gpa {

constexpr uint32_t kHotBlocks = 128;            // workgroups of k_hot (all resident: engine.hip hot_resident)
constexpr uint32_t kHotThreads = 512;
constexpr uint32_t kMaxHot = 4;                 // hot zones prepared per step (the lowest indices)
constexpr uint32_t kHotBins = 1u << 20;         // bins over a zone's big groups
constexpr uint32_t kHotBinItems = 8;            // records per bin aimed at
constexpr uint32_t kHotMaxBins = 4096;          // bins per big group
constexpr uint32_t kHotActors = 4096;           // actors per zone (both geometries)

// Grid barrier of a k_hot launch: a monotone arrival counter (never reset:
// every launch passes it a multiple of gridDim.x times). The hand-off of
// MI355X_MICROARCH.md's valid forms: every wave's stores waited
// (__syncthreads), lane 0's agent release with its own vmcnt wait (the
// compiler may drop the one after buffer_wbl2), the counter add; then one
// relaxed poll, an agent acquire (this CU's L1) and a barrier before any load.
// Every spin is bounded: a workgroup that times out (never expected — the host
// launches k_hot only when its grid is resident, engine.hip hot_resident)
// goes on without the phases after it and reports the miss at the zone's end
// (hot_zone_done), which then gives the zone back to k_step unprepared.
__device__ __forceinline__ bool hot_barrier()
{
  __shared__ uint32_t s_ok;
  __syncthreads();
  if(threadIdx.x == 0)
  {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(c_eng.hot_bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = (old / gridDim.x + 1u) * gridDim.x;
    uint32_t spins = 0;
    s_ok = 1;
    while((int32_t)(__hip_atomic_load(c_eng.hot_bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0)
    {
      __builtin_amdgcn_s_sleep(2);
      if(++spins > (1u << 26)) { s_ok = 0; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return s_ok != 0;
}

// Diagnostic build (-DGPA_STAMPS): workgroup 0 stamps the 100 MHz real-time
// clock at k_hot's phase boundaries into the last row of c_eng.dbg.
#ifdef GPA_STAMPS
#define HOT_RT(k) do { if(blockIdx.x == 0 && threadIdx.x == 0) \
  c_eng.dbg[(kMaxZones - 1) * kDbgSlots + (k)] = __builtin_amdgcn_s_memrealtime(); } while(0)
#else
#define HOT_RT(k) do {} while(0)
#endif

__device__ __forceinline__ uint32_t hot_bits(uint32_t v) { return v ? 32u - (uint32_t)__clz(v) : 0u; }

// per actor of a hot slot: [0] fmin, [1] fmax, [2] smax
__device__ __forceinline__ uint32_t* hot_aux(uint32_t slot, uint32_t k)
{
  return c_eng.hot_aux + ((size_t)slot * 3 + k) * kHotActors;
}

// The end of one hot zone, decided once for the whole grid by the last
// workgroup to finish it (an arrival counter, never reset, like hot_bar's):
// every workgroup first adds a miss to hot_bar[2] if it skipped a phase (its
// `ok` is false), then arrives. The last arriver sees every report: the zone
// is marked prepared only if it fits the bins (`fits`, the same in every
// workgroup) and no workgroup missed a phase; otherwise its arrival counts
// are cleared and k_step counts, places and sorts it itself from the landing
// buffer, which k_hot only reads — the result is the same, only slower. A
// miss is counted in hot_bar[3] (gpu_actor_debug_info).
__device__ __forceinline__ void hot_zone_done(bool ok, bool fits, uint32_t z, uint32_t h,
  uint32_t sidx, uint32_t za)
{
  __shared__ uint32_t s_clear;
  uint32_t* const fin = c_eng.hot_bar + 1;
  uint32_t* const bad = c_eng.hot_bar + 2;
  __syncthreads();
  if(threadIdx.x == 0)
  {
    if(!ok) __hip_atomic_fetch_add(bad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_clear = 0;
    if((old % gridDim.x) == gridDim.x - 1u)
    {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const uint32_t nbad = __hip_atomic_load(bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if(nbad)
      {
        __hip_atomic_store(bad, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(c_eng.hot_bar + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if(fits && nbad == 0u)
      {
        c_eng.hot_slot[z] = h;
        c_eng.hot_prep[z] = sidx + 1u;
      }
      else
        s_clear = nbad ? 2u : 1u;
    }
  }
  __syncthreads();
  if(s_clear)
  {
    uint32_t* const gcnt = c_eng.hot_cnt + (size_t)h * kHotActors;
    for(uint32_t a = threadIdx.x; a < za; a += blockDim.x) gcnt[a] = 0;
  }
  if(s_clear == 2u)
  {
    // after a missed phase nothing is known about who cleared what: every
    // bin, cursor and key range back to its resting value
    for(uint32_t j = threadIdx.x; j < kHotBins; j += blockDim.x)
    { c_eng.hot_hist[j] = 0; c_eng.hot_bcnt[j] = 0; c_eng.hot_cur[j] = 0; }
    for(uint32_t a = threadIdx.x; a < kHotActors; a += blockDim.x)
    {
      c_eng.hot_cur[kHotBins + a] = 0;
      hot_aux(h, 0)[a] = 0xFFFFFFFFu; hot_aux(h, 1)[a] = 0; hot_aux(h, 2)[a] = 0;
    }
  }
}

__global__ void __launch_bounds__(kHotThreads) k_hot(uint32_t cur, uint32_t sidx)
{
  extern __shared__ uint32_t s_h[];            // [5][za]
  __shared__ uint32_t s_list[kMaxHot];
  __shared__ uint32_t s_nlist, s_bins;
  __shared__ uint32_t s_tmp[kHotThreads / 64 + 1];
  __shared__ uint32_t s_tmp2[kHotThreads / 64 + 1];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t G = gridDim.x, bid = blockIdx.x;
  const uint32_t halt_now = c_eng.nranks == 1 ? (c_eng.spill_n[cur] != 0u || *c_eng.halt != 0u)
                                              : (*c_eng.spill_flag != 0u);
  if(halt_now) return;                         // k_step will not run this step
  const uint32_t nz = c_eng.n_zones, za = 1u << c_eng.zbits;
  // The hot zones with the kMaxHot lowest indices, in zone order — the same
  // list in every workgroup (the others go to k_step's own path): each pass
  // over kHotThreads zones ranks its hot ones by ballot, wave by wave.
  if(tid == 0) s_nlist = 0;
  __syncthreads();
  for(uint32_t z0 = 0; z0 < nz; z0 += kHotThreads)
  {
    const uint32_t z = z0 + tid;
    const bool is_hot = z < nz && min(c_eng.land_n[cur][z], c_eng.zcapz[z]) >= kHotMin;
    const unsigned long long m = __ballot(is_hot);
    if(lane == 0) s_tmp[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t k = s_nlist, tot = s_nlist;
    for(uint32_t w = 0; w < kHotThreads / 64; ++w)
    {
      if(w < wv) k += s_tmp[w];
      tot += s_tmp[w];
    }
    k += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if(is_hot && k < kMaxHot) s_list[k] = z;
    __syncthreads();
    if(tid == 0) s_nlist = tot;
    __syncthreads();
    if(tot >= kMaxHot) break;                  // uniform
  }
  const uint32_t nh = min(s_nlist, kMaxHot);
  if(nh == 0) return;                          // uniform over the grid
  uint32_t* const s_cnt = s_h;                 // counts; then segment offsets
  uint32_t* const s_a = s_h + za;              // fmin; then bin bases
  uint32_t* const s_b = s_h + 2 * za;          // fmax; then bins per actor
  uint32_t* const s_c = s_h + 3 * za;          // smax; then bin shift per actor
  uint32_t* const s_g = s_h + 4 * za;          // bin base per actor (P2 on)
  for(uint32_t h = 0; h < nh; ++h)
  {
    const uint32_t z = s_list[h];
    const uint32_t cap = c_eng.zcapz[z];
    const uint32_t nl = min(c_eng.land_n[cur][z], cap);
    const ZRec* Ld = c_eng.land[cur] + c_eng.zoff[z];
    ZRec* Sz = c_eng.S + 3 * c_eng.zoff[z];
    uint32_t* const gcnt = c_eng.hot_cnt + (size_t)h * kHotActors;
    uint32_t* const gfmin = hot_aux(h, 0);
    uint32_t* const gfmax = hot_aux(h, 1);
    uint32_t* const gsmax = hot_aux(h, 2);
    const uint32_t per = (nl + G - 1) / G;
    const uint32_t c0 = min(bid * per, nl), c1 = min(c0 + per, nl);
    HOT_RT(0);
    // ---- P1: counts and key ranges of this workgroup's slice
    for(uint32_t a = tid; a < za; a += kHotThreads)
    { s_cnt[a] = 0; s_a[a] = 0xFFFFFFFFu; s_b[a] = 0; s_c[a] = 0; }
    __syncthreads();
    for(uint32_t i = c0 + tid; i < c1; i += kHotThreads)
    {
      const uint32_t w0 = Ld[i].w0, from = Ld[i].from;
      const uint32_t a = w0 & (za - 1u);
      atomicAdd(&s_cnt[a], 1u);
      atomicMin(&s_a[a], from);
      atomicMax(&s_b[a], from);
      atomicMax(&s_c[a], w0 >> 16);
    }
    __syncthreads();
    for(uint32_t a = tid; a < za; a += kHotThreads)
      if(s_cnt[a])
      {
        atomicAdd(&gcnt[a], s_cnt[a]);
        atomicMin(&gfmin[a], s_a[a]);
        atomicMax(&gfmax[a], s_b[a]);
        atomicMax(&gsmax[a], s_c[a]);
      }
    HOT_RT(1);
    bool ok = hot_barrier();
    HOT_RT(2);
    // ---- P2: segment offsets, bins of the big groups, bin counts of the slice
    for(uint32_t a = tid; a < za; a += kHotThreads)
    {
      const uint32_t n = __hip_atomic_load(&gcnt[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_cnt[a] = n;
      uint32_t nb = 0, shift = 0;
      if(n > kBigGroup)
      {
        const uint32_t fmn = gfmin[a], fmx = gfmax[a], smx = gsmax[a];
        const uint32_t kbits = hot_bits(fmx - fmn) + hot_bits(smx);
        uint32_t lb = hot_bits((n + kHotBinItems - 1) / kHotBinItems - 1);   // ceil log2
        lb = min(min(lb, 12u), kbits);
        nb = 1u << lb;
        shift = kbits - lb;
        s_a[a] = fmn;
      }
      s_b[a] = nb;
      s_c[a] = shift | (hot_bits(gsmax[a]) << 8);
    }
    __syncthreads();
    // exclusive scans: counts -> offsets (s_cnt), bins -> bin bases (s_g; s_b
    // keeps the bin counts); each thread a run of za / kHotThreads actors
    {
      const uint32_t run = za / kHotThreads;
      uint32_t sn = 0, sb = 0;
      for(uint32_t k = 0; k < run; ++k) { sn += s_cnt[tid * run + k]; sb += s_b[tid * run + k]; }
      uint32_t pn = sn, pb = sb;
#pragma unroll
      for(int off = 1; off < 64; off <<= 1)
      {
        const uint32_t un = (uint32_t)__shfl_up((int)pn, off), ub = (uint32_t)__shfl_up((int)pb, off);
        if(lane >= (uint32_t)off) { pn += un; pb += ub; }
      }
      if(lane == 63) { s_tmp[wv] = pn; s_tmp2[wv] = pb; }
      __syncthreads();
      if(tid == 0)
      {
        uint32_t rn = 0, rb = 0;
        for(uint32_t w = 0; w < kHotThreads / 64; ++w)
        {
          const uint32_t tn = s_tmp[w], tb = s_tmp2[w];
          s_tmp[w] = rn; s_tmp2[w] = rb; rn += tn; rb += tb;
        }
        s_bins = rb;
      }
      __syncthreads();
      uint32_t rn = s_tmp[wv] + pn - sn, rb = s_tmp2[wv] + pb - sb;
      for(uint32_t k = 0; k < run; ++k)
      {
        const uint32_t a = tid * run + k;
        const uint32_t vn = s_cnt[a], vb = s_b[a];
        s_cnt[a] = rn; rn += vn;
        s_g[a] = rb; rb += vb;
      }
      __syncthreads();
    }
    const uint32_t nbins = s_bins;
    // fits: uniform over the grid when every barrier held (each workgroup
    // scanned the same counts); a zone past the bins is left to k_step's own
    // path. `ok`: this workgroup ran every phase so far.
    const bool fits = nbins <= kHotBins;
    uint32_t* const hist = c_eng.hot_hist;     // [nbins] records per bin -> (P2.5) bin starts
    uint32_t* const bcnt = c_eng.hot_bcnt;     // [nbins] records per bin (kept for P4)
    uint32_t* const bcur = c_eng.hot_cur;      // [nbins] cursors; [kHotBins + a] small groups
    if(ok && fits)
      for(uint32_t i = c0 + tid; i < c1; i += kHotThreads)
      {
        const uint32_t w0 = Ld[i].w0;
        const uint32_t a = w0 & (za - 1u);
        if(!s_b[a]) continue;
        const uint32_t from = Ld[i].from;
        const uint32_t sb = s_c[a] >> 8, sh = s_c[a] & 0xFFu;
        const uint64_t key = ((uint64_t)(from - s_a[a]) << sb) | (w0 >> 16);
        atomicAdd(&hist[s_g[a] + (uint32_t)(key >> sh)], 1u);
      }
    HOT_RT(3);
    ok = hot_barrier() && ok;
    HOT_RT(4);
    // ---- P2.5: each big group's bin starts (one workgroup per group)
    if(ok && fits)
    {
      // this workgroup's actors a = bid + k G (a serial walk over every actor
      // with a division per step took 139 us)
      for(uint32_t a = bid; a < za; a += G)
      {
        const uint32_t nb = s_b[a];             // uniform
        if(!nb) continue;
        const uint32_t b0 = s_g[a];
        // exclusive scan of hist[b0, b0 + nb) (nb <= 4096: 8 per thread)
        uint32_t v[kHotMaxBins / kHotThreads], sum = 0;
        const uint32_t per_t = kHotMaxBins / kHotThreads;
#pragma unroll
        for(uint32_t k2 = 0; k2 < per_t; ++k2)
        {
          const uint32_t j = tid * per_t + k2;
          v[k2] = j < nb ? hist[b0 + j] : 0u;
          sum += v[k2];
        }
        uint32_t incl = sum;
#pragma unroll
        for(int off = 1; off < 64; off <<= 1)
        {
          const uint32_t u = (uint32_t)__shfl_up((int)incl, off);
          if(lane >= (uint32_t)off) incl += u;
        }
        if(lane == 63) s_tmp[wv] = incl;
        __syncthreads();
        if(tid == 0)
        {
          uint32_t r = 0;
          for(uint32_t w = 0; w < kHotThreads / 64; ++w) { const uint32_t t = s_tmp[w]; s_tmp[w] = r; r += t; }
        }
        __syncthreads();
        uint32_t run = s_tmp[wv] + incl - sum;
#pragma unroll
        for(uint32_t k2 = 0; k2 < per_t; ++k2)
        {
          const uint32_t j = tid * per_t + k2;
          if(j < nb) { bcnt[b0 + j] = v[k2]; hist[b0 + j] = run; }
          run += v[k2];
        }
        __syncthreads();
      }
    }
    HOT_RT(5);
    ok = hot_barrier() && ok;
    HOT_RT(6);
    // (tests: the last workgroup misses P3 and P4, as after a barrier timeout)
    if(c_eng.hot_test && bid == G - 1u) ok = false;
    // ---- P3: every record to its place in S
    if(ok && fits)
      for(uint32_t i = c0 + tid; i < c1; i += kHotThreads)
      {
        const uint4 r = *reinterpret_cast<const uint4*>(Ld + i);
        const uint32_t a = r.x & (za - 1u);
        uint32_t pos = s_cnt[a];
        if(s_b[a])
        {
          const uint32_t sb = s_c[a] >> 8, sh = s_c[a] & 0xFFu;
          const uint64_t key = ((uint64_t)(r.y - s_a[a]) << sb) | (r.x >> 16);
          const uint32_t d = s_g[a] + (uint32_t)(key >> sh);
          pos += hist[d] + atomicAdd(&bcur[d], 1u);
        }
        else
          pos += atomicAdd(&bcur[kHotBins + a], 1u);
        *reinterpret_cast<uint4*>(Sz + pos) = r;
      }
    HOT_RT(7);
    ok = hot_barrier() && ok;
    HOT_RT(8);
    // ---- P4: each bin sorted in place by key (distinct keys); counters reset
    if(ok && fits)
      for(uint32_t j = bid * kHotThreads + tid; j < nbins; j += G * kHotThreads)
      {
        // the bin's actor: the last a with s_g[a] <= j (a small group after
        // it would start at the big group's end, past j)
        uint32_t lo = 0, hi = za - 1;
        while(lo < hi)
        {
          const uint32_t mid = (lo + hi + 1) / 2;
          if(s_g[mid] <= j) lo = mid; else hi = mid - 1;
        }
        ZRec* p = Sz + s_cnt[lo] + hist[j];
        const uint32_t m = bcnt[j];
        if(m > 1)
        {
          if(m <= 16)
          {
            uint64_t k[16];
            uint4 rr[16];
#pragma unroll
            for(int u = 0; u < 16; ++u)
              if((uint32_t)u < m)
              {
                rr[u] = *reinterpret_cast<const uint4*>(p + u);
                k[u] = ((uint64_t)rr[u].y << 16) | (rr[u].x >> 16);
              }
              else k[u] = ~0ull;
            // selection by rank: record u goes to the number of smaller keys
#pragma unroll
            for(int u = 0; u < 16; ++u)
              if((uint32_t)u < m)
              {
                uint32_t rk = 0;
#pragma unroll
                for(int t = 0; t < 16; ++t) rk += k[t] < k[u] ? 1u : 0u;
                *reinterpret_cast<uint4*>(p + rk) = rr[u];
              }
          }
          else
          {
            for(uint32_t i2 = 1; i2 < m; ++i2)
            {
              const uint4 x = *reinterpret_cast<const uint4*>(p + i2);
              const uint64_t kx = ((uint64_t)x.y << 16) | (x.x >> 16);
              uint32_t j2 = i2;
              while(j2 > 0)
              {
                const uint4 y = *reinterpret_cast<const uint4*>(p + j2 - 1);
                if((((uint64_t)y.y << 16) | (y.x >> 16)) <= kx) break;
                *reinterpret_cast<uint4*>(p + j2) = y;
                --j2;
              }
              *reinterpret_cast<uint4*>(p + j2) = x;
            }
          }
        }
        hist[j] = 0; bcnt[j] = 0; bcur[j] = 0;
      }
    else
      // a zone given back to k_step: this workgroup's share of the bins
      // cleared (a missed phase: the last workgroup clears them all below)
      for(uint32_t j = bid * kHotThreads + tid; j < min(nbins, kHotBins); j += G * kHotThreads)
      { hist[j] = 0; bcnt[j] = 0; bcur[j] = 0; }
    // per-actor scratch back to its resting values (hot_cnt stays when the
    // zone is prepared: k_step reads it and clears it)
    if(bid == 0)
      for(uint32_t a = tid; a < za; a += kHotThreads)
      {
        gfmin[a] = 0xFFFFFFFFu; gfmax[a] = 0; gsmax[a] = 0;
        bcur[kHotBins + a] = 0;
      }
    hot_zone_done(ok, fits, z, h, sidx, za);
    HOT_RT(9);
    // the next zone's P2 reuses the bins (after this one's P4 cleared them)
    if(h + 1 < nh) (void)hot_barrier();
    HOT_RT(10);
  }
}

} // namespace gpa

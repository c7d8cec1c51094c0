// zone_dev.h — the superstep kernel (k_step) and the injection kernels.
//
// k_step runs one 512-thread workgroup per zone of 2048 actors and replaces,
// for those actors, ponyint_actor_run's pop loop (actor.c:383-549), the MPSC
// push/pop (messageq.c:31-59,234-258) and the scheduler's run/steal loop
// (scheduler.c:752-1090):
//   1. count the zone's carried and newly landed records per actor (LDS
//      atomics; each landed record's rank comes back from its atomic) and
//      scan them into per-actor segments;
//   2. place an LDS index (u16) of every record at its segment position
//      (carry first, canonical; new arrivals after, in landing order) — or,
//      for a zone with more records than the index holds, the records
//      themselves into the scratch S;
//   3. per actor: handle min(batch, n) messages — carried mail, then the new
//      group in (from, seq) key order — with the actor's state in registers;
//      sends are parked in the zone outbox O and counted per destination
//      bucket (zone, or peer rank) in LDS; the unhandled tail is written to
//      the zone's carry buffer for the next step, already canonical;
//   4. reserve one contiguous chunk per destination bucket with ONE
//      atomicAdd per (zone, bucket) and scatter the outbox, sorted by bucket
//      in LDS tiles, into the destination zones' landing buffers (or the
//      per-peer exchange buffer).
// Workgroups never wait on each other: all inter-zone traffic goes through
// the next launch (the step boundary is the BSP barrier).
#pragma once
#include "engine_dev.h"

namespace gpa {

// Diagnostic build only (-DGPA_STAMPS): thread 0 of each zone stamps the
// shader clock at phase boundaries into c_eng.dbg[zone * 8 + k]. The shipped
// build compiles these away.
#ifdef GPA_STAMPS
#define GPA_STAMP(k)                                                         \
  do { if(threadIdx.x == 0) c_eng.dbg[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while(0)
#else
#define GPA_STAMP(k) do {} while(0)
#endif

constexpr int kUnroll = 8;   // independent records in flight per thread in streaming loops
#ifndef GPA_IDX_CAP
#define GPA_IDX_CAP 12288
#endif
#ifndef GPA_TILE
#define GPA_TILE 4096
#endif
constexpr uint32_t kIdxCap = GPA_IDX_CAP;  // LDS index budget per zone (records per step)
constexpr uint32_t kTile = GPA_TILE;       // outbox records sorted per scatter tile (64 KB of LDS)
constexpr int kTilePer = kTile / kZoneThreads;  // tile records per thread
constexpr int kIdxPer = kIdxCap / kZoneThreads; // landed records per thread on the LDS-index path
static_assert(kTile % kZoneThreads == 0 && kIdxCap % kZoneThreads == 0, "tile / index split");
// Arrival groups up to this size are loaded at once and ordered in registers.
// 16 where the handler does not read the message (pinger: the selection
// compiles away) or the table's state is small; 8 elsewhere, to stay within
// 128 VGPRs without spilling.
template <int HT> __host__ __device__ constexpr uint32_t small_regs()
{
  return (HT == GPU_ACTOR_HT_PINGER || HT == GPU_ACTOR_HT_FANIN_SENDER) ? 16u : 8u;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
  for(int off = 32; off > 0; off >>= 1)
    v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane)
{
#pragma unroll
  for(int off = 1; off < 64; off <<= 1)
  {
    const uint32_t u = (uint32_t)__shfl_up((int)v, off);
    if(lane >= (uint32_t)off) v += u;
  }
  return v;
}

// In-place exclusive scan of arr[kZone] (LDS) by a kZoneThreads workgroup;
// returns the total. All threads must call it.
__device__ uint32_t block_scan_zone(uint32_t* arr, uint32_t* s_tmp)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr uint32_t per = kZone / kZoneThreads;
  uint32_t v[per];
  uint32_t sum = 0;
#pragma unroll
  for(uint32_t k = 0; k < per; ++k) { v[k] = arr[tid * per + k]; sum += v[k]; }
  const uint32_t incl = wave_incl_scan(sum, lane);
  if(lane == 63) s_tmp[wv] = incl;
  __syncthreads();
  if(wv == 0)
  {
    uint32_t x = lane < (uint32_t)kZoneWaves ? s_tmp[lane] : 0u;
    x = wave_incl_scan(x, lane);
    if(lane < (uint32_t)kZoneWaves) s_tmp[lane] = x;
  }
  __syncthreads();
  uint32_t run = (wv ? s_tmp[wv - 1] : 0u) + incl - sum;
#pragma unroll
  for(uint32_t k = 0; k < per; ++k) { arr[tid * per + k] = run; run += v[k]; }
  const uint32_t total = s_tmp[kZoneWaves - 1];
  __syncthreads();
  return total;
}

// Phase-1 scans in one pass: off = exclusive scan of cnt + ccnt (segment
// starts), aux = exclusive scan of ccnt (carry starts). Two wave-level scans
// share the barriers, and waves 0 and 1 scan the two wave-total vectors side by
// side. s_tmp2 holds 2 * kZoneWaves entries. All threads call it; it ends
// behind a barrier.
__device__ void block_scan_zone_pair(const uint32_t* cnt, const uint32_t* ccnt, uint32_t* off,
                                     uint32_t* aux, uint32_t* s_tmp2)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  static_assert(kZoneWaves >= 2 && kZoneWaves <= 64, "pair scan: one wave per vector");
  constexpr uint32_t per = kZone / kZoneThreads;
  uint32_t va[per], vb[per];
  uint32_t sa = 0, sb = 0;
#pragma unroll
  for(uint32_t k = 0; k < per; ++k)
  {
    vb[k] = ccnt[tid * per + k];
    va[k] = cnt[tid * per + k] + vb[k];
    sa += va[k];
    sb += vb[k];
  }
  const uint32_t ia = wave_incl_scan(sa, lane);
  const uint32_t ib = wave_incl_scan(sb, lane);
  if(lane == 63) { s_tmp2[wv] = ia; s_tmp2[kZoneWaves + wv] = ib; }
  __syncthreads();
  if(wv < 2)
  {
    uint32_t* t = s_tmp2 + wv * kZoneWaves;
    uint32_t x = lane < (uint32_t)kZoneWaves ? t[lane] : 0u;
    x = wave_incl_scan(x, lane);
    if(lane < (uint32_t)kZoneWaves) t[lane] = x;
  }
  __syncthreads();
  uint32_t ra = (wv ? s_tmp2[wv - 1] : 0u) + ia - sa;
  uint32_t rb = (wv ? s_tmp2[kZoneWaves + wv - 1] : 0u) + ib - sb;
#pragma unroll
  for(uint32_t k = 0; k < per; ++k)
  {
    off[tid * per + k] = ra; ra += va[k];
    aux[tid * per + k] = rb; rb += vb[k];
  }
  __syncthreads();
}

// Exclusive scan of in[0, n) into out[0, n) (LDS; in place allowed) by a
// kZoneThreads workgroup, each thread taking a contiguous run; returns the
// total. Each wave adds the totals of the waves before it (no second scan
// level). All threads call it; it ends behind a barrier.
__device__ uint32_t block_scan_n(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* s_tmp)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t per = (n + kZoneThreads - 1) / kZoneThreads;
  const uint32_t lo = min(tid * per, n), hi = min(lo + per, n);
  uint32_t sum = 0;
  for(uint32_t i = lo; i < hi; ++i) sum += in[i];
  const uint32_t incl = wave_incl_scan(sum, lane);
  if(lane == 63) s_tmp[wv] = incl;
  __syncthreads();
  uint32_t run = incl - sum, total = 0;
  for(uint32_t w = 0; w < (uint32_t)kZoneWaves; ++w)
  {
    const uint32_t t = s_tmp[w];
    run += w < wv ? t : 0u;
    total += t;
  }
  for(uint32_t i = lo; i < hi; ++i) { const uint32_t v = in[i]; out[i] = run; run += v; }
  __syncthreads();
  return total;
}

// 16-B record moves built from their four words. Written this way, the
// scatter tile's records stay in registers and go to LDS as one ds_write_b128
// each; the plain uint4 copy made the compiler split the LDS stores and spill
// the tile to scratch (measured 40.8 -> 54.9 G msgs/s on C2). Non-temporal
// versions of these were slower (44 G msgs/s).
__device__ __forceinline__ void st16(uint4* p, const uint4& v)
{
  p->x = v.x; p->y = v.y; p->z = v.z; p->w = v.w;
}
__device__ __forceinline__ uint4 ld16(const uint4* p)
{
  uint4 v;
  v.x = p->x; v.y = p->y; v.z = p->z; v.w = p->w;
  return v;
}

__device__ __forceinline__ ZRec ld_rec(const ZRec* p)
{
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  ZRec r;
  r.w0 = v.x; r.from = v.y; r.arg = ((uint64_t)v.w << 32) | v.z;
  return r;
}

// An actor's segment of the zone's records, in segment order: [0, nc) carried
// mail (canonical), [nc, n) this step's arrival group (arrival order until
// sorted). The segment is a run of the zone's record index GI: u32 entries
// naming a record in the zone's carry buffer (kGiCarry), its landing buffer
// (injected / pushed records) or a sender's send region P (kGiPull).
constexpr uint32_t kGiPull = 0x80000000u;
constexpr uint32_t kGiCarry = 0x40000000u;
constexpr uint32_t kGiPosMask = 0x3FFFFFFFu;

struct AccG {
  uint32_t* gi;          // the actor's segment of GI
  const ZRec* C;         // zone carry[cur]
  const ZRec* Ld;        // zone land[cur]
  const ZRec* P;         // P[cur] (every zone's send region)
  __device__ __forceinline__ ZRec at(uint32_t e) const
  {
    if(e & kGiPull) return ld_rec(P + (e & ~kGiPull));
    if(e & kGiCarry) return ld_rec(C + (e & kGiPosMask));
    return ld_rec(Ld + e);
  }
  __device__ __forceinline__ ZRec rec(uint32_t j) const { return at(gi[j]); }
  // insertion sort of [lo, lo + g) by canonical key (stable)
  __device__ void sort(uint32_t lo, uint32_t g)
  {
    for(uint32_t i = 1; i < g; ++i)
    {
      const uint32_t x = gi[lo + i];
      const uint64_t kx = zkey(at(x));
      uint32_t j = i;
      while(j > 0)
      {
        const uint32_t y = gi[lo + j - 1];
        if(zkey(at(y)) <= kx) break;
        gi[lo + j] = y;
        --j;
      }
      gi[lo + j] = x;
    }
  }
};

template <int HT> __host__ __device__ constexpr bool may_yield()
{
  return HT == GPU_ACTOR_HT_FIFO_SINK;
}

// Drain one actor: handle up to min(batch, n) messages — carried mail, then
// the arrival group in (from, seq) key order — stopping early after a
// behaviour whose sends muted the actor or that yielded. Returns how many ran;
// the rest, [done, n) of acc, is left in canonical order for the carry-out
// pass (the group is sorted in place when it was not handled whole).
template <int HT, class Acc>
__device__ __forceinline__ uint32_t drain_zone(const TypeDev& Tref, ZoneCtx& a, Acc acc,
  uint32_t n, uint32_t nc, bool presorted)
{
  // a register copy of the type's fields: read once, not re-read after every
  // store the handlers make (the compiler cannot prove they do not alias)
  const TypeDev T = Tref;
  constexpr int NW = HT_Words<HT>::W;
  constexpr bool kY = may_yield<HT>();
  const uint32_t w = n < T.batch ? n : T.batch;
  uint64_t s[NW];
#pragma unroll
  for(int k = 0; k < NW; ++k) s[k] = T.state[(size_t)k * T.lcount + a.li];
  const uint32_t g = n - nc;
  const uint32_t hc = min(w, nc);                 // carried messages handled now
  constexpr uint32_t SM = small_regs<HT>();
  const bool small = g > 0 && w - hc >= g && g <= SM && !presorted;
  // small arrival group: its records are loaded with the state, before any
  // handler runs (one round of memory latency for the actor); the behaviour
  // rides in the key's low bits (key << 4 | beh sorts like the key)
  uint64_t k[SM], v[SM];
#pragma unroll
  for(int j = 0; j < (int)SM; ++j)
  {
    if(small && (uint32_t)j < g)
    {
      const ZRec r = acc.rec(nc + j);
      k[j] = (zkey(r) << 4) | ((r.w0 >> 12) & 0xFu); v[j] = r.arg;
    }
    else
    {
      k[j] = ~0ull; v[j] = 0;
    }
  }
  // Wait for those loads here, once: otherwise the wait lands at the head of
  // the handler loops, where it also waits for every outbox store the previous
  // message made (vmcnt counts stores too).
  __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
  uint32_t done = 0;
  bool stop = false, sorted = false;
  while(done < hc && !stop)
  {
    const ZRec r = acc.rec(done);
    handle(HtTag<HT>{}, T, a, s, (r.w0 >> 12) & 0xFu, r.arg);
    ++done;
    stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
  }
  if(g > 0 && !stop)
  {
    const uint32_t q = w - done;
    if(small)
    {
      // small group handled whole: all records in registers, select by key
      for(uint32_t r = 0; r < g && !stop; ++r)
      {
        uint64_t best = k[0], barg = v[0];
        uint32_t bi = 0;
#pragma unroll
        for(int j = 1; j < (int)SM; ++j)
          if(k[j] < best) { best = k[j]; barg = v[j]; bi = (uint32_t)j; }
#pragma unroll
        for(int j = 0; j < (int)SM; ++j)
          if((uint32_t)j == bi) k[j] = ~0ull;
        handle(HtTag<HT>{}, T, a, s, (uint32_t)best & 0xFu, barg);
        ++done;
        stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
      }
    }
    else if(q >= g && !presorted)
    {
      // large group handled whole: select in key order
      uint64_t last = 0;
      for(uint32_t r = 0; r < g && !stop; ++r)
      {
        uint64_t best = ~0ull;
        uint32_t bi = 0;
        for(uint32_t j = 0; j < g; ++j)
        {
          const uint64_t kk = zkey(acc.rec(nc + j));
          if((r == 0 || kk > last) && kk < best) { best = kk; bi = j; }
        }
        const ZRec rr = acc.rec(nc + bi);
        handle(HtTag<HT>{}, T, a, s, (rr.w0 >> 12) & 0xFu, rr.arg);
        last = best;
        ++done;
        stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
      }
    }
    else
    {
      // part of the group carries over (or it was sorted by the whole
      // workgroup already): canonical order first
      if(!presorted) acc.sort(nc, g);
      sorted = true;
      for(uint32_t k = 0; k < q && !stop; ++k)
      {
        const ZRec r = acc.rec(nc + k);
        handle(HtTag<HT>{}, T, a, s, (r.w0 >> 12) & 0xFu, r.arg);
        ++done;
        stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
      }
    }
  }
#pragma unroll
  for(int k = 0; k < NW; ++k) T.state[(size_t)k * T.lcount + a.li] = s[k];
  // what ran of the group were its smallest keys: sorted, the group's tail
  // is the canonical remainder
  if(done < n && g > 1 && !sorted && !presorted) acc.sort(nc, g);
  return done;
}

// The unhandled tail [done, n) of an actor's segment, already canonical, to
// the next step's carry buffer at carry position co (positions past the
// zone's capacity go to the spill list: never lost).
template <class Acc>
__device__ __forceinline__ void carry_out(Acc acc, uint32_t done, uint32_t n, uint32_t z,
  uint32_t co, uint32_t nxt)
{
  ZRec* cout = c_eng.carry[nxt] + c_eng.zoff[z];
  const uint32_t cap = zone_capacity(z);
  for(uint32_t k = done; k < n; ++k)
  {
    const ZRec r = acc.rec(k);
    uint4 u;
    u.x = r.w0; u.y = r.from; u.z = (uint32_t)r.arg; u.w = (uint32_t)(r.arg >> 32);
    const uint32_t pos = co + (k - done);
    if(pos < cap)
      *reinterpret_cast<uint4*>(cout + pos) = u;
    else
      spill_rec(nxt, kSpillCarry, z, pos, u);
  }
}

// ---- hot receivers: arrival groups sorted by the whole workgroup ------------------
// An actor with more than kBigGroup arrivals in one step (fan-in to a
// non-commutative receiver) would otherwise order them inside its own lane,
// O(g^2). Instead, before the behaviours run, the workgroup sorts each such
// group with a stable LSD radix sort (8-bit digits) over u64 items
// key << kPayBits | payload, the key compressed to (from - min from) << sbits
// | seq, the payload the record's idx entry (or its position in S).
constexpr uint32_t kBigGroup = 128;
constexpr uint32_t kMaxBig = 32;            // big groups sorted per round of the loop
constexpr uint32_t kPayBits = 20;           // payload bits of an item (group <= 2^20)
constexpr uint32_t kSortWork = 512 + kZoneWaves * 256;   // u32 of LDS the sort borrows

// Stable sort of n items in a by item bits [lo, hi); b is scratch of n items.
// The result ends in a. All threads call; ends behind a barrier.
__device__ void coop_radix_sort(uint64_t* a, uint64_t* b, uint32_t n, uint32_t lo, uint32_t hi,
  uint32_t* s_work)
{
  uint32_t* s_bin = s_work;                // [2][256] running base of each digit (double-buffered)
  uint32_t* s_wc = s_work + 512;           // [kZoneWaves][256] this tile's counts per wave
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t* src = a;
  uint64_t* dst = b;
  for(uint32_t sh = lo; sh < hi; sh += 8)
  {
    for(uint32_t d = tid; d < 256; d += kZoneThreads) s_bin[d] = 0;
    __syncthreads();
    for(uint32_t i = tid; i < n; i += kZoneThreads) atomicAdd(&s_bin[(src[i] >> sh) & 255u], 1u);
    __syncthreads();
    if(wv == 0)
    {
      uint32_t v[4], sum = 0;
#pragma unroll
      for(int k = 0; k < 4; ++k) { v[k] = s_bin[lane * 4 + k]; sum += v[k]; }
      uint32_t run = wave_incl_scan(sum, lane) - sum;
#pragma unroll
      for(int k = 0; k < 4; ++k) { s_bin[lane * 4 + k] = run; run += v[k]; }
    }
    uint32_t cb = 0;                       // which half of s_bin holds this tile's bases
    for(uint32_t t0 = 0; t0 < n; t0 += kZoneThreads)
    {
      const uint32_t i = t0 + tid;
      const bool valid = i < n;
      const uint64_t x = valid ? src[i] : 0ull;
      const uint32_t d = (uint32_t)(x >> sh) & 255u;
      // lanes of this wave holding the same digit: 8 ballots
      uint64_t same = __ballot(valid);
#pragma unroll
      for(int bit = 0; bit < 8; ++bit)
      {
        const uint64_t bb = __ballot(valid && ((d >> bit) & 1u));
        same &= ((d >> bit) & 1u) ? bb : ~bb;
      }
      for(uint32_t k = lane; k < 256; k += 64) s_wc[wv * 256 + k] = 0;
      __builtin_amdgcn_wave_barrier();
      const uint32_t rank = __popcll(same & lt);
      if(valid && rank == 0) s_wc[wv * 256 + d] = __popcll(same);
      __syncthreads();                     // counts (and, first time, the bases) visible
      if(valid)
      {
        uint32_t pre = s_bin[cb * 256 + d];
        for(uint32_t w = 0; w < wv; ++w) pre += s_wc[w * 256 + d];
        dst[pre + rank] = x;
      }
      for(uint32_t k = tid; k < 256; k += kZoneThreads)
      {
        uint32_t c = s_bin[cb * 256 + k];
        for(uint32_t w = 0; w < (uint32_t)kZoneWaves; ++w) c += s_wc[w * 256 + k];
        s_bin[(cb ^ 1u) * 256 + k] = c;
      }
      cb ^= 1u;
      __syncthreads();                     // every read of s_wc and the old bases done
    }
    uint64_t* t = src; src = dst; dst = t;
  }
  if(src != a)
  {
    for(uint32_t i = tid; i < n; i += kZoneThreads) a[i] = src[i];
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t bits_for(uint32_t v)
{
  return v ? 32u - (uint32_t)__clz(v) : 0u;
}

// Sort the arrival group [nc, nc + g) of one actor's segment by the whole
// workgroup: items key << kPayBits | position, then the GI entries permuted
// through `tmp` (g words). ia / ib hold g items each. Returns false (nothing
// changed) when the compressed key or the position does not fit.
__device__ bool coop_sort_group(const AccG& acc, uint32_t nc, uint32_t g, uint64_t* ia,
  uint64_t* ib, uint32_t* tmp, uint32_t* s_work, uint32_t* s_red3)
{
  const uint32_t tid = threadIdx.x;
  if(g > (1u << kPayBits)) return false;
  // key range: min/max sender, max sequence
  uint32_t fmin = 0xFFFFFFFFu, fmax = 0, smax = 0;
  for(uint32_t j = tid; j < g; j += kZoneThreads)
  {
    const ZRec r = acc.rec(nc + j);
    fmin = min(fmin, r.from); fmax = max(fmax, r.from); smax = max(smax, r.w0 >> 16);
  }
  if(tid < 3) s_red3[tid] = tid == 0 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  atomicMin(&s_red3[0], fmin); atomicMax(&s_red3[1], fmax); atomicMax(&s_red3[2], smax);
  __syncthreads();
  fmin = s_red3[0]; fmax = s_red3[1]; smax = s_red3[2];
  __syncthreads();
  const uint32_t sbits = bits_for(smax), kbits = bits_for(fmax - fmin) + sbits;
  if(kbits + kPayBits > 64u) return false;
  for(uint32_t j = tid; j < g; j += kZoneThreads)
  {
    const ZRec r = acc.rec(nc + j);
    const uint64_t key = ((uint64_t)(r.from - fmin) << sbits) | (r.w0 >> 16);
    ia[j] = (key << kPayBits) | (uint64_t)j;
  }
  __syncthreads();
  coop_radix_sort(ia, ib, g, kPayBits, kPayBits + ((kbits + 7u) & ~7u), s_work);
  const uint64_t pm = (1ull << kPayBits) - 1;
  for(uint32_t j = tid; j < g; j += kZoneThreads) tmp[j] = acc.gi[nc + (uint32_t)(ia[j] & pm)];
  __syncthreads();
  for(uint32_t j = tid; j < g; j += kZoneThreads) acc.gi[nc + j] = tmp[j];
  __syncthreads();
  return true;
}

// One actor of the zone: stays muted (nothing runs; its arrivals are put in
// canonical order for the carry) or drains.
template <int HT, class Acc>
__device__ __forceinline__ uint32_t zone_actor(const TypeDev& T, ZoneCtx& a, Acc acc, uint32_t n,
  uint32_t nc, bool stays, bool presorted)
{
  if(stays)
  {
    if(n - nc > 1 && !presorted) acc.sort(nc, n - nc);
    return 0;
  }
  return drain_zone<HT>(T, a, acc, n, nc, presorted);
}

// ---- k_step's LDS: one dynamic region (every carve offset a multiple of 16) ---------
// Two workgroups per CU, each with half of the CU's 160 KB: the fixed part,
// then the bucket arrays (outbox histogram [nb], tile counts [nbp + 1]), then
// the region that phase 0 (the segment table), the hot-group sort, the drain
// rounds (the LDS tile) and phase 4 (the outbox sort) take in turn.
constexpr uint32_t kLdsMax = 81920;                        // half of gfx950's 160 KB per CU
#ifndef GPA_LDS_STATIC
#define GPA_LDS_STATIC 2048
#endif
constexpr uint32_t kLdsStatic = GPA_LDS_STATIC;            // left for the compiler's own LDS
constexpr uint32_t kLdsDyn = kLdsMax - kLdsStatic;         // k_step's dynamic LDS
constexpr uint32_t kMaxT = kZone / kZoneThreads;           // drain rounds = tiles per zone per step
static_assert(kZone % kZoneThreads == 0, "whole rounds");
constexpr uint32_t L_OFF = 0;                              // s_off: counts, then segment offsets [kZone + 4]
constexpr uint32_t L_CCNT = L_OFF + (kZone + 4) * 4;       // carried records per actor
constexpr uint32_t L_AUX = L_CCNT + kZone * 4;             // carry start -> cursor -> remainder
constexpr uint32_t L_TB = L_AUX + kZone * 4;               // trigger byte per actor
constexpr uint32_t L_BIGBITS = L_TB + kZone;               // groups the workgroup sorted
constexpr uint32_t L_RED = L_BIGBITS + kZone / 8;          // counter reduction
constexpr uint32_t L_AGG = L_RED + kZoneWaves * 6 * 8;     // per-wave aggregation word
constexpr uint32_t L_BYTYPE = L_AGG + kZoneWaves * 8;      // delivered per type
constexpr uint32_t L_SMALL = L_BYTYPE + GPU_ACTOR_MAX_TYPES * 8;
constexpr uint32_t kSmallWords = 128;
constexpr uint32_t L_FAN = L_SMALL + kSmallWords * 4;      // fan-in apply accumulators (kFan only)
constexpr uint32_t L_VAR_FAN = L_FAN + 2 * kFanLds * 8;
static_assert(L_CCNT % 16 == 0 && L_AUX % 16 == 0 && L_TB % 16 == 0 && L_BIGBITS % 16 == 0 &&
              L_RED % 16 == 0 && L_AGG % 16 == 0 && L_BYTYPE % 16 == 0 && L_SMALL % 16 == 0 &&
              L_FAN % 16 == 0 && L_VAR_FAN % 16 == 0, "16-B carve");
// small words
constexpr uint32_t SW_TMP = 0;                 // kZoneWaves + 1
constexpr uint32_t SW_TMP2 = 20;               // 2 kZoneWaves
constexpr uint32_t SW_BIG = 52;                // kMaxBig
constexpr uint32_t SW_RED3 = 84;               // 3
constexpr uint32_t SW_NOUT = 88, SW_NTRIG = 89, SW_NBIG = 90, SW_TN = 91, SW_GMAX = 92, SW_NEED = 93;
constexpr uint32_t SW_TN1 = 97;                // the odd rounds' tile fill
constexpr uint32_t SW_GIB = 94;                // u64 pool base (8-B aligned)
constexpr uint32_t SW_GIOK = 96;
static_assert(SW_TMP2 >= kZoneWaves + 1 && SW_BIG >= SW_TMP2 + 2 * kZoneWaves &&
              SW_RED3 >= SW_BIG + kMaxBig && SW_GIOK < kSmallWords, "small words");

__host__ __device__ constexpr uint32_t al4(uint32_t words) { return (words + 3u) & ~3u; }
// byte offset of the fixed part's end (with or without the fan-in accumulators)
__host__ __device__ constexpr uint32_t step_var(bool fan) { return fan ? L_VAR_FAN : L_FAN; }
// byte offset of the shared region for nb outbox buckets and nbp tile buckets
// words of the tile-count array: tile buckets [nbp + 1], reused by phase 4 as
// its per-bucket tile counts [nb]
__host__ __device__ constexpr uint32_t step_tcw(uint32_t nb, uint32_t nbp)
{
  return al4(nbp + 1u > nb ? nbp + 1u : nb);
}
// [nb] outbox histogram, then two tile-count arrays (even / odd rounds). The
// region must hold a tile of a record per thread and the hot-group sort's work
// area; with very many zones it cannot, and every send takes the outbox
// (no tile: step_region without the count arrays, tcap 0).
__host__ __device__ constexpr uint32_t step_region_min()
{
  return (16u * kZoneThreads > kSortWork * 4u) ? 16u * kZoneThreads : kSortWork * 4u;
}
__host__ __device__ constexpr bool step_tiled(bool fan, uint32_t nb, uint32_t nbp)
{
  return step_var(fan) + 4u * (al4(nb) + 2u * step_tcw(nb, nbp)) + step_region_min() <= kLdsDyn;
}
__host__ __device__ constexpr uint32_t step_region(bool fan, uint32_t nb, uint32_t nbp)
{
  return step_var(fan) + 4u * (al4(nb) + (step_tiled(fan, nb, nbp) ? 2u * step_tcw(nb, nbp) : 0u));
}
// LDS tile capacity (records) in a region of `bytes`
__host__ __device__ constexpr uint32_t step_tcap(uint32_t bytes) { return bytes / 16u; }

// Handler tables whose behaviours never read the message (identical pings):
// their zones need the record index only for carried remainders and sorts.
template <int HT> __host__ __device__ constexpr bool ht_reads_msgs()
{
  return !(HT == GPU_ACTOR_HT_PINGER || HT == GPU_ACTOR_HT_FANIN_SENDER);
}

// Inclusive running max of a[0, n) (u16, LDS) by the workgroup. All threads
// call it; it ends behind a barrier.
__device__ void block_maxscan_u16(uint16_t* a, uint32_t n, uint32_t* s_tmp)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t per = (n + kZoneThreads - 1) / kZoneThreads;
  const uint32_t lo = min(tid * per, n), hi = min(lo + per, n);
  uint32_t m = 0;
  for(uint32_t i = lo; i < hi; ++i) m = max(m, (uint32_t)a[i]);
  uint32_t x = m;
#pragma unroll
  for(int off = 1; off < 64; off <<= 1)
  {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off);
    if(lane >= (uint32_t)off) x = max(x, y);
  }
  if(lane == 63) s_tmp[wv] = x;
  __syncthreads();
  if(wv == 0)
  {
    uint32_t y = lane < (uint32_t)kZoneWaves ? s_tmp[lane] : 0u;
#pragma unroll
    for(int off = 1; off < 64; off <<= 1)
    {
      const uint32_t q = (uint32_t)__shfl_up((int)y, off);
      if(lane >= (uint32_t)off) y = max(y, q);
    }
    if(lane < (uint32_t)kZoneWaves) s_tmp[lane] = y;
  }
  __syncthreads();
  const uint32_t xe = (uint32_t)__shfl_up((int)x, 1);
  uint32_t run = max(wv ? s_tmp[wv - 1] : 0u, lane ? xe : 0u);
  for(uint32_t i = lo; i < hi; ++i) { run = max(run, (uint32_t)a[i]); a[i] = (uint16_t)run; }
  __syncthreads();
}

// Sum over the workgroup (all threads call; ends behind a barrier).
__device__ uint32_t block_sum(uint32_t v, uint32_t* s_tmp)
{
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = (uint32_t)wave_sum(v);
  if(lane == 0) s_tmp[wv] = v;
  __syncthreads();
  uint32_t t = 0;
  for(uint32_t w = 0; w < (uint32_t)kZoneWaves; ++w) t += s_tmp[w];
  __syncthreads();
  return t;
}

constexpr int kFlPer = 8;    // tile records per thread at a flush (tcap <= kFlPer * kZoneThreads)

// Two 512-thread workgroups per zone... per CU: minimum waves per SIMD = 2 * 8 / 4 = 4.
// HTS >= 0: every serial actor of this engine runs handler table HTS (the host
// checks), so only that table is compiled in; HTS < 0: any mix of tables.
template <int HTS>
__global__ void __launch_bounds__(kZoneThreads, 4) k_step(uint32_t cur, uint32_t pend_slot,
  uint32_t sidx)
{
  constexpr bool kFan = HTS < 0 || HTS == GPU_ACTOR_HT_FANIN_SENDER;
  constexpr bool kReads = HTS < 0 || ht_reads_msgs<HTS < 0 ? 0 : HTS>();
  extern __shared__ __attribute__((aligned(16))) unsigned char s_lds[];
  uint32_t* const s_off = reinterpret_cast<uint32_t*>(s_lds + L_OFF);   // counts, then offsets
  uint32_t* const s_ccnt = reinterpret_cast<uint32_t*>(s_lds + L_CCNT);
  uint32_t* const s_aux = reinterpret_cast<uint32_t*>(s_lds + L_AUX);
  uint8_t* const s_tb = s_lds + L_TB;
  uint32_t* const s_bigbits = reinterpret_cast<uint32_t*>(s_lds + L_BIGBITS);
  unsigned long long* const s_red = reinterpret_cast<unsigned long long*>(s_lds + L_RED);
  unsigned long long* const s_agg = reinterpret_cast<unsigned long long*>(s_lds + L_AGG);
  unsigned long long* const s_bytype = reinterpret_cast<unsigned long long*>(s_lds + L_BYTYPE);
  uint32_t* const s_sw = reinterpret_cast<uint32_t*>(s_lds + L_SMALL);
  unsigned long long* const s_fan = reinterpret_cast<unsigned long long*>(s_lds + L_FAN);
  uint32_t* const s_tmp = s_sw + SW_TMP;
  uint32_t* const s_tmp2 = s_sw + SW_TMP2;
  uint32_t* const s_big = s_sw + SW_BIG;
  uint32_t* const s_red3 = s_sw + SW_RED3;

  const uint32_t z = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // One rank: a zone buffer overflowed into the spill list. The host grows the
  // zones and lands those records before another step runs; until then every
  // step is a no-op (spill_n[cur] is final for this launch; halt is set only
  // by skipped steps, so every zone of a launch decides alike).
  // With n_ranks > 1 the decision is the spill flag summed over ranks after
  // the last exchange, so every rank halts the same steps.
  const bool halt_now = c_eng.nranks == 1 ? (c_eng.spill_n[cur] != 0u || *c_eng.halt != 0u)
                                          : (*c_eng.spill_flag != 0u);
  if(halt_now)
  {
    if(z == 0 && tid == 0)
    {
      *c_eng.halt = 1u;
      c_eng.pend[pend_slot] = kPendSkipped;
      atomicAdd(c_eng.skipped, 1ull);
    }
    return;
  }
  const uint32_t nxt = cur ^ 1u;
  const uint32_t L0 = z * kZone;
  const uint32_t nact = min(kZone, c_eng.n_local - L0);
  const uint32_t R = c_eng.nranks, me = c_eng.rank;
  const uint32_t nz = c_eng.n_zones;
  const uint32_t nb = nz + (R > 1 ? R : 0u);
  const uint32_t nbp = c_eng.nbp, nper = c_eng.nper;
  const uint32_t cap = zone_capacity(z);
  uint32_t* const s_hist = reinterpret_cast<uint32_t*>(s_lds + step_var(kFan));
  uint32_t* const s_tc = s_hist + al4(nb);
  const uint32_t lds_region = step_region(kFan, nb, nbp);
  unsigned char* const s_reg = s_lds + lds_region;
  const uint32_t reg_bytes = kLdsDyn - lds_region;
  const uint32_t tcap = step_tiled(kFan, nb, nbp)
                        ? min(step_tcap(reg_bytes), (uint32_t)(kFlPer * kZoneThreads)) : 0u;

  if(tid < GPU_ACTOR_MAX_TYPES) s_bytype[tid] = 0;
  if constexpr(kFan)
    for(uint32_t j = tid; j < 2 * kFanLds; j += kZoneThreads) s_fan[j] = 0;

  // Backpressure bookkeeping: ztc = this zone's actors that
  // trigger muting after the last step (overloaded or muted); ztn = nonzero
  // bytes this zone left in trig_own[nxt] two steps ago. trig_n is indexed by
  // step mod 3: read this step's, add to the next's, clear the one after.
  const uint32_t ztc = c_eng.ztrig[cur][z];
  const uint32_t ztn = c_eng.ztrig[nxt][z];
  const bool gate = c_eng.trig_n[sidx % 3u] != 0u;
  if(z == 0 && tid == 0)
  {
    c_eng.trig_n[(sidx + 2u) % 3u] = 0u;
    c_eng.gi_n[(sidx + 1u) & 1u] = 0ull;      // the next step's record-index pool
  }
  uint8_t* const tb_out = c_eng.trig_own[nxt];

  for(uint32_t i = tid; i < kZone + 4; i += kZoneThreads) s_off[i] = 0;
  for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_ccnt[i] = 0;
  for(uint32_t b = tid; b < nb; b += kZoneThreads) s_hist[b] = 0;
  const uint32_t tcw = step_tcw(nb, nbp);
  if(tcap)
    for(uint32_t b = tid; b < tcw; b += kZoneThreads) s_tc[b] = 0;
  for(uint32_t k = tid; k < kZone / 32; k += kZoneThreads) s_bigbits[k] = 0;
  GPA_STAMP(0);
  if(tid == 0)
  {
    s_sw[SW_NOUT] = 0; s_sw[SW_NTRIG] = 0; s_sw[SW_NBIG] = 0; s_sw[SW_TN] = 0; s_sw[SW_GMAX] = 0;
    s_sw[SW_TN1] = 0;
    s_sw[SW_NEED] = (kReads || gate || ztc) ? 1u : 0u;
  }

  // ---- 0. this zone's segment of every tile sent to it last step ---------------------
  // slot g = sender zone s * kMaxT + tile t: its count and first record in
  // P[cur]; s_pre = exclusive scan of the counts (np = records pulled). When
  // the table does not fit the region (very many zones) only the total is
  // taken here and the slow path walks the slots in chunks.
  const uint32_t bz = xcd_slot(z, nper);
  const uint32_t nseg = nz * kMaxT;
  uint32_t* const s_pre = reinterpret_cast<uint32_t*>(s_reg);
  uint32_t* const s_pst = s_pre + al4(nseg + 1);
  const uint32_t seg_bytes = 4u * (al4(nseg + 1) + al4(nseg));
  const bool seg_fit = seg_bytes <= reg_bytes;
  // a tile its sender did not fill this step has an all-zero directory
  auto seg_at = [&](uint32_t gs, uint32_t& c, uint32_t& st) __attribute__((always_inline)) {
    const uint32_t s = gs / kMaxT;
    const uint16_t* d = c_eng.pdir[cur] + (size_t)gs * (nbp + 2u);
    const uint32_t lo = d[bz], hi = d[bz + 1], tb = d[nbp + 1];
    c = hi - lo;
    st = s * c_eng.pcap + tb + lo;
  };
  uint32_t np;
  if(seg_fit)
  {
    for(uint32_t gs = tid; gs < nseg; gs += kZoneThreads)
    {
      uint32_t c, st;
      seg_at(gs, c, st);
      s_pre[gs] = c;
      s_pst[gs] = st;
    }
    __syncthreads();
    np = block_scan_n(s_pre, s_pre, nseg, s_tmp);
    if(tid == 0) s_pre[nseg] = np;
  }
  else
  {
    uint32_t sum = 0;
    for(uint32_t gs = tid; gs < nseg; gs += kZoneThreads)
    {
      uint32_t c, st;
      seg_at(gs, c, st);
      sum += c;
    }
    np = block_sum(sum, s_tmp);
  }
  GPA_STAMP(1);

  // ---- 1. count --------------------------------------------------------------
  const uint32_t nc = min(c_eng.carry_n[cur][z], cap);
  const uint32_t nl = min(c_eng.land_n[cur][z], cap);
  const uint32_t na = nl + np;                 // arrivals: landed, then pulled
  if(nc + na == 0 && ztc == 0)
  {
    // an idle zone (uniform: every thread read the same counters) has
    // nothing to count, run or send — the quiet tail of a run, or zones of
    // a sparse workload; it only clears trigger bytes it left two steps ago
    if(tid == 0)
    {
      c_eng.carry_n[nxt][z] = 0;
      c_eng.pntile[nxt][z] = 0;
      c_eng.pn[nxt][z] = 0;
    }
    {
      uint16_t* const d = c_eng.pdir[nxt] + (size_t)z * kMaxT * (nbp + 2u);
      for(uint32_t j = tid; j < kMaxT * (nbp + 2u); j += kZoneThreads) d[j] = 0;
    }
    if(ztn)
    {
      for(uint32_t i = tid; i < nact; i += kZoneThreads) tb_out[(L0 + i) * R + me] = 0;
      if(tid == 0) c_eng.ztrig[nxt][z] = 0;
    }
    return;
  }
  // the trigger bytes of this zone's actors as the last step left them
  if(ztc)
    for(uint32_t i = tid; i < kZone; i += kZoneThreads)
      s_tb[i] = i < nact ? c_eng.trig[cur][(L0 + i) * R + me] : (uint8_t)0;
  else
    for(uint32_t i = tid; i < kZone / 4; i += kZoneThreads)
      reinterpret_cast<uint32_t*>(s_tb)[i] = 0;
  const ZRec* C = c_eng.carry[cur] + c_eng.zoff[z];
  const ZRec* Ld = c_eng.land[cur] + c_eng.zoff[z];
  const ZRec* Pc = c_eng.P[cur];
  // fast path: the segment table fits, arrivals fit the registers, pulled
  // record u -> its segment through marks at segment starts and a running max
  uint16_t* const s_mark = reinterpret_cast<uint16_t*>(s_reg + seg_bytes);
  const uint32_t mark_cap = seg_fit ? (reg_bytes - seg_bytes) / 2u : 0u;
  const bool fast = seg_fit && nc + na <= kIdxCap && np <= mark_cap;   // uniform
  if(fast && np)
  {
    for(uint32_t u = tid; u < np; u += kZoneThreads) s_mark[u] = 0;
    __syncthreads();
    for(uint32_t gs = tid; gs < nseg; gs += kZoneThreads)
      if(s_pre[gs + 1] != s_pre[gs]) s_mark[s_pre[gs]] = (uint16_t)gs;
    __syncthreads();
    block_maxscan_u16(s_mark, np, s_tmp);
  }
  else
    __syncthreads();
  auto e_w0 = [&](uint32_t e) __attribute__((always_inline)) -> uint32_t {
    return (e & kGiPull) ? Pc[e & ~kGiPull].w0 : Ld[e].w0;
  };
  // fast path: GI entry of arrival v
  auto arr_e = [&](uint32_t v) __attribute__((always_inline)) -> uint32_t {
    if(v < nl) return v;
    const uint32_t u = v - nl;
    const uint32_t gs = s_mark[u];
    return kGiPull | (s_pst[gs] + (u - s_pre[gs]));
  };
  // slow path: f(GI entry) for every pulled record, the slots taken in chunks
  // whose table fits the region (binary search per record)
  auto for_pulled = [&](auto&& f) __attribute__((always_inline)) {
    const uint32_t chunk = min(nseg, (reg_bytes / 8u) - 8u);
    for(uint32_t g0 = 0; g0 < nseg; g0 += chunk)
    {
      const uint32_t m = min(chunk, nseg - g0);
      uint32_t* const t_pre = reinterpret_cast<uint32_t*>(s_reg);
      uint32_t* const t_pst = t_pre + al4(m + 1);
      __syncthreads();                         // the last chunk's table is no longer read
      for(uint32_t k = tid; k < m; k += kZoneThreads)
      {
        uint32_t c, st;
        seg_at(g0 + k, c, st);
        t_pre[k] = c;
        t_pst[k] = st;
      }
      __syncthreads();
      const uint32_t cn = block_scan_n(t_pre, t_pre, m, s_tmp);
      for(uint32_t u = tid; u < cn; u += kZoneThreads)
      {
        uint32_t lo = 0, hi = m;               // t_pre[lo] <= u < t_pre[hi] (= cn)
        while(hi - lo > 1)
        {
          const uint32_t q = (lo + hi) >> 1;
          if(t_pre[q] <= u) lo = q; else hi = q;
        }
        f(kGiPull | (t_pst[lo] + (u - t_pre[lo])));
      }
    }
    __syncthreads();
  };
  // carried records counted apart (s_ccnt); arrivals in s_off (the counts)
  for(uint32_t i = tid; i < nc; i += kZoneThreads)
    atomicAdd(&s_ccnt[C[i].w0 & kZoneMask], 1u);
  // Arrivals: on the fast path each record's rank among its actor's arrivals
  // comes back from the counting atomic and stays in a register (packed
  // rank << 11 | actor), so placing it needs no second pass over the records.
  // kIdxPer loads in flight per thread.
  uint32_t wr[kIdxPer];
  if(fast)
  {
    // in three batches, so that the LDS reads and then the loads of all of a
    // thread's records are in flight together: segment of each pulled record,
    // its GI entry, its first word
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
    {
      const uint32_t v = u * kZoneThreads + tid;
      wr[u] = v >= nl && v < na ? s_mark[v - nl] : 0u;
    }
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
    {
      const uint32_t v = u * kZoneThreads + tid;
      wr[u] = v < nl ? v
            : v < na ? kGiPull | (s_pst[wr[u]] + (v - nl - s_pre[wr[u]]))
            : 0xFFFFFFFFu;
    }
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
      wr[u] = wr[u] != 0xFFFFFFFFu ? e_w0(wr[u]) : 0xFFFFFFFFu;
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
      if(wr[u] != 0xFFFFFFFFu)
      {
        const uint32_t act = wr[u] & kZoneMask;
        wr[u] = (atomicAdd(&s_off[act], 1u) << kZoneBits) | act;
      }
  }
  else
  {
    for(uint32_t v = tid; v < nl; v += kZoneThreads) atomicAdd(&s_off[Ld[v].w0 & kZoneMask], 1u);
    for_pulled([&](uint32_t e) { atomicAdd(&s_off[e_w0(e) & kZoneMask], 1u); });
  }
  __syncthreads();
  GPA_STAMP(2);
  if(tid == 0)
  {
    atomicAdd(&c_eng.pend[pend_slot], (unsigned long long)(nc + na));
    c_eng.carry_n[cur][z] = 0;
    c_eng.land_n[cur][z] = 0;
  }
  // counts -> segment offsets (in place), carry starts in s_aux; s_off[kZone] = total
  block_scan_zone_pair(s_off, s_ccnt, s_off, s_aux, s_tmp2);
  if(tid == 0) s_off[kZone] = nc + na;
  __syncthreads();
  auto n_of = [&](uint32_t i) __attribute__((always_inline)) { return s_off[i + 1] - s_off[i]; };
  // The zone's type when one type covers all of its slots, else -1. It is
  // wave-uniform, so that type's fields (batch, state, params) come through
  // scalar loads instead of a per-lane lookup chain.
  int tz = -1;
  for(uint32_t t = 0; t < c_eng.n_types; ++t)
    if(L0 >= c_types[t].lfirst && L0 + nact <= c_types[t].lfirst + c_types[t].lcount)
      tz = (int)t;
  tz = __builtin_amdgcn_readfirstlane(tz);
  // hot receivers (groups above kBigGroup, sorted by the whole workgroup), and
  // whether this zone's behaviours need the record index at all: a behaviour
  // that reads its message, a group the lane orders (more than the 16 held in
  // registers), a remainder to carry (more than a batch), muting
  {
    const uint32_t bmin = tz >= 0 ? c_types[tz].batch : 0u;
    uint32_t need = 0;
    for(uint32_t i = tid; i < nact; i += kZoneThreads)
    {
      const uint32_t n = n_of(i), g = n - s_ccnt[i];
      if(g > kBigGroup)
      {
        const uint32_t k = atomicAdd(&s_sw[SW_NBIG], 1u);
        if(k < kMaxBig)
        {
          s_big[k] = i;
          atomicMax(&s_sw[SW_GMAX], g);
        }
      }
      need |= (g > 16u || n > bmin) ? 1u : 0u;
    }
    if(need) s_sw[SW_NEED] = 1u;
  }
  __syncthreads();
  const uint32_t nbig = min(s_sw[SW_NBIG], kMaxBig);   // past kMaxBig: the lane sorts (slow, exact)
  const uint32_t gmax = s_sw[SW_GMAX];
  const bool need_gi = s_sw[SW_NEED] != 0u;
  // this step's record index (and sort scratch) from the pool
  const uint32_t ngi = need_gi ? (nc + na + 1u) & ~1u : 0u;
  if(tid == 0)
  {
    // even sizes keep every base 8-B aligned for the sort's u64 items
    const unsigned long long need = ngi + (nbig ? (5ull * gmax + 3ull) & ~1ull : 0ull);
    const unsigned long long base = need ? atomicAdd(&c_eng.gi_n[sidx & 1u], need) : 0ull;
    *reinterpret_cast<unsigned long long*>(s_sw + SW_GIB) = base;
    s_sw[SW_GIOK] = base + need <= c_eng.gi_cap ? 1u : 0u;
  }
  __syncthreads();
  if(!s_sw[SW_GIOK])
  {
    // cannot happen: the pool holds every record a step can have in flight
    if(tid == 0) atomicAdd(&c_eng.stats[ST_DROPPED], (unsigned long long)(nc + na));
    return;
  }
  uint32_t* const GI = c_eng.gi + *reinterpret_cast<const unsigned long long*>(s_sw + SW_GIB);
  GPA_STAMP(3);

  // ---- 2. place: GI in segment order (only where a behaviour or the carry will
  //      read it) -----------------------------------------------------------------------
  if(need_gi)
  {
    for(uint32_t i = tid; i < nc; i += kZoneThreads)
    {
      const uint32_t a = C[i].w0 & kZoneMask;
      GI[s_off[a] + (i - s_aux[a])] = kGiCarry | i;
    }
    if(fast)
    {
#pragma unroll
      for(int u = 0; u < kIdxPer; ++u)
        if(wr[u] != 0xFFFFFFFFu)
        {
          const uint32_t act = wr[u] & kZoneMask;
          GI[s_off[act] + s_ccnt[act] + (wr[u] >> kZoneBits)] = arr_e(u * kZoneThreads + tid);
        }
    }
    else
    {
      __syncthreads();
      for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_aux[i] = 0;
      __syncthreads();
      auto put = [&](uint32_t e) __attribute__((always_inline)) {
        const uint32_t a = e_w0(e) & kZoneMask;
        GI[s_off[a] + s_ccnt[a] + atomicAdd(&s_aux[a], 1u)] = e;
      };
      for(uint32_t v = tid; v < nl; v += kZoneThreads) put(v);
      for_pulled(put);
    }
  }
  __syncthreads();
  GPA_STAMP(4);

  // Hot receivers: their groups sorted by the whole workgroup (s_bigbits
  // marks them for drain_zone); the sort's work area is the LDS region, its
  // items in the pool after GI.
  if(nbig)
  {
    uint64_t* ia = reinterpret_cast<uint64_t*>(GI + ngi);
    uint64_t* ib = ia + gmax;
    uint32_t* tmp = reinterpret_cast<uint32_t*>(ib + gmax);
    for(uint32_t k = 0; k < nbig; ++k)
    {
      const uint32_t i = s_big[k];
      const uint32_t g = n_of(i) - s_ccnt[i];
      const bool ok = coop_sort_group(AccG{GI + s_off[i], C, Ld, Pc}, s_ccnt[i], g, ia, ib, tmp,
                                      reinterpret_cast<uint32_t*>(s_reg), s_red3);
      if(ok && tid == 0) s_bigbits[i >> 5] |= 1u << (i & 31);
    }
    __syncthreads();
  }
  auto big_sorted = [&](uint32_t i) __attribute__((always_inline)) {
    return ((s_bigbits[i >> 5] >> (i & 31)) & 1u) != 0u;
  };

  // s_aux will hold each actor's unhandled remainder (known after it ran)
  for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_aux[i] = 0;
  int any_rem = 0;

  // ---- 3. run handlers, one actor per thread per round; each round's local
  //      sends sorted in the LDS tile and written to this zone's send region ---------
  uint4* const s_tile = reinterpret_cast<uint4*>(s_reg);
  ZoneCtx a;
  a.reset_common();
  a.out = c_eng.O + c_eng.zoff[z];
  a.s_nout = &s_sw[SW_NOUT];
  a.ocap = cap;
  a.nxt = nxt;
  a.s_hist = s_hist;
  a.agg = &s_agg[wv];
  a.s_tile = s_tile;
  a.s_tn = &s_sw[SW_TN];
  a.tcap = tcap;
  // fan-in senders fold their analyzer applies per zone in LDS
  if constexpr(kFan)
    if(tz >= 0 && c_types[tz].ht == GPU_ACTOR_HT_FANIN_SENDER)
    {
      a.fan_t = type_of_global((uint32_t)c_types[tz].params[1]);
      if(a.fan_t >= 0) a.fan = s_fan;
    }
  uint32_t delivered = 0, active = 0, sent = 0, applied = 0;
  // drain local actor i, of type t (T = c_types[t])
  uint8_t* const trig_cur = gate ? c_eng.trig[cur] : nullptr;
  auto drain_actor = [&](const TypeDev& T, int t, uint32_t i) __attribute__((always_inline)) {
    const uint32_t n = n_of(i);
    const uint32_t L = L0 + i;
    a.li = L - T.lfirst;
    a.self = L * R + me;
    a.src_local = i;
    a.type = t;
    a.seq = 0;
    // backpressure: as the last step left this actor (bit 0 overloaded, bit
    // 1 muted); a muted actor waits while the receiver it is muted on is
    // overloaded (the release of ponyint_actor_unsetoverloaded, actor.c:1121)
    const uint32_t tb = s_tb[i];
    a.trig = trig_cur;
    a.prev_o = tb & 1u;
    a.mute_hit = 0;
    a.yield_req = 0;
    const bool stays = (tb & 2u) && (c_eng.trig[cur][c_eng.muted_on[L]] & 1u);
    uint32_t d = 0;
    const AccG acc{GI + s_off[i], C, Ld, Pc};
#define ZDRAIN(HT) d = zone_actor<HT>(T, a, acc, n, s_ccnt[i], stays, big_sorted(i));
    if constexpr(HTS >= 0)
    {
      ZDRAIN(HTS)
    }
    else
    {
      switch(T.ht)
      {
#define ZCASE(HT) case HT: { ZDRAIN(HT) } break;
        ZCASE(GPU_ACTOR_HT_RING)
        ZCASE(GPU_ACTOR_HT_PINGER)
        ZCASE(GPU_ACTOR_HT_PINGER_DET)
        ZCASE(GPU_ACTOR_HT_FANIN_SENDER)
        ZCASE(GPU_ACTOR_HT_GUPS_STREAMER)
        ZCASE(GPU_ACTOR_HT_STORM)
        ZCASE(GPU_ACTOR_HT_FIFO_SRC)
        ZCASE(GPU_ACTOR_HT_FIFO_SINK)
        ZCASE(GPU_ACTOR_HT_SPREADER)
#undef ZCASE
        default: break;
      }
    }
#undef ZDRAIN
    // overloaded iff a full batch ran and the actor was not muted
    // (batch_limit_reached, actor.c:369-381; maybe_mute first, 449-460)
    const uint32_t o = (d == T.batch && !a.mute_hit) ? 1u : 0u;
    const uint32_t m = (stays || a.mute_hit) ? 1u : 0u;
    if(a.mute_hit) c_eng.muted_on[L] = a.mute_to;
    const uint32_t nb_ = o | (m << 1);
    s_tb[i] = (uint8_t)nb_;
    if(nb_) atomicAdd(&s_sw[SW_NTRIG], 1u);
    s_aux[i] = n - d;
    any_rem |= (n - d) != 0u;
    delivered += d;
    active += d ? 1u : 0u;
    return d;
  };
  // Round r's tile: counting-sorted by XCD-major bucket slot (ranks from LDS
  // atomics, starts = exclusive scan of the counts), converted to landing
  // format and written to the send region at `cursor`; its bucket starts and
  // offset to the directory. Counters alternate between even and odd rounds:
  // a flush clears the next round's (their last reader passed the barrier
  // before it). Every thread calls it after the round's barrier.
  uint32_t tix = 0, cursor = 0;
  auto flush = [&](uint32_t r) __attribute__((always_inline)) {
    uint32_t* const tc = s_tc + (r & 1u) * tcw;
    uint32_t* const tc_next = s_tc + ((r + 1u) & 1u) * tcw;
    const uint32_t n = min(s_sw[(r & 1u) ? SW_TN1 : SW_TN], tcap);
    for(uint32_t j = tid; j < tcw; j += kZoneThreads) tc_next[j] = 0;
    if(tid == 0) s_sw[(r & 1u) ? SW_TN : SW_TN1] = 0;
    if(n == 0)
    {
      __syncthreads();
      return;
    }
    // the records go to registers here: the next round refills the tile as
    // soon as the scan's last barrier is passed
    uint32_t bk[kFlPer];
    uint4 rv[kFlPer];
#pragma unroll
    for(int u = 0; u < kFlPer; ++u)
    {
      const uint32_t slot = u * kZoneThreads + tid;
      if(slot < n)
      {
        rv[u] = s_tile[slot];
        const uint32_t bp = xcd_slot(rdiv(rv[u].x) >> kZoneBits, nper);
        bk[u] = bp << 16 | atomicAdd(&tc[bp], 1u);
      }
    }
    __syncthreads();
    (void)block_scan_n(tc, tc, nbp, s_tmp);
    ZRec* const Pz = c_eng.P[nxt] + (size_t)z * c_eng.pcap + cursor;
#pragma unroll
    for(int u = 0; u < kFlPer; ++u)
    {
      const uint32_t slot = u * kZoneThreads + tid;
      if(slot < n)
      {
        const uint4 r4 = rv[u];
        uint4 v;
        v.x = (r4.y & ~kZoneMask) | (rdiv(r4.x) & kZoneMask);
        v.y = (L0 + (r4.y & kZoneMask)) * R + me;
        v.z = r4.z;
        v.w = r4.w;
        st16(reinterpret_cast<uint4*>(Pz + tc[bk[u] >> 16] + (bk[u] & 0xFFFFu)), v);
      }
    }
    uint16_t* const d = c_eng.pdir[nxt] + (size_t)(z * kMaxT + tix) * (nbp + 2u);
    for(uint32_t j = tid; j < nbp; j += kZoneThreads) d[j] = (uint16_t)tc[j];
    if(tid == 0)
    {
      d[nbp] = (uint16_t)n;
      d[nbp + 1] = (uint16_t)cursor;
      c_eng.ptbase[nxt][z * kMaxT + tix] = cursor;
    }
    cursor += n;
    ++tix;
  };
  uint32_t dz = 0;
  const bool zred = tz >= 0 && c_types[tz].reducible;
  for(uint32_t r = 0; r < kMaxT; ++r)
  {
    a.s_tn = &s_sw[(r & 1u) ? SW_TN1 : SW_TN];
    const uint32_t i = r * kZoneThreads + tid;
    if(i < nact && !zred && (n_of(i) || s_tb[i]))
    {
      if(tz >= 0)
        dz += drain_actor(c_types[tz], tz, i);
      else
      {
        const int t = type_of_local(L0 + i);
        if(t >= 0 && !c_types[t].reducible)
        {
          const uint32_t d = drain_actor(c_types[t], t, i);
          if(d) atomicAdd(&s_bytype[t], (unsigned long long)d);
        }
      }
    }
    __syncthreads();
    GPA_STAMP(8 + 2 * r);
    flush(r);
    GPA_STAMP(9 + 2 * r);
  }
  // the tiles this zone did not fill: empty directories
  for(uint32_t t = tix; t < kMaxT; ++t)
  {
    uint16_t* const d = c_eng.pdir[nxt] + (size_t)(z * kMaxT + t) * (nbp + 2u);
    for(uint32_t j = tid; j < nbp + 2u; j += kZoneThreads) d[j] = 0;
  }
  if(tz >= 0 && dz) atomicAdd(&s_bytype[tz], (unsigned long long)dz);
  GPA_STAMP(5);
  if(tid == 0)
  {
    c_eng.pntile[nxt][z] = tix;
    c_eng.pn[nxt][z] = cursor;
  }
  sent = a.sent;
  applied = a.applied;
  if(applied && a.applied_type >= 0)
    atomicAdd(&s_bytype[a.applied_type], (unsigned long long)applied);
  // ---- 3b. carry-out: every actor's unhandled remainder, canonical, to the
  //      next step's carry buffer (none in the usual step) -----------------------------
  uint32_t ncout = 0;
  if(__syncthreads_or(any_rem))
  {
    ncout = block_scan_zone(s_aux, s_tmp);
    if(tid == 0) s_sw[SW_NBIG] = 0;
    __syncthreads();
    for(uint32_t i = tid; i < nact; i += kZoneThreads)
    {
      const uint32_t co = s_aux[i];
      const uint32_t rem = (i + 1 < kZone ? s_aux[i + 1] : ncout) - co;
      if(rem == 0) continue;
      if(rem > kBigGroup)
      {
        // a backlog (an overloaded receiver): copied by the whole workgroup
        const uint32_t k = atomicAdd(&s_sw[SW_NBIG], 1u);
        if(k < kMaxBig) { s_big[k] = i; continue; }
      }
      const uint32_t n = n_of(i);
      carry_out(AccG{GI + s_off[i], C, Ld, Pc}, n - rem, n, z, co, nxt);
    }
    __syncthreads();
    const uint32_t nbl = min(s_sw[SW_NBIG], kMaxBig);
    for(uint32_t k = 0; k < nbl; ++k)
    {
      const uint32_t i = s_big[k];
      const uint32_t co = s_aux[i];
      const uint32_t rem = (i + 1 < kZone ? s_aux[i + 1] : ncout) - co;
      const uint32_t n = n_of(i);
      const AccG acc{GI + s_off[i], C, Ld, Pc};
      ZRec* cout = c_eng.carry[nxt] + c_eng.zoff[z];
      for(uint32_t j = tid; j < rem; j += kZoneThreads)
      {
        const ZRec r = acc.rec(n - rem + j);
        uint4 u;
        u.x = r.w0; u.y = r.from; u.z = (uint32_t)r.arg; u.w = (uint32_t)(r.arg >> 32);
        const uint32_t pos = co + j;
        if(pos < cap)
          *reinterpret_cast<uint4*>(cout + pos) = u;
        else
          spill_rec(nxt, kSpillCarry, z, pos, u);
      }
    }
  }
  if(tid == 0) c_eng.carry_n[nxt][z] = ncout;   // past cap: the tail is in the spill list
  // trigger bytes for the next step (only where some are set, or were)
  const uint32_t ntrig = s_sw[SW_NTRIG];
  if(ntrig || ztn)
  {
    if(R == 1)
      for(uint32_t i = tid; i < kZone / 4; i += kZoneThreads)
      {
        if(4 * i < nact)
          reinterpret_cast<uint32_t*>(tb_out + L0)[i] = reinterpret_cast<const uint32_t*>(s_tb)[i];
      }
    else
      for(uint32_t i = tid; i < nact; i += kZoneThreads) tb_out[(L0 + i) * R + me] = s_tb[i];
    if(tid == 0)
    {
      c_eng.ztrig[nxt][z] = ntrig;
      if(ntrig) atomicAdd(&c_eng.trig_n[(sidx + 1u) % 3u], ntrig);
    }
  }
  __syncthreads();
  GPA_STAMP(6);
  if(tid < GPU_ACTOR_MAX_TYPES && s_bytype[tid])
    atomicAdd(&c_eng.stats[ST_BY_TYPE + tid], s_bytype[tid]);
  if constexpr(kFan)
    if(a.fan)
    {
      const TypeDev& F = c_types[a.fan_t];
      for(uint32_t j = tid; j < kFanLds && j < F.lcount; j += kZoneThreads)
        if(s_fan[j])
        {
          atomicAdd(reinterpret_cast<unsigned long long*>(&F.state[j]), s_fan[j]);
          atomicXor(reinterpret_cast<unsigned long long*>(&F.state[(size_t)F.lcount + j]),
            s_fan[kFanLds + j]);
        }
    }

  // ---- 4. the outbox (remote sends, tile overflow): one chunk per destination
  //      bucket, sorted in LDS tiles ----------------------------------------------------
  const uint32_t nout = min(s_sw[SW_NOUT], cap);
  uint32_t n_atom = 0, xover = 0;
  if(nout)
  {
    uint32_t* s_base = reinterpret_cast<uint32_t*>(s_reg);   // chunk base per bucket (region free again)
    const uint32_t nbw0 = tcap ? al4(nb) : 2u * al4(nb);
    uint32_t* s_tcnt = tcap ? s_tc : s_base + al4(nb);   // records of the tile per bucket
    uint32_t* s_tst = s_base + nbw0;        // bucket start within the sorted tile (tiled only)
    const uint32_t nbw = nbw0 + al4(nb);    // words of the bucket arrays in the region
    uint4* s_pool = reinterpret_cast<uint4*>(s_base + nbw);
    // the outbox sort tile, when the region holds one of at least a record per thread
    const bool tiled = reg_bytes >= 4u * nbw + 16u * kZoneThreads;
    const uint32_t ptile = tiled ? min(kTile, (reg_bytes - 4u * nbw) / 16u) : 0u;
    for(uint32_t b = tid; b < nb; b += kZoneThreads)
    {
      const uint32_t h = s_hist[b];
      if(h)
      {
        ++n_atom;
        if(b < nz)
          s_base[b] = atomicAdd(&c_eng.land_n[nxt][b], h);
        else
          s_base[b] = (uint32_t)atomicAdd(&c_eng.xcount[b - nz], (unsigned long long)h);
      }
      s_tcnt[b] = 0;
    }
    __syncthreads();
    const ORec* Oz = c_eng.O + c_eng.zoff[z];
    // r = {to, w, arg lo, arg hi} -> position pos of bucket b's chunk
    auto emit = [&](const uint4& r, uint32_t b, uint32_t pos) __attribute__((always_inline)) {
      const uint32_t from = (L0 + (r.y & kZoneMask)) * R + me;
      if(b < nz)
      {
        uint4 v;
        v.x = (r.y & ~kZoneMask) | (rdiv(r.x) & kZoneMask);
        v.y = from;
        v.z = r.z;
        v.w = r.w;
        if(pos < zone_capacity(b))
          st16(reinterpret_cast<uint4*>(c_eng.land[nxt] + c_eng.zoff[b] + pos), v);
        else
          spill_rec(nxt, 0u, b, pos, v);
      }
      else
      {
        if(pos < c_eng.xcap)
        {
          c_eng.xout[(size_t)(b - nz) * c_eng.xcap + pos] =
            xpack(r.x, r.y & ~kZoneMask, from, ((uint64_t)r.w << 32) | r.z);
        }
        else
          ++xover;
      }
    };
    if(nout <= kZoneThreads || !tiled)
    {
      // a sparse step (at most one record per thread), or no room for a tile:
      // rank each record in its bucket and store it straight away — the tile
      // sort only groups stores into runs, and a chunk's order is free
      // (receivers order by key)
      for(uint32_t i = tid; i < nout; i += kZoneThreads)
      {
        const uint4 r = ld16(reinterpret_cast<const uint4*>(Oz + i));
        const uint32_t b = bucket_of(r.x);
        emit(r, b, s_base[b] + atomicAdd(&s_tcnt[b], 1u));
      }
    }
    else
    for(uint32_t t0 = 0; t0 < nout; t0 += ptile)
    {
      const uint32_t m = min(ptile, nout - t0);
      uint4 ov[kTilePer];
      uint32_t bk[kTilePer], rk[kTilePer];
#pragma unroll
      for(int u = 0; u < kTilePer; ++u)
      {
        const uint32_t i = u * kZoneThreads + tid;
        if(i < m) ov[u] = ld16(reinterpret_cast<const uint4*>(Oz + t0 + i));
      }
#pragma unroll
      for(int u = 0; u < kTilePer; ++u)
      {
        const uint32_t i = u * kZoneThreads + tid;
        if(i < m)
        {
          bk[u] = bucket_of(ov[u].x);
          rk[u] = atomicAdd(&s_tcnt[bk[u]], 1u);
        }
      }
      __syncthreads();
      (void)block_scan_n(s_tcnt, s_tst, nb, s_tmp);
#pragma unroll
      for(int u = 0; u < kTilePer; ++u)
      {
        const uint32_t i = u * kZoneThreads + tid;
        if(i < m) s_pool[s_tst[bk[u]] + rk[u]] = ov[u];
      }
      __syncthreads();
      for(uint32_t p = tid; p < m; p += kZoneThreads)
      {
        const uint4 r = s_pool[p];
        const uint32_t b = bucket_of(r.x);
        emit(r, b, s_base[b] + (p - s_tst[b]));
      }
      __syncthreads();
      for(uint32_t b = tid; b < nb; b += kZoneThreads)
      {
        s_base[b] += s_tcnt[b];
        s_tcnt[b] = 0;
      }
      __syncthreads();
    }
  }

  // ---- counters: block reduction, one atomic per workgroup per counter ---------------
  unsigned long long v[6] = { delivered + applied, sent, active, 0ull, xover, n_atom };
#pragma unroll
  for(int k = 0; k < 6; ++k)
  {
    v[k] = wave_sum(v[k]);
    if(lane == 0) s_red[wv * 6 + k] = v[k];
  }
  __syncthreads();
  GPA_STAMP(7);
  if(tid < 6)
  {
    unsigned long long tot = 0;
    for(int w = 0; w < kZoneWaves; ++w) tot += s_red[w * 6 + tid];
    const int idx = tid == 0 ? ST_DELIVERED : tid == 1 ? ST_SENT : tid == 2 ? ST_ACTIVE
                  : tid == 3 ? ST_DROPPED : tid == 4 ? ST_XCHG_OVERFLOW : ST_ATOMICS;
    if(tot) atomicAdd(&c_eng.stats[idx], tot);
  }
}

// Pending mail (carried + landed + pulled) for parity `cur`, summed into pend[slot].
__global__ void __launch_bounds__(kBlock) k_pending(uint32_t cur, uint32_t slot)
{
  __shared__ unsigned long long s_red[kWaves];
  const uint32_t z = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long p = 0;
  if(z < c_eng.n_zones)
  {
    const uint32_t cap = zone_capacity(z);
    p = min(c_eng.carry_n[cur][z], cap) + min(c_eng.land_n[cur][z], cap) + c_eng.pn[cur][z];
  }
  p = wave_sum(p);
  if(__lane_id() == 0) s_red[threadIdx.x >> 6] = p;
  __syncthreads();
  if(threadIdx.x == 0)
  {
    unsigned long long tot = 0;
    for(int w = 0; w < kWaves; ++w) tot += s_red[w];
    if(tot) atomicAdd(&c_eng.pend[slot], tot);
  }
}

// Every record in the send regions of parity `cur` pushed into the landing
// buffers (one atomic each), for the paths that read only landing buffers:
// k_sparse, and a re-layout that changes the zone count. Block = one tile
// (sender zone s = blockIdx.x / kMaxT). The host clears pntile / pn after.
__global__ void __launch_bounds__(kBlock) k_pull_land(uint32_t cur)
{
  const uint32_t s = blockIdx.x / kMaxT, t = blockIdx.x % kMaxT;
  if(s >= c_eng.n_zones || t >= c_eng.pntile[cur][s]) return;
  const uint32_t nbp = c_eng.nbp, nper = c_eng.nper;
  const uint16_t* d = c_eng.pdir[cur] + (size_t)blockIdx.x * (nbp + 2u);
  const uint32_t n = d[nbp];
  const ZRec* src = c_eng.P[cur] + (size_t)s * c_eng.pcap + c_eng.ptbase[cur][blockIdx.x];
  for(uint32_t o = threadIdx.x; o < n; o += kBlock)
  {
    uint32_t lo = 0, hi = nbp;                 // d[lo] <= o < d[hi]
    while(hi - lo > 1)
    {
      const uint32_t m = (lo + hi) >> 1;
      if(d[m] <= o) lo = m; else hi = m;
    }
    const uint32_t b = (lo % nper) * 8u + lo / nper;
    const uint4 v = *reinterpret_cast<const uint4*>(src + o);
    const uint32_t pos = atomicAdd(&c_eng.land_n[cur][b], 1u);
    land_store(cur, b, pos, v);
  }
}

// Landing of records addressed to this rank's serial actors (host sends,
// records from other ranks): a block of kLandThreads threads takes
// kLandPer records each, counts them per destination zone in LDS, reserves one
// chunk per (block, zone) with a single atomicAdd, and writes them into it —
// ~kLandThreads * kLandPer / n_zones records per atomic instead of one.
constexpr int kLandThreads = 1024;
constexpr int kLandPer = 8;
constexpr uint32_t kLandRecs = kLandThreads * kLandPer;

struct LandRec {
  bool valid;
  uint32_t to, w, from;
  uint64_t arg;
};

__device__ __forceinline__ void land_records(LandRec (&r)[kLandPer], uint32_t cur,
  uint32_t* s_hist, uint32_t* s_base)
{
  const uint32_t nz = c_eng.n_zones;
  for(uint32_t b = threadIdx.x; b < nz; b += kLandThreads) s_hist[b] = 0;
  __syncthreads();
  uint32_t zt[kLandPer], rk[kLandPer];
#pragma unroll
  for(int u = 0; u < kLandPer; ++u)
    if(r[u].valid)
    {
      zt[u] = rdiv(r[u].to) >> kZoneBits;
      rk[u] = atomicAdd(&s_hist[zt[u]], 1u);
    }
  __syncthreads();
  for(uint32_t b = threadIdx.x; b < nz; b += kLandThreads)
    if(s_hist[b]) s_base[b] = atomicAdd(&c_eng.land_n[cur][b], s_hist[b]);
  __syncthreads();
#pragma unroll
  for(int u = 0; u < kLandPer; ++u)
    if(r[u].valid)
    {
      const uint32_t pos = s_base[zt[u]] + rk[u];
      uint4 v;
      v.x = r[u].w | (rdiv(r[u].to) & kZoneMask);
      v.y = r[u].from;
      v.z = (uint32_t)r[u].arg;
      v.w = (uint32_t)(r[u].arg >> 32);
      land_store(cur, zt[u], pos, v);
    }
}

// Host sends (pony_sendv from outside the runtime): hseq gives the canonical
// order; host senders rank above every actor id.
__global__ void __launch_bounds__(kLandThreads) k_inject(const gpu_msg_t* msgs, uint64_t n,
  uint64_t hseq_base, uint32_t cur)
{
  __shared__ uint32_t s_hist[kMaxZones];
  __shared__ uint32_t s_base[kMaxZones];
  LandRec r[kLandPer];
#pragma unroll
  for(int u = 0; u < kLandPer; ++u)
  {
    const uint64_t i = (uint64_t)blockIdx.x * kLandRecs + (uint64_t)u * kLandThreads + threadIdx.x;
    r[u].valid = false;
    if(i < n)
    {
      const gpu_msg_t m = msgs[i];
      const uint64_t hseq = hseq_base + i;
      if(!is_remote(m.to))
      {
        const int t = type_of_global(m.to);
        if(t >= 0 && c_types[t].reducible)
        {
          reducible_apply_local(m.to, m.behaviour, m.arg);
          atomicAdd(&c_eng.stats[ST_DELIVERED], 1ull);
          atomicAdd(&c_eng.stats[ST_BY_TYPE + t], 1ull);
        }
        else if(t >= 0)
        {
          r[u].valid = true;
          r[u].to = m.to;
          r[u].w = ((uint32_t)(hseq & 0xFFFFull) << 16) | ((m.behaviour & 0xFu) << 12);
          r[u].from = kHostFrom | (uint32_t)(hseq >> 16);
          r[u].arg = m.arg;
        }
      }
    }
  }
  land_records(r, cur, s_hist, s_base);
}

// Records received from other ranks: `in` holds each peer's records in rank
// order, rcnt[p] of them from peer p (clipped to xcap); the sender's rank of a
// record is the segment it lies in.
__global__ void __launch_bounds__(kLandThreads) k_xinject(const XRec* in, uint64_t n, uint32_t cur,
  const unsigned long long* rcnt)
{
  __shared__ uint32_t s_hist[kMaxZones];
  __shared__ uint32_t s_base[kMaxZones];
  __shared__ unsigned long long s_app[GPU_ACTOR_MAX_TYPES];
  __shared__ unsigned long long s_roff[kMaxRanks];
  const uint32_t R = c_eng.nranks, me = c_eng.rank;
  if(threadIdx.x < GPU_ACTOR_MAX_TYPES) s_app[threadIdx.x] = 0;
  if(threadIdx.x == 0)
  {
    unsigned long long acc = 0;
    for(uint32_t p = 0; p < R; ++p)
    {
      s_roff[p] = acc;
      acc += min(rcnt[p], (unsigned long long)c_eng.xcap);
    }
  }
  __syncthreads();
  LandRec r[kLandPer];
#pragma unroll
  for(int u = 0; u < kLandPer; ++u)
  {
    const uint64_t i = (uint64_t)blockIdx.x * kLandRecs + (uint64_t)u * kLandThreads + threadIdx.x;
    r[u].valid = false;
    if(i < n)
    {
      const XRec x = in[i];
      uint32_t src = 0;
      for(uint32_t p = 1; p < R; ++p)
        if(i >= s_roff[p]) src = p;
      const uint32_t seq = (x.w0 >> 27) << 9 | (x.w1 >> 23);
      const uint32_t beh = (x.w0 >> 23) & 0xFu;
      const uint32_t to = (x.w0 & 0x7FFFFFu) * R + me;
      if(seq == kXSeqApply)
      {
        reducible_apply_local(to, beh, x.arg);
        const int t = type_of_global(to);
        if(t >= 0) atomicAdd(&s_app[t], 1ull);
      }
      else
      {
        r[u].valid = true;
        r[u].to = to;
        r[u].w = seq << 16 | beh << 12;
        r[u].from = (x.w1 & 0x7FFFFFu) * R + src;
        r[u].arg = x.arg;
      }
    }
  }
  land_records(r, cur, s_hist, s_base);
  // land_records passed barriers after every s_app update
  if(threadIdx.x < GPU_ACTOR_MAX_TYPES && s_app[threadIdx.x])
  {
    atomicAdd(&c_eng.stats[ST_DELIVERED], s_app[threadIdx.x]);
    atomicAdd(&c_eng.stats[ST_BY_TYPE + threadIdx.x], s_app[threadIdx.x]);
  }
}

} // namespace gpa

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
// shader clock at phase boundaries into c_eng.dbg[zone * kDbgSlots + k]. The shipped
// build compiles these away.
#ifdef GPA_STAMPS
#define GPA_STAMP(k)                                                         \
  do { if(threadIdx.x == 0) c_eng.dbg[z * kDbgSlots + (k)] = __builtin_amdgcn_s_memtime(); } while(0)
// diagnostic build: add the clocks since t0 to slot k (thread 0)
#define GPA_ACC(k, t0)                                                        \
  do { if(threadIdx.x == 0) c_eng.dbg[z * kDbgSlots + (k)] += __builtin_amdgcn_s_memtime() - (t0); } while(0)
#else
#define GPA_STAMP(k) do {} while(0)
#endif

constexpr int kUnroll = 8;   // independent records in flight per thread in streaming loops
constexpr uint32_t kCarryRun = 256;   // carry records per sample when a backlog is counted
#ifndef GPA_IDX_CAP
#define GPA_IDX_CAP 16384
#endif
#ifndef GPA_TILE
#define GPA_TILE 4096
#endif
#ifndef GPA_EMIT_UNROLL
#define GPA_EMIT_UNROLL 4     // tile records a thread reads before its first store (two-pass emit)
#endif
constexpr uint32_t kIdxCap = GPA_IDX_CAP;  // LDS index budget per zone (records per step)
constexpr uint32_t kTile = GPA_TILE;       // outbox records sorted per scatter tile (64 KB of LDS)
constexpr int kTilePer = kTile / kZoneThreads;  // tile records per thread
constexpr int kIdxPer = kIdxCap / kZoneThreads; // landed records per thread on the LDS-index path
static_assert(kTile % kZoneThreads == 0 && kIdxCap % kZoneThreads == 0, "tile / index split");
// a zone k_hot prepared takes the scratch path, where k_step reads and clears
// its hot_cnt slot: it must never fit the LDS index
static_assert(kHotMin > kIdxCap, "hot zones take the scratch path");
// Arrival groups up to this size are loaded at once and ordered in registers.
// 16 where the handler does not read the message (pinger: the selection
// compiles away) or the table's state is small; 8 elsewhere, to stay within
// 128 VGPRs without spilling.
// (the run-time compiled program table, kHtJit: its generated code keeps the
// program's registers as locals, so it holds as many as the compiled tables)
template <int HT> __host__ __device__ constexpr uint32_t small_regs()
{
  return (HT == GPU_ACTOR_HT_PINGER || HT == GPU_ACTOR_HT_FANIN_SENDER ||
          HT == GPU_ACTOR_HT_PINGER_DET || HT == GPU_ACTOR_HT_STORM || HT == kHtJit) ? 16u
         : HT == GPU_ACTOR_HT_PROGRAM ? 4u : 8u;
}

// A workgroup barrier that orders LDS only. __syncthreads() also waits for
// every global store the wave has in flight (vmcnt counts stores on CDNA);
// inside a loop that scatters records to HBM between LDS phases, that wait
// costs a full store latency per iteration. Use this one where the threads
// share nothing through global memory across the barrier.
__device__ __forceinline__ void lds_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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

// Exclusive scan of in[0, n) into out[0, n) (LDS) by a kZoneThreads workgroup,
// each thread taking a contiguous run; returns the total. All threads call it;
// it ends behind a barrier (an LDS-only one: lds_sync).
__device__ uint32_t block_scan_n(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* s_tmp)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t per = (n + kZoneThreads - 1) / kZoneThreads;
  const uint32_t lo = min(tid * per, n), hi = min(lo + per, n);
  uint32_t sum = 0;
  for(uint32_t i = lo; i < hi; ++i) sum += in[i];
  const uint32_t incl = wave_incl_scan(sum, lane);
  if(lane == 63) s_tmp[wv] = incl;
  lds_sync();
  if(wv == 0)
  {
    uint32_t x = lane < (uint32_t)kZoneWaves ? s_tmp[lane] : 0u;
    x = wave_incl_scan(x, lane);
    if(lane < (uint32_t)kZoneWaves) s_tmp[lane] = x;
  }
  lds_sync();
  uint32_t run = (wv ? s_tmp[wv - 1] : 0u) + incl - sum;
  for(uint32_t i = lo; i < hi; ++i) { const uint32_t v = in[i]; out[i] = run; run += v; }
  const uint32_t total = s_tmp[kZoneWaves - 1];
  lds_sync();
  return total;
}

// Add 1 to ctr[key] for every valid lane and return each lane's rank among
// the lanes that added to the same counter (atomicAdd's return, in lane
// order). The lanes of up to 4 distinct keys per wave are folded into one LDS
// atomic each (carried backlogs, grouped by actor); the rest add one by one.
// kMinRun > 0 (landed records, usually spread over the zone): folding stops
// at the first key held by fewer lanes than that — only a hot receiver's
// arrivals, 64 lanes on a handful of counters, are worth the ballots.
template <int kMinRun = 0>
__device__ __forceinline__ uint32_t agg_add(uint32_t* ctr, uint32_t key, bool valid)
{
  const uint32_t lane = __lane_id();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t active = __ballot(valid);
  uint32_t res = 0;
  for(int it = 0; it < 4 && active; ++it)
  {
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t k = __builtin_amdgcn_readlane(key, leader);
    const uint64_t peers = __ballot(valid && key == k) & active;
    if(kMinRun > 0 && __popcll(peers) < kMinRun) break;
    uint32_t base = 0;
    if((int)lane == leader) base = atomicAdd(&ctr[k], (uint32_t)__popcll(peers));
    base = (uint32_t)__shfl((int)base, leader);
    if((peers >> lane) & 1ull) res = base + (uint32_t)__popcll(peers & lt);
    active &= ~peers;
  }
  if((active >> lane) & 1ull) res = atomicAdd(&ctr[key], 1u);
  return res;
}

// agg_add without the ranks: counting only (the leader's add returns nothing,
// so no lane waits for an LDS round trip).
template <int kMinRun = 0>
__device__ __forceinline__ void agg_count(uint32_t* ctr, uint32_t key, bool valid)
{
  const uint32_t lane = __lane_id();
  uint64_t active = __ballot(valid);
  for(int it = 0; it < 4 && active; ++it)
  {
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t k = __builtin_amdgcn_readlane(key, leader);
    const uint64_t peers = __ballot(valid && key == k) & active;
    if(kMinRun > 0 && __popcll(peers) < kMinRun) break;
    if((int)lane == leader) atomicAdd(&ctr[k], (uint32_t)__popcll(peers));
    active &= ~peers;
  }
  if((active >> lane) & 1ull) atomicAdd(&ctr[key], 1u);
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
// mail (canonical), [nc, n) this step's arrival group (landing order).
// AccIdx: an LDS index (u16) into carry ++ landing — the usual case.
// AccS:   records materialised in the zone scratch S — zones whose record count
//         exceeds the LDS index budget.
struct AccIdx {
  uint16_t* idx;
  const ZRec* C;
  const ZRec* Ld;
  uint32_t nc_zone;
  __device__ __forceinline__ ZRec rec(uint32_t j) const
  {
    const uint32_t i = idx[j];
    return i < nc_zone ? ld_rec(C + i) : ld_rec(Ld + (i - nc_zone));
  }
  // insertion sort of [lo, lo + g) by canonical key
  __device__ void sort(uint32_t lo, uint32_t g)
  {
    for(uint32_t i = 1; i < g; ++i)
    {
      const uint16_t x = idx[lo + i];
      const uint64_t kx = zkey(rec(lo + i));
      uint32_t j = i;
      while(j > 0 && zkey(rec(lo + j - 1)) > kx)
      {
        idx[lo + j] = idx[lo + j - 1];
        --j;
      }
      idx[lo + j] = x;
    }
  }
};

// AccS: the actor's carried mail read in place from the carry buffer (it is
// grouped by actor, in canonical order: no copy), its arrivals materialised
// in the zone scratch S.
struct AccS {
  ZRec* p;            // arrivals: p[0, g)
  const ZRec* c;      // carried mail: c[0, nc)
  uint32_t nc;
  // a group the workgroup sorted: its sorted items (key << kPayBits | position
  // in p), read through instead of permuting the records themselves
  const uint64_t* perm = nullptr;
  // the canonical prefix [0, nst) staged in LDS by the workgroup (k_step:
  // long sequential runs: a backlog's carried mail, a sorted hot group)
  const uint4* stg = nullptr;
  uint32_t nst = 0;
  __device__ __forceinline__ ZRec rec(uint32_t j) const
  {
    if(j < nst)
    {
      const uint4 v = stg[j];
      ZRec r;
      r.w0 = v.x; r.from = v.y; r.arg = ((uint64_t)v.w << 32) | v.z;
      return r;
    }
    if(j < nc) return ld_rec(c + j);
    return ld_rec(p + (perm ? (uint32_t)(perm[j - nc] & 0xFFFFFull) : j - nc));
  }
  // insertion sort of the arrival group [lo, lo + g), lo == nc
  __device__ void sort(uint32_t lo, uint32_t g)
  {
    ZRec* q = p + (lo - nc);
    for(uint32_t i = 1; i < g; ++i)
    {
      const ZRec x = q[i];
      const uint64_t kx = zkey(x);
      uint32_t j = i;
      while(j > 0)
      {
        const ZRec y = q[j - 1];
        if(zkey(y) <= kx) break;
        q[j] = y;
        --j;
      }
      q[j] = x;
    }
  }
};

// Staged runs (k_step 2b): actors whose canonical run this step is at least
// kStageMin records, at most kMaxStage of them, kStageCap records in all
// (the LDS index area past the carry starts).
constexpr uint32_t kStageMin = 32;
constexpr uint32_t kMaxStage = 64;
constexpr uint32_t kStageCap = (kIdxCap * sizeof(uint16_t) - kZone * sizeof(uint32_t)) / 16;

// Groups handled whole up to this size keep their keys in registers.
constexpr uint32_t kMedReg = 16;

// A table whose behaviours ignore the message (the message-ubench pinger:
// every ping has the same effect) needs no delivery order; the compiler then
// drops the key selection of its drain entirely.
// The tables the any-mix kernel compiles (all; a run-time compiled mix,
// jit_host.h, only the engine's)
#ifndef GPA_MIX_MASK
#define GPA_MIX_MASK 0xFFFFFFFFu
#endif

template <int HT> __host__ __device__ constexpr bool order_free()
{
  return HT == GPU_ACTOR_HT_PINGER;
}

// A table whose behaviours' sends depend on the message alone — target,
// behaviour and argument a function of (receiver, behaviour, argument), never
// of the state or of the order messages run in — and whose state updates
// commute: message-ubench-det's ping and the storm (det_ping: count += 1,
// acc ^= arg; the ring token to self + 1). Each behaviour sends at most one
// message. Its plain zones run in two passes (k_step's `dp`): the sends are
// counted per (drain round, bucket) while the landed records are counted, by
// running each behaviour once on a throwaway state, in landing order; then
// the zone drains straight into bucket-sorted LDS tiles — no outbox round
// trip — and an actor's messages run in position order, each send stamped
// with its message's canonical rank in the group (drain_commutative).
template <int HT> __host__ __device__ constexpr bool msg_local()
{
  return HT == GPU_ACTOR_HT_PINGER_DET || HT == GPU_ACTOR_HT_STORM;
}
// ... on the 2048-actor geometry (the 4096-actor one's static LDS leaves no
// room for the two more bucket arrays the counts take). GPA_DP=0: off (A/B).
#ifndef GPA_DP
#define GPA_DP 1
#endif
template <int HT> __host__ __device__ constexpr bool dp_table()
{
  return GPA_DP && HT >= 0 && msg_local<HT>() && kZoneBits == 11;
}

// A table set compiled as one k_step instantiation: the FIFO probe's source
// and sink tables (the hot-receiver shape: sources fan in to order-sensitive
// sinks). Its drain dispatches on the actor's table between these two only,
// where the any-mix kernel's switch over every table spilled 1,324 VGPRs.
constexpr int kHtFifoPair = 64;

// records a lane loads ahead in a sequential drain (drain_zone run_seq):
// the FIFO tables, whose receivers build backlogs; 1 elsewhere (registers)
template <int HT> __host__ __device__ constexpr uint32_t seq_batch()
{
  return (HT == GPU_ACTOR_HT_FIFO_SINK || HT == GPU_ACTOR_HT_FIFO_SRC) ? 4u : 1u;
}

// (kHtJit: when the compiled program set holds a YIELD, jit_host.h)
#ifndef GPA_JIT_YIELD
#define GPA_JIT_YIELD 1
#endif
template <int HT> __host__ __device__ constexpr bool may_yield()
{
  return HT == GPU_ACTOR_HT_FIFO_SINK || HT == GPU_ACTOR_HT_PROGRAM || (HT == kHtJit && GPA_JIT_YIELD);
}

// Drain one actor: handle up to min(batch, n) messages — carried mail, then
// the arrival group in (from, seq) key order — stopping early after a
// behaviour whose sends muted the actor or that yielded. Returns how many ran;
// the rest, [done, n) of acc, is left in canonical order for the carry-out
// pass (the group is sorted in place when it was not handled whole).
// The arrival group is handled, by its size:
//   small  (<= SM, handled whole): all records loaded with the state, in
//          registers; each message is the smallest key left (selection);
//   medium (<= kMedReg, tables with SM < kMedReg): keys in registers, each
//          record loaded again at its turn;
//   window (handled whole, larger): a sorted register window of the SM
//          smallest keys not yet handled (key << 16 | position), refilled by a
//          pass over the group when it runs dry — g * ceil(g / SM) key loads instead of a g^2 selection
//          from memory (C2-det: the ~15 actors per step with more than 16
//          arrivals held their zones ~75 us, profiles/r03_general.txt);
//   sorted (part of it carries over, or sorted by the workgroup): canonical
//          order first, then in position order.
// An order-free table (its behaviours ignore the message) handles a whole
// group in position order: nothing is loaded for it.
template <int HT, class Acc, class Ctx>
__device__ __forceinline__ uint32_t drain_zone(const TypeDev& Tref, Ctx& a, Acc acc,
  uint32_t n, uint32_t nc, bool presorted)
{
  // a register copy of the type's fields: read once, not re-read after every
  // store the handlers make (the compiler cannot prove they do not alias)
  const TypeDev T = Tref;
  constexpr int NW = HT_Words<HT>::W;
  constexpr bool kY = may_yield<HT>();
  // a priority type runs batch after batch: everything pending
  const uint32_t w = (T.prio || n < T.batch) ? n : T.batch;
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
  // records [j0, j0 + cnt) in order; FIFO tables keep kSeqB loads in flight
  // (a backlog's carried mail and a sorted group are runs of up to a batch:
  // one load round trip per record held a hot receiver's lane ~50 us a step)
#define GPA_RUN_SEQ(J0, CNT)                                                            \
  if constexpr(seq_batch<HT>() == 1)                                                    \
  {                                                                                     \
    for(uint32_t k_ = 0; k_ < (CNT) && !stop; ++k_)                                     \
    {                                                                                   \
      const ZRec r_ = acc.rec((J0) + k_);                                               \
      handle(HtTag<HT>{}, T, a, s, (r_.w0 >> 12) & 0xFu, r_.arg);                       \
      ++done;                                                                           \
      stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;                              \
    }                                                                                   \
  }                                                                                     \
  else                                                                                  \
  {                                                                                     \
    constexpr uint32_t kSeqB = seq_batch<HT>();                                         \
    for(uint32_t k0_ = 0; k0_ < (CNT) && !stop; k0_ += kSeqB)                           \
    {                                                                                   \
      ZRec r_[kSeqB];                                                                   \
      _Pragma("unroll")                                                                 \
      for(uint32_t u_ = 0; u_ < kSeqB; ++u_)                                            \
        if(k0_ + u_ < (CNT)) r_[u_] = acc.rec((J0) + k0_ + u_);                         \
      _Pragma("unroll")                                                                 \
      for(uint32_t u_ = 0; u_ < kSeqB; ++u_)                                            \
        if(k0_ + u_ < (CNT) && !stop)                                                   \
        {                                                                               \
          handle(HtTag<HT>{}, T, a, s, (r_[u_].w0 >> 12) & 0xFu, r_[u_].arg);           \
          ++done;                                                                       \
          stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;                          \
        }                                                                               \
    }                                                                                   \
  }
  GPA_RUN_SEQ(0u, hc)
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
    else if(SM < kMedReg && q >= g && g <= kMedReg && !presorted)
    {
      // medium group handled whole (more than the small path holds): keys in
      // registers with the record's position in the low bits; each record is
      // loaded again (a cache hit) when its turn comes
      uint64_t km[kMedReg];
#pragma unroll
      for(int j = 0; j < (int)kMedReg; ++j)
        km[j] = (uint32_t)j < g ? (zkey(acc.rec(nc + j)) << 4) | (uint64_t)j : ~0ull;
      for(uint32_t r = 0; r < g && !stop; ++r)
      {
        uint64_t best = km[0];
#pragma unroll
        for(int j = 1; j < (int)kMedReg; ++j) best = km[j] < best ? km[j] : best;
        const uint32_t bi = (uint32_t)best & 0xFu;
#pragma unroll
        for(int j = 0; j < (int)kMedReg; ++j)
          if((uint32_t)j == bi) km[j] = ~0ull;
        const ZRec rr = acc.rec(nc + bi);
        handle(HtTag<HT>{}, T, a, s, (rr.w0 >> 12) & 0xFu, rr.arg);
        ++done;
        stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
      }
    }
    else if(!order_free<HT>() && q >= g && g <= 0xFFFFu && !presorted)
    {
      // large group handled whole: key order through the window
      uint64_t km[SM];
#pragma unroll
      for(int t = 0; t < (int)SM; ++t) km[t] = ~0ull;
      uint64_t lo = 0;
      for(uint32_t r = 0; r < g && !stop; ++r)
      {
        if(km[0] == ~0ull)
        {
          // refill: the SM smallest keys >= lo, insertion-sorted
          for(uint32_t j = 0; j < g; j += 4)
          {
            uint64_t kk[4];
#pragma unroll
            for(int u = 0; u < 4; ++u)
              kk[u] = j + u < g ? zkey(acc.rec(nc + j + u)) : ~0ull;
#pragma unroll
            for(int u = 0; u < 4; ++u)
            {
              uint64_t x = (kk[u] << 16) | (j + u);
              if(j + u >= g || kk[u] < lo || x >= km[SM - 1]) continue;
#pragma unroll
              for(int t = 0; t < (int)SM; ++t)
              {
                const uint64_t m = km[t];
                const bool lt = x < m;
                km[t] = lt ? x : m;
                x = lt ? m : x;
              }
            }
          }
        }
        const uint32_t pos = (uint32_t)km[0] & 0xFFFFu;
        lo = (km[0] >> 16) + 1;
#pragma unroll
        for(int t = 0; t + 1 < (int)SM; ++t) km[t] = km[t + 1];
        km[SM - 1] = ~0ull;
        const ZRec rr = acc.rec(nc + pos);
        handle(HtTag<HT>{}, T, a, s, (rr.w0 >> 12) & 0xFu, rr.arg);
        ++done;
        stop = (a.mute_hit | (kY ? a.yield_req : 0u)) != 0u;
      }
    }
    else if(order_free<HT>() && q >= g && !presorted)
    {
      // order-free table, group handled whole: position order
      for(uint32_t r = 0; r < g && !stop; ++r)
      {
        const ZRec rr = acc.rec(nc + r);
        handle(HtTag<HT>{}, T, a, s, (rr.w0 >> 12) & 0xFu, rr.arg);
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
      GPA_RUN_SEQ(nc, q)
    }
  }
#pragma unroll
  for(int k = 0; k < NW; ++k) T.state[(size_t)k * T.lcount + a.li] = s[k];
  // what ran of the group were its smallest keys: sorted, the group's tail
  // is the canonical remainder
  if(done < n && g > 1 && !sorted && !presorted) acc.sort(nc, g);
  return done;
}
#undef GPA_RUN_SEQ

// An actor of a message-local, commutative table (msg_local) whose whole
// mail runs this step (no carried mail, no mute, no yield): the state ends
// the same whatever order its messages run in, and so do the sends — except
// their sequence numbers, which order them at their receivers. So the
// messages run in position order, each send stamped with its message's rank
// in the group by canonical key (the number of the group's keys below it):
// ranks rise with the canonical order, so every receiver sorts these sends
// exactly as it would sort seq 0, 1, 2, ... of a canonical drain (a message
// sends at most one; the ranks' gaps, where a message sent nothing, order
// nothing). Where drain_zone selects the smallest of 16 keys per message
// (~140 VALU instructions: C2-det's drain was VALU-bound), a rank is 16
// compares. A group past the register slots (<= kBigGroup in a plain zone;
// ~15 of C2-det's 1M actors a step) must come in canonical order: it runs in
// position order, each send stamped with its message's position.
template <int HT, class Acc, class Ctx>
__device__ __forceinline__ uint32_t drain_commutative(const TypeDev& Tref, Ctx& a, Acc acc, uint32_t g)
{
  constexpr uint32_t SM = small_regs<HT>();
  const TypeDev T = Tref;
  constexpr int NW = HT_Words<HT>::W;
  uint64_t s[NW];
#pragma unroll
  for(int k = 0; k < NW; ++k) s[k] = T.state[(size_t)k * T.lcount + a.li];
  uint64_t k[SM], v[SM];
  auto load_slots = [&](uint32_t c0) __attribute__((always_inline)) {
#pragma unroll
    for(int j = 0; j < (int)SM; ++j)
    {
      if(c0 + j < g)
      {
        const ZRec r = acc.rec(c0 + j);
        k[j] = (zkey(r) << 4) | ((r.w0 >> 12) & 0xFu); v[j] = r.arg;
      }
      else
      {
        k[j] = ~0ull; v[j] = 0;
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): the loads, once
  };
  if(g <= SM)
  {
    // the whole group in the slots: each rank from the registers
    load_slots(0u);
#pragma unroll
    for(int j = 0; j < (int)SM; ++j)
      if((uint32_t)j < g)
      {
        uint32_t rank = 0;
#pragma unroll
        for(int i = 0; i < (int)SM; ++i) rank += k[i] < k[j] ? 1u : 0u;
        a.seq = rank;
        handle(HtTag<HT>{}, T, a, s, (uint32_t)k[j] & 0xFu, v[j]);
      }
  }
  else
    // a larger group is in canonical order already (the workgroup put it
    // there: k_step's dp), so its position is its rank; four loads in flight
    for(uint32_t p0 = 0; p0 < g; p0 += 4)
    {
      ZRec r[4];
#pragma unroll
      for(uint32_t u = 0; u < 4; ++u)
        if(p0 + u < g) r[u] = acc.rec(p0 + u);
#pragma unroll
      for(uint32_t u = 0; u < 4; ++u)
        if(p0 + u < g)
        {
          a.seq = p0 + u;
          handle(HtTag<HT>{}, T, a, s, (r[u].w0 >> 12) & 0xFu, r[u].arg);
        }
    }
#pragma unroll
  for(int kk = 0; kk < NW; ++kk) T.state[(size_t)kk * T.lcount + a.li] = s[kk];
  return g;
}

// The unhandled tail [done, n) of an actor's segment, already canonical, to
// the next step's carry buffer at carry position co (positions past the
// zone's capacity go to the spill list: never lost).
template <bool SR, class Acc>
__device__ __forceinline__ void carry_out(Acc acc, uint32_t done, uint32_t n, uint32_t z,
  uint32_t co, uint32_t nxt)
{
  ZRec* cout = c_eng.carry[nxt] + (SR ? zone_off_s(z) : c_eng.zoff[z]);
  const uint32_t cap = SR ? zone_cap_s(z) : zone_capacity(z);
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
static_assert(kBigGroup < 256, "drain_commutative's 8-bit ranks");
constexpr uint32_t kMaxBig = 32;            // big groups sorted per round of the loop
constexpr uint32_t kPayBits = 20;           // payload bits of an item (group <= 2^20)
static_assert(kPayBits == 20, "AccS::perm masks positions with 0xFFFFF");
constexpr uint32_t kSortWork = 512 + kZoneWaves * 256;   // u32 of LDS the sort borrows

// Stable sort of n items in a by item bits [lo, hi); b is scratch of n items.
// The result ends in a. All threads call; ends behind a barrier.
__device__ void coop_radix_sort(uint64_t* a, uint64_t* b, uint32_t n, uint32_t lo, uint32_t hi,
  uint32_t* s_work)
{
  uint32_t* s_bin = s_work;                // [256] running base of each digit
  uint32_t* s_wc = s_work + 512;           // [kZoneWaves][256] this tile's counts per wave -> bases
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t* src = a;
  uint64_t* dst = b;
  for(uint32_t sh = lo; sh < hi; sh += 8)
  {
    for(uint32_t d = tid; d < 256; d += kZoneThreads) s_bin[d] = 0;
    lds_sync();
    for(uint32_t i0 = 0; i0 < n; i0 += kZoneThreads * kUnroll)
    {
      uint64_t x[kUnroll];
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        x[u] = i < n ? src[i] : 0ull;
      }
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
        if(i0 + u * kZoneThreads + tid < n) atomicAdd(&s_bin[(x[u] >> sh) & 255u], 1u);
    }
    lds_sync();
    if(wv == 0)
    {
      uint32_t v[4], sum = 0;
#pragma unroll
      for(int k = 0; k < 4; ++k) { v[k] = s_bin[lane * 4 + k]; sum += v[k]; }
      uint32_t run = wave_incl_scan(sum, lane) - sum;
#pragma unroll
      for(int k = 0; k < 4; ++k) { s_bin[lane * 4 + k] = run; run += v[k]; }
    }
    // Tiles of kZoneThreads * kUnroll items; wave wv ranks the contiguous
    // run [wv * 64 * kUnroll, +64 * kUnroll) of the tile, kUnroll rows of 64
    // in order, keeping a running count per digit in s_wc[wv] — item order
    // is (wave, row, lane), so the sort stays stable. Then, per digit, the
    // waves' counts become their bases (prefix over waves on top of the
    // running base s_bin) and every item goes to base + its rank. Three
    // barriers per 4096 items (512-thread zones).
    constexpr uint32_t kWaveItems = 64u * kUnroll;
    for(uint32_t t0 = 0; t0 < n; t0 += kZoneThreads * kUnroll)
    {
      for(uint32_t k = lane; k < 256; k += 64) s_wc[wv * 256 + k] = 0;
      uint64_t x[kUnroll];
      const uint32_t wbase = t0 + wv * kWaveItems + lane;
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = wbase + u * 64u;
        x[u] = i < n ? src[i] : 0ull;
      }
      __builtin_amdgcn_wave_barrier();
      uint32_t rk[kUnroll];
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const bool valid = wbase + u * 64u < n;
        const uint32_t d = (uint32_t)(x[u] >> sh) & 255u;
        // lanes of this row holding the same digit: 8 ballots
        uint64_t same = __ballot(valid);
#pragma unroll
        for(int bit = 0; bit < 8; ++bit)
        {
          const uint64_t bb = __ballot(valid && ((d >> bit) & 1u));
          same &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t r = __popcll(same & lt);
        const uint32_t c = s_wc[wv * 256 + d];   // this digit in the wave's earlier rows
        rk[u] = c + r;
        // (one wave: every lane's read above is done before this write)
        __builtin_amdgcn_wave_barrier();
        if(valid && r == 0) s_wc[wv * 256 + d] = c + (uint32_t)__popcll(same);
        __builtin_amdgcn_wave_barrier();
      }
      lds_sync();                          // the waves' counts (and, first time, the bases) visible
      for(uint32_t k = tid; k < 256; k += kZoneThreads)
      {
        uint32_t run = s_bin[k];
        for(uint32_t w = 0; w < (uint32_t)kZoneWaves; ++w)
        {
          const uint32_t c = s_wc[w * 256 + k];
          s_wc[w * 256 + k] = run;
          run += c;
        }
        s_bin[k] = run;
      }
      lds_sync();                          // per-wave bases visible
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
        if(wbase + u * 64u < n)
          dst[s_wc[wv * 256 + ((uint32_t)(x[u] >> sh) & 255u)] + rk[u]] = x[u];
      lds_sync();                          // every read of the bases done
    }
    // the pass's scattered stores are the next pass's loads (other threads)
    __syncthreads();
    uint64_t* t = src; src = dst; dst = t;
  }
  if(src != a)
  {
    for(uint32_t i0 = 0; i0 < n; i0 += kZoneThreads * kUnroll)
    {
      uint64_t x[kUnroll];
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        x[u] = i < n ? src[i] : 0ull;
      }
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        if(i < n) a[i] = x[u];
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t bits_for(uint32_t v)
{
  return v ? 32u - (uint32_t)__clz(v) : 0u;
}

// Items of a hot group have distinct keys (a sender's sequence numbers are),
// so the group need not be sorted stably: one MSD pass partitions the items by
// the top kMsdBits bits of their key into bins (a histogram, one scan, one
// scatter with LDS cursors), and each bin — about a dozen items at the group
// sizes that take this path — is then sorted whole by one thread in registers.
// Three passes over the items instead of the LSD sort's key-width / 8 passes
// of ranking and scattering each. Bins larger than kMsdReg items are sorted
// in memory; a group whose largest bin exceeds kMsdMaxBin (keys that cluster)
// takes the LSD sort.
constexpr uint32_t kMsdBits = 11;           // bins of the MSD pass (2048 u32 of the sort's LDS)
constexpr uint32_t kMsdReg = 16;            // items a thread sorts in registers
constexpr uint32_t kMsdMaxBin = 64;
static_assert((1u << kMsdBits) + kZoneWaves + 1 <= kSortWork, "MSD bins fit the sort's LDS");

// Sort n items in a by item bits [lo, lo + kbits) (keys distinct within
// them); b is scratch of n items. The result ends in a. All threads call;
// ends behind a barrier.
__device__ void coop_msd_sort(uint64_t* a, uint64_t* b, uint32_t n, uint32_t lo, uint32_t kbits,
  uint32_t* s_work)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t d = min(kMsdBits, kbits);
  const uint32_t sh = lo + kbits - d;
  const uint32_t nb = 1u << d;
  uint32_t* s_bin = s_work;                     // [nb] counts -> starts -> cursors (ends)
  uint32_t* s_tmp = s_work + (1u << kMsdBits);  // [kZoneWaves + 1]
  for(uint32_t k = tid; k < nb; k += kZoneThreads) s_bin[k] = 0;
  lds_sync();
  for(uint32_t i0 = 0; i0 < n; i0 += kZoneThreads * kUnroll)
  {
    uint64_t x[kUnroll];
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
    {
      const uint32_t i = i0 + u * kZoneThreads + tid;
      x[u] = i < n ? a[i] : 0ull;
    }
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
      if(i0 + u * kZoneThreads + tid < n) atomicAdd(&s_bin[(uint32_t)(x[u] >> sh) & (nb - 1u)], 1u);
  }
  lds_sync();
  // the largest bin decides the path (uniform)
  uint32_t mx = 0;
  for(uint32_t k = tid; k < nb; k += kZoneThreads) mx = max(mx, s_bin[k]);
#pragma unroll
  for(int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
  if(lane == 0) s_tmp[wv] = mx;
  lds_sync();
  mx = 0;
  for(uint32_t w = 0; w < (uint32_t)kZoneWaves; ++w) mx = max(mx, s_tmp[w]);
  lds_sync();
  if(mx > kMsdMaxBin)
  {
    coop_radix_sort(a, b, n, lo, lo + ((kbits + 7u) & ~7u), s_work);
    return;
  }
  (void)block_scan_n(s_bin, s_bin, nb, s_tmp);     // counts -> bin starts (in place)
  {
    // half-batches, software-pipelined (loads of one half before the other's stores)
    constexpr int kH = kUnroll / 2;
    constexpr uint32_t kStride = kZoneThreads * kH;
    auto load_half = [&](uint64_t (&x)[kH], uint32_t i0) __attribute__((always_inline)) {
#pragma unroll
      for(int u = 0; u < kH; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        x[u] = i < n ? a[i] : 0ull;
      }
    };
    auto scatter_half = [&](const uint64_t (&x)[kH], uint32_t i0) __attribute__((always_inline)) {
#pragma unroll
      for(int u = 0; u < kH; ++u)
        if(i0 + u * kZoneThreads + tid < n)
          b[atomicAdd(&s_bin[(uint32_t)(x[u] >> sh) & (nb - 1u)], 1u)] = x[u];
    };
    uint64_t xa[kH], xb[kH];
    load_half(xa, 0);
    for(uint32_t i0 = 0; i0 < n; i0 += 2 * kStride)
    {
      load_half(xb, i0 + kStride);
      scatter_half(xa, i0);
      load_half(xa, i0 + 2 * kStride);
      scatter_half(xb, i0 + kStride);
    }
  }
  // the scatter's stores are the bin sorts' loads (other threads); s_bin[k]
  // is now the end of bin k
  __syncthreads();
  for(uint32_t k = tid; k < nb; k += kZoneThreads)
  {
    const uint32_t e = s_bin[k], s0 = k ? s_bin[k - 1] : 0u, m = e - s0;
    if(m <= 1)
    {
      if(m) a[s0] = b[s0];
      continue;
    }
    if(m <= kMsdReg)
    {
      uint64_t r[kMsdReg];
#pragma unroll
      for(int j = 0; j < (int)kMsdReg; ++j) r[j] = (uint32_t)j < m ? b[s0 + j] : ~0ull;
      // insertion network over static indices (stays in registers)
#pragma unroll
      for(int i = 1; i < (int)kMsdReg; ++i)
#pragma unroll
        for(int j = i; j > 0; --j)
        {
          const uint64_t p = r[j - 1], q = r[j];
          r[j - 1] = p < q ? p : q;
          r[j] = p < q ? q : p;
        }
#pragma unroll
      for(int j = 0; j < (int)kMsdReg; ++j)
        if((uint32_t)j < m) a[s0 + j] = r[j];
    }
    else
    {
      // a larger bin: insertion sort in memory, into a
      for(uint32_t i = 0; i < m; ++i)
      {
        const uint64_t x = b[s0 + i];
        uint32_t j = i;
        while(j > 0 && a[s0 + j - 1] > x) { a[s0 + j] = a[s0 + j - 1]; --j; }
        a[s0 + j] = x;
      }
    }
  }
  __syncthreads();
}

// Sort the arrival group [nc, nc + g) of one actor's segment, by the whole
// workgroup. idx path: payload = the idx entry, written back in order; S
// path: payload = the record's position in the segment, and the sorted items
// are left in ia (g of them) for the actor's accessor to read through
// (AccS::perm) — the records themselves do not move. ib is scratch of g
// items. Returns false (nothing changed) when the compressed key does not fit.
template <class Acc>
__device__ bool coop_sort_group(Acc acc, uint16_t* idx, uint32_t nc, uint32_t g,
  uint64_t* ia, uint64_t* ib, uint32_t* s_work, uint32_t* s_red3)
{
  const uint32_t tid = threadIdx.x;
  // key range: min/max sender, max sequence
  uint32_t fmin = 0xFFFFFFFFu, fmax = 0, smax = 0;
  // kUnroll records in flight per thread (a group is tens of thousands of
  // records: one load per iteration would wait out a memory latency each time)
  for(uint32_t j0 = 0; j0 < g; j0 += kZoneThreads * kUnroll)
  {
    ZRec r[kUnroll];
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
    {
      const uint32_t j = j0 + u * kZoneThreads + tid;
      if(j < g) r[u] = acc.rec(nc + j);
    }
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
      if(j0 + u * kZoneThreads + tid < g)
      {
        fmin = min(fmin, r[u].from); fmax = max(fmax, r[u].from); smax = max(smax, r[u].w0 >> 16);
      }
  }
  if(tid < 3) s_red3[tid] = tid == 0 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  atomicMin(&s_red3[0], fmin); atomicMax(&s_red3[1], fmax); atomicMax(&s_red3[2], smax);
  __syncthreads();
  fmin = s_red3[0]; fmax = s_red3[1]; smax = s_red3[2];
  __syncthreads();
  const uint32_t sbits = bits_for(smax), kbits = bits_for(fmax - fmin) + sbits;
  const uint32_t pay = idx ? 16u : kPayBits;
  if(kbits + pay > 64u) return false;
  {
    // half-batches, software-pipelined: one half's record loads are issued
    // before the other half's item stores (vmcnt counts both, in order)
    constexpr int kH = kUnroll / 2;
    constexpr uint32_t kStride = kZoneThreads * kH;
    auto load_half = [&](ZRec (&r)[kH], uint32_t j0) __attribute__((always_inline)) {
#pragma unroll
      for(int u = 0; u < kH; ++u)
      {
        const uint32_t j = j0 + u * kZoneThreads + tid;
        if(j < g) r[u] = acc.rec(nc + j);
      }
    };
    auto store_half = [&](const ZRec (&r)[kH], uint32_t j0) __attribute__((always_inline)) {
#pragma unroll
      for(int u = 0; u < kH; ++u)
      {
        const uint32_t j = j0 + u * kZoneThreads + tid;
        if(j >= g) continue;
        const uint64_t key = ((uint64_t)(r[u].from - fmin) << sbits) | (r[u].w0 >> 16);
        ia[j] = (key << pay) | (idx ? (uint64_t)idx[nc + j] : (uint64_t)j);
      }
    };
    ZRec ra[kH], rb[kH];
    load_half(ra, 0);
    for(uint32_t j0 = 0; j0 < g; j0 += 2 * kStride)
    {
      load_half(rb, j0 + kStride);
      store_half(ra, j0);
      load_half(ra, j0 + 2 * kStride);
      store_half(rb, j0 + kStride);
    }
  }
  __syncthreads();
  coop_msd_sort(ia, ib, g, pay, kbits, s_work);
  const uint64_t pm = (1ull << pay) - 1;
  if(idx)
  {
    for(uint32_t j0 = 0; j0 < g; j0 += kZoneThreads * kUnroll)
    {
      uint64_t x[kUnroll];
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t j = j0 + u * kZoneThreads + tid;
        x[u] = j < g ? ia[j] : 0ull;
      }
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t j = j0 + u * kZoneThreads + tid;
        if(j < g) idx[nc + j] = (uint16_t)(x[u] & pm);
      }
    }
  }
  // (S path: the sorted items stay in ia, and the actor's records are read
  // through them: AccS::perm)
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

// ---- order-free zones in two passes (no outbox) -------------------------------------
// A zone of an order-free table whose mail all runs this step (k_step's `fast`
// case) runs its behaviours twice instead of parking every send in the zone
// outbox O and reading it back for the scatter: pass 1 (PlanCtx) only counts
// the sends per (drain round, destination bucket) in LDS; one chunk per bucket
// is reserved from the totals; pass 2 (TileCtx) runs the behaviours again on
// the same register copy of each actor's state and puts every send straight at
// its place in an LDS tile that is already sorted by bucket (the round's
// counts give each bucket's start), and the tile leaves as runs of one chunk
// each. The behaviours are deterministic functions of the state, so both
// passes make the same sends. A drain round is one actor per thread.
template <int HT> __host__ __device__ constexpr bool two_pass()
{
  return HT == GPU_ACTOR_HT_PINGER;     // order-free, at most one send per message
}
// state words a two-pass table keeps per actor (1 for the others: unused)
template <int HT> __host__ __device__ constexpr int plan_words()
{
  if constexpr(HT >= 0 && two_pass<HT>()) return HT_Words<HT>::W; else return 1;
}
constexpr uint32_t kRounds = kZone / kZoneThreads;
static_assert(kRounds == 4, "two rounds per packed count word, two words");
constexpr uint32_t kClasses = 16;   // message-count classes of the two-pass dealing (>= 15 share one)

// pass 2's tile: the whole LDS pool (the per-actor counts are in registers by then)
constexpr uint32_t kPlanTile = kTile;

// Store record r = {to, w | src_local, arg lo, arg hi} at position pos of
// bucket b's chunk: a destination zone's landing buffer (past its capacity:
// the spill list), or a peer rank's exchange segment. Returns 1 if the
// exchange lost it (its spill list full).
__device__ __forceinline__ uint32_t emit_rec(const uint4& r, uint32_t b, uint32_t pos, uint32_t L0,
  uint32_t nz, uint32_t nxt)
{
  const uint32_t from = (L0 + (r.y & kZoneMask)) * c_eng.nranks + c_eng.rank;
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
    return 0;
  }
  return xout_store(b - nz, pos, xpack(r.x, r.y & ~kZoneMask, from, ((uint64_t)r.w << 32) | r.z));
}

// A chunk's destination word, kept per bucket in LDS for the emit loops: the
// record offset of its first record in land[nxt] | kDirect when the whole
// chunk [base, base + h) fits its zone's capacity (the usual case: a record
// then needs one LDS read for its address, where emit_rec loads the zone's
// offset and capacity from HBM, a dependent L2 round trip per record), else
// the reserved position itself (a peer rank's segment, or a chunk that
// reaches past the zone: emit_rec checks each record).
constexpr uint32_t kDirect = 0x80000000u;
__device__ __forceinline__ uint32_t chunk_dst(uint32_t b, uint32_t base, uint32_t h, uint32_t nz)
{
  if(b < nz)
  {
    const uint64_t o = c_eng.zoff[b] + base;
    if(base + h <= c_eng.zcapz[b] && o + h <= 0x7FFFFFFFull) return (uint32_t)o | kDirect;
  }
  return base;
}

// Record r of bucket b at offset rel past its chunk's destination word d.
__device__ __forceinline__ uint32_t emit_at(const uint4& r, uint32_t b, uint32_t d, uint32_t rel,
  uint32_t L0, uint32_t nz, uint32_t nxt)
{
  if(d & kDirect)
  {
    uint4 v;
    v.x = (r.y & ~kZoneMask) | (rdiv(r.x) & kZoneMask);
    v.y = (L0 + (r.y & kZoneMask)) * c_eng.nranks + c_eng.rank;
    v.z = r.z;
    v.w = r.w;
    st16(reinterpret_cast<uint4*>(c_eng.land[nxt] + ((d & ~kDirect) + rel)), v);
    return 0;
  }
  return emit_rec(r, b, d + rel, L0, nz, nxt);
}

// pass 1: count each send in its (round, bucket) — two rounds per u32 word,
// 16 bits each (the zone's total is checked to fit)
// (kPlain: the plan path runs only with no backpressure anywhere and the
// zone's whole mail below seq_max; without the two checks in send_serial C2
// runs 70.9-71.5 -> 69.6-70.1 us, profiles/r06c_plain_ctx_ab.txt)
#ifndef GPA_PLAIN_CTX
#define GPA_PLAIN_CTX 1
#endif
struct PlanCtx : ActorBase {
  static constexpr bool kPlain = GPA_PLAIN_CTX;
  uint32_t* rh;
  uint32_t inc;
  __device__ __forceinline__ void put(uint32_t to, uint32_t w, uint64_t arg)
  {
    atomicAdd(&rh[bucket_of(to)], inc);
  }
};

// pass 2: the send's rank in its bucket comes from the round's cursor; the
// tile holds it at start + rank; past the tile it goes straight to its chunk
struct TileCtx : ActorBase {
  static constexpr bool kPlain = GPA_PLAIN_CTX;
  uint4* tile;
  uint32_t* cur;          // [nb] bucket cursors in the tile, two rounds per word (half sh)
  const uint32_t* st;     // [nb] bucket starts in the tile, likewise
  const uint32_t* bs;     // [nb] the bucket chunk's next free place (chunk_dst word)
  uint32_t sh, inc;       // this round's half: shift, and 1 << shift
  uint32_t L0, nz, nxt, xover;
  uint32_t tcap;          // records the tile holds
  __device__ __forceinline__ void put(uint32_t to, uint32_t w, uint64_t arg)
  {
    const uint32_t b = bucket_of(to);
    const uint32_t idx = (atomicAdd(&cur[b], inc) >> sh) & 0xFFFFu;
    uint4 r;
    r.x = to; r.y = w | src_local; r.z = (uint32_t)arg; r.w = (uint32_t)(arg >> 32);
    if(idx < tcap)
      tile[idx] = r;
    else
      xover += emit_at(r, b, bs[b], idx - ((st[b] >> sh) & 0xFFFFu), L0, nz, nxt);
  }
};

// The two-pass paths' shared steps (the pinger's plan path, and `dp` for the
// message-local tables). Counts per (round, bucket) come packed two rounds
// per u32 (16-bit halves): rh[0, nb) rounds 0-1, rh[nb, 2nb) rounds 2-3.
// (1) one chunk per bucket for the zone's sends: bs[b] = chunk_dst word
__device__ __forceinline__ uint32_t plan_reserve(const uint32_t* rh, uint32_t* bs, uint32_t nb,
  uint32_t nz, uint32_t nxt, uint32_t tid)
{
  uint32_t n_atom = 0;
  for(uint32_t b = tid; b < nb; b += kZoneThreads)
  {
    const uint32_t w0 = rh[b], w1 = rh[nb + b];
    const uint32_t h = (w0 & 0xFFFFu) + (w0 >> 16) + (w1 & 0xFFFFu) + (w1 >> 16);
    uint32_t base = 0;
    if(h)
    {
      ++n_atom;
      if(b < nz)
        base = atomicAdd(&c_eng.land_n[nxt][b], h);
      else
        base = (uint32_t)atomicAdd(&c_eng.xcount[b - nz], (unsigned long long)h);
    }
    bs[b] = chunk_dst(b, base, h, nz);
  }
  return n_atom;
}

// (2) every round's bucket starts in the tile at once: exclusive scans of the
// packed (round pair, bucket) counts, in place, each thread a contiguous run
// of buckets; the cursors start at them. Three barriers for the four rounds
// (a scan per round took three each). tot01 / tot23: the rounds' totals, packed.
__device__ __forceinline__ void plan_scan(uint32_t* rh, uint32_t* cur, uint32_t nb, uint32_t* tmp2,
  uint32_t tid, uint32_t& tot01, uint32_t& tot23)
{
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const uint32_t per = (nb + kZoneThreads - 1) / kZoneThreads;
  const uint32_t lo = min(tid * per, nb), hi = min(lo + per, nb);
  uint32_t a = 0, c = 0;
  for(uint32_t b = lo; b < hi; ++b) { a += rh[b]; c += rh[nb + b]; }
  const uint32_t ia = wave_incl_scan(a, lane), ic = wave_incl_scan(c, lane);
  if(lane == 63) { tmp2[wv] = ia; tmp2[kZoneWaves + wv] = ic; }
  lds_sync();
  if(wv < 2)
  {
    uint32_t* t = tmp2 + wv * kZoneWaves;
    uint32_t x = lane < (uint32_t)kZoneWaves ? t[lane] : 0u;
    x = wave_incl_scan(x, lane);
    if(lane < (uint32_t)kZoneWaves) t[lane] = x;
  }
  lds_sync();
  uint32_t ra = (wv ? tmp2[wv - 1] : 0u) + ia - a;
  uint32_t rc = (wv ? tmp2[kZoneWaves + wv - 1] : 0u) + ic - c;
  for(uint32_t b = lo; b < hi; ++b)
  {
    const uint32_t va = rh[b], vc = rh[nb + b];
    rh[b] = ra; cur[b] = ra; ra += va;
    rh[nb + b] = rc; cur[nb + b] = rc; rc += vc;
  }
  tot01 = tmp2[kZoneWaves - 1];
  tot23 = tmp2[2 * kZoneWaves - 1];
  lds_sync();
}

// (3) round r's tile (m records, sorted by bucket) to the chunks: runs of one
// chunk per wave store, every record of the thread read before the first
// store; then each chunk's next free place for the next round (the other
// half of bs: this round's emit still reads this one) = + the round's count
// of the bucket, the difference of consecutive starts. Returns the records
// the exchange lost (emit_rec).
__device__ __forceinline__ uint32_t plan_emit(const uint4* tile, uint32_t m, const uint32_t* rst,
  const uint32_t* bsr, uint32_t* bsw, uint32_t sh, uint32_t tr, uint32_t nb, uint32_t L0,
  uint32_t nz, uint32_t nxt, uint32_t tid)
{
  uint32_t xover = 0;
  constexpr uint32_t kEU = GPA_EMIT_UNROLL;
  for(uint32_t q0 = 0; q0 < m; q0 += kEU * kZoneThreads)
  {
    uint4 rec[kEU];
#pragma unroll
    for(uint32_t u = 0; u < kEU; ++u)
    {
      const uint32_t q = q0 + u * kZoneThreads + tid;
      if(q < m) rec[u] = tile[q];
    }
#pragma unroll
    for(uint32_t u = 0; u < kEU; ++u)
    {
      const uint32_t q = q0 + u * kZoneThreads + tid;
      if(q < m)
      {
        const uint32_t b = bucket_of(rec[u].x);
        xover += emit_at(rec[u], b, bsr[b], q - ((rst[b] >> sh) & 0xFFFFu), L0, nz, nxt);
      }
    }
  }
  for(uint32_t b = tid; b < nb; b += kZoneThreads)
  {
    const uint32_t s0 = (rst[b] >> sh) & 0xFFFFu;
    const uint32_t s1 = b + 1 < nb ? (rst[b + 1] >> sh) & 0xFFFFu : tr;
    bsw[b] = bsr[b] + (s1 - s0);
  }
  return xover;
}

// dp: the zone's LDS index at the end of the pool (nl entries, the start
// 16-B aligned), and the tile before it
__device__ __forceinline__ uint16_t* dp_index(uint4* pool, uint32_t nl)
{
  return reinterpret_cast<uint16_t*>(pool + kTile) - ((nl + 7u) & ~7u);
}
__device__ __forceinline__ uint32_t dp_tile_cap(uint32_t nl)
{
  return (uint32_t)(kTile * sizeof(uint4) - ((nl + 7u) & ~7u) * sizeof(uint16_t)) / (uint32_t)sizeof(uint4);
}

// 2 workgroups of kZoneThreads per CU: minimum waves per SIMD = 2 * 512 / 256 = 4
// HTS >= 0: every serial actor of this engine runs handler table HTS (the host
// checks), so only that table is compiled in; HTS < 0: any mix of tables.
// PM (two-pass tables): 0 every path in one kernel; or the step as two
// launches, so that the two-pass path gets registers of its own (alone it
// needs 99 VGPRs and spills none; beside the general path the kernel holds 128
// and spills 22): PM 1 runs only the zones that take the two-pass path — every
// other zone returns before it has written anything — and marks them in
// c_eng.zplan; PM 2, launched right behind it, runs the rest (the general
// path, as PM 0 would).
// A zone's static LDS, one object per table (HTS) whatever the launch form
// (PM): the fused step (PM 3) runs PM 1's and PM 2's code in one kernel, and
// function-local __shared__ arrays in the two instantiations would be two
// allocations.
template <int HTS> struct ZoneLds {
  // 64 KB pool. Phases 1-3: per-actor arrays + the segment index; phase 4:
  // the outbox sort tile (kTile records).
  uint4 pool[kTile];
  uint32_t tmp[kZoneWaves + 1];
  uint32_t tmp2[2 * kZoneWaves];
  uint32_t nout;
  uint32_t nmix;                    // carry runs that straddle actors (count phase)
  uint32_t tot;                     // messages pending in the zone (fast path)
  uint32_t ph[kClasses];            // two-pass path: actors per message-count class
  unsigned long long agg[kZoneWaves];
  unsigned long long bytype[GPU_ACTOR_MAX_TYPES];
  __attribute__((aligned(16))) uint8_t tb[kZone];   // trigger byte per actor
  uint32_t ntrig;
  uint32_t bigbits[kZone / 32];     // groups the workgroup sorted this step
  uint32_t red3[3];
  uint32_t big[kMaxBig];
  uint32_t nbig;
  uint32_t stn;
  // the staged runs' lists (phase 2b) and, once they are spent, the counters'
  // reduction (the end): apart, the pinger's zone held 160 B more than lets
  // two workgroups share a CU beside its 12 KB of bucket arrays
  union {
    struct { uint32_t stl[kMaxStage], stc[kMaxStage], sto[kMaxStage + 1]; } st;   // staged runs
    unsigned long long red[kZoneWaves][6];
  } u;
  unsigned long long fan[((HTS < 0 && ((GPA_MIX_MASK >> GPU_ACTOR_HT_FANIN_SENDER) & 1u)) ||
                          HTS == GPU_ACTOR_HT_FANIN_SENDER) ? 2 * kFanLds : 1];   // fan-in apply accumulators
};
template <int HTS> __device__ __forceinline__ ZoneLds<HTS>& zone_lds()
{
  __shared__ ZoneLds<HTS> lds;
  return lds;
}

// zone_step runs zone z's step; k_step (below) maps workgroups to zones.
template <int HTS, int PM>
__device__ __forceinline__ bool zone_step(const uint32_t z, uint32_t cur, uint32_t pend_slot,
  uint32_t sidx)
{
  ZoneLds<HTS>& Z = zone_lds<HTS>();
  uint4* const s_pool = Z.pool;
  static_assert(4 * kZone * sizeof(uint32_t) + kIdxCap * sizeof(uint16_t) <= sizeof(uint4) * kTile,
                "LDS pool too small");
  uint32_t* const s_cnt = reinterpret_cast<uint32_t*>(s_pool);   // records per actor this step
  uint32_t* const s_off = s_cnt + kZone;    // segment offset in S
  uint32_t* const s_ccnt = s_off + kZone;   // carried records per actor
  uint32_t* const s_aux = s_ccnt + kZone;   // carry start -> landing cursor -> carry-out offset
  uint16_t* const s_idx = reinterpret_cast<uint16_t*>(s_aux + kZone);  // index into carry ++ landing
  uint32_t* const s_cst = reinterpret_cast<uint32_t*>(s_idx);   // S path: carry start per actor
  extern __shared__ uint32_t s_dyn[];   // [nb] histogram, [nb] chunk bases, [nb] tile counts, [nb] tile starts
  auto& s_tmp = Z.tmp;
  auto& s_tmp2 = Z.tmp2;
  auto& s_nout = Z.nout;
  auto& s_nmix = Z.nmix;
  auto& s_tot = Z.tot;
  auto& s_ph = Z.ph;
  auto& s_agg = Z.agg;
  auto& s_red = Z.u.red;
  auto& s_bytype = Z.bytype;
  auto& s_tb = Z.tb;
  auto& s_ntrig = Z.ntrig;
  auto& s_bigbits = Z.bigbits;
  auto& s_red3 = Z.red3;
  auto& s_big = Z.big;
  auto& s_nbig = Z.nbig;
  auto& s_stn = Z.stn;
  auto& s_stl = Z.u.st.stl;
  auto& s_stc = Z.u.st.stc;
  auto& s_sto = Z.u.st.sto;
  auto& s_fan = Z.fan;
  constexpr bool kFan = (HTS < 0 && ((GPA_MIX_MASK >> GPU_ACTOR_HT_FANIN_SENDER) & 1u)) ||
                        HTS == GPU_ACTOR_HT_FANIN_SENDER;

  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  static_assert(PM == 0 || HTS >= 0, "split launches are for one-table engines");
  // PM 1 of a two-pass table takes the zones that plan; of any other table
  // the plain zones (kSimple): no backpressure, no carried mail, the LDS
  // index, no group over kBigGroup — the drain without the scratch path, the
  // hot-group sort and the mute checks, which then need no registers
  constexpr bool kPlanSplit = HTS >= 0 && two_pass<HTS>();
  constexpr bool kSimple = PM == 1 && !kPlanSplit;
  // ... of a message-local table, plain zones whose actors all drain whole
  // this step run in two passes (dp, below)
  constexpr bool kDP = kSimple && dp_table<HTS>();
  bool dp = false;
  // (the mark is the step's index + 1: nothing clears it, and a step that
  // halted — and runs again with the same index — marked no zone)
  if constexpr(PM == 2)
    if(__builtin_amdgcn_readfirstlane(c_eng.zplan[z]) == sidx + 1u) return false;
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
    if(PM != 1 && z == 0 && tid == 0)
    {
      *c_eng.halt = 1u;
      c_eng.pend[pend_slot] = kPendSkipped;
      atomicAdd(c_eng.skipped, 1ull);
    }
    return false;
  }
#ifdef GPA_STAMPS
  // the device's 100 MHz real-time clock (one for every XCD, unlike the
  // shader clock of GPA_STAMP): zone start [11] and end [12] across the grid
  if(tid == 0)
  {
    c_eng.dbg[z * kDbgSlots + 11] = __builtin_amdgcn_s_memrealtime();
    c_eng.dbg[z * kDbgSlots + 12] = 0;
  }
#endif
  if(tid < GPU_ACTOR_MAX_TYPES) s_bytype[tid] = 0;
  if(tid < kClasses) s_ph[tid] = 0;
  if constexpr(kFan)
    for(uint32_t j = tid; j < 2 * kFanLds; j += kZoneThreads) s_fan[j] = 0;
  const uint32_t nxt = cur ^ 1u;
  const uint32_t L0 = z * kZone;
  const uint32_t nact = min(kZone, c_eng.n_local - L0);
  const uint32_t R = c_eng.nranks, me = c_eng.rank;
  const uint32_t nz = c_eng.n_zones;
  const uint32_t nb = nz + (R > 1 ? R : 0u);
  // The zone's offset, capacity and counters through SGPRs (zone_cap_s):
  // measured faster for the pinger (C2) and the storm, slower for C2-det,
  // whose kernel then spills more SGPRs (profiles/r04y_split_sgpr_ab.txt)
  constexpr bool SR = HTS != GPU_ACTOR_HT_PINGER_DET;
  auto rfl = [](uint32_t v) __attribute__((always_inline)) {
    return SR ? __builtin_amdgcn_readfirstlane(v) : v;
  };
  const uint32_t cap = SR ? zone_cap_s(z) : zone_capacity(z);
  const uint64_t zo = SR ? zone_off_s(z) : c_eng.zoff[z];
  uint32_t* s_hist = s_dyn;
  uint32_t* s_base = s_dyn + nb;

  // Backpressure bookkeeping: ztc = this zone's actors that
  // trigger muting after the last step (overloaded or muted); ztn = nonzero
  // bytes this zone left in trig_own[nxt] two steps ago. trig_n is indexed by
  // step mod 3: read this step's, add to the next's, clear the one after.
  const uint32_t ztc = rfl(c_eng.ztrig[cur][z]);
  const uint32_t ztn = rfl(c_eng.ztrig[nxt][z]);
  const bool gate = rfl(c_eng.trig_n[sidx % 3u]) != 0u;
  // (every launch of the step clears it — PM 2's zone 0 returns above when PM
  // 1 ran it; no kernel of this step reads or adds to that slot). Likewise the
  // backlog list of the other parity, which the last k_carry_big copied.
  if(z == 0 && tid == 0)
  {
    c_eng.trig_n[(sidx + 2u) % 3u] = 0u;
    c_eng.bigc_n[cur ^ 1u] = 0ull;
  }
  if constexpr(PM == 1)
    if(gate || ztc != 0u || (kPlanSplit && c_eng.two_pass == 0u)) return false;
  uint8_t* const tb_out = c_eng.trig_own[nxt];

  for(uint32_t i = tid; i < kZone; i += kZoneThreads) { s_cnt[i] = 0; s_ccnt[i] = 0; }
  for(uint32_t b = tid; b < (kDP ? 2u : 1u) * nb; b += kZoneThreads) s_hist[b] = 0;
  if(tid == 0) { s_nout = 0; s_ntrig = 0; s_nmix = 0; s_tot = 0; }
  __syncthreads();
  GPA_STAMP(0);

  // ---- 1. count --------------------------------------------------------------
  const uint32_t nc = min(rfl(c_eng.carry_n[cur][z]), cap);
  const uint32_t nl = min(rfl(c_eng.land_n[cur][z]), cap);
  if(nc + nl == 0 && ztc == 0)
  {
    if constexpr(PM == 1) return false;
    // an idle zone (uniform: every thread read the same counters) has
    // nothing to count, run or send — the quiet tail of a run, or zones of
    // a sparse workload; it only clears trigger bytes it left two steps ago
    if(tid == 0) c_eng.carry_n[nxt][z] = 0;
    if(ztn)
    {
      for(uint32_t i = tid; i < nact; i += kZoneThreads) tb_out[(L0 + i) * R + me] = 0;
      if(tid == 0) c_eng.ztrig[nxt][z] = 0;
    }
    return false;
  }
  if constexpr(kSimple)
    if(nc != 0u || nl > kIdxCap) return false;
  // the trigger bytes of this zone's actors as the last step left them
  if(ztc)
    for(uint32_t i = tid; i < kZone; i += kZoneThreads)
      s_tb[i] = i < nact ? c_eng.trig[cur][(L0 + i) * R + me] : (uint8_t)0;
  else
    for(uint32_t i = tid; i < kZone / 4; i += kZoneThreads)
      reinterpret_cast<uint32_t*>(s_tb)[i] = 0;
  const ZRec* C = c_eng.carry[cur] + zo;
  const ZRec* Ld = c_eng.land[cur] + zo;
  const bool use_idx = kSimple || nc + nl <= kIdxCap;       // uniform per workgroup
  // a hot zone k_hot prepared: its arrivals are in S already, counted in
  // hot_cnt, each big group sorted (hot_dev.h)
  // (compiled for the tables whose engines run k_hot: engine.hip hot_on)
  constexpr bool kHotTables = !kSimple && (HTS < 0 || HTS == kHtFifoPair);
  const bool hot = kHotTables && c_eng.hot_on &&
                   __builtin_amdgcn_readfirstlane(c_eng.hot_prep[z]) == sidx + 1u;
  const uint32_t* const hot_cnt =
    c_eng.hot_cnt + (size_t)__builtin_amdgcn_readfirstlane(hot ? c_eng.hot_slot[z] : 0u) * 4096u;
  // carried records counted apart (s_ccnt); landed ones in s_cnt.
  // Carried mail is sorted by actor (carry-out writes each actor's remainder
  // at its scan offset). A large carry (a backlog) is counted from samples:
  // a run of kCarryRun records whose first and last belong to one actor is
  // all that actor's, and only the runs that straddle actors are read whole
  // (their positions listed in the index area, free until the place phase).
  // Elsewhere a wave's lanes mostly share one counter, folded into one atomic.
  uint32_t nmix = 0;
  const uint32_t nrun = (nc + kCarryRun - 1) / kCarryRun;
  const bool sampled = !kSimple && nc > kIdxCap && nrun <= kIdxCap / 2;     // uniform
  uint32_t* const s_mix = reinterpret_cast<uint32_t*>(s_idx);
  if(sampled)
  {
    for(uint32_t k = tid; k < nrun; k += kZoneThreads)
    {
      const uint32_t lo = k * kCarryRun, hi = min(lo + kCarryRun, nc);
      const uint32_t a0 = C[lo].w0 & kZoneMask, a1 = C[hi - 1].w0 & kZoneMask;
      if(a0 == a1)
        atomicAdd(&s_ccnt[a0], hi - lo);
      else
        s_mix[atomicAdd(&s_nmix, 1u)] = k;
    }
    __syncthreads();
    nmix = s_nmix;
  }
  const uint32_t ncount = sampled ? nmix * kCarryRun : nc;
  for(uint32_t base = 0; base < ncount; base += kZoneThreads * kUnroll)
  {
    uint32_t w[kUnroll];
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
    {
      const uint32_t j = base + u * kZoneThreads + tid;
      const uint32_t i = sampled ? s_mix[min(j, ncount - 1) / kCarryRun] * kCarryRun + j % kCarryRun : j;
      w[u] = (j < ncount && i < nc) ? C[i].w0 : 0xFFFFFFFFu;
    }
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
      agg_count(s_ccnt, w[u] & kZoneMask, w[u] != 0xFFFFFFFFu);
  }
  // Landed records: with the LDS index, each record's rank among its actor's
  // arrivals comes back from the counting atomic and stays in a register
  // (packed rank << 11 | actor), so placing it needs no second pass over the
  // landing buffer. kIdxPer loads in flight per thread.
  // The zone's type when one type covers all of its slots, else -1. It is
  // wave-uniform, so that type's fields (batch, state, params) come through
  // scalar loads instead of a per-lane lookup chain.
  int tz = -1;
  for(uint32_t t = 0; t < c_eng.n_types; ++t)
    if(L0 >= c_types[t].lfirst && L0 + nact <= c_types[t].lfirst + c_types[t].lcount)
      tz = (int)t;
  tz = __builtin_amdgcn_readfirstlane(tz);
  if constexpr(PM == 1)
    if(tz < 0) return false;
  // A zone of a two-pass table that may take that path (no backpressure
  // anywhere, one type) loads its actors' state now, coalesced, so that the
  // loads land while the landing buffer is counted; dropped if it does not.
  constexpr int kPW = plan_words<HTS>();
  uint64_t st[kRounds][kPW];
  if constexpr(HTS >= 0 && two_pass<HTS>())
    if(PM != 2 && !gate && ztc == 0 && tz >= 0)
    {
      const TypeDev& T = c_types[tz];
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t i = r * kZoneThreads + tid;
#pragma unroll
        for(int k = 0; k < kPW; ++k)
          st[r][k] = i < nact ? T.state[(size_t)k * T.lcount + (L0 + i - T.lfirst)] : 0ull;
      }
    }
  uint32_t wr[kIdxPer];
  if constexpr(kDP)
  {
    // dp's first pass rides on the count: each landed record, whole (its
    // line is read for the count anyway), in chunks of kDpChunk per thread;
    // its behaviour runs on a throwaway state with a counting context, whose
    // send is counted in the receiving actor's drain round and its bucket
    // (the sends of a message-local behaviour do not depend on the state or
    // the order: the second pass, in canonical order, makes the same ones)
    constexpr int kDpChunk = 8;
    static_assert(kIdxPer % kDpChunk == 0, "dp count chunks");
    const TypeDev& T = c_types[tz];
    PlanCtx pc;
    pc.reset_common();
    pc.type = tz;
#pragma unroll
    for(int u0 = 0; u0 < kIdxPer; u0 += kDpChunk)
    {
      uint4 rr[kDpChunk];
#pragma unroll
      for(int v = 0; v < kDpChunk; ++v)
      {
        const uint32_t i = (u0 + v) * kZoneThreads + tid;
        if(i < nl) rr[v] = ld16(reinterpret_cast<const uint4*>(Ld + i));
        else rr[v].x = 0xFFFFFFFFu;
      }
#pragma unroll
      for(int v = 0; v < kDpChunk; ++v)
      {
        wr[u0 + v] = rr[v].x;
        if(rr[v].x == 0xFFFFFFFFu) continue;
        const uint32_t act = rr[v].x & kZoneMask;
        wr[u0 + v] = (atomicAdd(&s_cnt[act], 1u) << kZoneBits) | act;
        const uint32_t rd = act / kZoneThreads;               // its drain round
        pc.rh = s_hist + (rd >> 1) * nb;
        pc.inc = (rd & 1u) ? 0x10000u : 1u;
        pc.self = (L0 + act) * R + me;
        pc.li = L0 + act - T.lfirst;
        pc.src_local = act;
        uint64_t junk[HT_Words<HTS>::W] = {};
        handle(HtTag<HTS>{}, T, pc, junk, (rr[v].x >> 12) & 0xFu,
               ((uint64_t)rr[v].w << 32) | rr[v].z);
      }
    }
  }
  else if(use_idx)
  {
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
    {
      const uint32_t i = u * kZoneThreads + tid;
      wr[u] = i < nl ? Ld[i].w0 : 0xFFFFFFFFu;
    }
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
      if(wr[u] != 0xFFFFFFFFu)
      {
        const uint32_t act = wr[u] & kZoneMask;
        wr[u] = (atomicAdd(&s_cnt[act], 1u) << kZoneBits) | act;
      }
  }
  else if(hot)
    for(uint32_t i = tid; i < kZone; i += kZoneThreads)
    {
      s_cnt[i] = hot_cnt[i];
      const_cast<uint32_t*>(hot_cnt)[i] = 0;     // (k_hot's next use of the slot is a later launch)
    }
  else
  for(uint32_t base = 0; base < nl; base += kZoneThreads * kUnroll)
  {
    uint32_t w[kUnroll];
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
    {
      const uint32_t i = base + u * kZoneThreads + tid;
      w[u] = i < nl ? Ld[i].w0 : 0xFFFFFFFFu;
    }
    // (a hot receiver's arrivals: lanes of one actor folded into one atomic)
#pragma unroll
    for(int u = 0; u < kUnroll; ++u)
      agg_count<8>(s_cnt, w[u] & kZoneMask, w[u] != 0xFFFFFFFFu);
  }
  __syncthreads();
  GPA_STAMP(1);
  // The zone takes its mail: its pending count, the reset of its counters of
  // parity cur and (PM 1) its mark are stored at the very end of the launch
  // (nothing in this launch reads them again). Stored here, they were waited
  // out by the zone's next __syncthreads — a store acknowledgement while the
  // whole GPU streams its landing buffers.
  bool took_mail = false;
  auto take_mail = [&]() __attribute__((always_inline)) { took_mail = true; };
  if constexpr(PM != 1) take_mail();


  // An order-free table (its behaviours ignore the message: the message-ubench
  // pinger) needs only each actor's message count when nothing can be left
  // over this step: no actor anywhere triggers muting (so none is muted or
  // mutes itself; none of this zone's carries a trigger byte either), and
  // every actor's mail fits its batch. Its records are
  // then never read — no segment scan, no index, no group sort. Otherwise
  // the zone takes the general path below.
  bool fast = false, plan = false;
  // two-pass tables: each round's own actor's message count, its count class
  // (busiest first) and its rank among the zone's actors of that class (the
  // plan path deals the actors to threads by count; the class histogram s_ph)
  uint32_t own_n[kRounds], pk[kRounds], prk[kRounds];
  if constexpr(HTS >= 0 && order_free<HTS>())
    if(!gate && ztc == 0 && tz >= 0)
    {
      const uint32_t bt = c_types[tz].prio ? 0xFFFFFFFFu : c_types[tz].batch;
      int over = 0;
      uint32_t tot = 0;
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t i = r * kZoneThreads + tid;
        const uint32_t c = s_cnt[i] + s_ccnt[i];
        over |= c > bt;
        tot += c;
        if constexpr(two_pass<HTS>())
          if(PM != 2)
          {
            own_n[r] = i < nact ? c : 0u;
            pk[r] = kClasses - 1u - min(own_n[r], kClasses - 1u);
            prk[r] = agg_add(s_ph, pk[r], true);
          }
      }
      GPA_STAMP(13);                         // diagnostic build: the class ranks are back
      tot = (uint32_t)min(wave_sum((unsigned long long)tot), 0xFFFFFFFFull);
      if(lane == 0 && tot) atomicAdd(&s_tot, tot);
      fast = !__syncthreads_or(over);
      GPA_STAMP(14);
      // two passes when every (round, bucket) count fits 16 bits and no
      // actor can run out of sequence numbers (pass 1 would count the
      // overflow again): the zone's messages, each sending at most one, are
      // fewer than seq_max
      if constexpr(two_pass<HTS>())
        plan = PM != 2 && fast && s_tot < c_eng.seq_max && c_eng.two_pass != 0u;
    }
  if constexpr(PM == 1)
  {
    if constexpr(kPlanSplit)
    {
      if(!plan) return false;                         // uniform: left to PM 2
    }
    else
    {
      int big = 0;
      for(uint32_t i = tid; i < kZone; i += kZoneThreads) big |= s_cnt[i] > kBigGroup;
      if(__syncthreads_or(big)) return false;         // a hot group: left to PM 2
      if constexpr(kDP)
      {
        // two passes when every actor's mail runs this step (its batch holds
        // it: nothing carries over, which the first pass could not know)
        // Groups past drain_commutative's register slots are put in
        // canonical order by the workgroup first (listed here, at most
        // kMaxStage of them with kZoneThreads records in all: else PM 2).
        const uint32_t bt = c_types[tz].prio ? 0xFFFFFFFFu : c_types[tz].batch;
        if(tid == 0) { s_stn = 0; s_sto[0] = 0; }
        __syncthreads();
        int over = 0;
        for(uint32_t i = tid; i < kZone; i += kZoneThreads)
        {
          const uint32_t c = s_cnt[i];
          over |= c > bt;
          if(c > small_regs<HTS>())
          {
            const uint32_t k = atomicAdd(&s_stn, 1u);
            if(k < kMaxStage) s_stl[k] = i;
            atomicAdd(&s_sto[0], c);
          }
        }
        __syncthreads();
        over |= s_stn > kMaxStage || s_sto[0] > (uint32_t)kZoneThreads;
        dp = !__syncthreads_or(over);
        // (otherwise left to PM 2's general path: PM 1 has written nothing
        // outside LDS, and keeps only the two-pass drain's registers)
        if(!dp) return false;
      }
    }
    take_mail();
  }
  ZRec* Sz = c_eng.S + 3 * zo;
  // S path: the sorted items of the groups the workgroup sorted, each at its
  // segment offset (S's last third, 2 cap items; read by the drain, the
  // carry-out and k_carry_big)
  uint64_t* const perm_s = reinterpret_cast<uint64_t*>(Sz + 2 * cap);
  if(fast)
  {
    // the actor's total (carried + landed); no group was sorted
    for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_cnt[i] += s_ccnt[i];
    for(uint32_t k = tid; k < kZone / 32; k += kZoneThreads) s_bigbits[k] = 0;
    __syncthreads();
  }
  else
  {
  block_scan_zone_pair(s_cnt, s_ccnt, s_off, s_aux, s_tmp2);
  GPA_STAMP(2);

  // ---- 2. place into the sorted inbox ---------------------------------------------
  // (the two forms apart: a record held across the branch went to scratch)
  if(use_idx)
    for(uint32_t i0 = 0; i0 < nc; i0 += kZoneThreads * kUnroll)
    {
      uint32_t w[kUnroll];
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        w[u] = i < nc ? C[i].w0 : 0u;
      }
#pragma unroll
      for(int u = 0; u < kUnroll; ++u)
      {
        const uint32_t i = i0 + u * kZoneThreads + tid;
        if(i >= nc) continue;
        const uint32_t a = w[u] & kZoneMask;
        s_idx[s_off[a] + (i - s_aux[a])] = (uint16_t)i;
      }
    }
  // (S path: carried mail stays where it is, read in place through AccS)
  if(use_idx)
  {
    // LDS index only: records stay in the landing buffer (dp: at the pool's
    // end, so that the rest of the pool is one tile once the per-actor arrays
    // are in registers)
    uint16_t* const s_ix = dp ? dp_index(s_pool, nl) : s_idx;
#pragma unroll
    for(int u = 0; u < kIdxPer; ++u)
      if(wr[u] != 0xFFFFFFFFu)
      {
        const uint32_t act = wr[u] & kZoneMask;
        s_ix[s_off[act] + s_ccnt[act] + (wr[u] >> kZoneBits)] = (uint16_t)(nc + u * kZoneThreads + tid);
      }
  }
  else
  {
    // each actor's carry start moves to s_cst (the index area, unused on this
    // path) and its S segment holds only arrivals: scan(cnt + ccnt) - scan(ccnt)
    __syncthreads();
    for(uint32_t i = tid; i < kZone; i += kZoneThreads)
    {
      s_cst[i] = s_aux[i];
      s_off[i] -= s_aux[i];
      s_aux[i] = 0;
    }
    __syncthreads();
    // Two half-batches of kUnroll / 2 records per thread, software-pipelined:
    // one half's loads are issued before the other half's stores, so waiting
    // for a load never waits out the stores before it (vmcnt counts both, in
    // issue order) — a hot receiver's zone places ~10^5 records here.
    constexpr int kH = kUnroll / 2;
    constexpr uint32_t kStride = kZoneThreads * kH;
    auto load_half = [&](uint4 (&r)[kH], uint32_t b0) __attribute__((always_inline)) {
#pragma unroll
      for(int u = 0; u < kH; ++u)
      {
        const uint32_t i = b0 + u * kZoneThreads + tid;
        // unconditional (clamped) loads: all in flight, the records in registers
        r[u] = *reinterpret_cast<const uint4*>(Ld + min(i, nl - 1));
        if(i >= nl) r[u].x = 0xFFFFFFFFu;
      }
    };
    auto place_half = [&](const uint4 (&r)[kH]) __attribute__((always_inline)) {
      uint32_t pos[kH];
#pragma unroll
      for(int u = 0; u < kH; ++u)
      {
        const uint32_t a = r[u].x & kZoneMask;
        pos[u] = s_off[a] + agg_add<8>(s_aux, a, r[u].x != 0xFFFFFFFFu);
      }
#pragma unroll
      for(int u = 0; u < kH; ++u)
        if(r[u].x != 0xFFFFFFFFu) *reinterpret_cast<uint4*>(Sz + pos[u]) = r[u];
    };
    if(nl && !hot)
    {
      uint4 ra[kH], rb[kH];
      load_half(ra, 0);
      for(uint32_t b0 = 0; b0 < nl; b0 += 2 * kStride)
      {
        load_half(rb, b0 + kStride);
        place_half(ra);
        load_half(ra, b0 + 2 * kStride);
        place_half(rb);
      }
    }
  }
  // from here on s_cnt is the actor's total: carried + landed
  for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_cnt[i] += s_ccnt[i];
  __syncthreads();
  GPA_STAMP(3);

  // Hot receivers: groups above kBigGroup sorted by the whole workgroup
  // (s_bigbits marks them for drain_zone). The sort borrows s_dyn, which the
  // behaviours' bucket counts use next, and the zone's outbox / S scratch.
  for(uint32_t k = tid; k < kZone / 32; k += kZoneThreads) s_bigbits[k] = 0;
  if(tid == 0) s_nbig = 0;
  __syncthreads();
  for(uint32_t i = tid; i < nact; i += kZoneThreads)
    if(s_cnt[i] - s_ccnt[i] > kBigGroup)
    {
      if(hot)
        atomicOr(&s_bigbits[i >> 5], 1u << (i & 31));   // sorted by k_hot, in place
      else
      {
        const uint32_t k = atomicAdd(&s_nbig, 1u);
        if(k < kMaxBig) s_big[k] = i;
      }
    }
  __syncthreads();
  {
    const uint32_t nbig = kSimple ? 0u : min(s_nbig, kMaxBig);     // past kMaxBig: the lane sorts (slow, exact)
    if(nbig)
    {
      uint64_t* ia = reinterpret_cast<uint64_t*>(c_eng.O + zo);
      for(uint32_t k = 0; k < nbig; ++k)
      {
        const uint32_t i = s_big[k];
        const uint32_t g = s_cnt[i] - s_ccnt[i];
        bool ok;
        if(use_idx)
          ok = coop_sort_group(AccIdx{s_idx + s_off[i], C, Ld, nc}, s_idx + s_off[i],
                               s_ccnt[i], g, ia, ia + g, s_dyn, s_red3);
        else
          ok = coop_sort_group(AccS{Sz + s_off[i], C + s_cst[i], s_ccnt[i]}, nullptr,
                               s_ccnt[i], g, perm_s + s_off[i], ia, s_dyn, s_red3);
        if(ok && tid == 0) s_bigbits[i >> 5] |= 1u << (i & 31);
      }
      for(uint32_t b = tid; b < max(nb, kSortWork); b += kZoneThreads) s_dyn[b] = 0;
      __syncthreads();
    }
  }
  }   // general path
  GPA_STAMP(7);                          // diagnostic build: the hot-group sort ends
  auto big_sorted = [&](uint32_t i) __attribute__((always_inline)) {
    return !kSimple && ((s_bigbits[i >> 5] >> (i & 31)) & 1u) != 0u;
  };
  // S path accessor of actor i (a group the workgroup sorted: read through its items)
  auto acc_s = [&](uint32_t i) __attribute__((always_inline)) {
    AccS a_{Sz + s_off[i], C + s_cst[i], s_ccnt[i]};
    if(big_sorted(i) && !hot) a_.perm = perm_s + s_off[i];
    return a_;
  };


  uint32_t delivered = 0, active = 0, sent = 0, applied = 0;
  uint32_t n_atom = 0, dropped = 0, xover = 0;
  uint32_t ncout = 0;
  ZoneCtx a;
  a.reset_common();
  if constexpr(HTS >= 0 && two_pass<HTS>())
    if(plan)
    {
      // ---- 3'. order-free zone: plan, reserve, emit (no outbox) -----------------------
      constexpr int NW = HT_Words<HTS>::W;
      const TypeDev T = c_types[tz];
      // per bucket, two rounds per u32 (16-bit halves: the zone's sends are
      // fewer than seq_max, so no half carries into the other):
      uint32_t* const s_rh = s_dyn;             // [2][nb] sends per (round, bucket) -> tile starts
      uint32_t* const s_cur = s_dyn + 2 * nb;   // [2][nb] tile cursors (from the starts)
      uint32_t* const s_bs = s_dyn + 4 * nb;    // [2][nb] each chunk's next free place (chunk_dst),
                                                //   round r reads half r & 1, writes the other
      uint4* const tile = s_pool;                // pass 2 (the whole pool)
      for(uint32_t b = tid; b < 2 * nb; b += kZoneThreads) s_rh[b] = 0;
      // Lanes of a wave run their actors' behaviours side by side, so a wave
      // takes as long as its busiest lane, and the four waves a SIMD holds
      // share its VALU. The zone's actors are therefore dealt to threads by
      // message count: counting-sorted (busiest first; the class histogram
      // s_ph was filled beside the fast check) into 64-actor blocks, and
      // block (wave w, round r) = 8g + (r or 7 - r) for j = w (or W - 1 - w
      // on odd rounds), g = j / 2 — every wave gets alike counts in its lanes
      // and a like total over its rounds, and every round a like share of
      // the zone's sends (the tile). The state moves through LDS (coalesced
      // loads — issued before the count phase — and stores; the permuted
      // threads read and write it there).
      constexpr bool kStageApart =
        kZone * sizeof(uint32_t) + NW * kZone * sizeof(uint64_t) + kZone * sizeof(uint16_t)
          <= kTile * sizeof(uint4);
      uint64_t* const s_stage = reinterpret_cast<uint64_t*>(s_pool) + (kStageApart ? kZone / 2 : 0);
      uint16_t* const s_perm = reinterpret_cast<uint16_t*>(s_pool + kTile) - kZone;
      static_assert(NW * kZone * sizeof(uint64_t) + kZone * sizeof(uint16_t) <= kTile * sizeof(uint4),
                    "two-pass state stage and permutation fit the pool");
      if(wv == 0)
      {
        const uint32_t c = lane < kClasses ? s_ph[lane] : 0u;
        const uint32_t x = wave_incl_scan(c, lane) - c;
        if(lane < kClasses) s_ph[lane] = x;
      }
      lds_sync();
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
        s_perm[s_ph[pk[r]] + prk[r]] = (uint16_t)(r * kZoneThreads + tid);
      lds_sync();
      uint32_t ai[kRounds], nm[kRounds];
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t j = (r & 1u) ? (uint32_t)kZoneWaves - 1u - wv : wv;
        const uint32_t blk = 8u * (j >> 1) + ((j & 1u) ? 7u - r : r);
        ai[r] = s_perm[64u * blk + lane];
        nm[r] = s_cnt[ai[r]];
      }
      if constexpr(!kStageApart)
        lds_sync();                            // every s_cnt read done: the stage overwrites it
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
#pragma unroll
        for(int k = 0; k < NW; ++k)
          s_stage[k * kZone + r * kZoneThreads + tid] = st[r][k];
      lds_sync();
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
#pragma unroll
        for(int k = 0; k < NW; ++k)
          st[r][k] = s_stage[k * kZone + ai[r]];
#ifdef GPA_STAMPS
      GPA_STAMP(8);                           // the permuted state is in registers
      if(tid == 0) { c_eng.dbg[z * kDbgSlots + 9] = 0; c_eng.dbg[z * kDbgSlots + 10] = 0; }
#endif
      // pass 1: count the sends of each round per bucket
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        if(!nm[r]) continue;
        const uint32_t i = ai[r];
        PlanCtx pc;
        pc.reset_common();
        pc.li = L0 + i - T.lfirst;
        pc.self = (L0 + i) * R + me;
        pc.src_local = i;
        pc.type = tz;
        pc.rh = s_rh + (r >> 1) * nb;
        pc.inc = (r & 1u) ? 0x10000u : 1u;
        uint64_t sc[NW];
#pragma unroll
        for(int k = 0; k < NW; ++k) sc[k] = st[r][k];
        for(uint32_t j = 0; j < nm[r]; ++j) handle(HtTag<HTS>{}, T, pc, sc, 0u, 0ull);
      }
      lds_sync();
      GPA_STAMP(3);
      // one chunk per bucket for the zone's sends
      n_atom += plan_reserve(s_rh, s_bs, nb, nz, nxt, tid);
      GPA_STAMP(5);
#ifdef GPA_STAMPS
      const unsigned long long t_scan = __builtin_amdgcn_s_memtime();
#endif
      // every round's bucket starts in the tile at once
      uint32_t tot01, tot23;
      plan_scan(s_rh, s_cur, nb, s_tmp2, tid, tot01, tot23);
#ifdef GPA_STAMPS
      GPA_ACC(9, t_scan);
#endif
      // pass 2, one round at a time
      TileCtx tc;
      tc.reset_common();
      tc.tile = tile;
      tc.tcap = kPlanTile;
      tc.L0 = L0; tc.nz = nz; tc.nxt = nxt; tc.xover = 0;
      uint32_t dz = 0;
#ifdef GPA_STAMPS
      unsigned long long emit_clk = 0, t_emit = 0;    // diagnostic build: Σ tile-emit time
#endif
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t sh = (r & 1u) * 16u;
        const uint32_t* const rst = s_rh + (r >> 1) * nb;       // the round's starts (half sh)
        const uint32_t tr = (((r >> 1) ? tot23 : tot01) >> sh) & 0xFFFFu;   // the round's sends
        tc.cur = s_cur + (r >> 1) * nb;
        const uint32_t* const bsr = s_bs + (r & 1u) * nb;
        uint32_t* const bsw = s_bs + ((r & 1u) ^ 1u) * nb;
        tc.st = rst; tc.bs = bsr;
        tc.sh = sh; tc.inc = 1u << sh;
#ifdef GPA_STAMPS
        const unsigned long long t_hand = __builtin_amdgcn_s_memtime();
#endif
        if(nm[r])
        {
          const uint32_t i = ai[r];
          const uint32_t L = L0 + i;
          tc.li = L - T.lfirst;
          tc.self = L * R + me;
          tc.src_local = i;
          tc.type = tz;
          tc.seq = 0;
          for(uint32_t j = 0; j < nm[r]; ++j) handle(HtTag<HTS>{}, T, tc, st[r], 0u, 0ull);
          // overloaded iff a full batch ran (batch_limit_reached, actor.c:369-381);
          // nothing here mutes
          const bool full = T.prio ? (nm[r] % T.batch == 0u) : nm[r] == T.batch;
          s_tb[i] = full ? 1u : 0u;
          if(full) atomicAdd(&s_ntrig, 1u);
          delivered += nm[r];
          active += 1;
          dz += nm[r];
        }
        lds_sync();
#ifdef GPA_STAMPS
        GPA_ACC(10, t_hand);
        t_emit = __builtin_amdgcn_s_memtime();
#endif
        // the tile, sorted by bucket, to the chunks; the chunks' next free
        // places for the next round
        xover += plan_emit(tile, min(tr, kPlanTile), rst, bsr, bsw, sh, tr, nb, L0, nz, nxt, tid);
        lds_sync();
#ifdef GPA_STAMPS
        emit_clk += __builtin_amdgcn_s_memtime() - t_emit;
#endif
      }
      // the new state back through the stage: permuted into LDS, coalesced out
      // (the last round's emit is behind a barrier: the pool is free)
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
#pragma unroll
        for(int k = 0; k < NW; ++k)
          s_stage[k * kZone + ai[r]] = st[r][k];
      lds_sync();
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t i = r * kZoneThreads + tid;
        if(own_n[r])
#pragma unroll
          for(int k = 0; k < NW; ++k)
            T.state[(size_t)k * T.lcount + (L0 + i - T.lfirst)] = s_stage[k * kZone + i];
      }
#ifdef GPA_STAMPS
      if(tid == 0) c_eng.dbg[z * kDbgSlots + 2] = emit_clk;
#endif
      sent = tc.sent;
      xover += tc.xover;
      if(dz) atomicAdd(&s_bytype[tz], (unsigned long long)dz);
    }
  if constexpr(kDP)
    if(dp)
    {
      // ---- 3''. message-local plain zone, second pass: the canonical drain
      //      straight into bucket-sorted LDS tiles, one per drain round -------
      const TypeDev& T = c_types[tz];
      {
        // the listed groups (past the register slots) into canonical order in
        // the index: one thread per record counts the group's keys below its
        // own, then every record moves to its rank (keys are distinct)
        uint16_t* const s_ix = dp_index(s_pool, nl);
        const uint32_t nbg = s_stn;                        // <= kMaxStage (dp)
        if(nbg)
        {
          if(tid == 0)
          {
            uint32_t o = 0;
            for(uint32_t k = 0; k < nbg; ++k) { s_sto[k] = o; o += s_cnt[s_stl[k]]; }
            s_sto[nbg] = o;                                  // <= kZoneThreads (dp)
          }
          lds_sync();
          uint16_t x = 0;
          uint32_t rank = 0, off = 0;
          if(tid < s_sto[nbg])
          {
            uint32_t k = 0;
            while(k + 1 < nbg && s_sto[k + 1] <= tid) ++k;
            const uint32_t i = s_stl[k], g = s_cnt[i];
            off = s_off[i];
            x = s_ix[off + tid - s_sto[k]];
            const uint64_t key = zkey(ld_rec(Ld + x));
            for(uint32_t j0 = 0; j0 < g; j0 += 4)
            {
              uint64_t kk[4];
#pragma unroll
              for(uint32_t u = 0; u < 4; ++u)
                kk[u] = j0 + u < g ? zkey(ld_rec(Ld + s_ix[off + j0 + u])) : ~0ull;
#pragma unroll
              for(uint32_t u = 0; u < 4; ++u) rank += kk[u] < key ? 1u : 0u;
            }
          }
          __syncthreads();
          if(tid < s_sto[nbg]) s_ix[off + rank] = x;
          __syncthreads();
        }
      }
      uint32_t* const s_rh = s_dyn;             // [2][nb] sends per (round, bucket) -> tile starts
      uint32_t* const s_cur = s_dyn + 2 * nb;   // [2][nb] tile cursors
      uint32_t* const s_bs = s_dyn + 4 * nb;    // [2][nb] chunks' next free places (ping-pong)
      n_atom += plan_reserve(s_rh, s_bs, nb, nz, nxt, tid);
      uint32_t tot01, tot23;
      plan_scan(s_rh, s_cur, nb, s_tmp2, tid, tot01, tot23);
      // each thread's actors (one a round) in registers: the per-actor arrays'
      // part of the pool becomes the tile, up to the index at its end
      // (packed: segment offset << 8 | count; plain zones' counts are at
      // most kBigGroup, their offsets below kIdxCap)
      static_assert(kBigGroup < 256 && kIdxCap <= (1u << 24), "dn / doff pack");
      uint32_t dno[kRounds];
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t i = r * kZoneThreads + tid;
        dno[r] = i < nact ? (s_off[i] << 8) | s_cnt[i] : 0u;
      }
      lds_sync();
      GPA_STAMP(8);                           // diagnostic build: the rounds start
#ifdef GPA_STAMPS
      if(tid == 0) { c_eng.dbg[z * kDbgSlots + 9] = 0; c_eng.dbg[z * kDbgSlots + 10] = 0; }
#endif
      const uint16_t* const s_ix = dp_index(s_pool, nl);
      TileCtx tc;
      tc.reset_common();
      tc.tile = s_pool;
      tc.tcap = dp_tile_cap(nl);
      tc.L0 = L0; tc.nz = nz; tc.nxt = nxt; tc.xover = 0;
      tc.type = tz;
      uint32_t dz = 0;
#pragma unroll
      for(uint32_t r = 0; r < kRounds; ++r)
      {
        const uint32_t sh = (r & 1u) * 16u;
        const uint32_t* const rst = s_rh + (r >> 1) * nb;
        const uint32_t tr = (((r >> 1) ? tot23 : tot01) >> sh) & 0xFFFFu;
        tc.cur = s_cur + (r >> 1) * nb;
        const uint32_t* const bsr = s_bs + (r & 1u) * nb;
        uint32_t* const bsw = s_bs + ((r & 1u) ^ 1u) * nb;
        tc.st = rst; tc.bs = bsr;
        tc.sh = sh; tc.inc = 1u << sh;
#ifdef GPA_STAMPS
        const unsigned long long t_dr = __builtin_amdgcn_s_memtime();
#endif
        if(dno[r] & 0xFFu)
        {
          const uint32_t i = r * kZoneThreads + tid;
          const uint32_t L = L0 + i;
          tc.li = L - T.lfirst;
          tc.self = L * R + me;
          tc.src_local = i;
          tc.seq = 0;
          const uint32_t d = drain_commutative<HTS>(T, tc,
            AccIdx{const_cast<uint16_t*>(s_ix) + (dno[r] >> 8), C, Ld, 0u}, dno[r] & 0xFFu);
          // overloaded iff a full batch ran (batch_limit_reached,
          // actor.c:369-381); nothing here mutes
          const bool full = T.prio ? (d % T.batch == 0u) : d == T.batch;
          s_tb[i] = full ? 1u : 0u;
          if(full) atomicAdd(&s_ntrig, 1u);
          delivered += d;
          active += 1;
          dz += d;
        }
        lds_sync();
#ifdef GPA_STAMPS
        GPA_ACC(9, t_dr);                     // the round's drain (to its barrier)
        const unsigned long long t_em = __builtin_amdgcn_s_memtime();
#endif
        xover += plan_emit(s_pool, min(tr, tc.tcap), rst, bsr, bsw, sh, tr, nb, L0, nz, nxt, tid);
        lds_sync();
#ifdef GPA_STAMPS
        GPA_ACC(10, t_em);                    // the round's tile emit
#endif
      }
      sent = tc.sent;
      xover += tc.xover;
      if(dz) atomicAdd(&s_bytype[tz], (unsigned long long)dz);
    }
  if(!(PM == 1 && kPlanSplit) && !plan && !dp)
  {
  // s_aux will hold each actor's unhandled remainder (known after it ran)
  for(uint32_t i = tid; i < kZone; i += kZoneThreads) s_aux[i] = 0;
  int any_rem = 0;

  // ---- 2b. staged runs (scratch path): an actor that handles a long run of
  // records in canonical order — its carried mail, then its arrivals when the
  // workgroup or k_hot sorted them — reads them one after another, a memory
  // round trip each (a hot receiver's backlog: 100 a step, ~40 us of its
  // zone). The workgroup loads the prefix each such actor handles this step
  // into LDS first (the index area past the carry starts, free on this path),
  // all loads in flight; s_aux[i] = stage offset << 16 | records until the
  // actor's own drain overwrites it.
  bool staged = false;
  uint4* const s_stage = reinterpret_cast<uint4*>(s_cst + kZone);
  if constexpr(!kSimple)
    if(!use_idx && !fast)
    {
      if(tid == 0) s_stn = 0;
      __syncthreads();
      for(uint32_t i = tid; i < nact; i += kZoneThreads)
      {
        const uint32_t n = s_cnt[i];
        if(n < kStageMin) continue;
        const int t = tz >= 0 ? tz : type_of_local(L0 + i);
        if(t < 0 || c_types[t].reducible) continue;
        const uint32_t w = c_types[t].prio ? n : min(n, c_types[t].batch);
        const uint32_t run = min(w, big_sorted(i) ? n : s_ccnt[i]);   // the canonical prefix handled
        if(run < kStageMin) continue;
        const uint32_t k = atomicAdd(&s_stn, 1u);
        if(k < kMaxStage) { s_stl[k] = i; s_stc[k] = run; }
      }
      __syncthreads();
      const uint32_t ns = min(s_stn, kMaxStage);
      if(ns)
      {
        if(tid == 0)
        {
          uint32_t o = 0;
          for(uint32_t k = 0; k < ns; ++k)
          {
            const uint32_t c = min(s_stc[k], kStageCap - o);
            s_sto[k] = o; s_stc[k] = c; o += c;
          }
          s_sto[ns] = o;
        }
        __syncthreads();
        if(tid < ns && s_stc[tid]) s_aux[s_stl[tid]] = (s_sto[tid] << 16) | s_stc[tid];
        const uint32_t tot = s_sto[ns];
        for(uint32_t t0 = tid; t0 < tot; t0 += kZoneThreads)
        {
          uint32_t k = 0;
          while(k + 1 < ns && s_sto[k + 1] <= t0) ++k;
          const ZRec r = acc_s(s_stl[k]).rec(t0 - s_sto[k]);
          s_stage[t0] = make_uint4(r.w0, r.from, (uint32_t)r.arg, (uint32_t)(r.arg >> 32));
        }
        __syncthreads();
        staged = true;
      }
    }
  GPA_STAMP(15);                         // diagnostic build: staged runs loaded

  // ---- 3. run handlers -------------------------------------------------------------
  a.out = c_eng.O + zo;
  a.s_nout = &s_nout;
  a.ocap = cap;
  a.nxt = nxt;
  a.s_hist = s_hist;
  a.agg = &s_agg[wv];
  // fan-in senders fold their analyzer applies per zone in LDS
  if constexpr(kFan)
    if(tz >= 0 && c_types[tz].ht == GPU_ACTOR_HT_FANIN_SENDER)
    {
      a.fan_t = type_of_global((uint32_t)c_types[tz].params[1]);
      if(a.fan_t >= 0) a.fan = s_fan;
    }
  // drain local actor i, of type t (T = c_types[t])
  uint8_t* const trig_cur = (!kSimple && gate) ? c_eng.trig[cur] : nullptr;
  auto drain_actor = [&](const TypeDev& T, int t, uint32_t i) __attribute__((always_inline)) {
    const uint32_t n = s_cnt[i];
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
#define ZDRAIN(HT)                                                                    \
    if(use_idx)                                                                       \
    {                                                                                 \
      AccIdx acc{s_idx + s_off[i], C, Ld, nc};                                        \
      d = zone_actor<HT>(T, a, acc, n, s_ccnt[i], stays, big_sorted(i));              \
    }                                                                                 \
    else                                                                              \
    {                                                                                 \
      AccS acc = acc_s(i);                                                            \
      if(staged)                                                                      \
      {                                                                               \
        const uint32_t sg = s_aux[i];                                                 \
        if(sg) { acc.stg = s_stage + (sg >> 16); acc.nst = sg & 0xFFFFu; }            \
      }                                                                               \
      d = zone_actor<HT>(T, a, acc, n, s_ccnt[i], stays, big_sorted(i));              \
    }
    if constexpr(HTS == kHtFifoPair)
    {
      if(T.ht == GPU_ACTOR_HT_FIFO_SRC)
      {
        ZDRAIN(GPU_ACTOR_HT_FIFO_SRC)
      }
      else
      {
        ZDRAIN(GPU_ACTOR_HT_FIFO_SINK)
      }
    }
    else if constexpr(HTS >= 0)
    {
      ZDRAIN(HTS)
    }
    else
    {
      switch(T.ht)
      {
// (GPA_MIX_MASK: the tables a run-time compiled any-mix step holds, bit
// per table id — engine.hip jit; the others' cases are not compiled)
#define ZCASE(HT) case HT: if constexpr(((GPA_MIX_MASK) >> (HT)) & 1u) { ZDRAIN(HT) } break;
        ZCASE(GPU_ACTOR_HT_RING)
        ZCASE(GPU_ACTOR_HT_PINGER)
        ZCASE(GPU_ACTOR_HT_PINGER_DET)
        ZCASE(GPU_ACTOR_HT_FANIN_SENDER)
        ZCASE(GPU_ACTOR_HT_GUPS_STREAMER)
        ZCASE(GPU_ACTOR_HT_STORM)
        ZCASE(GPU_ACTOR_HT_FIFO_SRC)
        ZCASE(GPU_ACTOR_HT_FIFO_SINK)
        ZCASE(GPU_ACTOR_HT_SPREADER)
        ZCASE(GPU_ACTOR_HT_PROGRAM)
#undef ZCASE
        default: break;
      }
    }
#undef ZDRAIN
    // overloaded iff a full batch ran (a priority type's last batch) and the
    // actor was not muted (batch_limit_reached, actor.c:369-381; maybe_mute
    // first, 449-460)
    const bool full = T.prio ? (d != 0u && d % T.batch == 0u) : d == T.batch;
    const uint32_t o = (full && !a.mute_hit) ? 1u : 0u;
    const uint32_t m = (stays || a.mute_hit) ? 1u : 0u;
    if(a.mute_hit) c_eng.muted_on[L] = a.mute_to;
    const uint32_t nb_ = o | (m << 1);
    s_tb[i] = (uint8_t)nb_;
    if(nb_) atomicAdd(&s_ntrig, 1u);
    s_aux[i] = n - d;
    any_rem |= (n - d) != 0u;
    delivered += d;
    active += d ? 1u : 0u;
    return d;
  };
  if(tz >= 0)
  {
    const TypeDev& T = c_types[tz];
    uint32_t dz = 0;
    if(!T.reducible)
      for(uint32_t i = tid; i < nact; i += kZoneThreads)
        if(s_cnt[i] || s_tb[i]) dz += drain_actor(T, tz, i);
    if(dz) atomicAdd(&s_bytype[tz], (unsigned long long)dz);
  }
  else
  {
    for(uint32_t i = tid; i < nact; i += kZoneThreads)
    {
      if(s_cnt[i] == 0 && s_tb[i] == 0) continue;
      const int t = type_of_local(L0 + i);
      if(t < 0 || c_types[t].reducible) continue;
      const uint32_t d = drain_actor(c_types[t], t, i);
      if(d) atomicAdd(&s_bytype[t], (unsigned long long)d);
    }
  }
  GPA_STAMP(16);                         // diagnostic build: the drain ends
  sent = a.sent;
  applied = a.applied;
  if(applied && a.applied_type >= 0)
    atomicAdd(&s_bytype[a.applied_type], (unsigned long long)applied);
  // ---- 3b. carry-out: every actor's unhandled remainder, canonical, to the
  //      next step's carry buffer (none in the usual step) -----------------------------
  if(__syncthreads_or(any_rem))
  {
    ncout = block_scan_zone(s_aux, s_tmp);
    if(tid == 0) s_nbig = 0;
    __syncthreads();
    for(uint32_t i = tid; i < nact; i += kZoneThreads)
    {
      const uint32_t co = s_aux[i];
      const uint32_t rem = (i + 1 < kZone ? s_aux[i + 1] : ncout) - co;
      if(rem == 0) continue;
      if(!kSimple && rem > kBigGroup)       // (kSimple: no group over kBigGroup)
      {
        // a backlog (an overloaded receiver): copied by the whole workgroup
        const uint32_t k = atomicAdd(&s_nbig, 1u);
        if(k < kMaxBig) { s_big[k] = i; continue; }
      }
      const uint32_t n = s_cnt[i];
      if(use_idx)
        carry_out<SR>(AccIdx{s_idx + s_off[i], C, Ld, nc}, n - rem, n, z, co, nxt);
      else
        carry_out<SR>(acc_s(i), n - rem, n, z, co, nxt);
    }
    __syncthreads();
    const uint32_t nbig = min(s_nbig, kMaxBig);
    for(uint32_t k = 0; k < nbig; ++k)
    {
      const uint32_t i = s_big[k];
      const uint32_t co = s_aux[i];
      const uint32_t rem = (i + 1 < kZone ? s_aux[i + 1] : ncout) - co;
      const uint32_t n = s_cnt[i];
      ZRec* cout = c_eng.carry[nxt] + zo;
      if(c_eng.defer_big && !use_idx && co + rem <= cap)
      {
        // listed for k_carry_big, which copies it with every CU right after
        // this launch (its sources, the carry buffer and S, stay untouched
        // until then); a full list: copied here
        if(tid == 0)
        {
          // one atomic gives the slot and the copy's place in the flat list
          const unsigned long long v = atomicAdd(&c_eng.bigc_n[cur], (1ull << 32) | rem);
          const uint32_t slot = (uint32_t)(v >> 32);
          uint32_t ok = 0;
          if(slot < c_eng.bigc_cap)
          {
            BigCopy b;
            b.c = C + s_cst[i]; b.p = Sz + s_off[i]; b.dst = cout + co;
            b.ncc = s_ccnt[i]; b.from = n - rem; b.rem = rem; b.base = (uint32_t)v;
            b.perm = big_sorted(i) && !hot ? perm_s + s_off[i] : nullptr;
            c_eng.bigc[slot] = b;
            ok = 1;
          }
          s_nmix = ok;
        }
        __syncthreads();
        const bool listed = s_nmix != 0u;
        __syncthreads();
        if(listed) continue;
      }
      // Two half-batches of kUnroll / 2 records per thread, software-pipelined:
      // one half's stores are issued behind the other half's loads, so waiting
      // for a load never waits out the stores before it (vmcnt counts both,
      // in issue order) and loads and stores stay in flight together.
      constexpr int kH = kUnroll / 2;
      constexpr uint32_t kStride = kZoneThreads * kH;
      auto load_half = [&](ZRec (&r)[kH], uint32_t j0) __attribute__((always_inline)) {
#pragma unroll
        for(int uu = 0; uu < kH; ++uu)
        {
          const uint32_t j = j0 + uu * kZoneThreads + tid;
          if(j < rem)
            r[uu] = use_idx ? AccIdx{s_idx + s_off[i], C, Ld, nc}.rec(n - rem + j)
                            : acc_s(i).rec(n - rem + j);
        }
      };
      auto store_half = [&](const ZRec (&r)[kH], uint32_t j0) __attribute__((always_inline)) {
#pragma unroll
        for(int uu = 0; uu < kH; ++uu)
        {
          const uint32_t j = j0 + uu * kZoneThreads + tid;
          if(j >= rem) continue;
          uint4 u;
          u.x = r[uu].w0; u.y = r[uu].from; u.z = (uint32_t)r[uu].arg; u.w = (uint32_t)(r[uu].arg >> 32);
          const uint32_t pos = co + j;
          if(pos < cap)
            *reinterpret_cast<uint4*>(cout + pos) = u;
          else
            spill_rec(nxt, kSpillCarry, z, pos, u);
        }
      };
      ZRec ra[kH], rb[kH];
      load_half(ra, 0);
      for(uint32_t j0 = 0; j0 < rem; j0 += 2 * kStride)
      {
        load_half(rb, j0 + kStride);
        store_half(ra, j0);
        load_half(ra, j0 + 2 * kStride);
        store_half(rb, j0 + kStride);
      }
    }
  }
  }   // !plan
  if(tid == 0) c_eng.carry_n[nxt][z] = ncout;   // past cap: the tail is in the spill list
  // trigger bytes for the next step (only where some are set, or were)
  const uint32_t ntrig = s_ntrig;
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
  GPA_STAMP(4);
  if(tid < GPU_ACTOR_MAX_TYPES && s_bytype[tid])
    stat_add_z(ST_BY_TYPE + tid, z, s_bytype[tid]);
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

  // ---- 4. one chunk per destination bucket ----------------------------------------
  if(!(PM == 1 && kPlanSplit) && !plan && !dp)
  {
  uint32_t* s_tcnt = s_dyn + 2 * nb;    // records of the tile per bucket
  uint32_t* s_tst = s_dyn + 3 * nb;     // bucket start within the sorted tile
  for(uint32_t b = tid; b < nb; b += kZoneThreads)
  {
    const uint32_t h = s_hist[b];
    if(h)
    {
      ++n_atom;
      const uint32_t base = b < nz ? atomicAdd(&c_eng.land_n[nxt][b], h)
                                   : (uint32_t)atomicAdd(&c_eng.xcount[b - nz], (unsigned long long)h);
      s_base[b] = chunk_dst(b, base, h, nz);
    }
    s_tcnt[b] = 0;
  }
  __syncthreads();
  GPA_STAMP(5);
  // Scatter in tiles sorted by bucket (LDS counting sort), so that a wave's
  // store instruction writes runs of consecutive records of one chunk rather
  // than 64 records to 64 chunks (measured 1.75x for a whole-zone sort,
  // scripts/ubench_scatter.hip).
  const uint32_t nout = min(s_nout, cap);
  const ORec* Oz = c_eng.O + zo;
  // r = {to, w, arg lo, arg hi} -> place rel of bucket b's chunk
  auto emit = [&](const uint4& r, uint32_t b, uint32_t rel) __attribute__((always_inline)) {
    xover += emit_at(r, b, s_base[b], rel, L0, nz, nxt);
  };
  if(nout <= kZoneThreads)
  {
    // a sparse step (at most one record per thread): rank each record in its
    // bucket and store it straight away — the tile sort only groups stores
    // into runs, and a chunk's order is free (receivers order by key)
    if(tid < nout)
    {
      const uint4 r = ld16(reinterpret_cast<const uint4*>(Oz + tid));
      const uint32_t b = bucket_of(r.x);
      emit(r, b, atomicAdd(&s_tcnt[b], 1u));
    }
  }
  else
  for(uint32_t t0 = 0; t0 < nout; t0 += kTile)
  {
    const uint32_t m = min(kTile, nout - t0);
    uint4 ov[kTilePer];
    uint32_t bk[kTilePer], rk[kTilePer];
    // every lane loads (past the tile's end: its last record, unused), so the
    // kTilePer loads are all in flight at once and the tile stays in registers
#pragma unroll
    for(int u = 0; u < kTilePer; ++u)
    {
      const uint32_t i = min(u * kZoneThreads + tid, m - 1);
      ov[u] = ld16(reinterpret_cast<const uint4*>(Oz + t0 + i));
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
    // the tile loop shares only LDS across its barriers: the previous tile's
    // landing stores drain while this one is sorted
    lds_sync();
    (void)block_scan_n(s_tcnt, s_tst, nb, s_tmp);
#pragma unroll
    for(int u = 0; u < kTilePer; ++u)
    {
      const uint32_t i = u * kZoneThreads + tid;
      if(i < m) s_pool[s_tst[bk[u]] + rk[u]] = ov[u];
    }
    lds_sync();
    for(uint32_t p = tid; p < m; p += kZoneThreads)
    {
      const uint4 r = s_pool[p];
      const uint32_t b = bucket_of(r.x);
      emit(r, b, p - s_tst[b]);
    }
    lds_sync();
    for(uint32_t b = tid; b < nb; b += kZoneThreads)
    {
      s_base[b] += s_tcnt[b];
      s_tcnt[b] = 0;
    }
    lds_sync();
  }
  }   // !plan

  // ---- counters: block reduction, one atomic per workgroup per counter ---------------
  unsigned long long v[6] = { delivered + applied, sent, active, dropped, xover, n_atom };
#pragma unroll
  for(int k = 0; k < 6; ++k)
  {
    v[k] = wave_sum(v[k]);
    if(lane == 0) s_red[wv][k] = v[k];
  }
  __syncthreads();
  GPA_STAMP(6);
  if(tid < 6)
  {
    unsigned long long tot = 0;
    for(int w = 0; w < kZoneWaves; ++w) tot += s_red[w][tid];
    const int idx = tid == 0 ? ST_DELIVERED : tid == 1 ? ST_SENT : tid == 2 ? ST_ACTIVE
                  : tid == 3 ? ST_DROPPED : tid == 4 ? ST_XCHG_OVERFLOW : ST_ATOMICS;
    if(tot) stat_add_z(idx, z, tot);
  }
  if(took_mail && tid == 0)
  {
    if(nc + nl) pend_add_z(pend_slot, z, (unsigned long long)(nc + nl));
    c_eng.carry_n[cur][z] = 0;
    c_eng.land_n[cur][z] = 0;
    if constexpr(PM == 1) c_eng.zplan[z] = sidx + 1u;
  }
#ifdef GPA_STAMPS
  if(tid == 0) c_eng.dbg[z * kDbgSlots + 12] = __builtin_amdgcn_s_memrealtime();
#endif
  return true;
}


// The general path of PM 3 (below) as a call: its registers apart from the
// two-pass path's (inlined beside it, the plan path spills and runs slower:
// profiles/r05s_split_pass2_ab.txt, one launch 107 us against 72.5)
template <int HTS>
__device__ __noinline__ void zone_step_rest(uint32_t z, uint32_t cur, uint32_t pend_slot, uint32_t sidx)
{
  zone_step<HTS, 2>(z, cur, pend_slot, sidx);
}

// One workgroup per zone. PM 3 (split tables): the step as one launch —
// PM 1's path, and for a zone it leaves, PM 2's through the call above
// (nothing is written before PM 1 leaves a zone, so PM 2 starts it afresh;
// the zone is unmarked, so PM 2 does not return at its mark).
template <int HTS, int PM>
__global__ void __launch_bounds__(kZoneThreads, 4) k_step(uint32_t cur, uint32_t pend_slot,
  uint32_t sidx)
{
  if constexpr(PM != 3)
    zone_step<HTS, PM>(blockIdx.x, cur, pend_slot, sidx);
  else if(!zone_step<HTS, 1>(blockIdx.x, cur, pend_slot, sidx))
  {
    __syncthreads();                     // PM 1's LDS reads are done
    zone_step_rest<HTS>(blockIdx.x, cur, pend_slot, sidx);
  }
}

// The helper kernels below belong to engine.hip's code object only (the
// step_*.hip units define GPA_STEP_TU and instantiate k_step alone).
#ifndef GPA_STEP_TU
// Pending mail (carried + landed) for parity `cur`, summed into pend[slot].
__global__ void __launch_bounds__(kBlock) k_pending(uint32_t cur, uint32_t slot)
{
  __shared__ unsigned long long s_red[kWaves];
  const uint32_t z = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long p = 0;
  if(z < c_eng.n_zones)
  {
    const uint32_t cap = zone_capacity(z);
    p = min(c_eng.carry_n[cur][z], cap) + min(c_eng.land_n[cur][z], cap);
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

#endif // GPA_STEP_TU

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
      zt[u] = zone_of_local(rdiv(r[u].to));
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
      v.x = r[u].w | slot_in_zone(rdiv(r[u].to));
      v.y = r[u].from;
      v.z = (uint32_t)r[u].arg;
      v.w = (uint32_t)(r[u].arg >> 32);
      land_store(cur, zt[u], pos, v);
    }
}

#ifndef GPA_STEP_TU
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
// order, rcnt[p] of them from peer p — back to back (stride 0: received by
// the collectives), or peer p's at in + p * stride (the inbox peers stored
// into, EngDev::peer_write); the sender's rank of a record is the segment it
// lies in.
__global__ void __launch_bounds__(kLandThreads) k_xinject(const XRec* in, uint64_t n, uint32_t cur,
  const unsigned long long* rcnt, uint64_t stride)
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
      acc += rcnt[p];
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
      uint32_t src = 0;
      for(uint32_t p = 1; p < R; ++p)
        if(i >= s_roff[p]) src = p;
      const XRec x = stride ? xrec_get(in + src * stride + (i - s_roff[src])) : in[i];
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
#endif // GPA_STEP_TU

} // namespace gpa

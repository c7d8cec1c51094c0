// sparse_dev.h — the small-step path: k_sparse runs whole supersteps inside
// ONE workgroup while the world's pending mail fits in its LDS.
//
// A sparse workload (examples/ring: 100 tokens among 100,000 actors) leaves
// k_step's zone machinery almost idle: every launch pays a kernel boundary and
// a zone's six barrier-separated phases over 2048-wide LDS arrays for a handful
// of records. The reference schedules only actors whose mailbox went from
// empty to non-empty (ponyint_sched_add, scheduler.c:1320-1338; run loop
// 953-1090). k_sparse does the same with the messages themselves as the
// schedule: the step's records live in an LDS list; each step it
//   1. ranks them by (receiver, sender, sender seq) — the canonical delivery
//      order — with every thread counting the keys below its record (n <=
//      kSpCap; the reads are LDS broadcasts);
//   2. hands each receiver's run of records to one lane, which loads the
//      actor's state, runs the behaviours in order and stores the state;
//   3. collects their sends into the next list (the run queue of the next
//      step) and loops — no kernel boundary, no zone scans, no HBM round trip
//      for the records.
// It exits, leaving every pending record in the zone landing buffers exactly
// as a k_step would have, when the world goes quiet, after max_steps, or when a
// step needs the dense path: more than kSpCap records, carried mail, or a
// receiver with more arrivals than its batch.
#pragma once
#include "engine_dev.h"

namespace gpa {

constexpr int kSpThreads = 1024;
constexpr int kSpWaves = kSpThreads / 64;
#ifndef GPA_SP_CAP
#define GPA_SP_CAP 1024
#endif
constexpr uint32_t kSpCap = GPA_SP_CAP;   // records one sparse step holds in LDS

enum SpReason : uint32_t { SP_QUIESCENT = 0, SP_MAX_STEPS = 1, SP_DENSE = 2 };

struct SparseCtl {
  unsigned long long steps;     // supersteps this launch ran
  unsigned long long pending;   // records pending at exit (all in landing[par])
  uint32_t reason;              // SpReason
  uint32_t par;                 // landing parity the next step reads
};

// a message list in LDS, struct of arrays
struct SpList {
  uint64_t* K;     // receiver's local slot << 32 | sender id (host: kHostFrom | hseq >> 16)
  uint32_t* W;     // seq << 16 | beh << 12
  uint64_t* A;     // argument
};

// the next list's length, two counters used on alternate steps (one is reset
// while the other fills, with no extra barrier)
__shared__ uint32_t sp_cnt[2];

static_assert(kSpCap <= 1024, "packed rank counts hold 10-bit fields");
static_assert(kSpCap <= kSpThreads, "one record per thread in the distinct-receiver check");
constexpr uint32_t kSpHashBits = 13;       // receiver occupancy table (LDS, u32)
constexpr uint32_t kSpHash = 1u << kSpHashBits;

// per-type fields the sparse steps read, cached in LDS
constexpr uint32_t kSpNoRun = 1u;     // reducible, or spawns actors: dense path only
struct SpType {
  uint32_t lfirst, lcount, batch, flags;
};

__device__ __forceinline__ int sp_type(const SpType* ti, uint32_t n_types, uint32_t L)
{
  for(uint32_t t = 0; t < n_types; ++t)
    if(L - ti[t].lfirst < ti[t].lcount) return (int)t;
  return -1;
}

struct SparseCtx : ActorBase {
  SpList nx;              // the next step's list
  uint32_t q;             // its length is sp_cnt[q] (may count past kSpCap)
  uint32_t* s_over;       // set when it overflowed into landing[nxt]
  uint32_t nxt;           // landing parity of this step's sends
  __device__ __forceinline__ void put(uint32_t to, uint32_t w, uint64_t arg)
  {
    // one address for the whole workgroup: said so, the compiler issues one
    // atomic per wave and a lane prefix count
    const uint32_t i = atomicAdd(&sp_cnt[__builtin_amdgcn_readfirstlane(q)], 1u);
    if(i < kSpCap)
    {
      nx.K[i] = ((uint64_t)rdiv(to) << 32) | self; nx.W[i] = w; nx.A[i] = arg;
    }
    else
    {
      // the list is full: land the record now; the step ends the launch
      *s_over = 1u;
      send_direct(nxt, self, to, w, arg);
    }
  }
};

// Land records [0, n) of a list into landing[p] (one atomic each: n <= kSpCap).
__device__ void sp_land(const SpList& l, uint32_t n, uint32_t p)
{
  for(uint32_t i = threadIdx.x; i < n; i += kSpThreads)
  {
    const uint32_t L = (uint32_t)(l.K[i] >> 32);
    const uint32_t z = zone_of_local(L);
    const uint32_t pos = atomicAdd(&c_eng.land_n[p][z], 1u);
    uint4 v;
    v.x = l.W[i] | slot_in_zone(L);
    v.y = (uint32_t)l.K[i];
    v.z = (uint32_t)l.A[i];
    v.w = (uint32_t)(l.A[i] >> 32);
    land_store(p, z, pos, v);
  }
}

// One receiver's run [i, i + g) of the sorted list, handled in order.
template <int HT>
__device__ __forceinline__ void sp_drain(const TypeDev& T, SparseCtx& a, const SpList& s,
  uint32_t i, uint32_t g)
{
  constexpr int NW = HT_Words<HT>::W;
  uint64_t st[NW];
#pragma unroll
  for(int k = 0; k < NW; ++k) st[k] = T.state[(size_t)k * T.lcount + a.li];
  for(uint32_t k = 0; k < g; ++k)
    handle(HtTag<HT>{}, T, a, st, (s.W[i + k] >> 12) & 0xFu, s.A[i + k]);
#pragma unroll
  for(int k = 0; k < NW; ++k) T.state[(size_t)k * T.lcount + a.li] = st[k];
}

// kProg: the engine holds program types (GPU_ACTOR_HT_PROGRAM); their
// interpreter is compiled into a k_sparse of its own (in the one kernel it
// cost the compiled ring 13 %: 41.2 -> 35.7 M msgs/s, profiles/r05p4_sparse_program_ab.txt).
// kGups: the same for the GUPS streamer, whose chunk listing and GF(2) jump
// (k_gups_apply) cost the ring 10 % in the one kernel (40.8 -> 36.7 M msgs/s,
// profiles/r06_ring_ab.txt).
template <bool kProg, bool kGups>
__device__ __forceinline__ void sp_dispatch(const TypeDev& Tref, SparseCtx& a, const SpList& S,
  uint32_t i, uint32_t g, uint32_t L)
{
  const TypeDev T = Tref;
  a.li = L - T.lfirst;
  switch(T.ht)
  {
#define SPCASE(HT) case HT: sp_drain<HT>(T, a, S, i, g); break;
    SPCASE(GPU_ACTOR_HT_RING)
    SPCASE(GPU_ACTOR_HT_PINGER)
    SPCASE(GPU_ACTOR_HT_PINGER_DET)
    SPCASE(GPU_ACTOR_HT_FANIN_SENDER)
    case GPU_ACTOR_HT_GUPS_STREAMER:
      if constexpr(kGups) sp_drain<GPU_ACTOR_HT_GUPS_STREAMER>(T, a, S, i, g);
      break;
    SPCASE(GPU_ACTOR_HT_STORM)
    SPCASE(GPU_ACTOR_HT_FIFO_SRC)
    SPCASE(GPU_ACTOR_HT_FIFO_SINK)
    case GPU_ACTOR_HT_PROGRAM:
      if constexpr(kProg) sp_drain<GPU_ACTOR_HT_PROGRAM>(T, a, S, i, g);
      break;
#undef SPCASE
    default: break;
  }
}

__device__ __forceinline__ uint32_t sp_block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t& total)
{
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for(int off = 1; off < 64; off <<= 1)
  {
    const uint32_t u = (uint32_t)__shfl_up((int)incl, off);
    if(lane >= (uint32_t)off) incl += u;
  }
  if(lane == 63) s_tmp[wv] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for(int w = 0; w < kSpWaves; ++w)
  {
    const uint32_t x = s_tmp[w];
    if(w < (int)wv) base += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return base + incl - v;
}

// Runs up to max_steps supersteps (0: no limit) starting from the records in
// landing[cur]; R == 1 and no spawning types (the host checks).
template <bool kProg, bool kGups>
__global__ void __launch_bounds__(kSpThreads) k_sparse(uint32_t cur, unsigned long long max_steps,
  SparseCtl* ctl, uint32_t sidx)
{
  __shared__ uint64_t bK[3][kSpCap], bA[3][kSpCap];
  __shared__ uint32_t bW[3][kSpCap];
  __shared__ uint32_t s_zpre[kMaxZones + 1];
  __shared__ uint32_t s_tmp[kSpWaves];
  __shared__ uint32_t s_over;
  __shared__ uint32_t s_acc[kSpThreads];        // packed rank counts (kSpCap <= kSpThreads)
  __shared__ SpType s_tinfo[GPU_ACTOR_MAX_TYPES];
  __shared__ uint32_t s_hcnt[kSpHash];          // records per receiver hash this step
  __shared__ unsigned long long s_agg[kSpWaves];
  __shared__ unsigned long long s_bytype[GPU_ACTOR_MAX_TYPES];
  __shared__ unsigned long long s_red[kSpWaves][4];

  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nz = c_eng.n_zones;
  const uint32_t n_types = c_eng.n_types;
  if(tid < GPU_ACTOR_MAX_TYPES)
  {
    s_bytype[tid] = 0;
    const TypeDev& T = c_types[tid];
    s_tinfo[tid].lfirst = T.lfirst;
    s_tinfo[tid].lcount = T.lcount;
    s_tinfo[tid].batch = T.batch;
    // reducible types never run; spawning and yielding ones need the zone path
    s_tinfo[tid].flags = (T.reducible || T.ht == GPU_ACTOR_HT_SPREADER ||
                          (T.ht == GPU_ACTOR_HT_PROGRAM && (!kProg || (T.prog_pad & 1u))) ||
                          (T.ht == GPU_ACTOR_HT_GUPS_STREAMER && !kGups) ||
                          (T.ht == GPU_ACTOR_HT_FIFO_SINK && T.params[1] != 0)) ? kSpNoRun : 0u;
  }
  if(tid == 0) { sp_cnt[0] = 0; sp_cnt[1] = 0; s_over = 0; }
  s_acc[tid] = 0;
  for(uint32_t h = tid; h < kSpHash; h += kSpThreads) s_hcnt[h] = 0;

  // ---- gather landing[cur] into list 0 ---------------------------------------------
  // per-thread run of zones, exclusive scan of their record counts
  const uint32_t per = (nz + kSpThreads - 1) / kSpThreads;
  const uint32_t z0 = min(tid * per, nz), z1 = min(z0 + per, nz);
  uint32_t mine = 0;
  int carried = 0;
  for(uint32_t z = z0; z < z1; ++z)
  {
    const uint32_t c = min(c_eng.land_n[cur][z], zone_capacity(z));
    s_zpre[z] = c;
    mine += c;
    carried |= c_eng.carry_n[cur][z] != 0u;
  }
  uint32_t total = 0;
  uint32_t run = sp_block_excl_scan(mine, s_tmp, total);
  for(uint32_t z = z0; z < z1; ++z) { const uint32_t c = s_zpre[z]; s_zpre[z] = run; run += c; }
  if(tid == 0) s_zpre[nz] = total;
  // spilled records wait for the host; an actor that triggers muting
  // (overloaded or muted) needs the zone path's backpressure
  const bool pending_fixup = c_eng.spill_n[cur] != 0u || *c_eng.halt != 0u ||
                             c_eng.trig_n[sidx % 3u] != 0u;
  if(__syncthreads_or(carried) || total > kSpCap || pending_fixup)
  {
    // the dense path owns this step: nothing was touched
    if(tid == 0)
    {
      ctl->steps = 0; ctl->pending = total; ctl->reason = SP_DENSE; ctl->par = cur;
    }
    return;
  }
  for(uint32_t i = tid; i < total; i += kSpThreads)
  {
    uint32_t lo = 0, hi = nz;          // zone z with s_zpre[z] <= i < s_zpre[z + 1]
    while(hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if(s_zpre[m] <= i) lo = m; else hi = m; }
    const uint4 v = *reinterpret_cast<const uint4*>(c_eng.land[cur] + c_eng.zoff[lo] + (i - s_zpre[lo]));
    const uint32_t zm = (1u << c_eng.zbits) - 1u;
    bK[0][i] = ((uint64_t)((lo << c_eng.zbits) + (v.x & zm)) << 32) | v.y;
    bW[0][i] = v.x & ~zm;
    bA[0][i] = ((uint64_t)v.w << 32) | v.z;
  }
  for(uint32_t z = z0; z < z1; ++z) c_eng.land_n[cur][z] = 0;
  // no actor triggers muting now; bytes a zone left in the other parity two
  // steps ago are cleared, so both parities read as all-quiet when the zone
  // path resumes
  for(uint32_t z = z0; z < z1; ++z)
    if(c_eng.ztrig[cur ^ 1u][z])
    {
      const uint32_t zs = 1u << c_eng.zbits;
      const uint32_t L0 = z * zs, nact = min(zs, c_eng.n_local - L0);
      for(uint32_t i = 0; i < nact; ++i) c_eng.trig_own[cur ^ 1u][L0 + i] = 0;
      c_eng.ztrig[cur ^ 1u][z] = 0;
    }
  __syncthreads();

  // ---- supersteps --------------------------------------------------------------------
  uint32_t la = 0, lb = 1;                 // current / next list; 2 = sorted
  uint32_t n = total;
  unsigned long long steps = 0;
  uint32_t reason = SP_QUIESCENT;
  unsigned long long delivered = 0, sent = 0, active = 0, applied = 0;
  int bt_t = 0;                            // per-type delivered counts, flushed when the type changes
  unsigned long long bt_n = 0;
  const SpList S{bK[2], bW[2], bA[2]};
  uint32_t q = 0;                          // which append counter this step's sends use
#ifdef GPA_STAMPS
  // diagnostic build: shader-clock cycles per phase, summed over the steps
  unsigned long long ph[4] = {0, 0, 0, 0};
  unsigned long long tk = __builtin_amdgcn_s_memtime();
#define SP_STAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph[k] += t_ - tk; tk = t_; } while(0)
#else
#define SP_STAMP(k) do {} while(0)
#endif
  for(;;)
  {
    if(n == 0) { reason = SP_QUIESCENT; break; }
    if(max_steps && steps >= max_steps) { reason = SP_MAX_STEPS; break; }
    const SpList Acur{bK[la], bW[la], bA[la]};
    const SpList Bnxt{bK[lb], bW[lb], bA[lb]};
    // 0. every receiver distinct (a ring's tokens, one message per actor)? A
    //    hashed occupancy count per receiver: no bucket above one means no
    //    receiver has two records, so every record is a run of its own and the
    //    order among runs is free — the rank sort is skipped. A collision
    //    (or a real repeat) takes the sort.
    // whether the record alone (a run of one) already needs the zone path
    // (the second record of a bucket sees a nonzero count come back from its
    // add, so one OR over the workgroup tells whether any bucket repeats)
    uint32_t hb = 0;
    int dense1 = 0;
    bool coll = false;
    if(tid < n)
    {
      const uint32_t L = (uint32_t)(Acur.K[tid] >> 32);
      hb = (L * 0x9E3779B1u) >> (32 - kSpHashBits);
      coll = atomicAdd(&s_hcnt[hb], 1u) != 0u;
      const int t = sp_type(s_tinfo, n_types, L);
      dense1 = (t < 0 || (s_tinfo[t].flags & kSpNoRun) || 1u >= s_tinfo[t].batch) ? 1 : 0;
    }
    // one barrier in the usual case (no repeat receiver, nothing for the zone
    // path); a second tells a repeat from a dense record
    const bool any_cd = __syncthreads_or(coll || dense1);
    const bool distinct = !(any_cd && __syncthreads_or(coll));
    if(tid < n) s_hcnt[hb] = 0;              // every add to it is behind the barrier above
    int dense = 0;
    uint32_t h_r = 0, h_g = 0;               // this thread's run: [h_r, h_r + h_g)
    const SpList* Srun = &S;
    if(distinct)
    {
      if(tid == 0) sp_cnt[q ^ 1u] = 0;       // the next step's counter, read last step
      if(tid < n) { h_r = tid; h_g = 1; }
      dense = any_cd ? 1 : 0;                // uniform: with no repeat, any_cd means a dense record
      Srun = &Acur;
    }
    else
    {
    // 1. canonical order. Record i's key (receiver, sender, seq) is compared
    //    with every other key by P threads, each over one slice of the list
    //    (consecutive lanes take consecutive records of the same slice, so
    //    their reads of key j are LDS broadcasts); each adds one packed
    //    partial count to s_acc[i]: keys below (rank), keys of the same
    //    receiver, and of those the ones below.
    {
      const uint32_t P = min(16u, max(1u, kSpThreads / n));
      const uint32_t span = (n + P - 1) / P;
      for(uint32_t task = tid; task < n * P; task += kSpThreads)
      {
        const uint32_t p = task / n, i = task - p * n;
        const uint64_t ki = Acur.K[i];
        const uint32_t li = (uint32_t)(ki >> 32);
        const uint32_t wi = Acur.W[i] >> 16;
        const uint32_t j0 = p * span, j1 = min(n, j0 + span);
        uint32_t lt = 0, same = 0, ltsame = 0;
        uint32_t j = j0;
        for(; j + 4 <= j1; j += 4)
        {
          uint64_t kj[4];
          uint32_t wj[4];
#pragma unroll
          for(int u = 0; u < 4; ++u) { kj[u] = Acur.K[j + u]; wj[u] = Acur.W[j + u] >> 16; }
#pragma unroll
          for(int u = 0; u < 4; ++u)
          {
            const uint32_t b = (uint32_t)(kj[u] < ki) | ((uint32_t)(kj[u] == ki) & (uint32_t)(wj[u] < wi));
            const uint32_t sm = (uint32_t)((uint32_t)(kj[u] >> 32) == li);
            lt += b; same += sm; ltsame += b & sm;
          }
        }
        for(; j < j1; ++j)
        {
          const uint64_t kj = Acur.K[j];
          const uint32_t wj = Acur.W[j] >> 16;
          const uint32_t b = (uint32_t)(kj < ki) | ((uint32_t)(kj == ki) & (uint32_t)(wj < wi));
          const uint32_t sm = (uint32_t)((uint32_t)(kj >> 32) == li);
          lt += b; same += sm; ltsame += b & sm;
        }
        atomicAdd(&s_acc[i], lt | (ltsame << 10) | (same << 20));
      }
    }
    __syncthreads();
    SP_STAMP(0);
    // 2. place each record at its rank; the first record of each receiver's
    //    run (no lower key of the same receiver) owns the run. A run longer
    //    than its type's batch needs carry: the step goes to the dense path.
    if(tid == 0) sp_cnt[q ^ 1u] = 0;         // the next step's counter, read last step
    if(tid < n)
    {
      const uint32_t c = s_acc[tid];
      const uint32_t r = c & 0x3FFu, ltsame = (c >> 10) & 0x3FFu, same = c >> 20;
      S.K[r] = Acur.K[tid]; S.W[r] = Acur.W[tid]; S.A[r] = Acur.A[tid];
      if(ltsame == 0)
      {
        h_r = r; h_g = same;
        const int t = sp_type(s_tinfo, n_types, (uint32_t)(Acur.K[tid] >> 32));
        // a full batch would leave the actor overloaded: the zone path owns that
        if(t < 0 || (s_tinfo[t].flags & kSpNoRun) || same >= s_tinfo[t].batch) dense = 1;
      }
    }
    s_acc[tid] = 0;                          // ready for the next step's counts
    }
    const int any_dense = distinct ? dense : __syncthreads_or(dense);   // uniform either way
    SP_STAMP(1);
    if(any_dense)
    {
      reason = SP_DENSE;                     // list la still holds the step, unsorted
      break;
    }
    // 3. behaviours: the owner of each run loads the actor's state, runs the
    //    run's behaviours in order and stores the state; sends go to list lb
    if(h_g)
    {
      const SpList& Sr = *Srun;
      const uint32_t L = (uint32_t)(Sr.K[h_r] >> 32);
      const int t = sp_type(s_tinfo, n_types, L);
      SparseCtx a;
      a.reset_common();
      a.self = L * c_eng.nranks + c_eng.rank;
      a.src_local = slot_in_zone(L);
      a.type = t;
      a.agg = &s_agg[wv];
      a.nx = Bnxt;
      a.q = q;
      a.s_over = &s_over;
      a.nxt = cur ^ 1u;
      // the usual case, one type for every run of the wave: its fields come
      // through scalar loads instead of a per-lane copy from constant memory
      const int tu = __builtin_amdgcn_readfirstlane(t);
      if(__ballot(t != tu) == 0ull) sp_dispatch<kProg, kGups>(c_types[tu], a, Sr, h_r, h_g, L);
      else sp_dispatch<kProg, kGups>(c_types[t], a, Sr, h_r, h_g, L);
      delivered += h_g;
      active += 1;
      sent += a.sent;
      applied += a.applied;
      if(t != bt_t) { if(bt_n) atomicAdd(&s_bytype[bt_t], bt_n); bt_t = t; bt_n = 0; }
      bt_n += h_g;
      if(a.applied && a.applied_type >= 0)
        atomicAdd(&s_bytype[a.applied_type], (unsigned long long)a.applied);
    }
    __syncthreads();
    SP_STAMP(2);
    const uint32_t nn = sp_cnt[q];
    ++steps;
    cur ^= 1u;
    q ^= 1u;
    const uint32_t t2 = la; la = lb; lb = t2;
    n = min(nn, kSpCap);
    SP_STAMP(3);
    if(s_over)
    {
      // the records past the list already sit in landing[cur]
      reason = SP_DENSE;
      break;
    }
  }
  // ---- hand the pending list back to the zone landing buffers ---------------------------
  const uint32_t over = s_over;
  {
    const SpList Acur{bK[la], bW[la], bA[la]};
    sp_land(Acur, n, cur);
  }
  if(bt_n) atomicAdd(&s_bytype[bt_t], bt_n);
  __syncthreads();
  unsigned long long v[4] = { delivered + applied, sent, active, 0 };
#pragma unroll
  for(int k = 0; k < 3; ++k)
  {
#pragma unroll
    for(int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if(lane == 0) s_red[wv][k] = v[k];
  }
  __syncthreads();
  if(tid < 3)
  {
    unsigned long long tot = 0;
    for(int w = 0; w < kSpWaves; ++w) tot += s_red[w][tid];
    const int idx = tid == 0 ? ST_DELIVERED : tid == 1 ? ST_SENT : ST_ACTIVE;
    if(tot) atomicAdd(&c_eng.stats[idx], tot);
  }
  if(tid < GPU_ACTOR_MAX_TYPES && s_bytype[tid])
    atomicAdd(&c_eng.stats[ST_BY_TYPE + tid], s_bytype[tid]);
#ifdef GPA_STAMPS
  if(tid == 0)
    for(int k = 0; k < 4; ++k) c_eng.dbg[k] = ph[k];
#endif
#undef SP_STAMP
  if(tid < 3) c_eng.trig_n[tid] = 0;       // nothing triggers after sparse steps
  if(tid == 0)
  {
    ctl->steps = steps;
    ctl->pending = over ? 0xFFFFFFFFFFFFFFFFull : n;   // unknown after an overflow: ask k_pending
    ctl->reason = reason;
    ctl->par = cur;
  }
}

} // namespace gpa

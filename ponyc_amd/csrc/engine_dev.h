// engine_dev.h — device-side data layout and handler tables of the gpu_actor
// engine. See DESIGN.md for the layout rationale.
//
// HBM layout (per rank; actor id a lives on rank a % R at local slot a / R):
//   per local slot (SoA, u32): head, sorted, end, lim, tail
//     head   next slot to handle             (written by the owner's drain)
//     sorted slots < sorted are in canonical order
//     end    tail snapshot at the step start (messages in [head,end) are visible)
//     lim    head at the step start + cap    (senders may fill slots < lim)
//     tail   next free slot                  (senders: atomicAdd)
//   per type: state[w][lcount] (u64, field-major) and a mailbox ring of
//   cap x 16-B records per actor: {u32 seq<<8|beh, u32 from, u64 arg}. The first
//   8 bytes read as one little-endian u64 are the canonical delivery key
//   (from << 32 | seq << 8 | beh).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/gpu_actor.h"
#include "rng_dev.h"

namespace gpa {

constexpr int      kBlock = 256;
constexpr int      kWaves = kBlock / 64;
constexpr uint32_t kHostFrom = 0xFF000000u;   // host senders: ids above every actor
constexpr uint32_t kSeqLimit = 1u << 24;      // per-sender sequence numbers per step

enum Stat : int {
  ST_DELIVERED = 0, ST_SENT = 1, ST_DROPPED = 2, ST_REMOTE_OUT = 3, ST_REMOTE_IN = 4,
  ST_SEQ_OVERFLOW = 5, ST_XCHG_OVERFLOW = 6, ST_ACTIVE = 7,
  ST_BY_TYPE = 16, ST_COUNT = 32
};

struct Rec {            // mailbox record, 16 B
  uint32_t sb;          // seq << 8 | behaviour
  uint32_t from;        // sender id (kHostFrom | hi bits for host sends)
  uint64_t arg;
};

struct XRec {           // cross-rank record, 24 B
  uint32_t to;
  uint32_t sb;
  uint32_t from;
  uint32_t beh_only;    // 1: reducible apply (seq unused)
  uint64_t arg;
};

struct TypeDev {
  uint32_t first, count;     // global id range
  uint32_t lfirst, lcount;   // local slot range on this rank
  uint32_t ht, words, batch, cap;
  uint32_t reducible, pad;
  uint64_t* state;           // [words][lcount]
  Rec*      mb;              // [lcount][cap]
  uint64_t  params[GPU_ACTOR_MAX_PARAMS];
};

struct EngDev {
  uint32_t n_types, rank, nranks, n_local;
  uint32_t *head, *sorted, *end, *lim, *tail;
  unsigned long long* stats;
  unsigned long long* pend;       // per-step pending counters
  XRec*  xout;                    // [nranks][xcap]
  unsigned long long* xcount;     // [nranks]
  uint32_t xcap, pad;
};

__constant__ TypeDev c_types[GPU_ACTOR_MAX_TYPES];
__constant__ EngDev  c_eng;

__device__ __forceinline__ int type_of_local(uint32_t L)
{
  for(uint32_t t = 0; t < c_eng.n_types; ++t)
    if(L - c_types[t].lfirst < c_types[t].lcount) return (int)t;
  return -1;
}

__device__ __forceinline__ int type_of_global(uint32_t id)
{
  for(uint32_t t = 0; t < c_eng.n_types; ++t)
    if(id - c_types[t].first < c_types[t].count) return (int)t;
  return -1;
}

__device__ __forceinline__ uint64_t rec_key(const Rec* r)
{
  return *reinterpret_cast<const uint64_t*>(r);
}

// Per-lane bookkeeping while one actor drains.
struct ActorCtx {
  uint32_t self;       // global id
  uint32_t li;         // index within its type (local)
  uint32_t seq;        // emissions this step
  uint32_t sent;
  uint32_t applied;    // reducible applies issued (delivered to applied_type)
  int      applied_type;
};

// ---- delivery ------------------------------------------------------------

__device__ __forceinline__ void remote_append(uint32_t to, uint32_t sb, uint32_t from,
  uint64_t arg, uint32_t beh_only)
{
  const uint32_t peer = to % c_eng.nranks;
  const unsigned long long k = atomicAdd(&c_eng.xcount[peer], 1ull);
  if(k >= c_eng.xcap)
  {
    atomicAdd(&c_eng.stats[ST_XCHG_OVERFLOW], 1ull);
    return;
  }
  XRec* x = c_eng.xout + (size_t)peer * c_eng.xcap + k;
  x->to = to; x->sb = sb; x->from = from; x->beh_only = beh_only; x->arg = arg;
}

// Append one record to a serial actor's ring (local target).
__device__ __forceinline__ void ring_push(uint32_t to, uint32_t sb, uint32_t from, uint64_t arg)
{
  const uint32_t L = to / c_eng.nranks;
  const int t = type_of_global(to);
  if(t < 0)
  {
    atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);
    return;
  }
  const TypeDev& T = c_types[t];
  const uint32_t slot = atomicAdd(&c_eng.tail[L], 1u);
  if((int32_t)(slot - c_eng.lim[L]) >= 0)
  {
    atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);
    return;
  }
  Rec* ring = T.mb + (size_t)(L - T.lfirst) * T.cap;
  Rec r;
  r.sb = sb; r.from = from; r.arg = arg;
  *reinterpret_cast<uint4*>(ring + (slot & (T.cap - 1))) = *reinterpret_cast<const uint4*>(&r);
}

// Reducible behaviours: applied as device atomics at the owner.
__device__ __forceinline__ void reducible_apply_local(uint32_t to, uint32_t beh, uint64_t arg)
{
  const int t = type_of_global(to);
  if(t < 0) return;
  const TypeDev& T = c_types[t];
  const uint32_t li = to / c_eng.nranks - T.lfirst;
  switch(T.ht)
  {
    case GPU_ACTOR_HT_FANIN_ANALYZER:
      atomicAdd(reinterpret_cast<unsigned long long*>(&T.state[li]), 1ull);
      atomicXor(reinterpret_cast<unsigned long long*>(&T.state[(size_t)T.lcount + li]),
        (unsigned long long)arg);
      break;
    case GPU_ACTOR_HT_GUPS_UPDATER: {
      const uint64_t k = arg & (T.params[0] - 1);
      atomicXor(reinterpret_cast<unsigned long long*>(&T.state[k * T.lcount + li]),
        (unsigned long long)arg);
      break;
    }
    default:
      break;
  }
  (void)beh;
}

__device__ __forceinline__ void send_serial(ActorCtx& a, uint32_t to, uint32_t beh, uint64_t arg)
{
  const uint32_t sb = (a.seq << 8) | beh;
  a.seq++;
  a.sent++;
  if(c_eng.nranks > 1 && to % c_eng.nranks != c_eng.rank)
  {
    remote_append(to, sb, a.self, arg, 0);
    return;
  }
  ring_push(to, sb, a.self, arg);
}

// fan-in Analyzer apply, aggregated per wavefront: lanes hitting the same
// analyzer fold their count and XOR through LDS and one lane issues the two
// global atomics (Guideline 12: one atomic per (wave, destination)).
__device__ __forceinline__ void send_analyzer(ActorCtx& a, uint32_t to, uint64_t arg,
  unsigned long long* s_agg)
{
  a.sent++;
  const bool remote = c_eng.nranks > 1 && to % c_eng.nranks != c_eng.rank;
  if(remote)
    remote_append(to, GPU_ACTOR_FANIN_MSG, a.self, arg, 1);   // counted by the owner
  else
  {
    a.applied++;
    if(a.applied_type < 0) a.applied_type = type_of_global(to);
  }
  const int lane = __lane_id();
  const int wv = threadIdx.x >> 6;
  unsigned long long active = __ballot(!remote);
  while(active != 0ull)
  {
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t tl = __builtin_amdgcn_readlane(to, leader);
    const bool mine = !remote && to == tl;
    const unsigned long long peers = __ballot(mine);
    if(lane == leader) s_agg[wv] = 0ull;
    __builtin_amdgcn_wave_barrier();
    if(mine) atomicXor(&s_agg[wv], (unsigned long long)arg);
    __builtin_amdgcn_wave_barrier();
    if(lane == leader)
    {
      const int t = type_of_global(tl);
      if(t >= 0)
      {
        const TypeDev& T = c_types[t];
        const uint32_t li = tl / c_eng.nranks - T.lfirst;
        atomicAdd(reinterpret_cast<unsigned long long*>(&T.state[li]),
          (unsigned long long)__popcll(peers));
        atomicXor(reinterpret_cast<unsigned long long*>(&T.state[(size_t)T.lcount + li]),
          s_agg[wv]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    active &= ~peers;
  }
}

__device__ __forceinline__ void send_updater(ActorCtx& a, uint32_t to, uint64_t d)
{
  a.sent++;
  if(c_eng.nranks > 1 && to % c_eng.nranks != c_eng.rank)
  {
    remote_append(to, GPU_ACTOR_GUPS_UPDATE, a.self, d, 1);   // counted by the owner
    return;
  }
  a.applied++;
  if(a.applied_type < 0) a.applied_type = type_of_global(to);
  reducible_apply_local(to, GPU_ACTOR_GUPS_UPDATE, d);
}

// ---- handler tables --------------------------------------------------------
// Each handle_* restates one reference behaviour set; s[] is the actor's state
// held in registers for the whole drain.

template <int HT> struct HT_Words;
template <> struct HT_Words<GPU_ACTOR_HT_RING>          { static constexpr int W = 4; };
template <> struct HT_Words<GPU_ACTOR_HT_PINGER>        { static constexpr int W = 3; };
template <> struct HT_Words<GPU_ACTOR_HT_PINGER_DET>    { static constexpr int W = 2; };
template <> struct HT_Words<GPU_ACTOR_HT_FANIN_SENDER>  { static constexpr int W = 4; };
template <> struct HT_Words<GPU_ACTOR_HT_GUPS_STREAMER> { static constexpr int W = 2; };
template <> struct HT_Words<GPU_ACTOR_HT_STORM>         { static constexpr int W = 2; };
template <> struct HT_Words<GPU_ACTOR_HT_FIFO_SRC>      { static constexpr int W = 3; };
template <> struct HT_Words<GPU_ACTOR_HT_FIFO_SINK>     { static constexpr int W = 11; };

template <int HT>
__device__ __forceinline__ void handle(const TypeDev& T, ActorCtx& a, uint64_t (&s)[HT_Words<HT>::W],
  uint32_t beh, uint64_t arg, unsigned long long* s_agg);

// examples/ring/main.pony:13-24
template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_RING>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[4], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  if(beh == GPU_ACTOR_RING_SET)
  {
    s[0] = arg;
    return;
  }
  s[2] += 1;
  if(arg > 0)
  {
    if(s[0] != GPU_ACTOR_NONE)
      send_serial(a, (uint32_t)s[0], GPU_ACTOR_RING_PASS, arg - 1);
  } else {
    s[3] += 1;
  }
}

// examples/message-ubench/main.pony:265-286 (+ forward budget)
template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_PINGER>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[3], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  s[2] += 1;
  if(s[2] <= T.params[2])
  {
    const uint64_t k = rand_int(s[0], s[1], T.params[0]);
    send_serial(a, (uint32_t)(T.params[1] + k), GPU_ACTOR_PINGER_PING, 42);
  }
}

__device__ __forceinline__ void det_ping(const TypeDev& T, ActorCtx& a, uint64_t& count,
  uint64_t& acc, uint32_t beh, uint64_t arg)
{
  count += 1;
  acc ^= arg;
  const uint64_t hop = arg & 0xFFFFFFFFull;
  if(hop < T.params[2])
  {
    const uint64_t k = mulhi64(splitmix_mix(T.params[3] ^ arg), T.params[0]);
    send_serial(a, (uint32_t)(T.params[1] + k), beh, (arg & 0xFFFFFFFF00000000ull) | (hop + 1));
  }
}

template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_PINGER_DET>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  det_ping(T, a, s[0], s[1], beh, arg);
}

template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_STORM>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  if(beh == GPU_ACTOR_STORM_TOKEN)
  {
    s[0] += 1;
    s[1] ^= arg;
    if(arg < T.params[2])
    {
      const uint32_t nxt = (a.self - T.first + 1 == T.count) ? T.first : a.self + 1;
      send_serial(a, nxt, GPU_ACTOR_STORM_TOKEN, arg + 1);
    }
    return;
  }
  det_ping(T, a, s[0], s[1], beh, arg);
}

// examples/fan-in/main.pony:241-250
template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_FANIN_SENDER>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[4], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  const uint64_t k = rand_int_unbiased(s[0], s[1], T.params[0]);
  const uint64_t i = a.self - T.first;
  send_analyzer(a, (uint32_t)(T.params[1] + k), (i << 32) | s[3], s_agg);
  s[3] += 1;
  if(s[2] > 0) s[2] -= 1;
  if(s[2] > 0)
    send_serial(a, a.self, GPU_ACTOR_FANIN_SEND_MSGS, 0);
}

// examples/gups_basic/main.pony:110-143, one message per datum
template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_GUPS_STREAMER>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  const uint64_t chunk = T.params[0], shift = T.params[1], mask = T.params[2];
  const uint32_t ubase = (uint32_t)T.params[3];
  uint64_t last = s[0];
  for(uint64_t c = 0; c < chunk; ++c)
  {
    const uint64_t d = polyrand_next(last);
    send_updater(a, ubase + (uint32_t)((d >> shift) & mask), d);
  }
  s[0] = last;
  if(arg > 0)
    send_serial(a, a.self, GPU_ACTOR_GUPS_APPLY, arg - 1);
  else
    s[1] = 1;
}

template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_FIFO_SRC>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[3], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  const uint64_t i = a.self - T.first;
  for(uint64_t j = 0; j < arg; ++j)
  {
    s[1] += 1;
    send_serial(a, (uint32_t)s[0], GPU_ACTOR_FIFO_PUSH, (i << 32) | s[1]);
  }
  if(s[2] > 0) s[2] -= 1;
  if(s[2] > 0)
    send_serial(a, a.self, GPU_ACTOR_FIFO_BURST, arg);
}

template <>
__device__ __forceinline__ void handle<GPU_ACTOR_HT_FIFO_SINK>(const TypeDev& T, ActorCtx& a,
  uint64_t (&s)[11], uint32_t beh, uint64_t arg, unsigned long long* s_agg)
{
  const uint64_t ns = T.params[0] ? T.params[0] : 1;
  const uint32_t slot = (uint32_t)(((arg >> 32) / ns) % 8);
  const uint64_t seq = arg & 0xFFFFFFFFull;
  s[1] += 1;
  s[0] = (s[0] ^ arg) * 0x100000001b3ull;
  // static-index select keeps s[] in registers
  uint64_t last = 0;
#pragma unroll
  for(int k = 0; k < 8; ++k) last = (slot == (uint32_t)k) ? s[3 + k] : last;
  if(seq != last + 1) s[2] += 1;
#pragma unroll
  for(int k = 0; k < 8; ++k) s[3 + k] = (slot == (uint32_t)k) ? seq : s[3 + k];
}

} // namespace gpa

// engine_dev.h — device-side data layout, delivery primitives and handler
// tables of the gpu_actor engine. See DESIGN.md for the rationale.
//
// HBM layout (per rank; actor id a lives on rank a % R at local slot L = a / R):
//   Local slots are cut into zones of kZone actors (2048, or 4096 for large
//   engines: step_entry.h). Zone z owns
//     land[p][z]   : landing buffer of step-p arrivals (unordered 16-B ZRecs),
//                    filled by producers in chunks, one atomicAdd on
//                    land_n[p][z] per (producer zone, destination zone);
//     carry[p][z]  : mail handed over from the previous step because of the
//                    batch limit, grouped by actor, in canonical order;
//     S[z], O[z]   : per-zone scratch (sorted inbox, outbox) that the zone's
//                    workgroup writes and reads back within one launch.
//   Per type: state[w][lcount] (u64, field-major).
// A ZRec is {u32 seq<<16 | beh<<12 | to_local, u32 from, u64 arg}; its
// canonical delivery key is (from << 16 | seq).
#pragma once
#ifndef __HIPCC_RTC__       // (also compiled at run time: engine.hip jit)
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>
#include "../../include/gpu_actor.h"
#include "rng_dev.h"

namespace gpa {

constexpr int      kBlock = 256;                 // helper kernels
constexpr int      kWaves = kBlock / 64;
// Zone geometry (A/B builds override it: scripts/build_variants.sh)
#ifndef GPA_ZONE_BITS
#define GPA_ZONE_BITS 11
#endif
#ifndef GPA_ZONE_THREADS
#define GPA_ZONE_THREADS 512
#endif
constexpr int      kZoneBits = GPA_ZONE_BITS;    // this code object's k_step geometry; to_local holds up to 12 bits
static_assert(kZoneBits <= 12, "to_local is 12 bits of a ZRec's w0");
constexpr uint32_t kZone = 1u << kZoneBits;      // actors per zone
constexpr uint32_t kZoneMask = kZone - 1;
constexpr int      kZoneThreads = GPA_ZONE_THREADS;  // one workgroup per zone
constexpr int      kZoneWaves = kZoneThreads / 64;
constexpr uint32_t kMaxZones = 4096;             // histogram bound (zones per rank)
constexpr uint32_t kMaxRanks = 64;
constexpr uint32_t kHostFrom = 0xFF000000u;      // host senders rank above every actor
constexpr uint32_t kSeqMax = 0xFFFEu;            // per-sender sends per step
constexpr uint32_t kSeqApply = 0xFFFFu;          // outbox marker: reducible apply
constexpr uint32_t kFanLds = 256;                // analyzers a zone accumulates in LDS
constexpr uint32_t kDbgSlots = 24;               // diagnostic build: clock stamps per zone

enum Stat : int {
  ST_DELIVERED = 0, ST_SENT = 1, ST_DROPPED = 2, ST_REMOTE_OUT = 3, ST_REMOTE_IN = 4,
  ST_SEQ_OVERFLOW = 5, ST_XCHG_OVERFLOW = 6, ST_ACTIVE = 7,
  ST_ATOMICS = 8,        // global reservation atomics issued by k_step
  ST_BY_TYPE = 16, ST_COUNT = 32
};

struct ZRec {            // landing / carry / sorted-inbox record, 16 B
  uint32_t w0;           // seq << 16 | beh << 12 | to_local
  uint32_t from;
  uint64_t arg;
};

struct ORec {            // outbox record (zone scratch), 16 B
  uint32_t to;
  uint32_t w;            // seq << 16 | beh << 12 | src_local
  uint64_t arg;
};

// Cross-rank record, 16 B: ids travel as local slots (the receiver is the
// owner of `to`; the sender's rank is known from which peer's segment the
// record arrived in), which leaves 14 bits for the sender's sequence number:
//   w0 = seq >> 9 << 27 | beh << 23 | to_local   (to_local < 2^23 = kMaxZones * kZone)
//   w1 = (seq & 511) << 23 | from_local
// seq == kXSeqApply marks a reducible apply. Per-step sends per actor are
// therefore limited to kXSeqMax when n_ranks > 1 (kSeqMax otherwise).
struct XRec {
  uint32_t w0;
  uint32_t w1;
  uint64_t arg;
};
// A record that found its zone buffer full: kept with the position it was
// given (landing: its reserved slot; carry: its canonical carry position), so
// once the host has grown the zone it lands exactly where it would have.
// tag = pos | kind << 30 (kSpillCarry) ; one list per parity of the buffer.
struct SpillRec {        // 32 B (16-B aligned halves)
  ZRec     rec;
  uint32_t z;
  uint32_t tag;
  uint32_t pad[2];
};
static_assert(sizeof(SpillRec) == 32, "SpillRec is 32 B");
constexpr uint32_t kSpillCarry = 1u << 30;
constexpr uint32_t kSpillPosMask = kSpillCarry - 1;
constexpr unsigned long long kPendSkipped = ~0ull;   // pend[] mark of a step that did not run

constexpr uint32_t kXSeqApply = 0x3FFFu;
constexpr uint32_t kXSeqMax = 0x3FFEu;
static_assert(sizeof(XRec) == 16, "XRec is 16 B");
// A cross-rank record past its peer segment's capacity (xcap): kept with its
// peer and reserved position; the host grows xout and places it before the
// exchange sends anything (messageq.c:31-59 is unbounded; so is the exchange).
struct XSpillRec {       // 32 B
  XRec     rec;
  uint32_t peer;
  uint32_t pos;
  uint32_t pad[2];
};
static_assert(sizeof(XSpillRec) == 32, "XSpillRec is 32 B");

__device__ __forceinline__ uint64_t zkey(const ZRec& r)
{
  return ((uint64_t)r.from << 16) | (r.w0 >> 16);
}

struct TypeDev {
  uint32_t first, count;     // global id range
  uint32_t lfirst, lcount;   // local slot range on this rank
  uint32_t ht, words, batch, cap;
  uint32_t reducible, prio;   // prio: priority > 0 (gpu_actor_type_priority)
  uint64_t* state;           // [words][lcount]
  uint64_t  params[GPU_ACTOR_MAX_PARAMS];
  const uint64_t* prog;      // GPU_ACTOR_HT_PROGRAM: the behaviours' program
  uint32_t  prog_n, prog_pad;   // prog_pad bit 0: the program holds a YIELD
};

// One deferred carry copy: records rec(from + j), j < rem, of an actor's
// canonical mail (rec(k) = k < ncc ? c[k] : p[k - ncc]: its carried mail,
// then its sorted arrivals — read through perm, the sorted items
// key << 20 | position, when the workgroup sorted them) to dst[j]. base: the
// copy's first record in the step's list of all listed records (copies in
// slot order have rising bases).
struct BigCopy {
  const ZRec* c;
  const ZRec* p;
  ZRec* dst;
  const uint64_t* perm;
  uint32_t ncc, from, rem, base;
};
static_assert(sizeof(BigCopy) == 48, "BigCopy is 48 B");

struct EngDev {
  uint32_t n_types, rank, nranks, n_local;
  uint32_t n_zones;
  uint32_t n_ids;                 // the world's actor ids (SEND of a program past them drops)
  uint64_t r_magic;               // floor(2^64 / nranks) + 1 (nranks > 1): rdiv
  const uint64_t* zoff;           // [n_zones] record offset of each zone's buffers
  const uint32_t* zcapz;          // [n_zones] records a zone buffer holds
  ZRec* land[2];                  // zone z: [zoff[z], zoff[z] + zcapz[z])
  ZRec* carry[2];
  uint32_t* land_n[2];            // [n_zones]
  uint32_t* carry_n[2];
  ZRec* S;                        // zone z: [3 zoff[z], 3 zoff[z] + 3 zcapz[z])
  ORec* O;                        // zone z: [zoff[z], zoff[z] + zcapz[z])
  unsigned long long* stats;
  unsigned long long* pend;       // per-step pending counters
  XRec*  xout;                    // [nranks][xcap] (unused with peer_write: xdst)
  unsigned long long* xcount;     // [nranks]
  uint32_t xcap;
  uint32_t seq_max;               // kSeqMax, or kXSeqMax with n_ranks > 1
  unsigned long long* dbg;        // [n_zones][8] phase stamps (diagnostic build)
  // actors created by behaviours this step (gpu_actor_type_reserve): sort key
  // type << 52 | creator << 20 | seq << 4 | beh, and the constructor's arg
  uint64_t* spawn_key;
  uint64_t* spawn_arg;
  unsigned int* spawn_n;          // records written (may exceed spawn_cap: overflow)
  uint32_t spawn_cap, pad3;
  // zone buffers past capacity (never dropped): spill[p] holds the records
  // for parity p's landing/carry buffers; a step that finds spill_n[cur] or
  // halt set does not run (one rank) until the host has grown the zones
  // backpressure (Pony's mute, restated per superstep): per
  // global id, the state the last step left, bit 0 overloaded, bit 1 muted
  // (trig[p] is read by senders in the step that reads parity p; with
  // n_ranks > 1 each rank writes its own actors into trig_own[p] and the
  // host merges them into trig[p]); per local slot the receiver a muted actor
  // waits on; per zone how many of its actors have a nonzero byte in trig[p];
  // per step (index mod 3) how many actors trigger muting
  uint8_t* trig[2];
  uint8_t* trig_own[2];
  uint32_t* muted_on;
  unsigned int* spill_flag;      // n_ranks > 1: spill lists in use on any rank
  uint32_t* ztrig[2];
  unsigned int* trig_n;           // [3]
  SpillRec* spill[2];
  unsigned int* spill_n;          // [2]
  unsigned int* halt;             // set by a skipped step: every later step skips too
  unsigned long long* skipped;    // steps skipped since the last fixup
  uint32_t spill_cap, pad4;
  // cross-rank records past xcap (n_ranks > 1): placed by the host after growing xout
  XSpillRec* xspill;
  unsigned int* xspill_n;
  uint32_t xspill_cap, pad5;
  // zone geometry of this engine (step_entry.h): actors per zone = 1 << zbits.
  // k_step is compiled per geometry (kZoneBits below is its own); the helper
  // kernels and the small-step path read it here.
  uint32_t zbits, pad6;
  // backlogs handed to the whole GPU: with defer_big set, a
  // zone whose actor leaves more than kBigGroup records over (an overloaded
  // receiver) lists the copy here instead of making it with its own
  // workgroup; k_carry_big, launched right behind k_step, copies every listed
  // remainder across all CUs and clears the list.
  BigCopy* bigc;
  unsigned long long* bigc_n;     // [2]: listed copies << 32 | their records, finished k_carry_big workgroups
  uint32_t bigc_cap, defer_big;
  // order-free zones run their behaviours twice instead of through the outbox
  // (zone_dev.h two_pass; PONYC_AMD_TWO_PASS=0 turns it off for A/B runs)
  uint32_t two_pass, pad7;
  // [n_zones] zones the step's two-pass launch ran: step index + 1 (k_step PM 1)
  uint32_t* zplan;
  // k_step's per-step counters, sharded (pend_sh[slot][kShards],
  // stats_sh[ST_COUNT][kShards]; zone z adds to shard z % kShards): 512 zones
  // adding to one word serialise at the memory-side atomic unit (~12 ns each,
  // MI355X_MICROARCH.md fan-in row), and a zone waits out its own add at its
  // next barrier. k_fold sums the shards into pend[] / stats[] before the host
  // reads them.
  unsigned long long* pend_sh;
  unsigned long long* stats_sh;
  // hot zones prepared by the whole GPU before k_step (hot_dev.h k_hot):
  // hot_prep[z] = step index + 1 of the step whose arrivals k_hot placed in
  // S, hot_slot[z] its slot; per slot the arrivals per actor (hot_cnt,
  // [kMaxHot][4096], cleared by k_step as it reads them) and key ranges
  // (hot_aux); bins and cursors over the zone's big groups; the grid
  // barrier's words (hot_bar: [0] arrivals, [1] finished workgroups, [2]
  // workgroups that missed a phase, [3] zones given back to k_step after such
  // a miss). hot_test (PONYC_AMD_HOT_TEST=1, tests only): the last workgroup
  // reports a missed phase for every hot zone, as a barrier timeout would.
  uint32_t hot_on, hot_test;
  uint32_t* hot_prep;
  uint32_t* hot_slot;
  uint32_t* hot_cnt;
  uint32_t* hot_aux;
  uint32_t* hot_hist;
  uint32_t* hot_bcnt;
  uint32_t* hot_cur;
  uint32_t* hot_bar;
  // GUPS streamers' chunks handed to the whole GPU (one rank, DESIGN.md §7
  // C4): a streamer of type gups_type (-1: none) lists its PolyRand state
  // before the chunk in gups_list and moves past the chunk with one jump
  // (gups_jump[gups_parts] = x^chunk); k_gups_apply, launched behind every
  // step, regenerates each chunk over gups_parts lanes, lane p from state *
  // gups_jump[p] (= x^(p * gups_l)), and applies it. The list is kGupsShards
  // segments of gups_seg chunks, a wave listing into segment (its global wave
  // index mod kGupsShards): one counter for 16,384 listing waves per step
  // serialised at the memory-side atomic unit (~13 ns each, 210 us of a C4
  // wide step). gups_n: [s] chunks listed in segment s (past gups_seg a
  // streamer applies its chunk itself), [kGupsShards] finished k_gups_apply
  // workgroups. gups_stat: per k_gups_apply workgroup, updates generated and
  // atomics issued (an update whose XOR operand is 0 changes no word and is
  // not issued; same-word updates of one wave are combined).
  uint64_t* gups_list;
  unsigned int* gups_n;
  const uint64_t* gups_jump;
  unsigned long long* gups_stat;
  uint32_t gups_seg, gups_l, gups_parts;
  int32_t gups_type;
  // cross-rank records for peer p go to xdst[p][pos], pos < xcap: this rank's
  // segment p of xout, or with peer_write (engine.hip peer_open) this rank's
  // segment of peer p's inbox, mapped over IPC, so that the records cross
  // xGMI as k_step stores them and only the counts go through the collectives
  // (their stores, and the owner's loads, at system scope: xrec_put/xrec_get)
  XRec* xdst[kMaxRanks];
  uint32_t peer_write, pad9;
};
constexpr uint32_t kGupsShards = 64;
constexpr uint32_t kShards = 32;
// landed records that make a zone hot (hot_dev.h). k_step consumes a prepared
// zone's counts only on its scratch path, so a hot zone must never fit the
// LDS index (zone_dev.h static_assert against kIdxCap).
constexpr uint32_t kHotMin = 32768;


__constant__ TypeDev c_types[GPU_ACTOR_MAX_TYPES];
__constant__ EngDev  c_eng;

// x / nranks and x % nranks without a division instruction sequence: for
// 32-bit x, mulhi(x, floor(2^64 / d) + 1) is exact (Lemire's fastdiv).
__device__ __forceinline__ uint32_t rdiv(uint32_t x)
{
  return c_eng.nranks == 1 ? x : (uint32_t)__umul64hi(c_eng.r_magic, (uint64_t)x);
}

__device__ __forceinline__ uint32_t rmod(uint32_t x)
{
  return x - rdiv(x) * c_eng.nranks;
}

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

// records a zone's landing/carry/outbox buffer holds: the sum over its serial
// actors of their type's mailbox capacity
__device__ __forceinline__ uint32_t zone_capacity(uint32_t z)
{
  return c_eng.zcapz[z];
}

// The same for a wave-uniform z (a workgroup's own zone): the values read
// through the table are uniform too, but the compiler cannot prove it and
// would hold them — and the zone's buffer pointers built from them — in
// vector registers, which the general drain spills (the outbox pointer was
// reloaded from scratch at every send). readfirstlane puts them in SGPRs.
__device__ __forceinline__ uint32_t zone_cap_s(uint32_t z)
{
  return __builtin_amdgcn_readfirstlane(c_eng.zcapz[z]);
}

__device__ __forceinline__ uint64_t zone_off_s(uint32_t z)
{
  const uint64_t o = c_eng.zoff[z];
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(o >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)o);
}

// zone of a local slot, and the slot within its zone (this engine's geometry)
__device__ __forceinline__ uint32_t zone_of_local(uint32_t L) { return L >> c_eng.zbits; }
__device__ __forceinline__ uint32_t slot_in_zone(uint32_t L) { return L & ((1u << c_eng.zbits) - 1u); }

// outbox bucket of a destination: its zone, or n_zones + peer rank if remote
__device__ __forceinline__ uint32_t bucket_of(uint32_t to)
{
  const uint32_t R = c_eng.nranks;
  if(R > 1)
  {
    const uint32_t owner = rmod(to);
    if(owner != c_eng.rank) return c_eng.n_zones + owner;
  }
  return zone_of_local(rdiv(to));
}

// Cross-rank record from global ids and a (seq << 16 | beh << 12) word.
__device__ __forceinline__ XRec xpack(uint32_t to, uint32_t w, uint32_t from, uint64_t arg)
{
  const uint32_t seq = (w >> 16) == kSeqApply ? kXSeqApply : (w >> 16);
  XRec x;
  x.w0 = (seq >> 9) << 27 | ((w >> 12) & 0xFu) << 23 | rdiv(to);
  x.w1 = (seq & 0x1FFu) << 23 | rdiv(from);
  x.arg = arg;
  return x;
}

// Per-lane bookkeeping while one actor drains: the fields every delivery
// context shares. A context type (ZoneCtx: k_step's zone outbox; SparseCtx:
// k_sparse's LDS message list) adds put(to, w, arg), the serial send.
struct ActorBase {
  uint32_t self;         // global id
  uint32_t li;           // index within its type (local)
  uint32_t src_local;    // slot within the zone
  uint32_t seq;          // sends this step
  uint32_t sent;
  uint32_t applied;      // local reducible applies issued
  int      applied_type;
  int      type;         // the draining actor's type
  unsigned long long* agg;   // this wave's LDS aggregation word
  unsigned long long* fan;   // zone accumulators of fan-in applies (LDS, 2 x kFanLds) or null
  int      fan_t;        // analyzer type those accumulators are for
  // the reducible type last applied to (gups updater), cached so that a run
  // of applies does not look the type up, and wait, once per message
  uint32_t rc_first, rc_count, rc_lfirst, rc_lcount;
  uint64_t* rc_state;
  uint64_t rc_mask;
  // backpressure while this actor runs: the step's trigger bytes (null when
  // no actor triggers muting), whether this actor was overloaded after the
  // last step, and what its sends and behaviours asked for
  const uint8_t* trig;
  uint32_t prev_o;
  uint32_t mute_hit;     // a send went to an overloaded or muted actor
  uint32_t mute_to;      // the first such receiver
  uint32_t yield_req;    // the behaviour yielded (ponyint_actor_yield)

  // kPlain: a context whose sends can neither run out of sequence numbers
  // nor mute (the two-pass path: no backpressure anywhere, the zone's whole
  // mail below seq_max) — send_serial then skips both checks
  static constexpr bool kPlain = false;

  __device__ __forceinline__ void reset_common()
  {
    trig = nullptr; prev_o = 0; mute_hit = 0; mute_to = 0; yield_req = 0;
    seq = 0; sent = 0; applied = 0; applied_type = -1;
    fan = nullptr; fan_t = -1;
    rc_first = rc_count = rc_lfirst = rc_lcount = 0;
    rc_state = nullptr;
    rc_mask = 0;
  }
};

struct ZoneCtx;
__device__ __forceinline__ void outbox_put(ZoneCtx& a, uint32_t to, uint32_t w, uint64_t arg);

struct ZoneCtx : ActorBase {
  ORec*     out;         // zone outbox (global scratch)
  uint32_t  ocap;        // its capacity
  uint32_t  nxt;         // landing parity of this step's sends
  uint32_t* s_nout;      // LDS outbox counter
  uint32_t* s_hist;      // LDS histogram by bucket
  __device__ __forceinline__ void put(uint32_t to, uint32_t w, uint64_t arg) { outbox_put(*this, to, w, arg); }
};
// ---- delivery --------------------------------------------------------------

// Reducible behaviours: applied as device atomics at the owner.
__device__ __forceinline__ void reducible_apply_local(uint32_t to, uint32_t beh, uint64_t arg)
{
  const int t = type_of_global(to);
  if(t < 0) return;
  const TypeDev& T = c_types[t];
  const uint32_t li = rdiv(to) - T.lfirst;
  switch(T.ht)
  {
    case GPU_ACTOR_HT_FANIN_ANALYZER:
      atomicAdd(reinterpret_cast<unsigned long long*>(&T.state[li]), 1ull);
      atomicXor(reinterpret_cast<unsigned long long*>(&T.state[(size_t)T.lcount + li]),
        (unsigned long long)arg);
      break;
    case GPU_ACTOR_HT_GUPS_UPDATER: {
      // t[d & m] ^= d
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

// Per-step counters of zone z (k_step), to its shard
__device__ __forceinline__ void pend_add_z(uint32_t slot, uint32_t z, unsigned long long v)
{
  atomicAdd(&c_eng.pend_sh[(size_t)slot * kShards + (z & (kShards - 1u))], v);
}
__device__ __forceinline__ void stat_add_z(int idx, uint32_t z, unsigned long long v)
{
  atomicAdd(&c_eng.stats_sh[(size_t)idx * kShards + (z & (kShards - 1u))], v);
}

// A record whose zone buffer (parity p, landing or carry) is full at `pos`.
__device__ __forceinline__ void spill_rec(uint32_t p, uint32_t kind, uint32_t z, uint32_t pos,
  const uint4& v)
{
  const unsigned int i = atomicAdd(&c_eng.spill_n[p], 1u);
  if(i < c_eng.spill_cap)
  {
    uint32_t* d = reinterpret_cast<uint32_t*>(c_eng.spill[p] + i);
    *reinterpret_cast<uint4*>(d) = v;
    *reinterpret_cast<uint4*>(d + 4) = make_uint4(z, pos | kind, 0u, 0u);
  }
  else
    atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);   // the spill list itself is full
}

// Store cross-rank record x at reserved position pos of peer segment `peer`;
// past the segment's capacity it goes to the exchange spill list (lost, and
// counted, only when that list is full too). Returns 1 if it was lost.
// A cross-rank record's store into its segment (EngDev::xdst) and its load by
// k_xinject: with peer_write the segment is another GPU's memory, written by
// this GPU's stores over xGMI and read by its owner while neither L2 may hold
// a copy, so both sides go to memory (system scope); plain otherwise.
__device__ __forceinline__ void xrec_put(XRec* d, const XRec& x)
{
  if(c_eng.peer_write)
  {
    uint64_t* q = reinterpret_cast<uint64_t*>(d);
    __hip_atomic_store(q, (uint64_t)x.w1 << 32 | x.w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, x.arg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  else
    *d = x;
}

__device__ __forceinline__ XRec xrec_get(const XRec* s)
{
  if(!c_eng.peer_write) return *s;
  const uint64_t* q = reinterpret_cast<const uint64_t*>(s);
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  XRec x;
  x.w0 = (uint32_t)a;
  x.w1 = (uint32_t)(a >> 32);
  x.arg = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return x;
}

__device__ __forceinline__ uint32_t xout_store(uint32_t peer, uint32_t pos, const XRec& x)
{
  if(pos < c_eng.xcap)
  {
    xrec_put(c_eng.xdst[peer] + pos, x);
    return 0;
  }
  const unsigned int i = atomicAdd(c_eng.xspill_n, 1u);
  if(i >= c_eng.xspill_cap) return 1;
  uint32_t* d = reinterpret_cast<uint32_t*>(c_eng.xspill + i);
  *reinterpret_cast<uint4*>(d) = make_uint4(x.w0, x.w1, (uint32_t)x.arg, (uint32_t)(x.arg >> 32));
  *reinterpret_cast<uint4*>(d + 4) = make_uint4(peer, pos, 0u, 0u);
  return 0;
}

// Store landing record v of zone z at reserved position pos of parity p.
__device__ __forceinline__ void land_store(uint32_t p, uint32_t z, uint32_t pos, const uint4& v)
{
  if(pos < zone_capacity(z))
    *reinterpret_cast<uint4*>(c_eng.land[p] + c_eng.zoff[z] + pos) = v;
  else
    spill_rec(p, 0u, z, pos, v);
}

// Outbox full (a zone sent more than its mailbox capacity this step): land the
// record directly with its own atomic on the destination bucket's counter. The
// receiver sorts by key, so where a record lands does not change delivery order.
__device__ __forceinline__ void send_direct(uint32_t nxt, uint32_t self, uint32_t to, uint32_t w, uint64_t arg)
{
  const uint32_t R = c_eng.nranks;
  const uint32_t nz = c_eng.n_zones;
  const uint32_t b = bucket_of(to);
  if(b < nz)
  {
    const uint32_t pos = atomicAdd(&c_eng.land_n[nxt][b], 1u);
    uint4 v;
    v.x = w | slot_in_zone(rdiv(to));
    v.y = self;
    v.z = (uint32_t)arg;
    v.w = (uint32_t)(arg >> 32);
    land_store(nxt, b, pos, v);
  }
  else
  {
    const unsigned long long pos = atomicAdd(&c_eng.xcount[b - nz], 1ull);
    if(pos > 0x3FFFFFFFull || xout_store(b - nz, (uint32_t)pos, xpack(to, w, self, arg)))
      atomicAdd(&c_eng.stats[ST_XCHG_OVERFLOW], 1ull);
  }
}

// Park one record in the zone outbox and count it in its destination bucket.
__device__ __forceinline__ void outbox_put(ZoneCtx& a, uint32_t to, uint32_t w, uint64_t arg)
{
  const uint32_t idx = atomicAdd(a.s_nout, 1u);
  if(idx >= a.ocap)
  {
    send_direct(a.nxt, a.self, to, w, arg);
    return;
  }
  ORec r;
  r.to = to; r.w = w | a.src_local; r.arg = arg;
  *reinterpret_cast<uint4*>(a.out + idx) = *reinterpret_cast<const uint4*>(&r);
  atomicAdd(&a.s_hist[bucket_of(to)], 1u);
}

// A handler's send: stamped with its canonical (sender, seq) key now.
template <class A>
__device__ __forceinline__ void send_serial(A& a, uint32_t to, uint32_t beh, uint64_t arg)
{
  a.sent++;
  if constexpr(!A::kPlain)
    if(a.seq >= c_eng.seq_max)
    {
      atomicAdd(&c_eng.stats[ST_SEQ_OVERFLOW], 1ull);
      return;
    }
  a.put(to, (a.seq << 16) | (beh << 12), arg);
  a.seq++;
  // ponyint_maybe_mute (actor.c:898-921): a send to an actor that is
  // overloaded or muted mutes a sender that is not overloaded itself, unless
  // it sends to itself; the sender stops after the behaviour it is running
  if constexpr(!A::kPlain)
    if(a.trig && !a.prev_o && !a.mute_hit && to != a.self && a.trig[to] != 0)
    {
      a.mute_hit = 1;
      a.mute_to = to;
    }
}

// ponyint_actor_yield (actor.c:675-679): end the actor's run after this
// behaviour; the rest of its mail waits for the next step.
template <class A>
__device__ __forceinline__ void actor_yield(A& a)
{
  a.yield_req = 1;
}

// pony_create inside a behaviour + its constructor message (actor.c:688-734,
// gencall.c:606-612): recorded with its canonical key; the id is assigned
// when the step ends (engine.hip: spawn_process), the constructor message is
// delivered in the next step. Counts as a send of the creator.
template <class A>
__device__ __forceinline__ void spawn_actor(A& a, uint32_t type, uint32_t beh, uint64_t arg)
{
  a.sent++;
  if(a.seq >= c_eng.seq_max)
  {
    atomicAdd(&c_eng.stats[ST_SEQ_OVERFLOW], 1ull);
    return;
  }
  const unsigned int pos = atomicAdd(c_eng.spawn_n, 1u);
  if(pos < c_eng.spawn_cap)
  {
    c_eng.spawn_key[pos] = ((uint64_t)type << 52) | ((uint64_t)a.self << 20) |
                           ((uint64_t)a.seq << 4) | (beh & 0xFu);
    c_eng.spawn_arg[pos] = arg;
  }
  else
    atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);
  a.seq++;
}

__device__ __forceinline__ bool is_remote(uint32_t to)
{
  return c_eng.nranks > 1 && rmod(to) != c_eng.rank;
}

// fan-in Analyzer apply, aggregated per wavefront: lanes hitting the same
// analyzer fold their count and XOR through LDS and one lane issues the two
// global atomics (Guideline 12: one atomic per (wave, destination)).
template <class A>
__device__ __forceinline__ void send_analyzer(A& a, uint32_t to, uint64_t arg)
{
  a.sent++;
  const bool remote = is_remote(to);
  if(remote)
    a.put(to, (kSeqApply << 16) | (GPU_ACTOR_FANIN_MSG << 12), arg);  // counted by owner
  else
  {
    a.applied++;
    if(a.applied_type < 0) a.applied_type = type_of_global(to);
  }
  const int lane = __lane_id();
  unsigned long long* agg = a.agg;
  unsigned long long active = __ballot(!remote);
  while(active != 0ull)
  {
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t tl = __builtin_amdgcn_readlane(to, leader);
    const bool mine = !remote && to == tl;
    const unsigned long long peers = __ballot(mine);
    if(lane == leader) *agg = 0ull;
    __builtin_amdgcn_wave_barrier();
    if(mine) atomicXor(agg, (unsigned long long)arg);
    __builtin_amdgcn_wave_barrier();
    if(lane == leader)
    {
      const int t = type_of_global(tl);
      if(t >= 0)
      {
        const TypeDev& T = c_types[t];
        const uint32_t li = rdiv(tl) - T.lfirst;
        if(a.fan && t == a.fan_t && li < kFanLds)
        {
          // zone accumulator: one global atomic per (zone, analyzer) at the end
          atomicAdd(&a.fan[li], (unsigned long long)__popcll(peers));
          atomicXor(&a.fan[kFanLds + li], *agg);
        }
        else
        {
          atomicAdd(reinterpret_cast<unsigned long long*>(&T.state[li]),
            (unsigned long long)__popcll(peers));
          atomicXor(reinterpret_cast<unsigned long long*>(&T.state[(size_t)T.lcount + li]),
            *agg);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    active &= ~peers;
  }
}

template <class A>
__device__ __forceinline__ void send_updater(A& a, uint32_t to, uint64_t d)
{
  a.sent++;
  if(is_remote(to))
  {
    a.put(to, (kSeqApply << 16) | (GPU_ACTOR_GUPS_UPDATE << 12), d);  // counted by owner
    return;
  }
  a.applied++;
  if(to - a.rc_first >= a.rc_count)
  {
    const int t = type_of_global(to);
    if(t < 0) return;
    const TypeDev& T = c_types[t];
    if(a.applied_type < 0) a.applied_type = t;
    a.rc_first = T.first; a.rc_count = T.count;
    a.rc_lfirst = T.lfirst; a.rc_lcount = T.lcount;
    a.rc_state = T.state;
    a.rc_mask = T.params[0] - 1;
  }
  // gups_basic Updater.apply: t[d & (size - 1)] ^= d, every update issued
  // (the streamers' chunks on one rank go through k_gups_apply instead)
  const uint32_t li = rdiv(to) - a.rc_lfirst;
  atomicXor(reinterpret_cast<unsigned long long*>(&a.rc_state[(d & a.rc_mask) * a.rc_lcount + li]),
    (unsigned long long)d);
}

// A GUPS streamer's chunk handed to k_gups_apply: its PolyRand state before
// the chunk listed (one list atomic per wave, on the wave's segment), the
// chunk's updates counted as sent and applied here. False when the segment is
// full: the streamer applies the chunk itself.
template <class A>
__device__ __forceinline__ bool gups_defer(A& a, uint64_t last, uint64_t chunk, uint32_t ubase)
{
  const uint64_t m = __ballot(1);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const uint32_t sh = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kGupsShards - 1u);
  unsigned int base = 0;
  if(below == 0) base = atomicAdd(&c_eng.gups_n[sh], (unsigned int)__popcll(m));
  base = __builtin_amdgcn_readfirstlane(base);
  const unsigned int i = base + below;
  if(i >= c_eng.gups_seg) return false;
  c_eng.gups_list[(size_t)sh * c_eng.gups_seg + i] = last;
  a.sent += (uint32_t)chunk;
  a.applied += (uint32_t)chunk;
  if(a.applied_type < 0) a.applied_type = type_of_global(ubase);
  return true;
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
template <> struct HT_Words<GPU_ACTOR_HT_SPREADER>      { static constexpr int W = 5; };
template <> struct HT_Words<GPU_ACTOR_HT_PROGRAM>       { static constexpr int W = 8; };
// Behaviours as programs compiled at run time (engine.hip jit): the program
// table's state, its handle() generated from the program words
constexpr int kHtJit = 13;
template <> struct HT_Words<kHtJit>                     { static constexpr int W = 8; };

template <int HT> struct HtTag {};

// examples/ring/main.pony:13-24
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_RING>, const TypeDev& T, A& a,
  uint64_t (&s)[4], uint32_t beh, uint64_t arg)
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
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_PINGER>, const TypeDev& T, A& a,
  uint64_t (&s)[3], uint32_t beh, uint64_t arg)
{
  s[2] += 1;
  if(s[2] <= T.params[2])
  {
    const uint64_t k = rand_int(s[0], s[1], T.params[0]);
    send_serial(a, (uint32_t)(T.params[1] + k), GPU_ACTOR_PINGER_PING, 42);
  }
}

template <class A>
__device__ __forceinline__ void det_ping(const TypeDev& T, A& a, uint64_t& count,
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

template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_PINGER_DET>, const TypeDev& T, A& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg)
{
  det_ping(T, a, s[0], s[1], beh, arg);
}

template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_STORM>, const TypeDev& T, A& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg)
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
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_FANIN_SENDER>, const TypeDev& T, A& a,
  uint64_t (&s)[4], uint32_t beh, uint64_t arg)
{
  const uint64_t k = rand_int_unbiased(s[0], s[1], T.params[0]);
  const uint64_t i = a.self - T.first;
  send_analyzer(a, (uint32_t)(T.params[1] + k), (i << 32) | s[3]);
  s[3] += 1;
  if(s[2] > 0) s[2] -= 1;
  if(s[2] > 0)
    send_serial(a, a.self, GPU_ACTOR_FANIN_SEND_MSGS, 0);
}

// examples/gups_basic/main.pony:110-143, one message per datum
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_GUPS_STREAMER>, const TypeDev& T, A& a,
  uint64_t (&s)[2], uint32_t beh, uint64_t arg)
{
  const uint64_t chunk = T.params[0], shift = T.params[1], mask = T.params[2];
  const uint32_t ubase = (uint32_t)T.params[3];
  uint64_t last = s[0];
  // one rank: the chunk goes to k_gups_apply, the state jumps past it
  if(a.type == c_eng.gups_type && gups_defer(a, last, chunk, ubase))
    last = polyrand_mulmod(last, c_eng.gups_jump[c_eng.gups_parts]);
  else
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

template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_FIFO_SRC>, const TypeDev& T, A& a,
  uint64_t (&s)[3], uint32_t beh, uint64_t arg)
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

template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_FIFO_SINK>, const TypeDev& T, A& a,
  uint64_t (&s)[11], uint32_t beh, uint64_t arg)
{
  // slot = ((arg >> 32) / ns) % 8. The sender index is 32 bits, so the
  // quotient is mulhi(floor(2^64 / ns) + 1, index) for ns >= 2 (rdiv's
  // fastdiv); the magic depends on the type's parameter only and leaves the
  // drain's loop (a 64-bit and then a 32-bit division per message were most of
  // a hot sink's per-behaviour instructions)
  const uint64_t ns = T.params[0] > 1 ? T.params[0] : 1;
  const uint64_t magic = ~0ull / ns + 1u;
  const uint32_t sx = (uint32_t)(arg >> 32);
  const uint32_t slot = ns > 0xFFFFFFFFull ? 0u
                      : ((ns == 1 ? sx : (uint32_t)__umul64hi(magic, (uint64_t)sx)) & 7u);
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
  // param 1: yield after every k-th message
  if(T.params[1] && s[1] % T.params[1] == 0) actor_yield(a);
}

// Behaviours as a program (include/gpu_actor.h GPU_ACTOR_HT_PROGRAM): the
// reference's generated dispatch (gentype.c:358-395) for any behaviour set,
// here one interpreter lane per actor. Registers r0-r7 are the state, r8 the
// argument, r9 self, r10 the behaviour; indexed at run time, they live in
// scratch. oracle/bsp.c restates it instruction for instruction.
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_PROGRAM>, const TypeDev& T, A& a,
  uint64_t (&s)[8], uint32_t beh, uint64_t arg)
{
  const uint64_t* const P = T.prog;
  const uint32_t np = T.prog_n;
  if(!P || np <= GPU_ACTOR_PROG_ENTRIES) return;
  uint32_t pc = (uint32_t)P[beh & 15u];
  if(pc == 0) return;
  uint64_t r[16];
#pragma unroll
  for(int k = 0; k < 8; ++k) r[k] = s[k];
  r[8] = arg; r[9] = a.self; r[10] = beh;
#pragma unroll
  for(int k = 11; k < 16; ++k) r[k] = 0;
  for(uint32_t step = 0; step < GPU_ACTOR_PROG_MAX_STEPS && pc < np; ++step)
  {
    const uint64_t ins = P[pc++];
    const uint32_t op = (uint32_t)ins & 0xFFu, d = ((uint32_t)ins >> 8) & 15u;
    const uint64_t x = r[((uint32_t)ins >> 12) & 15u], y = r[((uint32_t)ins >> 16) & 15u];
    const int64_t imm = (int32_t)(uint32_t)(ins >> 32);
    if(op == GPU_ACTOR_OP_HALT || op > GPU_ACTOR_OP_SPAWN) break;
    if(op == GPU_ACTOR_OP_JZ || op == GPU_ACTOR_OP_JNZ || op == GPU_ACTOR_OP_JMP)
    {
      const bool take = op == GPU_ACTOR_OP_JMP || ((x == 0) == (op == GPU_ACTOR_OP_JZ));
      if(take) pc = (uint32_t)((int64_t)pc + imm);
      continue;
    }
    if(op == GPU_ACTOR_OP_SEND)
    {
      if(x < c_eng.n_ids)
        send_serial(a, (uint32_t)x, (uint32_t)imm & 15u, y);
      else
        atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);
      continue;
    }
    if(op == GPU_ACTOR_OP_YIELD) { actor_yield(a); continue; }
    if(op == GPU_ACTOR_OP_SPAWN)
    {
      if(((uint32_t)imm & 0xFFu) < GPU_ACTOR_MAX_TYPES)
        spawn_actor(a, (uint32_t)imm & 0xFFu, ((uint32_t)imm >> 8) & 15u, y);
      else
        atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);
      continue;
    }
    uint64_t v;
    switch(op)
    {
      case GPU_ACTOR_OP_LDI:   v = (uint64_t)imm; break;
      case GPU_ACTOR_OP_LDP:   v = T.params[imm & 7]; break;
      case GPU_ACTOR_OP_MOV:   v = x; break;
      case GPU_ACTOR_OP_ADD:   v = x + y; break;
      case GPU_ACTOR_OP_SUB:   v = x - y; break;
      case GPU_ACTOR_OP_MUL:   v = x * y; break;
      case GPU_ACTOR_OP_MULHI: v = __umul64hi(x, y); break;
      case GPU_ACTOR_OP_AND:   v = x & y; break;
      case GPU_ACTOR_OP_OR:    v = x | y; break;
      case GPU_ACTOR_OP_XOR:   v = x ^ y; break;
      case GPU_ACTOR_OP_SHL:   v = x << (y & 63u); break;
      case GPU_ACTOR_OP_SHR:   v = x >> (y & 63u); break;
      case GPU_ACTOR_OP_ADDI:  v = x + (uint64_t)imm; break;
      case GPU_ACTOR_OP_LTU:   v = x < y ? 1u : 0u; break;
      case GPU_ACTOR_OP_EQ:    v = x == y ? 1u : 0u; break;
      default:                 v = splitmix_mix(x); break;     // GPU_ACTOR_OP_MIX
    }
    r[d] = v;
  }
#pragma unroll
  for(int k = 0; k < 8; ++k) s[k] = r[k];
}

// examples/spreader/main.pony:9-48
template <class A>
__device__ __forceinline__ void handle(HtTag<GPU_ACTOR_HT_SPREADER>, const TypeDev& T, A& a,
  uint64_t (&s)[5], uint32_t beh, uint64_t arg)
{
  if(beh == GPU_ACTOR_SPREADER_SPREAD)
  {
    // new create(env) / new spread(parent, count)
    const uint64_t parent = arg >> 32, count = arg & 0xFFFFFFFFull;
    s[0] = count;
    s[1] = parent == 0xFFFFFFFFull ? GPU_ACTOR_NONE : parent;
    if(count <= 1)
    {
      if(s[1] != GPU_ACTOR_NONE) send_serial(a, (uint32_t)s[1], GPU_ACTOR_SPREADER_RESULT, 1);
      else s[4] = 1;                                     // "1 actor"
    }
    else
    {
      // spawn_child() twice: Spreader.spread(this, _count - 1)
      const uint64_t ctor = ((uint64_t)a.self << 32) | (count - 1);
      spawn_actor(a, (uint32_t)a.type, GPU_ACTOR_SPREADER_SPREAD, ctor);
      spawn_actor(a, (uint32_t)a.type, GPU_ACTOR_SPREADER_SPREAD, ctor);
    }
    return;
  }
  // be result(i)
  s[3] += 1;
  s[2] += arg;
  if(s[3] == 2)
  {
    if(s[1] != GPU_ACTOR_NONE) send_serial(a, (uint32_t)s[1], GPU_ACTOR_SPREADER_RESULT, s[2] + 1);
    else s[4] = s[2] + 1;                               // "<n> actors"
  }
}

} // namespace gpa

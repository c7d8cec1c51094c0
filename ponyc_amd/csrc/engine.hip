// engine.hip — the gpu_actor engine for gfx950: kernels (zone_dev.h) and the
// C-ABI declared in include/gpu_actor.h.
//
// One superstep = one k_step launch (one workgroup per 2048-actor zone; see
// zone_dev.h). With n_ranks > 1, the records a step produced for actors on
// other ranks are swapped with RCCL after it (counts all-to-all, then grouped
// ncclSend/ncclRecv over xGMI) and k_xinject lands them before the next step.
// The launch boundary is the BSP barrier; quiescence ("no pending mail on any
// rank") replaces the CNF/ACK protocol (scheduler.c:303-480).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "engine_dev.h"
#include "zone_dev.h"
#include "sparse_dev.h"
#include "hot_dev.h"
#include "step_entry.h"
#include "jit_host.h"

// the 4096-actor-zone instantiations (step_*_z12.hip)
namespace gpa_z12 {
StepEntry step_entry_any();
StepEntry step_entry_ring();
StepEntry step_entry_pinger();
StepEntry step_entry_pinger_det();
StepEntry step_entry_fanin_sender();
StepEntry step_entry_gups_streamer();
StepEntry step_entry_storm();
StepEntry step_entry_spreader();
StepEntry step_entry_fifo_pair();
StepEntry step_entry_program();
} // namespace gpa_z12

using namespace gpa;

// gups Updater tables (gups_basic/main.pony:145-155: table[k] = k + index*size),
// one thread per word (field-major state[k * lcount + li]).
__global__ void __launch_bounds__(kBlock) k_construct_table(uint32_t t, uint32_t live)
{
  const TypeDev& T = c_types[t];
  const uint64_t n = T.lcount;
  const uint64_t size = T.params[0] < T.words ? T.params[0] : T.words;
  const uint64_t total = size * n;
  for(uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x; x < total;
      x += (uint64_t)gridDim.x * kBlock)
  {
    const uint64_t k = x / n, li = x - k * n;
    const uint64_t L = T.lfirst + li;
    const uint64_t i = L * c_eng.nranks + c_eng.rank - T.first;
    if(i >= live) continue;
    T.state[x] = k + i * size;
  }
}

// pony_create's constructor run: initial state of a freshly created type;
// the first `live` ids of the type (the rest are reserved for actors its
// behaviours create, and stay zeroed until then).
__global__ void __launch_bounds__(kBlock) k_construct(uint32_t t, uint32_t live)
{
  const TypeDev& T = c_types[t];
  const uint32_t li = blockIdx.x * kBlock + threadIdx.x;
  if(li >= T.lcount) return;
  const uint32_t L = T.lfirst + li;
  const uint64_t i = (uint64_t)L * c_eng.nranks + c_eng.rank - T.first;   // index in type
  if(i >= live) return;
  const size_t n = T.lcount;
  uint64_t* st = T.state;
  switch(T.ht)
  {
    case GPU_ACTOR_HT_RING: {
      const uint64_t size = T.params[0] ? T.params[0] : 1;
      const uint64_t ring = i / size, p = i % size;
      st[li] = (p == 0) ? GPU_ACTOR_NONE : T.first + ring * size + (p + 1) % size;
      st[n + li] = p + 1;
      break;
    }
    case GPU_ACTOR_HT_PINGER: {
      uint64_t x, y;
      xoro_create(x, y, T.params[3] + i + 1, 0x9E3779B97F4A7C15ull);
      (void)rand_int(x, y, 100); (void)rand_int(x, y, 100); (void)rand_int(x, y, 100);
      st[li] = x; st[n + li] = y;
      break;
    }
    case GPU_ACTOR_HT_FANIN_SENDER: {
      uint64_t x, y;
      xoro_create(x, y, T.params[3] ? 5489 + i : 5489, 0);
      st[li] = x; st[n + li] = y; st[2 * n + li] = T.params[2];
      break;
    }
    case GPU_ACTOR_HT_GUPS_STREAMER:
      st[li] = polyrand_seeded(T.params[5] * i);
      break;
    case GPU_ACTOR_HT_GUPS_UPDATER:      // the table: k_construct_table
      break;
    case GPU_ACTOR_HT_FIFO_SRC: {
      const uint64_t ns = T.params[1] ? T.params[1] : 1;
      st[li] = T.params[0] + i % ns;
      st[2 * n + li] = T.params[2];
      break;
    }
    case GPU_ACTOR_HT_FIFO_SINK:
      st[li] = 0xcbf29ce484222325ull;
      break;
    default:
      break;
  }
}

// Copy each zone's old buffer into its slot of a new layout (one block per zone).
__global__ void __launch_bounds__(kBlock) k_zone_copy(const ZRec* src, const uint64_t* src_off,
  const uint32_t* src_cap, ZRec* dst, const uint64_t* dst_off)
{
  const uint32_t z = blockIdx.x;
  const ZRec* s = src + src_off[z];
  ZRec* d = dst + dst_off[z];
  for(uint32_t i = threadIdx.x; i < src_cap[z]; i += kBlock) d[i] = s[i];
}

// ---- actors spawned by behaviours (gpu_actor_type_reserve) -------------------
// After a step: the spawn records, sorted by key (type, creator, seq), get ids
// first + live[type] + (rank within the type); each new actor's constructor
// message lands like any other arrival for the next step.
__global__ void __launch_bounds__(kBlock) k_spawn_scan(const uint64_t* key, uint32_t n,
  uint32_t* tstart, uint32_t* tcnt)
{
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  const uint32_t t = (uint32_t)(key[i] >> 52);
  atomicMin(&tstart[t], i);
  atomicAdd(&tcnt[t], 1u);
}

__global__ void __launch_bounds__(kLandThreads) k_spawn_land(const uint64_t* key, const uint64_t* arg,
  uint32_t n, const uint32_t* tstart, const unsigned long long* live, uint32_t cur)
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
      const uint64_t k = key[i];
      const uint32_t t = (uint32_t)(k >> 52);
      const TypeDev& T = c_types[t];
      const uint64_t slot = live[t] + (i - tstart[t]);
      if(slot < T.count)
      {
        // every rank numbers the same gathered list; it lands its own actors
        r[u].valid = c_eng.nranks == 1 || (T.first + slot) % c_eng.nranks == c_eng.rank;
        r[u].to = T.first + (uint32_t)slot;
        r[u].w = (uint32_t)(((k >> 4) & 0xFFFFull) << 16) | (uint32_t)((k & 0xFu) << 12);
        r[u].from = (uint32_t)(k >> 20);
        r[u].arg = arg[i];
      }
      else if(c_eng.rank == 0)
        atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);     // reserve exhausted
    }
  }
  land_records(r, cur, s_hist, s_base);
}

__global__ void k_spawn_commit(const uint32_t* tcnt, unsigned long long* live)
{
  const uint32_t t = threadIdx.x;
  if(t >= GPU_ACTOR_MAX_TYPES || tcnt[t] == 0) return;
  const unsigned long long room = c_types[t].count - live[t];
  live[t] += tcnt[t] < room ? tcnt[t] : room;
}

// ---- records past a zone's capacity (SpillRec, engine_dev.h) ----------------
// need[z] = largest position + 1 spilled into zone z (either buffer)
__global__ void __launch_bounds__(kBlock) k_spill_need(const SpillRec* s, uint32_t n, uint32_t* need)
{
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  atomicMax(&need[s[i].z], (s[i].tag & kSpillPosMask) + 1u);
}

// after the zones have grown: every spilled record to its own position
__global__ void __launch_bounds__(kBlock) k_spill_place(const SpillRec* s, uint32_t n, uint32_t p)
{
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  const SpillRec r = s[i];
  ZRec* base = (r.tag & kSpillCarry) ? c_eng.carry[p] : c_eng.land[p];
  base[c_eng.zoff[r.z] + (r.tag & kSpillPosMask)] = r.rec;
}

// Backlog copies listed by k_step (EngDev::bigc, defer_big): the listed
// records form one flat range (each copy's base, in slot order), cut into
// equal contiguous chunks, one per workgroup; a workgroup finds the first copy
// its chunk touches (binary search over the bases) and walks on from there,
// so one overloaded receiver's remainder moves at the whole GPU's bandwidth
// and no workgroup visits copies outside its chunk. With nothing listed the
// kernel returns at once. The list's counter is kept per step parity (cur):
// the next step's k_step clears this one (its zone 0, at its start), so no
// workgroup here signals another (the last-finisher count and fence took
// ~6 us a step: 512 adds on one word).
constexpr uint32_t kBigCopyCap = 4096;
constexpr uint32_t kBigCopyBlocks = 512;
__global__ void __launch_bounds__(kBlock) k_carry_big(uint32_t cur)
{
  // a step that did not run listed nothing (its counter may hold a list of
  // two steps before, already copied)
  const bool halt_now = c_eng.nranks == 1 ? (c_eng.spill_n[cur] != 0u || *c_eng.halt != 0u)
                                          : (*c_eng.spill_flag != 0u);
  if(halt_now) return;
  const unsigned long long v = c_eng.bigc_n[cur];  // final: k_step ran to completion before
  const uint32_t n = min((uint32_t)(v >> 32), c_eng.bigc_cap);
  if(n == 0) return;
  // the listed copies' records: the last one's base + its length (bigc_n's
  // low word also counts copies past bigc_cap, which their zones made)
  const uint32_t total = c_eng.bigc[n - 1].base + c_eng.bigc[n - 1].rem;
  const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint32_t c0 = blockIdx.x * per, c1 = min(c0 + per, total);
  if(c0 < c1)
  {
    uint32_t lo = 0, hi = n - 1;                   // last copy with base <= c0
    while(lo < hi)
    {
      const uint32_t mid = (lo + hi + 1) / 2;
      if(c_eng.bigc[mid].base <= c0) lo = mid; else hi = mid - 1;
    }
    for(uint32_t d = lo; d < n; ++d)
    {
      const BigCopy b = c_eng.bigc[d];
      if(b.base >= c1) break;
      const uint32_t j0 = c0 > b.base ? c0 - b.base : 0u;       // b.base < c1 here
      const uint32_t j1 = min(c1 - b.base, b.rem);
      for(uint32_t j = j0 + threadIdx.x; j < j1; j += kBlock)
      {
        const uint32_t k = b.from + j;
        const uint32_t q = k - b.ncc;
        const uint4 r = k < b.ncc ? *reinterpret_cast<const uint4*>(b.c + k)
                      : *reinterpret_cast<const uint4*>(b.p + (b.perm ? (uint32_t)(b.perm[q] & 0xFFFFFull) : q));
        *reinterpret_cast<uint4*>(b.dst + j) = r;
      }
    }
  }
}

// ===========================================================================
// Host side
// ===========================================================================

namespace {

constexpr uint32_t kChunk = 16;          // steps between quiescence readbacks
constexpr uint32_t kPendSlots = 4096;    // pend[] entries
constexpr uint32_t kPendPre = kPendSlots - 1;

struct HostType {
  bool registered = false, created = false;
  uint32_t words = 0, ht = 0, batch = 0, cap = 0;
  uint64_t params[GPU_ACTOR_MAX_PARAMS] = {};
  uint64_t first = 0, count = 0;
  uint32_t lfirst = 0, lcount = 0;
  uint64_t reserve = 0;                 // ids for actors spawned by behaviours
  int32_t priority = 0;                 // the fork's _priority() hint
  uint64_t* d_state = nullptr;
  uint64_t* d_prog = nullptr;           // GPU_ACTOR_HT_PROGRAM: the behaviours' program
  uint32_t prog_n = 0;
  bool prog_yields = false;             // it holds a YIELD or a SPAWN: the small-step path leaves it
  std::vector<uint64_t> prog_host;      // the program's words (the run-time compiled step, jit_host.h)
};

struct Engine {
  std::mutex mu;
  // asynchronous run (gpu_actor_run_async): one progress thread at a time;
  // wmu guards the thread object (joined or detached by whoever reaps it)
  std::mutex wmu;
  std::thread worker;
  // progress threads that chained a run from their own completion callback:
  // they cannot join themselves; gpu_actor_shutdown joins them
  std::vector<std::thread> detached;
  std::atomic<bool> async_busy{false};   // read without the lock
  std::atomic<bool> async_started{false};  // the progress thread holds mu
  int async_rc = 0;
  uint64_t async_steps = 0;
  bool init = false;
  gpu_actor_config_t cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  HostType types[GPU_ACTOR_MAX_TYPES];
  uint32_t n_types = 0;                 // 1 + highest created type id
  uint64_t n_actors = 0;                // global ids handed out
  uint32_t n_local = 0;
  // zones
  uint32_t n_zones = 0;
  uint64_t zone_records = 0;
  uint64_t* d_zoff = nullptr;
  uint32_t* d_zcap = nullptr;
  ZRec* d_land[2] = {nullptr, nullptr};
  ZRec* d_carry[2] = {nullptr, nullptr};
  uint32_t* d_land_n[2] = {nullptr, nullptr};
  uint32_t* d_carry_n[2] = {nullptr, nullptr};
  ZRec* d_S = nullptr;
  ORec* d_O = nullptr;
  uint32_t par = 0;                     // parity the next step reads
  unsigned long long* d_stats = nullptr;
  unsigned long long* d_pend = nullptr;
  unsigned long long* d_pend_sh = nullptr;    // [kPendSlots][kShards]: k_step's adds
  unsigned long long* d_stats_sh = nullptr;   // [ST_COUNT][kShards]
  // hot zones (hot_dev.h k_hot): one allocation, carved into EngDev's arrays
  uint32_t* d_hot = nullptr;
  bool hot_on = false;
  unsigned long long* d_dbg = nullptr;   // phase stamps of the diagnostic build
  gpu_msg_t* h_msgs = nullptr; uint64_t h_msgs_cap = 0;
  // gpu_actor_send appends here; flushed (one H2D + k_inject) before the
  // next operation that observes device state, so a send costs no sync
  std::vector<gpu_msg_t> deferred;
  gpu_msg_t* d_msgs = nullptr; uint64_t d_msgs_cap = 0;
  uint64_t host_seq = 0;
  uint64_t steps_total = 0;
  int sticky = 0;
  // behaviours as programs compiled at run time (jit_host.h): the module of
  // the current program set and geometry, the set a build failed for (kept
  // on the interpreter), the constants last uploaded (for a module loaded
  // later), and how many modules were built or loaded
  jit::Module jit;
  uint64_t jit_set = 0;                 // the program set (and geometry) the module is for
  uint64_t jit_failed = 0;
  uint32_t jit_builds = 0;
  bool jit_used = false;                // the last step ran the compiled module
  TypeDev td_host[GPU_ACTOR_MAX_TYPES];
  EngDev eng_host;
  bool consts_host = false;
  // GUPS streamers' chunks for k_gups_apply (EngDev::gups_*; gups_type -1: none)
  uint64_t* d_gups_list = nullptr;
  unsigned int* d_gups_n = nullptr;
  uint64_t* d_gups_jump = nullptr;
  unsigned long long* d_gups_stat = nullptr;
  uint64_t gups_jump_host[65] = {};
  uint32_t gups_cap = 0;
  int gups_type = -1;
  // One rank: device work that can change the spill status or the counters
  // bumps dev_epoch; a host read of either records the epoch it saw, so a
  // read that nothing could have changed since is skipped (run_fixed's and
  // gpu_actor_sync's host round trips, bench.py's timed region).
  uint64_t dev_epoch = 1, sstat_epoch = 0, sticky_epoch = 0;
  hipError_t last_hip = hipSuccess;
  std::vector<hipEvent_t> ev;
  double last_drain_ms = 0.0;
  // multi-rank exchange
  ncclComm_t comm = nullptr;
  XRec* d_xout = nullptr;
  XRec* d_xin = nullptr;
  unsigned long long* d_xc = nullptr;      // [2R + 2]: send counts, receive counts, scratch
  unsigned long long* d_xcount = nullptr;  // d_xc
  unsigned long long* d_xrecv = nullptr;   // d_xc + R
  unsigned long long* h_xc = nullptr;      // pinned mirror of d_xc
  unsigned int* d_spill_flag = nullptr;    // spill lists in use on any rank (summed)
  uint32_t xcap = 0;                       // records per peer segment of xout
  uint64_t xin_cap = 0;                    // records d_xin (and h_xin) hold
  XSpillRec* d_xspill = nullptr;           // cross-rank records past xcap
  unsigned int* d_xspill_n = nullptr;
  uint32_t xspill_cap = 0;
  std::vector<unsigned long long> h_xcount, h_xrecv;   // host transport
  uint64_t remote_total = 0;
  // peer writes (PONYC_AMD_PEER_WRITE=1, EngDev::peer_write): this rank's
  // inbox [R][xcap] (segment p: peer p's records, stored by peer p's k_step),
  // every peer's inbox mapped over IPC, and a small collective scratch
  bool peer_write = false;
  XRec* d_pin = nullptr;
  XRec* peer_ptr[kMaxRanks] = {};
  unsigned long long* d_hx = nullptr;      // [1 + R]
  // host transport (gpu_actor_set_transport)
  gpu_actor_alltoallv_fn xp_a2a = nullptr;
  gpu_actor_allreduce_fn xp_ar = nullptr;
  void* xp_ctx = nullptr;
  // host transport staging (pinned): what this rank sends, what it receives
  uint8_t* h_sbuf = nullptr;
  uint8_t* h_rbuf = nullptr;
  uint64_t h_sbuf_cap = 0, h_rbuf_cap = 0;
  // spawned actors (gpu_actor_type_reserve)
  uint32_t spawn_cap = 0;
  uint64_t *d_skey[2] = {nullptr, nullptr}, *d_sarg[2] = {nullptr, nullptr};
  unsigned int* d_spawn_n = nullptr;
  uint32_t *d_tstart = nullptr, *d_tcnt = nullptr;
  unsigned long long* d_live = nullptr;  // [GPU_ACTOR_MAX_TYPES] live actors per type
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  // records past zone capacity: spill lists, their counters, and the minimum
  // capacity each zone has grown to
  struct SpillStat {
    unsigned int spill_n[2];
    unsigned int halt;
    unsigned int pad;
    unsigned long long skipped;
  };
  // backpressure: trigger bytes per global id and parity
  // (d_trig_own: this rank's own bytes when n_ranks > 1, merged into d_trig),
  // the receiver each muted local actor waits on, per-zone trigger counts,
  // per-step counts (index = step mod 3), and the step index
  uint8_t* d_trig[2] = {nullptr, nullptr};
  uint8_t* d_trig_own[2] = {nullptr, nullptr};
  uint64_t trig_bytes = 0;
  bool trig_stale[2] = {false, false};
  uint32_t* d_muted_on = nullptr;
  uint64_t muted_on_cap = 0;
  uint32_t* d_ztrig[2] = {nullptr, nullptr};
  unsigned int* d_trig_n = nullptr;
  // zones the step's two-pass launch ran (EngDev::zplan); split_plan: run a
  // two-pass table's step as the two launches (PONYC_AMD_SPLIT_PLAN=0: one)
  uint32_t* d_zplan = nullptr;
  bool split_plan = true;
  // split tables: the step as one launch (k_step PM 3: the rest through a
  // call) instead of two (PONYC_AMD_FUSE=0: two)
  bool fuse = true;
  uint32_t sidx = 0;
  // backlog copies handed to k_carry_big (EngDev::bigc)
  BigCopy* d_bigc = nullptr;
  unsigned long long* d_bigc_n = nullptr;
  bool defer_big = false;
  SpillRec* d_spill[2] = {nullptr, nullptr};
  uint32_t spill_cap = 0;
  SpillStat* d_sstat = nullptr;
  SpillStat* h_sstat = nullptr;           // pinned
  uint32_t* d_need = nullptr;
  std::vector<uint32_t> zcap_min, zcap_host;
  uint64_t fixups = 0;
  // small-step path (k_sparse)
  SparseCtl* d_ctl = nullptr;
  SparseCtl* h_ctl = nullptr;             // pinned
  uint64_t sparse_launches = 0, sparse_steps = 0;
  // zone geometry: actors per zone = 1 << zbits (step_entry.h; chosen by
  // relayout_zones)
  uint32_t zbits = kZoneBits;
};

Engine g;

#define HIPCK(expr)                                                    \
  do {                                                                 \
    hipError_t e_ = (expr);                                            \
    if(e_ != hipSuccess) {                                             \
      g.last_hip = e_;                                                 \
      fprintf(stderr, "gpu_actor: %s failed: %s (%s:%d)\n", #expr,     \
        hipGetErrorString(e_), __FILE__, __LINE__);                    \
      return GPU_ACTOR_EHIP;                                           \
    }                                                                  \
  } while(0)

#define NCCLCK(expr)                                                   \
  do {                                                                 \
    ncclResult_t r_ = (expr);                                          \
    if(r_ != ncclSuccess) {                                            \
      fprintf(stderr, "gpu_actor: %s failed: %s\n", #expr,            \
        ncclGetErrorString(r_));                                       \
      return GPU_ACTOR_ECOMM;                                          \
    }                                                                  \
  } while(0)

inline uint32_t R() { return g.cfg.n_ranks; }
inline uint32_t rank() { return g.cfg.rank; }

// number of ids < x owned by this rank
inline uint64_t owned_below(uint64_t x)
{
  return x > rank() ? (x - rank() + R() - 1) / R() : 0;
}

inline uint32_t blocks_for(uint64_t n, uint32_t bs = kBlock) { return (uint32_t)((n + bs - 1) / bs); }

// actors per zone in this engine's geometry
inline uint32_t zone_actors() { return 1u << g.zbits; }

inline bool reducible_ht(uint32_t ht)
{
  return ht == GPU_ACTOR_HT_FANIN_ANALYZER || ht == GPU_ACTOR_HT_GUPS_UPDATER;
}

const std::vector<StepEntry>& step_entries()
{
  static const std::vector<StepEntry> v = {
    gpa::step_entry_any(), gpa::step_entry_ring(), gpa::step_entry_pinger(),
    gpa::step_entry_pinger_det(), gpa::step_entry_fanin_sender(),
    gpa::step_entry_gups_streamer(), gpa::step_entry_storm(), gpa::step_entry_spreader(),
    gpa_z12::step_entry_any(), gpa_z12::step_entry_ring(), gpa_z12::step_entry_pinger(),
    gpa_z12::step_entry_pinger_det(), gpa_z12::step_entry_fanin_sender(),
    gpa_z12::step_entry_gups_streamer(), gpa_z12::step_entry_storm(),
    gpa_z12::step_entry_spreader(), gpa::step_entry_fifo_pair(), gpa_z12::step_entry_fifo_pair(),
    gpa::step_entry_program(), gpa_z12::step_entry_program()};
  return v;
}

// Backlog copies go to k_carry_big (the whole GPU copies them right after
// k_step) in engines whose serial actors run more than one handler table —
// the fan-in shapes (sources and sinks of different kinds) that build
// backlogs of thousands of records per actor. The extra launch per step costs
// 2.4 % of a C2-det step and 1 % of a C5 step (profiles/r04j_hot_msd.txt,
// PONYC_AMD_DEFER_BIG=0/1), where backlogs over 128 records are rare and a
// zone copies one itself. PONYC_AMD_DEFER_BIG=0/1 forces it (tests, A/B).
bool defer_big_wanted()
{
  if(const char* f = getenv("PONYC_AMD_DEFER_BIG")) return atoi(f) != 0;
  int only = -1;
  for(const HostType& t : g.types)
  {
    if(!t.created || reducible_ht(t.ht)) continue;
    if(only >= 0 && (uint32_t)only != t.ht) return true;
    only = (int)t.ht;
  }
  return false;
}

StepEntry pick_step_entry();

// The hot-zone scratch words (hot_dev.h), in the order upload_types hands
// them to the device; hot_bar_words() is the grid barrier's [0] arrivals, [1]
// finished workgroups, [2] missed phases, [3] zones given back after a miss.
inline size_t hot_words_before_bar()
{
  return 2 * (size_t)kMaxZones + (size_t)kMaxHot * kHotActors + (size_t)kMaxHot * 3 * kHotActors +
         3 * (size_t)kHotBins + kHotActors;
}
inline uint32_t* hot_bar_words() { return g.d_hot + hot_words_before_bar(); }

// k_hot's workgroups must all be resident at once (its phases meet at grid
// barriers, hot_dev.h): kHotBlocks workgroups of kHotThreads with the LDS of
// the larger zone geometry, against the occupancy the runtime reports for
// this device (one workgroup per CU on half the CUs is what it needs; the
// reported figure can exceed the hardware's by one workgroup per CU,
// MI355X_MICROARCH.md, so one is taken off). Asked once per engine.
bool hot_resident()
{
  static int cached = -1;
  if(cached >= 0) return cached != 0;
  int per_cu = 0, cus = 0;
  const size_t lds = 5u * kHotActors * sizeof(uint32_t);
  if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_hot),
       (int)kHotThreads, lds) != hipSuccess ||
     hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g.device) != hipSuccess)
  {
    (void)hipGetLastError();
    cached = 0;
    return false;
  }
  cached = (uint64_t)std::max(per_cu - 1, per_cu > 0 ? 1 : 0) * (uint64_t)cus >= kHotBlocks ? 1 : 0;
  return cached != 0;
}

constexpr uint32_t kGupsBlocks = 1024;
__global__ void __launch_bounds__(256) k_gups_apply();

// The GUPS streamer type whose chunks k_gups_apply makes (EngDev::gups_*): the
// first with a nonzero chunk, on one rank (PONYC_AMD_GUPS_DEFER=0: none, every
// streamer applies its own chunk, for A/B runs). Chunks of L >= 16 updates per
// lane, at most 64 lanes per chunk.
int gups_setup(EngDev& e)
{
  g.gups_type = -1;
  e.gups_type = -1;
  const char* f = getenv("PONYC_AMD_GUPS_DEFER");
  if(R() != 1 || (f && atoi(f) == 0)) return 0;
  int t_def = -1;
  for(uint32_t t = 0; t < GPU_ACTOR_MAX_TYPES && t_def < 0; ++t)
    if(g.types[t].created && g.types[t].ht == GPU_ACTOR_HT_GUPS_STREAMER && g.types[t].params[0] > 0 &&
       g.types[t].params[0] <= 0xFFFFFFFFull)
      t_def = (int)t;
  if(t_def < 0) return 0;
  const HostType& h = g.types[t_def];
  const uint64_t chunk = h.params[0];
  const uint64_t L = std::max<uint64_t>(16, (chunk + 63) / 64);
  const uint64_t parts = (chunk + L - 1) / L;
  // kGupsShards segments, each at least 2^16 chunks (k_sparse lists from its
  // few waves' segments only)
  const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(1ull << 22, 2ull * h.lcount), 1ull << 28);
  if(cap > g.gups_cap)
  {
    HIPCK(hipStreamSynchronize(g.stream));      // no k_gups_apply still reads the old list
    if(g.d_gups_list) HIPCK(hipFree(g.d_gups_list));
    g.d_gups_list = nullptr;
    g.gups_cap = 0;
    HIPCK(hipMalloc(&g.d_gups_list, cap * sizeof(uint64_t)));
    g.gups_cap = (uint32_t)cap;
  }
  if(!g.d_gups_n)
  {
    HIPCK(hipMalloc(&g.d_gups_n, (kGupsShards + 1) * sizeof(unsigned int)));
    HIPCK(hipMemsetAsync(g.d_gups_n, 0, (kGupsShards + 1) * sizeof(unsigned int), g.stream));
    HIPCK(hipMalloc(&g.d_gups_jump, 65 * sizeof(uint64_t)));
    HIPCK(hipMalloc(&g.d_gups_stat, 2 * kGupsBlocks * sizeof(unsigned long long)));
    HIPCK(hipMemsetAsync(g.d_gups_stat, 0, 2 * kGupsBlocks * sizeof(unsigned long long), g.stream));
  }
  uint64_t jump[65] = {};
  for(uint64_t p = 0; p < parts; ++p) jump[p] = gpa::polyrand_xpow(p * L);
  jump[parts] = gpa::polyrand_xpow(chunk);
  if(memcmp(jump, g.gups_jump_host, sizeof(jump)) != 0)
  {
    HIPCK(hipStreamSynchronize(g.stream));      // no launch still reads the old table
    memcpy(g.gups_jump_host, jump, sizeof(jump));
    HIPCK(hipMemcpyAsync(g.d_gups_jump, g.gups_jump_host, sizeof(jump), hipMemcpyHostToDevice,
      g.stream));
  }
  e.gups_list = g.d_gups_list; e.gups_n = g.d_gups_n; e.gups_jump = g.d_gups_jump;
  e.gups_stat = g.d_gups_stat;
  e.gups_seg = g.gups_cap / kGupsShards;
  {
    // (tests: PONYC_AMD_GUPS_SEG=n lists at most n chunks per segment, so that
    // full segments send the rest through the streamers' own path)
    const char* sg = getenv("PONYC_AMD_GUPS_SEG");
    if(sg && atoi(sg) > 0) e.gups_seg = std::min<uint32_t>(e.gups_seg, (uint32_t)atoi(sg));
  }
  e.gups_l = (uint32_t)L; e.gups_parts = (uint32_t)parts;
  e.gups_type = t_def;
  g.gups_type = t_def;
  return 0;
}

// k_gups_apply behind a step's kernels (engines with a chunk-listing streamer
// type); the events, when given, end at its end
int gups_apply_launch(hipEvent_t e1)
{
  if(g.gups_type < 0) return 0;
  if(e1)
    hipExtLaunchKernelGGL(k_gups_apply, dim3(kGupsBlocks), dim3(256), 0, g.stream, nullptr, e1, 0u);
  else
    hipLaunchKernelGGL(k_gups_apply, dim3(kGupsBlocks), dim3(256), 0, g.stream);
  HIPCK(hipGetLastError());
  return 0;
}

int upload_types()
{
  TypeDev td[GPU_ACTOR_MAX_TYPES];
  memset(td, 0, sizeof(td));
  for(uint32_t t = 0; t < GPU_ACTOR_MAX_TYPES; ++t)
  {
    const HostType& h = g.types[t];
    TypeDev& d = td[t];
    if(!h.created) continue;
    d.first = (uint32_t)h.first; d.count = (uint32_t)h.count;
    d.lfirst = h.lfirst; d.lcount = h.lcount;
    d.ht = h.ht; d.words = h.words; d.batch = h.batch; d.cap = h.cap;
    d.reducible = reducible_ht(h.ht);
    d.prio = h.priority > 0 ? 1u : 0u;
    d.state = h.d_state;
    memcpy(d.params, h.params, sizeof(d.params));
    d.prog = h.d_prog;
    d.prog_n = h.prog_n;
    d.prog_pad = h.prog_yields ? 1u : 0u;
  }
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_types), td, sizeof(td), 0,
    hipMemcpyHostToDevice, g.stream));
  EngDev e;
  memset(&e, 0, sizeof(e));
  e.n_types = g.n_types; e.rank = rank(); e.nranks = R(); e.n_local = g.n_local;
  e.n_zones = g.n_zones; e.zoff = g.d_zoff; e.zcapz = g.d_zcap;
  e.n_ids = (uint32_t)std::min<uint64_t>(g.n_actors, 0xFFFFFFFFull);
  e.r_magic = R() > 1 ? ~0ull / R() + 1 : 0;
  for(int p = 0; p < 2; ++p)
  {
    e.land[p] = g.d_land[p]; e.carry[p] = g.d_carry[p];
    e.land_n[p] = g.d_land_n[p]; e.carry_n[p] = g.d_carry_n[p];
  }
  e.S = g.d_S; e.O = g.d_O;
  e.stats = g.d_stats; e.pend = g.d_pend;
  e.pend_sh = g.d_pend_sh; e.stats_sh = g.d_stats_sh;
  {
    uint32_t* h = g.d_hot;
    e.hot_prep = h; h += kMaxZones;
    e.hot_slot = h; h += kMaxZones;
    e.hot_cnt = h; h += kMaxHot * kHotActors;
    e.hot_aux = h; h += kMaxHot * 3 * kHotActors;
    e.hot_hist = h; h += kHotBins;
    e.hot_bcnt = h; h += kHotBins;
    e.hot_cur = h; h += kHotBins + kHotActors;
    e.hot_bar = h;
  }
  e.xout = g.d_xout; e.xcount = g.d_xcount; e.xcap = g.xcap;
  e.peer_write = g.peer_write ? 1u : 0u;
  for(uint32_t p = 0; p < R() && p < kMaxRanks; ++p)
    e.xdst[p] = g.peer_write ? (g.peer_ptr[p] ? g.peer_ptr[p] + (size_t)rank() * g.xcap : nullptr)
                             : (g.d_xout ? g.d_xout + (size_t)p * g.xcap : nullptr);
  e.seq_max = R() > 1 ? kXSeqMax : kSeqMax;
  e.dbg = g.d_dbg;
  e.spawn_key = g.d_skey[0]; e.spawn_arg = g.d_sarg[0];
  e.spawn_n = g.d_spawn_n; e.spawn_cap = g.spawn_cap;
  for(int p = 0; p < 2; ++p)
  {
    e.trig[p] = g.d_trig[p];
    e.trig_own[p] = R() > 1 ? g.d_trig_own[p] : g.d_trig[p];
    e.ztrig[p] = g.d_ztrig[p];
  }
  e.muted_on = g.d_muted_on;
  e.spill_flag = g.d_spill_flag;
  e.trig_n = g.d_trig_n;
  e.spill[0] = g.d_spill[0]; e.spill[1] = g.d_spill[1];
  e.spill_n = g.d_sstat ? g.d_sstat->spill_n : nullptr;
  e.halt = g.d_sstat ? &g.d_sstat->halt : nullptr;
  e.skipped = g.d_sstat ? &g.d_sstat->skipped : nullptr;
  e.spill_cap = g.spill_cap;
  e.xspill = g.d_xspill; e.xspill_n = g.d_xspill_n; e.xspill_cap = g.xspill_cap;
  e.zbits = g.zbits;
  g.defer_big = defer_big_wanted();
  // k_hot runs where backlogs build (the same engines as defer_big);
  // PONYC_AMD_HOT=0/1 forces it (tests, A/B)
  // It runs only where its grid is resident at once (hot_resident): its
  // phases meet at grid barriers.
  {
    const char* f = getenv("PONYC_AMD_HOT");
    g.hot_on = pick_step_entry().hot && (f ? atoi(f) != 0 : g.defer_big) && hot_resident();
    e.hot_on = g.hot_on ? 1u : 0u;
    const char* t = getenv("PONYC_AMD_HOT_TEST");
    e.hot_test = (t && atoi(t) != 0) ? 1u : 0u;
  }
  e.bigc = g.d_bigc; e.bigc_n = g.d_bigc_n; e.bigc_cap = kBigCopyCap;
  e.defer_big = g.defer_big ? 1u : 0u;
  {
    const char* f = getenv("PONYC_AMD_TWO_PASS");
    e.two_pass = (f && atoi(f) == 0) ? 0u : 1u;
    const char* sp = getenv("PONYC_AMD_SPLIT_PLAN");
    g.split_plan = !(sp && atoi(sp) == 0);
    const char* fu = getenv("PONYC_AMD_FUSE");
    g.fuse = !(fu && atoi(fu) == 0);
  }
  e.zplan = g.d_zplan;
  {
    const int rc = gups_setup(e);
    if(rc) return rc;
  }
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_eng), &e, sizeof(e), 0,
    hipMemcpyHostToDevice, g.stream));
  // every k_step code object holds its own copy of the constants
  for(const StepEntry& se : step_entries())
    HIPCK(se.upload(td, &e, g.stream));
  memcpy(g.td_host, td, sizeof(td));
  g.eng_host = e;
  g.consts_host = true;
  if(g.jit.mod)
  {
    HIPCK(hipMemcpyHtoDAsync(g.jit.types, g.td_host, sizeof(g.td_host), g.stream));
    HIPCK(hipMemcpyHtoDAsync(g.jit.eng, &g.eng_host, sizeof(g.eng_host), g.stream));
  }
  return 0;
}

// Spill lists of at least `cap` records per parity (they start empty between
// steps, so growing them moves nothing).
int ensure_spill(uint64_t cap)
{
  cap = std::min<uint64_t>(cap, 0x7FFFFFFFull);
  if(cap <= g.spill_cap) return 0;
  for(int p = 0; p < 2; ++p)
  {
    if(g.d_spill[p]) HIPCK(hipFree(g.d_spill[p]));
    g.d_spill[p] = nullptr;
    HIPCK(hipMalloc(&g.d_spill[p], cap * sizeof(SpillRec)));
  }
  g.spill_cap = (uint32_t)cap;
  return 0;
}

int relayout_zones(bool geometry = false);
StepEntry step_entry_for(bool z12);
bool step_fits(const StepEntry& se, uint64_t nb);
int upload_types();
int pend_read(uint32_t first, uint32_t n, std::vector<unsigned long long>& out);

// Spill list length for the current zone layout: a quarter of its records.
inline uint64_t spill_cap_for_zones()
{
  return std::max<uint64_t>(1u << 20, g.zone_records / 4);
}

int read_sstat()
{
  HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  g.sstat_epoch = g.dev_epoch;
  return 0;
}

inline bool spill_pending()
{
  return g.h_sstat->spill_n[0] || g.h_sstat->spill_n[1] || g.h_sstat->halt;
}

// Grow every zone that spilled, land the spilled records at the positions
// they were given, and release the halt (SpillRec, engine_dev.h). Uses the
// status last read into h_sstat. Nothing is dropped unless a spill list
// itself overflowed (counted; the run then fails with GPU_ACTOR_EMAILBOX).
// With n_ranks > 1 every rank calls it together (the decision is summed over
// ranks: settle_spills, run_locked) and it always clears the spill flag, even
// with nothing of its own to land, so that every rank's next step runs alike.
int fixup_spill()
{
  const Engine::SpillStat st = *g.h_sstat;
  g.dev_epoch++;
  if(R() == 1 && !st.spill_n[0] && !st.spill_n[1] && !st.halt) return 0;
  uint32_t n[2], most = 0;
  for(int p = 0; p < 2; ++p)
  {
    n[p] = std::min(st.spill_n[p], g.spill_cap);
    most = std::max(most, st.spill_n[p]);
  }
  if(n[0] || n[1])
  {
    const uint32_t nz = g.n_zones;
    HIPCK(hipMemsetAsync(g.d_need, 0, nz * sizeof(uint32_t), g.stream));
    for(int p = 0; p < 2; ++p)
      if(n[p])
        hipLaunchKernelGGL(k_spill_need, dim3(blocks_for(n[p])), dim3(kBlock), 0, g.stream,
          (const SpillRec*)g.d_spill[p], n[p], g.d_need);
    HIPCK(hipGetLastError());
    std::vector<uint32_t> need(nz);
    HIPCK(hipMemcpyAsync(need.data(), g.d_need, nz * sizeof(uint32_t), hipMemcpyDeviceToHost,
      g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    bool grow = false;
    for(uint32_t z = 0; z < nz; ++z)
      if(need[z] > g.zcap_host[z])
      {
        // double, or 1.5x what this step needed: a burst seldom grows a zone twice
        const uint64_t want = std::max<uint64_t>(2ull * g.zcap_host[z], need[z] + need[z] / 2);
        g.zcap_min[z] = (uint32_t)std::min<uint64_t>((want + 15) & ~15ull, kSpillPosMask);
        grow = true;
      }
    if(grow)
    {
      int rc = relayout_zones();
      if(rc) return rc;
      rc = upload_types();
      if(rc) return rc;
    }
    for(int p = 0; p < 2; ++p)
      if(n[p])
        hipLaunchKernelGGL(k_spill_place, dim3(blocks_for(n[p])), dim3(kBlock), 0, g.stream,
          (const SpillRec*)g.d_spill[p], n[p], (uint32_t)p);
    HIPCK(hipGetLastError());
  }
  HIPCK(hipMemsetAsync(g.d_sstat, 0, sizeof(Engine::SpillStat), g.stream));
  HIPCK(hipMemsetAsync(g.d_spill_flag, 0, sizeof(unsigned int), g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  memset(g.h_sstat, 0, sizeof(Engine::SpillStat));
  g.fixups++;
  // Only now, with every spilled record placed, may the lists be re-sized
  // (ensure_spill drops their contents): to the grown zones' share, and
  // larger when a list overflowed (those records were counted as dropped).
  // Re-sizing them inside relayout_zones, before k_spill_place had read them,
  // lost every spilled record of a burst that grew the zones past 4 M records
  // (round 3's 2048-sink backlog gap).
  const uint64_t want = std::max<uint64_t>(spill_cap_for_zones(),
                                           most > g.spill_cap ? 2ull * most : 0ull);
  if(want > g.spill_cap)
  {
    const int rc = ensure_spill(want);
    if(rc) return rc;
    return upload_types();
  }
  return 0;
}

// Re-lay the zone buffers after actors were created: zone z holds
// Σ_{serial actors in z} cap(type) records. Capacities only grow, so mail
// already landed or carried is copied zone by zone into the new layout.
// The zone geometry for n local actors (step_entry.h): 2048-actor zones with
// two 512-thread workgroups per CU while the buckets are few; past ~640
// buckets their four LDS bucket arrays no longer leave room for two
// workgroups per CU, and 4096-actor zones (half the buckets, twice the run
// length per bucket, one 1024-thread workgroup per CU) are faster — C5's 8M
// actors: 2.20 -> 1.58 ms per step (profiles/r03_general.txt). Their LDS
// holds up to ~2300 buckets.
uint32_t pick_zone_bits(uint64_t n)
{
  const uint64_t rb = R() > 1 ? R() : 0;
  const uint64_t nz11 = (n + 2047) / 2048, nz12 = (n + 4095) / 4096;
  if(const char* f = getenv("PONYC_AMD_ZONE_BITS"))      // test hook: force a geometry
    return atoi(f) == 12 ? 12u : 11u;
  // 4096-actor zones while their bucket arrays fit the LDS beside the z12
  // kernels' static LDS (~2,200 buckets; ~1,500 for the two-pass table's six
  // arrays); past that, 2048-actor zones at one workgroup per CU
  return (nz11 + rb > 640 && step_fits(step_entry_for(true), nz12 + rb)) ? 12u : 11u;
}

// No mail anywhere (landing or carried, either parity): a geometry change
// then moves nothing.
bool zones_empty()
{
  if(g.n_zones == 0) return true;
  std::vector<uint32_t> v(g.n_zones);
  for(int p = 0; p < 2; ++p)
    for(uint32_t* src : {g.d_land_n[p], g.d_carry_n[p]})
    {
      if(hipMemcpy(v.data(), src, g.n_zones * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return false;
      for(uint32_t x : v)
        if(x) return false;
    }
  return true;
}

// geometry: the zone geometry may be re-chosen (gpu_actor_create only: every
// rank creates alike, so the collective below is reached by all of them; a
// spill fixup can run on one rank alone and keeps the geometry).
int relayout_zones(bool geometry)
{
  // the geometry may change only before any step ran, with no mail landed
  // (zone buffers are copied zone by zone below)
  // Every rank must pick the same geometry (the trigger-byte merge and the
  // bucket layout assume it), so the choice follows the largest rank's share,
  // ceil(n_actors / R), not this rank's own count, which can be one less; and
  // whether mail has landed anywhere is summed over ranks (create is called
  // by every rank alike, so this collective is reached by all of them).
  bool fresh = false;
  {
    const uint32_t want = pick_zone_bits((g.n_actors + R() - 1) / R());
    if(geometry && want != g.zbits && g.steps_total == 0 && g.sparse_launches == 0)
    {
      HIPCK(hipStreamSynchronize(g.stream));
      bool empty = zones_empty();
      if(R() > 1)
      {
        const unsigned long long mine = empty ? 0ull : 1ull;
        HIPCK(hipMemcpyAsync(g.d_pend + kPendPre, &mine, sizeof(mine), hipMemcpyHostToDevice,
          g.stream));
        std::vector<unsigned long long> pv;
        const int rc = pend_read(kPendPre, 1, pv);
        if(rc) return rc;
        empty = pv[0] == 0;
      }
      if(empty)
      {
        g.zbits = want;
        g.zcap_min.clear();
        fresh = true;
      }
    }
  }
  const uint32_t za = zone_actors();
  const uint32_t nz = (uint32_t)((g.n_local + za - 1) / za);
  if(nz > kMaxZones) return GPU_ACTOR_ERANGE;
  std::vector<uint64_t> cap64(nz, 0);
  for(const HostType& t : g.types)
  {
    if(!t.created || reducible_ht(t.ht)) continue;
    for(uint64_t L = t.lfirst; L < (uint64_t)t.lfirst + t.lcount; )
    {
      const uint64_t z = L / za;
      const uint64_t hi = std::min<uint64_t>((z + 1) * za, (uint64_t)t.lfirst + t.lcount);
      cap64[z] += (hi - L) * t.cap;
      L = hi;
    }
  }
  std::vector<uint32_t> cap(nz);
  std::vector<uint64_t> off(nz);
  uint64_t total = 0;
  if(g.zcap_min.size() < nz) g.zcap_min.resize(nz, 0);
  for(uint32_t z = 0; z < nz; ++z)
  {
    cap64[z] = std::max<uint64_t>(cap64[z], g.zcap_min[z]);
    if(cap64[z] > (uint64_t)kSpillPosMask) return GPU_ACTOR_ERANGE;
    cap[z] = (uint32_t)cap64[z];
    off[z] = total;
    total += (cap[z] + 15u) & ~15u;          // keep every zone 256-B aligned
  }
  const size_t bytes = std::max<uint64_t>(total, 16) * sizeof(ZRec);
  uint64_t* d_off = nullptr;
  uint32_t* d_cap = nullptr;
  HIPCK(hipMalloc(&d_off, std::max<size_t>(nz, 1) * sizeof(uint64_t)));
  HIPCK(hipMalloc(&d_cap, std::max<size_t>(nz, 1) * sizeof(uint32_t)));
  HIPCK(hipMemcpyAsync(d_off, off.data(), nz * sizeof(uint64_t), hipMemcpyHostToDevice, g.stream));
  HIPCK(hipMemcpyAsync(d_cap, cap.data(), nz * sizeof(uint32_t), hipMemcpyHostToDevice, g.stream));
  for(int p = 0; p < 2; ++p)
  {
    ZRec *land = nullptr, *carry = nullptr;
    uint32_t *ln = nullptr, *cn = nullptr;
    HIPCK(hipMalloc(&land, bytes));
    HIPCK(hipMalloc(&carry, bytes));
    HIPCK(hipMalloc(&ln, std::max<size_t>(nz, 1) * sizeof(uint32_t)));
    HIPCK(hipMalloc(&cn, std::max<size_t>(nz, 1) * sizeof(uint32_t)));
    HIPCK(hipMemsetAsync(ln, 0, std::max<size_t>(nz, 1) * sizeof(uint32_t), g.stream));
    HIPCK(hipMemsetAsync(cn, 0, std::max<size_t>(nz, 1) * sizeof(uint32_t), g.stream));
    if(g.n_zones && !fresh)
    {
      hipLaunchKernelGGL(k_zone_copy, dim3(g.n_zones), dim3(kBlock), 0, g.stream,
        (const ZRec*)g.d_land[p], g.d_zoff, g.d_zcap, land, (const uint64_t*)d_off);
      hipLaunchKernelGGL(k_zone_copy, dim3(g.n_zones), dim3(kBlock), 0, g.stream,
        (const ZRec*)g.d_carry[p], g.d_zoff, g.d_zcap, carry, (const uint64_t*)d_off);
      HIPCK(hipGetLastError());
      HIPCK(hipMemcpyAsync(ln, g.d_land_n[p], g.n_zones * sizeof(uint32_t),
        hipMemcpyDeviceToDevice, g.stream));
      HIPCK(hipMemcpyAsync(cn, g.d_carry_n[p], g.n_zones * sizeof(uint32_t),
        hipMemcpyDeviceToDevice, g.stream));
    }
    HIPCK(hipStreamSynchronize(g.stream));
    if(g.d_land[p]) HIPCK(hipFree(g.d_land[p]));
    if(g.d_carry[p]) HIPCK(hipFree(g.d_carry[p]));
    if(g.d_land_n[p]) HIPCK(hipFree(g.d_land_n[p]));
    if(g.d_carry_n[p]) HIPCK(hipFree(g.d_carry_n[p]));
    g.d_land[p] = land; g.d_carry[p] = carry; g.d_land_n[p] = ln; g.d_carry_n[p] = cn;
  }
  if(g.d_S) HIPCK(hipFree(g.d_S));
  if(g.d_O) HIPCK(hipFree(g.d_O));
  if(g.d_zoff) HIPCK(hipFree(g.d_zoff));
  if(g.d_zcap) HIPCK(hipFree(g.d_zcap));
  HIPCK(hipMalloc(&g.d_S, 3 * bytes));     // 2 x: records of a zone; 1 x: sort scratch
  HIPCK(hipMalloc(&g.d_O, std::max<uint64_t>(total, 16) * sizeof(ORec)));
  g.d_zoff = d_off;
  g.d_zcap = d_cap;
  g.zone_records = total;
  g.n_zones = nz;
  g.zcap_host = cap;
  // the receiver each muted actor waits on, one word per local slot
  const uint64_t slots = (uint64_t)nz * za;
  if(slots > g.muted_on_cap)
  {
    uint32_t* mo = nullptr;
    HIPCK(hipMalloc(&mo, slots * sizeof(uint32_t)));
    HIPCK(hipMemsetAsync(mo, 0, slots * sizeof(uint32_t), g.stream));
    if(g.d_muted_on)
    {
      HIPCK(hipMemcpyAsync(mo, g.d_muted_on, g.muted_on_cap * sizeof(uint32_t),
        hipMemcpyDeviceToDevice, g.stream));
      HIPCK(hipStreamSynchronize(g.stream));
      HIPCK(hipFree(g.d_muted_on));
    }
    g.d_muted_on = mo;
    g.muted_on_cap = slots;
  }
  // (the spill lists are re-sized by the callers, once nothing is left in
  // them: fixup_spill relays the zones while its spilled records wait there)
  return 0;
}

uint32_t required_words(uint32_t ht)
{
  switch(ht)
  {
    case GPU_ACTOR_HT_RING: return 4;
    case GPU_ACTOR_HT_PINGER: return 3;
    case GPU_ACTOR_HT_PINGER_DET: return 2;
    case GPU_ACTOR_HT_FANIN_SENDER: return 4;
    case GPU_ACTOR_HT_FANIN_ANALYZER: return 2;
    case GPU_ACTOR_HT_GUPS_STREAMER: return 2;
    case GPU_ACTOR_HT_GUPS_UPDATER: return 1;
    case GPU_ACTOR_HT_STORM: return 2;
    case GPU_ACTOR_HT_FIFO_SRC: return 3;
    case GPU_ACTOR_HT_FIFO_SINK: return 11;
    case GPU_ACTOR_HT_SPREADER: return 5;
    case GPU_ACTOR_HT_PROGRAM: return 8;
    default: return 0;
  }
}

// Sum the sharded per-step counters of k_step (EngDev::pend_sh / stats_sh)
// into pend[first, first + n) and stats[], and clear the shards. One block;
// stream-ordered behind the steps, so plain adds.
__global__ void __launch_bounds__(kBlock) k_fold(uint32_t first, uint32_t n)
{
  for(uint32_t s = first + threadIdx.x; s < first + n; s += kBlock)
  {
    unsigned long long* sh = c_eng.pend_sh + (size_t)s * kShards;
    unsigned long long v = 0;
    for(uint32_t k = 0; k < kShards; ++k) { v += sh[k]; sh[k] = 0; }
    if(v) c_eng.pend[s] += v;
  }
  for(uint32_t i = threadIdx.x; i < ST_COUNT; i += kBlock)
  {
    unsigned long long* sh = c_eng.stats_sh + (size_t)i * kShards;
    unsigned long long v = 0;
    for(uint32_t k = 0; k < kShards; ++k) { v += sh[k]; sh[k] = 0; }
    if(v) c_eng.stats[i] += v;
  }
}

// k_step's sharded counters folded into pend[first, first + n) and stats[]
// (n == 0: stats only), ahead of a host read of either.
int fold_counters(uint32_t first, uint32_t n)
{
  hipLaunchKernelGGL(k_fold, dim3(1), dim3(kBlock), 0, g.stream, first, n);
  HIPCK(hipGetLastError());
  return 0;
}

// Zero pend[first, first + n) and their shards.
int pend_clear(uint32_t first, uint32_t n)
{
  HIPCK(hipMemsetAsync(g.d_pend + first, 0, n * sizeof(unsigned long long), g.stream));
  HIPCK(hipMemsetAsync(g.d_pend_sh + (size_t)first * kShards, 0,
    (size_t)n * kShards * sizeof(unsigned long long), g.stream));
  return 0;
}

void sticky_from(const unsigned long long* st)
{
  if(st[ST_DROPPED] || st[ST_XCHG_OVERFLOW]) g.sticky = GPU_ACTOR_EMAILBOX;
  else if(st[ST_SEQ_OVERFLOW]) g.sticky = GPU_ACTOR_ERANGE;
}

int check_sticky()
{
  if(R() == 1 && g.sticky_epoch == g.dev_epoch) return g.sticky;   // nothing ran since
  unsigned long long st[ST_COUNT];
  {
    const int rc = fold_counters(0, 0);
    if(rc) return rc;
  }
  HIPCK(hipMemcpyAsync(st, g.d_stats, sizeof(st), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  g.sticky_epoch = g.dev_epoch;
  sticky_from(st);
  return g.sticky;
}

// Cross-rank exchange after a step (n_ranks > 1), with ONE synchronisation:
//   device: counts all-to-all, trigger count summed (RCCL), then one pinned
//   readback of send counts, receive counts, the trigger count, the exchange
//   spill count and the spill status; host: grow xout / xin if this step
//   needs more room (exchange_room: records past xcap were kept in the
//   exchange spill list and are placed now — nothing is dropped, as
//   messageq.c:31-59 drops nothing), then grouped ncclSend/ncclRecv of the
//   records over xGMI; device: k_xinject lands them; the trigger bytes are
//   merged when any actor triggers muting (or did last time on this parity);
//   a spill flag summed over ranks (k_spill_flag + allreduce, no readback)
//   lets every rank's next k_step halt alike when any zone overflowed.
// The host transport (gpu_actor_set_transport) does the same through its
// callbacks, with the records staged through pinned host memory.
__global__ void k_spill_flag(unsigned int* flag)
{
  *flag = c_eng.spill_n[0] + c_eng.spill_n[1];
}

// This rank's spill status as one number (zone spill lists, halt, and the
// summed flag of the last exchange): summed over ranks by pend_read, it is
// the same on every rank, so every rank decides alike whether to fix up.
// The GUPS streamers' chunks listed since the last launch (EngDev::gups_list,
// one rank): gups_parts lanes per chunk, 64 / gups_parts chunks per wave; lane
// p regenerates updates p * L + 1 .. (p + 1) * L of its chunk (L = gups_l)
// from state * x^(p * L) — one GF(2) product, PolyRand._seed's own jump
// (gups_basic/main.pony:182-216) — and XORs each into its updater's word
// (Updater.apply, main.pony:145-155). Per update instruction the wave combines
// the lanes that share the first (then the second) remaining lane's word into
// one atomic, and issues no atomic for an XOR of 0 (the identity: a stream
// _seed left at 0 repeats word 0 of updater 0). The last workgroup to finish
// empties the list.
__global__ void __launch_bounds__(256) k_gups_apply()
{
  // the segments' chunk counts, and their prefix: chunk e (in segment order)
  // is entry e - s_pre[s] of the segment s with s_pre[s] <= e < s_pre[s + 1]
  __shared__ uint32_t s_pre[kGupsShards + 1];
  if(threadIdx.x < kGupsShards)
  {
    uint32_t c = min(__atomic_load_n(&c_eng.gups_n[threadIdx.x], __ATOMIC_RELAXED), c_eng.gups_seg);
    for(int off = 1; off < (int)kGupsShards; off <<= 1)
    {
      const uint32_t o = __shfl_up(c, off);
      if((int)threadIdx.x >= off) c += o;
    }
    s_pre[threadIdx.x + 1] = c;
    if(threadIdx.x == 0) s_pre[0] = 0;
  }
  __syncthreads();
  const uint32_t n = s_pre[kGupsShards];
  const TypeDev& S = c_types[c_eng.gups_type];
  const uint64_t chunk = S.params[0], shift = S.params[1], mask = S.params[2];
  const uint32_t ubase = (uint32_t)S.params[3];
  const uint32_t L = c_eng.gups_l, parts = c_eng.gups_parts, per_wave = 64u / parts;
  const uint32_t lane = threadIdx.x & 63u, sub = lane / parts, p = lane - sub * parts;
  const uint64_t jump = c_eng.gups_jump[p];
  const uint64_t first = (uint64_t)p * L;
  const uint32_t cnt = first < chunk ? (uint32_t)min<uint64_t>(L, chunk - first) : 0u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  // the updater type last written (gups updaters are one type in practice)
  uint32_t u_first = 0, u_count = 0, u_lfirst = 0, u_lcount = 0;
  uint64_t* u_state = nullptr;
  uint64_t u_mask = 0;
  uint32_t made = 0, issued = 0;
  for(uint64_t e0 = wave * per_wave; e0 < n; e0 += waves * per_wave)
  {
    const uint64_t e = e0 + sub;
    const bool live = sub < per_wave && e < n;
    uint64_t v = 0;
    if(live)
    {
      uint32_t lo = 0, hi = kGupsShards;
      while(hi - lo > 1u)
      {
        const uint32_t mid = (lo + hi) >> 1;
        if(s_pre[mid] <= e) lo = mid; else hi = mid;
      }
      v = c_eng.gups_list[(size_t)lo * c_eng.gups_seg + (e - s_pre[lo])];
    }
    if(live && p) v = polyrand_mulmod(v, jump);
    for(uint32_t j = 0; j < L; ++j)
    {
      unsigned long long* w = nullptr;
      if(live && j < cnt)
      {
        (void)polyrand_next(v);
        ++made;
        const uint32_t to = ubase + (uint32_t)((v >> shift) & mask);
        if(to - u_first >= u_count)
        {
          const int t = type_of_global(to);
          if(t >= 0)
          {
            const TypeDev& U = c_types[t];
            u_first = U.first; u_count = U.count; u_lfirst = U.lfirst; u_lcount = U.lcount;
            u_state = U.state; u_mask = U.params[0] - 1;
          }
        }
        if(to - u_first < u_count)
          w = reinterpret_cast<unsigned long long*>(&u_state[(v & u_mask) * u_lcount + (to - u_lfirst)]);
      }
      // the wave's update instruction: up to two combined words, then the rest
      const uint64_t wa = reinterpret_cast<uint64_t>(w);
      uint64_t left = __ballot(w != nullptr);
      for(int round = 0; round < 2 && left; ++round)
      {
        const uint32_t lead = (uint32_t)__ffsll((long long)left) - 1u;
        const uint64_t lw = __shfl(wa, (int)lead);
        const uint64_t peers = __ballot(((left >> lane) & 1ull) && wa == lw);
        uint64_t r = ((peers >> lane) & 1ull) ? v : 0ull;
        if(__popcll(peers) > 1)
          for(int off = 32; off; off >>= 1) r ^= __shfl_xor(r, off);
        if(lane == lead && r != 0)
        {
          atomicXor(w, (unsigned long long)r);
          ++issued;
        }
        left &= ~peers;
      }
      if(((left >> lane) & 1ull) && v != 0)
      {
        atomicXor(w, (unsigned long long)v);
        ++issued;
      }
    }
  }
  // per workgroup: updates made, atomics issued (each slot written by its own
  // workgroup only, summed by the host)
  __shared__ uint32_t s_sum[2];
  if(threadIdx.x < 2) s_sum[threadIdx.x] = 0;
  __syncthreads();
  if(made) atomicAdd(&s_sum[0], made);
  if(issued) atomicAdd(&s_sum[1], issued);
  __syncthreads();
  if(threadIdx.x == 0)
  {
    c_eng.gups_stat[blockIdx.x] += s_sum[0];
    c_eng.gups_stat[kGupsBlocks + blockIdx.x] += s_sum[1];
    __threadfence();
    const unsigned int done = atomicAdd(&c_eng.gups_n[kGupsShards], 1u);
    if(done == gridDim.x - 1u)
      for(uint32_t s = 0; s <= kGupsShards; ++s) atomicExch(&c_eng.gups_n[s], 0u);
  }
}

__global__ void k_spill_local(unsigned long long* out)
{
  *out = (unsigned long long)c_eng.spill_n[0] + c_eng.spill_n[1] + *c_eng.halt +
         (c_eng.nranks > 1 ? *c_eng.spill_flag : 0u);
}

// Only when the exchange spill list itself overflowed (records were lost and
// counted): send what xout holds, and count the kept spill records as lost too.
__global__ void k_xprep()
{
  const unsigned int xs = *c_eng.xspill_n;
  if(xs <= c_eng.xspill_cap) return;
  const uint32_t p = threadIdx.x;
  if(p < c_eng.nranks)
    c_eng.xcount[p] = min(c_eng.xcount[p], (unsigned long long)c_eng.xcap);
  if(p == 0) atomicAdd(&c_eng.stats[ST_XCHG_OVERFLOW], (unsigned long long)c_eng.xspill_cap);
}

__global__ void __launch_bounds__(kBlock) k_xspill_place(uint32_t n)
{
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  const XSpillRec r = c_eng.xspill[i];
  xrec_put(c_eng.xdst[r.peer] + r.pos, r.rec);
}

int alloc_xspill(uint32_t cap)
{
  if(g.d_xspill) HIPCK(hipFree(g.d_xspill));
  g.d_xspill = nullptr;
  HIPCK(hipMalloc(&g.d_xspill, (size_t)cap * sizeof(XSpillRec)));
  g.xspill_cap = cap;
  return 0;
}

// Room for this step's exchange: max_send records to one peer, total_recv
// records from all peers, xs records kept in the exchange spill list. xout's
// peer segments grow (kept records are copied to the new stride) and the
// spilled records go to their reserved positions; xin grows. Local decisions
// only: each side sizes its own buffers.
int peer_room(uint64_t max_send, uint64_t xs);
int exchange_room(uint64_t max_send, uint64_t total_recv, uint64_t xs)
{
  if(g.peer_write) return peer_room(max_send, xs);
  const bool lost = xs > g.xspill_cap;     // k_xprep clipped the counts to xcap
  if(max_send > g.xcap || lost)
  {
    uint64_t cap = std::max<uint64_t>(2ull * g.xcap, max_send + max_send / 2);
    cap = std::min<uint64_t>((cap + 63) & ~63ull, 0x40000000ull);
    XRec* nx = nullptr;
    HIPCK(hipMalloc(&nx, (size_t)R() * cap * sizeof(XRec)));
    HIPCK(hipMemcpy2DAsync(nx, cap * sizeof(XRec), g.d_xout, (size_t)g.xcap * sizeof(XRec),
      (size_t)g.xcap * sizeof(XRec), R(), hipMemcpyDeviceToDevice, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    HIPCK(hipFree(g.d_xout));
    g.d_xout = nx;
    g.xcap = (uint32_t)cap;
    const int rc = upload_types();
    if(rc) return rc;
  }
  if(xs)
  {
    if(!lost)
    {
      hipLaunchKernelGGL(k_xspill_place, dim3(blocks_for(xs)), dim3(kBlock), 0, g.stream,
        (uint32_t)xs);
      HIPCK(hipGetLastError());
    }
    HIPCK(hipMemsetAsync(g.d_xspill_n, 0, sizeof(unsigned int), g.stream));
    if(xs > g.xspill_cap / 2)
    {
      // a burst this large may come again: keep room for twice as much
      HIPCK(hipStreamSynchronize(g.stream));
      const int rc = alloc_xspill((uint32_t)std::min<uint64_t>(4ull * std::max<uint64_t>(xs,
        g.xspill_cap), 1ull << 27));
      if(rc) return rc;
      const int rc2 = upload_types();
      if(rc2) return rc2;
    }
  }
  if(total_recv > g.xin_cap)
  {
    const uint64_t cap = std::max<uint64_t>(2ull * g.xin_cap, total_recv + total_recv / 2);
    HIPCK(hipStreamSynchronize(g.stream));
    HIPCK(hipFree(g.d_xin));
    g.d_xin = nullptr;
    HIPCK(hipMalloc(&g.d_xin, cap * sizeof(XRec)));
    g.xin_cap = cap;
  }
  return 0;
}

// ---- cross-rank collectives on device buffers ---------------------
// Every cross-rank step of the engine — the exchange's counts and records,
// the trigger-byte and spill-flag merges, the spawn gather, the pending and
// counter sums — calls only these four, on device buffers in stream order.
// Each has two implementations: RCCL on the engine's stream (ncclAllReduce /
// ncclAllToAll / ncclAllGather / grouped ncclSend+ncclRecv over xGMI), and
// the host transport (gpu_actor_set_transport: the same device buffers
// staged through pinned host memory and the two callbacks). The control flow
// around them is one path, so the host-transport tests run it all; only the
// nccl* calls inside these functions are left to the RCCL runs.
enum XcType { XC_U8 = 0, XC_U32 = 1, XC_U64 = 2 };

int stage_room(uint64_t sbytes, uint64_t rbytes)
{
  if(sbytes > g.h_sbuf_cap)
  {
    if(g.h_sbuf) HIPCK(hipHostFree(g.h_sbuf));
    g.h_sbuf = nullptr;
    const uint64_t c = std::max<uint64_t>(sbytes, 2 * g.h_sbuf_cap);
    HIPCK(hipHostMalloc(&g.h_sbuf, c, hipHostMallocDefault));
    g.h_sbuf_cap = c;
  }
  if(rbytes > g.h_rbuf_cap)
  {
    if(g.h_rbuf) HIPCK(hipHostFree(g.h_rbuf));
    g.h_rbuf = nullptr;
    const uint64_t c = std::max<uint64_t>(rbytes, 2 * g.h_rbuf_cap);
    HIPCK(hipHostMalloc(&g.h_rbuf, c, hipHostMallocDefault));
    g.h_rbuf_cap = c;
  }
  return 0;
}

// d_out[i] = Σ over ranks of d_in[i], i < count (in place when d_in == d_out).
// XC_U8 on the host transport sums 8 bytes per word: every byte must have
// one nonzero contributor (the trigger bytes: each rank writes its own ids).
int xc_allreduce_sum(const void* d_in, void* d_out, uint64_t count, XcType t)
{
  if(count == 0) return 0;
  if(!g.xp_ar)
  {
    const ncclDataType_t nt = t == XC_U8 ? ncclUint8 : t == XC_U32 ? ncclUint32 : ncclUint64;
    NCCLCK(ncclAllReduce(d_in, d_out, count, nt, ncclSum, g.comm, g.stream));
    return 0;
  }
  const uint64_t esz = t == XC_U8 ? 1 : t == XC_U32 ? 4 : 8;
  const uint64_t bytes = count * esz;
  const uint64_t words = t == XC_U64 ? count : t == XC_U8 ? (bytes + 7) / 8 : count;
  int rc = stage_room(words * 8, bytes);
  if(rc) return rc;
  uint64_t* w = reinterpret_cast<uint64_t*>(g.h_sbuf);
  if(t == XC_U8) memset(w, 0, words * 8);
  HIPCK(hipMemcpyAsync(t == XC_U32 ? g.h_rbuf : g.h_sbuf, d_in, bytes, hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  if(t == XC_U32)
    for(uint64_t i = 0; i < count; ++i) w[i] = reinterpret_cast<const uint32_t*>(g.h_rbuf)[i];
  if(g.xp_ar(g.xp_ctx, w, words) != 0) return GPU_ACTOR_ECOMM;
  if(t == XC_U32)
  {
    for(uint64_t i = 0; i < count; ++i)
      reinterpret_cast<uint32_t*>(g.h_rbuf)[i] = (uint32_t)std::min<uint64_t>(w[i], 0xFFFFFFFFull);
    HIPCK(hipMemcpyAsync(d_out, g.h_rbuf, bytes, hipMemcpyHostToDevice, g.stream));
  }
  else
    HIPCK(hipMemcpyAsync(d_out, g.h_sbuf, bytes, hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));       // the staging is reused by the next call
  return 0;
}

// d_recv[p] = peer p's d_send[rank] (one u64 per peer).
int xc_alltoall_u64(const unsigned long long* d_send, unsigned long long* d_recv)
{
  const uint32_t n = R();
  if(!g.xp_a2a)
  {
    NCCLCK(ncclAllToAll(d_send, d_recv, 1, ncclUint64, g.comm, g.stream));
    return 0;
  }
  int rc = stage_room(n * 8, n * 8);
  if(rc) return rc;
  HIPCK(hipMemcpyAsync(g.h_sbuf, d_send, n * 8, hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  std::vector<uint64_t> b8(n, 8);
  if(g.xp_a2a(g.xp_ctx, g.h_sbuf, b8.data(), g.h_rbuf, b8.data()) != 0) return GPU_ACTOR_ECOMM;
  HIPCK(hipMemcpyAsync(d_recv, g.h_rbuf, n * 8, hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

// d_out[p] = rank p's d_in[0] (one u64 per rank).
int xc_allgather_u64(const unsigned long long* d_in, unsigned long long* d_out)
{
  const uint32_t n = R();
  if(!g.xp_a2a)
  {
    NCCLCK(ncclAllGather(d_in, d_out, 1, ncclUint64, g.comm, g.stream));
    return 0;
  }
  int rc = stage_room(n * 8, n * 8);
  if(rc) return rc;
  HIPCK(hipMemcpyAsync(g.h_sbuf, d_in, 8, hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  uint64_t* sw = reinterpret_cast<uint64_t*>(g.h_sbuf);
  for(uint32_t p = 1; p < n; ++p) sw[p] = sw[0];
  std::vector<uint64_t> b8(n, 8);
  if(g.xp_a2a(g.xp_ctx, g.h_sbuf, b8.data(), g.h_rbuf, b8.data()) != 0) return GPU_ACTOR_ECOMM;
  HIPCK(hipMemcpyAsync(d_out, g.h_rbuf, n * 8, hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

// One grouped exchange: to each peer p != rank, send[p] bytes from d_send[p];
// from it, recv[p] bytes into d_recv[p] (either may be 0).
struct XcPeer {
  const void* d_send = nullptr;
  uint64_t send = 0;
  void* d_recv = nullptr;
  uint64_t recv = 0;
};
int xc_sendrecv(const std::vector<XcPeer>& pp)
{
  const uint32_t n = R();
  if(!g.xp_a2a)
  {
    NCCLCK(ncclGroupStart());
    for(uint32_t p = 0; p < n; ++p)
    {
      if(p == rank()) continue;
      if(pp[p].send) NCCLCK(ncclSend(pp[p].d_send, pp[p].send, ncclUint8, p, g.comm, g.stream));
      if(pp[p].recv) NCCLCK(ncclRecv(pp[p].d_recv, pp[p].recv, ncclUint8, p, g.comm, g.stream));
    }
    NCCLCK(ncclGroupEnd());
    return 0;
  }
  std::vector<uint64_t> sb(n, 0), rb(n, 0);
  uint64_t st = 0, rt = 0;
  for(uint32_t p = 0; p < n; ++p)
  {
    if(p == rank()) continue;
    sb[p] = pp[p].send;
    rb[p] = pp[p].recv;
    st += sb[p];
    rt += rb[p];
  }
  int rc = stage_room(std::max<uint64_t>(st, 8), std::max<uint64_t>(rt, 8));
  if(rc) return rc;
  uint64_t off = 0;
  for(uint32_t p = 0; p < n; ++p)
  {
    if(sb[p]) HIPCK(hipMemcpyAsync(g.h_sbuf + off, pp[p].d_send, sb[p], hipMemcpyDeviceToHost, g.stream));
    off += sb[p];
  }
  HIPCK(hipStreamSynchronize(g.stream));
  if(g.xp_a2a(g.xp_ctx, g.h_sbuf, sb.data(), g.h_rbuf, rb.data()) != 0) return GPU_ACTOR_ECOMM;
  off = 0;
  for(uint32_t p = 0; p < n; ++p)
  {
    if(rb[p]) HIPCK(hipMemcpyAsync(pp[p].d_recv, g.h_rbuf + off, rb[p], hipMemcpyHostToDevice, g.stream));
    off += rb[p];
  }
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

// Trigger bytes in use: global ids L * R + r for every local slot L of the
// largest rank's zones (the same count on every rank, as the merge needs).
uint64_t trig_live_bytes()
{
  const uint64_t per_rank = (g.n_actors + R() - 1) / R();
  const uint64_t zones = (per_rank + zone_actors() - 1) / zone_actors();
  return std::min<uint64_t>(g.trig_bytes, (zones * zone_actors() * R() + 7) & ~7ull);
}

// Peer writes: map every peer's inbox (hipIpcGetMemHandle / hipIpcOpenMemHandle),
// the handles gathered word by word over the engine's collectives (RCCL or the
// host transport). Collective: every rank calls it at the same point.
void peer_close()
{
  for(uint32_t p = 0; p < kMaxRanks; ++p)
  {
    if(g.peer_ptr[p] && p != rank()) (void)hipIpcCloseMemHandle(g.peer_ptr[p]);
    g.peer_ptr[p] = nullptr;
  }
}

int peer_open()
{
  hipIpcMemHandle_t h;
  HIPCK(hipIpcGetMemHandle(&h, g.d_pin));
  static_assert(sizeof(hipIpcMemHandle_t) % 8 == 0, "IPC handle in u64 words");
  constexpr uint32_t kW = sizeof(hipIpcMemHandle_t) / 8;
  const uint32_t n = R();
  std::vector<unsigned long long> all((size_t)kW * n), got(n);
  for(uint32_t w = 0; w < kW; ++w)
  {
    unsigned long long v;
    memcpy(&v, reinterpret_cast<const char*>(&h) + 8 * w, 8);
    HIPCK(hipMemcpyAsync(g.d_hx, &v, 8, hipMemcpyHostToDevice, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    const int rc = xc_allgather_u64(g.d_hx, g.d_hx + 1);
    if(rc) return rc;
    HIPCK(hipMemcpyAsync(got.data(), g.d_hx + 1, n * 8, hipMemcpyDeviceToHost, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    for(uint32_t p = 0; p < n; ++p) all[(size_t)p * kW + w] = got[p];
  }
  for(uint32_t p = 0; p < n; ++p)
  {
    if(p == rank())
    {
      g.peer_ptr[p] = g.d_pin;
      continue;
    }
    hipIpcMemHandle_t hp;
    memcpy(&hp, &all[(size_t)p * kW], sizeof(hp));
    void* ptr = nullptr;
    HIPCK(hipIpcOpenMemHandle(&ptr, hp, hipIpcMemLazyEnablePeerAccess));
    g.peer_ptr[p] = static_cast<XRec*>(ptr);
  }
  return 0;
}

// exchange_room with peer writes: a segment lives in its receiver's inbox, so
// the segments grow on every rank alike — to the largest size any rank needs
// (one gather of each rank's need and whether it kept records in its exchange
// spill list), the kept records moved to the new stride by each inbox's owner,
// the inboxes mapped again; then the spilled records go to their peers, and
// when any rank placed some, one more collective orders those stores before
// every owner's k_xinject.
int peer_room(uint64_t max_send, uint64_t xs)
{
  const bool lost = xs > g.xspill_cap;     // k_xprep clipped the counts to xcap
  uint64_t want = 0;
  if(max_send > g.xcap || lost)
  {
    want = std::max<uint64_t>(2ull * g.xcap, max_send + max_send / 2);
    want = std::min<uint64_t>((want + 63) & ~63ull, 0x40000000ull);
  }
  const uint32_t n = R();
  const unsigned long long mine = want << 1 | (xs ? 1ull : 0ull);
  HIPCK(hipMemcpyAsync(g.d_hx, &mine, 8, hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  int rc = xc_allgather_u64(g.d_hx, g.d_hx + 1);
  if(rc) return rc;
  std::vector<unsigned long long> all(n);
  HIPCK(hipMemcpyAsync(all.data(), g.d_hx + 1, n * 8, hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  uint64_t cap = g.xcap;
  bool any_xs = false;
  for(uint32_t p = 0; p < n; ++p)
  {
    cap = std::max<uint64_t>(cap, all[p] >> 1);
    any_xs |= (all[p] & 1ull) != 0;
  }
  if(cap > g.xcap)
  {
    XRec* nx = nullptr;
    HIPCK(hipMalloc(&nx, (size_t)n * cap * sizeof(XRec)));
    HIPCK(hipMemcpy2DAsync(nx, cap * sizeof(XRec), g.d_pin, (size_t)g.xcap * sizeof(XRec),
      (size_t)g.xcap * sizeof(XRec), n, hipMemcpyDeviceToDevice, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    peer_close();
    HIPCK(hipFree(g.d_pin));
    g.d_pin = nx;
    g.xcap = (uint32_t)cap;
    rc = peer_open();
    if(rc) return rc;
    rc = upload_types();
    if(rc) return rc;
  }
  if(xs)
  {
    if(!lost)
    {
      hipLaunchKernelGGL(k_xspill_place, dim3(blocks_for(xs)), dim3(kBlock), 0, g.stream,
        (uint32_t)xs);
      HIPCK(hipGetLastError());
    }
    HIPCK(hipMemsetAsync(g.d_xspill_n, 0, sizeof(unsigned int), g.stream));
    if(xs > g.xspill_cap / 2)
    {
      HIPCK(hipStreamSynchronize(g.stream));
      rc = alloc_xspill((uint32_t)std::min<uint64_t>(4ull * std::max<uint64_t>(xs, g.xspill_cap),
        1ull << 27));
      if(rc) return rc;
      rc = upload_types();
      if(rc) return rc;
    }
  }
  if(any_xs)
  {
    rc = xc_allreduce_sum(g.d_hx, g.d_hx, 1, XC_U64);
    if(rc) return rc;
  }
  return 0;
}

int exchange_step(uint32_t step_sidx)
{
  const uint32_t n = R(), land_par = g.par, tslot = (step_sidx + 1) % 3;
  unsigned int tcount = 0;
  uint64_t total = 0;
  hipLaunchKernelGGL(k_xprep, dim3(1), dim3(64), 0, g.stream);
  HIPCK(hipGetLastError());
  // send counts to every peer (device), the step's trigger count summed
  int rc = xc_alltoall_u64(g.d_xcount, g.d_xrecv);
  if(rc) return rc;
  rc = xc_allreduce_sum(g.d_trig_n + tslot, g.d_trig_n + tslot, 1, XC_U32);
  if(rc) return rc;
  // the step's one readback: send and receive counts, trigger count, kept
  // exchange-spill records, spill status
  g.h_xc[2 * n] = 0;
  g.h_xc[2 * n + 1] = 0;
  HIPCK(hipMemcpyAsync(g.h_xc, g.d_xc, 2 * n * sizeof(unsigned long long), hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipMemcpyAsync(g.h_xc + 2 * n, g.d_trig_n + tslot, sizeof(unsigned int),
    hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipMemcpyAsync(g.h_xc + 2 * n + 1, g.d_xspill_n, sizeof(unsigned int),
    hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  tcount = (unsigned int)(g.h_xc[2 * n] & 0xFFFFFFFFull);
  const uint64_t xs = g.h_xc[2 * n + 1] & 0xFFFFFFFFull;
  std::vector<uint64_t> roff(n);
  uint64_t max_send = 0;
  for(uint32_t p = 0; p < n; ++p)
  {
    roff[p] = total;
    if(p == rank()) continue;
    total += g.h_xc[n + p];
    max_send = std::max<uint64_t>(max_send, g.h_xc[p]);
  }
  rc = exchange_room(max_send, total, xs);
  if(rc) return rc;
  // the records: each peer's segment of xout to it, its records into xin in
  // rank order (k_xinject tells the sender of a record by its segment)
  // (with peer writes they are in this rank's inbox already: every peer's
  // k_step stored them there before its counts went out)
  if(!g.peer_write)
  {
    std::vector<XcPeer> pp(n);
    for(uint32_t p = 0; p < n; ++p)
    {
      if(p == rank()) continue;
      pp[p].d_send = g.d_xout + (size_t)p * g.xcap;
      pp[p].send = g.h_xc[p] * sizeof(XRec);
      pp[p].d_recv = g.d_xin + roff[p];
      pp[p].recv = g.h_xc[n + p] * sizeof(XRec);
    }
    rc = xc_sendrecv(pp);
    if(rc) return rc;
  }
  g.remote_total += total;
  if(total)
  {
    hipLaunchKernelGGL(k_xinject, dim3(blocks_for(total, kLandRecs)), dim3(kLandThreads), 0, g.stream,
      (const XRec*)(g.peer_write ? g.d_pin : g.d_xin), total, land_par,
      (const unsigned long long*)g.d_xrecv, g.peer_write ? (uint64_t)g.xcap : 0ull);
    HIPCK(hipGetLastError());
  }
  HIPCK(hipMemsetAsync(g.d_xcount, 0, n * sizeof(unsigned long long), g.stream));
  // trigger bytes of parity land_par: every rank's own bytes summed (each
  // byte has one writer, so the sum is the merge), over the ids in use only
  if(tcount || g.trig_stale[land_par])
  {
    rc = xc_allreduce_sum(g.d_trig_own[land_par], g.d_trig[land_par], trig_live_bytes(), XC_U8);
    if(rc) return rc;
  }
  g.trig_stale[land_par] = tcount != 0;
  // did any rank's zone overflow (this step or its landing)? summed on device
  hipLaunchKernelGGL(k_spill_flag, dim3(1), dim3(1), 0, g.stream, g.d_spill_flag);
  HIPCK(hipGetLastError());
  return xc_allreduce_sum(g.d_spill_flag, g.d_spill_flag, 1, XC_U32);
}

// k_step compiled for the one handler table all serial actors share, when
// they do (smaller code, no spills); the any-mix instantiation otherwise.
StepEntry step_entry_for(bool z12)
{
  int only = -1;
  bool mixed = false;
  uint32_t set = 0;                     // tables of the serial actors, as bits
  for(const HostType& t : g.types)
  {
    if(!t.created || reducible_ht(t.ht)) continue;
    if(only >= 0 && (uint32_t)only != t.ht) mixed = true;
    only = (int)t.ht;
    set |= 1u << t.ht;
  }
  if(mixed) only = -1;
  if(set == ((1u << GPU_ACTOR_HT_FIFO_SRC) | (1u << GPU_ACTOR_HT_FIFO_SINK)))
    return z12 ? gpa_z12::step_entry_fifo_pair() : gpa::step_entry_fifo_pair();
  switch(only)
  {
    case GPU_ACTOR_HT_RING: return z12 ? gpa_z12::step_entry_ring() : gpa::step_entry_ring();
    case GPU_ACTOR_HT_PINGER: return z12 ? gpa_z12::step_entry_pinger() : gpa::step_entry_pinger();
    case GPU_ACTOR_HT_PINGER_DET:
      return z12 ? gpa_z12::step_entry_pinger_det() : gpa::step_entry_pinger_det();
    case GPU_ACTOR_HT_FANIN_SENDER:
      return z12 ? gpa_z12::step_entry_fanin_sender() : gpa::step_entry_fanin_sender();
    case GPU_ACTOR_HT_GUPS_STREAMER:
      return z12 ? gpa_z12::step_entry_gups_streamer() : gpa::step_entry_gups_streamer();
    case GPU_ACTOR_HT_STORM: return z12 ? gpa_z12::step_entry_storm() : gpa::step_entry_storm();
    case GPU_ACTOR_HT_SPREADER: return z12 ? gpa_z12::step_entry_spreader() : gpa::step_entry_spreader();
    case GPU_ACTOR_HT_PROGRAM: return z12 ? gpa_z12::step_entry_program() : gpa::step_entry_program();
    default: return z12 ? gpa_z12::step_entry_any() : gpa::step_entry_any();
  }
}

StepEntry pick_step_entry() { return step_entry_for(g.zbits == 12); }
StepEntry step_entry_for_any(bool z12) { return z12 ? gpa_z12::step_entry_any() : gpa::step_entry_any(); }

// LDS a workgroup may hold on gfx950 (the CU's whole 160 KB; two 512-thread
// zones per CU at <= 80 KB each)
constexpr size_t kLdsPerWorkgroup = 160 * 1024;

// Dynamic LDS of a step launch with nb destination buckets: the bucket
// arrays (zone_dev.h: histogram, chunk bases, tile counts, tile starts, and
// the two-pass table's round counts) or the hot-group sort's work area.
size_t step_dyn_bytes(const StepEntry& se, uint64_t nb)
{
  return sizeof(uint32_t) * std::max<uint64_t>((uint64_t)se.bucket_words * nb, se.sort_work);
}

// Whether a step launch with nb buckets fits a workgroup's LDS: static LDS of
// every kernel of the entry (hipFuncGetAttributes) + the dynamic part.
bool step_fits(const StepEntry& se, uint64_t nb)
{
  static std::map<step_kernel_t, size_t> cache;     // (callers hold g.mu)
  size_t st = 0;
  for(step_kernel_t k : {se.kernel, se.plan, se.rest, se.fused})
  {
    if(!k) continue;
    auto it = cache.find(k);
    if(it == cache.end())
    {
      hipFuncAttributes a;
      if(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k)) != hipSuccess) return false;
      it = cache.emplace(k, a.sharedSizeBytes).first;
    }
    st = std::max<size_t>(st, it->second);
  }
  return st + step_dyn_bytes(se, nb) <= kLdsPerWorkgroup;
}

// Ids and landing for the actors the last step's behaviours created: the
// records are sorted by (type, creator, seq) — the canonical order — and
// numbered after each type's live actors (k_spawn_*). One small readback per
// step, only for engines with a reserve. With n_ranks > 1 every rank gathers
// every rank's records (count allgather, then grouped send/recv, or the host
// transport), sorts the same list, numbers alike, and lands the constructor
// messages of the actors it owns (owner = id % n_ranks): the ids equal a
// single rank's (pony_create inside behaviours is rank-agnostic,
// actor.c:688-734).
int spawn_process(uint32_t cur)
{
  unsigned int n = 0;
  HIPCK(hipMemcpyAsync(&n, g.d_spawn_n, sizeof(n), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  n = std::min(n, g.spawn_cap);
  uint64_t* key = g.d_skey[0];
  uint64_t* arg = g.d_sarg[0];
  uint32_t total = n;
  if(R() > 1)
  {
    const uint32_t nr = R();
    std::vector<uint64_t> cnt(nr, 0);
    {
      unsigned long long* dc = g.d_xc + 2 * nr;     // scratch words of the counts block
      const unsigned long long mine = n;
      HIPCK(hipMemcpyAsync(dc, &mine, sizeof(mine), hipMemcpyHostToDevice, g.stream));
      unsigned long long* dall = nullptr;
      HIPCK(hipMalloc(&dall, nr * sizeof(unsigned long long)));
      int rc = xc_allgather_u64(dc, dall);
      if(rc) { (void)hipFree(dall); return rc; }
      HIPCK(hipMemcpyAsync(cnt.data(), dall, nr * sizeof(uint64_t), hipMemcpyDeviceToHost, g.stream));
      HIPCK(hipStreamSynchronize(g.stream));
      HIPCK(hipFree(dall));
    }
    // every rank's whole list, in rank order (each list holds at most
    // spawn_cap records; past that its own device counted the drops): the
    // reserve is applied per type after the canonical sort (k_spawn_land), so
    // which spawns get ids never depends on the rank layout
    std::vector<uint64_t> off(nr);
    uint64_t acc = 0;
    for(uint32_t p = 0; p < nr; ++p)
    {
      cnt[p] = std::min<uint64_t>(cnt[p], g.spawn_cap);
      off[p] = acc;
      acc += cnt[p];
    }
    if(acc > 0x7FFFFFFFull) return GPU_ACTOR_ERANGE;
    total = (uint32_t)acc;
    if(total == 0) return 0;
    n = (uint32_t)cnt[rank()];
    // gathered into [1], local records first copied to their own slot
    if(n)
    {
      HIPCK(hipMemcpyAsync(g.d_skey[1] + off[rank()], g.d_skey[0], n * sizeof(uint64_t),
        hipMemcpyDeviceToDevice, g.stream));
      HIPCK(hipMemcpyAsync(g.d_sarg[1] + off[rank()], g.d_sarg[0], n * sizeof(uint64_t),
        hipMemcpyDeviceToDevice, g.stream));
    }
    // every peer gets our n records; we get each peer's (keys, then args)
    for(int part = 0; part < 2; ++part)
    {
      uint64_t* mine_d = part ? g.d_sarg[0] : g.d_skey[0];
      uint64_t* all_d = part ? g.d_sarg[1] : g.d_skey[1];
      std::vector<XcPeer> pp(nr);
      for(uint32_t p = 0; p < nr; ++p)
      {
        if(p == rank()) continue;
        pp[p].d_send = mine_d;
        pp[p].send = (uint64_t)n * sizeof(uint64_t);
        pp[p].d_recv = all_d + off[p];
        pp[p].recv = cnt[p] * sizeof(uint64_t);
      }
      const int rc = xc_sendrecv(pp);
      if(rc) return rc;
    }
    // sort input: the gathered list
    HIPCK(hipMemcpyAsync(g.d_skey[0], g.d_skey[1], total * sizeof(uint64_t),
      hipMemcpyDeviceToDevice, g.stream));
    HIPCK(hipMemcpyAsync(g.d_sarg[0], g.d_sarg[1], total * sizeof(uint64_t),
      hipMemcpyDeviceToDevice, g.stream));
  }
  if(total == 0) return 0;
  size_t need = 0;
  HIPCK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, key, g.d_skey[1], arg,
    g.d_sarg[1], (int)total, 0, 56, g.stream));
  if(need > g.sort_tmp_bytes)
  {
    if(g.d_sort_tmp) HIPCK(hipFree(g.d_sort_tmp));
    HIPCK(hipMalloc(&g.d_sort_tmp, need));
    g.sort_tmp_bytes = need;
  }
  HIPCK(hipcub::DeviceRadixSort::SortPairs(g.d_sort_tmp, need, key, g.d_skey[1],
    arg, g.d_sarg[1], (int)total, 0, 56, g.stream));
  HIPCK(hipMemsetAsync(g.d_tstart, 0xFF, GPU_ACTOR_MAX_TYPES * sizeof(uint32_t), g.stream));
  HIPCK(hipMemsetAsync(g.d_tcnt, 0, GPU_ACTOR_MAX_TYPES * sizeof(uint32_t), g.stream));
  hipLaunchKernelGGL(k_spawn_scan, dim3(blocks_for(total)), dim3(kBlock), 0, g.stream,
    (const uint64_t*)g.d_skey[1], total, g.d_tstart, g.d_tcnt);
  hipLaunchKernelGGL(k_spawn_land, dim3(blocks_for(total, kLandRecs)), dim3(kLandThreads), 0,
    g.stream, (const uint64_t*)g.d_skey[1], (const uint64_t*)g.d_sarg[1], total,
    (const uint32_t*)g.d_tstart, (const unsigned long long*)g.d_live, cur);
  hipLaunchKernelGGL(k_spawn_commit, dim3(1), dim3(64), 0, g.stream,
    (const uint32_t*)g.d_tcnt, g.d_live);
  HIPCK(hipGetLastError());
  HIPCK(hipMemsetAsync(g.d_spawn_n, 0, sizeof(unsigned int), g.stream));
  return 0;
}

// One superstep: k_step on parity g.par (+ exchange), then flip parity.
// The run-time compiled step this engine's tables take (jit_host.h), built
// or loaded once per set (a set whose build fails stays on the compiled-in
// kernels; one seen before in this process, or on disk, loads at once), with
// PONYC_AMD_JIT not 0: 1 — every serial actor runs a program: the programs
// compiled (two launches, PM 1 plain zones and PM 2 the rest, with the split
// launches on); 2 — a mix of tables the any-mix kernel would run: that
// kernel with only those tables' drains; 0 — neither.
int step_after_launch(uint32_t slot, hipEvent_t e0, hipEvent_t e1);
int jit_ensure(const StepEntry& se)
{
  const char* f = getenv("PONYC_AMD_JIT");
  if((f && atoi(f) == 0) || !g.consts_host) return 0;
  const bool z12 = g.zbits == 12;
  std::vector<jit::Prog> progs;
  uint32_t mask = 0;
  bool all_prog = true;
  for(uint32_t t = 0; t < GPU_ACTOR_MAX_TYPES; ++t)
  {
    const HostType& h = g.types[t];
    if(!h.created || reducible_ht(h.ht)) continue;
    mask |= 1u << h.ht;
    if(h.ht != GPU_ACTOR_HT_PROGRAM || h.prog_host.empty()) all_prog = false;
    else progs.push_back({t, h.prog_host});
  }
  int kind = 0;
  uint64_t want = jit::fnv1a(z12 ? "z12" : "z11");
  if(all_prog && !progs.empty() && g.split_plan)
  {
    kind = 1;
    for(const jit::Prog& p : progs)
      want = jit::fnv1a(std::string(reinterpret_cast<const char*>(p.code.data()), p.code.size() * 8),
                        jit::fnv1a(std::to_string(p.type), want));
  }
  else if(se.kernel == step_entry_for_any(z12).kernel && mask)
  {
    kind = 2;
    want = jit::fnv1a("mix" + std::to_string(mask), want);
  }
  if(!kind) return 0;
  if(g.jit.mod && g.jit_set == want) return kind;
  if(g.jit_failed == want) return 0;
  jit::unload(g.jit);
  hipDeviceProp_t prop;
  if(hipGetDeviceProperties(&prop, g.device) != hipSuccess) { (void)hipGetLastError(); return 0; }
  std::string arch = prop.gcnArchName;
  arch = arch.substr(0, arch.find(':'));
  std::string log;
  const int rc = kind == 1 ? jit::build(progs, z12, arch, g.jit, log)
                           : jit::build_mix(mask, z12, arch, g.jit, log);
  if(getenv("PONYC_AMD_JIT_LOG"))
    fprintf(stderr, "gpu_actor jit: %s %s%s (rc %d) %s\n", kind == 1 ? "programs" : "mix",
            kind == 2 ? ("mask " + std::to_string(mask) + " ").c_str() : "", z12 ? "z12" : "z11", rc,
            log.c_str());
  if(rc != 0)
  {
    g.jit_failed = want;
    return 0;
  }
  g.jit_set = want;
  g.jit_builds++;
  if(hipMemcpyHtoDAsync(g.jit.types, g.td_host, sizeof(g.td_host), g.stream) != hipSuccess ||
     hipMemcpyHtoDAsync(g.jit.eng, &g.eng_host, sizeof(g.eng_host), g.stream) != hipSuccess)
  {
    (void)hipGetLastError();
    jit::unload(g.jit);
    g.jit_failed = want;
    return 0;
  }
  return kind;
}

int launch_step(uint32_t slot, hipEvent_t e0, hipEvent_t e1)
{
  if(g.n_zones == 0) return 0;
  g.dev_epoch++;
  const StepEntry se = pick_step_entry();
  if(se.stub) return GPU_ACTOR_EINVAL;      // an experiment build without this table
  // bucket arrays (4 x buckets; six for an order-free zone's two passes:
  // zone_dev.h two_pass) and, for hot receivers, the sort's work area
  const uint64_t nb = g.n_zones + (R() > 1 ? R() : 0);
  if(!step_fits(se, nb)) return GPU_ACTOR_ERANGE;    // more buckets than a workgroup's LDS holds
  const size_t dyn = step_dyn_bytes(se, nb);
  // the run-time compiled step (jit_ensure), when it builds and fits: the
  // programs' as two launches like the interpreter's, or a mix's one launch
  // with k_hot before it where hot zones are prepared
  g.jit_used = false;
  const int jk = jit_ensure(se);
  if(jk && g.jit.static_lds + dyn <= kLdsPerWorkgroup)
  {
    g.jit_used = true;
    uint32_t a_cur = g.par, a_slot = slot, a_sidx = g.sidx;
    void* args[] = {&a_cur, &a_slot, &a_sidx};
    if(e0) HIPCK(hipEventRecord(e0, g.stream));
    if(jk == 2 && g.hot_on)
      hipLaunchKernelGGL(k_hot, dim3(kHotBlocks), dim3(kHotThreads), 5u * zone_actors() * sizeof(uint32_t),
        g.stream, g.par, g.sidx);
    HIPCK(hipModuleLaunchKernel(g.jit.plan, g.n_zones, 1, 1, se.threads, 1, 1, (unsigned)dyn, g.stream,
      args, nullptr));
    if(jk == 1)
      HIPCK(hipModuleLaunchKernel(g.jit.rest, g.n_zones, 1, 1, se.threads, 1, 1, (unsigned)dyn, g.stream,
        args, nullptr));
    if(g.defer_big)
      hipLaunchKernelGGL(k_carry_big, dim3(kBigCopyBlocks), dim3(kBlock), 0, g.stream, g.par);
    const int grc = gups_apply_launch(nullptr);
    if(grc) return grc;
    if(e1) HIPCK(hipEventRecord(e1, g.stream));
    return step_after_launch(slot, e0, e1);
  }
  // a two-pass table's step as two launches: its two-pass zones, then the rest
  // (zone_dev.h k_step PM)
  // (fused: one launch of PM 3 in their place)
  const bool fused = se.plan && g.split_plan && g.fuse && se.fused;
  const bool split = se.plan && g.split_plan && !fused;
  step_kernel_t kern = fused ? se.fused : split ? se.plan : se.kernel;
  // hot zones first (hot_dev.h): the whole GPU prepares them for k_step
  const size_t hot_lds = 5u * zone_actors() * sizeof(uint32_t);
  if(e0)
  {
    // the events take the dispatch's own start/end timestamps: no marker
    // packets between steps
    const bool gups = g.gups_type >= 0;
    const bool more = split || g.defer_big || gups;
    if(g.hot_on)
      hipExtLaunchKernelGGL(k_hot, dim3(kHotBlocks), dim3(kHotThreads), (uint32_t)hot_lds, g.stream,
        e0, nullptr, 0u, g.par, g.sidx);
    hipExtLaunchKernelGGL(kern, dim3(g.n_zones), dim3(se.threads), (uint32_t)dyn, g.stream,
      g.hot_on ? nullptr : e0, more ? nullptr : e1, 0u, g.par, slot, g.sidx);
    if(split)
      hipExtLaunchKernelGGL(se.rest, dim3(g.n_zones), dim3(se.threads), (uint32_t)dyn, g.stream,
        nullptr, (g.defer_big || gups) ? nullptr : e1, 0u, g.par, slot, g.sidx);
    if(g.defer_big)
      hipExtLaunchKernelGGL(k_carry_big, dim3(kBigCopyBlocks), dim3(kBlock), 0, g.stream,
        nullptr, gups ? nullptr : e1, 0u, g.par);
    HIPCK(hipGetLastError());
    const int grc = gups_apply_launch(e1);
    if(grc) return grc;
  }
  else
  {
    if(g.hot_on)
      hipLaunchKernelGGL(k_hot, dim3(kHotBlocks), dim3(kHotThreads), hot_lds, g.stream, g.par, g.sidx);
    hipLaunchKernelGGL(kern, dim3(g.n_zones), dim3(se.threads), dyn, g.stream, g.par, slot, g.sidx);
    if(split)
      hipLaunchKernelGGL(se.rest, dim3(g.n_zones), dim3(se.threads), dyn, g.stream, g.par, slot, g.sidx);
    if(g.defer_big)
      hipLaunchKernelGGL(k_carry_big, dim3(kBigCopyBlocks), dim3(kBlock), 0, g.stream, g.par);
    HIPCK(hipGetLastError());
    const int grc = gups_apply_launch(nullptr);
    if(grc) return grc;
  }
  HIPCK(hipGetLastError());
  return step_after_launch(slot, e0, e1);
}

// After a step's launches: the parity and step index advance; the exchange
// (n_ranks > 1), the halted step's rerun, spawned actors.
int step_after_launch(uint32_t slot, hipEvent_t e0, hipEvent_t e1)
{
  HIPCK(hipGetLastError());
  const uint32_t step_sidx = g.sidx;
  g.par ^= 1u;
  g.sidx++;
  if(R() > 1)
  {
    int rc = exchange_step(step_sidx);
    if(rc) return rc;
    if(g.h_sstat->halt)
    {
      // this step did not run on any rank (a zone overflowed on some rank the
      // step before): grow, then run it again from the same parity and index
      rc = fixup_spill();
      if(rc) return rc;
      g.par ^= 1u;
      g.sidx--;
      rc = pend_clear(slot, 1);
      if(rc) return rc;
      return launch_step(slot, e0, e1);
    }
  }
  if(g.spawn_cap)
  {
    int rc = spawn_process(g.par);
    if(rc) return rc;
  }
  return 0;
}

int launch_pending(uint32_t slot)
{
  if(g.n_zones == 0) return 0;
  hipLaunchKernelGGL(k_pending, dim3(blocks_for(g.n_zones)), dim3(kBlock), 0, g.stream,
    g.par, slot);
  HIPCK(hipGetLastError());
  return 0;
}

// Sum over ranks of pend[first .. first+n) (host side, after sync).
int pend_read(uint32_t first, uint32_t n, std::vector<unsigned long long>& out)
{
  out.resize(n);
  {
    const int rc = fold_counters(first, n);
    if(rc) return rc;
  }
  if(R() > 1)
  {
    const int rc = xc_allreduce_sum(g.d_pend + first, g.d_pend + first, n, XC_U64);
    if(rc) return rc;
  }
  HIPCK(hipMemcpyAsync(out.data(), g.d_pend + first, n * sizeof(unsigned long long),
    hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

int ensure_events(size_t n)
{
  while(g.ev.size() < n)
  {
    hipEvent_t e;
    HIPCK(hipEventCreate(&e));
    g.ev.push_back(e);
  }
  return 0;
}

void free_all()
{
  jit::unload(g.jit);
  g.jit_set = g.jit_failed = 0;
  g.jit_builds = 0;
  g.jit_used = g.consts_host = false;
  if(g.d_gups_list) (void)hipFree(g.d_gups_list);
  if(g.d_gups_n) (void)hipFree(g.d_gups_n);
  if(g.d_gups_jump) (void)hipFree(g.d_gups_jump);
  if(g.d_gups_stat) (void)hipFree(g.d_gups_stat);
  g.d_gups_list = nullptr; g.d_gups_n = nullptr; g.d_gups_jump = nullptr; g.d_gups_stat = nullptr;
  memset(g.gups_jump_host, 0, sizeof(g.gups_jump_host));
  g.gups_cap = 0;
  g.gups_type = -1;
  for(auto& t : g.types)
  {
    if(t.d_state) (void)hipFree(t.d_state);
    if(t.d_prog) (void)hipFree(t.d_prog);
  }
  for(int p = 0; p < 2; ++p)
  {
    if(g.d_land[p]) (void)hipFree(g.d_land[p]);
    if(g.d_carry[p]) (void)hipFree(g.d_carry[p]);
    if(g.d_land_n[p]) (void)hipFree(g.d_land_n[p]);
    if(g.d_carry_n[p]) (void)hipFree(g.d_carry_n[p]);
  }
  if(g.d_S) (void)hipFree(g.d_S);
  if(g.d_O) (void)hipFree(g.d_O);
  if(g.d_zoff) (void)hipFree(g.d_zoff);
  if(g.d_zcap) (void)hipFree(g.d_zcap);
  for(int p = 0; p < 2; ++p)
  {
    if(g.d_skey[p]) (void)hipFree(g.d_skey[p]);
    if(g.d_sarg[p]) (void)hipFree(g.d_sarg[p]);
  }
  if(g.d_spawn_n) (void)hipFree(g.d_spawn_n);
  if(g.d_tstart) (void)hipFree(g.d_tstart);
  if(g.d_tcnt) (void)hipFree(g.d_tcnt);
  if(g.d_live) (void)hipFree(g.d_live);
  if(g.d_ctl) (void)hipFree(g.d_ctl);
  for(int p = 0; p < 2; ++p)
    if(g.d_spill[p]) (void)hipFree(g.d_spill[p]);
  if(g.d_sstat) (void)hipFree(g.d_sstat);
  if(g.h_sstat) (void)hipHostFree(g.h_sstat);
  if(g.d_need) (void)hipFree(g.d_need);
  for(int p = 0; p < 2; ++p)
  {
    if(g.d_trig[p]) (void)hipFree(g.d_trig[p]);
    if(g.d_trig_own[p]) (void)hipFree(g.d_trig_own[p]);
    if(g.d_ztrig[p]) (void)hipFree(g.d_ztrig[p]);
  }
  if(g.d_zplan) (void)hipFree(g.d_zplan);
  if(g.d_muted_on) (void)hipFree(g.d_muted_on);
  if(g.d_trig_n) (void)hipFree(g.d_trig_n);
  if(g.d_bigc) (void)hipFree(g.d_bigc);
  if(g.d_bigc_n) (void)hipFree(g.d_bigc_n);
  if(g.h_ctl) (void)hipHostFree(g.h_ctl);
  if(g.d_sort_tmp) (void)hipFree(g.d_sort_tmp);
  if(g.d_stats) (void)hipFree(g.d_stats);
  if(g.d_pend) (void)hipFree(g.d_pend);
  if(g.d_pend_sh) (void)hipFree(g.d_pend_sh);
  if(g.d_stats_sh) (void)hipFree(g.d_stats_sh);
  if(g.d_hot) (void)hipFree(g.d_hot);
  if(g.d_dbg) (void)hipFree(g.d_dbg);
  if(g.h_msgs) (void)hipHostFree(g.h_msgs);
  if(g.d_msgs) (void)hipFree(g.d_msgs);
  if(g.d_xout) (void)hipFree(g.d_xout);
  if(g.d_xin) (void)hipFree(g.d_xin);
  peer_close();
  if(g.d_pin) (void)hipFree(g.d_pin);
  if(g.d_hx) (void)hipFree(g.d_hx);
  if(g.d_xspill) (void)hipFree(g.d_xspill);
  if(g.d_xspill_n) (void)hipFree(g.d_xspill_n);
  if(g.d_xc) (void)hipFree(g.d_xc);
  if(g.h_xc) (void)hipHostFree(g.h_xc);
  if(g.d_spill_flag) (void)hipFree(g.d_spill_flag);
  if(g.h_sbuf) (void)hipHostFree(g.h_sbuf);
  if(g.h_rbuf) (void)hipHostFree(g.h_rbuf);
  for(hipEvent_t e : g.ev) (void)hipEventDestroy(e);
  if(g.comm) (void)ncclCommDestroy(g.comm);
  if(g.stream) (void)hipStreamDestroy(g.stream);
}

// A host send must name an actor of this rank (each rank injects its own
// share; k_inject lands only local mail).
inline bool host_msg_ok(const gpu_msg_t& m)
{
  return m.to < g.n_actors && m.behaviour <= 0xF && (R() == 1 || m.to % R() == rank());
}

int inject_locked(const gpu_msg_t* first, uint64_t n)
{
  if(g.host_seq + n >= (1ull << 40)) return GPU_ACTOR_ERANGE;
  g.dev_epoch++;
  if(n > g.d_msgs_cap)
  {
    if(g.d_msgs) HIPCK(hipFree(g.d_msgs));
    g.d_msgs = nullptr;
    HIPCK(hipMalloc(&g.d_msgs, n * sizeof(gpu_msg_t)));
    g.d_msgs_cap = n;
  }
  HIPCK(hipMemcpyAsync(g.d_msgs, first, n * sizeof(gpu_msg_t), hipMemcpyHostToDevice, g.stream));
  if(g.n_zones)
  {
    hipLaunchKernelGGL(k_inject, dim3(blocks_for(n, kLandRecs)), dim3(kLandThreads), 0, g.stream,
      (const gpu_msg_t*)g.d_msgs, n, g.host_seq, g.par);
    HIPCK(hipGetLastError());
  }
  g.host_seq += n;
  // the caller may reuse its buffer: this synchronises the stream
  int rc = read_sstat();
  if(rc) return rc;
  return spill_pending() ? fixup_spill() : 0;
}

// gpu_actor_send's deferred messages, injected in call order.
int flush_sends()
{
  if(g.deferred.empty()) return 0;
  const int rc = inject_locked(g.deferred.data(), g.deferred.size());
  g.deferred.clear();
  return rc;
}

int sendv_locked(const gpu_msg_t* first, uint64_t n)
{
  if(n == 0) return 0;
  if(!first) return GPU_ACTOR_EINVAL;
  for(uint64_t i = 0; i < n; ++i)
    if(!host_msg_ok(first[i])) return GPU_ACTOR_EINVAL;
  int rc = flush_sends();                   // earlier single sends go first
  if(rc) return rc;
  return inject_locked(first, n);
}

} // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

GPU_ACTOR_API const char* gpu_actor_strerror(int code)
{
  switch(code)
  {
    case GPU_ACTOR_OK: return "ok";
    case GPU_ACTOR_EINVAL: return "invalid argument";
    case GPU_ACTOR_ENOMEM: return "out of memory";
    case GPU_ACTOR_ENODEV: return "no usable GPU";
    case GPU_ACTOR_EMAILBOX: return "mailbox overflow (messages dropped)";
    case GPU_ACTOR_EHIP: return "HIP runtime error";
    case GPU_ACTOR_ESTATE: return "engine not initialised or already initialised";
    case GPU_ACTOR_ERANGE: return "sequence or id space exhausted";
    case GPU_ACTOR_ECOMM: return "RCCL exchange failure";
    case GPU_ACTOR_EBUSY: return "an asynchronous run is in flight";
    default: return "unknown error";
  }
}

GPU_ACTOR_API int gpu_actor_comm_id(void* out128)
{
  if(!out128) return GPU_ACTOR_EINVAL;
  ncclUniqueId id;
  NCCLCK(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

GPU_ACTOR_API int gpu_actor_init(const gpu_actor_config_t* cfg)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(g.init) return GPU_ACTOR_ESTATE;
  if(!cfg) return GPU_ACTOR_EINVAL;
  g.cfg = *cfg;
  if(g.cfg.n_ranks == 0) g.cfg.n_ranks = 1;
  if(g.cfg.rank >= g.cfg.n_ranks || g.cfg.n_ranks > kMaxRanks) return GPU_ACTOR_EINVAL;
  if(g.cfg.batch == 0) g.cfg.batch = 100;                 // PONY_SCHED_BATCH
  if(g.cfg.mailbox_cap == 0) g.cfg.mailbox_cap = 16;
  if(g.cfg.max_actors == 0) g.cfg.max_actors = 1ull << 26;
  if(g.cfg.max_actors > 0xFF000000ull) return GPU_ACTOR_EINVAL;

  int ndev = 0;
  if(hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GPU_ACTOR_ENODEV;
  g.device = cfg->device >= 0 ? cfg->device : 0;
  if(cfg->device < 0) (void)hipGetDevice(&g.device);
  if(g.device >= ndev) return GPU_ACTOR_ENODEV;
  HIPCK(hipSetDevice(g.device));
  HIPCK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));

  HIPCK(hipMalloc(&g.d_stats, ST_COUNT * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_stats, 0, ST_COUNT * sizeof(unsigned long long), g.stream));
  HIPCK(hipMalloc(&g.d_pend, kPendSlots * sizeof(unsigned long long)));
  HIPCK(hipMalloc(&g.d_pend_sh, (size_t)kPendSlots * kShards * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_pend_sh, 0, (size_t)kPendSlots * kShards * sizeof(unsigned long long),
    g.stream));
  {
    // hot-zone scratch (hot_dev.h): prep, slot, counts, key ranges (fmin
    // starts at ~0), bins, bin counts, cursors, barrier
    const size_t words = hot_words_before_bar() + 64;
    HIPCK(hipMalloc(&g.d_hot, words * sizeof(uint32_t)));
    HIPCK(hipMemsetAsync(g.d_hot, 0, words * sizeof(uint32_t), g.stream));
    uint32_t* aux = g.d_hot + 2 * kMaxZones + kMaxHot * kHotActors;
    for(uint32_t h = 0; h < kMaxHot; ++h)
      HIPCK(hipMemsetAsync(aux + (size_t)h * 3 * kHotActors, 0xFF, kHotActors * sizeof(uint32_t),
        g.stream));
  }
  HIPCK(hipMalloc(&g.d_stats_sh, (size_t)ST_COUNT * kShards * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_stats_sh, 0, (size_t)ST_COUNT * kShards * sizeof(unsigned long long),
    g.stream));
  HIPCK(hipMalloc(&g.d_dbg, kMaxZones * kDbgSlots * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_dbg, 0, kMaxZones * kDbgSlots * sizeof(unsigned long long), g.stream));
  HIPCK(hipMalloc(&g.d_spawn_n, sizeof(unsigned int)));
  HIPCK(hipMemsetAsync(g.d_spawn_n, 0, sizeof(unsigned int), g.stream));
  HIPCK(hipMalloc(&g.d_tstart, GPU_ACTOR_MAX_TYPES * sizeof(uint32_t)));
  HIPCK(hipMalloc(&g.d_tcnt, GPU_ACTOR_MAX_TYPES * sizeof(uint32_t)));
  HIPCK(hipMalloc(&g.d_live, GPU_ACTOR_MAX_TYPES * sizeof(unsigned long long)));
  HIPCK(hipMalloc(&g.d_ctl, sizeof(SparseCtl)));
  HIPCK(hipMalloc(&g.d_sstat, sizeof(Engine::SpillStat)));
  HIPCK(hipMemsetAsync(g.d_sstat, 0, sizeof(Engine::SpillStat), g.stream));
  HIPCK(hipHostMalloc(&g.h_sstat, sizeof(Engine::SpillStat), hipHostMallocDefault));
  memset(g.h_sstat, 0, sizeof(Engine::SpillStat));
  HIPCK(hipMalloc(&g.d_need, kMaxZones * sizeof(uint32_t)));
  HIPCK(hipMalloc(&g.d_zplan, kMaxZones * sizeof(uint32_t)));
  HIPCK(hipMemsetAsync(g.d_zplan, 0, kMaxZones * sizeof(uint32_t), g.stream));
  g.trig_bytes = (g.cfg.max_actors + 2 * 4096 + 7) & ~7ull;   // room for either zone size
  for(int p = 0; p < 2; ++p)
  {
    HIPCK(hipMalloc(&g.d_trig[p], g.trig_bytes));
    HIPCK(hipMemsetAsync(g.d_trig[p], 0, g.trig_bytes, g.stream));
    HIPCK(hipMalloc(&g.d_ztrig[p], kMaxZones * sizeof(uint32_t)));
    HIPCK(hipMemsetAsync(g.d_ztrig[p], 0, kMaxZones * sizeof(uint32_t), g.stream));
    if(R() > 1)
    {
      HIPCK(hipMalloc(&g.d_trig_own[p], g.trig_bytes));
      HIPCK(hipMemsetAsync(g.d_trig_own[p], 0, g.trig_bytes, g.stream));
    }
  }
  HIPCK(hipMalloc(&g.d_spill_flag, sizeof(unsigned int)));
  HIPCK(hipMemsetAsync(g.d_spill_flag, 0, sizeof(unsigned int), g.stream));
  HIPCK(hipMalloc(&g.d_trig_n, 4 * sizeof(unsigned int)));
  HIPCK(hipMemsetAsync(g.d_trig_n, 0, 4 * sizeof(unsigned int), g.stream));
  HIPCK(hipMalloc(&g.d_bigc, kBigCopyCap * sizeof(BigCopy)));
  HIPCK(hipMalloc(&g.d_bigc_n, 2 * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_bigc_n, 0, 2 * sizeof(unsigned long long), g.stream));
  HIPCK(hipHostMalloc(&g.h_ctl, sizeof(SparseCtl), hipHostMallocDefault));
  HIPCK(hipMemsetAsync(g.d_live, 0, GPU_ACTOR_MAX_TYPES * sizeof(unsigned long long), g.stream));

  if(R() > 1)
  {
    g.xcap = g.cfg.max_exchange ? g.cfg.max_exchange : (1u << 22);
    if(cfg->comm_id)
    {
      ncclUniqueId id;
      memcpy(&id, cfg->comm_id, sizeof(id));
      NCCLCK(ncclCommInitRank(&g.comm, (int)R(), id, (int)rank()));
      g.xp_a2a = nullptr;
      g.xp_ar = nullptr;
    }
    else
    {
      // host transport (callbacks registered with gpu_actor_set_transport);
      // its staging grows on demand (stage_room)
      if(!g.xp_a2a || !g.xp_ar) return GPU_ACTOR_EINVAL;
    }
    {
      const char* pw = getenv("PONYC_AMD_PEER_WRITE");
      g.peer_write = pw && atoi(pw) != 0;
    }
    if(g.peer_write)
    {
      HIPCK(hipMalloc(&g.d_pin, (size_t)R() * g.xcap * sizeof(XRec)));
      HIPCK(hipMalloc(&g.d_hx, (1 + R()) * sizeof(unsigned long long)));
    }
    else
    {
      HIPCK(hipMalloc(&g.d_xout, (size_t)R() * g.xcap * sizeof(XRec)));
      HIPCK(hipMalloc(&g.d_xin, (size_t)R() * g.xcap * sizeof(XRec)));
      g.xin_cap = (uint64_t)R() * g.xcap;
    }
    HIPCK(hipMalloc(&g.d_xspill_n, sizeof(unsigned int)));
    HIPCK(hipMemsetAsync(g.d_xspill_n, 0, sizeof(unsigned int), g.stream));
    {
      const int xrc = alloc_xspill(std::max<uint32_t>(1u << 18, g.xcap / 2));
      if(xrc) return xrc;
    }
    HIPCK(hipMalloc(&g.d_xc, (2 * R() + 2) * sizeof(unsigned long long)));
    HIPCK(hipMemsetAsync(g.d_xc, 0, (2 * R() + 2) * sizeof(unsigned long long), g.stream));
    HIPCK(hipHostMalloc(&g.h_xc, (2 * R() + 2) * sizeof(unsigned long long), hipHostMallocDefault));
    g.d_xcount = g.d_xc;
    g.d_xrecv = g.d_xc + R();
    g.h_xcount.assign(R(), 0);
    g.h_xrecv.assign(R(), 0);
    if(g.peer_write)
    {
      HIPCK(hipStreamSynchronize(g.stream));
      const int prc = peer_open();
      if(prc) return prc;
    }
  }
  g.init = true;
  int rc = upload_types();
  if(rc) return rc;
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

// Joins a finished (or running) asynchronous run; caller must NOT hold g.mu.
// Called on the progress thread itself (the completion callback chaining a
// run_async, wait or shutdown), it detaches instead: the thread ends right
// after its callback returns.
void join_worker()
{
  std::thread t;
  {
    std::lock_guard<std::mutex> wl(g.wmu);
    if(!g.worker.joinable()) return;
    if(g.worker.get_id() == std::this_thread::get_id())
    {
      // it cannot join itself: gpu_actor_shutdown joins it later, so its
      // completion callback has returned before anything it runs is freed
      g.detached.push_back(std::move(g.worker));
      return;
    }
    t = std::move(g.worker);
  }
  t.join();
}

// Joins the progress threads that chained runs from their callbacks (all
// but the calling thread itself); caller must NOT hold g.mu.
void join_detached()
{
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> wl(g.wmu);
    for(auto& t : g.detached)
    {
      if(t.get_id() == std::this_thread::get_id()) t.detach();   // returns after this call
      else ts.push_back(std::move(t));
    }
    g.detached.clear();
  }
  for(auto& t : ts)
    if(t.joinable()) t.join();
}

GPU_ACTOR_API int gpu_actor_shutdown(void)
{
  join_worker();                      // an async run finishes first
  join_detached();
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(g.stream) (void)hipStreamSynchronize(g.stream);
  free_all();
  for(auto& t : g.types) t = HostType();
  g.init = false; g.n_types = 0; g.n_actors = 0; g.n_local = 0;
  g.n_zones = 0; g.zone_records = 0; g.d_zoff = nullptr; g.d_zcap = nullptr; g.par = 0;
  g.zbits = kZoneBits;
  for(int p = 0; p < 2; ++p)
  {
    g.d_land[p] = g.d_carry[p] = nullptr;
    g.d_land_n[p] = g.d_carry_n[p] = nullptr;
  }
  g.d_S = nullptr; g.d_O = nullptr;
  g.d_stats = g.d_pend = g.d_dbg = nullptr;
  g.d_pend_sh = g.d_stats_sh = nullptr;
  g.d_hot = nullptr;
  g.spawn_cap = 0; g.d_spawn_n = nullptr; g.d_tstart = g.d_tcnt = nullptr; g.d_live = nullptr;
  g.d_ctl = nullptr; g.h_ctl = nullptr; g.sparse_launches = g.sparse_steps = 0;
  g.d_spill[0] = g.d_spill[1] = nullptr; g.spill_cap = 0; g.d_sstat = nullptr; g.h_sstat = nullptr;
  g.d_need = nullptr; g.zcap_min.clear(); g.zcap_host.clear(); g.fixups = 0;
  for(int p = 0; p < 2; ++p)
  {
    g.d_trig[p] = g.d_trig_own[p] = nullptr;
    g.d_ztrig[p] = nullptr;
    g.trig_stale[p] = false;
  }
  g.d_zplan = nullptr;
  g.trig_bytes = 0; g.d_muted_on = nullptr; g.muted_on_cap = 0; g.d_trig_n = nullptr; g.sidx = 0;
  g.d_bigc = nullptr; g.d_bigc_n = nullptr; g.defer_big = false;
  g.d_sort_tmp = nullptr; g.sort_tmp_bytes = 0;
  for(int p = 0; p < 2; ++p) g.d_skey[p] = g.d_sarg[p] = nullptr;
  g.h_msgs = nullptr; g.h_msgs_cap = 0; g.d_msgs = nullptr; g.d_msgs_cap = 0;
  g.host_seq = 0; g.steps_total = 0; g.sticky = 0; g.ev.clear(); g.last_drain_ms = 0;
  g.deferred.clear();
  g.comm = nullptr; g.d_xout = g.d_xin = nullptr;
  g.d_pin = nullptr; g.d_hx = nullptr; g.peer_write = false; g.d_xcount = g.d_xrecv = nullptr;
  g.d_xc = nullptr; g.h_xc = nullptr; g.d_spill_flag = nullptr;
  g.xcap = 0; g.remote_total = 0; g.stream = nullptr;
  g.xin_cap = 0; g.d_xspill = nullptr; g.d_xspill_n = nullptr; g.xspill_cap = 0;
  g.h_sbuf = g.h_rbuf = nullptr;
  g.h_sbuf_cap = g.h_rbuf_cap = 0;
  return 0;
}

GPU_ACTOR_API int gpu_actor_set_transport(gpu_actor_alltoallv_fn alltoallv,
  gpu_actor_allreduce_fn allreduce, void* ctx)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(g.init) return GPU_ACTOR_ESTATE;
  if((alltoallv == nullptr) != (allreduce == nullptr)) return GPU_ACTOR_EINVAL;
  g.xp_a2a = alltoallv;
  g.xp_ar = allreduce;
  g.xp_ctx = ctx;
  return 0;
}

GPU_ACTOR_API int gpu_actor_type_register(uint32_t type_id, uint32_t state_words,
  uint32_t handler_table)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  const uint32_t need = required_words(handler_table);
  if(need == 0 || state_words < need) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(t.registered) return GPU_ACTOR_EINVAL;
  t.registered = true;
  t.words = state_words;
  t.ht = handler_table;
  t.batch = g.cfg.batch;
  t.cap = g.cfg.mailbox_cap;
  return 0;
}

GPU_ACTOR_API int gpu_actor_type_config(uint32_t type_id, uint32_t batch, uint32_t mailbox_cap)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !g.types[type_id].registered) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(mailbox_cap & (mailbox_cap - 1)) return GPU_ACTOR_EINVAL;
  if(t.created && mailbox_cap && mailbox_cap != t.cap) return GPU_ACTOR_EINVAL;
  if(batch) t.batch = batch;
  if(mailbox_cap) t.cap = mailbox_cap;
  return t.created ? upload_types() : 0;
}

GPU_ACTOR_API int gpu_actor_type_priority(uint32_t type_id, int32_t priority)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !g.types[type_id].registered) return GPU_ACTOR_EINVAL;
  if(g.async_busy) return GPU_ACTOR_EBUSY;
  g.types[type_id].priority = priority;
  return g.types[type_id].created ? upload_types() : 0;
}

GPU_ACTOR_API int gpu_actor_type_param(uint32_t type_id, uint32_t idx, uint64_t value)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || idx >= GPU_ACTOR_MAX_PARAMS ||
    !g.types[type_id].registered) return GPU_ACTOR_EINVAL;
  g.types[type_id].params[idx] = value;
  return g.types[type_id].created ? upload_types() : 0;
}

GPU_ACTOR_API int gpu_actor_type_program(uint32_t type_id, const uint64_t* code, uint32_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !g.types[type_id].registered ||
     g.types[type_id].ht != GPU_ACTOR_HT_PROGRAM || !code || n <= GPU_ACTOR_PROG_ENTRIES ||
     n > (1u << 20)) return GPU_ACTOR_EINVAL;
  if(g.async_busy) return GPU_ACTOR_EBUSY;
  HostType& t = g.types[type_id];
  uint64_t* d = nullptr;
  HIPCK(hipMalloc(&d, (size_t)n * sizeof(uint64_t)));
  // on the engine's stream like every other upload; the new buffer is freed
  // if the copy fails
  if(hipMemcpyAsync(d, code, (size_t)n * sizeof(uint64_t), hipMemcpyHostToDevice, g.stream) !=
       hipSuccess || hipStreamSynchronize(g.stream) != hipSuccess)
  {
    (void)hipGetLastError();
    (void)hipFree(d);
    return GPU_ACTOR_EHIP;
  }
  if(t.d_prog)
  {
    HIPCK(hipStreamSynchronize(g.stream));          // no launch still reads the old one
    HIPCK(hipFree(t.d_prog));
  }
  t.d_prog = d;
  t.prog_n = n;
  t.prog_host.assign(code, code + n);
  t.prog_yields = false;
  for(uint32_t k = 0; k < n; ++k)                   // (a jump may run the entry words too)
    t.prog_yields |= (code[k] & 0xFFu) == GPU_ACTOR_OP_YIELD || (code[k] & 0xFFu) == GPU_ACTOR_OP_SPAWN;
  return t.created ? upload_types() : 0;
}

GPU_ACTOR_API int gpu_actor_create(uint32_t type_id, uint64_t count, uint64_t* first_id)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.registered || t.created || count == 0) return GPU_ACTOR_EINVAL;
  const uint64_t live = count;
  count += t.reserve;                    // ids for the type's spawned actors
  if(g.n_actors + count > g.cfg.max_actors) return GPU_ACTOR_ERANGE;
  if(g.spawn_cap + t.reserve > 0xFFFFFFFFull) return GPU_ACTOR_ERANGE;
  if(t.ht == GPU_ACTOR_HT_GUPS_UPDATER)
  {
    const uint64_t size = t.params[0];
    if(size == 0 || (size & (size - 1)) || size > t.words) return GPU_ACTOR_EINVAL;
  }
  const uint64_t lo = owned_below(g.n_actors), hi = owned_below(g.n_actors + count);
  const uint32_t n_local = (uint32_t)hi;
  if((n_local + kZone - 1) / kZone > kMaxZones) return GPU_ACTOR_ERANGE;
  t.first = g.n_actors;
  t.count = count;
  t.lfirst = (uint32_t)lo;
  t.lcount = (uint32_t)(hi - lo);
  const size_t lc = std::max<size_t>(t.lcount, 1);
  HIPCK(hipMalloc(&t.d_state, (size_t)t.words * lc * sizeof(uint64_t)));
  HIPCK(hipMemsetAsync(t.d_state, 0, (size_t)t.words * lc * sizeof(uint64_t), g.stream));
  t.created = true;
  g.n_actors += count;
  g.n_local = n_local;
  g.n_types = std::max(g.n_types, type_id + 1);
  int rc = relayout_zones(true);
  if(rc) return rc;
  rc = ensure_spill(spill_cap_for_zones());     // empty between calls: nothing to keep
  if(rc) return rc;
  rc = upload_types();
  if(rc) return rc;
  hipLaunchKernelGGL(k_construct, dim3(blocks_for(std::max<uint64_t>(t.lcount, 1))), dim3(kBlock), 0,
    g.stream, type_id, (uint32_t)live);
  if(t.ht == GPU_ACTOR_HT_GUPS_UPDATER)
    hipLaunchKernelGGL(k_construct_table, dim3(4096), dim3(kBlock), 0, g.stream,
      type_id, (uint32_t)live);
  HIPCK(hipGetLastError());
  const unsigned long long live_ull = live;
  HIPCK(hipMemcpyAsync(g.d_live + type_id, &live_ull, sizeof(live_ull), hipMemcpyHostToDevice,
    g.stream));
  if(t.reserve)
  {
    // the spawn buffers hold one record per reserved id; nothing is in them
    // between steps, so growing them drops nothing
    HIPCK(hipStreamSynchronize(g.stream));
    // the gathered list of n_ranks > 1 holds every rank's records
    const uint32_t cap = g.spawn_cap + (uint32_t)t.reserve;
    for(int p = 0; p < 2; ++p)
    {
      if(g.d_skey[p]) HIPCK(hipFree(g.d_skey[p]));
      if(g.d_sarg[p]) HIPCK(hipFree(g.d_sarg[p]));
      HIPCK(hipMalloc(&g.d_skey[p], (size_t)cap * R() * sizeof(uint64_t)));
      HIPCK(hipMalloc(&g.d_sarg[p], (size_t)cap * R() * sizeof(uint64_t)));
    }
    g.spawn_cap = cap;
    rc = upload_types();
    if(rc) return rc;
  }
  HIPCK(hipStreamSynchronize(g.stream));
  if(first_id) *first_id = t.first;
  return 0;
}

GPU_ACTOR_API int gpu_actor_type_reserve(uint32_t type_id, uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !g.types[type_id].registered ||
    g.types[type_id].created) return GPU_ACTOR_EINVAL;
  if(n > g.cfg.max_actors) return GPU_ACTOR_ERANGE;
  g.types[type_id].reserve = n;
  return 0;
}

GPU_ACTOR_API int gpu_actor_type_live(uint32_t type_id, uint64_t* live)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !live || !g.types[type_id].created)
    return GPU_ACTOR_EINVAL;
  unsigned long long v = 0;
  HIPCK(hipMemcpyAsync(&v, g.d_live + type_id, sizeof(v), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  *live = v;
  return 0;
}

GPU_ACTOR_API int gpu_actor_alloc_msgs(uint64_t n, gpu_msg_t** buf)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(!buf) return GPU_ACTOR_EINVAL;
  if(n > g.h_msgs_cap)
  {
    if(g.h_msgs) HIPCK(hipHostFree(g.h_msgs));
    g.h_msgs = nullptr;
    HIPCK(hipHostMalloc(&g.h_msgs, n * sizeof(gpu_msg_t), hipHostMallocDefault));
    g.h_msgs_cap = n;
  }
  *buf = g.h_msgs;
  return 0;
}

GPU_ACTOR_API int gpu_actor_sendv(const gpu_msg_t* first, uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  return sendv_locked(first, n);
}

GPU_ACTOR_API int gpu_actor_send(uint64_t to, uint32_t behaviour, uint64_t arg)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  gpu_msg_t m;
  m.to = (uint32_t)to; m.behaviour = behaviour; m.arg = arg;
  if(to >= g.n_actors || !host_msg_ok(m)) return GPU_ACTOR_EINVAL;
  if(g.host_seq + g.deferred.size() + 1 >= (1ull << 40)) return GPU_ACTOR_ERANGE;
  try { g.deferred.push_back(m); } catch(...) { return GPU_ACTOR_ENOMEM; }
  return 0;
}

// The small-step path applies to one rank without spawning types (spawned
// ids are numbered by the host after each dense step). GPA_NO_SPARSE=1 turns
// it off (A/B runs).
bool sparse_ok()
{
  const char* e = getenv("GPA_NO_SPARSE");
  return !(e && atoi(e) != 0) && R() == 1 && g.spawn_cap == 0 && g.n_zones > 0;
}

// One k_sparse launch from parity g.par: up to max_steps supersteps (0: no
// limit). Returns its control block after the launch completes.
int run_sparse(uint64_t max_steps, SparseCtl& out)
{
  g.dev_epoch++;
  bool prog = false, gups = false;
  for(const HostType& t : g.types)
  {
    prog |= t.created && t.ht == GPU_ACTOR_HT_PROGRAM;
    gups |= t.created && t.ht == GPU_ACTOR_HT_GUPS_STREAMER;
  }
#define GPA_SPARSE_LAUNCH(P, G)                                                         \
  hipLaunchKernelGGL((k_sparse<P, G>), dim3(1), dim3(kSpThreads), 0, g.stream, g.par,   \
    (unsigned long long)max_steps, g.d_ctl, g.sidx)
  if(prog && gups) GPA_SPARSE_LAUNCH(true, true);
  else if(prog) GPA_SPARSE_LAUNCH(true, false);
  else if(gups) GPA_SPARSE_LAUNCH(false, true);
  else GPA_SPARSE_LAUNCH(false, false);
#undef GPA_SPARSE_LAUNCH
  HIPCK(hipGetLastError());
  {
    // the chunks its supersteps listed (2^16 or more per segment)
    const int rc = gups_apply_launch(nullptr);
    if(rc) return rc;
  }
  HIPCK(hipMemcpyAsync(g.h_ctl, g.d_ctl, sizeof(SparseCtl), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  out = *g.h_ctl;
  g.par = out.par;
  g.sidx += (uint32_t)out.steps;
  g.sparse_launches++;
  g.sparse_steps += out.steps;
  return 0;
}

// Pending mail now (all ranks).
int pending_now(unsigned long long& out)
{
  int rc = pend_clear(kPendPre, 1);
  if(rc) return rc;
  rc = launch_pending(kPendPre);
  if(rc) return rc;
  std::vector<unsigned long long> pv;
  rc = pend_read(kPendPre, 1, pv);
  if(rc) return rc;
  out = pv[0];
  return 0;
}

// Zone overflow left by the last operation: grow the zones and land the
// spilled records. One rank decides from its own status. With n_ranks > 1 the
// decision is this status summed over ranks (k_spill_local + pend_read, a
// collective every rank makes at the same point), so all ranks run
// fixup_spill — and clear their spill flags — together or none does.
int settle_spills()
{
  if(R() == 1)
  {
    // (nothing ran since the last read: it stands)
    if(g.sstat_epoch == g.dev_epoch) return spill_pending() ? fixup_spill() : 0;
    const int rc = read_sstat();
    if(rc) return rc;
    return spill_pending() ? fixup_spill() : 0;
  }
  hipLaunchKernelGGL(k_spill_local, dim3(1), dim3(1), 0, g.stream, g.d_pend + kPendPre);
  HIPCK(hipGetLastError());
  HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
    g.stream));
  std::vector<unsigned long long> pv;
  const int rc = pend_read(kPendPre, 1, pv);
  if(rc) return rc;
  return pv[0] ? fixup_spill() : 0;
}

// The scheduler loop to quiescence (or max_steps); caller holds g.mu.
// One rank: chunks of kChunk k_step launches with one readback each, or
// k_sparse launches while few records are pending. A zone that overflowed
// halts the steps after it on the device; the host then grows the zones
// (fixup_spill) and resumes from the first step that did not run.
int run_locked(uint64_t max_steps, uint64_t* steps_done)
{
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  uint64_t done = 0;
  if(g.n_zones)
  {
    int rc = settle_spills();
    if(rc) return rc;
    unsigned long long before = 0;
    rc = pending_now(before);
    if(rc) return rc;
    std::vector<unsigned long long> pv;
    std::vector<uint32_t> par_at(kChunk + 1), sidx_at(kChunk + 1);
    const bool sp = sparse_ok();
    while(before > 0 && (max_steps == 0 || done < max_steps))
    {
      if(sp && before <= kSpCap)
      {
        // few messages in flight: whole supersteps in one workgroup until the
        // world is quiet, max_steps, or a step needs the zone path
        SparseCtl c;
        rc = run_sparse(max_steps ? max_steps - done : 0, c);
        if(rc) return rc;
        done += c.steps;
        if(spill_pending())
        {
          rc = fixup_spill();
          if(rc) return rc;
          rc = pending_now(before);
          if(rc) return rc;
          continue;
        }
        if(c.reason == SP_QUIESCENT) { before = 0; break; }
        if(c.reason == SP_MAX_STEPS) break;
        if(c.steps && c.pending == 0xFFFFFFFFFFFFFFFFull)
        {
          // the last step overflowed the list: count what is pending
          rc = pending_now(before);
          if(rc) return rc;
          if(before == 0) break;
        }
        if(max_steps && done >= max_steps) break;
        // SP_DENSE: the next steps go through k_step (at least one chunk)
      }
      uint32_t k = kChunk;
      if(max_steps) k = (uint32_t)std::min<uint64_t>(k, max_steps - done);
      // pend[j] = pending at the start of step j (k_step), pend[k] = after the
      // chunk, pend[k + 1] the spill status below (its shards cleared too: a
      // run_fixed before may have added to them)
      rc = pend_clear(0, k + 2);
      if(rc) return rc;
      for(uint32_t j = 0; j < k; ++j)
      {
        par_at[j] = g.par;
        sidx_at[j] = g.sidx;
        rc = launch_step(j, nullptr, nullptr);
        if(rc) return rc;
      }
      par_at[k] = g.par;
      rc = launch_pending(k);
      if(rc) return rc;
      // pend[k + 1]: the spill status, summed over ranks with the counts, so
      // every rank takes the same branch below (one rank: its own status)
      hipLaunchKernelGGL(k_spill_local, dim3(1), dim3(1), 0, g.stream, g.d_pend + k + 1);
      HIPCK(hipGetLastError());
      HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
        g.stream));
      rc = pend_read(0, k + 2, pv);
      if(rc) return rc;
      uint32_t j = 0;
      bool halted = false;
      for(; j < k && before > 0; ++j)
      {
        // one rank: a step the overflow halted; n_ranks > 1 re-runs halted
        // steps inside launch_step, so no summed slot reads as skipped
        if(R() == 1 && pv[j] == kPendSkipped) { halted = true; break; }
        ++done;
        before = pv[j + 1];
      }
      if(halted || pv[k + 1] != 0)
      {
        // steps from j on did not run: resume at the parity step j would have read
        if(halted) { g.par = par_at[j]; g.sidx = sidx_at[j]; }
        rc = fixup_spill();
        if(rc) return rc;
        rc = pending_now(before);
        if(rc) return rc;
      }
    }
  }
  g.steps_total += done;
  if(steps_done) *steps_done = done;
  g.host_seq = 0;     // a new host window starts after each run
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_run(uint64_t max_steps, uint64_t* steps_done)
{
  if(g.async_busy) return GPU_ACTOR_EBUSY;     // without waiting for the lock it holds
  std::lock_guard<std::mutex> lk(g.mu);
  if(g.async_busy) return GPU_ACTOR_EBUSY;
  return run_locked(max_steps, steps_done);
}

GPU_ACTOR_API int gpu_actor_run_async(uint64_t max_steps, gpu_actor_done_fn done, void* ctx)
{
  if(g.async_busy) return GPU_ACTOR_EBUSY;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    if(!g.init) return GPU_ACTOR_ESTATE;
    if(g.async_busy) return GPU_ACTOR_EBUSY;
  }
  join_worker();                      // reap the previous, finished run
  {
  std::lock_guard<std::mutex> lk(g.mu);
  if(g.async_busy) return GPU_ACTOR_EBUSY;
  g.async_busy = true;
  g.async_started = false;
  g.async_rc = 0;
  g.async_steps = 0;
  const int dev = g.device;
  try
  {
    std::lock_guard<std::mutex> wl(g.wmu);
    g.worker = std::thread([max_steps, done, ctx, dev]() {
      int rc;
      uint64_t steps = 0;
      {
        std::lock_guard<std::mutex> wl(g.mu);
        g.async_started = true;
        rc = hipSetDevice(dev) == hipSuccess ? run_locked(max_steps, &steps) : GPU_ACTOR_EHIP;
        g.async_rc = rc;
        g.async_steps = steps;
        g.async_busy = false;
      }
      // outside the lock: the callback may call back into the library
      if(done) done(ctx, rc, steps);
    });
  }
  catch(...)
  {
    g.async_busy = false;
    return GPU_ACTOR_ENOMEM;
  }
  }
  // return only once the progress thread holds the lock, so every later call
  // on this library is serialised behind the run it started
  while(!g.async_started) std::this_thread::yield();
  return 0;
}

GPU_ACTOR_API int gpu_actor_wait(uint64_t* steps_done)
{
  join_worker();
  std::lock_guard<std::mutex> lk(g.mu);
  if(steps_done) *steps_done = g.async_steps;
  const int rc = g.async_rc;
  g.async_rc = 0;
  return rc;
}

GPU_ACTOR_API int gpu_actor_busy(void)
{
  return g.async_busy ? 1 : 0;
}

GPU_ACTOR_API int gpu_actor_run_fixed(uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  if(g.n_zones == 0 || n == 0) return 0;
  // Two events on the engine's stream bracket the n launches: the average
  // step time they give includes each boundary between launches, so it can
  // only overstate the kernel's own duration (events bound to single
  // dispatches slowed those dispatches: r01 measured 94.8 us against a 93.5 us
  // wall step).
  int rc = ensure_events(2);
  if(rc) return rc;
  rc = settle_spills();
  if(rc) return rc;
  uint64_t left = n;
  double ms_total = 0.0;
  while(left)
  {
    // only the slots these launches add to (slot kPendPre is written whole);
    // one rank reads none of them here (its spill status decides), and every
    // reader of a slot clears it first (run, pending_now), so none at all
    if(R() > 1)
    {
      rc = pend_clear(0, (uint32_t)std::min<uint64_t>(left, kPendPre));
      if(rc) return rc;
    }
    const uint32_t par0 = g.par, sidx0 = g.sidx;
    HIPCK(hipEventRecord(g.ev[0], g.stream));
    for(uint64_t j = 0; j < left; ++j)
    {
      rc = launch_step((uint32_t)(j % kPendPre), nullptr, nullptr);
      if(rc) return rc;
    }
    HIPCK(hipEventRecord(g.ev[1], g.stream));
    bool any;
    if(R() == 1)
    {
      // the spill status and the counters (for the sticky errors) in one
      // host round trip
      unsigned long long st[ST_COUNT];
      rc = fold_counters(0, 0);
      if(rc) return rc;
      HIPCK(hipMemcpyAsync(st, g.d_stats, sizeof(st), hipMemcpyDeviceToHost, g.stream));
      rc = read_sstat();                    // synchronises the stream
      if(rc) return rc;
      g.sticky_epoch = g.dev_epoch;
      sticky_from(st);
      any = spill_pending();
    }
    else
    {
      // the same decision on every rank (see settle_spills)
      hipLaunchKernelGGL(k_spill_local, dim3(1), dim3(1), 0, g.stream, g.d_pend + kPendPre);
      HIPCK(hipGetLastError());
      HIPCK(hipMemcpyAsync(g.h_sstat, g.d_sstat, sizeof(Engine::SpillStat), hipMemcpyDeviceToHost,
        g.stream));
      std::vector<unsigned long long> pv;
      rc = pend_read(kPendPre, 1, pv);       // synchronises the stream
      if(rc) return rc;
      any = pv[0] != 0;
    }
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, g.ev[0], g.ev[1]));
    ms_total += ms;
    if(!any) break;
    // steps after an overflow did not run (one rank): grow, then run them
    const uint64_t skipped = std::min<uint64_t>(g.h_sstat->skipped, left);
    const uint64_t ran = left - skipped;
    if(R() == 1 && skipped)
    {
      g.par = par0 ^ (uint32_t)(ran & 1u);
      g.sidx = sidx0 + (uint32_t)ran;
    }
    rc = fixup_spill();
    if(rc) return rc;
    left = skipped;
  }
  g.last_drain_ms = ms_total / (double)n;
  g.steps_total += n;
  g.host_seq = 0;
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_sync(void)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  HIPCK(hipStreamSynchronize(g.stream));
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_state_read(uint32_t type_id, uint64_t first, uint64_t n,
  uint64_t* out)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  if(type_id >= GPU_ACTOR_MAX_TYPES || !out) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.created || first + n > t.lcount) return GPU_ACTOR_EINVAL;
  if(n == 0) return 0;
  // field-major [words][lcount] to [words][n]: one copy (a table type has
  // millions of words and few actors; a copy per word would take minutes)
  if(n == t.lcount)
    HIPCK(hipMemcpyAsync(out, t.d_state, (size_t)t.words * n * sizeof(uint64_t),
      hipMemcpyDeviceToHost, g.stream));
  else
    HIPCK(hipMemcpy2DAsync(out, n * sizeof(uint64_t), t.d_state + first,
      (size_t)t.lcount * sizeof(uint64_t), n * sizeof(uint64_t), t.words, hipMemcpyDeviceToHost,
      g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

GPU_ACTOR_API int gpu_actor_state_write(uint32_t type_id, uint64_t first, uint64_t n,
  const uint64_t* in)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  if(type_id >= GPU_ACTOR_MAX_TYPES || !in) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.created || first + n > t.lcount) return GPU_ACTOR_EINVAL;
  if(n == 0) return 0;
  if(n == t.lcount)
    HIPCK(hipMemcpyAsync(t.d_state, in, (size_t)t.words * n * sizeof(uint64_t),
      hipMemcpyHostToDevice, g.stream));
  else
    HIPCK(hipMemcpy2DAsync(t.d_state + first, (size_t)t.lcount * sizeof(uint64_t), in,
      n * sizeof(uint64_t), n * sizeof(uint64_t), t.words, hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

GPU_ACTOR_API int gpu_actor_counts(gpu_actor_counts_t* out)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  {
    const int frc = flush_sends();
    if(frc) return frc;
  }
  if(!out) return GPU_ACTOR_EINVAL;
  unsigned long long st[ST_COUNT];
  int rc = pend_clear(kPendPre, 1);
  if(rc) return rc;
  rc = fold_counters(0, 0);
  if(rc) return rc;
  rc = launch_pending(kPendPre);
  if(rc) return rc;
  const unsigned long long* src_stats = g.d_stats;
  if(R() > 1)
  {
    // sum counters and pending over ranks into scratch (pend[0 .. ST_COUNT))
    rc = xc_allreduce_sum(g.d_stats, g.d_pend, ST_COUNT, XC_U64);
    if(rc) return rc;
    rc = xc_allreduce_sum(g.d_pend + kPendPre, g.d_pend + kPendPre, 1, XC_U64);
    if(rc) return rc;
    src_stats = g.d_pend;
  }
  HIPCK(hipMemcpyAsync(st, src_stats, sizeof(st), hipMemcpyDeviceToHost, g.stream));
  unsigned long long pend = 0;
  HIPCK(hipMemcpyAsync(&pend, g.d_pend + kPendPre, sizeof(pend), hipMemcpyDeviceToHost,
    g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  memset(out, 0, sizeof(*out));
  out->steps = g.steps_total;
  out->delivered = st[ST_DELIVERED];
  out->sent = st[ST_SENT];
  out->pending = pend;
  out->dropped = st[ST_DROPPED] + st[ST_XCHG_OVERFLOW];
  out->remote = g.remote_total;
  out->active = st[ST_ACTIVE];
  for(int t = 0; t < GPU_ACTOR_MAX_TYPES; ++t) out->delivered_by_type[t] = st[ST_BY_TYPE + t];
  out->atomics = st[ST_ATOMICS];
  return 0;
}

GPU_ACTOR_API uint32_t gpu_actor_owner(uint64_t id)
{
  const uint32_t r = g.cfg.n_ranks ? g.cfg.n_ranks : 1;
  return (uint32_t)(id % r);
}

GPU_ACTOR_API void* gpu_actor_stream(void) { return (void*)g.stream; }

GPU_ACTOR_API double gpu_actor_last_drain_ms(void) { return g.last_drain_ms; }

// Diagnostic (not in the public header): engine internals for tests.
// out[0] spill fixups, [1] k_sparse launches, [2] supersteps run by k_sparse,
// [3] zone buffer records, [4] spill list capacity, [5] zones.
GPU_ACTOR_API int gpu_actor_debug_info(uint64_t* out, uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init || !out) return GPU_ACTOR_ESTATE;
  // + the trigger counts by step index mod 3 (zone_dev.h: read this step's,
  // add to the next's, clear the one after) and the zone geometry
  unsigned int tn[3] = {0, 0, 0};
  if(g.d_trig_n)
  {
    HIPCK(hipMemcpyAsync(tn, g.d_trig_n, sizeof(tn), hipMemcpyDeviceToHost, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
  }
  // + [10] hot zones k_hot gave back to k_step after a missed phase, [11]
  // whether k_hot runs in this engine
  uint32_t hb[4] = {0, 0, 0, 0};
  if(g.d_hot)
  {
    HIPCK(hipMemcpyAsync(hb, hot_bar_words(), sizeof(hb), hipMemcpyDeviceToHost, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
  }
  // + [12] whether the last step ran the module compiled from the programs
  // (jit_host.h), [13] modules built or loaded by this engine
  // + [14] updates k_gups_apply made, [15] the atomics it issued for them
  uint64_t gu[2] = {0, 0};
  if(g.d_gups_stat)
  {
    std::vector<unsigned long long> st(2 * kGupsBlocks);
    HIPCK(hipMemcpyAsync(st.data(), g.d_gups_stat, st.size() * sizeof(unsigned long long),
      hipMemcpyDeviceToHost, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    for(uint32_t b = 0; b < kGupsBlocks; ++b) { gu[0] += st[b]; gu[1] += st[kGupsBlocks + b]; }
  }
  // + [16] whether cross-rank records go straight into the peers' inboxes
  const uint64_t v[17] = {g.fixups, g.sparse_launches, g.sparse_steps, g.zone_records, g.spill_cap,
                          g.n_zones, tn[0], tn[1], tn[2], g.zbits, hb[3], g.hot_on ? 1u : 0u,
                          g.jit_used ? 1u : 0u, g.jit_builds, gu[0], gu[1], g.peer_write ? 1u : 0u};
  for(uint64_t i = 0; i < n && i < 17; ++i) out[i] = v[i];
  return 0;
}

// Diagnostic (not in the public header): compile the step for a program set
// into the code-object cache (jit_host.h) without a device — `nprog` programs,
// types[k] running words[off_k, off_k + lens[k]) (concatenated), at the
// 4096-actor geometry when z12 — so that a later run loads it at once.
// Returns 0, or GPU_ACTOR_EINVAL with hiprtc's log on stderr.
GPU_ACTOR_API int gpu_actor_debug_jit_compile(const uint32_t* types, const uint64_t* words,
  const uint32_t* lens, uint32_t nprog, int z12, const char* arch)
{
  if(!types || !words || !lens || nprog == 0 || nprog > GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  std::vector<jit::Prog> progs;
  uint64_t off = 0;
  for(uint32_t k = 0; k < nprog; ++k)
  {
    if(lens[k] <= GPU_ACTOR_PROG_ENTRIES || lens[k] > jit::kMaxWords) return GPU_ACTOR_EINVAL;
    progs.push_back({types[k], std::vector<uint64_t>(words + off, words + off + lens[k])});
    off += lens[k];
  }
  const std::string src = jit::unit_source(progs, z12 != 0);
  const std::string a = arch && *arch ? arch : "gfx950";
  std::string log;
  const std::string co = jit::code_object(src, a, jit::key_of(src, a), log);
  if(co.empty())
  {
    fprintf(stderr, "gpu_actor jit: %s\n", log.c_str());
    return GPU_ACTOR_EINVAL;
  }
  return 0;
}

// Diagnostic (not in the public header): the same for the any-mix step of a
// mix of compiled tables (bit per table id, jit_host.h build_mix).
GPU_ACTOR_API int gpu_actor_debug_jit_compile_mix(uint32_t mask, int z12, const char* arch)
{
  if(mask == 0) return GPU_ACTOR_EINVAL;
  const std::string src = jit::mix_source(mask, z12 != 0);
  const std::string a = arch && *arch ? arch : "gfx950";
  std::string log;
  if(jit::code_object(src, a, jit::key_of(src, a), log).empty())
  {
    fprintf(stderr, "gpu_actor jit: %s\n", log.c_str());
    return GPU_ACTOR_EINVAL;
  }
  return 0;
}

// Diagnostic (not in the public header): phase stamps of the last k_step of
// a -DGPA_STAMPS build, [n_zones][kDbgSlots] shader-clock values.
GPU_ACTOR_API int gpu_actor_debug_stamps(uint64_t* out, uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init || !out) return GPU_ACTOR_ESTATE;
  n = std::min<uint64_t>(n, (uint64_t)kMaxZones * kDbgSlots);
  HIPCK(hipMemcpyAsync(out, g.d_dbg, n * sizeof(uint64_t), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

// Diagnostic (not in the public header): the RCCL bodies of the four
// cross-rank collectives (xc_allreduce_sum for u8/u32/u64, xc_alltoall_u64,
// xc_allgather_u64) and a grouped ncclSend/ncclRecv — the calls
// xc_sendrecv makes — run once on a one-rank communicator over this engine's
// device (ncclCommInitAll: no bootstrap), on device buffers in the engine's
// stream, exactly as exchange_step calls them. One rank sums to itself, so
// out[] reads back what went in: out[0..4) the u64 sum, [4..8) u32,
// [8..16) u8, [16] all-to-all, [17] all-gather, [18..22) the self
// send/recv's received words; out[22] = the RCCL version. A one-rank engine
// only (the comm is swapped in for the call); returns GPU_ACTOR_ECOMM with the
// failing call on stderr if RCCL refuses.
GPU_ACTOR_API int gpu_actor_debug_rccl_selftest(uint64_t* out, uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init || !out || n < 23) return GPU_ACTOR_EINVAL;
  if(R() != 1 || g.comm || g.xp_ar || g.xp_a2a) return GPU_ACTOR_ESTATE;
  ncclComm_t comm = nullptr;
  int dev = g.device;
  NCCLCK(ncclCommInitAll(&comm, 1, &dev));
  g.comm = comm;
  unsigned long long* d = nullptr;
  int rc = 0;
  auto run = [&]() -> int {
    HIPCK(hipMalloc(&d, 64 * sizeof(unsigned long long)));
    unsigned long long h[64] = {};
    for(int i = 0; i < 4; ++i) h[i] = 0x1000000000ull * (i + 1) + i;           // u64
    uint32_t* h32 = reinterpret_cast<uint32_t*>(h + 4);
    for(int i = 0; i < 4; ++i) h32[i] = 0x10000u * (i + 1) + 7u;               // u32
    uint8_t* h8 = reinterpret_cast<uint8_t*>(h + 8);
    for(int i = 0; i < 64; ++i) h8[i] = (uint8_t)(3 * i + 1);                  // u8
    h[16] = 0xA2A0000000000001ull;                                               // all-to-all
    h[17] = 0xA770000000000002ull;                                               // all-gather
    for(int i = 0; i < 4; ++i) h[24 + i] = 0x5E4D000000000000ull + i;           // send source
    HIPCK(hipMemcpyAsync(d, h, sizeof(h), hipMemcpyHostToDevice, g.stream));
    int r = xc_allreduce_sum(d, d, 4, XC_U64);
    if(!r) r = xc_allreduce_sum(d + 4, d + 4, 8, XC_U32);
    if(!r) r = xc_allreduce_sum(d + 8, d + 8, 64, XC_U8);
    if(!r) r = xc_alltoall_u64(d + 16, d + 32);
    if(!r) r = xc_allgather_u64(d + 17, d + 33);
    if(r) return r;
    NCCLCK(ncclGroupStart());
    NCCLCK(ncclSend(d + 24, 4 * sizeof(unsigned long long), ncclUint8, 0, g.comm, g.stream));
    NCCLCK(ncclRecv(d + 40, 4 * sizeof(unsigned long long), ncclUint8, 0, g.comm, g.stream));
    NCCLCK(ncclGroupEnd());
    HIPCK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, g.stream));
    HIPCK(hipStreamSynchronize(g.stream));
    for(int i = 0; i < 16; ++i) out[i] = h[i];
    out[16] = h[32];
    out[17] = h[33];
    for(int i = 0; i < 4; ++i) out[18 + i] = h[40 + i];
    int ver = 0;
    NCCLCK(ncclGetVersion(&ver));
    out[22] = (uint64_t)ver;
    return 0;
  };
  rc = run();
  if(d) (void)hipFree(d);
  g.comm = nullptr;
  (void)ncclCommDestroy(comm);
  return rc;
}

} // extern "C"

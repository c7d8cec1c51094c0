// engine.hip — the gpu_actor engine: superstep kernels for gfx950 and the C-ABI
// declared in include/gpu_actor.h.
//
// One superstep = k_drain (every actor with visible mail drains up to `batch`
// messages in canonical order and runs its handlers; sends go straight into
// the receivers' HBM rings via one atomicAdd on the receiver's tail, or into a
// per-peer exchange buffer when the receiver lives on another rank) followed by
// k_snapshot (publishes the new tails as next step's visibility bound and
// counts pending mail for the quiescence test). With n_ranks > 1 the exchange
// buffers are swapped with RCCL between the two kernels and k_inject appends
// the received records. This replaces ponyint_actor_run's pop loop
// (actor.c:383-549), messageq push/pop (messageq.c:31-59,234-258), the run
// queue/steal machinery (scheduler.c:752-1090) and per-message pool
// allocation (pool.c:798-889).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "engine_dev.h"

using namespace gpa;

// ===========================================================================
// Kernels
// ===========================================================================

// Drain one actor: `W` state words in registers for the whole drain.
template <int HT>
__device__ __forceinline__ void drain_actor(uint32_t L, const TypeDev& T, ActorCtx& a,
  uint32_t& delivered, unsigned long long* s_agg)
{
  constexpr int W = HT_Words<HT>::W;
  uint32_t head = c_eng.head[L];
  const uint32_t end = c_eng.end[L];
  if(head == end) return;
  uint32_t sorted = c_eng.sorted[L];
  const uint32_t mask = T.cap - 1;
  Rec* ring = T.mb + (size_t)a.li * T.cap;
  const uint32_t avail = end - head;
  const uint32_t w = avail < T.batch ? avail : T.batch;

  uint64_t s[W];
#pragma unroll
  for(int k = 0; k < W; ++k) s[k] = T.state[(size_t)k * T.lcount + a.li];

  uint32_t done = 0;
  // 1. carried-over mail, already canonical
  while(done < w && head + done != sorted)
  {
    const Rec r = ring[(head + done) & mask];
    handle<HT>(T, a, s, r.sb & 0xFFu, r.arg, s_agg);
    ++done;
  }
  // 2. the newest arrival group [sorted, end): deliver in (from, seq) order
  if(sorted != end)
  {
    const uint32_t g = end - sorted;
    const uint32_t q = w - done;
    if(g == 1)
    {
      if(q >= 1)
      {
        const Rec r = ring[sorted & mask];
        handle<HT>(T, a, s, r.sb & 0xFFu, r.arg, s_agg);
        ++done;
      }
    }
    else if(q >= g)
    {
      // whole group handled now: select in key order, no write-back
      uint64_t last = 0;
      for(uint32_t r = 0; r < g; ++r)
      {
        uint64_t best = ~0ull;
        uint32_t bi = 0;
        for(uint32_t j = 0; j < g; ++j)
        {
          const uint64_t k = rec_key(ring + ((sorted + j) & mask));
          if((r == 0 || k > last) && k < best) { best = k; bi = j; }
        }
        const Rec rr = ring[(sorted + bi) & mask];
        handle<HT>(T, a, s, rr.sb & 0xFFu, rr.arg, s_agg);
        last = best;
      }
      done += g;
    }
    else
    {
      // part of the group carries over: canonicalise it in place first
      for(uint32_t i = 1; i < g; ++i)
      {
        const Rec x = ring[(sorted + i) & mask];
        const uint64_t kx = rec_key(&x);
        uint32_t j = i;
        while(j > 0)
        {
          const Rec y = ring[(sorted + j - 1) & mask];
          if(rec_key(&y) <= kx) break;
          ring[(sorted + j) & mask] = y;
          --j;
        }
        ring[(sorted + j) & mask] = x;
      }
      for(uint32_t k = 0; k < q; ++k)
      {
        const Rec r = ring[(sorted + k) & mask];
        handle<HT>(T, a, s, r.sb & 0xFFu, r.arg, s_agg);
      }
      done += q;
    }
    sorted = end;
  }

#pragma unroll
  for(int k = 0; k < W; ++k) T.state[(size_t)k * T.lcount + a.li] = s[k];
  c_eng.head[L] = head + done;
  c_eng.sorted[L] = sorted;
  delivered += done;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
  for(int off = 32; off > 0; off >>= 1)
    v += __shfl_xor(v, off);
  return v;
}

__global__ void __launch_bounds__(kBlock) k_drain()
{
  __shared__ unsigned long long s_agg[kWaves];
  const uint32_t L = blockIdx.x * kBlock + threadIdx.x;
  uint32_t delivered = 0;
  ActorCtx a;
  a.seq = 0; a.sent = 0; a.applied = 0; a.applied_type = -1;
  int t = -1;
  if(L < c_eng.n_local)
  {
    t = type_of_local(L);
    if(t >= 0 && !c_types[t].reducible)
    {
      const TypeDev& T = c_types[t];
      a.li = L - T.lfirst;
      a.self = L * c_eng.nranks + c_eng.rank;
      switch(T.ht)
      {
        case GPU_ACTOR_HT_RING:          drain_actor<GPU_ACTOR_HT_RING>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_PINGER:        drain_actor<GPU_ACTOR_HT_PINGER>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_PINGER_DET:    drain_actor<GPU_ACTOR_HT_PINGER_DET>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_FANIN_SENDER:  drain_actor<GPU_ACTOR_HT_FANIN_SENDER>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_GUPS_STREAMER: drain_actor<GPU_ACTOR_HT_GUPS_STREAMER>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_STORM:         drain_actor<GPU_ACTOR_HT_STORM>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_FIFO_SRC:      drain_actor<GPU_ACTOR_HT_FIFO_SRC>(L, T, a, delivered, s_agg); break;
        case GPU_ACTOR_HT_FIFO_SINK:     drain_actor<GPU_ACTOR_HT_FIFO_SINK>(L, T, a, delivered, s_agg); break;
        default: break;
      }
    }
  }
  // counters: one atomic per wave per counter (convergent here)
  const unsigned long long d = wave_sum(delivered);
  const unsigned long long snt = wave_sum(a.sent);
  const unsigned long long ap = wave_sum(a.applied);
  const unsigned long long so = wave_sum(a.seq >= kSeqLimit ? 1ull : 0ull);
  const unsigned long long act = wave_sum(delivered ? 1ull : 0ull);
  // per-type delivered: uniform type per wave is the common case
  const int t0 = __builtin_amdgcn_readfirstlane(t);
  const bool uniform = __all(t == t0);
  const int lane = __lane_id();
  if(lane == 0)
  {
    if(d + ap) atomicAdd(&c_eng.stats[ST_DELIVERED], d + ap);
    if(snt) atomicAdd(&c_eng.stats[ST_SENT], snt);
    if(so) atomicAdd(&c_eng.stats[ST_SEQ_OVERFLOW], so);
    if(act) atomicAdd(&c_eng.stats[ST_ACTIVE], act);
    if(uniform && d && t0 >= 0) atomicAdd(&c_eng.stats[ST_BY_TYPE + t0], d);
  }
  if(!uniform && delivered && t >= 0)
    atomicAdd(&c_eng.stats[ST_BY_TYPE + t], (unsigned long long)delivered);
  // local applies to a reducible type (one target type per handler table)
  if(a.applied && a.applied_type >= 0)
    atomicAdd(&c_eng.stats[ST_BY_TYPE + a.applied_type], (unsigned long long)a.applied);
}

// Publish next step's visibility bound and count pending mail.
__global__ void __launch_bounds__(kBlock) k_snapshot(uint32_t slot)
{
  __shared__ unsigned long long s_red[kWaves];
  const uint32_t L = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long pend = 0;
  if(L < c_eng.n_local)
  {
    const int t = type_of_local(L);
    if(t >= 0 && !c_types[t].reducible)
    {
      const uint32_t tail = c_eng.tail[L];
      const uint32_t head = c_eng.head[L];
      c_eng.end[L] = tail;
      c_eng.lim[L] = head + c_types[t].cap;
      pend = tail - head;
    }
  }
  pend = wave_sum(pend);
  if(__lane_id() == 0) s_red[threadIdx.x >> 6] = pend;
  __syncthreads();
  if(threadIdx.x == 0)
  {
    unsigned long long tot = 0;
    for(int w = 0; w < kWaves; ++w) tot += s_red[w];
    if(tot) atomicAdd(&c_eng.pend[slot], tot);
  }
}

// Host sends (pony_sendv from outside the runtime): hseq gives the canonical
// order; records are appended exactly like device sends.
__global__ void __launch_bounds__(kBlock) k_inject(const gpu_msg_t* msgs, uint64_t n,
  uint64_t hseq_base)
{
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  const gpu_msg_t m = msgs[i];
  const uint64_t hseq = hseq_base + i;
  const uint32_t from = kHostFrom | (uint32_t)(hseq >> 24);
  const uint32_t sb = (uint32_t)((hseq & 0xFFFFFFull) << 8) | (m.behaviour & 0xFFu);
  if(c_eng.nranks > 1 && m.to % c_eng.nranks != c_eng.rank) return;   // not ours
  const int t = type_of_global(m.to);
  if(t < 0) return;
  if(c_types[t].reducible)
  {
    reducible_apply_local(m.to, m.behaviour, m.arg);
    atomicAdd(&c_eng.stats[ST_DELIVERED], 1ull);
    atomicAdd(&c_eng.stats[ST_BY_TYPE + t], 1ull);
    return;
  }
  ring_push(m.to, sb, from, m.arg);
}

// Records received from other ranks.
__global__ void __launch_bounds__(kBlock) k_xinject(const XRec* in, uint64_t n)
{
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  const XRec x = in[i];
  if(x.beh_only)
    reducible_apply_local(x.to, x.sb, x.arg);
  else
    ring_push(x.to, x.sb, x.from, x.arg);
}

// Reducible deliveries that arrived from other ranks are counted at the
// receiver so per-type counts stay exact under sharding.
__global__ void k_xcount(const XRec* in, uint64_t n)
{
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if(i >= n) return;
  if(in[i].beh_only)
  {
    const int t = type_of_global(in[i].to);
    atomicAdd(&c_eng.stats[ST_DELIVERED], 1ull);
    if(t >= 0) atomicAdd(&c_eng.stats[ST_BY_TYPE + t], 1ull);
  }
}

// pony_create's constructor run: initial state of a freshly created type.
__global__ void __launch_bounds__(kBlock) k_construct(uint32_t t)
{
  const TypeDev& T = c_types[t];
  const uint32_t li = blockIdx.x * kBlock + threadIdx.x;
  if(li >= T.lcount) return;
  const uint32_t L = T.lfirst + li;
  const uint64_t i = (uint64_t)L * c_eng.nranks + c_eng.rank - T.first;   // index in type
  const size_t n = T.lcount;
  uint64_t* st = T.state;
  c_eng.head[L] = 0; c_eng.sorted[L] = 0; c_eng.end[L] = 0; c_eng.tail[L] = 0;
  c_eng.lim[L] = T.reducible ? 0u : T.cap;
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
    case GPU_ACTOR_HT_GUPS_UPDATER: {
      const uint64_t size = T.params[0];
      for(uint64_t k = 0; k < size && k < T.words; ++k) st[k * n + li] = k + i * size;
      break;
    }
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

// ===========================================================================
// Host side
// ===========================================================================

namespace {

constexpr uint32_t kChunk = 16;          // steps between quiescence readbacks
constexpr uint32_t kPendSlots = 4096;    // pend[] entries (chunk + run_fixed)

struct HostType {
  bool registered = false, created = false;
  uint32_t words = 0, ht = 0, batch = 0, cap = 0;
  uint64_t params[GPU_ACTOR_MAX_PARAMS] = {};
  uint64_t first = 0, count = 0;
  uint32_t lfirst = 0, lcount = 0;
  uint64_t* d_state = nullptr;
  Rec* d_mb = nullptr;
};

struct Engine {
  std::mutex mu;
  bool init = false;
  gpu_actor_config_t cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  HostType types[GPU_ACTOR_MAX_TYPES];
  uint32_t n_types = 0;                 // 1 + highest created type id
  uint64_t n_actors = 0;                // global ids handed out
  uint32_t n_local = 0, local_cap = 0;
  uint32_t *d_head = nullptr, *d_sorted = nullptr, *d_end = nullptr, *d_lim = nullptr,
           *d_tail = nullptr;
  unsigned long long* d_stats = nullptr;
  unsigned long long* d_pend = nullptr;
  gpu_msg_t* h_msgs = nullptr; uint64_t h_msgs_cap = 0;
  gpu_msg_t* d_msgs = nullptr; uint64_t d_msgs_cap = 0;
  uint64_t host_seq = 0;
  uint64_t steps_total = 0;
  int sticky = 0;
  hipError_t last_hip = hipSuccess;
  std::vector<hipEvent_t> ev;
  double last_drain_ms = 0.0;
  // multi-rank exchange
  ncclComm_t comm = nullptr;
  XRec* d_xout = nullptr;
  XRec* d_xin = nullptr;
  unsigned long long* d_xcount = nullptr;
  unsigned long long* d_xrecv = nullptr;   // counts from each peer
  uint32_t xcap = 0;
  std::vector<unsigned long long> h_xcount, h_xrecv;
  uint64_t remote_total = 0;
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

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

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
    d.reducible = (h.ht == GPU_ACTOR_HT_FANIN_ANALYZER || h.ht == GPU_ACTOR_HT_GUPS_UPDATER);
    d.state = h.d_state; d.mb = h.d_mb;
    memcpy(d.params, h.params, sizeof(d.params));
  }
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_types), td, sizeof(td), 0,
    hipMemcpyHostToDevice, g.stream));
  EngDev e;
  memset(&e, 0, sizeof(e));
  e.n_types = g.n_types; e.rank = rank(); e.nranks = R(); e.n_local = g.n_local;
  e.head = g.d_head; e.sorted = g.d_sorted; e.end = g.d_end; e.lim = g.d_lim; e.tail = g.d_tail;
  e.stats = g.d_stats; e.pend = g.d_pend;
  e.xout = g.d_xout; e.xcount = g.d_xcount; e.xcap = g.xcap;
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_eng), &e, sizeof(e), 0,
    hipMemcpyHostToDevice, g.stream));
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
    default: return 0;
  }
}

int check_sticky()
{
  unsigned long long st[ST_COUNT];
  HIPCK(hipMemcpyAsync(st, g.d_stats, sizeof(st), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  if(st[ST_DROPPED] || st[ST_XCHG_OVERFLOW]) g.sticky = GPU_ACTOR_EMAILBOX;
  else if(st[ST_SEQ_OVERFLOW]) g.sticky = GPU_ACTOR_ERANGE;
  return g.sticky;
}

// Cross-rank exchange of this step's remote records (RCCL over xGMI):
// counts all-to-all, then grouped point-to-point record transfers, then
// k_xinject appends them. Requires two small D2H reads of counts.
int exchange()
{
  const uint32_t n = R();
  HIPCK(hipMemcpyAsync(g.h_xcount.data(), g.d_xcount, n * sizeof(unsigned long long),
    hipMemcpyDeviceToHost, g.stream));
  NCCLCK(ncclAllToAll(g.d_xcount, g.d_xrecv, 1, ncclUint64, g.comm, g.stream));
  HIPCK(hipMemcpyAsync(g.h_xrecv.data(), g.d_xrecv, n * sizeof(unsigned long long),
    hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  uint64_t off = 0;
  std::vector<uint64_t> roff(n);
  for(uint32_t p = 0; p < n; ++p)
  {
    roff[p] = off;
    off += std::min<unsigned long long>(g.h_xrecv[p], g.xcap);
  }
  NCCLCK(ncclGroupStart());
  for(uint32_t p = 0; p < n; ++p)
  {
    if(p == rank()) continue;
    const uint64_t sc = std::min<unsigned long long>(g.h_xcount[p], g.xcap);
    const uint64_t rc = std::min<unsigned long long>(g.h_xrecv[p], g.xcap);
    if(sc) NCCLCK(ncclSend(g.d_xout + (size_t)p * g.xcap, sc * sizeof(XRec), ncclUint8, p,
      g.comm, g.stream));
    if(rc) NCCLCK(ncclRecv(g.d_xin + roff[p], rc * sizeof(XRec), ncclUint8, p, g.comm,
      g.stream));
  }
  NCCLCK(ncclGroupEnd());
  const uint64_t total = off;
  g.remote_total += total;
  if(total)
  {
    hipLaunchKernelGGL(k_xinject, dim3(blocks_for(total)), dim3(kBlock), 0, g.stream,
      g.d_xin, total);
    hipLaunchKernelGGL(k_xcount, dim3(blocks_for(total)), dim3(kBlock), 0, g.stream,
      g.d_xin, total);
    HIPCK(hipGetLastError());
  }
  HIPCK(hipMemsetAsync(g.d_xcount, 0, n * sizeof(unsigned long long), g.stream));
  return 0;
}

int launch_step(uint32_t slot, hipEvent_t e0, hipEvent_t e1)
{
  const uint32_t nb = blocks_for(g.n_local);
  if(nb == 0) return 0;
  if(e0) HIPCK(hipEventRecord(e0, g.stream));
  hipLaunchKernelGGL(k_drain, dim3(nb), dim3(kBlock), 0, g.stream);
  if(e1) HIPCK(hipEventRecord(e1, g.stream));
  HIPCK(hipGetLastError());
  if(R() > 1)
  {
    int rc = exchange();
    if(rc) return rc;
  }
  hipLaunchKernelGGL(k_snapshot, dim3(nb), dim3(kBlock), 0, g.stream, slot);
  HIPCK(hipGetLastError());
  return 0;
}

// Sum of pending over all ranks for pend[slot] entries (host side, after sync).
int pend_read(uint32_t first, uint32_t n, std::vector<unsigned long long>& out)
{
  out.resize(n);
  if(R() > 1)
  {
    NCCLCK(ncclAllReduce(g.d_pend + first, g.d_pend + first, n, ncclUint64, ncclSum, g.comm,
      g.stream));
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
  for(auto& t : g.types)
  {
    if(t.d_state) (void)hipFree(t.d_state);
    if(t.d_mb) (void)hipFree(t.d_mb);
  }
  uint32_t* u32s[] = { g.d_head, g.d_sorted, g.d_end, g.d_lim, g.d_tail };
  for(uint32_t* p : u32s) if(p) (void)hipFree(p);
  if(g.d_stats) (void)hipFree(g.d_stats);
  if(g.d_pend) (void)hipFree(g.d_pend);
  if(g.h_msgs) (void)hipHostFree(g.h_msgs);
  if(g.d_msgs) (void)hipFree(g.d_msgs);
  if(g.d_xout) (void)hipFree(g.d_xout);
  if(g.d_xin) (void)hipFree(g.d_xin);
  if(g.d_xcount) (void)hipFree(g.d_xcount);
  if(g.d_xrecv) (void)hipFree(g.d_xrecv);
  for(hipEvent_t e : g.ev) (void)hipEventDestroy(e);
  if(g.comm) (void)ncclCommDestroy(g.comm);
  if(g.stream) (void)hipStreamDestroy(g.stream);
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
  if(g.cfg.rank >= g.cfg.n_ranks) return GPU_ACTOR_EINVAL;
  if(g.cfg.batch == 0) g.cfg.batch = 100;                 // PONY_SCHED_BATCH
  if(g.cfg.mailbox_cap == 0) g.cfg.mailbox_cap = 64;
  if(g.cfg.mailbox_cap & (g.cfg.mailbox_cap - 1)) return GPU_ACTOR_EINVAL;
  if(g.cfg.max_actors == 0) g.cfg.max_actors = 1ull << 26;
  if(g.cfg.max_actors > 0xFF000000ull) return GPU_ACTOR_EINVAL;

  int ndev = 0;
  if(hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GPU_ACTOR_ENODEV;
  g.device = cfg->device >= 0 ? cfg->device : 0;
  if(cfg->device < 0) (void)hipGetDevice(&g.device);
  if(g.device >= ndev) return GPU_ACTOR_ENODEV;
  HIPCK(hipSetDevice(g.device));
  HIPCK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));

  g.local_cap = (uint32_t)((g.cfg.max_actors + R() - 1) / R());
  const size_t lb = (size_t)g.local_cap * sizeof(uint32_t);
  HIPCK(hipMalloc(&g.d_head, lb));
  HIPCK(hipMalloc(&g.d_sorted, lb));
  HIPCK(hipMalloc(&g.d_end, lb));
  HIPCK(hipMalloc(&g.d_lim, lb));
  HIPCK(hipMalloc(&g.d_tail, lb));
  HIPCK(hipMalloc(&g.d_stats, ST_COUNT * sizeof(unsigned long long)));
  HIPCK(hipMemsetAsync(g.d_stats, 0, ST_COUNT * sizeof(unsigned long long), g.stream));
  HIPCK(hipMalloc(&g.d_pend, kPendSlots * sizeof(unsigned long long)));

  if(R() > 1)
  {
    if(!cfg->comm_id) return GPU_ACTOR_EINVAL;
    ncclUniqueId id;
    memcpy(&id, cfg->comm_id, sizeof(id));
    NCCLCK(ncclCommInitRank(&g.comm, (int)R(), id, (int)rank()));
    g.xcap = g.cfg.max_exchange ? g.cfg.max_exchange : (1u << 22);
    HIPCK(hipMalloc(&g.d_xout, (size_t)R() * g.xcap * sizeof(XRec)));
    HIPCK(hipMalloc(&g.d_xin, (size_t)R() * g.xcap * sizeof(XRec)));
    HIPCK(hipMalloc(&g.d_xcount, R() * sizeof(unsigned long long)));
    HIPCK(hipMalloc(&g.d_xrecv, R() * sizeof(unsigned long long)));
    HIPCK(hipMemsetAsync(g.d_xcount, 0, R() * sizeof(unsigned long long), g.stream));
    g.h_xcount.assign(R(), 0);
    g.h_xrecv.assign(R(), 0);
  }
  g.init = true;
  int rc = upload_types();
  if(rc) return rc;
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

GPU_ACTOR_API int gpu_actor_shutdown(void)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(g.stream) (void)hipStreamSynchronize(g.stream);
  free_all();
  // reset to a pristine engine (mutex stays)
  for(auto& t : g.types) t = HostType();
  g.init = false; g.n_types = 0; g.n_actors = 0; g.n_local = 0; g.local_cap = 0;
  g.d_head = g.d_sorted = g.d_end = g.d_lim = g.d_tail = nullptr;
  g.d_stats = g.d_pend = nullptr;
  g.h_msgs = nullptr; g.h_msgs_cap = 0; g.d_msgs = nullptr; g.d_msgs_cap = 0;
  g.host_seq = 0; g.steps_total = 0; g.sticky = 0; g.ev.clear(); g.last_drain_ms = 0;
  g.comm = nullptr; g.d_xout = g.d_xin = nullptr; g.d_xcount = g.d_xrecv = nullptr;
  g.xcap = 0; g.remote_total = 0; g.stream = nullptr;
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
  if(t.created && mailbox_cap && mailbox_cap != t.cap) return GPU_ACTOR_EINVAL;
  if(mailbox_cap & (mailbox_cap - 1)) return GPU_ACTOR_EINVAL;
  if(batch) t.batch = batch;
  if(mailbox_cap) t.cap = mailbox_cap;
  return t.created ? upload_types() : 0;
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

GPU_ACTOR_API int gpu_actor_create(uint32_t type_id, uint64_t count, uint64_t* first_id)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.registered || t.created || count == 0) return GPU_ACTOR_EINVAL;
  if(g.n_actors + count > g.cfg.max_actors) return GPU_ACTOR_ERANGE;
  if(t.ht == GPU_ACTOR_HT_GUPS_UPDATER)
  {
    const uint64_t size = t.params[0];
    if(size == 0 || (size & (size - 1)) || size > t.words) return GPU_ACTOR_EINVAL;
  }
  t.first = g.n_actors;
  t.count = count;
  const uint64_t lo = owned_below(t.first), hi = owned_below(t.first + count);
  t.lfirst = (uint32_t)lo;
  t.lcount = (uint32_t)(hi - lo);
  const size_t lc = std::max<size_t>(t.lcount, 1);
  HIPCK(hipMalloc(&t.d_state, (size_t)t.words * lc * sizeof(uint64_t)));
  HIPCK(hipMemsetAsync(t.d_state, 0, (size_t)t.words * lc * sizeof(uint64_t), g.stream));
  const bool reducible = (t.ht == GPU_ACTOR_HT_FANIN_ANALYZER || t.ht == GPU_ACTOR_HT_GUPS_UPDATER);
  if(!reducible)
    HIPCK(hipMalloc(&t.d_mb, lc * t.cap * sizeof(Rec)));
  t.created = true;
  g.n_actors += count;
  g.n_local = (uint32_t)owned_below(g.n_actors);
  g.n_types = std::max(g.n_types, type_id + 1);
  int rc = upload_types();
  if(rc) return rc;
  if(t.lcount)
  {
    hipLaunchKernelGGL(k_construct, dim3(blocks_for(t.lcount)), dim3(kBlock), 0, g.stream,
      type_id);
    HIPCK(hipGetLastError());
  }
  HIPCK(hipStreamSynchronize(g.stream));
  if(first_id) *first_id = t.first;
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

static int sendv_locked(const gpu_msg_t* first, uint64_t n)
{
  if(n == 0) return 0;
  if(!first) return GPU_ACTOR_EINVAL;
  for(uint64_t i = 0; i < n; ++i)
    if(first[i].to >= g.n_actors || first[i].behaviour > 0xFF) return GPU_ACTOR_EINVAL;
  if(g.host_seq + n >= (1ull << 48)) return GPU_ACTOR_ERANGE;
  if(n > g.d_msgs_cap)
  {
    if(g.d_msgs) HIPCK(hipFree(g.d_msgs));
    g.d_msgs = nullptr;
    HIPCK(hipMalloc(&g.d_msgs, n * sizeof(gpu_msg_t)));
    g.d_msgs_cap = n;
  }
  HIPCK(hipMemcpyAsync(g.d_msgs, first, n * sizeof(gpu_msg_t), hipMemcpyHostToDevice, g.stream));
  hipLaunchKernelGGL(k_inject, dim3(blocks_for(n)), dim3(kBlock), 0, g.stream,
    (const gpu_msg_t*)g.d_msgs, n, g.host_seq);
  HIPCK(hipGetLastError());
  g.host_seq += n;
  HIPCK(hipStreamSynchronize(g.stream));    // caller may reuse its buffer
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
  if(to >= g.n_actors) return GPU_ACTOR_EINVAL;
  return sendv_locked(&m, 1);
}

GPU_ACTOR_API int gpu_actor_run(uint64_t max_steps, uint64_t* steps_done)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  const uint32_t nb = blocks_for(g.n_local);
  uint64_t done = 0;
  if(nb)
  {
    // slot kPendSlots-1: pending before the first step
    HIPCK(hipMemsetAsync(g.d_pend, 0, kPendSlots * sizeof(unsigned long long), g.stream));
    hipLaunchKernelGGL(k_snapshot, dim3(nb), dim3(kBlock), 0, g.stream, kPendSlots - 1);
    HIPCK(hipGetLastError());
    std::vector<unsigned long long> pv;
    int rc = pend_read(kPendSlots - 1, 1, pv);
    if(rc) return rc;
    unsigned long long before = pv[0];
    while(before > 0 && (max_steps == 0 || done < max_steps))
    {
      uint32_t k = kChunk;
      if(max_steps) k = (uint32_t)std::min<uint64_t>(k, max_steps - done);
      HIPCK(hipMemsetAsync(g.d_pend, 0, k * sizeof(unsigned long long), g.stream));
      for(uint32_t j = 0; j < k; ++j)
      {
        rc = launch_step(j, nullptr, nullptr);
        if(rc) return rc;
      }
      rc = pend_read(0, k, pv);
      if(rc) return rc;
      for(uint32_t j = 0; j < k && before > 0; ++j)
      {
        ++done;
        before = pv[j];
      }
    }
  }
  g.steps_total += done;
  if(steps_done) *steps_done = done;
  g.host_seq = 0;     // a new host window starts after each run
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_run_fixed(uint64_t n)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  const uint32_t nb = blocks_for(g.n_local);
  if(nb == 0 || n == 0) return 0;
  const uint64_t timed = std::min<uint64_t>(n, 2048);
  int rc = ensure_events(2 * timed);
  if(rc) return rc;
  HIPCK(hipMemsetAsync(g.d_pend, 0, kPendSlots * sizeof(unsigned long long), g.stream));
  hipLaunchKernelGGL(k_snapshot, dim3(nb), dim3(kBlock), 0, g.stream, kPendSlots - 1);
  for(uint64_t j = 0; j < n; ++j)
  {
    const bool tm = j >= n - timed;
    const uint64_t e = j - (n - timed);
    rc = launch_step((uint32_t)(j % (kPendSlots - 1)), tm ? g.ev[2 * e] : nullptr,
      tm ? g.ev[2 * e + 1] : nullptr);
    if(rc) return rc;
  }
  HIPCK(hipStreamSynchronize(g.stream));
  double tot = 0.0;
  for(uint64_t e = 0; e < timed; ++e)
  {
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, g.ev[2 * e], g.ev[2 * e + 1]));
    tot += ms;
  }
  g.last_drain_ms = tot / (double)timed;
  g.steps_total += n;
  g.host_seq = 0;
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_sync(void)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  HIPCK(hipStreamSynchronize(g.stream));
  return check_sticky();
}

GPU_ACTOR_API int gpu_actor_state_read(uint32_t type_id, uint64_t first, uint64_t n,
  uint64_t* out)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !out) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.created || first + n > t.lcount) return GPU_ACTOR_EINVAL;
  if(n == 0) return 0;
  for(uint32_t w = 0; w < t.words; ++w)
    HIPCK(hipMemcpyAsync(out + (size_t)w * n, t.d_state + (size_t)w * t.lcount + first,
      n * sizeof(uint64_t), hipMemcpyDeviceToHost, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

GPU_ACTOR_API int gpu_actor_state_write(uint32_t type_id, uint64_t first, uint64_t n,
  const uint64_t* in)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(type_id >= GPU_ACTOR_MAX_TYPES || !in) return GPU_ACTOR_EINVAL;
  HostType& t = g.types[type_id];
  if(!t.created || first + n > t.lcount) return GPU_ACTOR_EINVAL;
  if(n == 0) return 0;
  for(uint32_t w = 0; w < t.words; ++w)
    HIPCK(hipMemcpyAsync(t.d_state + (size_t)w * t.lcount + first, in + (size_t)w * n,
      n * sizeof(uint64_t), hipMemcpyHostToDevice, g.stream));
  HIPCK(hipStreamSynchronize(g.stream));
  return 0;
}

GPU_ACTOR_API int gpu_actor_counts(gpu_actor_counts_t* out)
{
  std::lock_guard<std::mutex> lk(g.mu);
  if(!g.init) return GPU_ACTOR_ESTATE;
  if(!out) return GPU_ACTOR_EINVAL;
  unsigned long long st[ST_COUNT];
  const uint32_t nb = blocks_for(g.n_local);
  HIPCK(hipMemsetAsync(g.d_pend + kPendSlots - 1, 0, sizeof(unsigned long long), g.stream));
  if(nb)
  {
    hipLaunchKernelGGL(k_snapshot, dim3(nb), dim3(kBlock), 0, g.stream, kPendSlots - 1);
    HIPCK(hipGetLastError());
  }
  const unsigned long long* src_stats = g.d_stats;
  if(R() > 1)
  {
    // sum counters and pending over ranks into scratch (pend[0 .. ST_COUNT])
    NCCLCK(ncclAllReduce(g.d_stats, g.d_pend, ST_COUNT, ncclUint64, ncclSum, g.comm, g.stream));
    NCCLCK(ncclAllReduce(g.d_pend + kPendSlots - 1, g.d_pend + kPendSlots - 1, 1, ncclUint64,
      ncclSum, g.comm, g.stream));
    src_stats = g.d_pend;
  }
  HIPCK(hipMemcpyAsync(st, src_stats, sizeof(st), hipMemcpyDeviceToHost, g.stream));
  unsigned long long pend = 0;
  HIPCK(hipMemcpyAsync(&pend, g.d_pend + kPendSlots - 1, sizeof(pend), hipMemcpyDeviceToHost,
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
  return 0;
}

GPU_ACTOR_API uint32_t gpu_actor_owner(uint64_t id)
{
  const uint32_t r = g.cfg.n_ranks ? g.cfg.n_ranks : 1;
  return (uint32_t)(id % r);
}

GPU_ACTOR_API void* gpu_actor_stream(void) { return (void*)g.stream; }

GPU_ACTOR_API double gpu_actor_last_drain_ms(void) { return g.last_drain_ms; }

} // extern "C"

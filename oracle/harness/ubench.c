/*
 * harness/ubench.c — TEST INFRASTRUCTURE ONLY. examples/message-ubench Pingers
 * on the reference runtime, with the workload made deterministic:
 *   --det 0 : faithful Pinger.ping/send_pings (message-ubench/main.pony:265-286)
 *             with a seeded Rand(seed+i+1, 0x9E3779B97F4A7C15) primed by three
 *             int(100) (main.pony:244-249) and a per-pinger forward budget B
 *             in place of the timer. Every ping is identical, so a pinger's
 *             state is a function of how many pings it has received: the
 *             network is abelian and its final state is schedule-independent.
 *   --det 1 : message-ubench-det: token<<32|hop payloads routed
 *             by splitmix64(seed ^ payload), H hops.
 * SyncLeader's role (tell_all_to_go, main.pony:201-218) is played by main():
 * each pinger receives I initial pings. Usage:
 *   harness_ubench --pingers N --initial I [--budget B | --det 1 --hops H]
 *                  [--seed S] [--threads T] [--out file]
 *                  [--warm-ms M --window-ms W]
 * Output (field-major u64): faithful: x, y, count; det: count, acc.
 *
 * Steady state (--window-ms W > 0, faithful form): no forward budget; as the
 * reference's report interval does (main.pony:86-88, Tick 288-299), a timer
 * thread lets the cascade run M ms, then counts the pings handled during
 * the next W ms (sum of the pingers' counts read at both ends), then stops
 * the pingers forwarding (Pinger.stop: _go = false, main.pony:257-259) so the
 * runtime drains and pony_start returns. The JSON line then carries
 * window_msgs_per_sec beside the whole-run figure.
 */
#include "harness.h"
#include <pthread.h>
#include <unistd.h>

enum { PING = 0 };

typedef struct pinger_t {
  pony_actor_pad_t pad;
  or_xoro_t rand;          /* _rand */
  uint64_t count;          /* _count */
  uint64_t acc;
  uint64_t idx;
} pinger_t;

static pinger_t** g_ps;    /* _ps */
static uint64_t g_n, g_budget, g_hops, g_seed;
static int g_det;
static uint64_t *g_x, *g_y, *g_count, *g_acc;
static volatile int g_stop;        /* steady state: Pinger._go cleared */
static uint64_t g_warm_ms, g_window_ms;
static double g_win_secs;
static uint64_t g_win_msgs;

static void pinger_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  pinger_t* p = (pinger_t*)self;
  uint64_t payload = (uint64_t)((pony_msgi_t*)m)->i;
  if(!g_det)
  {
    /* be ping(payload): _count = _count + 1; send_pings() while in budget */
    p->count += 1;
    if(p->count <= g_budget && !g_stop)
    {
      uint64_t k = or_rand_int(&p->rand, g_n);         /* _rand.int(_num_ps) */
      pony_sendi(ctx, (pony_actor_t*)g_ps[k], PING, 42);
    }
  } else {
    p->count += 1;
    p->acc ^= payload;
    uint64_t hop = payload & 0xFFFFFFFFULL;
    if(hop < g_hops)
    {
      uint64_t k = or_mulhi(or_splitmix_mix(g_seed ^ payload), g_n);
      pony_sendi(ctx, (pony_actor_t*)g_ps[k], PING,
        (intptr_t)((payload & 0xFFFFFFFF00000000ULL) | (hop + 1)));
    }
  }
}

/* a pinger's state to the output arrays (its finaliser, or after the run) */
static void pinger_out(const pinger_t* p)
{
  g_x[p->idx] = p->rand.x; g_y[p->idx] = p->rand.y;
  g_count[p->idx] = p->count; g_acc[p->idx] = p->acc;
}

static void pinger_final(void* self)
{
  const pinger_t* p = (const pinger_t*)self;
  pinger_out(p);
  h_fin[p->idx] = 1;
}

static pony_type_t pinger_type = { .id = 2, .size = sizeof(pinger_t), .dispatch = pinger_dispatch,
  .final = pinger_final };

/* pings handled so far: the pingers' counts, read in the live actors while
 * they run (rc = GC_INC_MORE: none is reaped during the run; each word is
 * written by its own pinger, and a read may be one ping stale) */
static uint64_t count_sum(void)
{
  uint64_t s = 0;
  for(uint64_t i = 0; i < g_n; i++) s += __atomic_load_n(&g_ps[i]->count, __ATOMIC_RELAXED);
  return s;
}

static void* window_timer(void* arg)
{
  (void)arg;
  usleep((useconds_t)(g_warm_ms * 1000));
  double t0 = h_now();
  uint64_t c0 = count_sum();
  usleep((useconds_t)(g_window_ms * 1000));
  double t1 = h_now();
  uint64_t c1 = count_sum();
  g_win_secs = t1 - t0;
  g_win_msgs = c1 - c0;
  g_stop = 1;
  return NULL;
}

int main(int argc, char** argv)
{
  g_n = h_arg(argc, argv, "--pingers", 8);
  uint64_t initial = h_arg(argc, argv, "--initial", 5);
  g_budget = h_arg(argc, argv, "--budget", 100);
  g_det = (int)h_arg(argc, argv, "--det", 0);
  g_hops = h_arg(argc, argv, "--hops", 32);
  g_seed = h_arg(argc, argv, "--seed", 5489);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");
  g_warm_ms = h_arg(argc, argv, "--warm-ms", 2000);
  g_window_ms = h_arg(argc, argv, "--window-ms", 0);
  if(g_window_ms && !g_det) g_budget = ~0ULL;

  g_ps = calloc(g_n, sizeof(pinger_t*));
  g_x = calloc(g_n, 8); g_y = calloc(g_n, 8); g_count = calloc(g_n, 8); g_acc = calloc(g_n, 8);
  h_fin = calloc(g_n, 1);

  pony_ctx_t* ctx = h_start(threads, noscale);

  for(uint64_t i = 0; i < g_n; i++)
  {
    pinger_t* p = (pinger_t*)pony_create(ctx, &pinger_type);
    p->idx = i;
    p->count = 0;
    p->acc = 0;
    if(!g_det)
    {
      or_xoro_create(&p->rand, g_seed + i + 1, 0x9E3779B97F4A7C15ULL);
      (void)or_rand_int(&p->rand, 100);
      (void)or_rand_int(&p->rand, 100);
      (void)or_rand_int(&p->rand, 100);
    }
    g_ps[i] = p;
  }
  /* tell_all_to_go: for i in initial: for p in ps: p.ping(payload) */
  for(uint64_t k = 0; k < initial; k++)
    for(uint64_t i = 0; i < g_n; i++)
    {
      uint64_t payload = g_det ? ((i * initial + k) << 32) : 42;
      pony_sendi(ctx, (pony_actor_t*)g_ps[i], PING, (intptr_t)payload);
    }

  pthread_t timer;
  const int windowed = g_window_ms && !g_det;
  if(windowed) pthread_create(&timer, NULL, window_timer, NULL);
  double secs = h_run(ctx);
  if(windowed) pthread_join(timer, NULL);
  for(uint64_t i = 0; i < g_n; i++)
    if(!h_fin[i]) pinger_out(g_ps[i]);

  uint64_t total = 0;
  for(uint64_t i = 0; i < g_n; i++) total += g_count[i];
  if(windowed)
  {
    printf("{\"harness\": \"ubench_steady\", \"threads\": %d, \"seconds\": %.6f, "
      "\"msgs\": %llu, \"msgs_per_sec\": %.1f, \"warm_ms\": %llu, \"window_seconds\": %.6f, "
      "\"window_msgs\": %llu, \"window_msgs_per_sec\": %.1f}\n", threads, secs,
      (unsigned long long)total, secs > 0 ? (double)total / secs : 0.0,
      (unsigned long long)g_warm_ms, g_win_secs, (unsigned long long)g_win_msgs,
      g_win_secs > 0 ? (double)g_win_msgs / g_win_secs : 0.0);
    fflush(stdout);
    return 0;
  }
  h_report(g_det ? "ubench_det" : "ubench", threads, secs, total);
  if(!g_det)
  {
    const uint64_t* f[3] = { g_x, g_y, g_count };
    return h_dump(out, f, 3, g_n);
  }
  const uint64_t* f[2] = { g_count, g_acc };
  return h_dump(out, f, 2, g_n);
}

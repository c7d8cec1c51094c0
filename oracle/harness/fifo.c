/*
 * harness/fifo.c — TEST INFRASTRUCTURE ONLY. Per-pair FIFO probe on the
 * reference runtime, the property CodegenOptimisationTest.
 * MergeSendMessageReordering pins (test/libponyc/codegen_optimisation.cc:13-41).
 * Source i sends `bursts` rounds of m PUSH(i << 32 | seq) to sink i % n_sinks,
 * re-sending BURST to itself between rounds. Each sink counts per-source
 * sequence breaks. The FNV fold h is interleaving-dependent on the CPU and is
 * reported only for information. Usage:
 *   harness_fifo --sources S --sinks K --bursts B --m M [--threads T] [--out f]
 * Output (field-major u64, K sinks): h, n, violations.
 */
#include "harness.h"

enum { BURST = 0, PUSH = 1 };

typedef struct sink_t {
  pony_actor_pad_t pad;
  uint64_t h, n, bad, last[8];
  uint64_t idx;
} sink_t;

typedef struct src_t {
  pony_actor_pad_t pad;
  sink_t* target;
  uint64_t seq, bursts, idx;
} src_t;

static uint64_t g_nsinks;
static uint64_t *g_h, *g_n, *g_bad;

static void sink_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  (void)ctx;
  sink_t* k = (sink_t*)self;
  uint64_t arg = (uint64_t)((pony_msgi_t*)m)->i;
  uint64_t slot = ((arg >> 32) / g_nsinks) % 8;
  uint64_t seq = arg & 0xFFFFFFFFULL;
  k->n += 1;
  k->h = (k->h ^ arg) * 0x100000001b3ULL;
  if(seq != k->last[slot] + 1) k->bad += 1;
  k->last[slot] = seq;
}

static sink_t** g_sinks;

static void sink_out(const sink_t* k)
{
  g_h[k->idx] = k->h; g_n[k->idx] = k->n; g_bad[k->idx] = k->bad;
}

static void sink_final(void* self)
{
  const sink_t* k = (const sink_t*)self;
  sink_out(k);
  h_fin[k->idx] = 1;
}

static void src_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  src_t* s = (src_t*)self;
  intptr_t burst = ((pony_msgi_t*)m)->i;
  for(intptr_t j = 0; j < burst; j++)
  {
    s->seq += 1;
    pony_sendi(ctx, (pony_actor_t*)s->target, PUSH, (intptr_t)((s->idx << 32) | s->seq));
  }
  if(s->bursts > 0) s->bursts -= 1;
  if(s->bursts > 0)
    pony_sendi(ctx, self, BURST, burst);
}

static pony_type_t sink_type = { .id = 7, .size = sizeof(sink_t), .dispatch = sink_dispatch,
  .final = sink_final };
static pony_type_t src_type = { .id = 8, .size = sizeof(src_t), .dispatch = src_dispatch };

int main(int argc, char** argv)
{
  uint64_t nsrc = h_arg(argc, argv, "--sources", 64);
  g_nsinks = h_arg(argc, argv, "--sinks", 8);
  uint64_t bursts = h_arg(argc, argv, "--bursts", 10);
  uint64_t mm = h_arg(argc, argv, "--m", 4);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");

  g_h = calloc(g_nsinks, 8); g_n = calloc(g_nsinks, 8); g_bad = calloc(g_nsinks, 8);
  sink_t** sinks = calloc(g_nsinks, sizeof(sink_t*));
  g_sinks = sinks;
  h_fin = calloc(g_nsinks, 1);

  pony_ctx_t* ctx = h_start(threads, noscale);
  for(uint64_t k = 0; k < g_nsinks; k++)
  {
    sink_t* s = (sink_t*)pony_create(ctx, &sink_type);
    s->h = 0xcbf29ce484222325ULL;
    s->idx = k;
    sinks[k] = s;
  }
  for(uint64_t i = 0; i < nsrc; i++)
  {
    src_t* s = (src_t*)pony_create(ctx, &src_type);
    s->target = sinks[i % g_nsinks];
    s->seq = 0;
    s->bursts = bursts;
    s->idx = i;
    pony_sendi(ctx, (pony_actor_t*)s, BURST, (intptr_t)mm);
  }

  double secs = h_run(ctx);
  for(uint64_t k = 0; k < g_nsinks; k++)
    if(!h_fin[k]) sink_out(g_sinks[k]);

  uint64_t total = 0;
  for(uint64_t k = 0; k < g_nsinks; k++) total += g_n[k];
  h_report("fifo", threads, secs, total + nsrc * bursts);
  const uint64_t* f[3] = { g_h, g_n, g_bad };
  return h_dump(out, f, 3, g_nsinks);
}

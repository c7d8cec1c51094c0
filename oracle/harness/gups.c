/*
 * harness/gups.c — TEST INFRASTRUCTURE ONLY. examples/gups_basic on the
 * reference runtime (gups_basic/main.pony:40-216). Streamer i draws
 * PolyRand(chunk * iterate * i) (main.pony:73-75) and, for iterate+1 calls of
 * apply, routes `chunk` data to Updater (d >> shift) & mask, which does
 * table[d & (size-1)] ^= d.
 *   --batched 1 (default): one Array[U64] message per updater per chunk, as the
 *                          reference does (main.pony:120-136);
 *   --batched 0          : one message per datum (the gpu_actor formulation).
 * Usage: harness_gups --logtable L --updaters U --streamers S --chunk C
 *                     --iterate I [--batched 0|1] [--threads T] [--out file]
 * Output: the whole table (U * size u64), updater-major.
 */
#include "harness.h"

enum { UPD_APPLY = 0, UPD_ONE = 1, STR_APPLY = 0 };

typedef struct updater_t {
  pony_actor_pad_t pad;
  uint64_t* table;
  uint64_t size;
} updater_t;

typedef struct streamer_t {
  pony_actor_pad_t pad;
  or_polyrand_t rand;
  uint64_t shift, mask, chunk;
} streamer_t;

/* Array[U64] val payload for the batched form (owned by the message). */
typedef struct { uint64_t n; uint64_t d[]; } batch_t;

static updater_t** g_up;
static uint64_t** g_tables;   /* table pointers outlive the actors */
static uint64_t g_nup;
static int g_batched;
static volatile uint64_t g_updates;

static void updater_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  (void)ctx;
  updater_t* u = (updater_t*)self;
  if(m->id == UPD_APPLY)
  {
    batch_t* b = (batch_t*)((pony_msgp_t*)m)->p;
    for(uint64_t k = 0; k < b->n; k++)
    {
      uint64_t d = b->d[k];
      uint64_t i = d & (u->size - 1);
      u->table[i] ^= d;
    }
    free(b);
  } else {
    uint64_t d = (uint64_t)((pony_msgi_t*)m)->i;
    u->table[d & (u->size - 1)] ^= d;
  }
}

static void streamer_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  streamer_t* s = (streamer_t*)self;
  intptr_t iterate = ((pony_msgi_t*)m)->i;
  if(g_batched)
  {
    batch_t** list = malloc(g_nup * sizeof(batch_t*));
    for(uint64_t i = 0; i < g_nup; i++)
    {
      list[i] = malloc(sizeof(batch_t) + s->chunk * sizeof(uint64_t));
      list[i]->n = 0;
    }
    for(uint64_t c = 0; c < s->chunk; c++)
    {
      uint64_t d = or_polyrand_next(&s->rand);
      uint64_t up = (d >> s->shift) & s->mask;
      list[up]->d[list[up]->n++] = d;
    }
    for(uint64_t i = 0; i < g_nup; i++)
    {
      if(list[i]->n > 0)
        pony_sendp(ctx, (pony_actor_t*)g_up[i], UPD_APPLY, list[i]);
      else
        free(list[i]);
    }
    free(list);
  } else {
    for(uint64_t c = 0; c < s->chunk; c++)
    {
      uint64_t d = or_polyrand_next(&s->rand);
      uint64_t up = (d >> s->shift) & s->mask;
      pony_sendi(ctx, (pony_actor_t*)g_up[up], UPD_ONE, (intptr_t)d);
    }
  }
  __atomic_fetch_add(&g_updates, s->chunk, __ATOMIC_RELAXED);
  if(iterate > 0)
    pony_sendi(ctx, self, STR_APPLY, iterate - 1);
}

static pony_type_t updater_type = { .id = 5, .size = sizeof(updater_t), .dispatch = updater_dispatch };
static pony_type_t streamer_type = { .id = 6, .size = sizeof(streamer_t), .dispatch = streamer_dispatch };

int main(int argc, char** argv)
{
  uint64_t logtable = h_arg(argc, argv, "--logtable", 20);
  g_nup = h_arg(argc, argv, "--updaters", 8);
  uint64_t nstr = h_arg(argc, argv, "--streamers", 4);
  uint64_t chunk = h_arg(argc, argv, "--chunk", 1024);
  uint64_t iterate = h_arg(argc, argv, "--iterate", 10000);
  g_batched = (int)h_arg(argc, argv, "--batched", 1);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");

  uint64_t size = (1ULL << logtable) / g_nup;             /* main.pony:57 */
  g_up = calloc(g_nup, sizeof(updater_t*));
  g_tables = calloc(g_nup, sizeof(uint64_t*));

  pony_ctx_t* ctx = h_start(threads, noscale);
  for(uint64_t i = 0; i < g_nup; i++)
  {
    updater_t* u = (updater_t*)pony_create(ctx, &updater_type);
    u->size = size;
    u->table = malloc(size * sizeof(uint64_t));
    for(uint64_t k = 0; k < size; k++) u->table[k] = k + i * size;   /* 148-155 */
    g_up[i] = u;
    g_tables[i] = u->table;
  }
  uint64_t shift = (uint64_t)(64 - __builtin_clzll(size));          /* 102 */
  for(uint64_t i = 0; i < nstr; i++)
  {
    streamer_t* s = (streamer_t*)pony_create(ctx, &streamer_type);
    or_polyrand_create(&s->rand, chunk * iterate * i);
    s->shift = shift;
    s->mask = g_nup - 1;
    s->chunk = chunk;
    pony_sendi(ctx, (pony_actor_t*)s, STR_APPLY, (intptr_t)iterate);
  }

  double secs = h_run(ctx);

  h_report(g_batched ? "gups_batched" : "gups", threads, secs, g_updates);
  if(out[0])
  {
    FILE* f = fopen(out, "wb");
    if(!f) { perror(out); return 1; }
    for(uint64_t i = 0; i < g_nup; i++)
      fwrite(g_tables[i], sizeof(uint64_t), size, f);
    fclose(f);
  }
  return 0;
}

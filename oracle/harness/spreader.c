/*
 * harness/spreader.c — TEST INFRASTRUCTURE ONLY. examples/spreader on the
 * reference runtime (spreader/main.pony:1-52): Spreader actors created by
 * behaviours — pony_create inside a behaviour, then the constructor
 * (`new spread(parent, count)`) delivered as the new actor's first message,
 * which is how generated code calls a constructor on a new actor
 * (gencall.c:606-612). Usage:
 *   harness_spreader --count C [--threads T] [--out file]
 * Output (field-major u64, 2^C - 1 entries each): every node's final _result,
 * sorted ascending; then [0] = the root's printed total (_result + 1), rest 0.
 * Actor identities are runtime pointers, so the tree is compared through the
 * multiset of node results and the total.
 */
#include "harness.h"

enum { SPREAD = 0, RESULT = 1 };

typedef struct spreader_t {
  pony_actor_pad_t pad;
  uint64_t count;                 /* _count */
  struct spreader_t* parent;      /* _parent: (Spreader | None) */
  uint64_t result;                /* _result */
  uint64_t received;              /* _received */
} spreader_t;

typedef struct {                  /* new spread(parent: Spreader, count: U64) */
  pony_msg_t msg;
  spreader_t* parent;
  uint64_t count;
} spread_msg_t;

static uint64_t* g_res;           /* final _result of each node, in finishing order */
static uint64_t g_nres;           /* atomic cursor */
static uint64_t g_total;          /* the root's print */
static uint64_t g_msgs;           /* behaviours run (for the rate line) */

static void record(uint64_t r)
{
  g_res[__atomic_fetch_add(&g_nres, 1, __ATOMIC_RELAXED)] = r;
}

static pony_type_t spreader_type;

/* fun spawn_child() => Spreader.spread(this, _count - 1) */
static void spawn_child(pony_ctx_t* ctx, spreader_t* self)
{
  spreader_t* c = (spreader_t*)pony_create(ctx, &spreader_type);
  spread_msg_t* m = (spread_msg_t*)pony_alloc_msg_size(sizeof(spread_msg_t), SPREAD);
  m->parent = self;
  m->count = self->count - 1;
  pony_sendv_single(ctx, (pony_actor_t*)c, &m->msg, &m->msg, true);
}

static void spreader_dispatch(pony_ctx_t* ctx, pony_actor_t* actor, pony_msg_t* msg)
{
  spreader_t* self = (spreader_t*)actor;
  __atomic_fetch_add(&g_msgs, 1, __ATOMIC_RELAXED);
  switch(msg->id)
  {
    case SPREAD: {                                /* main.pony:9-32 */
      spread_msg_t* m = (spread_msg_t*)msg;
      self->parent = m->parent;
      self->count = m->count;
      if(self->count <= 1)
      {
        record(0);                                /* a leaf keeps _result = 0 */
        if(self->parent != NULL)
          pony_sendi(ctx, (pony_actor_t*)self->parent, RESULT, 1);
        else
          g_total = 1;                            /* "1 actor" */
      }
      else
      {
        spawn_child(ctx, self);
        spawn_child(ctx, self);
      }
      break;
    }
    case RESULT: {                                /* main.pony:34-45 */
      self->received += 1;
      self->result += (uint64_t)((pony_msgi_t*)msg)->i;
      if(self->received == 2)
      {
        record(self->result);
        if(self->parent != NULL)
          pony_sendi(ctx, (pony_actor_t*)self->parent, RESULT, (intptr_t)(self->result + 1));
        else
          g_total = self->result + 1;             /* "<n> actors" */
      }
      break;
    }
  }
}

static pony_type_t spreader_type = { .id = 1, .size = sizeof(spreader_t),
  .dispatch = spreader_dispatch };

static int cmp_u64(const void* a, const void* b)
{
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv)
{
  uint64_t count = h_arg(argc, argv, "--count", 10);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");

  const uint64_t n = (1ull << count) - 1;
  g_res = calloc(n, sizeof(uint64_t));
  uint64_t* tot = calloc(n, sizeof(uint64_t));

  pony_ctx_t* ctx = h_start(threads, noscale);
  /* Main.create: Spreader(env) — the root's constructor, with no parent */
  spreader_t* root = (spreader_t*)pony_create(ctx, &spreader_type);
  spread_msg_t* m = (spread_msg_t*)pony_alloc_msg_size(sizeof(spread_msg_t), SPREAD);
  m->parent = NULL;
  m->count = count;
  pony_sendv_single(ctx, (pony_actor_t*)root, &m->msg, &m->msg, true);
  double secs = h_run(ctx);

  if(g_nres != n)
    fprintf(stderr, "spreader: %llu of %llu nodes finished\n", (unsigned long long)g_nres,
      (unsigned long long)n);
  qsort(g_res, n, sizeof(uint64_t), cmp_u64);
  tot[0] = g_total;
  h_report("spreader", threads, secs, g_msgs);
  const uint64_t* f[2] = { g_res, tot };
  return h_dump(out, f, 2, n);
}

/*
 * harness/ring.c — TEST INFRASTRUCTURE ONLY. examples/ring/main.pony on the
 * reference runtime. Usage:
 *   harness_ring --size S --count R --pass P [--threads T] [--out file]
 * Output (field-major u64, actor index = ring*S + (id-1)): recv, done.
 */
#include "harness.h"

enum { RING_SET = 0, RING_PASS = 1 };

typedef struct ring_t {
  pony_actor_pad_t pad;
  struct ring_t* next;     /* _next: (Ring | None) */
  uint32_t id;             /* _id */
  uint64_t idx;            /* ring*S + id-1 (harness bookkeeping) */
  uint64_t recv, done;     /* passes received; _env.out.print(_id) count */
} ring_t;

static uint64_t* g_recv;
static uint64_t* g_done;
static ring_t** g_rings;

static void ring_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  ring_t* r = (ring_t*)self;
  switch(m->id)
  {
    case RING_SET:                                   /* be set(neighbor) */
      r->next = (ring_t*)((pony_msgp_t*)m)->p;
      break;
    case RING_PASS: {                                /* be pass(i) */
      intptr_t i = ((pony_msgi_t*)m)->i;
      r->recv++;
      if(i > 0)
      {
        if(r->next != NULL)
          pony_sendi(ctx, (pony_actor_t*)r->next, RING_PASS, i - 1);
      } else {
        r->done++;                                   /* _env.out.print(_id) */
      }
      break;
    }
  }
}

static void ring_out(const ring_t* r)
{
  g_recv[r->idx] = r->recv; g_done[r->idx] = r->done;
}

static void ring_final(void* self)
{
  const ring_t* r = (const ring_t*)self;
  ring_out(r);
  h_fin[r->idx] = 1;
}

static pony_type_t ring_type = { .id = 1, .size = sizeof(ring_t), .dispatch = ring_dispatch,
  .final = ring_final };

int main(int argc, char** argv)
{
  uint32_t size = (uint32_t)h_arg(argc, argv, "--size", 3);
  uint32_t count = (uint32_t)h_arg(argc, argv, "--count", 1);
  uint64_t pass = h_arg(argc, argv, "--pass", 10);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");

  uint64_t n = (uint64_t)size * count;
  g_recv = calloc(n, sizeof(uint64_t));
  g_done = calloc(n, sizeof(uint64_t));
  g_rings = calloc(n, sizeof(ring_t*));
  h_fin = calloc(n, 1);

  pony_ctx_t* ctx = h_start(threads, noscale);

  /* setup_ring (ring/main.pony:61-72) */
  for(uint32_t j = 0; j < count; j++)
  {
    ring_t* first = (ring_t*)pony_create(ctx, &ring_type);
    first->id = 1; first->next = NULL; first->idx = (uint64_t)j * size;
    first->recv = 0; first->done = 0;
    g_rings[first->idx] = first;
    ring_t* next = first;
    for(uint32_t k = 0; k + 1 < size; k++)
    {
      ring_t* cur = (ring_t*)pony_create(ctx, &ring_type);
      cur->id = size - k;
      cur->next = next;
      cur->idx = (uint64_t)j * size + (cur->id - 1);
      cur->recv = 0; cur->done = 0;
      g_rings[cur->idx] = cur;
      next = cur;
    }
    pony_sendp(ctx, (pony_actor_t*)first, RING_SET, next);
    if(pass > 0)
      pony_sendi(ctx, (pony_actor_t*)first, RING_PASS, (intptr_t)pass);
  }

  double secs = h_run(ctx);
  for(uint64_t a = 0; a < n; a++)
    if(!h_fin[a]) ring_out(g_rings[a]);

  uint64_t total = 0;
  for(uint64_t a = 0; a < n; a++) total += g_recv[a];
  h_report("ring", threads, secs, total);
  const uint64_t* f[2] = { g_recv, g_done };
  return h_dump(out, f, 2, n);
}

/*
 * harness/fanin.c — TEST INFRASTRUCTURE ONLY. examples/fan-in Senders and
 * Analyzers on the reference runtime (fan-in/main.pony:212-254): each Sender
 * re-sends send_msgs() to itself and, per call, one msg_from_sender() to
 * _analyzers(_rand.int_unbiased(size)). The timer-driven `done()` is replaced
 * by P messages per sender; msg_from_sender carries (sender << 32 | n) so the
 * analyzers can also fold an XOR checksum. Usage:
 *   harness_fanin --senders S --analyzers A --msgs P [--seedmode 0|1]
 *                 [--threads T] [--out file]
 * Output (field-major u64): analyzer count, analyzer acc (A each).
 */
#include "harness.h"

enum { SEND_MSGS = 0, MSG_FROM_SENDER = 1 };

typedef struct analyzer_t {
  pony_actor_pad_t pad;
  uint64_t msgs_received;   /* _msgs_received */
  uint64_t acc;
  uint64_t idx;
} analyzer_t;

typedef struct sender_t {
  pony_actor_pad_t pad;
  or_xoro_t rand;           /* _rand: Rand = Rand() */
  uint64_t remaining;
  uint64_t sent;
  uint64_t idx;
} sender_t;

static analyzer_t** g_an;
static uint64_t g_na;
static uint64_t *g_count, *g_acc;

static void analyzer_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  (void)ctx;
  analyzer_t* a = (analyzer_t*)self;
  a->msgs_received += 1;                                   /* main.pony:219-220 */
  a->acc ^= (uint64_t)((pony_msgi_t*)m)->i;
}

static void analyzer_out(const analyzer_t* a)
{
  g_count[a->idx] = a->msgs_received;
  g_acc[a->idx] = a->acc;
}

static void analyzer_final(void* self)
{
  const analyzer_t* a = (const analyzer_t*)self;
  analyzer_out(a);
  h_fin[a->idx] = 1;
}

static void sender_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{
  (void)m;
  sender_t* s = (sender_t*)self;
  /* be send_msgs() (main.pony:241-250) */
  uint64_t k = or_rand_int_unbiased(&s->rand, g_na);
  pony_sendi(ctx, (pony_actor_t*)g_an[k], MSG_FROM_SENDER, (intptr_t)((s->idx << 32) | s->sent));
  s->sent += 1;
  if(s->remaining > 0) s->remaining -= 1;
  if(s->remaining > 0)
    pony_send(ctx, self, SEND_MSGS);
}

static pony_type_t analyzer_type = { .id = 3, .size = sizeof(analyzer_t), .dispatch = analyzer_dispatch,
  .final = analyzer_final };
static pony_type_t sender_type = { .id = 4, .size = sizeof(sender_t), .dispatch = sender_dispatch };

int main(int argc, char** argv)
{
  uint64_t ns = h_arg(argc, argv, "--senders", 1000);
  g_na = h_arg(argc, argv, "--analyzers", 4);
  uint64_t p = h_arg(argc, argv, "--msgs", 100);
  int seedmode = (int)h_arg(argc, argv, "--seedmode", 0);
  int threads = (int)h_arg(argc, argv, "--threads", 1);
  int noscale = (int)h_arg(argc, argv, "--noscale", 0);
  const char* out = h_sarg(argc, argv, "--out", "");

  g_an = calloc(g_na, sizeof(analyzer_t*));
  g_count = calloc(g_na, 8); g_acc = calloc(g_na, 8);
  h_fin = calloc(g_na, 1);

  pony_ctx_t* ctx = h_start(threads, noscale);
  for(uint64_t i = 0; i < g_na; i++)
  {
    analyzer_t* a = (analyzer_t*)pony_create(ctx, &analyzer_type);
    a->idx = i;
    g_an[i] = a;
  }
  for(uint64_t i = 0; i < ns; i++)
  {
    sender_t* s = (sender_t*)pony_create(ctx, &sender_type);
    or_xoro_create(&s->rand, seedmode ? 5489 + i : 5489, 0);
    s->remaining = p;
    s->sent = 0;
    s->idx = i;
    /* Sender.create calls send_msgs(): a message to itself */
    pony_send(ctx, (pony_actor_t*)s, SEND_MSGS);
  }

  double secs = h_run(ctx);
  for(uint64_t i = 0; i < g_na; i++)
    if(!h_fin[i]) analyzer_out(g_an[i]);

  uint64_t total = 0;
  for(uint64_t i = 0; i < g_na; i++) total += g_count[i];
  /* handler invocations: every analyzer message plus every send_msgs call */
  h_report("fanin", threads, secs, total + ns * p);
  const uint64_t* f[2] = { g_count, g_acc };
  return h_dump(out, f, 2, g_na);
}

/*
 * bsp.c — TEST INFRASTRUCTURE ONLY: single-threaded bulk-synchronous
 * restatement of the gpu_actor engine semantics (include/gpu_actor.h), used by
 * tests/ as the parity checker for the HIP engine. Written independently of
 * ponyc_amd/csrc: it restates the reference behaviours (file:line cited at each
 * handler) over the engine's delivery rules:
 *
 *   - step s visits actors in ascending id order (the canonical order);
 *   - an actor handles min(batch, mail pending at the start of s) messages
 *     from the head of its mailbox (actor.c:437-471, batch = PONY_SCHED_BATCH
 *     actor.c:20 or the per-type override, actor.c:410-416);
 *   - an emitted message is appended to the receiver's mailbox and is first
 *     visible in step s+1; so each step's arrivals are ordered by
 *     (sender id, sender sequence), after carried-over mail;
 *   - mailboxes are unbounded (as the reference's messageq is): nothing is
 *     ever dropped; `cap` only sizes the engine's first buffers;
 *   - messages to "reducible" types (all behaviours commutative) are applied
 *     when sent;
 *   - host sends are appended in call order (ids above every actor).
 *
 * Not thread-safe; one simulator per process.
 */
#include "oracle.h"
#include "../include/gpu_actor.h"

#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t beh; uint64_t arg; } orec_t;

typedef struct {
  orec_t*  buf;
  uint64_t cap_alloc;
  uint64_t head;          /* index of next message to handle (absolute)     */
  uint64_t tail;          /* number of messages ever appended (absolute)     */
  uint64_t tail0;         /* tail when step `stamp` started (appends in it wait) */
  uint64_t stamp;         /* step of the first append this step, + 1         */
} mbox_t;

/* Backpressure state of one actor (actor.c:340-381, 898-921, scheduler.c:
 * 1496-1635, restated for supersteps — see or_run): overloaded after the
 * last step it ran, muted, and the receiver it is muted on. */
typedef struct {
  uint8_t  o, m;
  uint32_t r;
} oflag_t;

typedef struct {
  int      registered, created;
  uint32_t words, ht, batch, cap, reducible;
  int32_t  priority;      /* the fork's _priority() hint (actor.c:414-416)   */
  uint64_t params[GPU_ACTOR_MAX_PARAMS];
  uint64_t first, count;  /* id range [first, first + count): created + reserve */
  uint64_t live;          /* created + spawned so far                        */
  uint64_t reserve;       /* room for actors spawned by behaviours           */
  uint64_t* state;        /* field-major: state[w * count + i] */
  uint64_t delivered;
  uint64_t* prog;         /* GPU_ACTOR_HT_PROGRAM: the behaviours' program */
  uint32_t prog_n;
} otype_t;

/* an actor created by a behaviour this step: id assigned at the step's end */
typedef struct { uint32_t type, beh; uint64_t arg; } ospawn_t;

static struct {
  int       init;
  otype_t   types[GPU_ACTOR_MAX_TYPES];
  uint64_t  n_actors;
  uint8_t*  type_of;      /* actor id -> type id */
  mbox_t*   mb;
  uint64_t  steps, delivered, sent, dropped;
  ospawn_t* spawns;       /* this step's, in (creator id, call order) order */
  uint64_t  n_spawns, spawns_alloc;
  /* backpressure: flags, the previous step's end state per actor (bit 0
   * overloaded, bit 1 muted: either triggers muting), and the actors a step
   * must visit (mail, muted or overloaded), as a bitmap scanned in id order */
  oflag_t*  fl;
  uint8_t*  trig;
  uint64_t  n_trig;
  uint64_t* live;
  uint64_t  pending;
  /* the actor running now, for send() */
  uint64_t  cur;
  int       cur_prev_o, mute_hit, yield_req, running;
  uint64_t  mute_to;
} S;

static const uint32_t DEFAULT_BATCH = 100;   /* PONY_SCHED_BATCH, actor.c:20 */
static const uint32_t DEFAULT_CAP = 16;   /* engine's initial zone sizing; no limit here */

static int ht_reducible(uint32_t ht)
{
  return ht == GPU_ACTOR_HT_FANIN_ANALYZER || ht == GPU_ACTOR_HT_GUPS_UPDATER;
}

int or_init(uint32_t n_types_max)
{
  (void)n_types_max;
  if(S.init) or_shutdown();
  memset(&S, 0, sizeof(S));
  S.init = 1;
  return 0;
}

void or_shutdown(void)
{
  for(int t = 0; t < GPU_ACTOR_MAX_TYPES; t++)
  {
    free(S.types[t].state);
    free(S.types[t].prog);
  }
  for(uint64_t a = 0; a < S.n_actors; a++)
    free(S.mb[a].buf);
  free(S.mb);
  free(S.type_of);
  free(S.spawns);
  free(S.fl);
  free(S.trig);
  free(S.live);
  memset(&S, 0, sizeof(S));
}

int or_type_reserve(uint32_t type_id, uint64_t n)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || !S.types[type_id].registered ||
    S.types[type_id].created) return GPU_ACTOR_EINVAL;
  S.types[type_id].reserve = n;
  return 0;
}

int or_type_live(uint32_t type_id, uint64_t* out)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || !S.types[type_id].created) return GPU_ACTOR_EINVAL;
  *out = S.types[type_id].live;
  return 0;
}

int or_type_register(uint32_t type_id, uint32_t state_words, uint32_t ht)
{
  if(!S.init || type_id >= GPU_ACTOR_MAX_TYPES || ht < 1 || ht > GPU_ACTOR_HT_PROGRAM) return GPU_ACTOR_EINVAL;
  if(ht == GPU_ACTOR_HT_PROGRAM && state_words < 8) return GPU_ACTOR_EINVAL;
  otype_t* t = &S.types[type_id];
  if(t->registered) return GPU_ACTOR_EINVAL;
  t->registered = 1;
  t->words = state_words;
  t->ht = ht;
  t->batch = DEFAULT_BATCH;
  t->cap = DEFAULT_CAP;
  t->reducible = (uint32_t)ht_reducible(ht);
  return 0;
}

int or_type_config(uint32_t type_id, uint32_t batch, uint32_t cap)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || !S.types[type_id].registered) return GPU_ACTOR_EINVAL;
  if(batch) S.types[type_id].batch = batch;
  if(cap) S.types[type_id].cap = cap;
  return 0;
}

/* scheduler.c:1053-1068: a rescheduled actor that outranks the next runnable
 * one keeps running; every default (0) actor ranks below a positive priority */
int or_type_priority(uint32_t type_id, int32_t priority)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || !S.types[type_id].registered) return GPU_ACTOR_EINVAL;
  S.types[type_id].priority = priority;
  return 0;
}

/* gpu_actor_type_program: the behaviours of a GPU_ACTOR_HT_PROGRAM type */
int or_type_program(uint32_t type_id, const uint64_t* code, uint32_t n)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || !S.types[type_id].registered ||
     S.types[type_id].ht != GPU_ACTOR_HT_PROGRAM || !code || n <= GPU_ACTOR_PROG_ENTRIES ||
     n > (1u << 20)) return GPU_ACTOR_EINVAL;
  uint64_t* p = malloc((size_t)n * sizeof(uint64_t));
  if(!p) return GPU_ACTOR_ENOMEM;
  memcpy(p, code, (size_t)n * sizeof(uint64_t));
  free(S.types[type_id].prog);
  S.types[type_id].prog = p;
  S.types[type_id].prog_n = n;
  return 0;
}

int or_type_param(uint32_t type_id, uint32_t idx, uint64_t value)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES || idx >= GPU_ACTOR_MAX_PARAMS ||
    !S.types[type_id].registered) return GPU_ACTOR_EINVAL;
  S.types[type_id].params[idx] = value;
  return 0;
}

/* ---- constructors (the reference `new create`) --------------------------- */
static void construct(uint32_t tid)
{
  otype_t* t = &S.types[tid];
  uint64_t n = t->count;
  uint64_t* st = t->state;
  for(uint64_t i = 0; i < t->live; i++)    /* reserved actors start zeroed */
  {
    switch(t->ht)
    {
      case GPU_ACTOR_HT_RING: {
        /* ring/main.pony:61-72: Ring(1) first, then Ring(size-k) whose
         * neighbour is the previously created actor; id m -> id m+1 -> ... */
        uint64_t size = t->params[0] ? t->params[0] : 1;
        uint64_t ring = i / size, p = i % size;
        st[0 * n + i] = (p == 0) ? GPU_ACTOR_NONE : t->first + ring * size + (p + 1) % size;
        st[1 * n + i] = p + 1;
        break;
      }
      case GPU_ACTOR_HT_PINGER: {
        /* message-ubench/main.pony:244-249 with a seeded Rand. */
        or_xoro_t r;
        or_xoro_create(&r, t->params[3] + i + 1, 0x9E3779B97F4A7C15ULL);
        (void)or_rand_int(&r, 100); (void)or_rand_int(&r, 100); (void)or_rand_int(&r, 100);
        st[0 * n + i] = r.x; st[1 * n + i] = r.y;
        break;
      }
      case GPU_ACTOR_HT_FANIN_SENDER: {
        /* fan-in/main.pony:235: `let _rand: Rand = Rand()` -> Rand(5489, 0). */
        or_xoro_t r;
        or_xoro_create(&r, t->params[3] ? 5489 + i : 5489, 0);
        st[0 * n + i] = r.x; st[1 * n + i] = r.y;
        st[2 * n + i] = t->params[2];
        break;
      }
      case GPU_ACTOR_HT_GUPS_STREAMER: {
        or_polyrand_t pr;
        or_polyrand_create(&pr, t->params[5] * i);
        st[0 * n + i] = pr.last;
        break;
      }
      case GPU_ACTOR_HT_GUPS_UPDATER: {
        /* gups_basic/main.pony:148-155: table[k] = k + index*size. */
        uint64_t size = t->params[0];
        for(uint64_t k = 0; k < size && k < t->words; k++)
          st[k * n + i] = k + i * size;
        break;
      }
      case GPU_ACTOR_HT_FIFO_SRC: {
        uint64_t ns = t->params[1] ? t->params[1] : 1;
        st[0 * n + i] = t->params[0] + i % ns;
        st[2 * n + i] = t->params[2];
        break;
      }
      case GPU_ACTOR_HT_FIFO_SINK:
        st[0 * n + i] = 0xcbf29ce484222325ULL;
        break;
      default:
        break;
    }
  }
}

int or_create(uint32_t type_id, uint64_t count, uint64_t* first_id)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  otype_t* t = &S.types[type_id];
  if(!t->registered || t->created) return GPU_ACTOR_EINVAL;
  const uint64_t live = count;
  count += t->reserve;
  uint64_t total = S.n_actors + count;
  uint8_t* to = realloc(S.type_of, total ? total : 1);
  mbox_t* mb = realloc(S.mb, (total ? total : 1) * sizeof(mbox_t));
  oflag_t* fl = realloc(S.fl, (total ? total : 1) * sizeof(oflag_t));
  uint8_t* tr = realloc(S.trig, total ? total : 1);
  const uint64_t words = (total + 63) / 64, old_words = (S.n_actors + 63) / 64;
  uint64_t* lv = realloc(S.live, (words ? words : 1) * sizeof(uint64_t));
  if(!to || !mb || !fl || !tr || !lv) return GPU_ACTOR_ENOMEM;
  S.type_of = to; S.mb = mb; S.fl = fl; S.trig = tr; S.live = lv;
  for(uint64_t w = old_words; w < words; w++) S.live[w] = 0;
  for(uint64_t a = S.n_actors; a < total; a++)
  {
    S.type_of[a] = (uint8_t)type_id;
    memset(&S.mb[a], 0, sizeof(mbox_t));
    memset(&S.fl[a], 0, sizeof(oflag_t));
    S.trig[a] = 0;
  }
  t->first = S.n_actors;
  t->count = count;
  t->live = live;
  t->state = calloc(t->words * count + 1, sizeof(uint64_t));
  if(!t->state) return GPU_ACTOR_ENOMEM;
  t->created = 1;
  S.n_actors = total;
  construct(type_id);
  if(first_id) *first_id = t->first;
  return 0;
}

/* ---- delivery ------------------------------------------------------------ */
static void apply_reducible(otype_t* t, uint64_t i, uint32_t beh, uint64_t arg)
{
  uint64_t n = t->count;
  switch(t->ht)
  {
    case GPU_ACTOR_HT_FANIN_ANALYZER:
      /* Analyzer.msg_from_sender (fan-in/main.pony:219-220): count += 1. */
      t->state[0 * n + i] += 1;
      t->state[1 * n + i] ^= arg;
      break;
    case GPU_ACTOR_HT_GUPS_UPDATER: {
      /* Updater.apply (gups_basic/main.pony:157-162). */
      uint64_t size = t->params[0];
      uint64_t k = arg & (size - 1);
      t->state[k * n + i] ^= arg;
      break;
    }
  }
  (void)beh;
  t->delivered++;
  S.delivered++;
}

static void deliver(uint64_t to, uint32_t beh, uint64_t arg)
{
  if(to >= S.n_actors) { S.dropped++; return; }
  otype_t* t = &S.types[S.type_of[to]];
  if(t->reducible)
  {
    apply_reducible(t, to - t->first, beh, arg);
    return;
  }
  mbox_t* m = &S.mb[to];
  if(m->tail - m->head >= m->cap_alloc)
  {
    uint64_t nc = m->cap_alloc ? m->cap_alloc * 2 : 8;
    orec_t* nb = malloc(nc * sizeof(orec_t));
    for(uint64_t k = m->head; k < m->tail; k++)
      nb[k % nc] = m->buf[k % m->cap_alloc];
    free(m->buf);
    m->buf = nb;
    m->cap_alloc = nc;
  }
  /* appended during a step: handled from the next one (BSP visibility) */
  if(S.running && m->stamp != S.steps + 1)
  {
    m->tail0 = m->tail;
    m->stamp = S.steps + 1;
  }
  m->buf[m->tail % m->cap_alloc].beh = beh;
  m->buf[m->tail % m->cap_alloc].arg = arg;
  m->tail++;
  S.pending++;
  S.live[to >> 6] |= 1ull << (to & 63);
}

static void send(uint64_t to, uint32_t beh, uint64_t arg)
{
  S.sent++;
  /* ponyint_maybe_mute (actor.c:898-921): a send to an actor that is
   * overloaded or muted (ponyint_triggers_muting, actor.c:1164-1169) mutes a
   * sender that is not itself overloaded, unless it sends to itself. The
   * sender stops after the message it is running (maybe_mute, actor.c:340-
   * 367); the first such receiver is the one it waits on. */
  if(S.n_trig && !S.cur_prev_o && to != S.cur && to < S.n_actors && S.trig[to] && !S.mute_hit)
  {
    S.mute_hit = 1;
    S.mute_to = to;
  }
  deliver(to, beh, arg);
}

int or_send(uint64_t to, uint32_t behaviour, uint64_t arg)
{
  if(!S.init) return GPU_ACTOR_ESTATE;
  if(to >= S.n_actors) return GPU_ACTOR_EINVAL;
  deliver(to, behaviour, arg);
  return 0;
}

int or_sendv(const void* msgs, uint64_t n)
{
  const gpu_msg_t* m = (const gpu_msg_t*)msgs;
  for(uint64_t k = 0; k < n; k++)
  {
    int rc = or_send(m[k].to, m[k].behaviour, m[k].arg);
    if(rc) return rc;
  }
  return 0;
}

/* pony_create inside a behaviour + the constructor message (actor.c:688-734,
 * gencall.c:606-612): the new actor's id is assigned when the step ends. */
static void spawn(uint32_t type, uint32_t beh, uint64_t arg)
{
  S.sent++;
  if(S.n_spawns == S.spawns_alloc)
  {
    uint64_t nc = S.spawns_alloc ? 2 * S.spawns_alloc : 64;
    ospawn_t* nb = realloc(S.spawns, nc * sizeof(ospawn_t));
    if(!nb) { S.dropped++; return; }
    S.spawns = nb;
    S.spawns_alloc = nc;
  }
  S.spawns[S.n_spawns].type = type;
  S.spawns[S.n_spawns].beh = beh;
  S.spawns[S.n_spawns].arg = arg;
  S.n_spawns++;
}

/* End of a step: spawned actors get ids per type in (creator id, call order)
 * order — the order they were recorded in, actors being visited by id — and
 * their constructor messages are appended to their (empty) mailboxes. */
static void place_spawns(void)
{
  for(uint32_t ty = 0; ty < GPU_ACTOR_MAX_TYPES; ty++)
    for(uint64_t k = 0; k < S.n_spawns; k++)
    {
      if(S.spawns[k].type != ty) continue;
      otype_t* t = &S.types[ty];
      if(t->live >= t->count) { S.dropped++; continue; }
      const uint64_t id = t->first + t->live;
      t->live++;
      deliver(id, S.spawns[k].beh, S.spawns[k].arg);
    }
  S.n_spawns = 0;
}

/* ---- behaviours ---------------------------------------------------------- */
/* GPU_ACTOR_HT_PROGRAM (include/gpu_actor.h): one behaviour of the type's
 * program; w0 points at state word 0, word k at w0[k * stride]. */
static void run_program(const otype_t* t, uint64_t self, uint32_t beh, uint64_t arg,
  uint64_t* w0, uint64_t stride)
{
  const uint64_t* P = t->prog;
  const uint32_t np = t->prog_n;
  if(!P || np <= GPU_ACTOR_PROG_ENTRIES) return;
  uint32_t pc = (uint32_t)P[beh & 15];
  if(pc == 0) return;
  uint64_t r[16] = {0};
  for(int k = 0; k < 8; k++) r[k] = w0[(uint64_t)k * stride];
  r[8] = arg; r[9] = self; r[10] = beh;
  for(uint32_t step = 0; step < GPU_ACTOR_PROG_MAX_STEPS && pc < np; step++)
  {
    const uint64_t ins = P[pc++];
    const uint32_t op = (uint32_t)(ins & 0xFF), d = (uint32_t)(ins >> 8) & 15;
    const uint64_t x = r[(ins >> 12) & 15], y = r[(ins >> 16) & 15];
    const int64_t imm = (int32_t)(uint32_t)(ins >> 32);
    if(op == GPU_ACTOR_OP_HALT || op > GPU_ACTOR_OP_SPAWN) break;
    switch(op)
    {
      case GPU_ACTOR_OP_JZ:    if(x == 0) pc = (uint32_t)((int64_t)pc + imm); continue;
      case GPU_ACTOR_OP_JNZ:   if(x != 0) pc = (uint32_t)((int64_t)pc + imm); continue;
      case GPU_ACTOR_OP_JMP:   pc = (uint32_t)((int64_t)pc + imm); continue;
      case GPU_ACTOR_OP_SEND:
        if(x < S.n_actors) send(x, (uint32_t)imm & 15, y);
        else S.dropped++;
        continue;
      case GPU_ACTOR_OP_YIELD: S.yield_req = 1; continue;
      case GPU_ACTOR_OP_SPAWN:
        if(((uint32_t)imm & 0xFF) < GPU_ACTOR_MAX_TYPES)
          spawn((uint32_t)imm & 0xFF, ((uint32_t)imm >> 8) & 15, y);
        else
          S.dropped++;
        continue;
      case GPU_ACTOR_OP_LDI:   r[d] = (uint64_t)imm; break;
      case GPU_ACTOR_OP_LDP:   r[d] = t->params[imm & 7]; break;
      case GPU_ACTOR_OP_MOV:   r[d] = x; break;
      case GPU_ACTOR_OP_ADD:   r[d] = x + y; break;
      case GPU_ACTOR_OP_SUB:   r[d] = x - y; break;
      case GPU_ACTOR_OP_MUL:   r[d] = x * y; break;
      case GPU_ACTOR_OP_MULHI: r[d] = or_mulhi(x, y); break;
      case GPU_ACTOR_OP_AND:   r[d] = x & y; break;
      case GPU_ACTOR_OP_OR:    r[d] = x | y; break;
      case GPU_ACTOR_OP_XOR:   r[d] = x ^ y; break;
      case GPU_ACTOR_OP_SHL:   r[d] = x << (y & 63); break;
      case GPU_ACTOR_OP_SHR:   r[d] = x >> (y & 63); break;
      case GPU_ACTOR_OP_ADDI:  r[d] = x + (uint64_t)imm; break;
      case GPU_ACTOR_OP_LTU:   r[d] = x < y; break;
      case GPU_ACTOR_OP_EQ:    r[d] = x == y; break;
      default:                 r[d] = or_splitmix_mix(x); break;     /* GPU_ACTOR_OP_MIX */
    }
  }
  for(int k = 0; k < 8; k++) w0[(uint64_t)k * stride] = r[k];
}

static void handle(otype_t* t, uint64_t self, uint32_t beh, uint64_t arg)
{
  uint64_t n = t->count, i = self - t->first;
  uint64_t* st = t->state;
#define W(k) st[(uint64_t)(k) * n + i]
  switch(t->ht)
  {
    case GPU_ACTOR_HT_RING:
      if(beh == GPU_ACTOR_RING_SET)
      {
        W(0) = arg;                                 /* ring/main.pony:13-14 */
      } else {
        W(2) += 1;                                  /* ring/main.pony:16-24 */
        if(arg > 0)
        {
          if(W(0) != GPU_ACTOR_NONE)
            send(W(0), GPU_ACTOR_RING_PASS, arg - 1);
        } else {
          W(3) += 1;                                /* _env.out.print(_id)  */
        }
      }
      break;

    case GPU_ACTOR_HT_PINGER: {
      /* message-ubench/main.pony:265-286 (ping + send_pings). */
      or_xoro_t r = { W(0), W(1) };
      W(2) += 1;
      if(W(2) <= t->params[2])
      {
        uint64_t k = or_rand_int(&r, t->params[0]);
        send(t->params[1] + k, GPU_ACTOR_PINGER_PING, 42);
      }
      W(0) = r.x; W(1) = r.y;
      break;
    }

    case GPU_ACTOR_HT_PINGER_DET:
    case GPU_ACTOR_HT_STORM: {
      W(0) += 1;
      if(t->ht == GPU_ACTOR_HT_STORM && beh == GPU_ACTOR_STORM_TOKEN)
      {
        W(1) ^= arg;
        if(arg < t->params[2])
        {
          uint64_t nxt = (i + 1 == n) ? t->first : self + 1;
          send(nxt, GPU_ACTOR_STORM_TOKEN, arg + 1);
        }
        break;
      }
      W(1) ^= arg;
      uint64_t hop = arg & 0xFFFFFFFFULL;
      if(hop < t->params[2])
      {
        uint64_t k = or_mulhi(or_splitmix_mix(t->params[3] ^ arg), t->params[0]);
        send(t->params[1] + k, beh, (arg & 0xFFFFFFFF00000000ULL) | (hop + 1));
      }
      break;
    }

    case GPU_ACTOR_HT_FANIN_SENDER: {
      /* Sender.send_msgs (fan-in/main.pony:241-250). */
      or_xoro_t r = { W(0), W(1) };
      uint64_t k = or_rand_int_unbiased(&r, t->params[0]);
      send(t->params[1] + k, GPU_ACTOR_FANIN_MSG, (i << 32) | W(3));
      W(3) += 1;
      W(0) = r.x; W(1) = r.y;
      if(W(2) > 0) W(2) -= 1;
      if(W(2) > 0)
        send(self, GPU_ACTOR_FANIN_SEND_MSGS, 0);
      break;
    }

    case GPU_ACTOR_HT_GUPS_STREAMER: {
      /* Streamer.apply (gups_basic/main.pony:110-143), one message per datum. */
      or_polyrand_t pr = { W(0) };
      uint64_t chunk = t->params[0], shift = t->params[1], mask = t->params[2];
      for(uint64_t c = 0; c < chunk; c++)
      {
        uint64_t d = or_polyrand_next(&pr);
        uint64_t u = (d >> shift) & mask;
        send(t->params[3] + u, GPU_ACTOR_GUPS_UPDATE, d);
      }
      W(0) = pr.last;
      if(arg > 0)
        send(self, GPU_ACTOR_GUPS_APPLY, arg - 1);
      else
        W(1) = 1;                                  /* main.streamer_done() */
      break;
    }

    case GPU_ACTOR_HT_FIFO_SRC: {
      for(uint64_t j = 0; j < arg; j++)
      {
        W(1) += 1;
        send(W(0), GPU_ACTOR_FIFO_PUSH, (i << 32) | W(1));
      }
      if(W(2) > 0) W(2) -= 1;
      if(W(2) > 0)
        send(self, GPU_ACTOR_FIFO_BURST, arg);
      break;
    }

    case GPU_ACTOR_HT_SPREADER:
      if(beh == GPU_ACTOR_SPREADER_SPREAD)
      {
        /* new create / new spread (spreader/main.pony:9-32) */
        const uint64_t parent = arg >> 32, count = arg & 0xFFFFFFFFULL;
        W(0) = count;
        W(1) = parent == 0xFFFFFFFFULL ? GPU_ACTOR_NONE : parent;
        if(count <= 1)
        {
          if(W(1) != GPU_ACTOR_NONE) send(W(1), GPU_ACTOR_SPREADER_RESULT, 1);
          else W(4) = 1;                           /* env.out.print("1 actor") */
        }
        else
        {
          /* spawn_child() x 2 (spreader/main.pony:47-48) */
          spawn(S.type_of[self], GPU_ACTOR_SPREADER_SPREAD, (self << 32) | (count - 1));
          spawn(S.type_of[self], GPU_ACTOR_SPREADER_SPREAD, (self << 32) | (count - 1));
        }
      }
      else
      {
        /* be result(i) (spreader/main.pony:34-45) */
        W(3) += 1;
        W(2) += arg;
        if(W(3) == 2)
        {
          if(W(1) != GPU_ACTOR_NONE) send(W(1), GPU_ACTOR_SPREADER_RESULT, W(2) + 1);
          else W(4) = W(2) + 1;                    /* print(_result + 1 " actors") */
        }
      }
      break;

    case GPU_ACTOR_HT_PROGRAM:
      run_program(t, self, beh, arg, &W(0), n);
      break;

    case GPU_ACTOR_HT_FIFO_SINK: {
      uint64_t ns = t->params[0] ? t->params[0] : 1;
      uint64_t slot = ((arg >> 32) / ns) % 8;
      uint64_t seq = arg & 0xFFFFFFFFULL;
      W(1) += 1;
      W(0) = (W(0) ^ arg) * 0x100000001b3ULL;
      if(seq != W(3 + slot) + 1) W(2) += 1;
      W(3 + slot) = seq;
      /* param 1: yield after every k-th message (ponyint_actor_yield) */
      if(t->params[1] && W(1) % t->params[1] == 0) S.yield_req = 1;
      break;
    }
  }
#undef W
}

/* ---- run ----------------------------------------------------------------- */
static uint64_t pending_total(void)
{
  return S.pending;
}

static void trig_set(uint64_t a, int v)
{
  if(S.trig[a] == (uint8_t)v) return;
  S.trig[a] = (uint8_t)v;
  if(v) S.n_trig++; else S.n_trig--;
}

/* One superstep, actors visited in id order (those with mail, muted or
 * overloaded). Backpressure, restated for supersteps from actor.c:340-381,
 * 449-471, 898-921 and scheduler.c:1496-1635:
 *   - flags are read as the previous step left them;
 *   - a muted actor stays muted (runs nothing, keeps its mail) while the
 *     receiver it is muted on is overloaded; otherwise it is unmuted and runs
 *     this step (Pony unmutes a receiver's senders when it clears OVERLOADED,
 *     ponyint_actor_unsetoverloaded, actor.c:1121-1134; muted actors wait only
 *     on overloaded ones, which always run, so muting cannot deadlock);
 *   - an actor runs min(batch, mail at step start) messages and stops early
 *     after a message whose sends muted it (send()) or that yielded
 *     (ponyint_actor_yield, actor.c:675-679); the rest waits, in order;
 *   - an actor of a type with priority > 0 runs batch after batch
 *     (scheduler.c:1053-1068 keeps it running while it outranks the next
 *     runnable actor): all the mail at step start, with the same early stops;
 *   - it is overloaded after the step iff it ran a full batch (a priority
 *     type: its last batch) and was not muted (batch_limit_reached,
 *     actor.c:369-381); an actor that did not run is not overloaded. */
static void run_step(void)
{
  typedef struct { uint64_t a; int t; } upd_t;
  static upd_t* upd = NULL;
  static uint64_t upd_alloc = 0;
  uint64_t n_upd = 0;
  S.running = 1;
  const uint64_t words = (S.n_actors + 63) / 64;
  for(uint64_t w = 0; w < words; w++)
  {
    uint64_t bits = S.live[w];
    while(bits)
    {
      const uint64_t a = w * 64 + (uint64_t)__builtin_ctzll(bits);
      bits &= bits - 1;
      otype_t* t = &S.types[S.type_of[a]];
      mbox_t* m = &S.mb[a];
      oflag_t* f = &S.fl[a];
      const int prev_o = f->o;
      uint64_t handled = 0;
      int muted_now = 0;
      if(f->m && (S.trig[f->r] & 1u))
        muted_now = 1;                 /* still waiting: nothing runs */
      else
      {
        f->m = 0;
        const uint64_t avail = (m->stamp == S.steps + 1 ? m->tail0 : m->tail) - m->head;
        const uint64_t w_ = (t->priority > 0 || avail < t->batch) ? avail : t->batch;
        S.cur = a; S.cur_prev_o = prev_o; S.mute_hit = 0; S.yield_req = 0;
        for(uint64_t k = 0; k < w_; k++)
        {
          orec_t r = m->buf[m->head % m->cap_alloc];
          m->head++;
          S.pending--;
          t->delivered++;
          S.delivered++;
          handled++;
          handle(t, a, r.beh, r.arg);
          if(S.mute_hit || S.yield_req) break;
        }
        if(S.mute_hit) { muted_now = 1; f->r = (uint32_t)S.mute_to; }
      }
      f->m = (uint8_t)muted_now;
      const int full = t->priority > 0 ? (handled != 0 && handled % t->batch == 0)
                                       : handled == t->batch;
      f->o = (uint8_t)(full && !muted_now);
      if(n_upd == upd_alloc)
      {
        upd_alloc = upd_alloc ? 2 * upd_alloc : 1024;
        upd = realloc(upd, upd_alloc * sizeof(upd_t));
      }
      upd[n_upd].a = a;
      upd[n_upd].t = (int)f->o | ((int)f->m << 1);
      n_upd++;
    }
  }
  S.running = 0;
  /* the next step reads the flags this one left */
  for(uint64_t k = 0; k < n_upd; k++)
  {
    const uint64_t a = upd[k].a;
    trig_set(a, upd[k].t);
    if(S.mb[a].tail == S.mb[a].head && !S.fl[a].m && !S.fl[a].o)
      S.live[a >> 6] &= ~(1ull << (a & 63));
  }
}

int or_run(uint64_t max_steps, uint64_t* steps_done)
{
  if(!S.init) return GPU_ACTOR_ESTATE;
  uint64_t done = 0;
  /* runs while mail is pending; flags left by the last step are honoured by
   * the next run */
  while((max_steps == 0 || done < max_steps) && pending_total() > 0)
  {
    run_step();
    place_spawns();
    S.steps++;
    done++;
  }
  if(steps_done) *steps_done = done;
  return S.dropped ? GPU_ACTOR_EMAILBOX : 0;
}

int or_state_read(uint32_t type_id, uint64_t first, uint64_t n, uint64_t* out)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  otype_t* t = &S.types[type_id];
  if(!t->created || first + n > t->count) return GPU_ACTOR_EINVAL;
  for(uint32_t w = 0; w < t->words; w++)
    memcpy(out + (uint64_t)w * n, t->state + (uint64_t)w * t->count + first, n * sizeof(uint64_t));
  return 0;
}

int or_state_write(uint32_t type_id, uint64_t first, uint64_t n, const uint64_t* in)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  otype_t* t = &S.types[type_id];
  if(!t->created || first + n > t->count) return GPU_ACTOR_EINVAL;
  for(uint32_t w = 0; w < t->words; w++)
    memcpy(t->state + (uint64_t)w * t->count + first, in + (uint64_t)w * n, n * sizeof(uint64_t));
  return 0;
}

/* Actors whose trigger byte the last step left nonzero (overloaded or muted):
 * the oracle's side of the engine's per-step trigger count (trig_n). */
uint64_t or_trig_count(void)
{
  return S.init ? S.n_trig : 0;
}

int or_counts(uint64_t* out)
{
  out[0] = S.steps;
  out[1] = S.delivered;
  out[2] = S.sent;
  out[3] = pending_total();
  out[4] = S.dropped;
  return 0;
}

int or_type_delivered(uint32_t type_id, uint64_t* out)
{
  if(type_id >= GPU_ACTOR_MAX_TYPES) return GPU_ACTOR_EINVAL;
  *out = S.types[type_id].delivered;
  return 0;
}

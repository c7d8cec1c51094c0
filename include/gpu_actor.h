/*
 * gpu_actor.h — C-ABI of the MI355X actor-dispatch engine (libgpuactor.so).
 *
 * Drop-in boundary for the Pony runtime's data-parallel hot path: the entry
 * points below replace, for GPU-resident POD-state actors, the pony.h calls a
 * compiled Pony program makes on that path. Actors are
 * addressed by 32-bit ids instead of pony_actor_t*, state is plain words,
 * and behaviours come from a fixed table of device handlers (the analogue of
 * pony_type_t.dispatch, pony.h:114-115,171-195).
 *
 * Conventions mirrored from pony.h:
 *   - ownership of a message passes to the library at send (pony_sendv,
 *     pony.h:271-279); messages in one gpu_actor_sendv call keep their order
 *     (a pony_chain, pony.h:296-305);
 *   - per-sender->receiver FIFO and causal delivery (the guarantee
 *     codegen_optimisation.cc:13-41 pins) hold;
 *   - unlike pony.h, errors are returned as codes (0 ok, <0 error), never
 *     raised, so every entry point is safe to declare as Pony FFI without `?`;
 *   - calls from different host threads are serialised internally.
 *
 * Execution model: bulk-synchronous supersteps. In step s every actor with
 * pending mail drains up to `batch` messages (PONY_SCHED_BATCH = 100,
 * actor.c:20, overridable per type like the fork's _batch() hint,
 * pony.h:156-162) and runs the handler for each; messages sent in step s are
 * delivered from step s+1 on. Each step's arrivals at an actor are delivered
 * in (sender id, sender sequence) order, after any carried-over mail; host
 * sends count as senders with ids above every actor id.
 */
#ifndef GPU_ACTOR_H
#define GPU_ACTOR_H

#include <stdint.h>
#ifndef __HIPCC_RTC__   /* (the run-time compiled step: engine.hip jit) */
#include <stddef.h>
#endif

#if defined(__cplusplus)
extern "C" {
#endif

#define GPU_ACTOR_API __attribute__((visibility("default")))

/* ---- error codes ------------------------------------------------------- */
#define GPU_ACTOR_OK            0
#define GPU_ACTOR_EINVAL       -1   /* bad argument / unknown type / bad id   */
#define GPU_ACTOR_ENOMEM       -2   /* device or host allocation failed        */
#define GPU_ACTOR_ENODEV       -3   /* no usable GPU                           */
#define GPU_ACTOR_EMAILBOX     -4   /* messages lost: the per-step overflow list
                                       was exhausted, or behaviours spawned past
                                       a type's reserve (zone buffers that fill
                                       spill and grow; they never drop)        */
#define GPU_ACTOR_EHIP         -5   /* HIP runtime error                       */
#define GPU_ACTOR_ESTATE       -6   /* not initialised / already initialised   */
#define GPU_ACTOR_ERANGE       -7   /* sequence or id space exhausted: more than
                                       65,534 sends by one actor in one superstep
                                       (16,382 with n_ranks > 1), or more than
                                       2^23 actors on one rank                  */
#define GPU_ACTOR_ECOMM        -8   /* RCCL / exchange failure                 */
#define GPU_ACTOR_EBUSY        -9   /* an asynchronous run is in flight         */

#define GPU_ACTOR_MAX_TYPES    16
#define GPU_ACTOR_MAX_PARAMS   8

/* ---- messages ------------------------------------------------------------ */
/* One application message: the POD analogue of pony_msgi_t (pony.h:53-58). */
typedef struct gpu_msg_t
{
  uint32_t to;          /* receiver actor id                           */
  uint32_t behaviour;   /* behaviour index within the receiver's table */
  uint64_t arg;         /* the single machine-word argument            */
} gpu_msg_t;

/* ---- configuration ------------------------------------------------------ */
typedef struct gpu_actor_config_t
{
  int32_t  device;          /* HIP device ordinal for this process (-1: current)  */
  uint32_t n_ranks;         /* processes (one per GPU) sharing the actor space   */
  uint32_t rank;            /* this process's rank, 0 <= rank < n_ranks          */
  uint32_t batch;           /* default per-step drain limit (0 -> 100)           */
  uint32_t mailbox_cap;     /* default mailbox ring capacity, power of 2 (0->16) */
  uint32_t max_exchange;    /* per-peer records per step for n_ranks>1 (0->auto) */
  uint64_t max_actors;      /* capacity of the global id space (0 -> 1<<26)      */
  const void* comm_id;      /* 128-byte ncclUniqueId from rank 0 (n_ranks > 1)  */
} gpu_actor_config_t;

/* Counters read back by gpu_actor_counts (device-side counters, summed over
 * ranks when n_ranks > 1). */
typedef struct gpu_actor_counts_t
{
  uint64_t steps;       /* supersteps run since init                        */
  uint64_t delivered;   /* application messages handled (handler invocations) */
  uint64_t sent;        /* application messages emitted by handlers          */
  uint64_t pending;     /* messages waiting in mailboxes now                 */
  uint64_t dropped;     /* messages lost to mailbox overflow (error)          */
  uint64_t remote;      /* messages that crossed ranks                       */
  uint64_t active;      /* actor-steps that handled at least one message     */
  uint64_t delivered_by_type[GPU_ACTOR_MAX_TYPES];
  uint64_t atomics;     /* global chunk-reservation atomics the drain kernel
                           issued (one per (zone, destination bucket) per step) */
} gpu_actor_counts_t;

/* ---- lifecycle (pony_init / pony_start / pony_stop, pony.h:486-559) ------ */
GPU_ACTOR_API int gpu_actor_init(const gpu_actor_config_t* cfg);
GPU_ACTOR_API int gpu_actor_shutdown(void);
/* 128-byte communicator id to broadcast from rank 0 before gpu_actor_init. */
GPU_ACTOR_API int gpu_actor_comm_id(void* out128);

/* Host transport for n_ranks > 1 when no RCCL communicator is given (comm_id
 * NULL): the per-step exchange and the cross-rank sums are routed through these
 * host callbacks (e.g. gloo), with records staged through pinned host memory.
 * alltoallv: send_bytes[p] bytes at offset Σ_{q<p} send_bytes[q] of `send` go
 * to rank p; recv_bytes[p] bytes from rank p land likewise in `recv`. Returns
 * 0 on success. allreduce: in-place sum of n u64 over ranks. Set before
 * gpu_actor_init; NULL restores RCCL. */
typedef int (*gpu_actor_alltoallv_fn)(void* ctx, const void* send, const uint64_t* send_bytes,
  void* recv, const uint64_t* recv_bytes);
typedef int (*gpu_actor_allreduce_fn)(void* ctx, uint64_t* buf, uint64_t n);
GPU_ACTOR_API int gpu_actor_set_transport(gpu_actor_alltoallv_fn alltoallv,
  gpu_actor_allreduce_fn allreduce, void* ctx);

/* ---- types (pony_type_t, pony.h:171-195) -------------------------------- */
/* Register actor type `type_id` (< GPU_ACTOR_MAX_TYPES) with `state_words`
 * 64-bit words of POD state, dispatching to handler table `handler_table`
 * (GPU_ACTOR_HT_*). */
GPU_ACTOR_API int gpu_actor_type_register(uint32_t type_id, uint32_t state_words,
  uint32_t handler_table);
/* Per-type drain limit (the fork's _batch() hint, actor.c:410-416) and mailbox
 * ring capacity (power of two). 0 keeps the config default. */
GPU_ACTOR_API int gpu_actor_type_config(uint32_t type_id, uint32_t batch,
  uint32_t mailbox_cap);
/* Per-type scheduling priority (the fork's _priority() hint, actor.c:414-416;
 * default PONY_DEFAULT_ACTOR_PRIORITY = 0, scheduler.h:20). In the reference a
 * rescheduled actor whose priority exceeds the next runnable actor's keeps its
 * scheduler thread and runs its next batch at once (scheduler.c:1053-1068);
 * every default actor ranks below a positive priority. Restated per
 * superstep: an actor of a type with priority > 0 runs batch after batch
 * while mail is pending at the step's start — it handles all of it unless a
 * behaviour mutes it or yields — and is overloaded afterwards iff its last
 * batch was full (handled a positive multiple of its batch) and it was not
 * muted. Priorities <= 0 keep one batch per step. Any time between runs. */
GPU_ACTOR_API int gpu_actor_type_priority(uint32_t type_id, int32_t priority);
/* Handler-table parameter `idx` (< GPU_ACTOR_MAX_PARAMS) of a type; set before
 * gpu_actor_create, which runs the table's constructor with them. */
GPU_ACTOR_API int gpu_actor_type_param(uint32_t type_id, uint32_t idx, uint64_t value);
/* The behaviours of a GPU_ACTOR_HT_PROGRAM type, given at run time: `n`
 * instruction words (below), copied to the device. Replaces the generated
 * per-type dispatch switch (src/libponyc/codegen/gentype.c:358-395, the
 * pony_type_t.dispatch the runtime calls in actor.c:437-480) for behaviour
 * sets the compiled tables do not hold — no library rebuild. Any time while
 * no run is in flight; an engine that holds programs runs them on the zone
 * path (never the small-step path). */
GPU_ACTOR_API int gpu_actor_type_program(uint32_t type_id, const uint64_t* code, uint32_t n);

/* ---- actors (pony_create, actor.c:688-734) ------------------------------ */
/* Bulk-create `count` actors of a type (once per type); ids are
 * [*first_id, *first_id + count). Runs the table's constructor on device. */
GPU_ACTOR_API int gpu_actor_create(uint32_t type_id, uint64_t count, uint64_t* first_id);
/* Room for `n` more actors of a type that behaviours create while running
 * (pony_create inside a behaviour + its constructor message, actor.c:688-734,
 * gencall.c:606-612). Call before gpu_actor_create; the type's id range
 * becomes [first, first + count + n). A spawned actor's id is assigned at the
 * end of the superstep that created it, in (creator id, creator send
 * sequence) order after the type's live actors; its constructor message is
 * delivered in the next superstep like any other send. With n_ranks > 1
 * every rank gathers every rank's spawn records and numbers them alike, so
 * the ids equal a single rank's; the owner (id % n_ranks) lands the message. */
GPU_ACTOR_API int gpu_actor_type_reserve(uint32_t type_id, uint64_t n);
/* Live (created + spawned) actors of a type. */
GPU_ACTOR_API int gpu_actor_type_live(uint32_t type_id, uint64_t* live);

/* ---- sending from the host (pony_alloc_msg + pony_sendv, actor.c:749-817) */
/* Host staging buffer for up to n messages, owned by the library and valid
 * until the next gpu_actor_alloc_msgs / gpu_actor_shutdown. */
GPU_ACTOR_API int gpu_actor_alloc_msgs(uint64_t n, gpu_msg_t** buf);
/* Send n messages in order (a chain). Ownership passes to the library. With
 * n_ranks > 1 every message must be addressed to an actor this rank owns
 * (gpu_actor_owner(to) == rank): each rank injects its own share, and a
 * message for another rank's actor fails the whole call with
 * GPU_ACTOR_EINVAL before anything is sent. */
GPU_ACTOR_API int gpu_actor_sendv(const gpu_msg_t* first, uint64_t n);
/* pony_sendi (actor.c:959-968) analogue. The message is appended to a host
 * staging list (no device work, no synchronisation) and injected, in call
 * order and before any later gpu_actor_sendv, by the next call that runs or
 * observes the engine (run*, sync, state_*, counts). Same ownership rule as
 * gpu_actor_sendv. */
GPU_ACTOR_API int gpu_actor_send(uint64_t to, uint32_t behaviour, uint64_t arg);

/* ---- running (the scheduler run loop, scheduler.c:953-1090) ------------- */
/* Run up to max_steps supersteps (0: until quiescent, i.e. no pending mail on
 * any rank). *steps_done receives the number of steps that handled mail. */
GPU_ACTOR_API int gpu_actor_run(uint64_t max_steps, uint64_t* steps_done);
/* Run exactly n supersteps without any host synchronisation between them
 * (benchmark form: no quiescence test, no readback). */
GPU_ACTOR_API int gpu_actor_run_fixed(uint64_t n);
/* Block until all queued device work is done; returns the sticky error. */
GPU_ACTOR_API int gpu_actor_sync(void);
/* Asynchronous run (the ASIO delivery pattern, event.c:116-135):
 * gpu_actor_run(max_steps) on a library progress thread; returns at once.
 * When the run ends, done(ctx, rc, steps_done) is called ON THAT THREAD,
 * outside the library's lock (it may call back into the library). A Pony
 * binding's `done` calls pony_register_thread() (pony.h:520-528) once and then
 * pony_sendv_single()s a completion message to the notify actor passed as ctx
 * (INTEGRATION.md). While the run is in flight the other entry points block
 * behind it (calls are serialised), and gpu_actor_run/run_async return
 * GPU_ACTOR_EBUSY. done may be NULL (poll gpu_actor_busy / gpu_actor_wait). */
typedef void (*gpu_actor_done_fn)(void* ctx, int rc, uint64_t steps_done);
GPU_ACTOR_API int gpu_actor_run_async(uint64_t max_steps, gpu_actor_done_fn done, void* ctx);
/* Join the last asynchronous run: its return code and steps (0 if none). */
GPU_ACTOR_API int gpu_actor_wait(uint64_t* steps_done);
/* 1 while an asynchronous run is in flight, else 0. */
GPU_ACTOR_API int gpu_actor_busy(void);

/* ---- state and counters ------------------------------------------------- */
/* Copy state of actors [first, first+n) of a type (indices relative to the
 * type's first id; only actors owned by this rank are meaningful when
 * n_ranks > 1). Layout: field-major, out[w * n + i] = word w of actor i. */
GPU_ACTOR_API int gpu_actor_state_read(uint32_t type_id, uint64_t first, uint64_t n,
  uint64_t* out);
GPU_ACTOR_API int gpu_actor_state_write(uint32_t type_id, uint64_t first, uint64_t n,
  const uint64_t* in);
GPU_ACTOR_API int gpu_actor_counts(gpu_actor_counts_t* out);
/* Id of the rank owning actor `id` (hash partition; id % n_ranks). */
GPU_ACTOR_API uint32_t gpu_actor_owner(uint64_t id);
/* Device stream the engine runs on (hipStream_t), for profiling/overlap. */
GPU_ACTOR_API void* gpu_actor_stream(void);
/* Average step time (ms) of the last gpu_actor_run_fixed: two HIP events on
 * the engine's stream around its n launches, divided by n (an upper bound on
 * the step kernel's own duration); 0 if unavailable. */
GPU_ACTOR_API double gpu_actor_last_drain_ms(void);
GPU_ACTOR_API const char* gpu_actor_strerror(int code);

/* ======================================================================== */
/* Fixed handler tables. Each table is the device restatement of one         */
/* reference actor's behaviours. Behaviour ids, state words and params:     */
/* ======================================================================== */

/* Ring (examples/ring/main.pony:3-24).
 *   state: [0] next (actor id; ~0 = None)  [1] ring id (1..size)
 *          [2] pass messages received        [3] pass(0) received ("print")
 *   params: [0] ring size (constructor: actor k of ring j gets id k%size+1,
 *           next = the actor with id+1, except id 1 whose next comes by set)
 *   behaviours: SET(arg = neighbour id), PASS(arg = i)                      */
#define GPU_ACTOR_HT_RING            1
#define GPU_ACTOR_RING_SET           0
#define GPU_ACTOR_RING_PASS          1

/* Pinger of examples/message-ubench/main.pony:229-286 with a per-pinger
 * forward budget in place of the wall-clock interval. Rand is seeded
 * Rand(seed + i + 1, 0x9E3779B97F4A7C15) and primed with three int(100).
 *   state: [0] rng x  [1] rng y  [2] pings received
 *   params: [0] N pingers  [1] first pinger id  [2] budget  [3] seed
 *   behaviours: PING(arg): count += 1; if count <= budget:
 *               ping(42) to pinger rand.int(N)                               */
#define GPU_ACTOR_HT_PINGER          2
#define GPU_ACTOR_PINGER_PING        0

/* message-ubench-det: a token's route depends only on its
 * payload. arg = token << 32 | hop.
 *   state: [0] pings received  [1] xor of payloads
 *   params: [0] N  [1] first id  [2] hops H  [3] seed
 *   behaviours: PING(arg): count++, acc ^= arg; if hop < H: send
 *               (token<<32 | hop+1) to first + mulhi(splitmix64(seed^arg), N) */
#define GPU_ACTOR_HT_PINGER_DET      3
#define GPU_ACTOR_PINGER_DET_PING    0

/* fan-in Sender (examples/fan-in/main.pony:231-254), P messages each.
 *   state: [0] rng x [1] rng y [2] remaining [3] sent
 *   params: [0] analyzers A [1] first analyzer id [2] P
 *           [3] seed mode (0: every sender Rand() = Rand(5489, 0) as in the
 *               reference, fan-in/main.pony:235; 1: Rand(5489 + i, 0))
 *   behaviours: SEND_MSGS: MSG(i << 32 | sent) to analyzer
 *               rand.int_unbiased(A); sent++; if --remaining: SEND_MSGS to self */
#define GPU_ACTOR_HT_FANIN_SENDER    4
#define GPU_ACTOR_FANIN_SEND_MSGS    0

/* fan-in Analyzer (fan-in/main.pony:212-229). Commutative ("reducible"):
 * messages are applied as device atomics when sent.
 *   state: [0] messages received  [1] xor of args
 *   behaviours: MSG(arg)                                                     */
#define GPU_ACTOR_HT_FANIN_ANALYZER  5
#define GPU_ACTOR_FANIN_MSG          0

/* gups Streamer (examples/gups_basic/main.pony:93-143), one message per
 * update. Streamer i uses PolyRand(i * stride).
 *   state: [0] PolyRand last  [1] finished flag
 *   params: [0] chunk [1] shift [2] updater mask [3] first updater id
 *           [4] unused [5] seed stride
 *   behaviours: APPLY(iterate): chunk x UPDATE(d) to updater (d>>shift)&mask;
 *               if iterate > 0: APPLY(iterate-1) to self else finished = 1   */
#define GPU_ACTOR_HT_GUPS_STREAMER   6
#define GPU_ACTOR_GUPS_APPLY         0

/* gups Updater (gups_basic/main.pony:145-165). Reducible (XOR).
 *   state: `size` words, table[k] = k + index*size initially
 *   params: [0] size (power of two)
 *   behaviours: UPDATE(d): table[d & (size-1)] ^= d                           */
#define GPU_ACTOR_HT_GUPS_UPDATER    7
#define GPU_ACTOR_GUPS_UPDATE        0

/* Message storm: a ring token plus random-target traffic.
 *   state: [0] messages received  [1] xor of args
 *   params: [0] N [1] first id [2] hops H [3] seed
 *   behaviours: TOKEN(hop): count++, acc ^= hop; if hop < H: TOKEN(hop+1)
 *               to the next actor (wrapping); STORM(arg): as PINGER_DET.PING */
#define GPU_ACTOR_HT_STORM           8
#define GPU_ACTOR_STORM_TOKEN        0
#define GPU_ACTOR_STORM_STORM        1

/* Per-pair FIFO probe (order-sensitive; codegen_optimisation.cc:13-41).
 * Source i targets sink first_sink + i % n_sinks.
 *   FIFO_SRC state: [0] target [1] seq [2] bursts left
 *            params: [0] first sink id [1] n sinks [2] bursts
 *            BURST(m): m x PUSH(i << 32 | ++seq); if --bursts: BURST(m) to self
 *   FIFO_SINK state: [0] h (FNV-1a fold of args, order-sensitive) [1] n
 *            [2] FIFO violations [3..10] last seq per source slot
 *            params: [0] n sinks [1] yield period k (0 = never): the sink
 *            calls the yield rule (pony_yield analogue) after
 *            every k-th message it has received
 *            PUSH(arg): slot = ((arg >> 32) / n_sinks) % 8                   */
#define GPU_ACTOR_HT_FIFO_SRC        9
#define GPU_ACTOR_FIFO_BURST         0
#define GPU_ACTOR_HT_FIFO_SINK       10
#define GPU_ACTOR_FIFO_PUSH          0

/* Spreader (examples/spreader/main.pony:1-48): builds a binary tree of
 * 2^count - 1 actors by spawning, then sums the node counts back up.
 *   state: [0] count [1] parent id (~0 = none: the root)
 *          [2] _result [3] _received [4] root's printed total (result + 1)
 *   behaviours: SPREAD(parent << 32 | count) — the constructor
 *               (new create / new spread): if count == 1: RESULT(1) to parent
 *               (the root sets [4] = 1) else spawn two Spreaders with
 *               SPREAD(self << 32 | count - 1);
 *               RESULT(i): received++, result += i; at 2: RESULT(result + 1)
 *               to parent, or the root sets [4] = result + 1                */
#define GPU_ACTOR_HT_SPREADER        11
#define GPU_ACTOR_SPREADER_SPREAD    0
#define GPU_ACTOR_SPREADER_RESULT    1

/* 12: behaviours as a program (gpu_actor_type_program), interpreted per
 * message. state: 8 words. Registers r0-r7 are the state words, r8 the
 * message argument, r9 the actor's id, r10 the behaviour, r11-r15 zero at
 * entry; r0-r7 are the state afterwards. Words 0-15 of the program are the
 * entry index of behaviour 0-15's code (0: the behaviour does nothing); code
 * follows. An instruction is one u64:
 *   op | d << 8 | a << 12 | b << 16 | (uint32_t)imm << 32   (imm: int32)
 * and pc indexes the next instruction while one runs. A behaviour ends at
 * HALT, at an invalid op or pc, or after GPU_ACTOR_PROG_MAX_STEPS
 * instructions. SEND to an id past the world's ids is dropped (counted).   */
#define GPU_ACTOR_HT_PROGRAM         12
#define GPU_ACTOR_PROG_ENTRIES       16
#define GPU_ACTOR_PROG_MAX_STEPS     4096
#define GPU_ACTOR_OP_HALT   0   /* end the behaviour                          */
#define GPU_ACTOR_OP_LDI    1   /* r[d] = (int64)imm                          */
#define GPU_ACTOR_OP_LDP    2   /* r[d] = type param (imm & 7)                */
#define GPU_ACTOR_OP_MOV    3   /* r[d] = r[a]                                */
#define GPU_ACTOR_OP_ADD    4   /* r[d] = r[a] + r[b]                         */
#define GPU_ACTOR_OP_SUB    5   /* r[d] = r[a] - r[b]                         */
#define GPU_ACTOR_OP_MUL    6   /* r[d] = r[a] * r[b] (low 64 bits)           */
#define GPU_ACTOR_OP_MULHI  7   /* r[d] = (r[a] * r[b]) >> 64, unsigned       */
#define GPU_ACTOR_OP_AND    8
#define GPU_ACTOR_OP_OR     9
#define GPU_ACTOR_OP_XOR    10
#define GPU_ACTOR_OP_SHL    11  /* r[d] = r[a] << (r[b] & 63)                 */
#define GPU_ACTOR_OP_SHR    12  /* r[d] = r[a] >> (r[b] & 63), logical        */
#define GPU_ACTOR_OP_ADDI   13  /* r[d] = r[a] + (int64)imm                   */
#define GPU_ACTOR_OP_LTU    14  /* r[d] = r[a] < r[b] (unsigned), 0 or 1      */
#define GPU_ACTOR_OP_EQ     15  /* r[d] = r[a] == r[b], 0 or 1                */
#define GPU_ACTOR_OP_JZ     16  /* if r[a] == 0: pc += imm                    */
#define GPU_ACTOR_OP_JNZ    17  /* if r[a] != 0: pc += imm                    */
#define GPU_ACTOR_OP_JMP    18  /* pc += imm                                  */
#define GPU_ACTOR_OP_SEND   19  /* send behaviour (imm & 15), arg r[b], to r[a] */
#define GPU_ACTOR_OP_MIX    20  /* r[d] = splitmix64 finaliser of r[a]        */
#define GPU_ACTOR_OP_YIELD  21  /* end this actor's run after this behaviour  */
#define GPU_ACTOR_OP_SPAWN  22  /* create an actor of type (imm & 0xFF) whose
                                   constructor behaviour (imm >> 8 & 15) gets
                                   arg r[b] (pony_create + its constructor
                                   message, actor.c:688-734, gencall.c:606-612;
                                   gpu_actor_type_reserve gives the room, past
                                   it the spawn is dropped and counted)      */

#define GPU_ACTOR_NONE 0xFFFFFFFFFFFFFFFFULL

#if defined(__cplusplus)
}
#endif
#endif

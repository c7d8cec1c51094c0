"""
# gpu_actor package

Pony binding of libgpuactor.so (include/gpu_actor.h), the MI355X actor-dispatch
engine. Examples opt in with `use "gpu_actor"`; the engine replaces, for the
actors it holds, libponyrt's mailbox drain (ponyint_actor_run, actor.c:383-549),
messageq push/pop (messageq.c) and the scheduler run loop (scheduler.c).

Every FFI entry point is declared with its exact prototype: undeclared FFI
calls are emitted as varargs (gencall.c:1196-1198). All return an I32 error
code (0 = ok, include/gpu_actor.h GPU_ACTOR_E*), never a Pony error, so no `?`.

Not compiled in the build image: ponyc needs LLVM <= 7 (SURVEY §8 c1). The C
ABI these declarations bind is exercised by tests/test_cabi.py and the GPU
parity tests through the same symbols.
"""
use "lib:gpuactor"

use @gpu_actor_init[I32](cfg: GpuActorConfig tag)
use @gpu_actor_shutdown[I32]()
use @gpu_actor_comm_id[I32](out128: Pointer[U8] tag)
use @gpu_actor_type_register[I32](type_id: U32, state_words: U32, table: U32)
use @gpu_actor_type_config[I32](type_id: U32, batch: U32, mailbox_cap: U32)
use @gpu_actor_type_priority[I32](type_id: U32, priority: I32)
use @gpu_actor_type_param[I32](type_id: U32, idx: U32, value: U64)
use @gpu_actor_type_program[I32](type_id: U32, code: Pointer[U64] tag, n: U32)
use @gpu_actor_create[I32](type_id: U32, count: U64, first: Pointer[U64])
use @gpu_actor_type_reserve[I32](type_id: U32, n: U64)
use @gpu_actor_type_live[I32](type_id: U32, live: Pointer[U64])
use @gpu_actor_alloc_msgs[I32](n: U64, buf: Pointer[Pointer[GpuMsg]])
use @gpu_actor_sendv[I32](first: Pointer[U64] tag, n: U64)
use @gpu_actor_send[I32](to: U64, behaviour: U32, arg: U64)
use @gpu_actor_run[I32](max_steps: U64, steps_done: Pointer[U64])
use @gpu_actor_run_fixed[I32](n: U64)
use @gpu_actor_run_async[I32](max_steps: U64,
  done: @{(GpuRunNotify, I32, U64)}, ctx: GpuRunNotify)
use @gpu_actor_wait[I32](steps_done: Pointer[U64])
use @gpu_actor_busy[I32]()
use @gpu_actor_sync[I32]()
use @gpu_actor_state_read[I32](type_id: U32, first: U64, n: U64, out: Pointer[U64] tag)
use @gpu_actor_state_write[I32](type_id: U32, first: U64, n: U64, src: Pointer[U64] tag)
use @gpu_actor_counts[I32](out: GpuActorCounts tag)
use @gpu_actor_owner[U32](id: U64)
use @gpu_actor_strerror[Pointer[U8] val](code: I32)
use @pony_register_thread[None]()
use @pony_unregister_thread[None]()

primitive HtRing fun apply(): U32 => 1            // examples/ring
primitive HtPinger fun apply(): U32 => 2          // examples/message-ubench
primitive HtPingerDet fun apply(): U32 => 3
primitive HtFaninSender fun apply(): U32 => 4     // examples/fan-in
primitive HtFaninAnalyzer fun apply(): U32 => 5
primitive HtGupsStreamer fun apply(): U32 => 6    // examples/gups_basic
primitive HtGupsUpdater fun apply(): U32 => 7
primitive HtStorm fun apply(): U32 => 8
primitive HtFifoSrc fun apply(): U32 => 9         // examples/overload shape
primitive HtFifoSink fun apply(): U32 => 10
primitive HtSpreader fun apply(): U32 => 11       // examples/spreader

struct GpuMsg
  """gpu_msg_t: {u32 to, u32 behaviour, u64 arg} (pony_msgi_t's payload)."""
  var to: U32 = 0
  var behaviour: U32 = 0
  var arg: U64 = 0

class GpuMsgs
  """
  A chain of messages for one gpu_actor_sendv (pony_chain + pony_sendv,
  actor.c:773-817, 923-927): gpu_msg_t records packed two U64 words each
  (to | behaviour << 32 little-endian, then arg), so one FFI call hands the
  whole chain over, in order.
  """
  let _words: Array[U64]

  new create(capacity: USize = 0) =>
    _words = Array[U64](capacity * 2)

  fun ref push(to: U64, behaviour: U32, arg: U64) =>
    _words.push((to and 0xFFFF_FFFF) or (behaviour.u64() << 32))
    _words.push(arg)

  fun size(): USize => _words.size() / 2

  fun cpointer(): Pointer[U64] tag => _words.cpointer()

struct GpuActorConfig
  """gpu_actor_config_t."""
  var device: I32 = 0
  var n_ranks: U32 = 1
  var rank: U32 = 0
  var batch: U32 = 0
  var mailbox_cap: U32 = 0
  var max_exchange: U32 = 0
  var max_actors: U64 = 0
  var comm_id: Pointer[U8] tag = Pointer[U8]

struct GpuActorCounts
  """gpu_actor_counts_t (GPU_ACTOR_MAX_TYPES = 16 per-type counters)."""
  var steps: U64 = 0
  var delivered: U64 = 0
  var sent: U64 = 0
  var pending: U64 = 0
  var dropped: U64 = 0
  var remote: U64 = 0
  var active: U64 = 0
  embed delivered_by_type: GpuTypeCounts = GpuTypeCounts
  var atomics: U64 = 0

struct GpuTypeCounts
  var t0: U64 = 0
  var t1: U64 = 0
  var t2: U64 = 0
  var t3: U64 = 0
  var t4: U64 = 0
  var t5: U64 = 0
  var t6: U64 = 0
  var t7: U64 = 0
  var t8: U64 = 0
  var t9: U64 = 0
  var t10: U64 = 0
  var t11: U64 = 0
  var t12: U64 = 0
  var t13: U64 = 0
  var t14: U64 = 0
  var t15: U64 = 0

interface tag GpuRunNotify
  """Receives the completion of an asynchronous run."""
  be gpu_run_done(rc: I32, steps: U64)

primitive GpuRunDone
  """
  Completion callback handed to gpu_actor_run_async. The library calls it on
  its progress thread; registering that thread with the runtime first
  (pony.h:520-528) makes the behaviour call below a plain pony_sendv from an
  external thread — the pattern ASIO uses to deliver events (event.c:116-135).
  """
  fun apply(): @{(GpuRunNotify, I32, U64)} =>
    @{(notify: GpuRunNotify, rc: I32, steps: U64) =>
      @pony_register_thread()
      notify.gpu_run_done(rc, steps)
      // pair the registration (pony.h:520-536, as asio/epoll.c does): the
      // library may run the next asynchronous run on a new thread
      @pony_unregister_thread()
    }

class GpuActors
  """
  Thin owner of the engine for one process: init on create, shutdown on
  dispose. Error codes are returned as-is.
  """
  let _cfg: GpuActorConfig

  new create(device: I32 = 0, batch: U32 = 0, mailbox_cap: U32 = 0) =>
    _cfg = GpuActorConfig
    _cfg.device = device
    _cfg.batch = batch
    _cfg.mailbox_cap = mailbox_cap
    @gpu_actor_init(_cfg)

  fun register(type_id: U32, state_words: U32, table: U32): I32 =>
    @gpu_actor_type_register(type_id, state_words, table)

  fun param(type_id: U32, idx: U32, value: U64): I32 =>
    @gpu_actor_type_param(type_id, idx, value)

  fun reserve(type_id: U32, n: U64): I32 =>
    @gpu_actor_type_reserve(type_id, n)

  fun create_actors(type_id: U32, count: U64): U64 =>
    """pony_create in bulk; returns the first id (GPU_ACTOR_NONE on error)."""
    var first: U64 = -1
    if @gpu_actor_create(type_id, count, addressof first) != 0 then
      first = -1
    end
    first

  fun config(type_id: U32, batch: U32, mailbox_cap: U32 = 0): I32 =>
    """The fork's _batch() hint (actor.c:410-416) and the zone sizing hint."""
    @gpu_actor_type_config(type_id, batch, mailbox_cap)

  fun priority(type_id: U32, priority': I32): I32 =>
    """The fork's _priority() hint (actor.c:414-416, scheduler.c:1053-1068)."""
    @gpu_actor_type_priority(type_id, priority')

  fun send(to: U64, behaviour: U32, arg: U64): I32 =>
    """pony_sendi: staged on the host, injected by the next run (no sync)."""
    @gpu_actor_send(to, behaviour, arg)

  fun sendv(msgs: GpuMsgs box): I32 =>
    """pony_sendv of a chain: one H2D copy for all of it."""
    @gpu_actor_sendv(msgs.cpointer(), msgs.size().u64())

  fun run(max_steps: U64 = 0): U64 =>
    var steps: U64 = 0
    @gpu_actor_run(max_steps, addressof steps)
    steps

  fun run_async(notify: GpuRunNotify, max_steps: U64 = 0): I32 =>
    """Returns at once; notify.gpu_run_done(rc, steps) arrives when the run ends."""
    @gpu_actor_run_async(max_steps, GpuRunDone(), notify)

  fun live(type_id: U32): U64 =>
    var n: U64 = 0
    @gpu_actor_type_live(type_id, addressof n)
    n

  fun state(type_id: U32, first: U64, n: U64, words: USize): Array[U64] iso^ =>
    """Field-major: out(w * n + i) = word w of actor first + i."""
    let out = recover Array[U64].init(0, words * n.usize()) end
    @gpu_actor_state_read(type_id, first, n, out.cpointer())
    out

  fun counts(): GpuActorCounts =>
    let c = GpuActorCounts
    @gpu_actor_counts(c)
    c

  fun strerror(code: I32): String =>
    String.copy_cstring(@gpu_actor_strerror(code))

  fun dispose() =>
    @gpu_actor_wait(Pointer[U64])
    @gpu_actor_shutdown()

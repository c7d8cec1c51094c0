"""
examples/fan-in (main.pony:103-254) on the GPU engine, the shape SURVEY C3
measures: `senders` Sender actors (Sender.send_msgs, main.pony:241-250: pick an
Analyzer with rand.int_unbiased, send msg_from_sender, send itself send_msgs
again) into `analyzers` Analyzer actors (msg_from_sender: count += 1,
main.pony:219-220). The Coordinator/Receiver/timer reporting loop is host-side
in the reference and is replaced by one run to quiescence with a message
budget per sender. Every Sender is seeded Rand() = Rand(5489, 0) as in the
reference (main.pony:235). Analyzers are commutative ("reducible" handler
table): their messages are applied as device atomics when sent.
Mirrors ponyc_amd/workloads.py:fanin and tests/golden/fanin_1000_a4_p100.
"""
use "gpu_actor"

actor Main is GpuRunNotify
  let _env: Env
  let _gpu: GpuActors
  let _senders: U64 = 100_000
  let _analyzers: U64 = 4
  let _msgs: U64 = 100

  new create(env: Env) =>
    _env = env
    _gpu = GpuActors
    _gpu.register(0, 2, HtFaninAnalyzer())
    let afirst = _gpu.create_actors(0, _analyzers)
    _gpu.register(1, 4, HtFaninSender())
    _gpu.param(1, 0, _analyzers)
    _gpu.param(1, 1, afirst)
    _gpu.param(1, 2, _msgs)               // send_msgs budget per Sender
    _gpu.param(1, 3, 0)                   // every Sender: Rand() (seed 5489)
    let sfirst = _gpu.create_actors(1, _senders)
    // Sender.create calls send_msgs(): one chain for all of them
    let m = GpuMsgs(_senders.usize())
    var i: U64 = 0
    while i < _senders do m.push(sfirst + i, 0, 0); i = i + 1 end
    _gpu.sendv(m)
    _gpu.run_async(this)

  be gpu_run_done(rc: I32, steps: U64) =>
    // analyzer state: [count, xor of payloads] per analyzer
    let st = _gpu.state(0, 0, _analyzers, 2)
    var total: U64 = 0
    var a: USize = 0
    while a < _analyzers.usize() do
      try total = total + st(a)? end
      a = a + 1
    end
    _env.out.print("rc " + rc.string() + ": " + total.string() +
      " messages at the analyzers in " + steps.string() + " supersteps")
    _gpu.dispose()

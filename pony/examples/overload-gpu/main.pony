"""
examples/overload (main.pony:1-60) on the GPU engine: many senders fire at
few receivers that cannot keep up; backpressure mutes the senders while a
receiver is overloaded (actor.c:340-381, 898-921; DESIGN.md §2) instead of
letting its mailbox grow without bound. The receivers here are the FIFO probe
sinks (order-sensitive fold of every message), so the run is also a per-pair
FIFO check: the sinks' violation counters stay 0.
Mirrors ponyc_amd/workloads.py:fifo and tests/test_gpu_backpressure.py.
"""
use "gpu_actor"

actor Main is GpuRunNotify
  let _env: Env
  let _gpu: GpuActors
  let _sinks: U64 = 4

  new create(env: Env) =>
    _env = env
    _gpu = GpuActors(0, 100, 16)          // device 0, batch 100, mailbox_cap 16
    let senders: U64 = 100_000
    _gpu.register(0, 11, HtFifoSink())
    _gpu.param(0, 0, _sinks)
    let kfirst = _gpu.create_actors(0, _sinks)
    _gpu.register(1, 3, HtFifoSrc())
    _gpu.param(1, 0, kfirst)
    _gpu.param(1, 1, _sinks)
    _gpu.param(1, 2, 10)                  // Sender.fire() ten times each
    let sfirst = _gpu.create_actors(1, senders)
    let m = GpuMsgs(senders.usize())
    var i: U64 = 0
    while i < senders do m.push(sfirst + i, 0, 1); i = i + 1 end
    _gpu.sendv(m)
    _gpu.run_async(this)

  be gpu_run_done(rc: I32, steps: U64) =>
    let st = _gpu.state(0, 0, _sinks, 11)   // [h, n, violations, last seq x 8] per sink
    var n: U64 = 0
    var bad: U64 = 0
    var k: USize = 0
    while k < _sinks.usize() do
      try
        n = n + st(_sinks.usize() + k)?
        bad = bad + st((2 * _sinks.usize()) + k)?
      end
      k = k + 1
    end
    _env.out.print("rc " + rc.string() + ": " + n.string() + " messages received, " +
      bad.string() + " FIFO violations, " + steps.string() + " supersteps")
    _gpu.dispose()

"""
examples/message-ubench (main.pony:54-56, 223-286) on the GPU engine: N
pingers, each started with `initial` pings; every ping is forwarded to pinger
rand.int(N) until the per-pinger forward budget is spent. The run is
asynchronous: Main stays responsive and prints the totals when the engine's
completion message arrives (gpu_actor_run_async -> GpuRunNotify).
Mirrors ponyc_amd/workloads.py:ubench and bench.py (C2).
"""
use "gpu_actor"

actor Main is GpuRunNotify
  let _env: Env
  let _gpu: GpuActors
  let _n: U64 = 1_048_576

  new create(env: Env) =>
    _env = env
    _gpu = GpuActors
    _gpu.register(0, 3, HtPinger())
    _gpu.param(0, 0, _n)                  // N
    _gpu.param(0, 2, 100)                 // forward budget
    _gpu.param(0, 3, 5489)                // seed
    let first = _gpu.create_actors(0, _n)
    _gpu.param(0, 1, first)
    // SyncLeader.tell_all_to_go: 5 rounds of pings as one chain (one sendv)
    let m = GpuMsgs((5 * _n).usize())
    var k: U64 = 0
    while k < 5 do
      var i: U64 = 0
      while i < _n do m.push(first + i, 0, 42); i = i + 1 end
      k = k + 1
    end
    _gpu.sendv(m)
    _gpu.run_async(this)

  be gpu_run_done(rc: I32, steps: U64) =>
    let c = _gpu.counts()
    _env.out.print("rc " + rc.string() + ": " + c.delivered.string() +
      " pings in " + steps.string() + " supersteps")
    _gpu.dispose()

"""
examples/ring (main.pony:3-24, 46-85) on the GPU engine: `count` rings of
`size` actors; the first actor of each ring is told its neighbour (set) and
then passes a token `pass` times around. Mirrors ponyc_amd/workloads.py:ring
and tests/golden/ring_1000x10_p500.
"""
use "gpu_actor"

actor Main
  new create(env: Env) =>
    let size: U64 = 1000
    let count: U64 = 100
    let pass: U64 = 10000
    let gpu = GpuActors
    gpu.register(0, 4, HtRing())
    gpu.param(0, 0, size)
    let first = gpu.create_actors(0, size * count)
    var j: U64 = 0
    while j < count do
      let head = first + (j * size)
      gpu.send(head, 0, head + 1)           // set(next)
      gpu.send(head, 1, pass)               // pass(pass)
      j = j + 1
    end
    let steps = gpu.run()
    let c = gpu.counts()
    env.out.print(c.delivered.string() + " messages, " + steps.string() + " supersteps")
    gpu.dispose()

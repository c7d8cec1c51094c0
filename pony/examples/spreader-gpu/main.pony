"""
examples/spreader (main.pony:1-48) on the GPU engine: the root's behaviour
spawns two Spreaders (pony_create inside a behaviour, actor.c:688-734), down to
depth `count`; results are summed back to the root, which records
"<2^count - 1> actors". Ids of spawned actors are reserved up front
(gpu_actor_type_reserve). Mirrors tests/golden/spreader_c12.
"""
use "gpu_actor"

actor Main
  new create(env: Env) =>
    let count: U64 = 12
    let gpu = GpuActors
    gpu.register(0, 5, HtSpreader())
    gpu.reserve(0, (1 << count) - 2)
    let root = gpu.create_actors(0, 1)
    gpu.send(root, 0, (U64(0xFFFF_FFFF) << 32) or count)   // Spreader(env) -> spread
    gpu.run()
    let st = gpu.state(0, 0, 1, 5)
    try env.out.print(st(4)?.string() + " actors") end
    gpu.dispose()

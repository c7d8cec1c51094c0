"""
examples/gups_basic (main.pony:40-216) on the GPU engine: `updaters` Updater
actors hold the table slices (table[k] = k + index * size, main.pony:148-155)
and `streamers` Streamer actors stream PolyRand data (main.pony:167-216), each
datum d as one message to updater (d >> shift) and mask, which applies
table[d & (size - 1)] ^= d (main.pony:157-162). Streamer i is seeded
chunk * iterate * i and runs `iterate` + 1 chunks (apply(iterate) recursing
down to 0). Updaters are commutative (XOR): applied as device atomics.
The elapsed time and GUPS are printed as the reference does.
Mirrors ponyc_amd/workloads.py:gups and tests/golden/gups_l16_u8_s4_c1024_i10.
"""
use "gpu_actor"
use "time"

actor Main is GpuRunNotify
  let _env: Env
  let _gpu: GpuActors
  let _start: U64
  let _updates: U64

  new create(env: Env) =>
    _env = env
    _gpu = GpuActors
    let logtable: U64 = 20
    let updaters: U64 = 8
    let streamers: U64 = 4
    let chunk: U64 = 1024
    let iterate: U64 = 10000
    let size = (U64(1) << logtable) / updaters
    _updates = streamers * chunk * (iterate + 1)
    _gpu.register(0, size.u32(), HtGupsUpdater())
    _gpu.param(0, 0, size)
    let ufirst = _gpu.create_actors(0, updaters)
    _gpu.register(1, 2, HtGupsStreamer())
    _gpu.param(1, 0, chunk)
    _gpu.param(1, 1, size.bitwidth() - size.clz())   // shift (main.pony:102)
    _gpu.param(1, 2, updaters - 1)                   // mask
    _gpu.param(1, 3, ufirst)
    _gpu.param(1, 5, chunk * iterate)                // seed stride
    let sfirst = _gpu.create_actors(1, streamers)
    let m = GpuMsgs(streamers.usize())
    var i: U64 = 0
    while i < streamers do m.push(sfirst + i, 0, iterate); i = i + 1 end
    _start = Time.nanos()
    _gpu.sendv(m)
    _gpu.run_async(this)

  be gpu_run_done(rc: I32, steps: U64) =>
    let elapsed = (Time.nanos() - _start).f64()
    _env.out.print("rc " + rc.string() + " Time: " + (elapsed / 1e9).string() +
      " GUPS: " + (_updates.f64() / elapsed).string())
    _gpu.dispose()

import sys, time, json, os
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from ponyc_amd import workloads as W
from ponyc_amd.engine import Engine
for name, setup in [("ring", lambda e: W.ring(e, 1000, 100, 10000)), ("ring_prog", lambda e: W.ring_prog(e, 1000, 100, 10000)), ("ring_one", lambda e: W.ring(e, 1000, 1, 10000))]:
    res = []
    for _ in range(3):
        e = Engine(device=0); setup(e); e.sync()
        t0 = time.perf_counter(); steps = e.run(); e.sync(); secs = time.perf_counter() - t0
        c = e.counts(); e.shutdown(); res.append(round(c["delivered"] / secs / 1e6, 2))
    print(json.dumps({"case": name, "mmsgs_per_s": res, "steps": steps}), flush=True)

"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

  * rng_kats.json   : the known-answer vectors of packages/random/_test.pony
                      (xoroshiro128+ and SplitMix64, seed 5489), extracted from
                      the reference test file as data;
  * <workload>.npz  : final per-actor state produced by the reference runtime
                      (oracle/_ref/libponyrt.so, built from /root/reference by
                      oracle/Makefile) running the C drivers in oracle/harness/
                      with 4 scheduler threads;
  * manifest.json   : configs, seeds and totals.

Run from the repo root in the build container (needs /root/reference):
    python tests/golden/gen_golden.py [fixture names...]   (default: all)
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

REF_TEST = "/root/reference/packages/random/_test.pony"

# (fixture name, harness, args, field names, reshape rows)
CONFIGS = [
    ("ring_64x4_p100", "ring", {"size": 64, "count": 4, "pass": 100}, ["recv", "done"]),
    ("ring_1000x10_p500", "ring", {"size": 1000, "count": 10, "pass": 500}, ["recv", "done"]),
    ("ubench_4096_i4_b32", "ubench", {"pingers": 4096, "initial": 4, "budget": 32},
     ["x", "y", "count"]),
    ("ubench_1000_i5_b10", "ubench", {"pingers": 1000, "initial": 5, "budget": 10},
     ["x", "y", "count"]),
    ("ubench_det_4096_i4_h32", "ubench", {"pingers": 4096, "initial": 4, "det": 1, "hops": 32},
     ["count", "acc"]),
    ("fanin_1000_a4_p100", "fanin", {"senders": 1000, "analyzers": 4, "msgs": 100},
     ["count", "acc"]),
    ("fanin_5000_a16_p20_s1", "fanin", {"senders": 5000, "analyzers": 16, "msgs": 20,
                                        "seedmode": 1}, ["count", "acc"]),
    ("gups_l16_u8_s4_c1024_i10", "gups", {"logtable": 16, "updaters": 8, "streamers": 4,
                                          "chunk": 1024, "iterate": 10}, ["table"]),
    ("fifo_64_8_b10_m4", "fifo", {"sources": 64, "sinks": 8, "bursts": 10, "m": 4},
     ["h", "n", "violations"]),
    # every node's final _result (sorted: ids are runtime pointers) + the root's total
    ("spreader_c12", "spreader", {"count": 12}, ["results_sorted", "total"]),
]


def extract_kats() -> dict:
    src = open(REF_TEST).read()
    out = {}
    for cls, key in (("_TestXorOshiro128Plus", "xoroshiro128plus_5489"),
                     ("_TestSplitMix64", "splitmix64_5489")):
        body = src.split(f"class iso {cls}")[1].split("class iso ")[0]
        out[key] = [int(v) for v in re.findall(r"assert_eq\[U64\]\(\w+\.next\(\), (\d+)\)", body)]
    return out


def main() -> None:
    pyoracle.build(reference=True)
    only = set(sys.argv[1:])
    manifest = {"generator": "tests/golden/gen_golden.py",
                "reference": "KittyMac/ponyc src/libponyrt @ VERSION 0.33.0, unmodified",
                "threads": 4, "fixtures": {}}
    mpath = os.path.join(HERE, "manifest.json")
    if only and os.path.exists(mpath):
        with open(mpath) as f:
            manifest = json.load(f)
    if not only:
        kats = extract_kats()
        with open(os.path.join(HERE, "rng_kats.json"), "w") as f:
            json.dump(kats, f, indent=1)
    tmp = os.path.join(HERE, "_tmp")
    os.makedirs(tmp, exist_ok=True)
    for name, harness, args, fields in CONFIGS:
        if only and name not in only:
            continue
        a = dict(args)
        a["threads"] = 4
        out = os.path.join(tmp, name + ".bin")
        info, data = pyoracle.run_harness(harness, a, out)
        arrays = {}
        if fields == ["table"]:
            arrays["table"] = data
        else:
            rows = data.reshape(len(fields), -1)
            for i, fld in enumerate(fields):
                arrays[fld] = rows[i]
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        manifest["fixtures"][name] = {"harness": harness, "args": args, "fields": fields,
                                      "msgs": info["msgs"]}
        print(name, info)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()

"""Build A/B variants of the engine (compile-time toggles) into
ponyc_amd/variants/lib_<name>.so, one after another (each build compiles
its units in parallel).
    python scripts/build_ab.py name=-DFOO=1,-DBAR=0 name2=... [--only HT]
--only HT compiles one k_step table (GPA_STEP_ONLY, ~30 s per variant)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ponyc_amd import build as b  # noqa: E402

args = sys.argv[1:]
only = None
if "--only" in args:
    i = args.index("--only")
    only = args[i + 1]
    del args[i:i + 2]
os.makedirs(os.path.join(ROOT, "ponyc_amd", "variants"), exist_ok=True)
for spec in args:
    name, _, defs = spec.partition("=")
    d = [x for x in defs.split(",") if x]
    if only is not None:
        d.append(f"-DGPA_STEP_ONLY={only}")
    out = os.path.join(ROOT, "ponyc_amd", "variants", f"lib_{name}.so")
    print(b.build(defines=d, out=out), flush=True)

"""Regenerates tests/golden/jsf32_seed1.json from oracle/_ref/ref_jsf (the reference's jsf.h
compiled in place by oracle/Makefile); only where /root/reference exists."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
v = [int(x) for x in subprocess.check_output([os.path.join(ROOT, "oracle", "_ref", "ref_jsf"), "200000"]).split()]
json.dump({"_doc": "first draws of the reference's jsf32 (3rd/rng/jsf.h, default seed) from oracle/_ref/ref_jsf "
                   "(tests/gen_jsf32.py)", "first": v[:256], "n": len(v), "last_index": len(v) - 1, "last": v[-1],
           "pct_lt_50": sum(1 for x in v if x % 100 < 50)},
          open(os.path.join(ROOT, "tests", "golden", "jsf32_seed1.json"), "w"))

"""Generates tests/golden/cpc_vectors.json by running the reference's vendored
datasketches (compiled in place by oracle/Makefile into oracle/_ref/ref_sketch)
on seeded uint32 streams. Run from the repo root in the container that has
/root/reference; the committed JSON is what tests use elsewhere."""
import json
import subprocess

import numpy as np

SIZES = [1, 2, 3, 17, 191, 192, 193, 1000, 6911, 6912, 20000, 100000, 700000, 2500000]


def main():
    rng = np.random.default_rng(0x5eedc0c)
    cases = []
    for n in SIZES:
        seed = int(rng.integers(0, 2**31))
        v = np.random.default_rng(seed).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        body = " ".join(map(str, v.tolist()))
        inp = f"cpc_u32 0 {n} {body}\ncpc_u32 1 {n} {body}\n"
        out = subprocess.run(["oracle/_ref/ref_sketch"], input=inp.encode(), capture_output=True, check=True)
        hip, icon = [float(x) for x in out.stdout.split()]
        cases.append({"n": n, "seed": seed, "hip": hip, "icon": icon})
    json.dump({"_doc": "CPC lg_k=11 estimates from the reference datasketches for numpy default_rng(seed).integers(0,2**32,n) as uint32 items",
               "cases": cases}, open("tests/golden/cpc_vectors.json", "w"), indent=1)


if __name__ == "__main__":
    main()

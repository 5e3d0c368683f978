"""device vs host record index on synthetic blobs: report the first mismatching field / offset"""
import sys
import numpy as np
sys.path.insert(0, '.')
import pktvisor_amd as pa
from tests.test_index_parallel import blob
h = pa.PvHandlers(num_periods=1, max_records=1 << 22)
F = ("n_records", "bytes_used", "first_sec", "first_nsec", "last_sec", "last_nsec", "monotone", "n_sec_changes")
for kind, n in (("small", 120000), ("mixed", 4000), ("adv", 1500)):
    for seed in range(3):
        b = blob(np.random.default_rng(seed), n, kind)
        if len(b) > (60 << 20):
            continue
        a = pa.RecordIndex(b)
        offs, sci, scs, info = h.index_device(b)
        bad = [f for f in F if getattr(a.info, f) != getattr(info, f)]
        d = np.nonzero(a.offsets[: len(offs)] != offs[: len(a.offsets)])[0]
        k = a.info.n_sec_changes
        sc_ok = np.array_equal(a.sc_idx[:k], sci[:k]) and np.array_equal(a.sc_sec[:k], scs[:k])
        print(kind, seed, len(b), "bad", [(f, getattr(a.info, f), getattr(info, f)) for f in bad], "offdiff", d[:3], "sc_ok", sc_ok)
        if bad:
            ln = a.info.n_records
            last = int(a.offsets[ln - 1])
            print("  host last off", last, "sec", np.frombuffer(b, np.uint32, 1, last)[0], "dev last off", int(offs[ln - 1]))

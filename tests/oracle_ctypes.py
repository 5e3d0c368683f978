"""ctypes loader for oracle/liboracle.so — test infrastructure only (the checker)."""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        lib.pvo_run.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        lib.pvo_run.restype = ctypes.c_int
        lib.pvo_free.argtypes = [ctypes.c_void_p]
        lib.pvo_cpc_u32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        lib.pvo_cpc_u32.restype = ctypes.c_double
        lib.pvo_icon.argtypes = [ctypes.c_uint32]
        lib.pvo_icon.restype = ctypes.c_double

    def run_bytes(self, data: bytes, **cfg) -> dict:
        s = ";".join(f"{k}={v}" for k, v in cfg.items() if v is not None and v != "")
        out = ctypes.c_void_p()
        rc = self.lib.pvo_run(data, len(data), s.encode(), ctypes.byref(out))
        txt = ctypes.string_at(out.value).decode() if out.value else ""
        self.lib.pvo_free(out)
        if rc != 0:
            raise RuntimeError(f"oracle failed ({rc}): {txt}")
        return json.loads(txt)

    def run_policy(self, files, period: int = 0, merged: bool = False, prometheus: bool = False, **cfg) -> dict:
        """Policy::_get_merged_buckets over like handlers, one per capture (pvo_run_policy)."""
        s = ";".join(f"{k}={v}" for k, v in cfg.items() if v is not None and v != "")
        bufs = [ctypes.create_string_buffer(f, len(f)) for f in files]
        arr = (ctypes.c_void_p * len(files))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
        lens = (ctypes.c_size_t * len(files))(*[len(f) for f in files])
        out = ctypes.c_void_p()
        self.lib.pvo_run_policy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p,
                                            ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        rc = self.lib.pvo_run_policy(arr, lens, len(files), s.encode(), period, int(merged), int(prometheus),
                                     ctypes.byref(out))
        txt = ctypes.string_at(out.value).decode() if out.value else ""
        self.lib.pvo_free(out)
        if rc != 0:
            raise RuntimeError(f"oracle failed ({rc}): {txt}")
        return json.loads(txt)

    def run_file(self, path, **cfg) -> dict:
        with open(path, "rb") as f:
            return self.run_bytes(f.read(), **cfg)


def load() -> Oracle:
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
    return Oracle(ctypes.CDLL(LIB))


def jget(d, path):
    for p in path.split("."):
        if isinstance(d, list):
            d = d[int(p)]
        else:
            d = d[p]
    return d

"""Start WORLD ranks of tests/dist_worker.py as child processes (127.0.0.1 rendezvous)."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, args, timeout=240):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs.append(subprocess.Popen([sys.executable, "-m", "tests.dist_worker", *args], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    failed = [(r, p.returncode, o) for r, (p, o) in enumerate(zip(procs, outs)) if p.returncode != 0]
    if failed:
        # the root cause first: a rank whose peers then saw their connection close
        failed.sort(key=lambda f: "Connection closed by peer" in f[2])
        raise RuntimeError("\n".join(f"rank {r} failed ({rc}):\n{o[-2500:]}" for r, rc, o in failed[:2]))
    return outs

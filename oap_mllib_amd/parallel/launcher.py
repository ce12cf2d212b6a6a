"""Standalone gang launcher: starts all ranks of a job together, one process per GPU.

The reference relies on Spark running all ``executorNum`` tasks concurrently with no barrier and
forces ``spark.task.maxFailures=1`` so a retried task cannot rejoin a stale KVS
(SURVEY.md §2.4 "Gang scheduling", examples/kmeans/run.sh:24).  This launcher gives the
standalone (non-Spark) deployment gang semantics: every rank starts together on 127.0.0.1 with a
fresh port, ranks are pinned to GPUs through LOCAL_RANK, and if any rank exits non-zero the
others are terminated (no hung peers) and the launcher returns that exit code.

    python -m oap_mllib_amd.parallel.launcher --nproc 8 my_job.py --arg ...
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(host: str = "127.0.0.1", start: int = 0) -> int:
    """A free TCP port (kernel-assigned, or the first bindable one >= start)."""
    if start <= 0:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind((host, 0))
            return s.getsockname()[1]
    for p in range(start, 65535):
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind((host, p))
                return p
            except OSError:
                continue
    raise RuntimeError("no free port")


def launch(cmd: list[str], nproc: int, host: str = "127.0.0.1", port: int = 0,
           env: dict | None = None, timeout_s: float | None = None) -> int:
    port = port or free_port(host)
    procs = []
    base = dict(os.environ if env is None else env)
    for r in range(nproc):
        e = dict(base)
        e.update(RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_RANK=str(r),
                 LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=host, MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = False
            for p in procs:
                c = p.poll()
                if c is None:
                    alive = True
                elif c != 0 and rc == 0:
                    rc = c
            if rc != 0 or not alive:
                break
            if timeout_s is not None and time.time() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    return launch([sys.executable, a.script] + a.args, a.nproc, a.host, a.port,
                  timeout_s=a.timeout)


if __name__ == "__main__":
    raise SystemExit(main())

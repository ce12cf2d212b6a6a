"""Runs a test worker function in N processes (a gloo world on 127.0.0.1)."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RUNNER = r'''
import json, os, sys, importlib
sys.path.insert(0, {root!r})
sys.path.insert(0, os.path.join({root!r}, "tests"))
mod = importlib.import_module({module!r})
res = getattr(mod, {func!r})(**json.loads({kwargs!r}))
with open(os.path.join({outdir!r}, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump(res, f)
'''


def run_world(module: str, func: str, nproc: int = 2, timeout: float = 240.0,
              env: dict | None = None, **kwargs):
    from oap_mllib_amd.parallel.launcher import launch

    with tempfile.TemporaryDirectory() as d:
        script = os.path.join(d, "runner.py")
        with open(script, "w") as f:
            f.write(_RUNNER.format(root=ROOT, module=module, func=func,
                                   kwargs=json.dumps(kwargs), outdir=d))
        e = dict(os.environ)
        e.update(env or {})
        e.setdefault("OMP_NUM_THREADS", "2")
        rc = launch([sys.executable, script], nproc, env=e, timeout_s=timeout)
        outs = []
        for r in range(nproc):
            p = os.path.join(d, f"rank{r}.json")
            outs.append(json.load(open(p)) if os.path.exists(p) else None)
        return rc, outs

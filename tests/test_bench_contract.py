"""bench.py's driver contract on the CPU: presets, argument handling, the self-launch of N ranks."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("oap_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_world_size_mismatch_is_refused(monkeypatch, capsys):
    monkeypatch.setenv("WORLD_SIZE", "3")
    assert _bench().main(["--gpus", "2"]) == 2
    assert "WORLD_SIZE=3" in capsys.readouterr().err


def _run_bench(args, extra_env=None):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env.update(OAP_BENCH_DEVICE="cpu", MASTER_ADDR="127.0.0.1")
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    return json.loads(lines[0])


SMALL = ["--rows", "6000", "--dim", "8", "--k", "5", "--steps", "3", "--warmup", "1",
         "--skip-fit", "--box", "4", "--sigma", "3"]


def test_self_launch_two_ranks_cpu():
    """`bench.py --gpus 2` with no launcher environment starts its own 2-rank world (the driver's
    8-GPU sweep path), every rank joins the collectives, rank 0 prints one JSON line."""
    one = _run_bench(["--gpus", "1"] + SMALL)
    two = _run_bench(["--gpus", "2"] + SMALL)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["extra"]["world_size"] == 2 and two["config"]["parallelism"] == "dp2"
    assert two["steps"] == 3 and two["warmup"] == 1 and two["scaling"] == "strong"
    # strong scaling over identical global data: same fit for any world size
    assert one["extra"]["cost"] == two["extra"]["cost"]
    assert one["extra"]["center_shift_history"] == two["extra"]["center_shift_history"]
    assert two["extra"]["max_center_shift_last"] > 0  # overlapping blobs: centers still move
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "vs_baseline",
                "dtype", "data", "config"):
        assert key in two


def test_presets_match_baseline_configs(monkeypatch):
    b = _bench()
    seen = {}

    def fake(args, w):  # capture the resolved preset instead of running on a GPU
        seen.update(rows=args.rows, dim=args.dim, k=args.k, dtype=args.dtype)
        raise SystemExit(0)

    monkeypatch.setattr(b, "bench_kmeans", fake)
    import oap_mllib_amd as O

    monkeypatch.setattr(O, "init_world", lambda *a, **k: None)
    for cfg, want in [("kmeans", (100_000_000, 50, 200, "f32")),
                      ("kmeans_bf16", (1_000_000_000, 100, 1000, "bf16"))]:
        seen.clear()
        with pytest.raises(SystemExit):
            b.main(["--config", cfg])
        assert (seen["rows"], seen["dim"], seen["k"], seen["dtype"]) == want
    with pytest.raises(SystemExit):
        b.main(["--config", "kmeans", "--rows", "1000", "--k", "7"])
    assert seen["rows"] == 1000 and seen["k"] == 7 and seen["dim"] == 50


def test_cpu_baseline_proxies_report_rates():
    """The CPU-proxy baselines (benchmarks/cpu_baseline.py) return labelled, positive rates."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    from cpu_baseline import kmeans_proxy, pca_proxy

    rng = np.random.default_rng(0)
    X = rng.normal(size=(20000, 8))
    km = kmeans_proxy(X, X[:5].copy(), iters=2)
    assert km["samples_per_sec"] > 0 and km["rows"] == 20000 and "proxy" in km["note"]
    pc = pca_proxy(X, 3, full_rows=1_000_000)
    assert pc["fit_s_scaled"] > 0 and pc["rows_scaled_to"] == 1_000_000

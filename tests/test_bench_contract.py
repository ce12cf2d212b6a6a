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


def _run_script(script, args):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env.update(OAP_BENCH_DEVICE="cpu", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)] + args, env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    return json.loads(lines[0])


def test_kmeans_bench_eight_ranks_cpu():
    """The driver's 8-GPU sweep, rehearsed on CPU ranks: `bench.py --gpus 8` self-launches an
    8-rank world over the same global rows; the fixed-point statistics make the fit bitwise
    the 1-rank one (every center shift; the cost to fp64 summation order)."""
    one = _run_bench(["--gpus", "1"] + SMALL)
    eight = _run_bench(["--gpus", "8"] + SMALL)
    assert eight["n_gpus"] == 8 and eight["extra"]["world_size"] == 8
    assert eight["config"]["parallelism"] == "dp8"
    # (centers: bitwise — the shift history is computed from them; the cost is an fp64 sum of
    # per-row costs over 8 shards, so its last bits follow the summation order)
    assert one["extra"]["center_shift_history"] == eight["extra"]["center_shift_history"]
    assert abs(one["extra"]["cost"] - eight["extra"]["cost"]) <= 1e-12 * one["extra"]["cost"]


def test_pca_bench_self_launch_eight_ranks_cpu():
    """benchmarks/bench_pca.py --gpus 8: one global dataset sharded 8 ways; the statistics are
    fp64 sums allreduced in another order, so eigenvalues agree to ~1e-12 relative."""
    args = ["--rows", "4000", "--dim", "16", "--k", "4", "--reps", "1", "--cpu-rows", "0",
            "--precision", "exact"]
    one = _run_script("benchmarks/bench_pca.py", ["--gpus", "1"] + args)
    eight = _run_script("benchmarks/bench_pca.py", ["--gpus", "8"] + args)
    assert one["n_gpus"] == 1 and eight["n_gpus"] == 8
    assert eight["extra"]["world_size"] == 8 and eight["config"]["parallelism"] == "dp8"
    a, b = one["extra"]["explained_variance"], eight["extra"]["explained_variance"]
    assert len(a) == len(b) == 4
    for x, y in zip(a, b):
        assert abs(x - y) <= 1e-10 * max(abs(x), 1e-300)
    assert abs(one["extra"]["pc_abs_sum"] - eight["extra"]["pc_abs_sum"]) <= 1e-8


def test_als_bench_self_launch_eight_ranks_cpu():
    """benchmarks/bench_als.py --gpus 8: the same global ratings (block-keyed generator) sharded
    8 ways through the distributed shuffle; the factors match the 1-rank fit (fp64 Gramian sums
    in another order: agreement to float rounding)."""
    args = ["--ratings", "20000", "--users", "600", "--items", "150", "--rank", "6",
            "--iters", "2", "--cpu-ratings", "0"]
    one = _run_script("benchmarks/bench_als.py", ["--gpus", "1"] + args)
    eight = _run_script("benchmarks/bench_als.py", ["--gpus", "8"] + args)
    assert eight["n_gpus"] == 8 and eight["extra"]["world_size"] == 8
    assert one["config"]["ratings"] == eight["config"]["ratings"]
    assert one["config"]["users"] == eight["config"]["users"]
    assert one["extra"]["failed_rows"] == eight["extra"]["failed_rows"] == 0
    for key in ("user_factor_sum", "item_factor_sum"):
        x, y = one["extra"][key], eight["extra"][key]
        assert abs(x - y) <= 1e-5 * abs(x), (key, x, y)
    import numpy as np

    np.testing.assert_allclose(one["extra"]["factor_head"], eight["extra"]["factor_head"],
                               rtol=1e-4, atol=1e-5)

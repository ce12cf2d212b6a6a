"""bench.py's driver contract on the CPU: presets, argument handling, refusal without a launcher."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("oap_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_multi_gpu_without_launcher_is_refused(monkeypatch, capsys):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert _bench().main(["--gpus", "2"]) == 2
    assert "torch.distributed.run" in capsys.readouterr().err


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

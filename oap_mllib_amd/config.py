"""One configuration object for the whole framework.

The reference scatters its knobs over Spark conf keys (``spark.oap.mllib.oneccl.kvs.ip`` /
``.port``, KMeansDALImpl.scala:40-44), ``spark.executor.cores`` (Utils.scala:51-58), env vars set
programmatically (``CCL_ATL_TRANSPORT``, OneCCL.scala:26-30) and hard-coded dispatch thresholds
(PCA ``numFeatures < 65535``, PCA.scala:103).  Here every knob has one documented name, resolved
in increasing priority from: defaults < environment (``OAP_MLLIB_<NAME>``) < Spark conf
(``spark.oap.mllib.<name>``, reference keys kept as aliases) < explicit overrides.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Mapping

# reference Spark-conf keys that keep working as aliases
SPARK_ALIASES = {
    "spark.oap.mllib.oneccl.kvs.ip": "rendezvous_host",
    "spark.oap.mllib.oneccl.kvs.port": "rendezvous_port",
    "spark.executor.cores": "cpu_threads",
}


@dataclasses.dataclass
class Config:
    #: "auto" (GPU when one is visible and the native engine loaded), "gpu", "cpu" (native CPU
    #: engine) or "vanilla" (pure numpy reference implementation, the Spark-MLlib fallback analog)
    device: str = "auto"
    #: explicit GPU ordinal; default = LOCAL_RANK % visible GPUs (one rank per GPU)
    device_id: int = -1
    #: share of free HBM the per-process arena may reserve
    hbm_fraction: float = 0.92
    #: host threads of the native CPU engine (0 = min(cores, 16))
    cpu_threads: int = 0
    #: storage dtype of GPU K-Means tables: "f32" or "bf16" (bf16 halves HBM bytes and uses 2
    #: instead of 3 MFMA products; assignments stay exact for the bf16 values)
    storage_dtype: str = "f32"
    #: collective watchdog (seconds); <= 0 disables
    comm_timeout_s: float = 600.0
    #: use RCCL for GPU ranks (else host/gloo collectives staged through pinned memory)
    use_rccl: bool = True
    #: a world of ONE GPU rank forms a real 1-rank RCCL communicator instead of the no-op local
    #: comm, so every device-collective branch of the multi-GPU drivers (grouped allreduces,
    #: comm-stream overlap, send/recv shuffles, chunked broadcasts) runs on a single GPU
    force_device_comm: bool = False
    rendezvous_host: str = "127.0.0.1"
    rendezvous_port: int = 0
    #: PCA statistics precision on the GPU: "exact" = the reference's fp64 (fp64 products and
    #: sums on the fp64 MFMA; fp64 input rows are kept as they are), "fast" = bf16-split products
    #: accumulated in fp32 then fp64 (~1e-6 relative; ~2.5x faster)
    pca_precision: str = "exact"
    #: PCA dispatch cap (the reference hard-codes numFeatures < 65535, PCA.scala:103)
    pca_max_features: int = 65535
    #: rows per pinned staging chunk during ingestion
    ingest_chunk_rows: int = 1 << 18
    #: K-Means rows per rank beyond which the fit streams them from host memory through HBM
    #: chunk buffers every iteration (0 = automatic: 60% of the device's total memory)
    hbm_budget_bytes: int = 0
    #: rows per HBM chunk of the streamed (out-of-core) K-Means fit
    stream_chunk_rows: int = 1 << 22
    log_level: str = "warn"
    log_file: str = ""
    #: directory for periodic training snapshots ("" = off; the sc.checkpointDir analogue)
    checkpoint_dir: str = ""
    #: K-Means iterations between snapshots (ALS uses its checkpointInterval param)
    checkpoint_interval: int = 10
    #: Spark version written into saved models' metadata (and PMML headers); "" = the
    #: installed pyspark's, else 3.1.1.  The reference builds one jar per Spark profile
    #: (3.0.0, 3.0.1, 3.0.2, 3.1.1, mllib-dal/pom.xml:151-224); here it is one knob.
    spark_version: str = ""
    #: native-layer tuning / diagnostic knobs ({"OAP_KMEANS_ROW_SCAN": "0", ...}), installed by
    #: init_world; the complete documented list is ``_native.knob_table()`` (runtime/knobs.cpp,
    #: docs/ARCHITECTURE.md "Knobs").  A knob not given here falls back to the environment
    #: variable of the same name.  From the environment / Spark conf: "NAME=value,NAME=value".
    native_knobs: dict = dataclasses.field(default_factory=dict)

    def replace(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)


def _coerce(field: dataclasses.Field, value: Any) -> Any:
    if field.name == "native_knobs":
        if isinstance(value, Mapping):
            return {str(k): str(v) for k, v in value.items()}
        out = {}
        for item in str(value).split(","):
            if item.strip():
                k, _, v = item.partition("=")
                out[k.strip()] = v.strip()
        return out
    t = field.type if isinstance(field.type, type) else {"str": str, "int": int, "float": float,
                                                         "bool": bool}.get(str(field.type), str)
    if t is bool:
        if isinstance(value, str):
            return value.strip().lower() in ("1", "true", "yes", "on")
        return bool(value)
    return t(value)


def resolve(overrides: Mapping[str, Any] | None = None,
            spark_conf: Mapping[str, str] | None = None,
            environ: Mapping[str, str] | None = None) -> Config:
    env = os.environ if environ is None else environ
    fields = {f.name: f for f in dataclasses.fields(Config)}
    values: dict[str, Any] = {}
    for name, f in fields.items():
        ev = env.get("OAP_MLLIB_" + name.upper())
        if ev is not None and ev != "":
            values[name] = _coerce(f, ev)
    if spark_conf:
        for key, val in spark_conf.items():
            name = SPARK_ALIASES.get(key)
            if name is None and key.startswith("spark.oap.mllib."):
                name = key[len("spark.oap.mllib."):].replace(".", "_")
            if name in fields:
                values[name] = _coerce(fields[name], val)
    for key, val in (overrides or {}).items():
        if key not in fields:
            raise KeyError(f"unknown config key '{key}'")
        values[key] = _coerce(fields[key], val)
    return Config(**values)


_current: Config | None = None


def get_config() -> Config:
    global _current
    if _current is None:
        _current = resolve()
    return _current


def set_config(cfg: Config | None = None, **overrides) -> Config:
    """Installs a process-wide configuration (``set_config(device="cpu")``)."""
    global _current
    base = cfg if cfg is not None else get_config()
    _current = base.replace(**overrides) if overrides else base
    return _current

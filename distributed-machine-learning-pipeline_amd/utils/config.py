"""Typed configuration with CLI flags, config files and environment overrides.

The reference has no configuration system at all: ports, addresses,
hyper-parameters and the health interval are compile-time constants
(``DSML/client/client.go:21-33,518,527``, ``DSML/cmd/gpu_device_server/main.go:13,23``,
``DSML/cmd/gpu_coordinator_server/main.go:13``,
``DSML/gpu_coordinator_service/gpu_coordinator_server.go:57``).
Here every such constant is a dataclass field whose default reproduces the
reference, and each field can be set (lowest to highest precedence) by

  1. the dataclass default,
  2. a YAML / JSON file (``--config path``; YAML read with ``safe_load``),
  3. an environment variable ``HIPDSML_<FIELD>`` (upper-case),
  4. an explicit command-line flag ``--field-name``.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, fields
from typing import Any, Dict, List, Optional, Sequence, Type, TypeVar

T = TypeVar("T")
ENV_PREFIX = "HIPDSML_"


@dataclass
class TrainConfig:
    """Data-parallel training job (one process per GPU under torchrun)."""
    model: str = "784-128-64-10"          # layer list; reference code: 784-128-10
    engine: str = "auto"                  # auto | fused (fp32 HIP step) | wide (bf16 MFMA GEMMs)
    batch: int = 64                       # per-replica batch (client.go:22)
    lr: float = 0.01                      # client.go:27
    momentum: float = 0.0
    weight_decay: float = 0.0
    epochs: int = 10                      # client.go:28
    steps: int = 0                        # >0: stop after this many steps (overrides epochs)
    init: str = "auto"                    # reference: U(-0.05, 0.05) (client.go:44-51) | kaiming;
                                          # auto = reference for fused, kaiming for wide
    seed: int = 0
    data: str = "synthetic"               # synthetic | mnist (idx files under data_dir)
    data_dir: str = ""
    samples: int = 60032                  # synthetic samples per replica
    sync: str = "auto"                    # auto | pkx | pkg | pkg2 | pk | pk2 | xact | xgmi | rccl | ring | torch
    ring_chunk_bytes: int = 1 << 20
    graph_steps: int = 50                 # steps per hipGraph (fused-exchange steps too); 0 = eager
    backend: str = "auto"                 # torch.distributed backend: auto | nccl | gloo
    device: str = "auto"                  # auto | cuda | cpu
    checkpoint: str = ""                  # path to write checkpoints to
    checkpoint_every: int = 0             # steps between checkpoints (0: end of each epoch)
    keep_checkpoints: int = 2
    resume: str = ""                      # checkpoint to resume from ("auto": latest at `checkpoint`)
    metrics: str = ""                     # JSON-lines metrics file ("-" = stdout)
    log_every: int = 0                    # steps between metric records (0: per epoch)
    eval: bool = True                     # run the test set after training
    trace: bool = False                   # roctx ranges around phases


@dataclass
class DeviceServerConfig:
    host: str = "127.0.0.1"
    ports: str = "5003,5004,5005"         # cmd/gpu_device_server/main.go:13-23
    gpus: str = ""
    device_ids: str = ""                  # default 1..n like the reference
    backend: str = "auto"                 # auto | host | hip
    mem_size: int = 64 << 20


@dataclass
class CoordinatorConfig:
    host: str = "127.0.0.1"
    port: int = 50051                     # cmd/gpu_coordinator_server/main.go:13
    health_interval: float = 5.0          # gpu_coordinator_server.go:57
    health_timeout: float = 2.0           # gpu_coordinator_server.go:103


def _parse_bool(s: str) -> bool:
    v = str(s).strip().lower()
    if v in ("1", "true", "yes", "on"):
        return True
    if v in ("0", "false", "no", "off", ""):
        return False
    raise ValueError(f"not a boolean: {s!r}")


def _coerce(tp: Any, raw: Any) -> Any:
    tp = {"int": int, "float": float, "str": str, "bool": bool}.get(tp, tp) if isinstance(tp, str) else tp
    if tp is bool:
        return raw if isinstance(raw, bool) else _parse_bool(raw)
    if tp is int and isinstance(raw, str):
        return int(raw, 0)
    return tp(raw)


def _field_type(f: dataclasses.Field) -> Any:
    return f.type if not isinstance(f.type, str) else {"int": int, "float": float, "str": str,
                                                        "bool": bool}[f.type]


def add_arguments(ap: argparse.ArgumentParser, cls: Type) -> None:
    """One ``--flag`` per dataclass field (default None = "not given")."""
    for f in fields(cls):
        tp = _field_type(f)
        flag = "--" + f.name.replace("_", "-")
        if tp is bool:
            ap.add_argument(flag, dest=f.name, default=None, type=_parse_bool, nargs="?", const=True,
                            help=f"(bool, default {f.default})")
        else:
            ap.add_argument(flag, dest=f.name, default=None, type=str,
                            help=f"({tp.__name__}, default {f.default})")
    if not any(a.dest == "config" for a in ap._actions):
        ap.add_argument("--config", default=None, help="YAML/JSON config file")


def load_file(path: str) -> Dict[str, Any]:
    with open(path) as fh:
        text = fh.read()
    if path.endswith(".json"):
        data = json.loads(text)
    else:
        import yaml

        data = yaml.safe_load(text) or {}
    if not isinstance(data, dict):
        raise ValueError(f"{path}: expected a mapping")
    return data


def resolve(cls: Type[T], ns: Optional[argparse.Namespace] = None,
            env: Optional[Dict[str, str]] = None, file_values: Optional[Dict[str, Any]] = None) -> T:
    env = os.environ if env is None else env
    names = {f.name: f for f in fields(cls)}
    vals: Dict[str, Any] = {}
    if ns is not None and getattr(ns, "config", None):
        file_values = {**load_file(ns.config), **(file_values or {})}
    for k, v in (file_values or {}).items():
        k = k.replace("-", "_")
        if k not in names:
            raise ValueError(f"unknown config key {k!r} for {cls.__name__}")
        vals[k] = _coerce(_field_type(names[k]), v)
    for k, f in names.items():
        e = env.get(ENV_PREFIX + k.upper())
        if e is not None:
            vals[k] = _coerce(_field_type(f), e)
    if ns is not None:
        for k, f in names.items():
            v = getattr(ns, k, None)
            if v is not None:
                vals[k] = _coerce(_field_type(f), v)
    return cls(**vals)


def parse(cls: Type[T], argv: Optional[Sequence[str]] = None, prog: Optional[str] = None) -> T:
    ap = argparse.ArgumentParser(prog=prog)
    add_arguments(ap, cls)
    return resolve(cls, ap.parse_args(argv))


def to_dict(cfg: Any) -> Dict[str, Any]:
    return dataclasses.asdict(cfg)


def dims_of(model: str) -> List[int]:
    return [int(x) for x in model.replace("x", "-").split("-") if x]
